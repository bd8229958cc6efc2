// Winograd F(2x2, 3x3) on bf16 MFMAs with fp32-exact operand splitting ("bf16x6"): the same
// layers and the same transforms as sp_wino.hip, but the 16 GEMMs
// M_xi = sum_ci U_xi[co][ci] V_xi[ci][tile] run on v_mfma_f32_32x32x16_bf16 (16x the MACs per
// cycle of the fp32 MFMA) with every fp32 operand split EXACTLY into three bf16 terms,
//
//   a = a_h + a_m + a_l     a_h = a truncated to bf16, a_m = (a - a_h) truncated, a_l = rest
//
// (a 24-bit significand is three 8-bit ones: every split is exact, no rounding), and the
// product taken as the six terms down to 2^-16 relative,
//
//   u v ~ u_h v_h + u_h v_m + u_m v_h + u_h v_l + u_l v_h + u_m v_m    (dropped: <= 3 * 2^-24)
//
// each a bf16 x bf16 product (exact in fp32) accumulated in fp32 by the MFMA.  The error of
// a layer is that of an fp32 GEMM (tests/test_conv_gpu.py pins it against fp64 next to the
// fp32-MFMA tile); it is an fp32 computation carried on the bf16 datapath, not a bf16 one.
//
// Tile: one workgroup = 32 output channels x 16 x 32 outputs; its four waves each own 2 x 16
// output tiles (4 x 32 outputs) of the same 32 channels, all 16 GEMMs in 256 AGPRs.  A k-step
// is 16 input channels (the MFMA's K): U for the workgroup's 32 channels (48 KB: 16 xi x 3
// terms x 32 co x 16 ci) comes into LDS by direct global->LDS loads one k-step ahead (two
// buffers, one barrier per k-step); each wave's input block (16 channels x 6 rows x 34
// columns) is loaded into registers one k-step ahead and written to a wave-private LDS
// region; each lane builds V for one tile and 8 channels, one row of xi at a time, splits it
// and packs channel pairs into the MFMA's B fragment.

#include "sp_common.h"

#include <algorithm>

namespace sp {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned uvec4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#ifndef X6_EXP
#define X6_EXP 0  // diagnostics only (wrong results, timing): 1 no loads in the k loop, 2 no
                  // MFMA work, 3 no waits / barrier between k-steps
#endif
constexpr int X6_CO = 32;                  // output channels per workgroup
constexpr int X6_KC = 16;                  // input channels per k-step (the MFMA's K)
constexpr int X6_ROW = 40;                 // LDS floats per block row: col -1 at 3, cols 0.. at 4..
constexpr int X6_CI = 252;                 // per channel: 6 rows; 8 channels = 32 banks apart
constexpr int X6_WAVE = X6_KC * X6_CI;     // floats of a wave's input block
constexpr int X6_USTAGE = 16 * 3 * 64 * 16;  // bytes of U per k-step (48 KB)
constexpr int X6_WG_ROWS = 16, X6_WG_COLS = 32;
// row r of a channel's block: rows two apart sit 84 floats (20 banks) apart, every row
// 16-byte aligned for the staging writes
__device__ constexpr int x6_row(int r) { return r * X6_ROW + 4 * (r >> 1); }

struct X6Geom {
    int64_t batch;
    const float* x;
    const unsigned short* up;  // packed U terms (sp_wino3x3_x6_pack)
    float* out;
    const float* bias;
    const float* res;
    int cin, cout, H, W, plane;
    int ntiles, cob, tiles_w, per_img, nsteps;
};

struct X6Tile { int n, oh0, ow0, cb; };

__device__ __forceinline__ X6Tile x6_tile(const X6Geom& g, int t) {
    // XCD-aware: tiles t and t + 8 run on one XCD, so consecutive logical tiles (the channel
    // blocks of one spatial tile, then its neighbours) share an L2
    const int lb = (g.ntiles & 7) ? t : (t & 7) * (g.ntiles >> 3) + (t >> 3);
    const int cb = lb % g.cob, rest = lb / g.cob;
    const int n = rest / g.per_img, r = rest - n * g.per_img;
    const int ty = r / g.tiles_w;
    return X6Tile{n, ty * X6_WG_ROWS, (r - ty * g.tiles_w) * X6_WG_COLS, cb};
}

// A wave's input-block loads for one k-step (16 channels x 6 rows x 34 columns).  Interior:
// 12 16-byte loads; load i covers block rows i, i + 12, ..., i + 84 (lane >> 3 picks one, lane
// & 7 the 16-byte piece), i.e. channel 2 (lane >> 3) + i / 6 at row i % 6, so the lane part of
// the address is one tile-independent VGPR and the load's row is uniform (a row outside the
// image is a uniform out-of-range scalar offset: the buffer returns zeros).  Halo columns: 4
// dword loads (channel half h, side), lanes 0..47 one block row each.
struct X6Lane {
    int vi, li;   // interior: byte offset (2q plane + 4k) * 4, LDS index 2q CI + 4 + 4k
    int mh;       // halo: (m / 6) plane + (m % 6) W for lane m < 48, else -1
    int lh;       // halo: LDS index (m / 6) CI + row(m % 6)
};
struct X6Src {
    __amdgpu_buffer_rsrc_t rs;
    int base;        // (row0 * W + ow0) * 4 (negative only at the top edge, row 0 unused there)
    int nrec;        // the buffer's size: a scalar offset at least this reads zeros
    int row0;
    int hl, hr;      // halo byte offsets (left / right column) of this lane, or out of range
};
struct X6Regs { f32x4 a[12]; float h[4]; };

constexpr int X6_OOB = 0x7FFFFFF0;

__device__ __forceinline__ X6Lane x6_lane(const X6Geom& g, int lane) {
    X6Lane L;
    const int q = lane >> 3, k = lane & 7;
    L.vi = (2 * q * g.plane + 4 * k) * 4;
    L.li = 2 * q * X6_CI + 4 + 4 * k;
    const int m = lane < 48 ? lane : 0;
    L.mh = lane < 48 ? (m / 6) * g.plane + (m % 6) * g.W : -1;
    L.lh = (m / 6) * X6_CI + x6_row(m % 6);
    return L;
}

__device__ __forceinline__ X6Src x6_src(const X6Geom& g, const X6Lane& L, const X6Tile& ti, int wv,
                                        int lane) {
    X6Src s;
    s.rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.x + (int64_t)ti.n * g.cin * g.plane),
                                             (short)0, g.cin * g.plane * 4, 0x00020000);
    s.nrec = g.cin * g.plane * 4;
    s.row0 = ti.oh0 + 4 * wv - 1;
    s.base = (s.row0 * g.W + ti.ow0) * 4;
    const int r = lane < 48 ? lane % 6 : 0;
    const bool rowok = L.mh >= 0 && (unsigned)(s.row0 + r) < (unsigned)g.H;
    const int hb = L.mh + s.row0 * g.W + ti.ow0;
    s.hl = rowok && ti.ow0 > 0 ? (hb - 1) * 4 : X6_OOB;
    s.hr = rowok && ti.ow0 + 32 < g.W ? (hb + 32) * 4 : X6_OOB;
    return s;
}

__device__ __forceinline__ void x6_load(const X6Src& s, const X6Lane& L, int so, X6Regs& r, int plane,
                                        int W, int H) {
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const int row = i % 6;
        const bool ok = (unsigned)(s.row0 + row) < (unsigned)H;  // uniform
        const int sof = ok ? so + ((i / 6) * plane + row * W) * 4 + s.base : s.nrec;
        r.a[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(s.rs, L.vi, sof, 0));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
        r.h[j] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            s.rs, (j & 1) ? s.hr : s.hl, so + (j >> 1) * 8 * plane * 4, 0));
}

__device__ __forceinline__ void x6_stage(float* xw, const X6Lane& L, int lane, const X6Regs& r) {
#pragma unroll
    for (int i = 0; i < 12; ++i)
        *reinterpret_cast<f32x4*>(xw + L.li + (i / 6) * X6_CI + x6_row(i % 6)) = r.a[i];
    if (lane < 48) {
#pragma unroll
        for (int j = 0; j < 4; ++j) xw[L.lh + (j >> 1) * 8 * X6_CI + ((j & 1) ? 36 : 3)] = r.h[j];
    }
}

// U terms of one k-step (48 KB, contiguous in the packed layout) -> LDS buffer, 12 direct
// buffer loads of 1 KB per wave (lane offset lane * 16 in one VGPR, the chunk as a scalar).
// Written as inline asm: the compiler's wait insertion does not see these loads, so it does not
// drain them (vmcnt(0)) before every LDS read of the k-step; the kernel waits for them itself.
__device__ __forceinline__ void x6_lds_dma(__amdgpu_buffer_rsrc_t rs, const void* lds, int voff, int soff) {
    const unsigned la = static_cast<unsigned>(reinterpret_cast<size_t>((lds_void*)lds));
    unsigned keep;  // m0 is reserved to the compiler: saved and restored around the load
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(__builtin_amdgcn_readfirstlane(la)), "v"(voff), "s"(rs), "s"(soff)
                 : "memory");
}
__device__ __forceinline__ void x6_load_u(__amdgpu_buffer_rsrc_t urs, int stage, int wv, int lane,
                                          unsigned char* ubuf) {
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const int chunk = 12 * wv + i;
        x6_lds_dma(urs, ubuf + chunk * 1024, lane * 16, stage * X6_USTAGE + chunk * 1024);
    }
}

// exact three-way split of an fp32 value into bf16 terms (truncation: each step exact)
__device__ __forceinline__ void x6_split(float v, unsigned& h, unsigned& m, unsigned& l) {
    const unsigned vb = __float_as_uint(v);
    h = vb & 0xffff0000u;
    const float r = v - __uint_as_float(h);
    m = __float_as_uint(r) & 0xffff0000u;
    l = __float_as_uint(r - __uint_as_float(m));  // low 16 bits are zero
}
// (bf16 of a, bf16 of b) -> one register, a in the low half
__device__ __forceinline__ unsigned x6_pack(unsigned a, unsigned b) {
    return __builtin_amdgcn_perm(b, a, 0x07060302u);
}

__device__ __forceinline__ f32x16 x6_mfma(uvec4 a, uvec4 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// One k-step's MFMA work: V for this lane's tile and 8 channels from the staged block, one
// row of xi at a time, 6 MFMAs per xi, software-pipelined by hand: the region of xi issues
// the LDS reads of U(xi + 1) and of the next xi-row's window rows first, then its 6 MFMAs
// with the VALU work of V(xi + 1) (transform, split, pack: ~60 instructions) between them —
// beside bf16 MFMAs independent f32 VALU work issues in the MFMA's shadow, unlike beside
// fp32 ones (tools/mfma_gap.hip) — and ends at a scheduling wall.
struct X6Op { uvec4 h, m, l; };

// t_r = (B^T d)_r per column for channel j: r0 = d0 - d2, r1 = d1 + d2, r2 = d2 - d1, r3 = d1 - d3
__device__ __forceinline__ void x6_trow(const float* xr, int r, int j, float (&t)[4]) {
    constexpr int RO[4] = {0, X6_ROW, x6_row(2), x6_row(3)};  // window rows (both tile rows)
    const int ra = r == 0 ? 0 : (r == 2 ? 2 : 1);
    const int rb = r == 0 ? 2 : (r == 1 ? 2 : (r == 2 ? 1 : 3));
    const float* b = xr + j * X6_CI;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float a = b[RO[ra] + c], d = b[RO[rb] + c];
        t[c] = r == 1 ? a + d : a - d;
    }
}
// the window rows of t_r for channel j, read (the subtraction follows a region later)
struct X6Rows { float a[4], d[4]; };
__device__ __forceinline__ X6Rows x6_rows(const float* xr, int r, int j) {
    constexpr int RO[4] = {0, X6_ROW, x6_row(2), x6_row(3)};
    const int ra = r == 0 ? 0 : (r == 2 ? 2 : 1);
    const int rb = r == 0 ? 2 : (r == 1 ? 2 : (r == 2 ? 1 : 3));
    const float* b = xr + j * X6_CI;
    X6Rows w;
#pragma unroll
    for (int c = 0; c < 4; ++c) w.a[c] = b[RO[ra] + c], w.d[c] = b[RO[rb] + c];
    return w;
}
__device__ __forceinline__ void x6_tfrom(const X6Rows& w, int r, float (&t)[4]) {
#pragma unroll
    for (int c = 0; c < 4; ++c) t[c] = r == 1 ? w.a[c] + w.d[c] : w.a[c] - w.d[c];
}

// B fragments (three terms) of V_xi, xi = 4 r + cc, from t_r of the 8 channels
__device__ __forceinline__ X6Op x6_v(const float (&t)[8][4], int cc) {
    X6Op o;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const float* a = t[2 * p];
        const float* e = t[2 * p + 1];
        // v = t B per row: (t0 - t2, t1 + t2, t2 - t1, t1 - t3)
        const float v0 = cc == 0 ? a[0] - a[2] : cc == 1 ? a[1] + a[2] : cc == 2 ? a[2] - a[1] : a[1] - a[3];
        const float v1 = cc == 0 ? e[0] - e[2] : cc == 1 ? e[1] + e[2] : cc == 2 ? e[2] - e[1] : e[1] - e[3];
        unsigned h0, m0, l0, h1, m1, l1;
        x6_split(v0, h0, m0, l0);
        x6_split(v1, h1, m1, l1);
        o.h[p] = x6_pack(h0, h1);
        o.m[p] = x6_pack(m0, m1);
        o.l[p] = x6_pack(l0, l1);
    }
    return o;
}

__device__ __forceinline__ X6Op x6_u(const unsigned char* ub, int xi, int lane) {
    const uvec4* uq = reinterpret_cast<const uvec4*>(ub) + xi * 3 * 64 + lane;
    return X6Op{uq[0], uq[64], uq[128]};
}

__device__ __forceinline__ void x6_compute(const float* xr, const unsigned char* ub, int lane,
                                           f32x16 (&acc)[16]) {
    float t[8][4], tn[8][4];
    X6Rows w[3];
    // prologue: t_0, U(0), V(0)
#pragma unroll
    for (int j = 0; j < 8; ++j) x6_trow(xr, 0, j, t[j]);
    X6Op u = x6_u(ub, 0, lane);
    X6Op v = x6_v(t, 0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) {
        const int r = xi >> 2, cc = xi & 3;
        // LDS reads first: U(xi + 1); window rows of t_{r+1}, channels 3cc .. 3cc+2 (cc < 3)
        X6Op un = u;
        if (xi < 15) un = x6_u(ub, xi + 1, lane);
        X6Rows wn[3];
        if (r < 3 && cc < 3) {
#pragma unroll
            for (int k = 0; k < 3; ++k)
                if (3 * cc + k < 8) wn[k] = x6_rows(xr, r + 1, 3 * cc + k);
        }
        // this xi's 6 products (small terms first)
        f32x16 c = acc[xi];
        c = x6_mfma(u.l, v.h, c);
        c = x6_mfma(u.h, v.l, c);
        c = x6_mfma(u.m, v.m, c);
        c = x6_mfma(u.m, v.h, c);
        c = x6_mfma(u.h, v.m, c);
        acc[xi] = x6_mfma(u.h, v.h, c);
        // t_{r+1} of the channels read in the previous region
        if (r < 3 && cc > 0) {
#pragma unroll
            for (int k = 0; k < 3; ++k)
                if (3 * (cc - 1) + k < 8) x6_tfrom(w[k], r + 1, tn[3 * (cc - 1) + k]);
        }
        // V(xi + 1)
        X6Op vn = v;
        if (xi < 15) vn = x6_v(cc == 3 ? tn : t, (xi + 1) & 3);
        // issue order: the reads, then MFMA / VALU alternating
        __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 12, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        u = un;
        v = vn;
#pragma unroll
        for (int k = 0; k < 3; ++k) w[k] = wn[k];
        if (cc == 3) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) t[j][q] = tn[j][q];
        }
    }
}

// Y = A^T M A per (channel, tile) in registers, + bias (+ residual), as sp_wino.hip: register
// q of every accumulator is channel co0 + (q&3) + 8(q>>2) + 4hh, tile l = lane & 31.
template <bool RES>
__device__ __forceinline__ void x6_epilogue(const X6Geom& g, const X6Tile& ti, int wv, int lane,
                                            const f32x16 (&acc)[16]) {
    const int hh = lane >> 5, l = lane & 31, tr = l >> 4, tc = l & 15;
    const int co0 = ti.cb * X6_CO;
    const int64_t img = (int64_t)ti.n * g.cout * g.plane;
    const auto ors = __builtin_amdgcn_make_buffer_rsrc(g.out + img, (short)0, g.cout * g.plane * 4, 0x00020000);
    const auto rrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(RES ? g.res + img : g.out), (short)0,
                                                       RES ? g.cout * g.plane * 4 : 0, 0x00020000);
    const int vo = ((co0 + 4 * hh) * g.plane + (ti.oh0 + 4 * wv + 2 * tr) * g.W + ti.ow0 + 2 * tc) * 4;
    const auto brs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.bias ? g.bias : g.out), (short)0,
                                                       g.bias ? g.cout * 4 : 0, 0x00020000);
    const float bl = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(brs, (co0 + l) * 4, 0, 0));
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        float s0[4], s1[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const float m0 = acc[a * 4 + 0][q], m1 = acc[a * 4 + 1][q];
            const float m2 = acc[a * 4 + 2][q], m3 = acc[a * 4 + 3][q];
            s0[a] = m0 + m1 + m2;
            s1[a] = m1 - m2 - m3;
        }
        const int c = (q & 3) + 8 * (q >> 2);
        const float b0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, bl), c));
        const float b1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, bl), c + 4));
        const float bv = hh ? b1 : b0;
        const int so = c * g.plane * 4;
        f32x2 y0 = {s0[0] + s0[1] + s0[2] + bv, s1[0] + s1[1] + s1[2] + bv};
        f32x2 y1 = {s0[1] - s0[2] - s0[3] + bv, s1[1] - s1[2] - s1[3] + bv};
        if constexpr (RES) {
            y0 += __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rrs, vo, so, 0));
            y1 += __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rrs, vo, so + g.W * 4, 0));
        }
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y0), ors, vo, so, 0);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y1), ors, vo, so + g.W * 4, 0);
        // one register row at a time (the next tile's operands are live: no hoisted reads)
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Persistent: one workgroup per CU walks tiles t = blockIdx.x, + gridDim.x, ...; the k-step
// stream runs on across tile boundaries (the next tile's first block and U are fetched
// during this tile's last k-step).
template <bool RES>
__global__ __launch_bounds__(kBlock, 1) void k_wino3x3_x6(X6Geom g) {
    __shared__ __attribute__((aligned(16))) unsigned char ulds[2 * X6_USTAGE];
    __shared__ __attribute__((aligned(16))) float xlds[4 * X6_WAVE];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar offsets
    float* const xw = xlds + wv * X6_WAVE;
    const int l = lane & 31;
    const float* const xr = xw + (lane >> 5) * 8 * X6_CI + x6_row(2 * (l >> 4)) + 3 + 2 * (l & 15);
    const int so_step = X6_KC * g.plane * 4;
    const auto urs = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(g.up), (short)0,
                                                       g.cob * g.nsteps * X6_USTAGE, 0x00020000);

    int t = blockIdx.x;
    X6Tile ti = x6_tile(g, t);
    const X6Lane xl = x6_lane(g, lane);
    X6Src cur = x6_src(g, xl, ti, wv, lane);
    X6Regs xr_next;
    // prologue: step 0 of the first tile
    x6_load(cur, xl, 0, xr_next, g.plane, g.W, g.H);
    x6_load_u(urs, ti.cb * g.nsteps, wv, lane, ulds);
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0) expcnt(0)
    x6_stage(xw, xl, lane, xr_next);
    __syncthreads();

    f32x16 acc[16];
    int buf = 0;
    for (;;) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = f32x16{};
        for (int s = 0; s + 1 < g.nsteps; ++s) {
#if X6_EXP != 1
            x6_load(cur, xl, (s + 1) * so_step, xr_next, g.plane, g.W, g.H);
            x6_load_u(urs, ti.cb * g.nsteps + s + 1, wv, lane, ulds + (buf ^ 1) * X6_USTAGE);
#endif
#if X6_EXP != 2
            x6_compute(xr, ulds + buf * X6_USTAGE, lane, acc);
#endif
#if X6_EXP != 3
            __builtin_amdgcn_s_waitcnt(0);
#endif
#if X6_EXP != 1
            x6_stage(xw, xl, lane, xr_next);
#endif
#if X6_EXP != 3
            __syncthreads();
#endif
            buf ^= 1;
        }
        // last k-step: fetch the next tile's first block and U meanwhile
        const int tn = t + (int)gridDim.x;
        const bool more = tn < g.ntiles;
        const X6Tile tin = x6_tile(g, more ? tn : t);
        const X6Src nxt = x6_src(g, xl, tin, wv, lane);
        if (more) {
            x6_load(nxt, xl, 0, xr_next, g.plane, g.W, g.H);
            x6_load_u(urs, tin.cb * g.nsteps, wv, lane, ulds + (buf ^ 1) * X6_USTAGE);
        }
        x6_compute(xr, ulds + buf * X6_USTAGE, lane, acc);
        x6_epilogue<RES>(g, ti, wv, lane, acc);
        if (!more) break;
        __builtin_amdgcn_s_waitcnt(0);
        x6_stage(xw, xl, lane, xr_next);
        __syncthreads();
        buf ^= 1;
        t = tn;
        ti = tin;
        cur = nxt;
    }
}

// U = G g G^T per (co, ci) (as sp_wino.hip), split into three bf16 terms and packed as the
// MFMA's A fragments: u16 index ((((cb * nsteps + s) * 16 + xi) * 3 + term) * 64 + lane) * 8 + j
// for output row orow = 32 cb + (lane & 31) and input ci = 16 s + 8 (lane >> 5) + j.
__global__ void k_wino3x3_x6_pack(const float* __restrict__ w, int cout, int cin, int flip,
                                  unsigned short* __restrict__ up) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (co, ci) of W
    if (i >= (int64_t)cout * cin) return;
    const int co = static_cast<int>(i / cin), ci = static_cast<int>(i - (int64_t)co * cin);
    float g[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) g[k] = flip ? w[i * 9 + (8 - k)] : w[i * 9 + k];
    const int orow = flip ? ci : co, kin = flip ? co : ci, kin_n = flip ? cout : cin;
    float tg[12];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        tg[0 * 3 + c] = g[0 * 3 + c];
        tg[1 * 3 + c] = 0.5f * (g[0 * 3 + c] + g[1 * 3 + c] + g[2 * 3 + c]);
        tg[2 * 3 + c] = 0.5f * (g[0 * 3 + c] - g[1 * 3 + c] + g[2 * 3 + c]);
        tg[3 * 3 + c] = g[2 * 3 + c];
    }
    float u[16];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float a = tg[r * 3 + 0], b = tg[r * 3 + 1], c = tg[r * 3 + 2];
        u[r * 4 + 0] = a;
        u[r * 4 + 1] = 0.5f * (a + b + c);
        u[r * 4 + 2] = 0.5f * (a - b + c);
        u[r * 4 + 3] = c;
    }
    const int nsteps = kin_n / X6_KC, cb = orow / X6_CO, s = kin / X6_KC;
    const int lane = (orow & 31) + 32 * ((kin & 15) >> 3), j = kin & 7;
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) {
        unsigned h, m, l;
        x6_split(u[xi], h, m, l);
        const int64_t base = ((((int64_t)cb * nsteps + s) * 16 + xi) * 3) * 64;
        up[((base + 0 * 64) + lane) * 8 + j] = static_cast<unsigned short>(h >> 16);
        up[((base + 1 * 64) + lane) * 8 + j] = static_cast<unsigned short>(m >> 16);
        up[((base + 2 * 64) + lane) * 8 + j] = static_cast<unsigned short>(l >> 16);
    }
}

}  // namespace sp

using namespace sp;

extern "C" {

int sp_wino3x3_x6_supported(int32_t cin, int32_t cout, int32_t height, int32_t width) {
    return cin >= X6_KC && cin % X6_KC == 0 && cout >= X6_CO && cout % X6_CO == 0 &&
           height > 0 && height % X6_WG_ROWS == 0 && width > 0 && width % X6_WG_COLS == 0;
}

// packed U terms: cin * cout * 16 xi * 3 terms bf16 = cin * cout * 24 floats of storage
int64_t sp_wino3x3_x6_packed_size(int32_t cin, int32_t cout) { return (int64_t)cin * cout * 24; }

int sp_wino3x3_x6_pack(const float* w, int32_t cout, int32_t cin, int32_t input_vjp, float* up,
                       sp_stream_t stream) {
    if (!w || !up || cout <= 0 || cin <= 0) return SP_EINVAL;
    const int kin = input_vjp ? cout : cin, nout = input_vjp ? cin : cout;
    if (kin % X6_KC || nout % X6_CO) return SP_EINVAL;
    const int64_t total = (int64_t)cout * cin;
    launch(0, k_wino3x3_x6_pack, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256),
           static_cast<hipStream_t>(stream), w, cout, cin, input_vjp,
           reinterpret_cast<unsigned short*>(up));
    return check_launch("sp_wino3x3_x6_pack");
}

static int x6_cu_count() {
    static int cached[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cached[dev]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            v = 256;
        cached[dev] = v;
    }
    return cached[dev];
}

static int wino3x3_x6(int kind, const float* x, const float* up, const float* bias, const float* res,
                      int64_t n, int32_t cin, int32_t cout, int32_t height, int32_t width, float* y,
                      sp_stream_t stream, const char* what) {
    if (!sp_wino3x3_x6_supported(cin, cout, height, width) || n < 0) return SP_EINVAL;
    if (n == 0) return SP_OK;
    if (!x || !up || !y) return SP_EINVAL;
    const int64_t tiles = n * (height / X6_WG_ROWS) * (width / X6_WG_COLS) * (cout / X6_CO);
    if (tiles >= (int64_t(1) << 31) || (int64_t)cin * height * width * 4 >= (int64_t(1) << 31) ||
        (int64_t)cout * height * width * 4 >= (int64_t(1) << 31))
        return SP_EINVAL;
    X6Geom g;
    g.batch = n;
    g.x = x;
    g.up = reinterpret_cast<const unsigned short*>(up);
    g.out = y;
    g.bias = bias;
    g.res = res;
    g.cin = cin;
    g.cout = cout;
    g.H = height;
    g.W = width;
    g.plane = height * width;
    g.ntiles = static_cast<int>(tiles);
    g.cob = cout / X6_CO;
    g.tiles_w = width / X6_WG_COLS;
    g.per_img = g.tiles_w * (height / X6_WG_ROWS);
    g.nsteps = cin / X6_KC;
    const int grid = static_cast<int>(std::min<int64_t>(tiles, x6_cu_count()));
    // algorithmic Winograd work (the fp32 tile's executed MFMA FLOPs; the bf16 MFMAs execute
    // 6x that on the split terms)
    const double flops = 8.0 * n * cin * cout * height * width;
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (res) launch_w(kind, flops, k_wino3x3_x6<true>, dim3(grid), dim3(kBlock), st, g);
    else launch_w(kind, flops, k_wino3x3_x6<false>, dim3(grid), dim3(kBlock), st, g);
    return check_launch(what);
}

int sp_wino3x3_x6_fwd(const float* x, const float* up, const float* bias, const float* res, int64_t n,
                      int32_t cin, int32_t cout, int32_t height, int32_t width, float* y,
                      sp_stream_t stream) {
    if (res && res == y) return SP_EINVAL;
    return wino3x3_x6(TK_WINO3X3_FWD, x, up, bias, res, n, cin, cout, height, width, y, stream,
                      "sp_wino3x3_x6_fwd");
}

int sp_wino3x3_x6_bwd_input(const float* dy, const float* up_vjp, int64_t n, int32_t cin,
                            int32_t cout, int32_t height, int32_t width, float* dx,
                            sp_stream_t stream) {
    return wino3x3_x6(TK_WINO3X3_BWD_INPUT, dy, up_vjp, nullptr, nullptr, n, cout, cin, height,
                      width, dx, stream, "sp_wino3x3_x6_bwd_input");
}

}  // extern "C"

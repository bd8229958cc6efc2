// Winograd F(2x2, 3x3) convolution on fp32 MFMA: the same 3x3 / stride 1 / pad 1
// layers as sp_conv.hip (ResnetBlock / mid / up-sampling convolutions of the SD VAE
// and the DDPM UNet) with 2.25x fewer multiplies.
//
//   U = G g G^T   (4x4 per (co, ci); weights transformed + packed once per layer)
//   V = B^T d B   (4x4 per (ci, tile) from the 4x4 input window of a 2x2 output tile)
//   M_xi = sum_ci U_xi[co][ci] * V_xi[ci][tile]      16 GEMMs on v_mfma_f32_32x32x2_f32
//   Y = A^T M A   (2x2 outputs per (co, tile))
//
// Kernel structure: see k_wino3x3_r below (register-resident, one persistent workgroup
// per CU) and its ξ-split form k_wino3x3_xi (the default for the W % 32 layers: the waves of
// a pair split the 16 GEMMs by ξ, so each transforms half of V).  Earlier layouts, measured
// and replaced: an LDS-staged workgroup tile (U and V through double-buffered LDS, one
// barrier per 4 input channels, 4 waves splitting the 16 GEMMs by rows of M and reducing the
// output transform through LDS): 167-203 effective TFLOP/s, barrier- and wait-bound (42 % of
// wave time parked); round 3: V shared between the co-half waves through LDS (-0.6 %), a
// four-way ξ-row split (-1.7 % against the two-way one).
//
// Numerics: exact fp32 MFMA accumulation of fp32 transforms; the transforms add the
// usual F(2,3) rounding (|coefficients| <= 1, one 0.5 factor), comparable to MIOpen's
// own Winograd f2x3 solver that these layers ran on before.

#define SP_TU 6  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

#include <algorithm>
#include <utility>

namespace sp {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// f(std::integral_constant<int, I>) for I = B .. E - 1, unrolled at compile time
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

// V = B^T d B for a 4x4 window d (row-major), B^T = [[1,0,-1,0],[0,1,1,0],[0,-1,1,0],[0,1,0,-1]]
__device__ __forceinline__ void wino_in(const float (&d)[16], float (&v)[16]) {
    float t[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {  // columns: t = B^T d
        t[0 * 4 + c] = d[0 * 4 + c] - d[2 * 4 + c];
        t[1 * 4 + c] = d[1 * 4 + c] + d[2 * 4 + c];
        t[2 * 4 + c] = d[2 * 4 + c] - d[1 * 4 + c];
        t[3 * 4 + c] = d[1 * 4 + c] - d[3 * 4 + c];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // rows: v = t B
        v[r * 4 + 0] = t[r * 4 + 0] - t[r * 4 + 2];
        v[r * 4 + 1] = t[r * 4 + 1] + t[r * 4 + 2];
        v[r * 4 + 2] = t[r * 4 + 2] - t[r * 4 + 1];
        v[r * 4 + 3] = t[r * 4 + 1] - t[r * 4 + 3];
    }
}

// The same V on packed fp32 (v_pk_add_f32, two lanes per instruction).  Window row r is
// held as its two natural register pairs, p = (d[r][0], d[r][1]) and q = (d[r][2], d[r][3])
// (ds_read2 results, used in place: no register moves), so every step below is one packed
// add with operand swizzles:
//   t = B^T d on pairs:  t0 = d0 - d2, t1 = d1 + d2, t2 = d2 - d1, t3 = d1 - d3
//   v = t B per row:     (v0, v1) = (p.x - q.x, p.y + q.x),  (v2, v3) = (q.x - p.y, p.y - q.y)
// 16 instructions for the 4x4 window instead of 32 scalar ones; every element is the same
// single IEEE add or subtract as the scalar transform (bit-identical).
// (The compiler does not form the swizzled packed adds from vector code, so they are
// written out.)
struct WinRow { f32x2 p, q; };

__device__ __forceinline__ f32x2 pk_add(f32x2 a, f32x2 b) {  // a + b
    f32x2 r;
    asm("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f32x2 pk_sub(f32x2 a, f32x2 b) {  // a - b
    f32x2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ f32x2 pk_row01(f32x2 p, f32x2 q) {  // (p.x - q.x, p.y + q.x)
    f32x2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,0] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(p), "v"(q));
    return r;
}
__device__ __forceinline__ f32x2 pk_row23(f32x2 p, f32x2 q) {  // (q.x - p.y, p.y - q.y)
    f32x2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,1] neg_lo:[0,1] neg_hi:[1,0]"
        : "=v"(r) : "v"(q), "v"(p));
    return r;
}

__device__ __forceinline__ WinRow wpk_t(int k, const WinRow (&d)[4]) {  // row k of B^T d
    switch (k) {
        case 0: return WinRow{pk_sub(d[0].p, d[2].p), pk_sub(d[0].q, d[2].q)};
        case 1: return WinRow{pk_add(d[1].p, d[2].p), pk_add(d[1].q, d[2].q)};
        case 2: return WinRow{pk_sub(d[2].p, d[1].p), pk_sub(d[2].q, d[1].q)};
        default: return WinRow{pk_sub(d[1].p, d[3].p), pk_sub(d[1].q, d[3].q)};
    }
}

__device__ __forceinline__ void wpk_v(const WinRow& t, float* v) {  // row of t B
    const f32x2 a = pk_row01(t.p, t.q);  // (t0 - t2, t1 + t2)
    const f32x2 b = pk_row23(t.p, t.q);  // (t2 - t1, t1 - t3)
    v[0] = a.x, v[1] = a.y, v[2] = b.x, v[3] = b.y;
}

// U = G g G^T (4x4, row-major) for a 3x3 filter g, G = [[1,0,0],[.5,.5,.5],[.5,-.5,.5],[0,0,1]]
__device__ __forceinline__ void wino_filter(const float (&g)[9], float (&u)[16]) {
    float tg[12];  // G g (4 x 3)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        tg[0 * 3 + c] = g[0 * 3 + c];
        tg[1 * 3 + c] = 0.5f * (g[0 * 3 + c] + g[1 * 3 + c] + g[2 * 3 + c]);
        tg[2 * 3 + c] = 0.5f * (g[0 * 3 + c] - g[1 * 3 + c] + g[2 * 3 + c]);
        tg[3 * 3 + c] = g[2 * 3 + c];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float a = tg[r * 3 + 0], b = tg[r * 3 + 1], c = tg[r * 3 + 2];
        u[r * 4 + 0] = a;
        u[r * 4 + 1] = 0.5f * (a + b + c);
        u[r * 4 + 2] = 0.5f * (a - b + c);
        u[r * 4 + 3] = c;
    }
}

// ---------------------------------------------------------------------------------------
// Register-resident kernel.  A wave's MFMA operands are
// disjoint from its neighbours' — U rows by output channel, V by tile — so each wave runs
// on its own: it computes all 16 transformed GEMMs of 32 output channels x 32 tiles (16 x
// 16 accumulators per lane, in AGPRs at one wave per SIMD), reads its packed U straight
// into registers (64 contiguous bytes per lane per k-step), and applies Y = A^T M A in
// registers at the end.  Its input block per k-step (2 channels x 6 rows x 34 columns) is
// read with coalesced 16-byte loads, written to a wave-private LDS region with even and
// odd columns apart, and read back as each lane's 4x4 window (conflict-free ds_read2)
// for V = B^T d B.  No barrier anywhere: the four waves of a workgroup (2 channel halves x
// 2 tile-row pairs: 64 channels x 8 x 32 outputs) only share cache lines.  Loads run
// three k-steps ahead for the input, two for U.
// (A first version loaded the 16 window pixels per lane with dword loads: 2.5x re-reads,
// uncoalesced; the address unit was 74 % busy and the MFMAs 48 %.)
// ---------------------------------------------------------------------------------------
constexpr int WR_CO = 64;   // output channels per workgroup (2 waves x 32)
#ifndef SP_WINO_EXP
#define SP_WINO_EXP 0  // diagnostics only: 1 = no loads in the k loop, 2 = no output stores,
                       // 3 = no input transform, 6 = the ξ-split tile without its epilogue
                       // (wrong results, timing only)
#endif
#ifndef SP_WINO_BURST
#define SP_WINO_BURST 1  // the transform's placement in the k-step: 0 one row per MFMA gap, 1 one
                         // burst, 2 two bursts (see wr_step)
#endif
#ifndef SP_WINO_SPLITK
#define SP_WINO_SPLITK 32  // most split-K parts a launch may use (1: no split)
#endif
constexpr int WR_NS = 4;    // unroll of the k-step ring (cin % (2 WR_NS) == 0)
// Tile geometry of a wave: 32 tiles (the MFMA's N) as TRW tile rows x TCW tile columns.
// TCW = 16 (images with W % 32 == 0): 2 x 16 tiles = 4 x 32 outputs; TCW = 8 (W = 16, the
// UNet's 16x16 level): 4 x 8 tiles = 8 x 16 outputs.  A workgroup stacks two waves' rows
// (and two 32-channel halves): 64 co x (4 TRW) x (2 TCW) outputs.
template <int TCW_, bool MOSAIC_ = false, bool SPLIT_ = false, int UP_ = 0>
struct WGeo {
    static constexpr int TCW = TCW_;
    // UP (diffusers Upsample2D: a nearest 2x upsample feeding this conv, fused; the W % 32
    // geometry of the xi tile, unsplit): 1 = the input is the half-resolution source, each
    // 16-byte piece of an upsampled row loaded as the 8 source bytes it repeats; 2 = the
    // output (the input VJP of conv(upsample(x))) summed over each 2x2 block into the
    // half-resolution gradient in the epilogue, in the upsample VJP's order.  Either way the
    // upsampled tensor is never written.
    static constexpr int UP = UP_;
    // SPLIT (launches whose tiles leave CUs idle: small batches, the low-resolution levels):
    // K cut into g.ksplit parts, one tile each; part kh stores its partial sums (no bias, no
    // residual) to workspace slice kh, and k_wino_split_reduce adds the slices in order, the
    // bias and the residual (deterministic; a compile-time variant: the other kernels keep
    // their register allocation)
    static constexpr bool SPLIT = SPLIT_;
    // MOSAIC (8x8 images, the UNet's 8x8 level): the W = 16 geometry over two images side by
    // side; in LDS image 1's columns start one position later, so one zero column (never
    // written) is image 0's right and image 1's left padding.
    static constexpr bool MOSAIC = MOSAIC_;
    static constexpr int TRW = 32 / TCW;
    static constexpr int ROWS = 2 * TRW + 2;     // input block rows per channel
    static constexpr int PPR = TCW / 2;          // 16-byte pieces per block row
    static constexpr int RC = 2 * ROWS;          // block rows of the k-step's two channels
    static constexpr int ROW = TCW == 16 ? 40 : 25;  // LDS floats per block row (cols -1.. at 3..)
    static constexpr int CI = TCW == 16 ? 6 * 40 : 10 * 25 + 8;  // per input channel
    static constexpr int WAVE = 2 * CI;
    static constexpr int WG_ROWS = 4 * TRW;      // output rows per workgroup
    static constexpr int WG_COLS = 2 * TCW;      // output columns per workgroup
    static_assert(RC - 64 / PPR == 4 && 2 * RC <= 64, "piece / halo lane mapping");
    // row r of a channel at r * ROW + r / 2: rows two apart sit an odd bank distance apart
    __device__ static constexpr int row(int r) { return r * ROW + (r >> 1); }
};

struct WrX { f32x4 a, b; float h; };  // a lane's share of one k-step's input block
struct WrU { f32x4 u[4]; };           // a lane's 16 U values (xi = 0..15) for one k-step
struct WxLane {                       // per-lane LDS indices (the same for every tile)
    int wa, wb, wh;   // where the two 16-byte pieces and the halo dword are written
    int rd;           // the window's first even-column read
};
struct WrTile {                       // one tile: 64 channels x 8 x 32 outputs of one image
    int n, oh0, ow0, co0;             // co0: this wave's first channel
    int kh;                           // split-K part (input channels kh * cin / ksplit ..)
};
struct WrSrc {                        // a tile's load sources
    __amdgpu_buffer_rsrc_t rs;        // the image's input planes
    int oa, ob, oh;                   // byte offsets of this lane's pieces (or OOB)
    int uso;                          // byte offset of the wave's packed U rows at k-step 0
                                      // (wave-uniform; a lane adds lane * 64)
};
struct WrGeom {
    int64_t batch;
    const float* x;
    const float* up;
    float* out;
    const float* bias;
    const float* res;   // NULL, or a tensor shaped like out added in the epilogue
    int cin, cout, H, W, plane;
    int ntiles, cob, tiles_w, per_img;
    int64_t u_step;                   // floats of packed U per k-step
    int so_step;                      // bytes of input per k-step (two channels)
    int nsteps;                       // k-steps per tile (of one split-K part)
    int ksplit;                       // split-K parts of the SPLIT kernels, else 1
    float* ws;                        // SPLIT: the parts' partial outputs [ksplit][batch][cout][H][W]
    int64_t ws_stride;                // floats per part slice
    int hplane, Wh;                   // UP: the half-resolution plane (H/2 x W/2) and row
};

// First image of a wave's data and how many of its images exist (MOSAIC: 2 per wave).
template <class GE>
__device__ __forceinline__ int64_t wr_img0(const WrGeom& g, const WrTile& ti, int wv) {
    return GE::MOSAIC ? ti.n + 2 * (wv >> 1) : ti.n;
}
template <class GE>
__device__ __forceinline__ int wr_nimg(const WrGeom& g, const WrTile& ti, int wv) {
    if constexpr (!GE::MOSAIC) return 1;
    const int64_t left = g.batch - wr_img0<GE>(g, ti, wv);
    return left <= 0 ? 0 : (left >= 2 ? 2 : 1);
}

template <class GE>
__device__ __forceinline__ WrTile wr_tile(const WrGeom& g, int t, int wv) {
    // XCD-aware order: tiles t and t + 8 run on one XCD (persistent workgroups b and b + 8
    // share one), so consecutive logical tiles (the channel blocks of one tile group, then
    // its neighbours) share an L2
    int lb = (g.ntiles & 7) ? t : (t & 7) * (g.ntiles >> 3) + (t >> 3);
    SP_DCHECK(t >= 0 && t < g.ntiles && lb < g.ntiles);
    int kh = 0;
    if constexpr (GE::SPLIT) kh = lb % g.ksplit, lb /= g.ksplit;
    const int co_blk = lb % g.cob, rest = lb / g.cob;
    if constexpr (GE::MOSAIC)  // four images per workgroup, two per wave
        return WrTile{4 * rest, 0, 0, co_blk * WR_CO + 32 * (wv & 1), kh};
    const int n = rest / g.per_img, r = rest - n * g.per_img;
    const int ty = r / g.tiles_w;
    return WrTile{n, ty * GE::WG_ROWS, (r - ty * g.tiles_w) * GE::WG_COLS, co_blk * WR_CO + 32 * (wv & 1),
                  kh};
}

template <class GE>
__device__ __forceinline__ WrSrc wr_src(const WrGeom& g, const WrTile& ti, int wv, int lane) {
    constexpr int OOB = 0x7FFFFFF0;  // outside the image: the buffer returns 0
    const int row0 = GE::MOSAIC ? -1 : ti.oh0 + 2 * GE::TRW * (wv >> 1) - 1;  // first input row
    const int ka = lane % GE::PPR, rca = lane / GE::PPR, rcb = 64 / GE::PPR + ((lane / GE::PPR) & 3);
    const int rch = (lane % (2 * GE::RC)) >> 1, side = lane & 1;
    // split-K part kh reads input channels kofs .. kofs + 2 nsteps - 1 (and the matching U)
    const int kofs = GE::SPLIT ? ti.kh * 2 * g.nsteps : 0, nimg = wr_nimg<GE>(g, ti, wv);
    auto goff = [&](int rc, int col) {
        const int ci = rc / GE::ROWS, gr = row0 + rc % GE::ROWS;
        if constexpr (GE::MOSAIC) {  // virtual column -> (image, column); rows 0..7; a column of
                                     // an image past the batch reads zeros (OOB)
            return (unsigned)gr < (unsigned)g.H && col >= 0 && col < 2 * g.W && (col >> 3) < nimg
                       ? ((col >> 3) * g.cin * g.plane + ci * g.plane + gr * g.W + (col & 7)) * 4
                       : OOB;
        }
        if constexpr (GE::UP == 1)  // upsampled (row, col) -> its source pixel (col even for pieces)
            return ((unsigned)gr < (unsigned)g.H && (unsigned)col < (unsigned)g.W)
                       ? (ci * g.hplane + (gr >> 1) * g.Wh + (col >> 1)) * 4 : OOB;
        return ((unsigned)gr < (unsigned)g.H && (unsigned)col < (unsigned)g.W)
                   ? (ci * g.plane + gr * g.W + col) * 4 : OOB;
    };
    const int pin = GE::UP == 1 ? g.hplane : g.plane;  // floats per input plane
    WrSrc s;
    s.rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(g.x + wr_img0<GE>(g, ti, wv) * g.cin * pin + (int64_t)kofs * pin),
        (short)0, nimg ? (nimg * g.cin - kofs) * pin * 4 : 0, 0x00020000);
    s.oa = goff(rca, ti.ow0 + 4 * ka);
    s.ob = goff(rcb, ti.ow0 + 4 * ka);
    s.oh = GE::MOSAIC ? OOB : goff(rch, side ? ti.ow0 + 2 * GE::TCW : ti.ow0 - 1);
    s.uso = __builtin_amdgcn_readfirstlane(
        static_cast<int>(((GE::SPLIT ? (int64_t)ti.kh * g.nsteps * g.u_step : 0) +
                          (int64_t)(ti.co0 >> 5) * 64 * 16) * 4));
#if SP_DEBUG
    {   // every k-step's input pieces inside this tile's planes — of the images that exist (a
        // MOSAIC wave's pieces of an image past the batch are OOB) —, U rows inside the packed U
        const int64_t span = nimg ? (int64_t)(nimg * g.cin - kofs) * pin * 4 : 0;
        const int64_t last = (int64_t)(g.nsteps - 1) * g.so_step;
        constexpr int piece = GE::UP == 1 ? 8 : 16;
        SP_DCHECK(s.oa == OOB || (s.oa >= 0 && s.oa + last + piece <= span));
        SP_DCHECK(s.ob == OOB || (s.ob >= 0 && s.ob + last + piece <= span));
        SP_DCHECK(s.oh == OOB || (s.oh >= 0 && s.oh + last + 4 <= span));
        SP_DCHECK(s.uso >= 0 && (int64_t)s.uso + ((int64_t)(g.nsteps - 1) * g.u_step + 64 * 16) * 4 <=
                                   (int64_t)g.nsteps * g.ksplit * g.u_step * 4);
        SP_DCHECK(ti.co0 + 32 <= g.cout && ti.n < g.batch);
    }
#endif
    return s;
}

template <class GE>
__device__ __forceinline__ void wr_load_x(const WrSrc& s, int so, WrX& x) {
    if constexpr (GE::UP == 1) {  // four upsampled columns = two source pixels, each twice
        const f32x2 a = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(s.rs, s.oa, so, 0));
        const f32x2 b = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(s.rs, s.ob, so, 0));
        x.a = f32x4{a.x, a.x, a.y, a.y};
        x.b = f32x4{b.x, b.x, b.y, b.y};
    } else {
        x.a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(s.rs, s.oa, so, 0));
        x.b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(s.rs, s.ob, so, 0));
    }
    x.h = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(s.rs, s.oh, so, 0));
}

// U rows of k-step `step` by buffer loads: the lane's offset is a fixed VGPR (lane * 64), the
// step's a scalar — no per-step vector address arithmetic beside the MFMAs.
__device__ __forceinline__ f32x4 wr_u4(__amdgpu_buffer_rsrc_t urs, int lane, int soff, int i) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(urs, lane * 64 + 16 * i, soff, 0));
}

__device__ __forceinline__ void wr_load_u(__amdgpu_buffer_rsrc_t urs, int lane, int soff, WrU& u) {
#pragma unroll
    for (int i = 0; i < 4; ++i) u.u[i] = wr_u4(urs, lane, soff, i);
}

// Block piece -> LDS (columns in natural order; dword pairs, so no register shuffles).
__device__ __forceinline__ void wr_stage_x(float* xw, const WxLane& xl, const WrX& x) {
#pragma unroll
    for (int i = 0; i < 4; ++i) xw[xl.wa + i] = x.a[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) xw[xl.wb + i] = x.b[i];
    xw[xl.wh] = x.h;
}

// Row r of this lane's 4x4 window (columns 2tc-1 .. 2tc+2 of the wave's rows 2tr .. 2tr+3)
// as the pairs of the packed transform.
template <class GE>
__device__ __forceinline__ WinRow wr_window_row(const float* xw, const WxLane& xl, int r) {
    const float* row = xw + xl.rd + GE::row(r);
    return WinRow{f32x2{row[0], row[1]}, f32x2{row[2], row[3]}};
}

struct WrRing {          // k-steps in flight
    WrX xs[4];
    WrU us[4];
    float v[2][16];      // V of the current and the next step
};

// One k-step q (slot K = q mod 4) of the current tile.  A wave issues in order and its
// vector work does not overlap an MFMA it has to wait behind, so the step is laid out by
// hand, one small piece of side work after each of the 16 MFMAs (each runs 64 cycles),
// with scheduling walls in between:
//   gap 0     input block loads for step q + 3
//   gap 1, 2  U loads for step q + 2
//   gap 3, 4  stage the block of step q + 1 in LDS
//   gap 5, 6  read this lane's window of it
//   gap 8-15  V = B^T d B of step q + 1, two packed operations per gap
// (Four bursts after every fourth MFMA ran 12-14 % slower: the MFMA pipe idled while the
// burst issued.)  Loads run 3 steps ahead for the input block, 2 for U; near the end of
// a tile they fetch the next tile's first steps (XN / UN), so its operands arrive during
// this tile's epilogue.
template <class GE, int K, bool FIRST, bool XN, bool UN>
__device__ __forceinline__ void wr_step(const WrGeom& g, const WrSrc& cur, const WrSrc& nxt,
                                        __amdgpu_buffer_rsrc_t urs, int lane, float* xw,
                                        const WxLane& xl, int q, WrRing& r, f32x16 (&acc)[16]) {
    const WrU& u = r.us[K];
    const float(&vc)[16] = r.v[K & 1];
    float(&vn)[16] = r.v[(K + 1) & 1];
    WinRow d[4], t[4];
    const WrX& xb = r.xs[(K + 1) % 4];  // block of step q + 1
#define WR_MFMA(xi)                                                                          \
    acc[xi] = __builtin_amdgcn_mfma_f32_32x32x2f32(u.u[(xi) >> 2][(xi) & 3], vc[xi],         \
                                                   FIRST ? f32x16{} : acc[xi], 0, 0, 0);     \
    __builtin_amdgcn_sched_barrier(0)
#define WR_WALL                                \
    asm volatile("" ::: "memory");             \
    __builtin_amdgcn_sched_barrier(0)
    WR_MFMA(0);
#if SP_WINO_EXP != 1
    wr_load_x<GE>(XN ? nxt : cur, (XN ? q + 3 - g.nsteps : q + 3) * g.so_step, r.xs[(K + 3) % 4]);
#endif
    WR_WALL;
    WR_MFMA(1);
    const int uso = (UN ? nxt.uso : cur.uso) + (UN ? q + 2 - g.nsteps : q + 2) * g.u_step * 4;
    WrU& un = r.us[(K + 2) % 4];
#if SP_WINO_EXP != 1
    un.u[0] = wr_u4(urs, lane, uso, 0);
    un.u[1] = wr_u4(urs, lane, uso, 1);
#endif
    WR_WALL;
    WR_MFMA(2);
#if SP_WINO_EXP != 1
    un.u[2] = wr_u4(urs, lane, uso, 2);
    un.u[3] = wr_u4(urs, lane, uso, 3);
#endif
    WR_WALL;
    WR_MFMA(3);
#pragma unroll
    for (int i = 0; i < 4; ++i) xw[xl.wa + i] = xb.a[i];
    WR_WALL;
    WR_MFMA(4);
#pragma unroll
    for (int i = 0; i < 4; ++i) xw[xl.wb + i] = xb.b[i];
    xw[xl.wh] = xb.h;
    WR_WALL;
    WR_MFMA(5);
    d[0] = wr_window_row<GE>(xw, xl, 0);
    d[1] = wr_window_row<GE>(xw, xl, 1);
    WR_WALL;
    WR_MFMA(6);
    d[2] = wr_window_row<GE>(xw, xl, 2);
    d[3] = wr_window_row<GE>(xw, xl, 3);
    WR_WALL;
#if SP_WINO_BURST == 0
    WR_MFMA(7);
    WR_MFMA(8);
    // t = B^T d, one row (two packed adds) per gap
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        t[k] = wpk_t(k, d);
        WR_WALL;
        WR_MFMA(9 + k);
    }
    // v = t B, one row per gap
#pragma unroll
    for (int rr = 0; rr < 3; ++rr) {
        wpk_v(t[rr], vn + 4 * rr);
        WR_WALL;
        WR_MFMA(13 + rr);
    }
    wpk_v(t[3], vn + 12);
#elif SP_WINO_BURST == 1
    // the whole transform as one burst: beside fp32 MFMAs the first VALU instruction of a gap
    // costs ~14 cycles and each further one ~4-5 (tools/mfma_gap.hip), so one burst of 16
    // packed adds costs about a third of 16 gaps with one each
    WR_MFMA(7);
    WR_MFMA(8);
    WR_MFMA(9);
    WR_MFMA(10);
    WR_MFMA(11);
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = wpk_t(k, d);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) wpk_v(t[rr], vn + 4 * rr);
    WR_WALL;
    WR_MFMA(12);
    WR_MFMA(13);
    WR_MFMA(14);
    WR_MFMA(15);
#else
    // two bursts: t = B^T d after MFMA 9, v = t B after MFMA 13
    WR_MFMA(7);
    WR_MFMA(8);
    WR_MFMA(9);
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = wpk_t(k, d);
    WR_WALL;
    WR_MFMA(10);
    WR_MFMA(11);
    WR_MFMA(12);
    WR_MFMA(13);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) wpk_v(t[rr], vn + 4 * rr);
    WR_WALL;
    WR_MFMA(14);
    WR_MFMA(15);
#endif
#if SP_WINO_EXP == 3
#pragma unroll
    for (int i = 0; i < 4; ++i)  // diagnostics: no input transform
        vn[4 * i] = d[i].p.x, vn[4 * i + 1] = d[i].p.y, vn[4 * i + 2] = d[i].q.x, vn[4 * i + 3] = d[i].q.y;
#endif
    WR_WALL;
#undef WR_MFMA
#undef WR_WALL
}

// Y = A^T M A, A^T = [[1,1,1,0],[0,1,-1,-1]], per (channel, tile) in registers: register r
// of every accumulator is channel co0 + (r&3) + 8(r>>2) + 4hh, tile l.  Buffer stores:
// one per-lane offset, the register row's channel offset as a scalar.
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

template <class GE>
__device__ __forceinline__ int wr_out_voff(const WrGeom& g, const WrTile& ti, int wv, int lane) {
    const int hh = lane >> 5, l = lane & 31;
    if constexpr (GE::MOSAIC) {
        const int tr = l / GE::TCW, tc = l % GE::TCW;
        return ((tc >> 2) * g.cout * g.plane + (ti.co0 + 4 * hh) * g.plane + 2 * tr * g.W +
                2 * (tc & 3)) * 4;
    }
    const int tr = GE::TRW * (wv >> 1) + l / GE::TCW, tc = l % GE::TCW;
    return ((ti.co0 + 4 * hh) * g.plane + (ti.oh0 + 2 * tr) * g.W + ti.ow0 + 2 * tc) * 4;
}

// The residual this lane adds to its 2x2 outputs of the tile (RES): loaded before the
// tile's last k-steps so the loads land while the MFMAs finish.
struct WrRes { f32x2 v[16][2]; };

template <class GE>
__device__ __forceinline__ void wr_load_res(const WrGeom& g, const WrTile& ti, int wv, int lane,
                                            WrRes& rv) {
    const auto rrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(g.res) + wr_img0<GE>(g, ti, wv) * g.cout * g.plane, (short)0,
        wr_nimg<GE>(g, ti, wv) * g.cout * g.plane * 4, 0x00020000);
    const int vo = wr_out_voff<GE>(g, ti, wv, lane);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int so = ((r & 3) + 8 * (r >> 2)) * g.plane * 4;
        rv.v[r][0] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rrs, vo, so, 0));
        rv.v[r][1] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rrs, vo, so + g.W * 4, 0));
    }
}

template <class GE, bool RES>
__device__ __forceinline__ void wr_epilogue(const WrGeom& g, const WrTile& ti, int wv, int lane,
                                            const f32x16 (&acc)[16], const WrRes& rv) {
    static_assert(!(GE::SPLIT && RES), "split-K parts add no residual (the reduce does)");
    const int hh = lane >> 5, l = lane & 31;
    // SPLIT: part kh's slice of the workspace, laid out like the output
    float* const obase = GE::SPLIT ? g.ws + (int64_t)ti.kh * g.ws_stride : g.out;
    const auto ors = __builtin_amdgcn_make_buffer_rsrc(
        obase + wr_img0<GE>(g, ti, wv) * g.cout * g.plane, (short)0,
        wr_nimg<GE>(g, ti, wv) * g.cout * g.plane * 4, 0x00020000);
    const int vo = wr_out_voff<GE>(g, ti, wv, lane);
    // the lane's last output row (channel co0 + 27 + 4 hh, second image row) inside the images
    SP_DCHECK(wr_nimg<GE>(g, ti, wv) == 0 || GE::MOSAIC ||
              (int64_t)vo + (27 * (int64_t)g.plane + g.W) * 4 + 8 <= (int64_t)wr_nimg<GE>(g, ti, wv) * g.cout * g.plane * 4);
    // bias[co0 + (lane & 31)] in one register, each row's two values (channels c and c + 4)
    // read out with v_readlane; no bias: a zero-length buffer, whose loads return 0.
    // (Sixteen vector bias registers here get hoisted and spilled while the next tile's
    // operands are live.)
    const auto brs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(g.bias ? g.bias : g.up), (short)0,
        g.bias && !GE::SPLIT ? g.cout * 4 : 0, 0x00020000);  // SPLIT: the reduce adds it
    const float bl = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(brs, (ti.co0 + l) * 4, 0, 0));
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        float s0[4], s1[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const float m0 = acc[a * 4 + 0][r], m1 = acc[a * 4 + 1][r];
            const float m2 = acc[a * 4 + 2][r], m3 = acc[a * 4 + 3][r];
            s0[a] = m0 + m1 + m2;
            s1[a] = m1 - m2 - m3;
        }
        const int c = (r & 3) + 8 * (r >> 2);  // channel co0 + c + 4 hh
        const float b0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, bl), c));
        const float b1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, bl), c + 4));
        const float bv = hh ? b1 : b0;
        const int so = c * g.plane * 4;
#if SP_WINO_EXP == 2
        if (g.W >= 0) continue;  // never true at run time: the stores are skipped, all math kept
#endif
        f32x2 y0 = {s0[0] + s0[1] + s0[2] + bv, s1[0] + s1[1] + s1[2] + bv};
        f32x2 y1 = {s0[1] - s0[2] - s0[3] + bv, s1[1] - s1[2] - s1[3] + bv};
        if constexpr (RES) y0 += rv.v[r][0], y1 += rv.v[r][1];
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y0), ors, vo, so, 0);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y1), ors, vo, so + g.W * 4, 0);
        // one register row at a time: the next tile's operands are live across the
        // epilogue, so its accumulator reads must not all be hoisted
        __builtin_amdgcn_sched_barrier(0);
    }
}

// Persistent: one workgroup per CU walks tiles t = blockIdx.x, + gridDim.x, ...; the load
// ring runs on across tile boundaries, so a tile's prologue latency and its predecessor's
// store drain overlap MFMA work instead of leaving the CU idle (at one wave per SIMD no
// other workgroup can fill those gaps).
template <bool RES, int TCW, bool MOSAIC = false, bool SPLIT = false>
__global__ __launch_bounds__(kBlock, 1) void k_wino3x3_r(WrGeom g) {
    using GE = WGeo<TCW, MOSAIC, SPLIT>;
    __shared__ __attribute__((aligned(16))) float xlds[4 * GE::WAVE];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    float* const xw = xlds + wv * GE::WAVE;
    WxLane xl;
    {
        auto loff = [](int rc) { return (rc / GE::ROWS) * GE::CI + GE::row(rc % GE::ROWS); };
        const int ka = lane % GE::PPR, rca = lane / GE::PPR, rcb = 64 / GE::PPR + ((lane / GE::PPR) & 3);
        const int rch = (lane % (2 * GE::RC)) >> 1, side = lane & 1;
        const int l = lane & 31;
        if constexpr (GE::MOSAIC) {
            // image 1's columns one position later: cols 0..7 at 4..11 / 13..20; positions
            // 3, 12, 21 hold the zero padding (12 is rewritten with the halo loads' zeros)
            xl.wa = loff(rca) + 4 + 4 * ka + (ka >= 2);
            xl.wb = loff(rcb) + 4 + 4 * ka + (ka >= 2);
            xl.wh = loff(rch) + 12;
            const int tc = l % GE::TCW;
            xl.rd = (lane >> 5) * GE::CI + GE::row(2 * (l / GE::TCW)) + 3 + 2 * tc + (tc >= 4);
            for (int i = lane; i < GE::WAVE; i += 64) xw[i] = 0.f;
        } else {
            xl.wa = loff(rca) + 4 + 4 * ka;
            xl.wb = loff(rcb) + 4 + 4 * ka;
            xl.wh = loff(rch) + (side ? 4 + 2 * GE::TCW : 3);
            xl.rd = (lane >> 5) * GE::CI + GE::row(2 * (l / GE::TCW)) + 3 + 2 * (l % GE::TCW);
        }
    }
    // all of packed U: (cin / 2) k-steps of u_step floats
    const auto urs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.up), (short)0,
                                                       g.nsteps * g.ksplit * static_cast<int>(g.u_step) * 4,
                                                       0x00020000);
    int t = blockIdx.x;
    const int stride = gridDim.x;
    WrTile ti = wr_tile<GE>(g, t, wv);
    WrSrc cur = wr_src<GE>(g, ti, wv, lane);
    int tn = t + stride;
    WrTile tin = wr_tile<GE>(g, tn < g.ntiles ? tn : t, wv);  // no next tile: harmless re-loads
    WrSrc nxt = wr_src<GE>(g, tin, wv, lane);

    // prologue in the loop's own issue order (..., X(q+1), U(q), X(q+2), U(q+1))
    WrRing r;
    wr_load_x<GE>(cur, 0, r.xs[0]);
    __builtin_amdgcn_sched_barrier(0);
    wr_load_x<GE>(cur, g.so_step, r.xs[1]);
    __builtin_amdgcn_sched_barrier(0);
    wr_load_u(urs, lane, cur.uso, r.us[0]);
    __builtin_amdgcn_sched_barrier(0);
    wr_load_x<GE>(cur, 2 * g.so_step, r.xs[2]);
    __builtin_amdgcn_sched_barrier(0);
    wr_load_u(urs, lane, cur.uso + g.u_step * 4, r.us[1]);
    __builtin_amdgcn_sched_barrier(0);
    {
        wr_stage_x(xw, xl, r.xs[0]);
        WinRow d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = wr_window_row<GE>(xw, xl, k);
#pragma unroll
        for (int k = 0; k < 4; ++k) wpk_v(wpk_t(k, d), r.v[0] + 4 * k);
    }
    f32x16 acc[16];
    const int last = g.nsteps - 4;  // >= 4 (cin >= 16)
    for (;;) {
        wr_step<GE, 0, true, false, false>(g, cur, nxt, urs, lane, xw, xl, 0, r, acc);
        wr_step<GE, 1, false, false, false>(g, cur, nxt, urs, lane, xw, xl, 1, r, acc);
        wr_step<GE, 2, false, false, false>(g, cur, nxt, urs, lane, xw, xl, 2, r, acc);
        wr_step<GE, 3, false, false, false>(g, cur, nxt, urs, lane, xw, xl, 3, r, acc);
        for (int p = 4; p < last; p += 4) {
            wr_step<GE, 0, false, false, false>(g, cur, nxt, urs, lane, xw, xl, p + 0, r, acc);
            wr_step<GE, 1, false, false, false>(g, cur, nxt, urs, lane, xw, xl, p + 1, r, acc);
            wr_step<GE, 2, false, false, false>(g, cur, nxt, urs, lane, xw, xl, p + 2, r, acc);
            wr_step<GE, 3, false, false, false>(g, cur, nxt, urs, lane, xw, xl, p + 3, r, acc);
        }
        WrRes rv;
        if constexpr (RES) {
            wr_load_res<GE>(g, ti, wv, lane, rv);
            __builtin_amdgcn_sched_barrier(0);
        }
        // last four steps: the ring starts fetching the next tile's steps 0..2 / 0..1
        wr_step<GE, 0, false, false, false>(g, cur, nxt, urs, lane, xw, xl, last + 0, r, acc);
        wr_step<GE, 1, false, true, false>(g, cur, nxt, urs, lane, xw, xl, last + 1, r, acc);
        wr_step<GE, 2, false, true, true>(g, cur, nxt, urs, lane, xw, xl, last + 2, r, acc);
        wr_step<GE, 3, false, true, true>(g, cur, nxt, urs, lane, xw, xl, last + 3, r, acc);
        wr_epilogue<GE, RES>(g, ti, wv, lane, acc, rv);
        t = tn;
        if (t >= g.ntiles) break;
        ti = tin;
        cur = nxt;
        tn = t + stride;
        tin = wr_tile<GE>(g, tn < g.ntiles ? tn : t, wv);
        nxt = wr_src<GE>(g, tin, wv, lane);
    }
}

// ---------------------------------------------------------------------------------------
// ξ-split tile (SP_WINO_XI, the W % 32 geometry): the two waves of a tile-row pair split the
// 16 transformed GEMMs by ξ instead of by output channel.  Wave H holds ξ 8H .. 8H + 7 for all
// 64 channels of the workgroup (8 ξ x 2 channel blocks x 16 accumulator registers = the same
// 256 AGPRs), so per k-step it transforms only its half of V (ξ rows 2H, 2H + 1: 8 packed adds
// instead of 16, three window rows instead of four) and feeds each V value to two MFMAs.  No
// barrier in the k-loop: each wave stages the whole input block in its own LDS region as
// before.  The output transform needs all four ξ rows: once per tile the waves exchange the
// row sums of the channel block the other one finishes (16 KB per wave through LDS, two
// barriers), and each completes and stores one 32-channel block — in the same operation order
// as wr_epilogue, so results are bit-identical to k_wino3x3_r.
// ---------------------------------------------------------------------------------------
#ifndef SP_WINO_XI
#define SP_WINO_XI 1
#endif
// Load distances of the ξ-split tile (k-steps ahead of use): the input block DX, U DU.  The
// wave's vector loads complete in issue order (one vmcnt), so the wait for U(q) also waits for
// every block load issued before it: the two distances have to grow together, or the shorter
// one sets the effective depth of both.  Round 4 measured deeper rings (XI_NR = 8 slots, the
// k loop unrolled 8 steps) in the headline step (profiles/round4/wino/ring_depth_ab.txt):
// (DX, DU) = (3, 2) 220.1 samples/s, (4, 4) 220.5, (5, 4) 219.8, (5, 5) 218.2, (6, 5) 219.4,
// (6, 6) 218.7, (7, 6) 218.2 — no gain: the k-steps do not wait on load latency (SQ_WAIT_ANY
// is 5 % of wave cycles; the MFMA pipe is busy 0.85 of the cycles at the clock the chip holds,
// profiles/round4/wino/sq_counters.txt).  The shallow ring keeps the registers.
#ifndef SP_WINO_XI16
#define SP_WINO_XI16 1  // the ξ-split tile on the W = 16 geometry too (the UNets' 16x16 levels)
#endif
#ifndef SP_WINO_DX
#define SP_WINO_DX 3
#endif
#ifndef SP_WINO_DU
#define SP_WINO_DU 2
#endif
constexpr int XI_DX = SP_WINO_DX, XI_DU = SP_WINO_DU;
constexpr int XI_NR = (XI_DX > 3 || XI_DU > 3) ? 8 : 4;  // ring slots = unroll of the k loop
static_assert(XI_DX >= 2 && XI_DX < XI_NR && XI_DU >= 1 && XI_DU < XI_NR, "ring distances");

struct XiRing {
    WrX xs[XI_NR];
    WrU us[XI_NR];   // u[2 cb + j]: channel block cb, ξ 8H + 4j .. + 3
    float v[2][8];   // this wave's half of V (slot i = ξ 8H + i) for the current / next step
};

constexpr int XI_EX = 16 * 64 * 4;  // floats per wave of the epilogue exchange

template <int H>
__device__ __forceinline__ void xi_load_u(__amdgpu_buffer_rsrc_t urs, int lane, int soff, WrU& u) {
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
        for (int j = 0; j < 2; ++j)
            u.u[2 * cb + j] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(urs, lane * 64 + 32 * H + 16 * j,
                                                             soff + cb * 64 * 64, 0));
}

// this wave's half of V from window rows e0, e1, e2 (= rows H .. H + 2 of the window)
template <int H>
__device__ __forceinline__ void xi_half(const WinRow& e0, const WinRow& e1, const WinRow& e2, float* vn) {
    const WinRow f{pk_sub(e0.p, e2.p), pk_sub(e0.q, e2.q)};
    if constexpr (H == 0) {  // ξ row 0 = t0 = d0 - d2, row 1 = t1 = d1 + d2
        wpk_v(f, vn);
        wpk_v(WinRow{pk_add(e1.p, e2.p), pk_add(e1.q, e2.q)}, vn + 4);
    } else {                 // ξ row 2 = t2 = d2 - d1, row 3 = t3 = d1 - d3
        wpk_v(WinRow{pk_sub(e1.p, e0.p), pk_sub(e1.q, e0.q)}, vn);
        wpk_v(f, vn + 4);
    }
}

// One k-step q (ring slot K = q mod XI_NR): MFMAs on U(q) and V(q); beside them the loads of
// the block of step q + DX and of U(q + DU) (XN / UN: those steps belong to the next tile), the
// block of step q + 1 staged in LDS, its window read and half of V(q + 1) transformed.
template <class GE, int H, int K, bool FIRST, bool XN, bool UN>
__device__ __forceinline__ void xi_step(const WrGeom& g, const WrSrc& cur, const WrSrc& nxt,
                                        __amdgpu_buffer_rsrc_t urs, int lane, float* xw,
                                        const WxLane& xl, int q, XiRing& r, f32x16 (&acc)[16]) {
    // (GE: the W % 32 geometry or the W = 16 one)
    // q as an opaque scalar: the step's load offsets are computed here from it (two scalar
    // multiply-adds), not hoisted out of the unrolled loop as XI_NR sets of live SGPRs (spills)
    asm volatile("" : "+s"(q));
    const WrU& u = r.us[K];
    const float(&vc)[8] = r.v[K & 1];
    float(&vn)[8] = r.v[(K + 1) & 1];
    WinRow e[3];
    const WrX& xb = r.xs[(K + 1) % XI_NR];  // block of step q + 1
#define XI_MFMA(sl)                                                                               \
    acc[sl] = __builtin_amdgcn_mfma_f32_32x32x2f32(u.u[2 * ((sl) >> 3) + (((sl) & 7) >> 2)][(sl) & 3], \
                                                   vc[(sl) & 7], FIRST ? f32x16{} : acc[sl], 0, 0, 0); \
    __builtin_amdgcn_sched_barrier(0)
#define XI_WALL                                \
    asm volatile("" ::: "memory");             \
    __builtin_amdgcn_sched_barrier(0)
    XI_MFMA(0);
#if SP_WINO_EXP != 1
    wr_load_x<GE>(XN ? nxt : cur, (XN ? q + XI_DX - g.nsteps : q + XI_DX) * g.so_step, r.xs[(K + XI_DX) % XI_NR]);
#endif
    XI_WALL;
    XI_MFMA(1);
    const int uso = (UN ? nxt.uso : cur.uso) + (UN ? q + XI_DU - g.nsteps : q + XI_DU) * g.u_step * 4;
    WrU& un = r.us[(K + XI_DU) % XI_NR];
#if SP_WINO_EXP != 1
    un.u[0] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(urs, lane * 64 + 32 * H, uso, 0));
    un.u[1] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(urs, lane * 64 + 32 * H + 16, uso, 0));
#endif
    XI_WALL;
    XI_MFMA(2);
#if SP_WINO_EXP != 1
    un.u[2] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(urs, lane * 64 + 32 * H, uso + 64 * 64, 0));
    un.u[3] = __builtin_bit_cast(f32x4,
                                 __builtin_amdgcn_raw_buffer_load_b128(urs, lane * 64 + 32 * H + 16, uso + 64 * 64, 0));
#endif
    XI_WALL;
    XI_MFMA(3);
#pragma unroll
    for (int i = 0; i < 4; ++i) xw[xl.wa + i] = xb.a[i];
    XI_WALL;
    XI_MFMA(4);
#pragma unroll
    for (int i = 0; i < 4; ++i) xw[xl.wb + i] = xb.b[i];
    xw[xl.wh] = xb.h;
    XI_WALL;
    XI_MFMA(5);
    e[0] = wr_window_row<GE>(xw, xl, H + 0);
    e[1] = wr_window_row<GE>(xw, xl, H + 1);
    XI_WALL;
    XI_MFMA(6);
    e[2] = wr_window_row<GE>(xw, xl, H + 2);
    XI_WALL;
    XI_MFMA(7);
    XI_MFMA(8);
    XI_MFMA(9);
    XI_MFMA(10);
    XI_MFMA(11);
    xi_half<H>(e[0], e[1], e[2], vn);
    XI_WALL;
    XI_MFMA(12);
    XI_MFMA(13);
    XI_MFMA(14);
    XI_MFMA(15);
    XI_WALL;
#undef XI_MFMA
#undef XI_WALL
}

// k-steps p + K0 + K for K in the sequence (p % XI_NR == 0).  LAST: the tile's final XI_NR
// steps, whose loads beyond the tile's last step fetch the next tile's first steps.
template <class GE, int H, bool FIRST, bool LAST, int K0, int... K>
__device__ __forceinline__ void xi_steps(std::integer_sequence<int, K...>, const WrGeom& g, const WrSrc& cur,
                                         const WrSrc& nxt, __amdgpu_buffer_rsrc_t urs, int lane, float* xw,
                                         const WxLane& xl, int p, XiRing& r, f32x16 (&acc)[16]) {
    (xi_step<GE, H, K0 + K, FIRST && K0 + K == 0, LAST && (K0 + K + XI_DX >= XI_NR),
             LAST && (K0 + K + XI_DU >= XI_NR)>(g, cur, nxt, urs, lane, xw, xl, p + K0 + K, r, acc),
     ...);
}

// Epilogue: row sums of this wave's ξ rows for both channel blocks; the block the partner
// completes goes through LDS, the partner's rows of this wave's block come back; then the
// output transform, bias, residual and stores as wr_epilogue (same order of operations).
template <class GE, int H, bool RES>
__device__ __forceinline__ void xi_epilogue(const WrGeom& g, const WrTile& ti, int wv, int lane,
                                            const f32x16 (&acc)[16], const WrRes& rv, float* ex) {

    float* mine = ex + H * XI_EX;          // written by this wave (the partner's block)
    const float* theirs = ex + (1 - H) * XI_EX;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
        float o[4];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const int b = (1 - H) * 8 + a * 4;  // the partner's channel block, ξ row 2H + a
            o[a] = acc[b + 0][rr] + acc[b + 1][rr] + acc[b + 2][rr];
            o[2 + a] = acc[b + 1][rr] - acc[b + 2][rr] - acc[b + 3][rr];
        }
        *reinterpret_cast<f32x4*>(mine + (rr * 64 + lane) * 4) = f32x4{o[0], o[1], o[2], o[3]};
        __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_barrier();
    WrTile tf = ti;
    tf.co0 = ti.co0 + 32 * H;  // this wave completes channel block H
    const int hh = lane >> 5, l = lane & 31;
    static_assert(!(GE::UP == 2 && RES), "the pooled input VJP adds no residual");
    const int pout = GE::UP == 2 ? g.hplane : g.plane;  // floats per output plane
    const auto ors = __builtin_amdgcn_make_buffer_rsrc(g.out + (int64_t)tf.n * g.cout * pout, (short)0,
                                                       g.cout * pout * 4, 0x00020000);
    int vo = wr_out_voff<GE>(g, tf, wv, lane);
    if constexpr (GE::UP == 2) {  // the lane's 2x2 block -> its half-resolution pixel
        const int tr = GE::TRW * (wv >> 1) + l / GE::TCW, tc = l % GE::TCW;
        vo = ((tf.co0 + 4 * hh) * g.hplane + (tf.oh0 / 2 + tr) * g.Wh + tf.ow0 / 2 + tc) * 4;
        SP_DCHECK(tf.n < g.batch && (int64_t)vo + 27 * (int64_t)g.hplane * 4 + 4 <= (int64_t)g.cout * g.hplane * 4);
    } else {
        SP_DCHECK(tf.n < g.batch && (int64_t)vo + (27 * (int64_t)g.plane + g.W) * 4 + 8 <= (int64_t)g.cout * g.plane * 4);
    }
    const auto brs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.bias ? g.bias : g.up), (short)0,
                                                       g.bias ? g.cout * 4 : 0, 0x00020000);
    const float bl = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(brs, (tf.co0 + l) * 4, 0, 0));
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
        const f32x4 p = *reinterpret_cast<const f32x4*>(theirs + (rr * 64 + lane) * 4);
        float s0[4], s1[4];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
            const int b = H * 8 + a * 4;  // this wave's rows of its own block: ξ row 2H + a
            s0[2 * H + a] = acc[b + 0][rr] + acc[b + 1][rr] + acc[b + 2][rr];
            s1[2 * H + a] = acc[b + 1][rr] - acc[b + 2][rr] - acc[b + 3][rr];
            s0[2 * (1 - H) + a] = p[a];
            s1[2 * (1 - H) + a] = p[2 + a];
        }
        const int c = (rr & 3) + 8 * (rr >> 2);
        const float b0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, bl), c));
        const float b1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, bl), c + 4));
        const float bv = hh ? b1 : b0;
        const int so = c * pout * 4;
        f32x2 y0 = {s0[0] + s0[1] + s0[2] + bv, s1[0] + s1[1] + s1[2] + bv};
        f32x2 y1 = {s0[1] - s0[2] - s0[3] + bv, s1[1] - s1[2] - s1[3] + bv};
        if constexpr (RES) y0 += rv.v[rr][0], y1 += rv.v[rr][1];
        if constexpr (GE::UP == 2) {  // k_upsample2x_vjp's order: ((row 0) + row 1, left first)
            const float p = ((y0.x + y0.y) + y1.x) + y1.y;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(p), ors, vo, so, 0);
        } else {
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y0), ors, vo, so, 0);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y1), ors, vo, so + g.W * 4, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // the partner's rows are read before it writes again
    __builtin_amdgcn_s_barrier();
}

template <class GE, bool RES, int H>
__device__ __forceinline__ void xi_body(const WrGeom& g, int wv, int lane, float* xw, float* ex) {

    const int wq = wv & ~1;  // tile geometry of channel half 0 (the pair covers all 64 channels)
    WxLane xl;
    {
        auto loff = [](int rc) { return (rc / GE::ROWS) * GE::CI + GE::row(rc % GE::ROWS); };
        const int ka = lane % GE::PPR, rca = lane / GE::PPR, rcb = 64 / GE::PPR + ((lane / GE::PPR) & 3);
        const int rch = (lane % (2 * GE::RC)) >> 1, side = lane & 1;
        const int l = lane & 31;
        xl.wa = loff(rca) + 4 + 4 * ka;
        xl.wb = loff(rcb) + 4 + 4 * ka;
        xl.wh = loff(rch) + (side ? 4 + 2 * GE::TCW : 3);
        xl.rd = (lane >> 5) * GE::CI + GE::row(2 * (l / GE::TCW)) + 3 + 2 * (l % GE::TCW);
    }
    const auto urs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.up), (short)0,
                                                       g.nsteps * static_cast<int>(g.u_step) * 4, 0x00020000);
    int t = blockIdx.x;
    const int stride = gridDim.x;
    WrTile ti = wr_tile<GE>(g, t, wq);
    WrSrc cur = wr_src<GE>(g, ti, wq, lane);
    int tn = t + stride;
    WrTile tin = wr_tile<GE>(g, tn < g.ntiles ? tn : t, wq);
    WrSrc nxt = wr_src<GE>(g, tin, wq, lane);

    // prologue in the loop's own issue order: X(s), U(s) for s = 0 .. (the first step's loads
    // are X(DX), U(DU))
    XiRing r;
    static_for<0, (XI_DX > XI_DU ? XI_DX : XI_DU)>([&](auto S) {
        constexpr int s = decltype(S)::value;
        if constexpr (s < XI_DX) wr_load_x<GE>(cur, s * g.so_step, r.xs[s]);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (s < XI_DU) xi_load_u<H>(urs, lane, cur.uso + s * static_cast<int>(g.u_step) * 4, r.us[s]);
        __builtin_amdgcn_sched_barrier(0);
    });
    {
        wr_stage_x(xw, xl, r.xs[0]);
        const WinRow e0 = wr_window_row<GE>(xw, xl, H + 0), e1 = wr_window_row<GE>(xw, xl, H + 1),
                     e2 = wr_window_row<GE>(xw, xl, H + 2);
        xi_half<H>(e0, e1, e2, r.v[0]);
    }
    f32x16 acc[16];
    const int last = g.nsteps - XI_NR;  // >= XI_NR, a multiple of XI_NR (wino3x3's dispatch rule)
    constexpr auto ring = std::make_integer_sequence<int, XI_NR>{};
    // the residual (RES: 64 registers per lane) is loaded two steps before the tile's end, so it
    // does not hold registers across the deep ring's whole last block
    constexpr int RES_AT = XI_NR - 2;
    for (;;) {
        xi_steps<GE, H, true, false, 0>(ring, g, cur, nxt, urs, lane, xw, xl, 0, r, acc);
        for (int p = XI_NR; p < last; p += XI_NR)
            xi_steps<GE, H, false, false, 0>(ring, g, cur, nxt, urs, lane, xw, xl, p, r, acc);
        WrRes rv;
        xi_steps<GE, H, false, true, 0>(std::make_integer_sequence<int, RES_AT>{}, g, cur, nxt, urs, lane, xw, xl,
                                    last, r, acc);
        if constexpr (RES) {
            WrTile tf = ti;
            tf.co0 = ti.co0 + 32 * H;
            wr_load_res<GE>(g, tf, wv, lane, rv);
            __builtin_amdgcn_sched_barrier(0);
        }
        xi_steps<GE, H, false, true, RES_AT>(std::make_integer_sequence<int, XI_NR - RES_AT>{}, g, cur, nxt, urs, lane,
                                         xw, xl, last, r, acc);
#if SP_WINO_EXP == 6
        if (g.W < 0)  // never true at run time: no epilogue (the MFMAs stay live)
#endif
        xi_epilogue<GE, H, RES>(g, ti, wv, lane, acc, rv, ex);
        t = tn;
        if (t >= g.ntiles) break;
        ti = tin;
        cur = nxt;
        tn = t + stride;
        tin = wr_tile<GE>(g, tn < g.ntiles ? tn : t, wq);
        nxt = wr_src<GE>(g, tin, wq, lane);
    }
}

template <bool RES, int TCW, int UP = 0>
__global__ __launch_bounds__(kBlock, 1) void k_wino3x3_xi(WrGeom g) {
    using GE = WGeo<TCW, false, false, UP>;
    __shared__ __attribute__((aligned(16))) float xlds[4 * GE::WAVE];
    __shared__ __attribute__((aligned(16))) float exlds[2 * 2 * XI_EX];  // [pair][writer][...]
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float* const xw = xlds + wv * GE::WAVE;
    float* const ex = exlds + (wv >> 1) * 2 * XI_EX;
    if (wv & 1) xi_body<GE, RES, 1>(g, wv, lane, xw, ex);
    else xi_body<GE, RES, 0>(g, wv, lane, xw, ex);
}

// Split-K reduce: out = (((ws_0 + ws_1) + ws_2) + ...) + bias[c] (+ res), four outputs per
// thread (plane % 4 == 0), the parts added in a fixed order (bitwise reproducible)
__global__ __launch_bounds__(kBlock) void k_wino_split_reduce(const float* __restrict__ ws, int ks,
                                                              int64_t stride4, int plane4, int cout,
                                                              const float* __restrict__ bias,
                                                              const float* __restrict__ res,
                                                              float* __restrict__ out) {
    const f32x4* w4 = reinterpret_cast<const f32x4*>(ws);
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < stride4; i += (int64_t)gridDim.x * kBlock) {
        f32x4 a = w4[i];
        for (int k = 1; k < ks; ++k) a += w4[(int64_t)k * stride4 + i];
        if (bias) a += bias[(i / plane4) % cout];
        if (res) a += reinterpret_cast<const f32x4*>(res)[i];
        reinterpret_cast<f32x4*>(out)[i] = a;
    }
}

// Pack for k_wino3x3_r (U = G g G^T per (co, ci), G = [[1,0,0],[.5,.5,.5],[.5,-.5,.5],[0,0,1]]): up[((kin / 2 * (cout_p / 32) + orow / 32) * 64 + lane) * 16 + xi],
// lane = 32 (kin & 1) + orow % 32.
__global__ void k_wino3x3_pack(const float* __restrict__ w, int cout, int cin, int flip,
                                 float* __restrict__ up) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (co, ci) of W
    if (i >= (int64_t)cout * cin) return;
    const int co = static_cast<int>(i / cin), ci = static_cast<int>(i - (int64_t)co * cin);
    float g[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) g[k] = flip ? w[i * 9 + (8 - k)] : w[i * 9 + k];
    const int orow = flip ? ci : co, kin = flip ? co : ci, cout_p = flip ? cin : cout;
    float u[16];
    wino_filter(g, u);
    float* dst = up + (((int64_t)(kin >> 1) * (cout_p >> 5) + (orow >> 5)) * 64 +
                       32 * (kin & 1) + (orow & 31)) * 16;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        reinterpret_cast<f32x4*>(dst)[q] = f32x4{u[q * 4 + 0], u[q * 4 + 1], u[q * 4 + 2], u[q * 4 + 3]};
}

}  // namespace sp

using namespace sp;

extern "C" {

int sp_wino3x3_supported(int32_t cin, int32_t cout, int32_t height, int32_t width) {
    // W % 32: 32-column workgroup tiles of 8 rows; W = 16 (UNet 16x16 level): 16 x 16
    const bool geo = (width % WGeo<16>::WG_COLS == 0 && height % WGeo<16>::WG_ROWS == 0) ||
                     (width == WGeo<8>::WG_COLS && height % WGeo<8>::WG_ROWS == 0) ||
                     (width == 8 && height == 8);  // MOSAIC
    return cin >= 16 && cout > 0 && cin % (2 * WR_NS) == 0 && cout % WR_CO == 0 && geo &&
           height > 0 && width > 0;
}

int64_t sp_wino3x3_packed_size(int32_t cin, int32_t cout) { return (int64_t)cin * cout * 16; }

int sp_wino3x3_pack(const float* w, int32_t cout, int32_t cin, int32_t input_vjp, float* up,
                    sp_stream_t stream) {
    if (!w || !up || cout <= 0 || cin <= 0) return SP_EINVAL;
    const int kin = input_vjp ? cout : cin, nout = input_vjp ? cin : cout;
    if (kin % 2 || nout % 32) return SP_EINVAL;
    const int64_t total = (int64_t)cout * cin;
    launch(0, k_wino3x3_pack, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256),
           static_cast<hipStream_t>(stream), w, cout, cin, input_vjp, up);
    return check_launch("sp_wino3x3_pack");
}

static int cu_count() {
    static int cached[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cached[dev]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            v <= 0)
            v = 256;
        cached[dev] = v;
    }
    return cached[dev];
}

// Split-K parts for a launch of `tiles` tiles over cin input channels: doubled while the
// doubled count still fits one persistent wave of workgroups and every part keeps at least two
// rings of k-steps (k_wino3x3_r's first and last blocks)
static int wino_ksplit(int64_t tiles, int32_t cin) {
    const int nst = cin / 2;
    int ks = 1;
    while (ks * 2 <= SP_WINO_SPLITK && tiles * ks * 2 <= cu_count() && nst % (ks * 2 * WR_NS) == 0 &&
           nst / (ks * 2) >= 2 * WR_NS)
        ks *= 2;
    return ks;
}

static int64_t wino_tiles(int64_t n, int32_t cout, int32_t height, int32_t width) {
    const bool mosaic = width == 8;
    const bool narrow = !mosaic && width % WGeo<16>::WG_COLS != 0;
    const int wg_rows = narrow ? WGeo<8>::WG_ROWS : WGeo<16>::WG_ROWS;
    const int wg_cols = narrow ? WGeo<8>::WG_COLS : WGeo<16>::WG_COLS;
    return mosaic ? (n + 3) / 4 * (cout / WR_CO) : n * (height / wg_rows) * (width / wg_cols) * (cout / WR_CO);
}

// the xi tile serves the launch (W % 32 geometry, K a multiple of its ring)
static bool wino_xi(int32_t cin, int32_t height, int32_t width) {
    return SP_WINO_XI && width % WGeo<16>::WG_COLS == 0 && height % WGeo<16>::WG_ROWS == 0 &&
           cin % (2 * XI_NR) == 0 && cin >= 4 * XI_NR;
}

// up_mode (Upsample2D fused, height x width the conv's = the upsampled size): 1 = x is the
// half-resolution source, 2 = y is the half-resolution 2x2-block sum; the xi tile, unsplit.
static int wino3x3(int kind, const float* x, const float* up, const float* bias,
                   const float* res, int64_t n, int32_t cin, int32_t cout, int32_t height,
                   int32_t width, float* y, float* ws, size_t ws_bytes, sp_stream_t stream,
                   const char* what, int up_mode = 0) {
    if (!sp_wino3x3_supported(cin, cout, height, width) || n < 0) return SP_EINVAL;
    if (up_mode && (!wino_xi(cin, height, width) || res)) return SP_EINVAL;
    if (n == 0) return SP_OK;
    if (!x || !up || !y) return SP_EINVAL;
    const bool mosaic = width == 8;                     // 8x8 images, 4 per workgroup
    const bool narrow = !mosaic && width % WGeo<16>::WG_COLS != 0;  // the W = 16 geometry
    const int wg_rows = narrow ? WGeo<8>::WG_ROWS : WGeo<16>::WG_ROWS;
    const int wg_cols = narrow ? WGeo<8>::WG_COLS : WGeo<16>::WG_COLS;
    const int64_t tiles = wino_tiles(n, cout, height, width);
    // per-sample planes are addressed by 32-bit buffer offsets (bytes < 2^31)
    if (tiles >= (int64_t(1) << 31) || (int64_t)cin * height * width * 4 >= (int64_t(1) << 31) ||
        (int64_t)cout * height * width * 4 >= (int64_t(1) << 31))
        return SP_EINVAL;
    // split K where the tiles leave CUs idle (small batches, the low-resolution levels), when
    // the caller's workspace holds every part's partial output
    const int64_t out_floats = n * cout * (int64_t)height * width;
    int ksplit = ws && !up_mode ? wino_ksplit(tiles, cin) : 1;
    if (ksplit > 1 && ws_bytes < (size_t)ksplit * out_floats * sizeof(float)) ksplit = 1;
    if (tiles * ksplit >= (int64_t(1) << 31)) ksplit = 1;
    WrGeom g;
    g.x = x;
    g.up = up;
    g.out = y;
    g.bias = bias;
    g.res = res;
    g.cin = cin;
    g.cout = cout;
    g.H = height;
    g.W = width;
    g.plane = height * width;
    g.ntiles = static_cast<int>(tiles * ksplit);
    g.ksplit = ksplit;
    g.ws = ksplit > 1 ? ws : nullptr;
    g.ws_stride = out_floats;
    g.cob = cout / WR_CO;
    g.tiles_w = mosaic ? 1 : width / wg_cols;
    g.per_img = mosaic ? 1 : g.tiles_w * (height / wg_rows);
    g.batch = n;
    g.u_step = (int64_t)cout * 32;
    g.hplane = (height / 2) * (width / 2);
    g.Wh = width / 2;
    g.so_step = 2 * (up_mode == 1 ? g.hplane : height * width) * 4;
    g.nsteps = cin / 2 / ksplit;
    // one persistent workgroup per CU (a 512-register wave per SIMD: one workgroup fits)
    const int grid = static_cast<int>(std::min<int64_t>(tiles * ksplit, cu_count()));
    // executed MFMA work: 16 GEMMs of 2*cin*cout per 2x2 tile = 8*cin*cout per pixel
    // (the direct-conv equivalent is 18*cin*cout per pixel, 2.25x more)
    const double flops = 8.0 * n * cin * cout * height * width;
    const dim3 gd(static_cast<unsigned>(grid)), bd(kBlock);
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (up_mode == 1) {
        launch_w(kind, flops, k_wino3x3_xi<false, 16, 1>, gd, bd, st, g);
        return check_launch(what);
    }
    if (up_mode == 2) {
        launch_w(kind, flops, k_wino3x3_xi<false, 16, 2>, gd, bd, st, g);
        return check_launch(what);
    }
    if (ksplit > 1) {
        if (mosaic) launch_w(kind, flops, k_wino3x3_r<false, 8, true, true>, gd, bd, st, g);
        else if (narrow) launch_w(kind, flops, k_wino3x3_r<false, 8, false, true>, gd, bd, st, g);
        else launch_w(kind, flops, k_wino3x3_r<false, 16, false, true>, gd, bd, st, g);
        // the parts' sum + bias + residual (plane % 4 == 0 on every supported geometry)
        const int64_t v4 = out_floats / 4;
        const unsigned rb = static_cast<unsigned>(std::min<int64_t>((v4 + kBlock - 1) / kBlock, 4 * cu_count()));
        launch(0, k_wino_split_reduce, dim3(rb), dim3(kBlock), st, static_cast<const float*>(ws), ksplit, v4,
               height * width / 4, cout, bias, res, y);
    } else if (mosaic) {
        if (res) launch_w(kind, flops, k_wino3x3_r<true, 8, true>, gd, bd, st, g);
        else launch_w(kind, flops, k_wino3x3_r<false, 8, true>, gd, bd, st, g);
    } else if (narrow) {
#if SP_WINO_XI16
        if (SP_WINO_XI && cin % (2 * XI_NR) == 0 && cin >= 4 * XI_NR) {  // the ξ-split tile, W = 16
            if (res) launch_w(kind, flops, k_wino3x3_xi<true, 8>, gd, bd, st, g);
            else launch_w(kind, flops, k_wino3x3_xi<false, 8>, gd, bd, st, g);
            return check_launch(what);
        }
#endif
        if (res) launch_w(kind, flops, k_wino3x3_r<true, 8>, gd, bd, st, g);
        else launch_w(kind, flops, k_wino3x3_r<false, 8>, gd, bd, st, g);
    } else if (SP_WINO_XI && cin % (2 * XI_NR) == 0 && cin >= 4 * XI_NR) {
        if (res) launch_w(kind, flops, k_wino3x3_xi<true, 16>, gd, bd, st, g);
        else launch_w(kind, flops, k_wino3x3_xi<false, 16>, gd, bd, st, g);
    } else {
        if (res) launch_w(kind, flops, k_wino3x3_r<true, 16>, gd, bd, st, g);
        else launch_w(kind, flops, k_wino3x3_r<false, 16>, gd, bd, st, g);
    }
    return check_launch(what);
}

int64_t sp_wino3x3_workspace(int64_t n, int32_t cin, int32_t cout, int32_t height, int32_t width) {
    if (!sp_wino3x3_supported(cin, cout, height, width) || n <= 0) return 0;
    const int ks = wino_ksplit(wino_tiles(n, cout, height, width), cin);
    return ks > 1 ? (int64_t)ks * n * cout * height * width * (int64_t)sizeof(float) : 0;
}

int sp_wino3x3_fwd(const float* x, const float* up, const float* bias, int64_t n, int32_t cin,
                   int32_t cout, int32_t height, int32_t width, float* y, sp_stream_t stream) {
    return wino3x3(TK_WINO3X3_FWD, x, up, bias, nullptr, n, cin, cout, height, width, y, nullptr, 0,
                   stream, "sp_wino3x3_fwd");
}

int sp_wino3x3_fwd_res(const float* x, const float* up, const float* bias, const float* res,
                       int64_t n, int32_t cin, int32_t cout, int32_t height, int32_t width,
                       float* y, sp_stream_t stream) {
    if (!res || res == y) return SP_EINVAL;
    return wino3x3(TK_WINO3X3_FWD, x, up, bias, res, n, cin, cout, height, width, y, nullptr, 0,
                   stream, "sp_wino3x3_fwd_res");
}

int sp_wino3x3_bwd_input(const float* dy, const float* up_vjp, int64_t n, int32_t cin,
                         int32_t cout, int32_t height, int32_t width, float* dx,
                         sp_stream_t stream) {
    return wino3x3(TK_WINO3X3_BWD_INPUT, dy, up_vjp, nullptr, nullptr, n, cout, cin, height,
                   width, dx, nullptr, 0, stream, "sp_wino3x3_bwd_input");
}

int sp_wino3x3_fwd_ws(const float* x, const float* up, const float* bias, const float* res,
                      int64_t n, int32_t cin, int32_t cout, int32_t height, int32_t width,
                      float* y, float* ws, int64_t ws_bytes, sp_stream_t stream) {
    if (res == y && res) return SP_EINVAL;
    if (ws && (ws == y || ws_bytes < 0)) return SP_EINVAL;
    return wino3x3(TK_WINO3X3_FWD, x, up, bias, res, n, cin, cout, height, width, y, ws,
                   static_cast<size_t>(ws_bytes > 0 ? ws_bytes : 0), stream, "sp_wino3x3_fwd_ws");
}

int sp_wino3x3_up_supported(int32_t cin, int32_t cout, int32_t height, int32_t width) {
    // forward (K = cin) and input VJP (K = cout) both on the xi tile, even upsampled sizes
    return sp_wino3x3_supported(cin, cout, height, width) && sp_wino3x3_supported(cout, cin, height, width) &&
           wino_xi(cin, height, width) && wino_xi(cout, height, width) && height % 2 == 0 && width % 2 == 0;
}

int sp_wino3x3_fwd_up(const float* x, const float* up, const float* bias, int64_t n, int32_t cin,
                      int32_t cout, int32_t height, int32_t width, float* y, sp_stream_t stream) {
    if (!sp_wino3x3_up_supported(cin, cout, height, width)) return SP_EINVAL;
    return wino3x3(TK_WINO3X3_FWD, x, up, bias, nullptr, n, cin, cout, height, width, y, nullptr, 0,
                   stream, "sp_wino3x3_fwd_up", 1);
}

int sp_wino3x3_bwd_input_pool(const float* dy, const float* up_vjp, int64_t n, int32_t cin,
                              int32_t cout, int32_t height, int32_t width, float* dx,
                              sp_stream_t stream) {
    if (!sp_wino3x3_up_supported(cin, cout, height, width)) return SP_EINVAL;
    return wino3x3(TK_WINO3X3_BWD_INPUT, dy, up_vjp, nullptr, nullptr, n, cout, cin, height, width, dx,
                   nullptr, 0, stream, "sp_wino3x3_bwd_input_pool", 2);
}

int sp_wino3x3_bwd_input_ws(const float* dy, const float* up_vjp, int64_t n, int32_t cin,
                            int32_t cout, int32_t height, int32_t width, float* dx, float* ws,
                            int64_t ws_bytes, sp_stream_t stream) {
    if (ws && (ws == dx || ws_bytes < 0)) return SP_EINVAL;
    return wino3x3(TK_WINO3X3_BWD_INPUT, dy, up_vjp, nullptr, nullptr, n, cout, cin, height,
                   width, dx, ws, static_cast<size_t>(ws_bytes > 0 ? ws_bytes : 0), stream,
                   "sp_wino3x3_bwd_input_ws");
}

}  // extern "C"

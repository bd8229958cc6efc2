// Winograd F(2x2, 3x3) convolution on fp32 MFMA: the same 3x3 / stride 1 / pad 1
// layers as sp_conv.hip (ResnetBlock / mid / up-sampling convolutions of the SD VAE
// and the DDPM UNet) with 2.25x fewer multiplies.
//
//   U = G g G^T   (4x4 per (co, ci); weights transformed + packed once per layer)
//   V = B^T d B   (4x4 per (ci, tile) from the 4x4 input window of a 2x2 output tile)
//   M_xi = sum_ci U_xi[co][ci] * V_xi[ci][tile]      16 GEMMs on v_mfma_f32_32x32x2_f32
//   Y = A^T M A   (2x2 outputs per (co, tile))
//
// Workgroup: 64 output channels x 32 tiles (4 x 32 output pixels of one image), 4 waves,
// wave r owning row r of the transformed 4x4 tile M (xi = 4r .. 4r+3) for all 64 co x 32
// tiles (128 fp32 per lane), so two workgroups fit a CU (48 KB LDS, <= 256 registers per
// lane) and one workgroup's transforms / LDS stores overlap the other's MFMAs.  The
// output transform is linear in M, so each wave applies A^T (.) A to its own row and the
// four shares are summed through LDS.  K walks the input channels 4 at a
// time: per chunk the workgroup writes U (16 xi x 4 ci x 64 co) and V (16 xi x 4 ci x 32
// tiles) to LDS (double-buffered: the next chunk's global loads are in flight during the
// MFMAs).  MFMA lane half h carries input channel 2kk + h.
//
// Numerics: exact fp32 MFMA accumulation of fp32 transforms; the transforms add the
// usual F(2,3) rounding (|coefficients| <= 1, one 0.5 factor), comparable to MIOpen's
// own Winograd f2x3 solver that these layers ran on before.

#include "sp_common.h"

namespace sp {

constexpr int WG_CO = 64;     // output channels per workgroup
constexpr int WG_TR = 2;      // tile rows per workgroup   (4 output rows)
constexpr int WG_TC = 16;     // tile columns per workgroup (32 output columns)
constexpr int WG_T = WG_TR * WG_TC;  // 32 tiles
constexpr int WG_CI = 4;      // input channels per K chunk
constexpr int WG_U = 16 * WG_CI * WG_CO;  // floats of U per chunk (4096)
constexpr int WG_V = 16 * WG_CI * WG_T;   // floats of V per chunk (2048)
constexpr int WG_NPAIR = WG_CI * WG_T;    // (ci, tile) transforms per chunk: 128 (threads < 128)
// (measured: 32 co x 64 tiles per workgroup, every thread transforming, was 10 % slower)

#ifndef SP_WINO_REG
#define SP_WINO_REG 1  // register-resident kernel (k_wino3x3_r); 0: LDS-staged k_wino3x3
#endif
#ifndef SP_WINO_HOIST
#define SP_WINO_HOIST 1  // read a chunk's MFMA operands from LDS before its MFMAs
#endif

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

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

// Global -> registers for chunk cc: packed U rows (float4).
__device__ __forceinline__ void wg_load_u(const float* __restrict__ up, int cc, int cout, int co0,
                                          int tid, f32x4 (&ru)[WG_U / 4 / kBlock]) {
    // U chunk layout: [xi][ci_l][cout] rows of cout floats; this workgroup takes co0..+63
    const float* src = up + (int64_t)cc * 16 * WG_CI * cout + co0;
#pragma unroll
    for (int i = 0; i < WG_U / 4 / kBlock; ++i) {
        const int idx = tid + kBlock * i;          // float4 index in [xi*4+ci][16 float4]
        const int row = idx >> 4, c4 = idx & 15;
        ru[i] = *reinterpret_cast<const f32x4*>(src + (int64_t)row * cout + c4 * 4);
    }
}

// Global -> registers for chunk cc: this thread's 4x4 input window (threads < 128).
// Buffer loads: the chunk offset is a scalar (soffset), each lane's 16 pixel offsets are
// fixed per workgroup, and a pixel outside the image has an out-of-range offset, which
// the hardware returns as 0 (the padding) — no branches, no clamping.
struct WinWindow {  // a thread's 4x4 input window: byte offset of its corner + validity
    int base;         // ((ci_l * H + gr) * W + gc) * 4
    unsigned mask;    // bit r*4+c: pixel inside the image
};

__device__ __forceinline__ void wg_load_x(__amdgpu_buffer_rsrc_t rs, int cc, int64_t plane, int W,
                                          WinWindow win, int tid, float (&rd)[16]) {
    if (tid < WG_NPAIR) {  // waves 0, 1: pair = tid, ci = tid / 32 (in base), tile = tid % 32
        const int so = static_cast<int>((int64_t)cc * WG_CI * plane * 4);  // wave-uniform
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int off = ((win.mask >> (r * 4 + c)) & 1u) ? win.base + (r * W + c) * 4
                                                                 : 0x7FFFFFF0;  // OOB -> 0
                rd[r * 4 + c] =
                    __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, off, so, 0));
            }
    }
}

__device__ __forceinline__ void wg_store(float* Us, float* Vs, int tid,
                                         const f32x4 (&ru)[WG_U / 4 / kBlock],
                                         const float (&rd)[16]) {
#pragma unroll
    for (int i = 0; i < WG_U / 4 / kBlock; ++i)
        *reinterpret_cast<f32x4*>(&Us[(tid + kBlock * i) * 4]) = ru[i];
    if (tid < WG_NPAIR) {
        const int ci = tid >> 5, tile = tid & 31;
        float v[16];
        wino_in(rd, v);
#pragma unroll
        for (int xi = 0; xi < 16; ++xi) Vs[(xi * WG_CI + ci) * WG_T + tile] = v[xi];
    }
}

// LDS-visibility barrier that leaves global loads in flight.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
}

// One K chunk: MFMAs on buffer `buf`, stage chunk cc+1 (loaded before the previous
// barrier) into the other buffer, then issue the loads of chunk cc+2.
__device__ __forceinline__ void wg_chunk(float* Us0, float* Vs0, int buf, int cc, int nchunks,
                                         const float* __restrict__ up, int cout, int co0,
                                         int64_t plane, int W, __amdgpu_buffer_rsrc_t rs,
                                         WinWindow win, int tid, int xr, int hh,
                                         int l, f32x4 (&ru)[WG_U / 4 / kBlock], float (&rnext)[16],
                                         f32x16 (&acc)[4][2]) {
    const bool more = cc + 1 < nchunks;
    // wave xr owns row xr of M: xi = 4 xr + j, both 32-channel halves (one B read feeds
    // two MFMAs: 1.5 LDS reads per MFMA)
    const float* Ub = Us0 + buf * WG_U + (4 * xr * WG_CI + hh) * WG_CO + l;
    const float* Vb = Vs0 + buf * WG_V + (4 * xr * WG_CI + hh) * WG_T + l;
#if SP_WINO_HOIST == 0
#pragma unroll
    for (int kk = 0; kk < WG_CI / 2; ++kk)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float a0 = Ub[(j * WG_CI + 2 * kk) * WG_CO];
            const float a1 = Ub[(j * WG_CI + 2 * kk) * WG_CO + 32];
            const float b = Vb[(j * WG_CI + 2 * kk) * WG_T];
            acc[j][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b, acc[j][0], 0, 0, 0);
            acc[j][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b, acc[j][1], 0, 0, 0);
        }
#else
    // all 24 operands of the chunk are read up front: the LDS latency of the second
    // half (kk = 1) hides under the first half's eight MFMAs instead of stalling each pair
    float a[WG_CI / 2][4][2], b[WG_CI / 2][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int kk = 0; kk < WG_CI / 2; ++kk) b[kk][j] = Vb[(j * WG_CI + 2 * kk) * WG_T];
#pragma unroll
    for (int kk = 0; kk < WG_CI / 2; ++kk)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            a[kk][j][0] = Ub[(j * WG_CI + 2 * kk) * WG_CO];
            a[kk][j][1] = Ub[(j * WG_CI + 2 * kk) * WG_CO + 32];
        }
    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the MFMAs
#pragma unroll
    for (int kk = 0; kk < WG_CI / 2; ++kk)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            acc[j][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk][j][0], b[kk][j], acc[j][0], 0, 0, 0);
            acc[j][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk][j][1], b[kk][j], acc[j][1], 0, 0, 0);
        }
#endif
    if (more) {
        wg_store(Us0 + (buf ^ 1) * WG_U, Vs0 + (buf ^ 1) * WG_V, tid, ru, rnext);
        if (cc + 2 < nchunks) {
            wg_load_u(up, cc + 2, cout, co0, tid, ru);
            wg_load_x(rs, cc + 2, plane, W, win, tid, rnext);
        }
    }
    lds_barrier();
}

// One wave's share of the output transform: MODE 0 writes it to LDS, 1 adds the LDS value
// and writes back, 2 adds the LDS value and the bias and stores the 2x2 outputs.
template <int MODE>
__device__ __forceinline__ void wg_share(const f32x16 (&acc)[4][2], float c0, float c1, int hh,
                                         int tile, float* ex, const float* __restrict__ bias,
                                         float* __restrict__ on, int co0, int64_t plane,
                                         int64_t pix = 0, int W = 0) {
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const float u0 = acc[0][m][r] + acc[1][m][r] + acc[2][m][r];
            const float u1 = acc[1][m][r] - acc[2][m][r] - acc[3][m][r];
            f32x4 y = {c0 * u0, c0 * u1, c1 * u0, c1 * u1};
            const int col = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * hh;
            f32x4* e = reinterpret_cast<f32x4*>(&ex[(col * WG_T + tile) * 4]);
            if (MODE > 0) y += *e;
            if (MODE < 2) {
                *e = y;
            } else {
                const float bv = bias ? bias[co0 + col] : 0.f;
                float* dst = on + (int64_t)(co0 + col) * plane + pix;
                *reinterpret_cast<float2*>(dst) = make_float2(y[0] + bv, y[1] + bv);
                *reinterpret_cast<float2*>(dst + W) = make_float2(y[2] + bv, y[3] + bv);
            }
        }
}

__global__ __launch_bounds__(kBlock, 2) void k_wino3x3(const float* __restrict__ x,
                                                       const float* __restrict__ up,
                                                       const float* __restrict__ bias,
                                                       float* __restrict__ out, int cin, int cout,
                                                       int H, int W) {
    // one array: U double buffer, then V double buffer; the epilogue reuses U's space
    __shared__ __attribute__((aligned(16))) float lds[2 * WG_U + 2 * WG_V];
    float* const Us0 = lds;
    float* const Vs0 = lds + 2 * WG_U;

    const int tiles_w = W / (2 * WG_TC), per_img = tiles_w * (H / (2 * WG_TR));
    const int n = blockIdx.x / per_img, t = blockIdx.x - n * per_img;
    const int oh0 = (t / tiles_w) * 2 * WG_TR, ow0 = (t - (t / tiles_w) * tiles_w) * 2 * WG_TC;
    const int co0 = blockIdx.y * WG_CO;
    const int64_t plane = (int64_t)H * W;
    const float* __restrict__ xn = x + (int64_t)n * cin * plane;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5, l = lane & 31;
    const int xr = wv;  // wave's row of the 4x4 transformed tile M
    const int nchunks = cin / WG_CI;

    f32x4 ru[WG_U / 4 / kBlock];
    float rd[16];
    // the input window of this thread's tile (threads < 128: tile = tid % 32)
    WinWindow win;
    {
        const int tile = tid & 31;
        const int gr = oh0 + 2 * (tile / WG_TC) - 1, gc = ow0 + 2 * (tile % WG_TC) - 1;
        win.base = (int)(((tid >> 5) & 3) * plane + gr * W + gc) * 4;
        win.mask = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if ((unsigned)(gr + r) < (unsigned)H && (unsigned)(gc + c) < (unsigned)W)
                    win.mask |= 1u << (r * 4 + c);
    }
    const int64_t ci_bytes = (int64_t)cin * plane * 4;
    f32x16 acc[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j][0] = acc[j][1] = f32x16{};

    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xn), (short)0,
                                                      static_cast<int>(ci_bytes), 0x00020000);
    // The next chunk's U rows and input windows are loaded right after the previous
    // chunk's stage was written, before the barrier, so their latency is covered by the
    // barrier wait plus a whole MFMA phase.  The barrier is a raw s_barrier after an
    // LDS-only wait: __syncthreads()'s release fence would also wait for these loads.
    wg_load_u(up, 0, cout, co0, tid, ru);
    wg_load_x(rs, 0, plane, W, win, tid, rd);
    wg_store(Us0, Vs0, tid, ru, rd);
    if (nchunks > 1) {
        wg_load_u(up, 1, cout, co0, tid, ru);
        wg_load_x(rs, 1, plane, W, win, tid, rd);
    }
    lds_barrier();
    for (int cc = 0; cc < nchunks; ++cc)
        wg_chunk(Us0, Vs0, cc & 1, cc, nchunks, up, cout, co0, plane, W, rs, win, tid, xr, hh, l,
                 ru, rd, acc);

    // output transform Y = A^T M A, A^T = [[1,1,1,0],[0,1,-1,-1]]: wave xr holds row xr of
    // M, whose share of Y is A^T[:, xr] (x) (M[xr, :] A).  The four shares are summed in a
    // fixed order through LDS (wave 3, then 2, 1, and 0 writes the output).  Lane column
    // = tile l, register r = co row (r&3)+8(r>>2)+4h of channel half m.
    float* ex = lds;  // [64 co][32 tiles][4] (8192 floats of the 12288)
    const float c0 = xr == 3 ? 0.f : 1.f;                       // A^T[0][xr]
    const float c1 = xr == 0 ? 0.f : (xr == 1 ? 1.f : -1.f);    // A^T[1][xr]
    const int tile = l;
    const int oh = oh0 + 2 * (tile / WG_TC), ow = ow0 + 2 * (tile % WG_TC);
    float* on = out + (int64_t)n * cout * plane;
    if (xr == 3) wg_share<0>(acc, c0, c1, hh, tile, ex, nullptr, nullptr, 0, 0, 0);
    __syncthreads();
    if (xr == 2) wg_share<1>(acc, c0, c1, hh, tile, ex, nullptr, nullptr, 0, 0, 0);
    __syncthreads();
    if (xr == 1) wg_share<1>(acc, c0, c1, hh, tile, ex, nullptr, nullptr, 0, 0, 0);
    __syncthreads();
    if (xr == 0) wg_share<2>(acc, c0, c1, hh, tile, ex, bias, on, co0, plane, (int64_t)oh * W + ow, W);
}

// ---------------------------------------------------------------------------------------
// Register-resident variant (SP_WINO_REG=1, the default).  A wave's MFMA operands are
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
constexpr int WR_TR = 4;    // tile rows per workgroup (2 per wave): 8 output rows
constexpr int WR_TC = 16;   // tile columns: 32 output columns
constexpr int WR_NS = 4;    // unroll of the k-step ring (cin % (2 WR_NS) == 0)
constexpr int WX_ROW = 40;           // LDS floats per block row: even columns 0..16, odd 19..35
constexpr int WX_CI = 6 * WX_ROW;    // per input channel of the block
constexpr int WX_WAVE = 2 * WX_CI;   // per wave

struct WrX { f32x4 a, b; float h; };  // a lane's share of one k-step's input block
struct WrU { f32x4 u[4]; };           // a lane's 16 U values (xi = 0..15) for one k-step
struct WxLane {                       // per-lane constants of the block's loads and LDS traffic
    int oa, ob, oh;   // byte offsets of the two 16-byte pieces and the halo dword (or OOB)
    int wa, wb, wh;   // LDS indices (in the wave's region) the pieces are written to
    int rd;           // LDS index of the window's first even-column read
};

__device__ __forceinline__ void wr_load_x(__amdgpu_buffer_rsrc_t rs, const WxLane& xl, int so,
                                          WrX& x) {
    x.a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, xl.oa, so, 0));
    x.b = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, xl.ob, so, 0));
    x.h = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, xl.oh, so, 0));
}

__device__ __forceinline__ void wr_load_u(const float* __restrict__ src, WrU& u) {
#pragma unroll
    for (int i = 0; i < 4; ++i) u.u[i] = reinterpret_cast<const f32x4*>(src)[i];
}

// Block piece -> LDS: columns 4k..4k+3 go to even slots 2k, 2k+1 and odd slots 20+2k, 21+2k.
__device__ __forceinline__ void wr_stage_x(float* xw, const WxLane& xl, const WrX& x) {
    *reinterpret_cast<float2*>(xw + xl.wa) = make_float2(x.a[0], x.a[2]);
    *reinterpret_cast<float2*>(xw + xl.wa + 20) = make_float2(x.a[1], x.a[3]);
    *reinterpret_cast<float2*>(xw + xl.wb) = make_float2(x.b[0], x.b[2]);
    *reinterpret_cast<float2*>(xw + xl.wb + 20) = make_float2(x.b[1], x.b[3]);
    xw[xl.wh] = x.h;
}

// This lane's 4x4 window (columns 2tc-1 .. 2tc+2 = odd tc-1, even tc, odd tc, even tc+1).
__device__ __forceinline__ void wr_window(const float* xw, const WxLane& xl, float (&d)[16]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float* row = xw + xl.rd + r * WX_ROW;
        d[r * 4 + 0] = row[19];
        d[r * 4 + 1] = row[0];
        d[r * 4 + 2] = row[20];
        d[r * 4 + 3] = row[1];
    }
}

struct WrRing {          // k-steps in flight
    WrX xs[4];
    WrU us[4];
    float v[2][16];      // V of the current and the next step
};
struct WrCtx {
    __amdgpu_buffer_rsrc_t rs;
    WxLane xl;
    float* xw;
    const float* ub;
    int64_t u_step;
    int so_step, nsteps;
};

// One k-step q (slot K = q mod 4), laid out by hand with scheduling walls between the
// pieces — 4 MFMAs, stage the next block, 4 MFMAs, read the next windows, 4 MFMAs, the
// next V and the block loads, 4 MFMAs, the U loads — so the waits land where the data is
// due and the vector / LDS work issues in the MFMA pipe's shadow.  (Spreading the same
// work over all 16 MFMA gaps with scheduling groups measured the same.)
template <int K, bool FIRST>
__device__ __forceinline__ void wr_step(const WrCtx& c, int q, WrRing& g, f32x16 (&acc)[16]) {
    const int nx = min(q + 3, c.nsteps - 1);  // clamped: harmless re-loads at the end
    const int nu = min(q + 2, c.nsteps - 1);
    const WrU& u = g.us[K];
    const float(&vc)[16] = g.v[K & 1];
    float(&vn)[16] = g.v[(K + 1) & 1];
    float d[16];
    auto mfma = [&](int xi, float a) {
        acc[xi] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, vc[xi], FIRST ? f32x16{} : acc[xi],
                                                       0, 0, 0);
    };
#pragma unroll
    for (int xi = 0; xi < 4; ++xi) mfma(xi, u.u[0][xi]);
    __builtin_amdgcn_sched_barrier(0);
    wr_stage_x(c.xw, c.xl, g.xs[(K + 1) % 4]);  // block of step q + 1
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int xi = 4; xi < 8; ++xi) mfma(xi, u.u[1][xi - 4]);
    __builtin_amdgcn_sched_barrier(0);
    wr_window(c.xw, c.xl, d);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int xi = 8; xi < 12; ++xi) mfma(xi, u.u[2][xi - 8]);
    __builtin_amdgcn_sched_barrier(0);
    wino_in(d, vn);
    wr_load_x(c.rs, c.xl, nx * c.so_step, g.xs[(K + 3) % 4]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int xi = 12; xi < 16; ++xi) mfma(xi, u.u[3][xi - 12]);
    __builtin_amdgcn_sched_barrier(0);
    wr_load_u(c.ub + nu * c.u_step, g.us[(K + 2) % 4]);
    __builtin_amdgcn_sched_barrier(0);
}

__global__ __launch_bounds__(kBlock, 1) void k_wino3x3_r(const float* __restrict__ x,
                                                         const float* __restrict__ up,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ out, int cin,
                                                         int cout, int H, int W) {
    __shared__ __attribute__((aligned(16))) float xlds[4 * WX_WAVE];
    // XCD-aware order: blocks b and b + 8 share an L2, so consecutive logical blocks (the
    // channel blocks of one tile group, then its neighbours) are dealt to one XCD
    const int nb = gridDim.x, b = blockIdx.x;
    const int lb = (nb & 7) ? b : (b & 7) * (nb >> 3) + (b >> 3);
    const int cob = cout / WR_CO;
    const int co_blk = lb % cob, rest = lb / cob;
    const int tiles_w = W / (2 * WR_TC), per_img = tiles_w * (H / (2 * WR_TR));
    const int n = rest / per_img, t = rest - n * per_img;
    const int oh0 = (t / tiles_w) * 2 * WR_TR, ow0 = (t - (t / tiles_w) * tiles_w) * 2 * WR_TC;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int hh = lane >> 5, l = lane & 31;
    const int co0 = co_blk * WR_CO + 32 * (wv & 1);
    const int trl = l >> 4, tc = l & 15;          // this lane's tile within the wave
    const int tr = 2 * (wv >> 1) + trl;           // ... within the workgroup
    const int plane = H * W;                      // < 2^29 (checked on the host)
    const int row0 = oh0 + 4 * (wv >> 1) - 1;     // the wave's first input row
    float* const xw = xlds + wv * WX_WAVE;

    WxLane xl;
    {
        constexpr int OOB = 0x7FFFFFF0;  // outside the image: the buffer returns 0
        const int ka = lane & 7, rca = lane >> 3;                 // piece a: rows 0..7
        const int rcb = 8 + ((lane >> 3) & 3);                    // piece b: rows 8..11
        const int rch = (lane % 24) >> 1, side = lane & 1;        // halo: 12 rows x 2 sides
        auto goff = [&](int rc, int col) {
            const int ci = rc / 6, gr = row0 + rc % 6;
            return ((unsigned)gr < (unsigned)H && (unsigned)col < (unsigned)W)
                       ? (ci * plane + gr * W + col) * 4 : OOB;
        };
        auto loff = [](int rc) { return (rc / 6) * WX_CI + (rc % 6) * WX_ROW; };
        xl.oa = goff(rca, ow0 + 4 * ka);
        xl.ob = goff(rcb, ow0 + 4 * ka);
        xl.oh = goff(rch, side ? ow0 + 32 : ow0 - 1);
        xl.wa = loff(rca) + 2 * ka;
        xl.wb = loff(rcb) + 2 * ka;
        xl.wh = loff(rch) + (side ? 16 : 19);
        xl.rd = hh * WX_CI + 2 * trl * WX_ROW + tc;
    }
    const float* xn = x + (int64_t)n * cin * plane;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xn), (short)0,
                                                      cin * plane * 4, 0x00020000);
    const int so_step = 2 * plane * 4;  // bytes per k-step (two input channels)
    // packed U: [k-step][cout / 32][lane][16]
    const int64_t u_step = (int64_t)cout * 32;
    const float* ub = up + ((int64_t)(co0 >> 5) * 64 + lane) * 16;
    const int nsteps = cin / 2;  // a multiple of WR_NS (cin % (2 WR_NS) == 0)

    // Step q's input block is loaded during step q - 3 and staged + turned into V during
    // step q - 1; its U rows are loaded at the end of step q - 2 (wr_step).  The prologue
    // issues loads in the loop's own order, so the waits at the loop head are the same from
    // either predecessor.
    WrRing ring;
    wr_load_x(rs, xl, 0, ring.xs[0]);
    __builtin_amdgcn_sched_barrier(0);
    wr_load_x(rs, xl, so_step, ring.xs[1]);
    __builtin_amdgcn_sched_barrier(0);
    wr_load_u(ub, ring.us[0]);
    __builtin_amdgcn_sched_barrier(0);
    wr_load_x(rs, xl, 2 * so_step, ring.xs[2]);
    __builtin_amdgcn_sched_barrier(0);
    wr_load_u(ub + u_step, ring.us[1]);
    __builtin_amdgcn_sched_barrier(0);
    {
        float d[16];
        wr_stage_x(xw, xl, ring.xs[0]);
        wr_window(xw, xl, d);
        wino_in(d, ring.v[0]);
    }
    const WrCtx ctx{rs, xl, xw, ub, u_step, so_step, nsteps};
    f32x16 acc[16];
    // first round: step 0 starts the accumulators from zero (no 256 AGPR clears)
    wr_step<0, true>(ctx, 0, ring, acc);
    wr_step<1, false>(ctx, 1, ring, acc);
    wr_step<2, false>(ctx, 2, ring, acc);
    wr_step<3, false>(ctx, 3, ring, acc);
    for (int p = WR_NS; p < nsteps; p += WR_NS) {
        wr_step<0, false>(ctx, p + 0, ring, acc);
        wr_step<1, false>(ctx, p + 1, ring, acc);
        wr_step<2, false>(ctx, p + 2, ring, acc);
        wr_step<3, false>(ctx, p + 3, ring, acc);
    }

    // Y = A^T M A, A^T = [[1,1,1,0],[0,1,-1,-1]], per (channel, tile) in registers:
    // register r of every accumulator is channel co0 + (r&3) + 8(r>>2) + 4hh, tile l
    const int oh = oh0 + 2 * tr, ow = ow0 + 2 * tc;
    float* on = out + (int64_t)n * cout * plane + (int64_t)oh * W + ow;
    float bv[16];  // all bias loads in flight together (one wait, not sixteen)
#pragma unroll
    for (int r = 0; r < 16; ++r) bv[r] = 0.f;
    if (bias) {
#pragma unroll
        for (int r = 0; r < 16; ++r) bv[r] = bias[co0 + (r & 3) + 8 * (r >> 2) + 4 * hh];
    }
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
        const int co = co0 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        float* dst = on + (int64_t)co * plane;
        *reinterpret_cast<float2*>(dst) =
            make_float2(s0[0] + s0[1] + s0[2] + bv[r], s1[0] + s1[1] + s1[2] + bv[r]);
        *reinterpret_cast<float2*>(dst + W) =
            make_float2(s0[1] - s0[2] - s0[3] + bv[r], s1[1] - s1[2] - s1[3] + bv[r]);
    }
}

// Pack for k_wino3x3_r: up[((kin / 2 * (cout_p / 32) + orow / 32) * 64 + lane) * 16 + xi],
// lane = 32 (kin & 1) + orow % 32.
__global__ void k_wino3x3_pack_r(const float* __restrict__ w, int cout, int cin, int flip,
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

// U = G g G^T, G = [[1,0,0],[.5,.5,.5],[.5,-.5,.5],[0,0,1]], packed
// up[((cc*16 + xi)*WG_CI + ci_l)*cout_p + co].  input_vjp: transform W'[ci][co] = W[co][ci]
// flipped (the input VJP's weights; cout_p = cin of W).
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
    const int cc = kin / WG_CI, cl = kin - cc * WG_CI;
#pragma unroll
    for (int xi = 0; xi < 16; ++xi)
        up[(((int64_t)cc * 16 + xi) * WG_CI + cl) * cout_p + orow] = u[xi];
}

}  // namespace sp

using namespace sp;

extern "C" {

int sp_wino3x3_supported(int32_t cin, int32_t cout, int32_t height, int32_t width) {
#if SP_WINO_REG
    return cin > 0 && cout > 0 && cin % (2 * WR_NS) == 0 && cout % WR_CO == 0 &&
           height % (2 * WR_TR) == 0 && width % (2 * WR_TC) == 0 && height > 0 && width > 0;
#else
    return cin > 0 && cout > 0 && cin % WG_CI == 0 && cout % WG_CO == 0 &&
           height % (2 * WG_TR) == 0 && width % (2 * WG_TC) == 0 && height > 0 && width > 0;
#endif
}

int64_t sp_wino3x3_packed_size(int32_t cin, int32_t cout) { return (int64_t)cin * cout * 16; }

int sp_wino3x3_pack(const float* w, int32_t cout, int32_t cin, int32_t input_vjp, float* up,
                    sp_stream_t stream) {
    if (!w || !up || cout <= 0 || cin <= 0) return SP_EINVAL;
    const int kin = input_vjp ? cout : cin, nout = input_vjp ? cin : cout;
    const int64_t total = (int64_t)cout * cin;
#if SP_WINO_REG
    if (kin % 4 || nout % 32) return SP_EINVAL;
    launch(0, k_wino3x3_pack_r, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256),
           static_cast<hipStream_t>(stream), w, cout, cin, input_vjp, up);
    return check_launch("sp_wino3x3_pack");
#endif
    if (kin % WG_CI) return SP_EINVAL;
    (void)nout;
    launch(0, k_wino3x3_pack, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256),
           static_cast<hipStream_t>(stream), w, cout, cin, input_vjp, up);
    return check_launch("sp_wino3x3_pack");
}

static int wino3x3(int kind, const float* x, const float* up, const float* bias, int64_t n,
                   int32_t cin, int32_t cout, int32_t height, int32_t width, float* y,
                   sp_stream_t stream, const char* what) {
    if (!sp_wino3x3_supported(cin, cout, height, width) || n < 0) return SP_EINVAL;
    if (n == 0) return SP_OK;
    if (!x || !up || !y) return SP_EINVAL;
#if SP_WINO_REG
    const int64_t blocks = n * (height / (2 * WR_TR)) * (width / (2 * WR_TC)) * (cout / WR_CO);
#else
    const int64_t blocks = n * (height / (2 * WG_TR)) * (width / (2 * WG_TC));
#endif
    // per-sample input planes are addressed by 32-bit buffer offsets (bytes < 2^31)
    if (blocks >= (int64_t(1) << 31) || (int64_t)cin * height * width * 4 >= (int64_t(1) << 31) ||
        (int64_t)cout * height * width * 4 >= (int64_t(1) << 31))
        return SP_EINVAL;
    // executed MFMA work: 16 GEMMs of 2*cin*cout per 2x2 tile = 8*cin*cout per pixel
    // (the direct-conv equivalent is 18*cin*cout per pixel, 2.25x more)
    const double flops = 8.0 * n * cin * cout * height * width;
#if SP_WINO_REG
    launch_w(kind, flops, k_wino3x3_r, dim3(static_cast<unsigned>(blocks)), dim3(kBlock),
             static_cast<hipStream_t>(stream), x, up, bias, y, cin, cout, height, width);
    return check_launch(what);
#endif
    launch_w(kind, flops, k_wino3x3, dim3(static_cast<unsigned>(blocks), cout / WG_CO),
             dim3(kBlock), static_cast<hipStream_t>(stream), x, up, bias, y, cin, cout, height,
             width);
    return check_launch(what);
}

int sp_wino3x3_fwd(const float* x, const float* up, const float* bias, int64_t n, int32_t cin,
                   int32_t cout, int32_t height, int32_t width, float* y, sp_stream_t stream) {
    return wino3x3(TK_WINO3X3_FWD, x, up, bias, n, cin, cout, height, width, y, stream,
                   "sp_wino3x3_fwd");
}

int sp_wino3x3_bwd_input(const float* dy, const float* up_vjp, int64_t n, int32_t cin,
                         int32_t cout, int32_t height, int32_t width, float* dx,
                         sp_stream_t stream) {
    return wino3x3(TK_WINO3X3_BWD_INPUT, dy, up_vjp, nullptr, n, cout, cin, height, width, dx,
                   stream, "sp_wino3x3_bwd_input");
}

}  // extern "C"

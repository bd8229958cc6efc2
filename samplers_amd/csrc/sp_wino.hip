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
#pragma unroll
    for (int kk = 0; kk < WG_CI / 2; ++kk) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float a0 = Ub[(j * WG_CI + 2 * kk) * WG_CO];
            const float a1 = Ub[(j * WG_CI + 2 * kk) * WG_CO + 32];
            const float b = Vb[(j * WG_CI + 2 * kk) * WG_T];
            acc[j][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b, acc[j][0], 0, 0, 0);
            acc[j][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b, acc[j][1], 0, 0, 0);
        }
    }
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
    float tg[12];  // G g (4 x 3)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        tg[0 * 3 + c] = g[0 * 3 + c];
        tg[1 * 3 + c] = 0.5f * (g[0 * 3 + c] + g[1 * 3 + c] + g[2 * 3 + c]);
        tg[2 * 3 + c] = 0.5f * (g[0 * 3 + c] - g[1 * 3 + c] + g[2 * 3 + c]);
        tg[3 * 3 + c] = g[2 * 3 + c];
    }
    const int cc = kin / WG_CI, cl = kin - cc * WG_CI;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const float a = tg[r * 3 + 0], b = tg[r * 3 + 1], c = tg[r * 3 + 2];
        const float u[4] = {a, 0.5f * (a + b + c), 0.5f * (a - b + c), c};
#pragma unroll
        for (int q = 0; q < 4; ++q)
            up[(((int64_t)cc * 16 + r * 4 + q) * WG_CI + cl) * cout_p + orow] = u[q];
    }
}

}  // namespace sp

using namespace sp;

extern "C" {

int sp_wino3x3_supported(int32_t cin, int32_t cout, int32_t height, int32_t width) {
    return cin > 0 && cout > 0 && cin % WG_CI == 0 && cout % WG_CO == 0 &&
           height % (2 * WG_TR) == 0 && width % (2 * WG_TC) == 0 && height > 0 && width > 0;
}

int64_t sp_wino3x3_packed_size(int32_t cin, int32_t cout) { return (int64_t)cin * cout * 16; }

int sp_wino3x3_pack(const float* w, int32_t cout, int32_t cin, int32_t input_vjp, float* up,
                    sp_stream_t stream) {
    if (!w || !up || cout <= 0 || cin <= 0) return SP_EINVAL;
    if (input_vjp ? (cout % WG_CI) : (cin % WG_CI)) return SP_EINVAL;
    const int64_t total = (int64_t)cout * cin;
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
    const int64_t blocks = n * (height / (2 * WG_TR)) * (width / (2 * WG_TC));
    // per-sample input planes are addressed by 32-bit buffer offsets (bytes < 2^31)
    if (blocks >= (int64_t(1) << 31) || (int64_t)cin * height * width * 4 >= (int64_t(1) << 31) ||
        (int64_t)cout * height * width * 4 >= (int64_t(1) << 31))
        return SP_EINVAL;
    // executed MFMA work: 16 GEMMs of 2*cin*cout per 2x2 tile = 8*cin*cout per pixel
    // (the direct-conv equivalent is 18*cin*cout per pixel, 2.25x more)
    const double flops = 8.0 * n * cin * cout * height * width;
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

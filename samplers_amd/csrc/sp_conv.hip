// 3x3 / stride 1 / pad 1 convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32: exact fp32,
// the result of each output is a k-ordered fmaf chain) — the convolution tile of the
// SD VAE and UNet ResnetBlocks (SURVEY.md §8f row f1, §8b "vae_conv3x3_fwd/bwd_input";
// reached from /root/reference/samplers/networks/diffusers/stable_diffusion.py:330-345
// and ddpm.py:40-43).  Input VJP = the same kernel on transposed + flipped weights.
//
// Implicit GEMM: out[n, co, p] = sum_{ci, r, s} W[co, ci, r, s] * x[n, ci, p + (r-1, s-1)]
//   M = Cout (128 per workgroup), N = pixels (8 rows x 32 columns of one image per
//   workgroup), K = Cin*9 walked in chunks of 4 input channels (36 k).
// Per chunk the workgroup stages in LDS
//   A: packed weights [36 k][128 co]          (host-packed once per layer: row k of a
//                                              chunk = 128 contiguous co, float4 loads)
//   P: input patch    [4 ci][10 rows][34 cols] (zero outside the image = the padding)
// and each wave (2 x 4 tiles of 32 x 32: 64 co x 4 pixel rows) issues 144 MFMAs.  Lane
// half h of an MFMA carries k-index kk + 18h, i.e. the same (r, s) and input channel
// ci + 2h, so every LDS address is a per-lane base + a compile-time offset.  Chunks are
// double-buffered: the next chunk's global loads are in flight during the MFMAs.
// Measured on MI355X (tools/bench_conv.py): 136-137.5 TFLOP/s = 0.87 of the 157.3 TF
// fp32-MFMA peak on the UNet/VAE layer shapes (MIOpen: 104-130); 4x8 / 8x4 / 8x8 /
// 2x8 (channels x rows) tiles measured 133 / 114-121 / 126-129 / 132-136.

#define SP_TU 5  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

namespace sp {

#ifndef SP_CONV_CI
#define SP_CONV_CI 4
#endif
#ifndef SP_CONV_TPH
#define SP_CONV_TPH 8
#endif
#ifndef SP_CONV_MINB
#define SP_CONV_MINB 2
#endif

constexpr int CV_M = 128;            // output channels per workgroup
constexpr int CV_TPH = SP_CONV_TPH;  // pixel rows per workgroup (each wave: TPH/2 rows)
constexpr int CV_TPW = 32;           // pixel columns per workgroup
constexpr int CV_CI = SP_CONV_CI;    // input channels per K chunk (even)
constexpr int CV_K = CV_CI * 9;
constexpr int CV_KH = CV_K / 2;      // k-steps per chunk: lane half h takes k = kk + KH*h
constexpr int CV_NR = CV_TPH / 2;    // MFMA pixel tiles (rows) per wave
static_assert(CV_CI % 2 == 0 && CV_TPH % 2 == 0, "conv tile");
constexpr int CV_PW = CV_TPW + 2;
constexpr int CV_PH = CV_TPH + 2;
constexpr int CV_PATCH = CV_PH * CV_PW;                    // 204
constexpr int CV_A4 = CV_K * CV_M / 4;                     // float4 of A per chunk: 1152
constexpr int CV_NA = (CV_A4 + kBlock - 1) / kBlock;       // 5
constexpr int CV_NP = (CV_CI * CV_PATCH + kBlock - 1) / kBlock;  // 4

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Global -> registers for K chunk cc: packed weight rows (float4) and the input patch
// (zero outside the image).
__device__ __forceinline__ void cv_load(const float* __restrict__ wp, const float* __restrict__ xn,
                                        int cc, int cout, int co0, int h0, int w0, int H, int W,
                                        int64_t plane, int tid, f32x4 (&ra)[CV_NA],
                                        float (&rp)[CV_NP]) {
    const float* src = wp + (int64_t)cc * CV_K * cout + co0;
#pragma unroll
    for (int i = 0; i < CV_NA; ++i) {
        const int idx = tid + kBlock * i;
        if (i < CV_NA - 1 || idx < CV_A4)
            ra[i] = *reinterpret_cast<const f32x4*>(src + (int64_t)(idx >> 5) * cout + (idx & 31) * 4);
    }
#pragma unroll
    for (int i = 0; i < CV_NP; ++i) {
        const int idx = tid + kBlock * i;
        const int ci = idx / CV_PATCH, rem = idx - ci * CV_PATCH;
        const int pr = rem / CV_PW, pc = rem - pr * CV_PW;
        const int gh = h0 - 1 + pr, gw = w0 - 1 + pc;
        const bool ok = (i < CV_NP - 1 || idx < CV_CI * CV_PATCH) && (unsigned)gh < (unsigned)H &&
                        (unsigned)gw < (unsigned)W;
        rp[i] = ok ? xn[(int64_t)(cc * CV_CI + ci) * plane + gh * W + gw] : 0.f;
    }
}

__device__ __forceinline__ void cv_store(float* As, float* Ps, int tid, const f32x4 (&ra)[CV_NA],
                                         const float (&rp)[CV_NP]) {
#pragma unroll
    for (int i = 0; i < CV_NA; ++i) {
        const int idx = tid + kBlock * i;
        if (i < CV_NA - 1 || idx < CV_A4) *reinterpret_cast<f32x4*>(&As[idx * 4]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < CV_NP; ++i) {
        const int idx = tid + kBlock * i;
        if (i < CV_NP - 1 || idx < CV_CI * CV_PATCH) Ps[idx] = rp[i];
    }
}

__global__ __launch_bounds__(kBlock, SP_CONV_MINB) void k_conv3x3(const float* __restrict__ x,
                                                       const float* __restrict__ wp,
                                                       const float* __restrict__ bias,
                                                       float* __restrict__ out, int cin,
                                                       int cout, int H, int W) {
    __shared__ __attribute__((aligned(16))) float As[2][CV_K * CV_M];
    __shared__ float Ps[2][CV_CI * CV_PATCH];

    const int tiles_w = W / CV_TPW, per_img = tiles_w * (H / CV_TPH);
    const int n = blockIdx.x / per_img, t = blockIdx.x - n * per_img;
    const int h0 = (t / tiles_w) * CV_TPH, w0 = (t - (t / tiles_w) * tiles_w) * CV_TPW;
    const int co0 = blockIdx.y * CV_M;
    SP_DCHECK(W % CV_TPW == 0 && H % CV_TPH == 0 && co0 + CV_M <= cout && cin % CV_CI == 0 &&
              h0 + CV_TPH <= H && w0 + CV_TPW <= W);
    const int64_t plane = (int64_t)H * W;
    const float* __restrict__ xn = x + (int64_t)n * cin * plane;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5, l = lane & 31;
    const int m_w = (wv & 1) * 64, prow = (wv >> 1) * CV_NR;
    const int nchunks = cin / CV_CI;

    f32x4 ra[CV_NA];
    float rp[CV_NP];
    f32x16 acc[2][CV_NR];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < CV_NR; ++b) acc[a][b] = f32x16{};

    cv_load(wp, xn, 0, cout, co0, h0, w0, H, W, plane, tid, ra, rp);
    cv_store(As[0], Ps[0], tid, ra, rp);
    __syncthreads();
    for (int cc = 0; cc < nchunks; ++cc) {
        const int buf = cc & 1;
        if (cc + 1 < nchunks) cv_load(wp, xn, cc + 1, cout, co0, h0, w0, H, W, plane, tid, ra, rp);
        const float* Ab = &As[buf][(CV_KH * hh) * CV_M + m_w + l];
        const float* Pb = &Ps[buf][(CV_CI / 2 * hh) * CV_PATCH + prow * CV_PW + l];
#pragma unroll
        for (int kk = 0; kk < CV_KH; ++kk) {
            const int koff = (kk / 9) * CV_PATCH + ((kk % 9) / 3) * CV_PW + (kk % 3);
            const float a0 = Ab[kk * CV_M], a1 = Ab[kk * CV_M + 32];
            float b[CV_NR];
#pragma unroll
            for (int ni = 0; ni < CV_NR; ++ni) b[ni] = Pb[koff + ni * CV_PW];
#pragma unroll
            for (int ni = 0; ni < CV_NR; ++ni) {
                acc[0][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b[ni], acc[0][ni], 0, 0, 0);
                acc[1][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b[ni], acc[1][ni], 0, 0, 0);
            }
        }
        if (cc + 1 < nchunks) cv_store(As[buf ^ 1], Ps[buf ^ 1], tid, ra, rp);
        __syncthreads();
    }

    // epilogue: C/D map col = lane & 31 (pixel column), row = (r&3) + 8(r>>2) + 4h (co)
    float* on = out + (int64_t)n * cout * plane;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = co0 + m_w + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const float bv = bias ? bias[co] : 0.f;
#pragma unroll
            for (int ni = 0; ni < CV_NR; ++ni)
                on[(int64_t)co * plane + (h0 + prow + ni) * W + w0 + l] = acc[mi][ni][r] + bv;
        }
    }
}

// wp[(cc*36 + k)*cout_p + co] for k = ci_l*9 + r*3 + s.  flip: pack the input-VJP
// weights W'[ci][co][r][s] = W[co][ci][2-r][2-s] (cout_p = cin of W).
__global__ void k_conv3x3_pack(const float* __restrict__ w, int cout, int cin, int flip,
                               float* __restrict__ wp) {
    const int64_t total = (int64_t)cout * cin * 9;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int co = static_cast<int>(i / ((int64_t)cin * 9));
    const int rem = static_cast<int>(i - (int64_t)co * cin * 9);
    const int ci = rem / 9, rs = rem - ci * 9, r = rs / 3, s = rs - r * 3;
    if (!flip) {
        // GEMM roles: rows = co (cout), k = (ci, r, s)
        const int cc = ci / CV_CI, k = (ci % CV_CI) * 9 + rs;
        wp[((int64_t)cc * CV_K + k) * cout + co] = w[i];
    } else {
        // input VJP: rows = ci (cin of W), k = (co, 2-r, 2-s)
        const int cc = co / CV_CI, k = (co % CV_CI) * 9 + (2 - r) * 3 + (2 - s);
        wp[((int64_t)cc * CV_K + k) * cin + ci] = w[i];
    }
}

}  // namespace sp

using namespace sp;

extern "C" {

int sp_conv3x3_supported(int32_t cin, int32_t cout, int32_t height, int32_t width) {
    return cin > 0 && cout > 0 && cin % CV_CI == 0 && cout % CV_M == 0 && height % CV_TPH == 0 &&
           width % CV_TPW == 0 && height > 0 && width > 0;
}

int64_t sp_conv3x3_packed_size(int32_t cin, int32_t cout) { return (int64_t)cin * cout * 9; }

int sp_conv3x3_pack(const float* w, int32_t cout, int32_t cin, int32_t input_vjp, float* wp,
                    sp_stream_t stream) {
    if (!w || !wp || cout <= 0 || cin <= 0) return SP_EINVAL;
    if (input_vjp ? (cout % CV_CI) : (cin % CV_CI)) return SP_EINVAL;
    const int64_t total = (int64_t)cout * cin * 9;
    launch(0, k_conv3x3_pack, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256),
           static_cast<hipStream_t>(stream), w, cout, cin, input_vjp, wp);
    return check_launch("sp_conv3x3_pack");
}

static int conv3x3(int kind, const float* x, const float* wp, const float* bias, int64_t n,
                   int32_t cin, int32_t cout, int32_t height, int32_t width, float* y,
                   sp_stream_t stream, const char* what) {
    if (!sp_conv3x3_supported(cin, cout, height, width) || n < 0) return SP_EINVAL;
    if (n == 0) return SP_OK;
    if (!x || !wp || !y) return SP_EINVAL;
    const int64_t tiles = n * (height / CV_TPH) * (width / CV_TPW);
    if (tiles >= (int64_t(1) << 31) || (int64_t)cin * height * width >= (int64_t(1) << 31))
        return SP_EINVAL;
    const double flops = 18.0 * n * cin * cout * height * width;  // 2 * 9 MACs per tap
    launch_w(kind, flops, k_conv3x3, dim3(static_cast<unsigned>(tiles), cout / CV_M),
             dim3(kBlock), static_cast<hipStream_t>(stream), x, wp, bias, y, cin, cout, height,
             width);
    return check_launch(what);
}

int sp_conv3x3_fwd(const float* x, const float* wp, const float* bias, int64_t n, int32_t cin,
                   int32_t cout, int32_t height, int32_t width, float* y, sp_stream_t stream) {
    return conv3x3(TK_CONV3X3_FWD, x, wp, bias, n, cin, cout, height, width, y, stream,
                   "sp_conv3x3_fwd");
}

int sp_conv3x3_bwd_input(const float* dy, const float* wp_vjp, int64_t n, int32_t cin,
                         int32_t cout, int32_t height, int32_t width, float* dx,
                         sp_stream_t stream) {
    // dx (n, cin, h, w) = conv3x3(dy (n, cout, h, w), W') with W' packed by input_vjp=1
    return conv3x3(TK_CONV3X3_BWD_INPUT, dy, wp_vjp, nullptr, n, cout, cin, height, width, dx,
                   stream, "sp_conv3x3_bwd_input");
}

}  // extern "C"

// Transformer-block glue of the SD 1.5 eps-UNet (diffusers BasicTransformerBlock inside
// Transformer2DModel, called from /root/reference/samplers/networks/diffusers/
// stable_diffusion.py:306-313): LayerNorm over the channels of
// token-major activations and the GEGLU gate of the feed-forward, forward and input VJP.
// The surrounding linears run on sp_linear_x6 and the attention on sp_attention.hip; these
// kernels replace the torch LayerNorm / chunk / gelu / mul chain and its autograd VJP
// (one pass over the bytes each way instead of three to five).
//
// All of them stream HBM: one wave per LayerNorm row (C = 320 / 640 / 1280 channels held
// in registers, two wave reductions), float4 lanes for GEGLU.  fp32 throughout.

#define SP_TU 12  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

#include <algorithm>
#include <cmath>

namespace sp {

constexpr int LN_ROWS = kBlock / 64;  // rows per workgroup (one per wave)

// Row r of a [T][C] matrix: lane l holds float4 groups l, l + 64, ... (NV of them, masked
// past C / 4).
template <int NV>
__device__ __forceinline__ void ln_load(const float* __restrict__ row, int c4, int lane, float4 (&v)[NV]) {
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = lane + 64 * j;
        v[j] = i < c4 ? reinterpret_cast<const float4*>(row)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

__device__ __forceinline__ float sum4(float4 a) { return (a.x + a.y) + (a.z + a.w); }

// y = (x - mean) / sqrt(var + eps) * w + b (biased variance, as torch.nn.LayerNorm); the
// row's mean and 1/sqrt(var + eps) are kept for the VJP.
template <int NV>
__global__ __launch_bounds__(kBlock) void k_layernorm_fwd(const float* __restrict__ x,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ b, int64_t rows,
                                                          int c, float eps, float* __restrict__ y,
                                                          float* __restrict__ mean,
                                                          float* __restrict__ rstd) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * LN_ROWS + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int c4 = c >> 2;
    SP_DCHECK(c % 4 == 0 && c4 <= NV * 64);  // the row fits the lane's registers
    float4 v[NV];
    ln_load<NV>(x + r * c, c4, lane, v);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) s += sum4(v[j]);
    const float mu = wave_sum(s) / static_cast<float>(c);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        if (lane + 64 * j < c4) {
            const float4 d = make_float4(v[j].x - mu, v[j].y - mu, v[j].z - mu, v[j].w - mu);
            q += (d.x * d.x + d.y * d.y) + (d.z * d.z + d.w * d.w);
        }
    }
    const float rs = 1.f / sqrtf(wave_sum(q) / static_cast<float>(c) + eps);
    float* yr = y + r * c;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = lane + 64 * j;
        if (i < c4) {
            const float4 g = reinterpret_cast<const float4*>(w)[i];
            const float4 o = reinterpret_cast<const float4*>(b)[i];
            reinterpret_cast<float4*>(yr)[i] =
                make_float4((v[j].x - mu) * rs * g.x + o.x, (v[j].y - mu) * rs * g.y + o.y,
                            (v[j].z - mu) * rs * g.z + o.z, (v[j].w - mu) * rs * g.w + o.w);
        }
    }
    if (lane == 0) mean[r] = mu, rstd[r] = rs;
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * w, xhat = (x - mean) * rstd
// (the weights are frozen: no dw / db); add != NULL: dx += add (the residual branch's
// gradient of the same tensor, summed here instead of in a separate pass).
template <int NV>
__global__ __launch_bounds__(kBlock) void k_layernorm_bwd(const float* __restrict__ dy,
                                                          const float* __restrict__ x,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd,
                                                          const float* __restrict__ add, int64_t rows,
                                                          int c, float* __restrict__ dx) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * LN_ROWS + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int c4 = c >> 2;
    const float mu = mean[r], rs = rstd[r];
    float4 g[NV], h[NV];
    ln_load<NV>(dy + r * c, c4, lane, g);
    ln_load<NV>(x + r * c, c4, lane, h);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = lane + 64 * j;
        if (i < c4) {
            const float4 ww = reinterpret_cast<const float4*>(w)[i];
            g[j] = make_float4(g[j].x * ww.x, g[j].y * ww.y, g[j].z * ww.z, g[j].w * ww.w);
            h[j] = make_float4((h[j].x - mu) * rs, (h[j].y - mu) * rs, (h[j].z - mu) * rs, (h[j].w - mu) * rs);
            s1 += (g[j].x * h[j].x + g[j].y * h[j].y) + (g[j].z * h[j].z + g[j].w * h[j].w);
            s2 += sum4(g[j]);
        }
    }
    const float inv_c = 1.f / static_cast<float>(c);
    const float m1 = wave_sum(s1) * inv_c, m2 = wave_sum(s2) * inv_c;
    float* dr = dx + r * c;
    const float* ar = add ? add + r * c : nullptr;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = lane + 64 * j;
        if (i < c4) {
            float4 o = make_float4(rs * (g[j].x - m2 - h[j].x * m1), rs * (g[j].y - m2 - h[j].y * m1),
                                   rs * (g[j].z - m2 - h[j].z * m1), rs * (g[j].w - m2 - h[j].w * m1));
            if (ar) {
                const float4 a = reinterpret_cast<const float4*>(ar)[i];
                o = make_float4(o.x + a.x, o.y + a.y, o.z + a.z, o.w + a.w);
            }
            reinterpret_cast<float4*>(dr)[i] = o;
        }
    }
}

// exact GELU (torch.nn.functional.gelu, approximate='none') and its derivative
__device__ __forceinline__ float gelu(float g) { return 0.5f * g * (1.f + erff(g * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float g) {
    const float cdf = 0.5f * (1.f + erff(g * 0.70710678118654752f));
    const float pdf = expf(-0.5f * g * g) * 0.39894228040143268f;
    return cdf + g * pdf;
}

// h = [a | gate] ([T][2F], the GEGLU projection's output): y = a * gelu(gate)  ([T][F])
__global__ __launch_bounds__(kBlock) void k_geglu_fwd(const float* __restrict__ h, int64_t rows, int f,
                                                      float* __restrict__ y) {
    const int f4 = f >> 2;
    const int n4 = static_cast<int>(rows) * f4;  // < 2^31 (checked on the host)
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n4; i += gridDim.x * kBlock) {
        const int r = i / f4;
        const int j = i - r * f4;
        const float4* hr = reinterpret_cast<const float4*>(h + (int64_t)r * 2 * f);
        const float4 a = hr[j], g = hr[f4 + j];
        reinterpret_cast<float4*>(y)[i] =
            make_float4(a.x * gelu(g.x), a.y * gelu(g.y), a.z * gelu(g.z), a.w * gelu(g.w));
    }
}

// VJP: dh = [dy * gelu(gate) | dy * a * gelu'(gate)]
__global__ __launch_bounds__(kBlock) void k_geglu_bwd(const float* __restrict__ h,
                                                      const float* __restrict__ dy, int64_t rows, int f,
                                                      float* __restrict__ dh) {
    const int f4 = f >> 2;
    const int n4 = static_cast<int>(rows) * f4;  // < 2^31 (checked on the host)
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n4; i += gridDim.x * kBlock) {
        const int r = i / f4;
        const int j = i - r * f4;
        const float4* hr = reinterpret_cast<const float4*>(h + (int64_t)r * 2 * f);
        const float4 a = hr[j], g = hr[f4 + j];
        const float4 d = reinterpret_cast<const float4*>(dy)[i];
        float4* o = reinterpret_cast<float4*>(dh + (int64_t)r * 2 * f);
        o[j] = make_float4(d.x * gelu(g.x), d.y * gelu(g.y), d.z * gelu(g.z), d.w * gelu(g.w));
        o[f4 + j] = make_float4(d.x * a.x * gelu_grad(g.x), d.y * a.y * gelu_grad(g.y),
                                d.z * a.z * gelu_grad(g.z), d.w * a.w * gelu_grad(g.w));
    }
}

// Row softmax of materialised attention scores (the single-head d = 512 attention of the
// VAE mid blocks and the DDPM UNet, whose score GEMMs stay on hipBLASLt): one wave per row of
// n scores held in registers; in place, lse[row] = max + log(sum) kept for the record.
template <int NV>
__global__ __launch_bounds__(kBlock) void k_softmax_rows(float* __restrict__ s, int64_t rows, int n,
                                                         float* __restrict__ lse) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * LN_ROWS + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int n4 = n >> 2;
    float* row = s + r * n;
    float4 v[NV];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = lane + 64 * j;
        v[j] = i < n4 ? reinterpret_cast<const float4*>(row)[i]
                      : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
        mx = fmaxf(mx, fmaxf(fmaxf(v[j].x, v[j].y), fmaxf(v[j].z, v[j].w)));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        v[j] = make_float4(expf(v[j].x - mx), expf(v[j].y - mx), expf(v[j].z - mx), expf(v[j].w - mx));
        sum += sum4(v[j]);
    }
    sum = wave_sum(sum);
    const float inv = 1.f / sum;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = lane + 64 * j;
        if (i < n4)
            reinterpret_cast<float4*>(row)[i] = make_float4(v[j].x * inv, v[j].y * inv, v[j].z * inv, v[j].w * inv);
    }
    if (lse && lane == 0) lse[r] = mx + logf(sum);
}

// Its VJP, scaled: ds = scale * p * (dp - sum(p * dp)) per row, written over dp.
template <int NV>
__global__ __launch_bounds__(kBlock) void k_softmax_bwd_rows(const float* __restrict__ p, float* __restrict__ dp,
                                                             int64_t rows, int n, float scale) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * LN_ROWS + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int n4 = n >> 2;
    float4 a[NV], g[NV];
    ln_load<NV>(p + r * n, n4, lane, a);
    ln_load<NV>(dp + r * n, n4, lane, g);
    float d = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) d += (a[j].x * g[j].x + a[j].y * g[j].y) + (a[j].z * g[j].z + a[j].w * g[j].w);
    d = wave_sum(d);
    float* row = dp + r * n;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = lane + 64 * j;
        if (i < n4)
            reinterpret_cast<float4*>(row)[i] =
                make_float4(scale * a[j].x * (g[j].x - d), scale * a[j].y * (g[j].y - d),
                            scale * a[j].z * (g[j].z - d), scale * a[j].w * (g[j].w - d));
    }
}

// 1x1 convolution over few channels (the SD VAE's quant_conv 8 -> 8 and post_quant_conv
// 4 -> 4, stable_diffusion.py:330-345): y[n][o][p] = sum_c w[o][c] x[n][c][p] (+ b[o]), one
// thread per 4 pixels; trans = 1 applies W^T (the input VJP, no bias).
template <int CI, int CO>
__global__ __launch_bounds__(kBlock) void k_conv1x1_small(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ b, int64_t n, int hw,
                                                          int trans, float* __restrict__ y) {
    __shared__ float ws[CI * CO + CO];
    for (int i = threadIdx.x; i < CI * CO; i += kBlock) {
        const int o = i / CI, c = i - o * CI;
        ws[i] = trans ? w[c * CO + o] : w[i];  // ws[o][c]; trans: w is stored [CI][CO]
    }
    for (int i = threadIdx.x; i < CO; i += kBlock) ws[CI * CO + i] = b ? b[i] : 0.f;
    __syncthreads();
    const int hw4 = hw >> 2;
    const int64_t total = n * hw4;
    for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += (int64_t)gridDim.x * kBlock) {
        const int64_t img = t / hw4;
        const int p = static_cast<int>(t - img * hw4);
        float4 xv[CI];
#pragma unroll
        for (int c = 0; c < CI; ++c) xv[c] = reinterpret_cast<const float4*>(x + (img * CI + c) * hw)[p];
#pragma unroll
        for (int o = 0; o < CO; ++o) {
            const float bb = ws[CI * CO + o];
            float4 acc = make_float4(bb, bb, bb, bb);
#pragma unroll
            for (int c = 0; c < CI; ++c) {
                const float ww = ws[o * CI + c];
                acc.x = fmaf(ww, xv[c].x, acc.x);
                acc.y = fmaf(ww, xv[c].y, acc.y);
                acc.z = fmaf(ww, xv[c].z, acc.z);
                acc.w = fmaf(ww, xv[c].w, acc.w);
            }
            reinterpret_cast<float4*>(y + (img * CO + o) * hw)[p] = acc;
        }
    }
}

static int ln_nv(int c) { return (c / 4 + 63) / 64; }

static unsigned stream_grid(int64_t n4) {
    const int64_t blocks = (n4 + kBlock - 1) / kBlock;
    return static_cast<unsigned>(blocks < 8192 ? blocks : 8192);
}

}  // namespace sp

using namespace sp;

extern "C" {

int sp_layernorm_supported(int64_t rows, int32_t c) {
    return rows >= 0 && c > 0 && c % 4 == 0 && ln_nv(c) <= 8 && rows * (int64_t)c < (int64_t(1) << 40);
}

#define SP_LN_DISPATCH(NVV, ...) \
    switch (NVV) {               \
        case 1: __VA_ARGS__(1); break; \
        case 2: __VA_ARGS__(2); break; \
        case 3: __VA_ARGS__(3); break; \
        case 4: __VA_ARGS__(4); break; \
        case 5: __VA_ARGS__(5); break; \
        case 6: __VA_ARGS__(6); break; \
        case 7: __VA_ARGS__(7); break; \
        default: __VA_ARGS__(8); break; \
    }

int sp_layernorm_fwd(const float* x, const float* w, const float* b, int64_t rows, int32_t c, float eps,
                     float* y, float* mean, float* rstd, sp_stream_t stream) {
    if (!sp_layernorm_supported(rows, c)) return SP_EINVAL;
    if (rows == 0) return SP_OK;
    if (!x || !w || !b || !y || !mean || !rstd || x == y) return SP_EINVAL;
    const dim3 grid(static_cast<unsigned>((rows + LN_ROWS - 1) / LN_ROWS));
    hipStream_t s = static_cast<hipStream_t>(stream);
#define SP_LN_F(N) launch(0, k_layernorm_fwd<N>, grid, dim3(kBlock), s, x, w, b, rows, c, eps, y, mean, rstd)
    SP_LN_DISPATCH(ln_nv(c), SP_LN_F)
#undef SP_LN_F
    return check_launch("sp_layernorm_fwd");
}

int sp_layernorm_bwd(const float* dy, const float* x, const float* w, const float* mean, const float* rstd,
                     const float* add, int64_t rows, int32_t c, float* dx, sp_stream_t stream) {
    if (!sp_layernorm_supported(rows, c)) return SP_EINVAL;
    if (rows == 0) return SP_OK;
    if (!dy || !x || !w || !mean || !rstd || !dx || dx == x) return SP_EINVAL;
    const dim3 grid(static_cast<unsigned>((rows + LN_ROWS - 1) / LN_ROWS));
    hipStream_t s = static_cast<hipStream_t>(stream);
#define SP_LN_B(N) launch(0, k_layernorm_bwd<N>, grid, dim3(kBlock), s, dy, x, w, mean, rstd, add, rows, c, dx)
    SP_LN_DISPATCH(ln_nv(c), SP_LN_B)
#undef SP_LN_B
    return check_launch("sp_layernorm_bwd");
}

static int sm_nv(int n) {
    const int nv = (n / 4 + 63) / 64;
    return nv <= 1 ? 1 : nv <= 2 ? 2 : nv <= 4 ? 4 : nv <= 8 ? 8 : 16;
}

int sp_softmax_rows_supported(int64_t rows, int32_t n) {
    return rows >= 0 && n > 0 && n % 4 == 0 && n <= 4096 && rows * (int64_t)n < (int64_t(1) << 40);
}

int sp_softmax_rows(float* s, int64_t rows, int32_t n, float* lse, sp_stream_t stream) {
    if (!sp_softmax_rows_supported(rows, n)) return SP_EINVAL;
    if (rows == 0) return SP_OK;
    if (!s) return SP_EINVAL;
    const dim3 grid(static_cast<unsigned>((rows + LN_ROWS - 1) / LN_ROWS));
    hipStream_t st = static_cast<hipStream_t>(stream);
    switch (sm_nv(n)) {
        case 1: launch(0, k_softmax_rows<1>, grid, dim3(kBlock), st, s, rows, static_cast<int>(n), lse); break;
        case 2: launch(0, k_softmax_rows<2>, grid, dim3(kBlock), st, s, rows, static_cast<int>(n), lse); break;
        case 4: launch(0, k_softmax_rows<4>, grid, dim3(kBlock), st, s, rows, static_cast<int>(n), lse); break;
        case 8: launch(0, k_softmax_rows<8>, grid, dim3(kBlock), st, s, rows, static_cast<int>(n), lse); break;
        default: launch(0, k_softmax_rows<16>, grid, dim3(kBlock), st, s, rows, static_cast<int>(n), lse); break;
    }
    return check_launch("sp_softmax_rows");
}

int sp_softmax_bwd_rows(const float* p, float* dp, int64_t rows, int32_t n, float scale, sp_stream_t stream) {
    if (!sp_softmax_rows_supported(rows, n)) return SP_EINVAL;
    if (rows == 0) return SP_OK;
    if (!p || !dp || p == dp) return SP_EINVAL;
    const dim3 grid(static_cast<unsigned>((rows + LN_ROWS - 1) / LN_ROWS));
    hipStream_t st = static_cast<hipStream_t>(stream);
    const int ni = static_cast<int>(n);
    switch (sm_nv(n)) {
        case 1: launch(0, k_softmax_bwd_rows<1>, grid, dim3(kBlock), st, p, dp, rows, ni, scale); break;
        case 2: launch(0, k_softmax_bwd_rows<2>, grid, dim3(kBlock), st, p, dp, rows, ni, scale); break;
        case 4: launch(0, k_softmax_bwd_rows<4>, grid, dim3(kBlock), st, p, dp, rows, ni, scale); break;
        case 8: launch(0, k_softmax_bwd_rows<8>, grid, dim3(kBlock), st, p, dp, rows, ni, scale); break;
        default: launch(0, k_softmax_bwd_rows<16>, grid, dim3(kBlock), st, p, dp, rows, ni, scale); break;
    }
    return check_launch("sp_softmax_bwd_rows");
}

int sp_conv1x1_small_supported(int32_t cin, int32_t cout, int64_t hw) {
    return ((cin == 4 && cout == 4) || (cin == 8 && cout == 8)) && hw > 0 && hw % 4 == 0;
}

int sp_conv1x1_small(const float* x, const float* w, const float* b, int64_t n, int32_t cin, int32_t cout,
                     int64_t hw, int32_t trans, float* y, sp_stream_t stream) {
    if (!sp_conv1x1_small_supported(cin, cout, hw) || n < 0 || hw >= (int64_t(1) << 31)) return SP_EINVAL;
    if (n == 0) return SP_OK;
    if (!x || !w || !y || x == y || (trans && b)) return SP_EINVAL;
    const int64_t total = n * (hw / 4);
    const dim3 grid(static_cast<unsigned>(std::min<int64_t>((total + kBlock - 1) / kBlock, 4096)));
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (cin == 4)
        launch(0, k_conv1x1_small<4, 4>, grid, dim3(kBlock), st, x, w, b, n, static_cast<int>(hw), trans, y);
    else
        launch(0, k_conv1x1_small<8, 8>, grid, dim3(kBlock), st, x, w, b, n, static_cast<int>(hw), trans, y);
    return check_launch("sp_conv1x1_small");
}

int sp_geglu_fwd(const float* h, int64_t rows, int32_t f, float* y, sp_stream_t stream) {
    if (rows < 0 || f <= 0 || f % 4 || rows * (int64_t)f >= (int64_t(1) << 31)) return SP_EINVAL;
    if (rows == 0) return SP_OK;
    if (!h || !y) return SP_EINVAL;
    const int64_t n4 = rows * (f / 4);
    launch(0, k_geglu_fwd, dim3(stream_grid(n4)), dim3(kBlock), static_cast<hipStream_t>(stream), h, rows,
           static_cast<int>(f), y);
    return check_launch("sp_geglu_fwd");
}

int sp_geglu_bwd(const float* h, const float* dy, int64_t rows, int32_t f, float* dh, sp_stream_t stream) {
    if (rows < 0 || f <= 0 || f % 4 || rows * (int64_t)f >= (int64_t(1) << 31)) return SP_EINVAL;
    if (rows == 0) return SP_OK;
    if (!h || !dy || !dh || dh == h) return SP_EINVAL;
    const int64_t n4 = rows * (f / 4);
    launch(0, k_geglu_bwd, dim3(stream_grid(n4)), dim3(kBlock), static_cast<hipStream_t>(stream), h, dy,
           rows, static_cast<int>(f), dh);
    return check_launch("sp_geglu_bwd");
}

}  // extern "C"

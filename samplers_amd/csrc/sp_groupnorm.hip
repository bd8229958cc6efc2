// GroupNorm (+ optional SiLU, + optional per-(sample, channel) input bias) forward
// and input-VJP for the priors around the hot path: every ResnetBlock of the DDPM
// UNet and of the SD VAE runs norm -> SiLU -> conv, and the UNet adds its time
// embedding right before norm2 (diffusers ResnetBlock2D, called from
// /root/reference/samplers/networks/diffusers/ddpm.py:40-43 and
// stable_diffusion.py:330-345).  PyTorch runs this as RowwiseMoments + GroupNorm
// apply + SiLU (+ the bias add), 4-5 HBM passes forward and ~7 backward; here it
// is 2 kernels each way:
//   fwd: stats  — shifted sums S1 = sum(x - K), S2 = sum((x - K)^2) per chunk
//        apply  — mean/rstd from the group's chunk partials, z = silu(x*a_c + b_c)
//   bwd: stats  — A = sum(dy*gamma), B = sum(dy*gamma*xhat) per chunk (y recomputed)
//        apply  — dx = rstd*(dy*gamma - A/n - xhat*B/n)
// x is NCHW, so one group (sample n, channels g*Cg .. g*Cg+Cg-1) is one contiguous
// run of Cg*HW floats; it is cut into chunks of 16384 floats, one workgroup each, so
// the launch fills the chip even at batch 1.  The shift K is the group's first
// element (removes the cancellation of plain sum/sum-of-squares); chunk partials are
// combined in a fixed order (deterministic).  All four passes are HBM-bound.

#include "sp_common.h"

namespace sp {

constexpr int GN_CHUNK = 16384;  // elements per workgroup

// n / d for 0 <= n < 2^31 by multiply-high (d >= 1).
struct FastDiv {
    uint32_t mul, shr;
};

static FastDiv make_fastdiv(uint32_t d) {
    uint32_t l = 0;
    while ((uint64_t(1) << l) < d) ++l;
    const uint64_t m = ((uint64_t(1) << 32) * ((uint64_t(1) << l) - d)) / d + 1;
    return FastDiv{static_cast<uint32_t>(m), l};
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) {
    return (__umulhi(n, f.mul) + n) >> f.shr;
}

struct GnGeom {
    const float* bias;   // [N, C] added to x before normalisation, or NULL
    const float* gamma;  // [C] or NULL (1)
    const float* beta;   // [C] or NULL (0)
    int C, G, Cg;
    uint32_t gs;         // elements per group
    int chunks;          // workgroups per group
    FastDiv hw_div;      // element (or float4) index in group -> channel in group
    float eps;
    // The input may be the channel concatenation of two tensors, x = cat(x1, x2), x1 with
    // c1 channels (c1hw = c1 * HW elements per sample), x2 with the rest; x2 == NULL: one
    // tensor.  The same split applies to the input gradient (dx1, dx2) and its addends.
    const float* x2;
    uint32_t c1hw, s2;   // elements per sample of x1 and of x2
};

// Element e of group blockIdx.y of a (possibly two-part) NCHW tensor: p1 + e before the
// group's split point, p2 + e after it (a float4 never straddles: HW % 4 == 0 when V = 4).
template <typename T>
struct Parts {
    T* p1;
    T* p2;
    uint32_t split;
    __device__ __forceinline__ T* at(uint32_t e) const { return (e < split ? p1 : p2) + e; }
};

template <typename T>
__device__ __forceinline__ Parts<T> parts_of(T* x1, T* x2, const GnGeom& G) {
    const int64_t gi = blockIdx.y;
    const int64_t n = gi / G.G;
    const int64_t g0 = (gi - n * G.G) * (int64_t)G.gs;  // group start within the sample
    Parts<T> p;
    if (!x2) {
        p.p1 = p.p2 = x1 + gi * (int64_t)G.gs;
        p.split = G.gs;
        return p;
    }
    p.p1 = x1 + n * (int64_t)G.c1hw + g0;
    p.p2 = x2 + n * (int64_t)G.s2 + (g0 - (int64_t)G.c1hw);
    const int64_t sp = (int64_t)G.c1hw - g0;
    p.split = static_cast<uint32_t>(sp < 0 ? 0 : (sp > (int64_t)G.gs ? G.gs : sp));
    return p;
}

__device__ __forceinline__ float silu_f(float y) { return y / (1.f + __expf(-y)); }

// dsilu/dy * dz
__device__ __forceinline__ float silu_bwd(float y, float dz) {
    const float s = 1.f / (1.f + __expf(-y));
    return dz * s * (1.f + y * (1.f - s));
}

// Per-group quantities every kernel needs.
struct GroupCtx {
    int64_t n;             // sample
    int g;                 // group within sample
    Parts<const float> x;  // the group's input elements
    int64_t zoff;          // group base in the (one-part) output / dz tensors
    uint32_t lo, hi;       // this chunk's vector range [lo, hi) in units of V elements
};

template <int V>
__device__ __forceinline__ GroupCtx group_ctx(const float* base, const GnGeom& G) {
    GroupCtx c;
    const int64_t gi = blockIdx.y;
    c.n = gi / G.G;
    c.g = static_cast<int>(gi - c.n * G.G);
    c.x = parts_of<const float>(base, G.x2, G);
    c.zoff = gi * (int64_t)G.gs;
    const uint32_t nv = G.gs / V, per = GN_CHUNK / V;
    c.lo = blockIdx.x * per;
    c.hi = min(nv, c.lo + per);
    return c;
}

template <int V>
__device__ __forceinline__ int chan_of(uint32_t j, const GroupCtx& c, const GnGeom& G) {
    return c.g * G.Cg + static_cast<int>(fdiv(j, G.hw_div));
}

constexpr int GN_UNROLL = 4;

// ---- forward: chunk partial shifted moments ----------------------------------------
template <int V>
__global__ __launch_bounds__(kBlock) void k_gn_stats(const float* __restrict__ x, GnGeom G,
                                                     float* __restrict__ partial) {
    __shared__ float red[8];
    const GroupCtx c = group_ctx<V>(x, G);
    const float K = *c.x.at(0) + (G.bias ? G.bias[c.n * G.C + c.g * G.Cg] : 0.f);
    float s1 = 0.f, s2 = 0.f;
    for (uint32_t j0 = c.lo + threadIdx.x; j0 < c.hi; j0 += GN_UNROLL * kBlock) {
        float v[GN_UNROLL][V];
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
            const uint32_t j = j0 + u * kBlock;
            if (j < c.hi) load_v<V>(c.x.at(j * V), v[u]);
        }
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
            const uint32_t j = j0 + u * kBlock;
            if (j < c.hi) {
                const float b = G.bias ? G.bias[c.n * G.C + chan_of<V>(j, c, G)] : 0.f;
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    const float d = v[u][e] + b - K;
                    s1 += d;
                    s2 = fmaf(d, d, s2);
                }
            }
        }
    }
    s1 = wave_sum(s1);
    s2 = wave_sum(s2);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = s1, red[4 + wid] = s2;
    __syncthreads();
    if (threadIdx.x == 0) {
        float* p = partial + ((int64_t)blockIdx.y * G.chunks + blockIdx.x) * 2;
        p[0] = (red[0] + red[1]) + (red[2] + red[3]);
        p[1] = (red[4] + red[5]) + (red[6] + red[7]);
    }
}

// Sum of the group's chunk partials (pairs), redundantly in every wave.
__device__ __forceinline__ void group_sums(const float* __restrict__ partial, int chunks, float& a,
                                           float& b) {
    const float* p = partial + (int64_t)blockIdx.y * chunks * 2;
    a = 0.f, b = 0.f;
    for (int i = threadIdx.x & 63; i < chunks; i += 64) a += p[2 * i], b += p[2 * i + 1];
    a = wave_sum(a);
    b = wave_sum(b);
}

// ---- forward: normalise + affine (+ SiLU) --------------------------------------------
template <int V, bool ACT>
__global__ __launch_bounds__(kBlock) void k_gn_apply(const float* __restrict__ x, GnGeom G,
                                                     const float* __restrict__ partial,
                                                     float* __restrict__ z,
                                                     float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out) {
    const GroupCtx c = group_ctx<V>(x, G);
    float S1, S2;
    group_sums(partial, G.chunks, S1, S2);
    const float K = *c.x.at(0) + (G.bias ? G.bias[c.n * G.C + c.g * G.Cg] : 0.f);
    const float inv_n = 1.f / static_cast<float>(G.gs);
    const float m1 = S1 * inv_n;
    const float mean = K + m1;
    const float var = fmaxf(S2 * inv_n - m1 * m1, 0.f);
    const float rstd = rsqrtf(var + G.eps);
    if (blockIdx.x == 0 && threadIdx.x == 0) mean_out[blockIdx.y] = mean, rstd_out[blockIdx.y] = rstd;
    float* zg = z + c.zoff;
    for (uint32_t j0 = c.lo + threadIdx.x; j0 < c.hi; j0 += GN_UNROLL * kBlock) {
        float v[GN_UNROLL][V];
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
            const uint32_t j = j0 + u * kBlock;
            if (j < c.hi) load_v<V>(c.x.at(j * V), v[u]);
        }
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
            const uint32_t j = j0 + u * kBlock;
            if (j >= c.hi) continue;
            const int ch = chan_of<V>(j, c, G);
            const float b = G.bias ? G.bias[c.n * G.C + ch] : 0.f;
            const float sc = rstd * (G.gamma ? G.gamma[ch] : 1.f);
            const float sh = (G.beta ? G.beta[ch] : 0.f) - mean * sc;
            float o[V];
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const float y = fmaf(v[u][e] + b, sc, sh);
                o[e] = ACT ? silu_f(y) : y;
            }
            store_v<V>(zg + (size_t)j * V, o);
        }
    }
}

// dy*gamma and xhat for one element group (y recomputed exactly as the forward did).
template <int V, bool ACT>
__device__ __forceinline__ void gn_grad_terms(const float (&v)[V], const float (&dz)[V], float b,
                                              float mean, float rstd, float ga, float be,
                                              float (&gdy)[V], float (&xh)[V]) {
    const float sc = rstd * ga, sh = be - mean * sc;
#pragma unroll
    for (int e = 0; e < V; ++e) {
        const float xb = v[e] + b;
        const float y = fmaf(xb, sc, sh);
        const float dy = ACT ? silu_bwd(y, dz[e]) : dz[e];
        gdy[e] = dy * ga;
        xh[e] = (xb - mean) * rstd;
    }
}

// ---- backward: chunk partials of sum(dy*gamma), sum(dy*gamma*xhat) ------------------
template <int V, bool ACT>
__global__ __launch_bounds__(kBlock) void k_gn_bwd_stats(const float* __restrict__ dz,
                                                         const float* __restrict__ x, GnGeom G,
                                                         const float* __restrict__ mean_in,
                                                         const float* __restrict__ rstd_in,
                                                         float* __restrict__ partial) {
    __shared__ float red[8];
    const GroupCtx c = group_ctx<V>(x, G);
    const float mean = mean_in[blockIdx.y], rstd = rstd_in[blockIdx.y];
    const float* dzg = dz + c.zoff;
    float sa = 0.f, sb = 0.f;
    for (uint32_t j0 = c.lo + threadIdx.x; j0 < c.hi; j0 += GN_UNROLL * kBlock) {
        float v[GN_UNROLL][V], g[GN_UNROLL][V];
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
            const uint32_t j = j0 + u * kBlock;
            if (j < c.hi) {
                load_v<V>(c.x.at(j * V), v[u]);
                load_v<V>(dzg + (size_t)j * V, g[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
            const uint32_t j = j0 + u * kBlock;
            if (j >= c.hi) continue;
            const int ch = chan_of<V>(j, c, G);
            float gdy[V], xh[V];
            gn_grad_terms<V, ACT>(v[u], g[u], G.bias ? G.bias[c.n * G.C + ch] : 0.f, mean, rstd,
                                  G.gamma ? G.gamma[ch] : 1.f, G.beta ? G.beta[ch] : 0.f, gdy, xh);
#pragma unroll
            for (int e = 0; e < V; ++e) {
                sa += gdy[e];
                sb = fmaf(gdy[e], xh[e], sb);
            }
        }
    }
    sa = wave_sum(sa);
    sb = wave_sum(sb);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = sa, red[4 + wid] = sb;
    __syncthreads();
    if (threadIdx.x == 0) {
        float* p = partial + ((int64_t)blockIdx.y * G.chunks + blockIdx.x) * 2;
        p[0] = (red[0] + red[1]) + (red[2] + red[3]);
        p[1] = (red[4] + red[5]) + (red[6] + red[7]);
    }
}

// ---- backward: dx ---------------------------------------------------------------------
template <int V, bool ACT>
__global__ __launch_bounds__(kBlock) void k_gn_bwd_apply(const float* __restrict__ dz,
                                                         const float* __restrict__ x, GnGeom G,
                                                         const float* __restrict__ mean_in,
                                                         const float* __restrict__ rstd_in,
                                                         const float* __restrict__ partial,
                                                         float* __restrict__ dx,
                                                         float* __restrict__ dx2,
                                                         const float* __restrict__ add1,
                                                         const float* __restrict__ add2) {
    const GroupCtx c = group_ctx<V>(x, G);
    float A, B;
    group_sums(partial, G.chunks, A, B);
    const float inv_n = 1.f / static_cast<float>(G.gs);
    const float mA = A * inv_n, mB = B * inv_n;
    const float mean = mean_in[blockIdx.y], rstd = rstd_in[blockIdx.y];
    const float* dzg = dz + c.zoff;
    const Parts<float> dxg = parts_of<float>(dx, G.x2 ? dx2 : nullptr, G);
    const Parts<const float> adg = parts_of<const float>(add1, G.x2 ? add2 : nullptr, G);
    for (uint32_t j0 = c.lo + threadIdx.x; j0 < c.hi; j0 += GN_UNROLL * kBlock) {
        float v[GN_UNROLL][V], g[GN_UNROLL][V];
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
            const uint32_t j = j0 + u * kBlock;
            if (j < c.hi) {
                load_v<V>(c.x.at(j * V), v[u]);
                load_v<V>(dzg + (size_t)j * V, g[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < GN_UNROLL; ++u) {
            const uint32_t j = j0 + u * kBlock;
            if (j >= c.hi) continue;
            const int ch = chan_of<V>(j, c, G);
            float gdy[V], xh[V], o[V];
            gn_grad_terms<V, ACT>(v[u], g[u], G.bias ? G.bias[c.n * G.C + ch] : 0.f, mean, rstd,
                                  G.gamma ? G.gamma[ch] : 1.f, G.beta ? G.beta[ch] : 0.f, gdy, xh);
#pragma unroll
            for (int e = 0; e < V; ++e) o[e] = rstd * (gdy[e] - mA - xh[e] * mB);
            if (add1) {  // dx = GN input VJP + addend (a residual branch's gradient)
                float ad[V];
                load_v<V>(adg.at(j * V), ad);
#pragma unroll
                for (int e = 0; e < V; ++e) o[e] += ad[e];
            }
            store_v<V>(dxg.at(j * V), o);
        }
    }
}

// ---- host side --------------------------------------------------------------------------
static int gn_geom(int64_t n, int32_t c, int64_t hw, int32_t groups, const float* bias,
                   const float* gamma, const float* beta, float eps, GnGeom* G, int* V,
                   dim3* grid) {
    if (n < 0 || c <= 0 || hw <= 0 || groups <= 0 || c % groups) return SP_EINVAL;
    const int64_t gs = (int64_t)(c / groups) * hw;
    if (gs >= (int64_t(1) << 31) || n * groups >= 65536) return SP_EINVAL;
    *V = (hw % 4 == 0) ? 4 : 1;
    G->bias = bias, G->gamma = gamma, G->beta = beta;
    G->C = c, G->G = groups, G->Cg = c / groups;
    G->gs = static_cast<uint32_t>(gs);
    G->chunks = static_cast<int>((gs + GN_CHUNK - 1) / GN_CHUNK);
    G->hw_div = make_fastdiv(static_cast<uint32_t>(hw / *V));
    G->eps = eps;
    G->x2 = nullptr;
    G->c1hw = static_cast<uint32_t>(c * hw);
    G->s2 = 0;
    *grid = dim3(G->chunks, static_cast<unsigned>(n * groups));
    return SP_OK;
}

}  // namespace sp

using namespace sp;

extern "C" {

int64_t sp_groupnorm_workspace(int64_t n, int32_t channels, int64_t hw, int32_t groups) {
    if (n < 0 || channels <= 0 || hw <= 0 || groups <= 0 || channels % groups) return -1;
    const int64_t gs = (int64_t)(channels / groups) * hw;
    return n * groups * ((gs + GN_CHUNK - 1) / GN_CHUNK) * 2;
}

// second part of a channel-concatenated input: x2 != NULL holds channels c1 .. channels-1
static int gn_split(GnGeom* G, const float* x2, int32_t c1, int32_t channels, int64_t hw) {
    if (!x2) return SP_OK;
    if (c1 <= 0 || c1 >= channels || (int64_t)channels * hw >= (int64_t(1) << 31)) return SP_EINVAL;
    G->x2 = x2;
    G->c1hw = static_cast<uint32_t>(c1 * hw);
    G->s2 = static_cast<uint32_t>((channels - c1) * hw);
    return SP_OK;
}

int sp_groupnorm_silu_fwd(const float* x, const float* chan_bias, const float* gamma,
                          const float* beta, int64_t n, int32_t channels, int64_t hw,
                          int32_t groups, float eps, int32_t act, float* z, float* mean,
                          float* rstd, float* work, sp_stream_t stream) {
    return sp_groupnorm_silu_fwd2(x, nullptr, channels, chan_bias, gamma, beta, n, channels, hw,
                                  groups, eps, act, z, mean, rstd, work, stream);
}

int sp_groupnorm_silu_fwd2(const float* x, const float* x2, int32_t c1, const float* chan_bias,
                           const float* gamma, const float* beta, int64_t n, int32_t channels,
                           int64_t hw, int32_t groups, float eps, int32_t act, float* z,
                           float* mean, float* rstd, float* work, sp_stream_t stream) {
    GnGeom G;
    int V;
    dim3 grid;
    int rc = gn_geom(n, channels, hw, groups, chan_bias, gamma, beta, eps, &G, &V, &grid);
    if (rc == SP_OK) rc = gn_split(&G, x2, c1, channels, hw);
    if (rc != SP_OK) return rc;
    if (n == 0) return SP_OK;  // empty batch: nothing to read or write
    if (!x || !z || !mean || !rstd || !work) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 blk(kBlock);
    if (V == 4) {
        launch(0, k_gn_stats<4>, grid, blk, s, x, G, work);
        if (act) launch(0, k_gn_apply<4, true>, grid, blk, s, x, G, (const float*)work, z, mean, rstd);
        else launch(0, k_gn_apply<4, false>, grid, blk, s, x, G, (const float*)work, z, mean, rstd);
    } else {
        launch(0, k_gn_stats<1>, grid, blk, s, x, G, work);
        if (act) launch(0, k_gn_apply<1, true>, grid, blk, s, x, G, (const float*)work, z, mean, rstd);
        else launch(0, k_gn_apply<1, false>, grid, blk, s, x, G, (const float*)work, z, mean, rstd);
    }
    return check_launch("sp_groupnorm_silu_fwd");
}

int sp_groupnorm_silu_bwd(const float* dz, const float* x, const float* chan_bias,
                          const float* gamma, const float* beta, const float* mean,
                          const float* rstd, int64_t n, int32_t channels, int64_t hw,
                          int32_t groups, int32_t act, float* dx, float* work,
                          sp_stream_t stream) {
    return sp_groupnorm_silu_bwd2(dz, x, nullptr, channels, chan_bias, gamma, beta, mean, rstd,
                                  n, channels, hw, groups, act, dx, nullptr, nullptr, nullptr,
                                  work, stream);
}

int sp_groupnorm_silu_bwd2(const float* dz, const float* x, const float* x2, int32_t c1,
                           const float* chan_bias, const float* gamma, const float* beta,
                           const float* mean, const float* rstd, int64_t n, int32_t channels,
                           int64_t hw, int32_t groups, int32_t act, float* dx, float* dx2,
                           const float* add1, const float* add2, float* work,
                           sp_stream_t stream) {
    GnGeom G;
    int V;
    dim3 grid;
    int rc = gn_geom(n, channels, hw, groups, chan_bias, gamma, beta, 0.f, &G, &V, &grid);
    if (rc == SP_OK) rc = gn_split(&G, x2, c1, channels, hw);
    if (rc != SP_OK) return rc;
    if (n == 0) return SP_OK;
    if (!dz || !x || !mean || !rstd || !dx || !work || (x2 && !dx2) || (x2 && add1 && !add2))
        return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 blk(kBlock);
#define SP_GN_BWD(VV, AA)                                                                      \
    launch(0, k_gn_bwd_stats<VV, AA>, grid, blk, s, dz, x, G, mean, rstd, work);              \
    launch(0, k_gn_bwd_apply<VV, AA>, grid, blk, s, dz, x, G, mean, rstd, (const float*)work, dx, \
           dx2, add1, add2)
    if (V == 4) {
        if (act) { SP_GN_BWD(4, true); } else { SP_GN_BWD(4, false); }
    } else {
        if (act) { SP_GN_BWD(1, true); } else { SP_GN_BWD(1, false); }
    }
#undef SP_GN_BWD
    return check_launch("sp_groupnorm_silu_bwd");
}

}  // extern "C"

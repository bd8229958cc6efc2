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
// run of Cg*HW floats; it is cut into chunks (8192-16384 floats, see GN_CHUNK_*), one
// workgroup each, so the launch fills the chip even at batch 1.  Where the input is
// float4-aligned, single-pass variants of both directions (below) replace the pairs.  The shift K is the group's first
// element (removes the cancellation of plain sum/sum-of-squares); chunk partials are
// combined in a fixed order (deterministic).  All four passes are HBM-bound.

#define SP_TU 4  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

#include <algorithm>
#include <utility>

// No implicit mul+add contraction: which products the backend fuses depends on the code
// around them, and the single-pass and two-pass kernels must round identically.
#pragma clang fp contract(off)

namespace sp {

// Elements per workgroup (chunk).  Forward: 16384 for groups of >= 2^17 elements, 8192 below
// (fewer, larger chunks stream better on big groups; small groups need the chunks to fill the
// chip); backward: 8192.  Measured on the UNet's shapes (tools/bench_gn.py, MI355X).  The
// chunk is a function of the shape only, so every path over one call sums in the same order.
#ifndef SP_GN_CHUNK_FWD_BIG
#define SP_GN_CHUNK_FWD_BIG 16384
#endif
#ifndef SP_GN_CHUNK_FWD
#define SP_GN_CHUNK_FWD 8192
#endif
#ifndef SP_GN_CHUNK_BWD
#define SP_GN_CHUNK_BWD 8192
#endif
#ifndef SP_GN_FWD_WPC
#define SP_GN_FWD_WPC 2  // workgroups per CU the single-pass forward is compiled for
#endif
#ifndef SP_GN_BWD_WPC
#define SP_GN_BWD_WPC 2  // ... and the single-pass input VJP
#endif
constexpr int GN_CHUNK_FWD_BIG = SP_GN_CHUNK_FWD_BIG, GN_CHUNK_FWD = SP_GN_CHUNK_FWD,
              GN_CHUNK_BWD = SP_GN_CHUNK_BWD;
constexpr int GN_FWD_BIG_GROUP = 1 << 17;
constexpr int GN_CHUNK_MIN = GN_CHUNK_FWD < GN_CHUNK_BWD ? GN_CHUNK_FWD : GN_CHUNK_BWD;
static_assert(GN_CHUNK_FWD_BIG >= GN_CHUNK_MIN, "workspace sizing");

static int gn_fwd_chunk(int64_t gs) { return gs >= GN_FWD_BIG_GROUP ? GN_CHUNK_FWD_BIG : GN_CHUNK_FWD; }

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
    uint32_t chunk;      // elements per workgroup (GN_CHUNK_FWD / _BWD)
    int chunks;          // workgroups per group
    FastDiv hw_div;      // element (or float4) index in group -> channel in group
    float eps;
    // The input may be the channel concatenation of two tensors, x = cat(x1, x2), x1 with
    // c1 channels (c1hw = c1 * HW elements per sample), x2 with the rest; x2 == NULL: one
    // tensor.  The same split applies to the input gradient (dx1, dx2) and its addends.
    const float* x2;
    uint32_t c1hw, s2;   // elements per sample of x1 and of x2
    // input VJP only: a second addend (one-part inputs), added after add1 — a UNet skip
    // tensor's gradient from its up-block consumer, instead of an autograd accumulation add
    const float* add1b;
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
__device__ __forceinline__ Parts<T> parts_at(T* x1, T* x2, const GnGeom& G, int64_t gi) {
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

template <typename T>
__device__ __forceinline__ Parts<T> parts_of(T* x1, T* x2, const GnGeom& G) {
    return parts_at<T>(x1, x2, G, blockIdx.y);
}

// The logistic as v_exp + v_rcp (1 ulp) instead of an IEEE division (a ten-instruction
// sequence per element in kernels that do little else per element).
__device__ __forceinline__ float sigmoid_f(float y) { return __builtin_amdgcn_rcpf(1.f + __expf(-y)); }

__device__ __forceinline__ float silu_f(float y) { return y * sigmoid_f(y); }

// dsilu/dy * dz
__device__ __forceinline__ float silu_bwd(float y, float dz) {
    const float s = sigmoid_f(y);
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
__device__ __forceinline__ GroupCtx group_ctx_at(const float* base, const GnGeom& G, int64_t gi,
                                                 uint32_t chunk) {
    GroupCtx c;
    c.n = gi / G.G;
    c.g = static_cast<int>(gi - c.n * G.G);
    c.x = parts_at<const float>(base, G.x2, G, gi);
    c.zoff = gi * (int64_t)G.gs;
    const uint32_t nv = G.gs / V, per = G.chunk / V;
    c.lo = chunk * per;
    c.hi = min(nv, c.lo + per);
    SP_DCHECK(chunk < static_cast<uint32_t>(G.chunks) && c.lo < nv && G.chunk % V == 0 && c.g < G.G);
    return c;
}

template <int V>
__device__ __forceinline__ GroupCtx group_ctx(const float* base, const GnGeom& G) {
    return group_ctx_at<V>(base, G, blockIdx.y, blockIdx.x);
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
            if (G.add1b) {  // + the skip gradient (one-part inputs)
                float ad[V];
                load_v<V>(G.add1b + c.zoff + (size_t)j * V, ad);
#pragma unroll
                for (int e = 0; e < V; ++e) o[e] += ad[e];
            }
            store_v<V>(dxg.at(j * V), o);
        }
    }
}


// ---- single-pass kernels: one team of workgroups per group -------------------------------
// The two-pass kernels read their inputs twice (forward: x for the moments, then x again to
// normalise; backward: x and dz for the two sums, then again for dx).  Here the workgroups of
// a team (one per chunk of the group) keep their chunk in registers across the group
// reduction: each publishes its chunk partials as two 64-bit words {value, 1} with
// agent-scope atomic stores (coherent across the XCDs' L2s, no cache flush), then polls the
// team's words until all are present (the words are zeroed before the launch).  The grid is
// persistent and no larger than the chip's resident capacity, so a team's members are
// resident together; each team walks groups gi = team, team + nteams, ...  A workgroup keeps
// two groups in flight: once a group's partials are published, the poll of the team's words
// is ISSUED FIRST and the next group's chunk is loaded right behind it, so the wait for the
// team (a cross-XCD hand-off: 1.5-3 us under load, against ~8 us of streaming per group)
// overlaps the next chunk's HBM traffic — the poll's result is older than the prefetch, so
// the wait for it leaves the prefetch in flight.  Chunking, the per-thread element order and
// the summation order are those of the two-pass kernels, so the results are bit-identical.
// HBM traffic: forward 2 passes (was 3), backward 3 + the addends (was 5 + the addends).
// Poll bound: a member still absent after this many polls (~5-20 ms) is taken to be missing
// (not resident: another process or stream holds CUs, so the grid's co-residency assumption
// failed) and the waiting workgroup recomputes that member's chunk partials itself from the
// chunk's inputs, in the member's own element order and block reduction — bit-identical to
// what the member publishes.  The result is therefore exact whatever the residency; a missing
// member costs one extra read of its chunk.  g_gnt_spin_limit overrides the bound
// (sp_groupnorm_set_spin_limit; 0 = recompute every word not present at the first poll, which
// tests use to exercise the recompute path).
constexpr int GNT_MAX_SPINS = 1 << 16;

__device__ unsigned int g_gnt_timeouts;  // chunk partials recomputed (sp_groupnorm_team_timeouts)
__device__ int g_gnt_spin_limit = GNT_MAX_SPINS;

__device__ __forceinline__ void gnt_publish(uint64_t* slot, float a, float b) {
    __hip_atomic_store(slot, (uint64_t(1) << 32) | __float_as_uint(a), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(slot + 1, (uint64_t(1) << 32) | __float_as_uint(b), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int GNT_MAX_CHUNKS = 256;  // chunks per group (words polled per team)

// Self-cleaning words (the slot region is all zero again when a launch ends, so the next
// launch needs no memset).  A team walks its groups in step: a member publishes group g's words
// only after it has read all of the previous group's, so once a member has read all of g's words
// nobody reads the previous group's any more, and it clears its own two words of that group
// (plain stores, nothing waited for).  The last group's words are cleared by the member that
// counts itself out of the team last (one returning atomic per workgroup and launch).  With a
// member that timed out, words may be cleared before it read them: it then recomputes those
// partials as it does for any absent word, and still clears its own words afterwards.
__device__ __forceinline__ void gnt_clear_own(uint64_t* slots, int chunks, int64_t gprev, uint32_t m) {
    if (gprev >= 0 && threadIdx.x == 0) {
        uint64_t* w = slots + (gprev * chunks + m) * 2;
        __hip_atomic_store(w, uint64_t(0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(w + 1, uint64_t(0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__device__ __forceinline__ void gnt_release_last(uint64_t* slots, int* done, int chunks, int64_t glast,
                                                 int64_t team) {
    if (threadIdx.x >= 64) return;  // wave 0
    int old = 0;
    if (threadIdx.x == 0)
        old = __hip_atomic_fetch_add(done + team, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__builtin_amdgcn_readfirstlane(old) != chunks - 1) return;
    uint64_t* w = slots + glast * chunks * 2;
    for (int i = threadIdx.x; i < 2 * chunks; i += 64)
        __hip_atomic_store(w + i, uint64_t(0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0) __hip_atomic_store(done + team, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Block-reduce (a, b) as the two-pass kernels do and publish them as chunk m's words.
// threadIdx.x re-read opaque to the compiler: values derived from it (LDS addresses, buffer
// offsets) are then formed where they are used instead of being held live across a group —
// in the VJP kernel (256 VGPRs: two groups' chunks and the addends in flight) such values were
// spilled to scratch, and each reload's vmcnt(0) waited for the next group's chunk loads
// (OPQ = false: the plain index, the forward kernels' form, which did not spill and measured
// ~1 % faster with it)
template <bool OPQ = true>
__device__ __forceinline__ int gn_tid() {
    int t = threadIdx.x;
    if constexpr (OPQ) asm volatile("" : "+v"(t));
    return t;
}

__device__ __forceinline__ void gnt_reduce_publish(float a, float b, float* red, uint64_t* slot) {
    a = wave_sum(a);
    b = wave_sum(b);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) red[wid] = a, red[4 + wid] = b;
    __syncthreads();
    if (threadIdx.x == 0) gnt_publish(slot, (red[0] + red[1]) + (red[2] + red[3]),
                                      (red[4] + red[5]) + (red[6] + red[7]));
}

// A chunk's elements in one tensor part (the single-pass kernels require that no chunk straddles
// the two parts of a concatenated input): buffer resource over the chunk's first `lim`
// float4 of the group, so accesses past the chunk end read 0 / are dropped.  The range
// check covers the VGPR offset only (not soffset), so a thread's float4 i is addressed as
// voffset (lo + tid + i * kBlock) * 16.
template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t gnt_rsrc(const Parts<T>& p, uint32_t lo, uint32_t lim) {
    // a group straddling the two parts is served when the split falls on a chunk boundary
    // (the host checks): the chunk [lo, lim) then lies in one part
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(lo * 4u < p.split ? p.p1 : p.p2), (short)0,
                                             lim * 16, 0x00020000);
}

typedef float gnt_f4 __attribute__((ext_vector_type(4)));

#ifndef SP_GN_NTL
#define SP_GN_NTL 2  // cache-policy bits of the chunk loads: non-temporal (once-read streams)
#endif
__device__ __forceinline__ void gnt_load(__amdgpu_buffer_rsrc_t r, uint32_t vo, int i, float (&d)[4]) {
    const gnt_f4 t = __builtin_bit_cast(
        gnt_f4, __builtin_amdgcn_raw_buffer_load_b128(r, vo + i * kBlock * 16, 0, SP_GN_NTL));
    d[0] = t[0], d[1] = t[1], d[2] = t[2], d[3] = t[3];
}

#ifndef SP_GN_NT
#define SP_GN_NT 2  // non-temporal output stores.  With non-temporal loads as well: GroupNorm
                    // -8 / -9 % (fwd / VJP) and the DPS step +1.4 % (profiles/round3/wino/
                    // xi_ab.txt); non-temporal stores alone measured -0.9 % in round 2
#endif
__device__ __forceinline__ void gnt_store(__amdgpu_buffer_rsrc_t r, uint32_t vo, int i, const float (&d)[4]) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, gnt_f4{d[0], d[1], d[2], d[3]}), r,
                                           vo + i * kBlock * 16, 0, SP_GN_NT);
}

// The group's per-channel gamma / beta / bias come along with its chunk (one value per thread
// t < Cg) and are read from a double-buffered LDS table.
constexpr int GNP_MAX_CG = 128;  // channels per group the LDS table holds

struct GnpBuf {  // one group's per-thread prefetch state besides the chunk itself
    float ga, be, bi;  // thread t < Cg: gamma / beta / bias of the group's channel t
    float kx, kb;      // the group's first element and that channel's bias: the shift K is
                       // their sum, formed where it is used (forming it here would wait for
                       // the whole prefetch)
};

// Issue the loads of group gi's chunk m and its per-channel state.  live == false: the chunk
// loads get an empty range (no memory access, zeros) — the caller issues them anyway so that
// the code after the prefetch has one path (see gnp_poll_finish).
template <int PER, bool OPQ = false>
__device__ __forceinline__ void gnp_issue(const float* __restrict__ base, const GnGeom& G,
                                          int64_t gi, uint32_t m, float (&v)[PER][4], GnpBuf& b,
                                          bool live = true) {
    const GroupCtx c = group_ctx_at<4>(base, G, gi, m);
    const auto r = gnt_rsrc(c.x, c.lo, live ? c.hi : 0u);
    const uint32_t vo = (c.lo + gn_tid<OPQ>()) * 16;
#pragma unroll
    for (int i = 0; i < PER; ++i) gnt_load(r, vo, i, v[i]);
    // every thread loads, from the input itself where a table is absent (threads t >= Cg
    // re-read the last channel): no branch around a load, see above
    const int ch = c.g * G.Cg + min(static_cast<int>(threadIdx.x), G.Cg - 1);
    const float ga = (G.gamma ? G.gamma : base)[ch];
    const float be = (G.beta ? G.beta : base)[ch];
    const float bi = (G.bias ? G.bias : base)[c.n * G.C + ch];
    b.ga = G.gamma ? ga : 1.f;
    b.be = G.beta ? be : 0.f;
    b.bi = G.bias ? bi : 0.f;
    b.kx = *c.x.at(0);
    const float kb = (G.bias ? G.bias : base)[c.n * G.C + c.g * G.Cg];
    b.kb = G.bias ? kb : 0.f;
}

// Poll words of a team: every thread issues its loads (threads past the team re-read word 0),
// so the loads precede anything issued after this call.
template <bool OPQ = false>
__device__ __forceinline__ void gnp_poll_issue(const uint64_t* slots, int chunks, uint64_t& wa,
                                               uint64_t& wb) {
    const int tt = gn_tid<OPQ>(), t = tt < chunks ? tt : 0;
    wa = __hip_atomic_load(slots + 2 * t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    wb = __hip_atomic_load(slots + 2 * t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Finish the poll (threads t < chunks spin on their words) and form the team's sums as
// gnt_sums does.  Every thread tests its issued words first, outside any branch and loop: the
// wait for them then leaves the younger prefetch loads in flight (at a loop header or a join
// the compiler merges paths and waits for everything).  Words still absent after the poll
// bound are recomputed by the whole workgroup with `recompute(mm, a, b)` (a block-wide call
// that leaves chunk mm's two partials in thread 0's a, b).
template <bool OPQ = false, typename Recompute>
__device__ __forceinline__ void gnp_poll_finish(const uint64_t* slots, int chunks, uint64_t wa,
                                                uint64_t wb, float* sv, int* miss, float& a,
                                                float& b, Recompute recompute) {
    const int t = gn_tid<OPQ>();
    bool ready = (wa >> 32) && (wb >> 32);
    if (t == 0) miss[GNT_MAX_CHUNKS] = 0;
    if ((t < chunks) & !ready) {
        const int limit = g_gnt_spin_limit;
#pragma nounroll
        for (int spins = 0; spins < limit; ++spins) {
            __builtin_amdgcn_s_sleep(2);
            wa = __hip_atomic_load(slots + 2 * t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            wb = __hip_atomic_load(slots + 2 * t + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ready = (wa >> 32) && (wb >> 32);
            if (ready) break;
        }
    }
    __syncthreads();  // miss[] count cleared before any thread records a missing word
    if (t < chunks) {
        sv[t] = __uint_as_float(static_cast<uint32_t>(wa));
        sv[GNT_MAX_CHUNKS + t] = __uint_as_float(static_cast<uint32_t>(wb));
        if (!ready) miss[atomicAdd(&miss[GNT_MAX_CHUNKS], 1)] = t;
    }
    __syncthreads();
    const int nmiss = miss[GNT_MAX_CHUNKS];
    if (nmiss) {  // rare (block-uniform): a team member did not publish in time
        if (t == 0) atomicAdd(&g_gnt_timeouts, static_cast<unsigned>(nmiss));
        for (int q = 0; q < nmiss; ++q) {
            const int mm = miss[q];
            float ra, rb;
            recompute(mm, ra, rb);
            if (t == 0) sv[mm] = ra, sv[GNT_MAX_CHUNKS + mm] = rb;
            __syncthreads();
        }
    }
    a = 0.f, b = 0.f;
    for (int i = t & 63; i < chunks; i += 64) a += sv[i], b += sv[GNT_MAX_CHUNKS + i];
    a = wave_sum(a);
    b = wave_sum(b);
}

// Block-reduce (a, b) exactly as gnt_reduce_publish does; thread 0 gets the chunk's words.
__device__ __forceinline__ void gnt_reduce_local(float& a, float& b, float* red) {
    a = wave_sum(a);
    b = wave_sum(b);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();  // red[] may still be read by a previous reduction
    if (lane == 0) red[wid] = a, red[4 + wid] = b;
    __syncthreads();
    a = (red[0] + red[1]) + (red[2] + red[3]);
    b = (red[4] + red[5]) + (red[6] + red[7]);
}

// Forward chunk mm's shifted moments, recomputed from x (the terms and order of gnp_fwd_group).
template <int PER>
__device__ __forceinline__ void gnp_fwd_recompute(const float* __restrict__ x, const GnGeom& G,
                                               int64_t gi, uint32_t mm, float K,
                                               const float (*tab)[GNP_MAX_CG], float* red,
                                               float& a, float& b) {
    const int t = threadIdx.x;
    const GroupCtx c = group_ctx_at<4>(x, G, gi, mm);
    const auto r = gnt_rsrc(c.x, c.lo, c.hi);
    const uint32_t vo = (c.lo + t) * 16;
    float s1 = 0.f, s2 = 0.f;
#pragma nounroll
    for (int i = 0; i < PER; ++i) {
        float v[4];
        gnt_load(r, vo, i, v);
        const uint32_t j = c.lo + t + i * kBlock;
        const bool in = j < c.hi;
        const float bb = G.bias ? tab[2][fdiv(in ? j : c.lo, G.hw_div)] : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float d = in ? v[e] + bb - K : 0.f;
            s1 += d;
            s2 = fmaf(d, d, s2);
        }
    }
    gnt_reduce_local(s1, s2, red);
    a = s1, b = s2;
}

// One forward group: chunk v (loaded), state bf; prefetches group gn (< 0: none) into vn / bn.
template <bool ACT, int PER>
__device__ __forceinline__ void gnp_fwd_group(const float* __restrict__ x, const GnGeom& G,
                                              uint64_t* __restrict__ slots, int64_t gi, int64_t gn,
                                              uint32_t m, float (&v)[PER][4], const GnpBuf& bf,
                                              float (&vn)[PER][4], GnpBuf& bn, float (*tab)[GNP_MAX_CG],
                                              float* red, float* sv, int* miss, float* __restrict__ z,
                                              float* __restrict__ mean_out,
                                              float* __restrict__ rstd_out, int64_t gprev) {
    const int t = threadIdx.x;
    const GroupCtx c = group_ctx_at<4>(x, G, gi, m);
    SP_DCHECK(G.Cg <= GNP_MAX_CG);  // the group's channels fit the LDS table
    if (t < G.Cg) tab[0][t] = bf.ga, tab[1][t] = bf.be, tab[2][t] = bf.bi;
    __syncthreads();
    const float K = bf.kx + bf.kb;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint32_t j = c.lo + t + i * kBlock;
        const bool in = j < c.hi;  // past the chunk end: adds exact zeros
        const float b = G.bias ? tab[2][fdiv(in ? j : c.lo, G.hw_div)] : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float d = in ? v[i][e] + b - K : 0.f;
            s1 += d;
            s2 = fmaf(d, d, s2);
        }
    }
    uint64_t* gslots = slots + gi * G.chunks * 2;
    gnt_reduce_publish(s1, s2, red, gslots + 2 * m);
    uint64_t wa, wb;
    gnp_poll_issue(gslots, G.chunks, wa, wb);
    gnp_issue<PER>(x, G, gn >= 0 ? gn : gi, m, vn, bn, gn >= 0);
    float S1, S2;
    gnp_poll_finish(gslots, G.chunks, wa, wb, sv, miss, S1, S2, [&](int mm, float& ra, float& rb) {
        gnp_fwd_recompute<PER>(x, G, gi, static_cast<uint32_t>(mm), K, tab, red, ra, rb);
    });
    const float inv_n = 1.f / static_cast<float>(G.gs);
    const float m1 = S1 * inv_n;
    const float mean = K + m1;
    const float var = fmaxf(S2 * inv_n - m1 * m1, 0.f);
    const float rstd = rsqrtf(var + G.eps);
    if (m == 0 && t == 0) mean_out[gi] = mean, rstd_out[gi] = rstd;
    const Parts<float> zp{z + c.zoff, z + c.zoff, G.gs};
    const auto rz = gnt_rsrc(zp, c.lo, c.hi);
    const uint32_t vo = (c.lo + t) * 16;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint32_t j = c.lo + t + i * kBlock;
        const uint32_t cl = fdiv(j < c.hi ? j : c.lo, G.hw_div);
        const float b = G.bias ? tab[2][cl] : 0.f;
        const float sc = rstd * tab[0][cl];
        const float sh = tab[1][cl] - mean * sc;
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const float y = fmaf(v[i][e] + b, sc, sh);
            o[e] = ACT ? silu_f(y) : y;
        }
        gnt_store(rz, vo, i, o);  // past the chunk end: dropped
    }
    gnt_clear_own(slots, G.chunks, gprev, m);
}

template <bool ACT, int PER>
__global__ __launch_bounds__(kBlock, SP_GN_FWD_WPC) void k_gn_fwd_pipe(const float* __restrict__ x, GnGeom G,
                                                           uint64_t* __restrict__ slots, int* done, int nteams,
                                                           int64_t ngroups, float* __restrict__ z,
                                                           float* __restrict__ mean_out,
                                                           float* __restrict__ rstd_out) {
    __shared__ float red[8];
    __shared__ float sv[2 * GNT_MAX_CHUNKS];
    __shared__ int miss[GNT_MAX_CHUNKS + 1];
    __shared__ float tab[2][3][GNP_MAX_CG];
    const uint32_t m = blockIdx.x % G.chunks;
    int64_t gi = blockIdx.x / G.chunks;
    if (gi >= ngroups) return;
    // a chunk fits the registers the kernel was built for; the team words of every group it
    // visits lie in the region sized for ngroups
    SP_DCHECK(G.chunk / 4 <= PER * kBlock && G.chunks <= GNT_MAX_CHUNKS && nteams > 0);
    float va[PER][4], vb[PER][4];
    GnpBuf ba, bb;
    const int64_t team = gi;
    gnp_issue<PER>(x, G, gi, m, va, ba);
    for (;;) {  // two groups per trip: the register buffers are named, not indexed
        int64_t gn = gi + nteams < ngroups ? gi + nteams : -1;
        gnp_fwd_group<ACT, PER>(x, G, slots, gi, gn, m, va, ba, vb, bb, tab[0], red, sv, miss, z,
                                mean_out, rstd_out, gi - nteams);
        if (gn < 0) break;
        gi = gn;
        gn = gi + nteams < ngroups ? gi + nteams : -1;
        gnp_fwd_group<ACT, PER>(x, G, slots, gi, gn, m, vb, bb, va, ba, tab[1], red, sv, miss, z,
                                mean_out, rstd_out, gi - nteams);
        if (gn < 0) break;
        gi = gn;
    }
    gnt_release_last(slots, done, G.chunks, gi, team);
}

// Backward chunk mm's sums of dy*gamma and dy*gamma*xhat, recomputed from x and dz (the terms
// and order of gnp_bwd_group).
template <bool ACT, int PER>
__device__ __forceinline__ void gnp_bwd_recompute(const float* __restrict__ dz,
                                               const float* __restrict__ x, const GnGeom& G,
                                               int64_t gi, uint32_t mm, float mean, float rstd,
                                               const float (*tab)[GNP_MAX_CG], float* red,
                                               float& a, float& b) {
    const int t = threadIdx.x;
    const GroupCtx c = group_ctx_at<4>(x, G, gi, mm);
    const auto r = gnt_rsrc(c.x, c.lo, c.hi);
    const auto rg = gnt_rsrc(Parts<const float>{dz + c.zoff, dz + c.zoff, G.gs}, c.lo, c.hi);
    const uint32_t vo = (c.lo + t) * 16;
    float sa = 0.f, sb = 0.f;
#pragma nounroll
    for (int i = 0; i < PER; ++i) {
        float v[4], g[4];
        gnt_load(r, vo, i, v);
        gnt_load(rg, vo, i, g);
        const uint32_t j = c.lo + t + i * kBlock;
        const bool in = j < c.hi;
        const uint32_t cl = fdiv(in ? j : c.lo, G.hw_div);
        float gdy[4], xh[4];
        gn_grad_terms<4, ACT>(v, g, G.bias ? tab[2][cl] : 0.f, mean, rstd, tab[0][cl], tab[1][cl],
                              gdy, xh);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            sa += in ? gdy[e] : 0.f;
            sb = fmaf(in ? gdy[e] : 0.f, xh[e], sb);
        }
    }
    gnt_reduce_local(sa, sb, red);
    a = sa, b = sb;
}

// One backward group: x chunk v and dz chunk g (loaded); prefetches group gn into vn / gq.
template <bool ACT, int PER>
__device__ __forceinline__ void gnp_bwd_group(
    const float* __restrict__ dz, const float* __restrict__ x, const GnGeom& G,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    uint64_t* __restrict__ slots, int64_t gi, int64_t gn, uint32_t m, float (&v)[PER][4],
    float (&g)[PER][4], const GnpBuf& bf, float (&vn)[PER][4], float (&gq)[PER][4], GnpBuf& bn,
    float (*tab)[GNP_MAX_CG], float* red, float* sv, int* miss, float* __restrict__ dx,
    float* __restrict__ dx2, const float* __restrict__ add1, const float* __restrict__ add2,
    int64_t gprev) {
    const int t = threadIdx.x;
    const GroupCtx c = group_ctx_at<4>(x, G, gi, m);
    SP_DCHECK(G.Cg <= GNP_MAX_CG);  // the group's channels fit the LDS table
    if (t < G.Cg) tab[0][t] = bf.ga, tab[1][t] = bf.be, tab[2][t] = bf.bi;
    __syncthreads();
    const float mean = mean_in[gi], rstd = rstd_in[gi];
    // v, g are replaced by xhat and dy*gamma: the dx pass needs nothing else
    float sa = 0.f, sb = 0.f;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const uint32_t j = c.lo + t + i * kBlock;
        const bool in = j < c.hi;  // past the chunk end: adds exact zeros
        const uint32_t cl = fdiv(in ? j : c.lo, G.hw_div);
        float gdy[4], xh[4];
        gn_grad_terms<4, ACT>(v[i], g[i], G.bias ? tab[2][cl] : 0.f, mean, rstd, tab[0][cl],
                              tab[1][cl], gdy, xh);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            sa += in ? gdy[e] : 0.f;
            sb = fmaf(in ? gdy[e] : 0.f, xh[e], sb);
            g[i][e] = gdy[e];
            v[i][e] = xh[e];
        }
    }
    uint64_t* gslots = slots + gi * G.chunks * 2;
    gnt_reduce_publish(sa, sb, red, gslots + 2 * m);
    // the addends of this group, issued before the poll and the prefetch (an absent addend
    // gets an empty range: zeros, no memory access, no branch around the loads)
    const uint32_t vo = (c.lo + t) * 16;
    float a1[PER][4], a1b[PER][4];
    {
        const auto ra = gnt_rsrc(parts_at<const float>(add1 ? add1 : x, G.x2 ? (add1 ? add2 : x) : nullptr,
                                                       G, gi), c.lo, add1 ? c.hi : 0u);
        const Parts<const float> abp{(G.add1b ? G.add1b : x) + c.zoff, (G.add1b ? G.add1b : x) + c.zoff,
                                     G.gs};
        const auto rb = gnt_rsrc(abp, c.lo, G.add1b ? c.hi : 0u);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            gnt_load(ra, vo, i, a1[i]);
            gnt_load(rb, vo, i, a1b[i]);
        }
    }
    uint64_t wa, wb;
    gnp_poll_issue<true>(gslots, G.chunks, wa, wb);
    {
        const int64_t gq_i = gn >= 0 ? gn : gi;
        gnp_issue<PER, true>(x, G, gq_i, m, vn, bn, gn >= 0);
        const auto rg = gnt_rsrc(Parts<const float>{dz + gq_i * (int64_t)G.gs,
                                                    dz + gq_i * (int64_t)G.gs, G.gs},
                                 c.lo, gn >= 0 ? c.hi : 0u);
#pragma unroll
        for (int i = 0; i < PER; ++i) gnt_load(rg, vo, i, gq[i]);
    }
    float A, B;
    gnp_poll_finish<true>(gslots, G.chunks, wa, wb, sv, miss, A, B, [&](int mm, float& ra, float& rb) {
        gnp_bwd_recompute<ACT, PER>(dz, x, G, gi, static_cast<uint32_t>(mm), mean, rstd, tab, red,
                                    ra, rb);
    });
    const float inv_n = 1.f / static_cast<float>(G.gs);
    const float mA = A * inv_n, mB = B * inv_n;
    const auto rd = gnt_rsrc(parts_at<float>(dx, G.x2 ? dx2 : nullptr, G, gi), c.lo, c.hi);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rstd * (g[i][e] - mA - v[i][e] * mB);
        if (add1) {  // as k_gn_bwd_apply (same rounding)
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] += a1[i][e];
        }
        if (G.add1b) {  // + the skip gradient, as k_gn_bwd_apply
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] += a1b[i][e];
        }
        gnt_store(rd, vo, i, o);
    }
    gnt_clear_own(slots, G.chunks, gprev, m);
}

template <bool ACT, int PER>
__global__ __launch_bounds__(kBlock, SP_GN_BWD_WPC) void k_gn_bwd_pipe(
    const float* __restrict__ dz, const float* __restrict__ x, GnGeom G,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    uint64_t* __restrict__ slots, int* done, int nteams, int64_t ngroups, float* __restrict__ dx,
    float* __restrict__ dx2, const float* __restrict__ add1, const float* __restrict__ add2) {
    __shared__ float red[8];
    __shared__ float sv[2 * GNT_MAX_CHUNKS];
    __shared__ int miss[GNT_MAX_CHUNKS + 1];
    __shared__ float tab[2][3][GNP_MAX_CG];
    const uint32_t m = blockIdx.x % G.chunks;
    int64_t gi = blockIdx.x / G.chunks;
    if (gi >= ngroups) return;
    SP_DCHECK(G.chunk / 4 <= PER * kBlock && G.chunks <= GNT_MAX_CHUNKS && nteams > 0);
    float va[PER][4], ga[PER][4], vb[PER][4], gb[PER][4];
    GnpBuf ba, bb;
    gnp_issue<PER>(x, G, gi, m, va, ba);
    {
        const GroupCtx c = group_ctx_at<4>(x, G, gi, m);
        const auto rg = gnt_rsrc(Parts<const float>{dz + c.zoff, dz + c.zoff, G.gs}, c.lo, c.hi);
        const uint32_t vo = (c.lo + threadIdx.x) * 16;
#pragma unroll
        for (int i = 0; i < PER; ++i) gnt_load(rg, vo, i, ga[i]);
    }
    const int64_t team = gi;
    for (;;) {
        int64_t gn = gi + nteams < ngroups ? gi + nteams : -1;
        gnp_bwd_group<ACT, PER>(dz, x, G, mean_in, rstd_in, slots, gi, gn, m, va, ga, ba, vb, gb,
                                bb, tab[0], red, sv, miss, dx, dx2, add1, add2, gi - nteams);
        if (gn < 0) break;
        gi = gn;
        gn = gi + nteams < ngroups ? gi + nteams : -1;
        gnp_bwd_group<ACT, PER>(dz, x, G, mean_in, rstd_in, slots, gi, gn, m, vb, gb, bb, va, ga,
                                ba, tab[1], red, sv, miss, dx, dx2, add1, add2, gi - nteams);
        if (gn < 0) break;
        gi = gn;
    }
    gnt_release_last(slots, done, G.chunks, gi, team);
}

// ---- host side --------------------------------------------------------------------------
static int gn_geom(int64_t n, int32_t c, int64_t hw, int32_t groups, const float* bias,
                   const float* gamma, const float* beta, float eps, int chunk, GnGeom* G,
                   int* V, dim3* grid) {
    if (n < 0 || c <= 0 || hw <= 0 || groups <= 0 || c % groups) return SP_EINVAL;
    const int64_t gs = (int64_t)(c / groups) * hw;
    if (gs >= (int64_t(1) << 31) || n * groups >= 65536) return SP_EINVAL;
    *V = (hw % 4 == 0) ? 4 : 1;
    G->bias = bias, G->gamma = gamma, G->beta = beta;
    G->C = c, G->G = groups, G->Cg = c / groups;
    G->gs = static_cast<uint32_t>(gs);
    G->chunk = static_cast<uint32_t>(chunk);
    G->chunks = static_cast<int>((gs + chunk - 1) / chunk);
    G->hw_div = make_fastdiv(static_cast<uint32_t>(hw / *V));
    G->eps = eps;
    G->x2 = nullptr;
    G->add1b = nullptr;
    G->c1hw = static_cast<uint32_t>(c * hw);
    G->s2 = 0;
    *grid = dim3(G->chunks, static_cast<unsigned>(n * groups));
    return SP_OK;
}

static int g_single_pass = 1;  // sp_groupnorm_single_pass

// A stream being captured into a graph takes the two-pass kernels (bit-identical results): a
// replayed graph let the single-pass teams wait on members that were not resident at B = 64
// (1.27 M recomputed partials, 3.3x the eager step; profiles/round4/graph/), and the two-pass
// form waits on nobody.
static bool gn_capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
}

// Bytes of the single-pass kernels' team region: two 64-bit words per chunk and a done count per
// group, at the smallest chunk either direction uses (an upper bound for both).
static int64_t gnt_region_bytes(int64_t ngroups, int chunks) { return ngroups * chunks * 16 + ngroups * 4; }

// The single-pass kernels' team words and done counts.  `team` (the caller's, team_bytes long,
// zeroed once by the caller and left zero by every launch — gnt_clear_own / gnt_release_last —
// so a call needs no memset), else the call's workspace, zeroed first.  The library allocates
// nothing: a caller that keeps one zeroed region per stream saves the memset launch.
static int gnt_slots(int64_t ngroups, int chunks, float* work, void* team, int64_t team_bytes,
                     hipStream_t s, uint64_t** slots, int** done) {
    const int64_t words = ngroups * chunks * 16, bytes = gnt_region_bytes(ngroups, chunks);
    if (team) {
        if (team_bytes < bytes) return SP_EINVAL;
        *slots = static_cast<uint64_t*>(team);
        *done = reinterpret_cast<int*>(static_cast<char*>(team) + words);
        return SP_OK;
    }
    *slots = reinterpret_cast<uint64_t*>(work);
    *done = reinterpret_cast<int*>(reinterpret_cast<char*>(work) + words);
    if (hipMemsetAsync(work, 0, bytes, s) != hipSuccess) return check_launch("groupnorm slots (memset)");
    return SP_OK;
}

// Teams that fit the chip at once for a single-pass kernel (0: the kernel cannot run).
static int64_t gnt_teams(const void* kernel, int64_t ngroups, int chunks) {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess)
        return 0;
    const int64_t teams = (int64_t)cus * per_cu / chunks;
    return teams < ngroups ? teams : ngroups;
}

}  // namespace sp

using namespace sp;

extern "C" {

int64_t sp_groupnorm_workspace(int64_t n, int32_t channels, int64_t hw, int32_t groups) {
    if (n < 0 || channels <= 0 || hw <= 0 || groups <= 0 || channels % groups) return -1;
    const int64_t gs = (int64_t)(channels / groups) * hw;
    // two-pass: 2 floats per chunk; single pass: 2 64-bit words per chunk and a count per group
    return n * groups * ((gs + GN_CHUNK_MIN - 1) / GN_CHUNK_MIN) * 4 + n * groups;
}

int64_t sp_groupnorm_team_bytes(int64_t n, int32_t channels, int64_t hw, int32_t groups) {
    if (n < 0 || channels <= 0 || hw <= 0 || groups <= 0 || channels % groups) return -1;
    const int64_t gs = (int64_t)(channels / groups) * hw;
    return gnt_region_bytes(n * groups, static_cast<int>((gs + GN_CHUNK_MIN - 1) / GN_CHUNK_MIN));
}

int sp_groupnorm_single_pass(int32_t enable) {
    const int prev = g_single_pass;
    if (enable >= 0) g_single_pass = enable ? 1 : 0;
    return prev;
}

int sp_groupnorm_set_spin_limit(int32_t spins) {
    const int32_t v = spins < 0 ? GNT_MAX_SPINS : spins;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_gnt_spin_limit), &v, sizeof(v)) != hipSuccess)
        return check_launch("sp_groupnorm_set_spin_limit");
    return SP_OK;
}

int64_t sp_groupnorm_team_timeouts(void) {
    unsigned int v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_gnt_timeouts), sizeof(v)) != hipSuccess) return -1;
    return v;
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
                                  groups, eps, act, z, mean, rstd, work, nullptr, 0, stream);
}

int sp_groupnorm_silu_fwd2(const float* x, const float* x2, int32_t c1, const float* chan_bias,
                           const float* gamma, const float* beta, int64_t n, int32_t channels,
                           int64_t hw, int32_t groups, float eps, int32_t act, float* z,
                           float* mean, float* rstd, float* work, void* team, int64_t team_bytes,
                           sp_stream_t stream) {
    GnGeom G;
    int V;
    dim3 grid;
    const int chunk = gn_fwd_chunk((int64_t)(channels / (groups > 0 ? groups : 1)) * hw);
    int rc = gn_geom(n, channels, hw, groups, chan_bias, gamma, beta, eps, chunk, &G, &V, &grid);
    if (rc == SP_OK) rc = gn_split(&G, x2, c1, channels, hw);
    if (rc != SP_OK) return rc;
    if (n == 0) return SP_OK;  // empty batch: nothing to read or write
    if (!x || !z || !mean || !rstd || !work) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 blk(kBlock);
    if (V == 4 && g_single_pass && !gn_capturing(s) && G.Cg <= GNP_MAX_CG && G.chunks <= GNT_MAX_CHUNKS &&
        (!x2 || (int64_t)(c1 % G.Cg) * hw % chunk == 0)) {
        const int64_t ngroups = n * groups;
        const void* kern;
        if (chunk == GN_CHUNK_FWD_BIG)
            kern = act ? (const void*)k_gn_fwd_pipe<true, GN_CHUNK_FWD_BIG / 4 / kBlock>
                       : (const void*)k_gn_fwd_pipe<false, GN_CHUNK_FWD_BIG / 4 / kBlock>;
        else
            kern = act ? (const void*)k_gn_fwd_pipe<true, GN_CHUNK_FWD / 4 / kBlock>
                       : (const void*)k_gn_fwd_pipe<false, GN_CHUNK_FWD / 4 / kBlock>;
        const int64_t teams = gnt_teams(kern, ngroups, G.chunks);
        if (teams > 0) {
            uint64_t* slots;
            int* done;
            if (int e = gnt_slots(ngroups, G.chunks, work, team, team_bytes, s, &slots, &done)) return e;
            const dim3 grid1(static_cast<unsigned>(teams * G.chunks));
            const int nt = static_cast<int>(teams);
#define SP_GN_FWD_PIPE(AA, PP) \
    launch(0, k_gn_fwd_pipe<AA, PP>, grid1, blk, s, x, G, slots, done, nt, ngroups, z, mean, rstd)
            if (chunk == GN_CHUNK_FWD_BIG) {
                if (act) { SP_GN_FWD_PIPE(true, GN_CHUNK_FWD_BIG / 4 / kBlock); }
                else { SP_GN_FWD_PIPE(false, GN_CHUNK_FWD_BIG / 4 / kBlock); }
            } else {
                if (act) { SP_GN_FWD_PIPE(true, GN_CHUNK_FWD / 4 / kBlock); }
                else { SP_GN_FWD_PIPE(false, GN_CHUNK_FWD / 4 / kBlock); }
            }
#undef SP_GN_FWD_PIPE
            return check_launch("sp_groupnorm_silu_fwd");
        }
    }
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
                                  nullptr, work, nullptr, 0, stream);
}

int sp_groupnorm_silu_bwd2(const float* dz, const float* x, const float* x2, int32_t c1,
                           const float* chan_bias, const float* gamma, const float* beta,
                           const float* mean, const float* rstd, int64_t n, int32_t channels,
                           int64_t hw, int32_t groups, int32_t act, float* dx, float* dx2,
                           const float* add1, const float* add2, const float* add1b,
                           float* work, void* team, int64_t team_bytes, sp_stream_t stream) {
    GnGeom G;
    int V;
    dim3 grid;
    int rc = gn_geom(n, channels, hw, groups, chan_bias, gamma, beta, 0.f, GN_CHUNK_BWD, &G, &V,
                     &grid);
    if (rc == SP_OK) rc = gn_split(&G, x2, c1, channels, hw);
    if (rc != SP_OK) return rc;
    if (n == 0) return SP_OK;
    if (!dz || !x || !mean || !rstd || !dx || !work || (x2 && !dx2) || (x2 && add1 && !add2) ||
        (x2 && add1b))
        return SP_EINVAL;
    G.add1b = add1b;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 blk(kBlock);
    if (V == 4 && g_single_pass && !gn_capturing(s) && G.Cg <= GNP_MAX_CG && G.chunks <= GNT_MAX_CHUNKS &&
        (!x2 || (int64_t)(c1 % G.Cg) * hw % GN_CHUNK_BWD == 0)) {
        const int64_t ngroups = n * groups;
        constexpr int PER = GN_CHUNK_BWD / 4 / kBlock;
        auto kern = act ? k_gn_bwd_pipe<true, PER> : k_gn_bwd_pipe<false, PER>;
        const int64_t teams = gnt_teams(reinterpret_cast<const void*>(kern), ngroups, G.chunks);
        if (teams > 0) {
            uint64_t* slots;
            int* done;
            if (int e = gnt_slots(ngroups, G.chunks, work, team, team_bytes, s, &slots, &done)) return e;
            launch(0, kern, dim3(static_cast<unsigned>(teams * G.chunks)), blk, s, dz, x, G, mean,
                   rstd, slots, done, static_cast<int>(teams), ngroups, dx, dx2, add1, add2);
            return check_launch("sp_groupnorm_silu_bwd");
        }
    }
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

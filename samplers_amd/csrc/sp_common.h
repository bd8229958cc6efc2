// Shared device helpers for libsamplers_hip: Philox4x32-10 normals, wave64 /
// block reductions, vector load/store, launch-error bookkeeping.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/samplers_hip.h"

namespace sp {

#ifndef SP_KITER
#define SP_KITER 2
#endif
#ifndef SP_NT_STORE
#define SP_NT_STORE 0
#endif

// ---------------------------------------------------------------------------
// Bounds-checked debug build (`make debug`: -DSP_DEBUG=1, samplers_amd/lib/debug/).
// SP_DCHECK(cond) states an index / range invariant of a kernel.  In the debug build a
// violated one is counted in a per-translation-unit device word, with the site of the first
// (SP_TU << 16 | __LINE__; SP_TU numbers the source files, 0 = this header); the kernel then
// goes on unchanged (a check never alters what a kernel reads or writes — the buffer range
// checks of the release build stay as they are), and sp_debug_violations() reads the counts
// after a device sync.  The release build compiles the checks away.
// ---------------------------------------------------------------------------
#ifndef SP_DEBUG
#define SP_DEBUG 0
#endif
#ifndef SP_TU
#define SP_TU 0
#endif
#if SP_DEBUG
static __device__ unsigned int g_dcheck[2];  // violations, first site
__attribute__((unused)) static __device__ __noinline__ void dcheck_fail(unsigned site) {
    if (atomicAdd(&g_dcheck[0], 1u) == 0u) atomicExch(&g_dcheck[1], site);
}
#define SP_DCHECK(cond)                                                     \
    do {                                                                    \
        if (!(cond)) ::sp::dcheck_fail((unsigned(SP_TU) << 16) | __LINE__); \
    } while (0)
// host side: every translation unit registers a reader of its two words (sp_dps.hip)
typedef int (*dcheck_reader)(unsigned* out, int reset);
void dcheck_register(dcheck_reader r);
static int dcheck_read_tu(unsigned* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dcheck), sizeof(g_dcheck)) != hipSuccess) return -1;
    if (reset) {
        const unsigned zero[2] = {0u, 0u};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_dcheck), zero, sizeof(zero)) != hipSuccess) return -1;
    }
    return 0;
}
static const int g_dcheck_registered = (dcheck_register(&dcheck_read_tu), 0);
#else
#define SP_DCHECK(cond) \
    do {                \
    } while (0)
#endif

constexpr int kBlock = 256;       // 4 waves of 64 lanes
constexpr int kIter = SP_KITER;   // float4 groups per thread per block (elementwise kernels)

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11).  Counter = (element group, sample, step lo,
// step hi), key = seed.  The same (seed, step, sample, element) gives the same
// normal on every shard, so a batch split over N GPUs reproduces the 1-GPU draw.
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
    constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t lo0 = M0 * c.x, hi0 = __umulhi(M0, c.x);
        const uint32_t lo1 = M1 * c.z, hi1 = __umulhi(M1, c.z);
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// Uniform in (0,1), exactly representable: ((u >> 9) + 0.5) * 2^-23.
__device__ __forceinline__ float u01(uint32_t u) {
    return (static_cast<float>(u >> 9) + 0.5f) * 1.1920928955078125e-07f;
}

// Four standard normals for element group `grp` (elements 4*grp .. 4*grp+3).
// Box-Muller on the hardware transcendentals: v_log_f32 is log2, v_sin_f32 /
// v_cos_f32 take revolutions, so sin(2*pi*u) = __builtin_amdgcn_sinf(u).
__device__ __forceinline__ void philox_normal4(uint64_t seed, int64_t step, int64_t sample,
                                               int64_t grp, float out[4]) {
    const u32x4 c{static_cast<uint32_t>(grp), static_cast<uint32_t>(sample),
                  static_cast<uint32_t>(static_cast<uint64_t>(step)),
                  static_cast<uint32_t>(static_cast<uint64_t>(step) >> 32)};
    const u32x4 r = philox4x32_10(c, static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
    constexpr float kM2Ln2 = -1.3862943611198906f;  // -2 ln 2
    const float rad0 = __builtin_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u01(r.x)));
    const float rad1 = __builtin_sqrtf(kM2Ln2 * __builtin_amdgcn_logf(u01(r.z)));
    const float t0 = u01(r.y), t1 = u01(r.w);
    out[0] = rad0 * __builtin_amdgcn_cosf(t0);
    out[1] = rad0 * __builtin_amdgcn_sinf(t0);
    out[2] = rad1 * __builtin_amdgcn_cosf(t1);
    out[3] = rad1 * __builtin_amdgcn_sinf(t1);
}

// ---------------------------------------------------------------------------
// Reductions (wave64 butterfly; fixed order -> deterministic).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Block sum for kBlock threads; result valid in thread 0.
__device__ __forceinline__ float block_sum(float v, float* lds4) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) lds4[wid] = v;
    __syncthreads();
    float t = 0.f;
    if (threadIdx.x == 0) t = (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
    return t;
}

// Sum of the P partials of one sample, computed redundantly by every wave
// (all lanes end with the total; no LDS, no barrier).
__device__ __forceinline__ float sum_partials(const float* __restrict__ p, int P) {
    float s = 0.f;
    for (int i = threadIdx.x & 63; i < P; i += 64) s += p[i];
    return wave_sum(s);
}

// The same total for a whole block of kBlock threads: wave w adds its quarter of the partials
// (lane-strided), the four wave sums meet in LDS in a fixed order — deterministic and equal in
// every block of the sample, a quarter of sum_partials' loads per wave (at 3x512² P = 384:
// the update pass spent 8 µs of 50 re-reading them, round 4).  Every thread must call it.
__device__ __forceinline__ float block_sum_partials(const float* __restrict__ p, int P, float* lds4) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q = (P + 3) >> 2, lo = w * q, hi = min(P, lo + q);
    float s = 0.f;
    for (int i = lo + lane; i < hi; i += 64) s += p[i];
    s = wave_sum(s);
    if (lane == 0) lds4[w] = s;
    __syncthreads();
    return (lds4[0] + lds4[1]) + (lds4[2] + lds4[3]);
}

// ---------------------------------------------------------------------------
// Vector access
// ---------------------------------------------------------------------------
// NT = non-temporal (streamed-once inputs)
template <int V, bool NT = false>
__device__ __forceinline__ void load_v(const float* __restrict__ p, float (&r)[V]) {
    if constexpr (V == 4) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        f4v t;
        if constexpr (NT)
            t = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(p));
        else
            t = *reinterpret_cast<const f4v*>(p);
        r[0] = t.x; r[1] = t.y; r[2] = t.z; r[3] = t.w;
    } else {
#pragma unroll
        for (int e = 0; e < V; ++e) r[e] = p[e];
    }
}

// NT = non-temporal (streamed-once outputs: the updated sample of the DPS step).
template <int V, bool NT = false>
__device__ __forceinline__ void store_v(float* __restrict__ p, const float (&r)[V]) {
    if constexpr (V == 4) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v t = {r[0], r[1], r[2], r[3]};
        if constexpr (NT || SP_NT_STORE)
            __builtin_nontemporal_store(t, reinterpret_cast<f4v*>(p));
        else
            *reinterpret_cast<f4v*>(p) = t;
    } else {
#pragma unroll
        for (int e = 0; e < V; ++e) p[e] = r[e];
    }
}

// Normals for elements j..j+V-1 of one sample (V = 4 with j % 4 == 0, or V = 1).
template <int V>
__device__ __forceinline__ void philox_normals(uint64_t seed, int64_t step, int64_t sample,
                                               int64_t j, float (&z)[V]) {
    float q[4];
    philox_normal4(seed, step, sample, j >> 2, q);
    if constexpr (V == 4) {
        z[0] = q[0]; z[1] = q[1]; z[2] = q[2]; z[3] = q[3];
    } else {
        const int c = static_cast<int>(j & 3);
        z[0] = c == 0 ? q[0] : c == 1 ? q[1] : c == 2 ? q[2] : q[3];
    }
}

// ---------------------------------------------------------------------------
// Inpainting index: observed rank of element j (= its index in the packed y).
// keep_bits bit (j & 63) of word (j >> 6) is 1 when x[j] is observed; the rank
// is word_rank[j >> 6] + popcount of the lower bits of that word.  Equals the
// position of j in torch.nonzero(~mask.flatten()) (inpainting.py:49-50).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void inpaint_lookup(const sp_op& op, int64_t j, uint32_t& bits4,
                                               int64_t& rank0) {
    const uint64_t word = op.keep_bits[j >> 6];
    const int sh = static_cast<int>(j & 63);
    bits4 = static_cast<uint32_t>(word >> sh) & 0xFu;
    rank0 = op.word_rank[j >> 6] + __popcll(word & ((1ull << sh) - 1ull));
}

// Observed bits of elements j..j+3 (MASK operator: m == n, no ranks needed).
__device__ __forceinline__ uint32_t mask_bits(const sp_op& op, int64_t j) {
    return static_cast<uint32_t>(op.keep_bits[j >> 6] >> (j & 63)) & 0xFu;
}

// ---------------------------------------------------------------------------
// host-side error bookkeeping
// ---------------------------------------------------------------------------
void set_error(const char* what, hipError_t e);
int check_launch(const char* what);

// Kernel timing (sp_timing_enable): the start/stop events of a timed launch are
// attached to its dispatch packet (hipExtLaunchKernel), so they bracket the
// kernel alone — the same interval rocprofv3's kernel trace reports.
// Each record carries the launch's algorithmic work (samples for the DPS passes,
// FLOPs for the convolution tile) for sp_timing_collect_work.
bool timing_on();
void timing_events(int kind, double work, hipEvent_t* start, hipEvent_t* stop);

enum {
    TK_DPS_RESIDUAL = 1,
    TK_DPS_UPDATE = 2,
    TK_CONV3X3_FWD = 3,
    TK_CONV3X3_BWD_INPUT = 4,
    TK_WINO3X3_FWD = 5,
    TK_WINO3X3_BWD_INPUT = 6,
    TK_CONV_BF16 = 7
};

template <typename K, typename... Args>
inline void launch_w(int kind, double work, K kernel, dim3 grid, dim3 block, hipStream_t s,
                     Args... args) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (kind && timing_on()) timing_events(kind, work, &e0, &e1);
    hipExtLaunchKernelGGL(kernel, grid, block, 0, s, e0, e1, 0, args...);
}

template <typename K, typename... Args>
inline void launch(int kind, K kernel, dim3 grid, dim3 block, hipStream_t s, Args... args) {
    launch_w(kind, 0.0, kernel, grid, block, s, args...);
}

}  // namespace sp

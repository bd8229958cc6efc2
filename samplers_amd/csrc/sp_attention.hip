// Fused self-attention softmax(q k^T * scale) v and its input VJP on fp32 MFMA
// (v_mfma_f32_16x16x4_f32) for the SD 1.5 ε-UNet's transformer blocks (attn1 over the
// 64x64 / 32x32 / 16x16 / 8x8 latent tokens, head dims 40 / 80 / 160; diffusers
// UNet2DConditionModel, called from /root/reference/samplers/networks/diffusers/
// stable_diffusion.py:306-313).  The score matrix (32 latents x 8 heads x 4096^2 x 4 B =
// 17 GiB per layer at configs[3]'s batch) never reaches HBM: every kernel keeps a 16 x 16
// score block in registers (the FlashAttention recurrence, exact fp32 MFMA accumulation).
//
// Layouts: row i of head h of batch b of q, k, v, dq, dk, dv starts at (b n + i) rs + h d, of
// out and dout at (b n + i) ro + h d: the token-major [b][n][heads x d] activations the
// projections read and write (rs = 3 heads d when q, k, v are the thirds of one fused
// projection), so no head split / merge copies exist.  heads = 1, rs = ro = d is the plain
// [bh][n][d] layout.  lse, delta are [bh][n].
// MFMA operand maps (16x16x4 f32): A[m = l & 15][k = l >> 4], B[k = l >> 4][n = l & 15],
// C[row = 4 (l >> 4) + i][col = l & 15], i = 0..3 (cdna_hip_programming.md §3).
//
// Every kernel computes a score block TRANSPOSED or not so that the per-query softmax state
// is lane-local:
//   forward, dq:  S^T = K Q^T  (C: key 4(l>>4)+i, query l&15); O^T / dQ^T += V^T / K^T . P^T
//                 take P^T straight from the C registers as their B operand, k-step i
//                 pairing key 4(l>>4)+i (the key order inside the MFMA's K is a permutation,
//                 applied to the A operand's reads too);
//   dk, dv:       S = Q K^T   (C: query 4(l>>4)+i, key l&15); dK^T / dV^T += Q^T / dO^T . dS / P.
// The running max, the row sum and the rescale of the accumulators then need no lane
// exchange except two xor-shuffles for the block max.  Scores are scaled by scale*log2(e) and
// exponentiated with exp2; lse is stored in natural-log units.
//
// Work per 16 x 16 (query, key) block at head dim d: forward d/4 + 4 ceil(d/16) MFMAs, dq
// 2 d/4 + 4 ceil(d/16), dk/dv 2 d/4 + 8 ceil(d/16) (useful FLOP: 4 d per block entry forward,
// 10 d backward).

#define SP_TU 10  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

#include <algorithm>
#include <cmath>

namespace sp {

typedef float at_f4 __attribute__((ext_vector_type(4)));

constexpr int AT_WAVES = 4;
constexpr float AT_LOG2E = 1.4426950408889634f;
constexpr float AT_LN2 = 0.6931471805599453f;

template <int D>
struct AtGeo {
    static_assert(D % 4 == 0 && D <= 160, "head dim");
    static constexpr int DP = D + 4;                 // LDS row stride: conflict-free reads
    static constexpr int DS = D / 4;                 // k-steps over d
    static constexpr int DT = (D + 15) / 16;         // 16-row tiles over d (rows >= D unused)
    static constexpr int QT = D <= 80 ? 2 : 1;       // 16-row tiles per wave (queries or keys)
    static constexpr int SB = D <= 80 ? 64 : 32;     // rows (keys or queries) per LDS stage
    static constexpr int WB = AT_WAVES * QT * 16;    // rows a workgroup owns
    static constexpr int PAD = 16;                   // tail so padding-row reads stay in LDS
    static constexpr int NF4 = (SB * D / 4 + kBlock - 1) / kBlock;  // float4 per thread per tensor
};

// 2^x as the bare v_exp_f32: exp2f adds a range check and rescale for results below 2^-126
// (five instructions per score); here x <= 0 and such weights vanish beside the row's largest
// (2^0) in every sum they enter.  exp2(-inf) = 0 as before.
__device__ __forceinline__ float at_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ at_f4 at_mfma(float a, float b, at_f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Stage rows [r0, r0 + SB) of a [n][D] matrix (contiguous: SB*D floats) into LDS rows of
// stride DP, through registers (issued one stage ahead).
template <int D>
struct AtStage {
    float4 r[AtGeo<D>::NF4];
};

// rows >= lim (past the last key of a cross-attention context) are staged as zeros
template <int D>
__device__ __forceinline__ void at_load(const float* __restrict__ src, int rs, AtStage<D>& st,
                                        int lim = 1 << 30) {
    using G = AtGeo<D>;
#pragma unroll
    for (int j = 0; j < G::NF4; ++j) {
        const int i = threadIdx.x + j * kBlock;
        if (i < G::SB * D / 4) {
            const int row = (4 * i) / D, col = 4 * i - row * D;
            st.r[j] = row < lim ? *reinterpret_cast<const float4*>(src + (int64_t)row * rs + col)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
}

// first element of head h = bh % heads of batch bh / heads, in a layout of row stride rs
__device__ __forceinline__ int64_t at_base(int bh, int heads, int n, int rs, int d) {
    const int b = bh / heads;
    return (int64_t)b * n * rs + (int64_t)(bh - b * heads) * d;
}

// The keys / values: m rows of stride rs per sample; shared = one sample for the whole batch
// (cross-attention to one context row broadcast over the batch)
struct AtKV {
    int m, rs, shared;
    __device__ __forceinline__ int64_t base(int bh, int heads, int d) const {
        return at_base(shared ? bh % heads : bh, heads, m, rs, d);
    }
};

template <int D>
__device__ __forceinline__ void at_store(float* dst, const AtStage<D>& st) {
    using G = AtGeo<D>;
#pragma unroll
    for (int j = 0; j < G::NF4; ++j) {
        const int i = threadIdx.x + j * kBlock;
        if (i < G::SB * D / 4) {
            const int row = (4 * i) / D, col = 4 * i - row * D;
            *reinterpret_cast<float4*>(dst + row * G::DP + col) = st.r[j];
        }
    }
}

__device__ __forceinline__ float at_max4(at_f4 s) { return fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3])); }

// max over the four lanes l, l^16, l^32, l^48 (the rows of one C column)
__device__ __forceinline__ float at_colmax(float v) {
    v = fmaxf(v, __shfl_xor(v, 16));
    return fmaxf(v, __shfl_xor(v, 32));
}
__device__ __forceinline__ float at_colsum(float v) {
    v += __shfl_xor(v, 16);
    return v + __shfl_xor(v, 32);
}

// ---- forward --------------------------------------------------------------------------------
// Workgroup: WB queries of one (batch, head); wave w owns query tiles; keys streamed through
// LDS in stages of SB rows (K and V), 16 keys per score block.
template <int D>
__global__ __launch_bounds__(kBlock) void k_attn_fwd(const float* __restrict__ q,
                                                     const float* __restrict__ k,
                                                     const float* __restrict__ v, int n, int heads,
                                                     int rs, int ro, AtKV kv, float sl2,
                                                     float* __restrict__ out,
                                                     float* __restrict__ lse) {
    using G = AtGeo<D>;
    __shared__ __attribute__((aligned(16))) float Ks[G::SB * G::DP + G::PAD];
    __shared__ __attribute__((aligned(16))) float Vs[G::SB * G::DP + G::PAD];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, li = lane & 15, kl = lane >> 4;
    const int64_t base = at_base(blockIdx.y, heads, n, rs, D);
    const int q0 = blockIdx.x * G::WB + wv * G::QT * 16;
    const int64_t kvb = kv.base(blockIdx.y, heads, D);
    SP_DCHECK(rs >= heads * D && ro >= heads * D && (int64_t)blockIdx.x * G::WB < n && kv.m > 0);
    const float* __restrict__ kb = k + kvb;
    const float* __restrict__ vb = v + kvb;
    const int m_keys = kv.m;

    float qr[G::QT][G::DS];  // B operand of S^T = K Q^T: Q[q][4s + kl] * scale * log2 e
#pragma unroll
    for (int t = 0; t < G::QT; ++t)
#pragma unroll
        for (int s = 0; s < G::DS; ++s) qr[t][s] = q[base + (int64_t)(q0 + 16 * t + li) * rs + 4 * s + kl] * sl2;
    at_f4 o[G::QT][G::DT];
    float m[G::QT], l[G::QT];
#pragma unroll
    for (int t = 0; t < G::QT; ++t) {
        m[t] = -INFINITY, l[t] = 0.f;
#pragma unroll
        for (int dt = 0; dt < G::DT; ++dt) o[t][dt] = at_f4{0.f, 0.f, 0.f, 0.f};
    }

    AtStage<D> sk, sv;
    const int rk = kv.rs;
    at_load<D>(kb, rk, sk, m_keys);
    at_load<D>(vb, rk, sv, m_keys);
    const int nst = (m_keys + G::SB - 1) / G::SB;
    for (int st = 0; st < nst; ++st) {
        __syncthreads();  // the previous stage's reads are done
        at_store<D>(Ks, sk);
        at_store<D>(Vs, sv);
        __syncthreads();
        if (st + 1 < nst) {  // next stage's rows in flight during this stage's MFMAs
            at_load<D>(kb + (int64_t)(st + 1) * G::SB * rk, rk, sk, m_keys - (st + 1) * G::SB);
            at_load<D>(vb + (int64_t)(st + 1) * G::SB * rk, rk, sv, m_keys - (st + 1) * G::SB);
        }
#pragma unroll
        for (int sb = 0; sb < G::SB / 16; ++sb) {
            const int key0 = st * G::SB + sb * 16;
            if (key0 >= m_keys) break;  // past the context's last key (uniform)
            const float* kr = Ks + (sb * 16 + li) * G::DP + kl;       // K[key li][4s + kl]
            at_f4 s[G::QT];
#pragma unroll
            for (int t = 0; t < G::QT; ++t) s[t] = at_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ss = 0; ss < G::DS; ++ss) {
                const float a = kr[4 * ss];
#pragma unroll
                for (int t = 0; t < G::QT; ++t) s[t] = at_mfma(a, qr[t][ss], s[t]);
            }
            if (key0 + 16 > m_keys) {  // keys past the last one score -inf (p = 0)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (key0 + 4 * kl + i >= m_keys)
#pragma unroll
                        for (int t = 0; t < G::QT; ++t) s[t][i] = -INFINITY;
            }
            float p[G::QT][4], corr[G::QT];
            bool moved = false;
#pragma unroll
            for (int t = 0; t < G::QT; ++t) {
                const float mn = fmaxf(m[t], at_colmax(at_max4(s[t])));
                corr[t] = at_exp2(m[t] - mn);  // 0 on the first block (m = -inf)
                moved |= corr[t] != 1.f;
                m[t] = mn;
                float ps = 0.f;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    p[t][i] = at_exp2(s[t][i] - mn);
                    ps += p[t][i];
                }
                l[t] = fmaf(l[t], corr[t], ps);  // this lane's partial row sum
            }
            // rescale the outputs only when some query's running max moved (a wave-uniform
            // branch; skipping a multiply by exactly 1 changes no bit)
            if (__builtin_amdgcn_ballot_w64(moved))
#pragma unroll
                for (int t = 0; t < G::QT; ++t)
#pragma unroll
                    for (int dt = 0; dt < G::DT; ++dt) o[t][dt] *= corr[t];
            // O^T += V^T P^T: k-step i takes key 4 kl + i (A: V[key][dt*16 + li])
            const float* vr = Vs + (sb * 16 + 4 * kl) * G::DP + li;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int dt = 0; dt < G::DT; ++dt) {
                    const float a = vr[i * G::DP + 16 * dt];
#pragma unroll
                    for (int t = 0; t < G::QT; ++t) o[t][dt] = at_mfma(a, p[t][i], o[t][dt]);
                }
        }
    }
    // O = O^T / rowsum; lane: d = dt*16 + 4 kl + i of query q0 + 16 t + li
#pragma unroll
    for (int t = 0; t < G::QT; ++t) {
        const float tot = at_colsum(l[t]);
        const float inv = 1.f / tot;
        const int qq = q0 + 16 * t + li;
        float* orow = out + at_base(blockIdx.y, heads, n, ro, D) + (int64_t)qq * ro;
#pragma unroll
        for (int dt = 0; dt < G::DT; ++dt) {
            const int d0 = dt * 16 + 4 * kl;
            if (d0 < D) *reinterpret_cast<float4*>(orow + d0) = make_float4(
                o[t][dt][0] * inv, o[t][dt][1] * inv, o[t][dt][2] * inv, o[t][dt][3] * inv);
        }
        if (kl == 0) lse[(int64_t)blockIdx.y * n + qq] = (m[t] + log2f(tot)) * AT_LN2;
    }
}

// ---- backward: delta = rowsum(dout * out) -----------------------------------------------------
template <int D>
__global__ __launch_bounds__(kBlock) void k_attn_delta(const float* __restrict__ out,
                                                       const float* __restrict__ dout, int64_t rows,
                                                       int n, int heads, int ro,
                                                       float* __restrict__ delta) {
    const int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x;  // (bh, token) = (r / n, r % n)
    if (r >= rows) return;
    const int bh = static_cast<int>(r / n), tok = static_cast<int>(r - (int64_t)bh * n);
    const int64_t off = at_base(bh, heads, n, ro, D) + (int64_t)tok * ro;
    const float4* a = reinterpret_cast<const float4*>(out + off);
    const float4* b = reinterpret_cast<const float4*>(dout + off);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < D / 4; ++j) {
        const float4 x = a[j], y = b[j];
        s += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
    delta[r] = s;
}

// ---- backward: dq ---------------------------------------------------------------------------
// As the forward, with dP^T = V dO^T beside S^T and dQ^T += K^T dS^T, dS = P (dP - delta).
template <int D>
__global__ __launch_bounds__(kBlock) void k_attn_dq(const float* __restrict__ q,
                                                    const float* __restrict__ k,
                                                    const float* __restrict__ v,
                                                    const float* __restrict__ dout,
                                                    const float* __restrict__ lse,
                                                    const float* __restrict__ delta, int n,
                                                    int heads, int rs, int ro, AtKV kv, float sl2,
                                                    float scale, float* __restrict__ dq) {
    using G = AtGeo<D>;
    __shared__ __attribute__((aligned(16))) float Ks[G::SB * G::DP + G::PAD];
    __shared__ __attribute__((aligned(16))) float Vs[G::SB * G::DP + G::PAD];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, li = lane & 15, kl = lane >> 4;
    const int64_t base = at_base(blockIdx.y, heads, n, rs, D);
    const int64_t obase = at_base(blockIdx.y, heads, n, ro, D);
    const int q0 = blockIdx.x * G::WB + wv * G::QT * 16;
    const int64_t kvb = kv.base(blockIdx.y, heads, D);
    const float* __restrict__ kb = k + kvb;
    const float* __restrict__ vb = v + kvb;
    const int m_keys = kv.m;

    float qr[G::QT][G::DS], dr[G::QT][G::DS], ls[G::QT], de[G::QT];
#pragma unroll
    for (int t = 0; t < G::QT; ++t) {
        const int64_t row = base + (int64_t)(q0 + 16 * t + li) * rs;
        const int64_t orow = obase + (int64_t)(q0 + 16 * t + li) * ro;
#pragma unroll
        for (int s = 0; s < G::DS; ++s) {
            qr[t][s] = q[row + 4 * s + kl] * sl2;
            dr[t][s] = dout[orow + 4 * s + kl];
        }
        const int64_t r = (int64_t)blockIdx.y * n + q0 + 16 * t + li;
        ls[t] = lse[r] * AT_LOG2E;
        de[t] = delta[r];
    }
    at_f4 acc[G::QT][G::DT];
#pragma unroll
    for (int t = 0; t < G::QT; ++t)
#pragma unroll
        for (int dt = 0; dt < G::DT; ++dt) acc[t][dt] = at_f4{0.f, 0.f, 0.f, 0.f};

    AtStage<D> sk, sv;
    const int rk = kv.rs;
    at_load<D>(kb, rk, sk, m_keys);
    at_load<D>(vb, rk, sv, m_keys);
    const int nst = (m_keys + G::SB - 1) / G::SB;
    for (int st = 0; st < nst; ++st) {
        __syncthreads();
        at_store<D>(Ks, sk);
        at_store<D>(Vs, sv);
        __syncthreads();
        if (st + 1 < nst) {
            at_load<D>(kb + (int64_t)(st + 1) * G::SB * rk, rk, sk, m_keys - (st + 1) * G::SB);
            at_load<D>(vb + (int64_t)(st + 1) * G::SB * rk, rk, sv, m_keys - (st + 1) * G::SB);
        }
#pragma unroll
        for (int sb = 0; sb < G::SB / 16; ++sb) {
            const int key0 = st * G::SB + sb * 16;
            if (key0 >= m_keys) break;  // past the context's last key (uniform)
            const float* kr = Ks + (sb * 16 + li) * G::DP + kl;
            const float* vr = Vs + (sb * 16 + li) * G::DP + kl;
            at_f4 s[G::QT], dp[G::QT];
#pragma unroll
            for (int t = 0; t < G::QT; ++t) s[t] = dp[t] = at_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ss = 0; ss < G::DS; ++ss) {
                const float a = kr[4 * ss], b = vr[4 * ss];
#pragma unroll
                for (int t = 0; t < G::QT; ++t) {
                    s[t] = at_mfma(a, qr[t][ss], s[t]);
                    dp[t] = at_mfma(b, dr[t][ss], dp[t]);
                }
            }
            if (key0 + 16 > m_keys) {  // keys past the last one: p = 0
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (key0 + 4 * kl + i >= m_keys)
#pragma unroll
                        for (int t = 0; t < G::QT; ++t) s[t][i] = -INFINITY;
            }
            float ds[G::QT][4];
#pragma unroll
            for (int t = 0; t < G::QT; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) ds[t][i] = at_exp2(s[t][i] - ls[t]) * (dp[t][i] - de[t]);
            // dQ^T += K^T dS^T: k-step i takes key 4 kl + i (A: K[key][dt*16 + li])
            const float* kt = Ks + (sb * 16 + 4 * kl) * G::DP + li;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int dt = 0; dt < G::DT; ++dt) {
                    const float a = kt[i * G::DP + 16 * dt];
#pragma unroll
                    for (int t = 0; t < G::QT; ++t) acc[t][dt] = at_mfma(a, ds[t][i], acc[t][dt]);
                }
        }
    }
#pragma unroll
    for (int t = 0; t < G::QT; ++t) {
        float* drow = dq + base + (int64_t)(q0 + 16 * t + li) * rs;
#pragma unroll
        for (int dt = 0; dt < G::DT; ++dt) {
            const int d0 = dt * 16 + 4 * kl;
            if (d0 < D) *reinterpret_cast<float4*>(drow + d0) = make_float4(
                acc[t][dt][0] * scale, acc[t][dt][1] * scale, acc[t][dt][2] * scale,
                acc[t][dt][3] * scale);
        }
    }
}

// ---- backward: dk, dv -----------------------------------------------------------------------
// Workgroup: WB keys; wave w owns key tiles; queries (Q, dO rows, lse, delta) streamed through
// LDS.  S = Q K^T and dP = dO V^T (C: query 4(l>>4)+i, key l&15), dV^T += dO^T P,
// dK^T += Q^T dS.
template <int D>
__global__ __launch_bounds__(kBlock) void k_attn_dkv(const float* __restrict__ q,
                                                     const float* __restrict__ k,
                                                     const float* __restrict__ v,
                                                     const float* __restrict__ dout,
                                                     const float* __restrict__ lse,
                                                     const float* __restrict__ delta, int n,
                                                     int heads, int rs, int ro, float sl2, float scale,
                                                     float* __restrict__ dk, float* __restrict__ dv) {
    using G = AtGeo<D>;
    __shared__ __attribute__((aligned(16))) float Qs[G::SB * G::DP + G::PAD];
    __shared__ __attribute__((aligned(16))) float Os[G::SB * G::DP + G::PAD];  // dO rows
    __shared__ float Ls[G::SB], Es[G::SB];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, li = lane & 15, kl = lane >> 4;
    const int64_t base = at_base(blockIdx.y, heads, n, rs, D);
    const int64_t rbase = (int64_t)blockIdx.y * n;
    const int k0 = blockIdx.x * G::WB + wv * G::QT * 16;
    const float* __restrict__ qb = q + base;
    const float* __restrict__ ob = dout + at_base(blockIdx.y, heads, n, ro, D);

    float kr[G::QT][G::DS], vr[G::QT][G::DS];  // B operands: K[key li][4s + kl] * sl2, V[..]
#pragma unroll
    for (int t = 0; t < G::QT; ++t) {
        const int64_t row = base + (int64_t)(k0 + 16 * t + li) * rs;
#pragma unroll
        for (int s = 0; s < G::DS; ++s) {
            kr[t][s] = k[row + 4 * s + kl] * sl2;
            vr[t][s] = v[row + 4 * s + kl];
        }
    }
    at_f4 ak[G::QT][G::DT], av[G::QT][G::DT];
#pragma unroll
    for (int t = 0; t < G::QT; ++t)
#pragma unroll
        for (int dt = 0; dt < G::DT; ++dt) ak[t][dt] = av[t][dt] = at_f4{0.f, 0.f, 0.f, 0.f};

    AtStage<D> sq, so;
    float sl = 0.f, se = 0.f;
    auto load_rows = [&](int st) {
        at_load<D>(qb + (int64_t)st * G::SB * rs, rs, sq);
        at_load<D>(ob + (int64_t)st * G::SB * ro, ro, so);
        if (threadIdx.x < G::SB) {
            sl = lse[rbase + st * G::SB + threadIdx.x] * AT_LOG2E;
            se = delta[rbase + st * G::SB + threadIdx.x];
        }
    };
    load_rows(0);
    const int nst = n / G::SB;
    for (int st = 0; st < nst; ++st) {
        __syncthreads();
        at_store<D>(Qs, sq);
        at_store<D>(Os, so);
        if (threadIdx.x < G::SB) Ls[threadIdx.x] = sl, Es[threadIdx.x] = se;
        __syncthreads();
        if (st + 1 < nst) load_rows(st + 1);
#pragma unroll
        for (int sb = 0; sb < G::SB / 16; ++sb) {
            const float* qa = Qs + (sb * 16 + li) * G::DP + kl;  // Q[query li][4s + kl]
            const float* oa = Os + (sb * 16 + li) * G::DP + kl;
            at_f4 s[G::QT], dp[G::QT];
#pragma unroll
            for (int t = 0; t < G::QT; ++t) s[t] = dp[t] = at_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ss = 0; ss < G::DS; ++ss) {
                const float a = qa[4 * ss], b = oa[4 * ss];
#pragma unroll
                for (int t = 0; t < G::QT; ++t) {
                    s[t] = at_mfma(a, kr[t][ss], s[t]);
                    dp[t] = at_mfma(b, vr[t][ss], dp[t]);
                }
            }
            // rows of the C registers: queries sb*16 + 4 kl + i
            float pl[4], pe[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) pl[i] = Ls[sb * 16 + 4 * kl + i], pe[i] = Es[sb * 16 + 4 * kl + i];
            float p[G::QT][4], ds[G::QT][4];
#pragma unroll
            for (int t = 0; t < G::QT; ++t)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    p[t][i] = at_exp2(s[t][i] - pl[i]);
                    ds[t][i] = p[t][i] * (dp[t][i] - pe[i]);
                }
            // dV^T += dO^T P, dK^T += Q^T dS: k-step i takes query 4 kl + i
            const float* ot = Os + (sb * 16 + 4 * kl) * G::DP + li;
            const float* qt = Qs + (sb * 16 + 4 * kl) * G::DP + li;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int dt = 0; dt < G::DT; ++dt) {
                    const float ao = ot[i * G::DP + 16 * dt], aq = qt[i * G::DP + 16 * dt];
#pragma unroll
                    for (int t = 0; t < G::QT; ++t) {
                        av[t][dt] = at_mfma(ao, p[t][i], av[t][dt]);
                        ak[t][dt] = at_mfma(aq, ds[t][i], ak[t][dt]);
                    }
                }
        }
    }
#pragma unroll
    for (int t = 0; t < G::QT; ++t) {
        const int64_t row = base + (int64_t)(k0 + 16 * t + li) * rs;
#pragma unroll
        for (int dt = 0; dt < G::DT; ++dt) {
            const int d0 = dt * 16 + 4 * kl;
            if (d0 < D) {
                *reinterpret_cast<float4*>(dk + row + d0) = make_float4(
                    ak[t][dt][0] * scale, ak[t][dt][1] * scale, ak[t][dt][2] * scale,
                    ak[t][dt][3] * scale);
                *reinterpret_cast<float4*>(dv + row + d0) =
                    make_float4(av[t][dt][0], av[t][dt][1], av[t][dt][2], av[t][dt][3]);
            }
        }
    }
}

template <int D>
static int attn_fwd_d(const float* q, const float* k, const float* v, int64_t bh, int heads, int64_t n,
                      int rs, int ro, AtKV kv, float scale, float* out, float* lse, hipStream_t s) {
    using G = AtGeo<D>;
    const double flops = 4.0 * bh * n * kv.m * D;
    launch_w(0, flops, k_attn_fwd<D>, dim3(static_cast<unsigned>(n / G::WB), static_cast<unsigned>(bh)),
             dim3(kBlock), s, q, k, v, static_cast<int>(n), heads, rs, ro, kv, scale * AT_LOG2E, out, lse);
    return check_launch("sp_attention_fwd");
}

template <int D>
static int attn_bwd_d(const float* q, const float* k, const float* v, const float* out,
                      const float* dout, const float* lse, int64_t bh, int heads, int64_t n, int rs, int ro,
                      AtKV kv, float scale, float* delta, float* dq, float* dk, float* dv, hipStream_t s) {
    using G = AtGeo<D>;
    const int64_t rows = bh * n;
    launch(0, k_attn_delta<D>, dim3(static_cast<unsigned>((rows + kBlock - 1) / kBlock)), dim3(kBlock), s,
           out, dout, rows, static_cast<int>(n), heads, ro, delta);
    const dim3 grid(static_cast<unsigned>(n / G::WB), static_cast<unsigned>(bh));
    const float sl2 = scale * AT_LOG2E;
    if (dq) launch(0, k_attn_dq<D>, grid, dim3(kBlock), s, q, k, v, dout, lse, (const float*)delta,
                   static_cast<int>(n), heads, rs, ro, kv, sl2, scale, dq);
    if (dk || dv) {
        if (!dk || !dv) return SP_EINVAL;
        launch(0, k_attn_dkv<D>, grid, dim3(kBlock), s, q, k, v, dout, lse, (const float*)delta,
               static_cast<int>(n), heads, rs, ro, sl2, scale, dk, dv);
    }
    return check_launch("sp_attention_bwd");
}

}  // namespace sp

using namespace sp;

extern "C" {

int sp_attention_supported(int64_t bh, int64_t n, int64_t m, int32_t d) {
    if (bh <= 0 || bh > 65535 || n <= 0 || m != n || n > (int64_t(1) << 24)) return 0;
    switch (d) {
        case 40: return n % AtGeo<40>::WB == 0 && n % AtGeo<40>::SB == 0;
        case 80: return n % AtGeo<80>::WB == 0 && n % AtGeo<80>::SB == 0;
        case 160: return n % AtGeo<160>::WB == 0 && n % AtGeo<160>::SB == 0;
        default: return 0;
    }
}

int sp_attention_mh_supported(int64_t batch, int32_t heads, int64_t n, int64_t m, int32_t d) {
    if (batch <= 0 || heads <= 0 || batch * heads > 65535 || n <= 0 || m <= 0 || n > (int64_t(1) << 24) ||
        m > (int64_t(1) << 24))
        return 0;
    switch (d) {
        case 40: return n % AtGeo<40>::WB == 0 && (m != n || n % AtGeo<40>::SB == 0);
        case 80: return n % AtGeo<80>::WB == 0 && (m != n || n % AtGeo<80>::SB == 0);
        case 160: return n % AtGeo<160>::WB == 0 && (m != n || n % AtGeo<160>::SB == 0);
        default: return 0;
    }
}

static bool mh_ok(int64_t batch, int32_t heads, int64_t n, int64_t m, int32_t d, int32_t rs, int32_t ro,
                  int32_t rs_kv, int64_t kv_batch) {
    const int32_t c = heads * d;
    return sp_attention_mh_supported(batch, heads, n, m, d) && rs >= c && ro >= c && rs_kv >= c &&
           rs % 4 == 0 && ro % 4 == 0 && rs_kv % 4 == 0 && (kv_batch == 1 || kv_batch == batch) &&
           batch * n * (int64_t)std::max(rs, ro) < (int64_t(1) << 40);
}

int sp_attention_fwd_mh(const float* q, const float* k, const float* v, int64_t batch, int32_t heads,
                        int64_t n, int64_t m, int32_t d, int32_t rs, int32_t rs_kv, int64_t kv_batch,
                        int32_t ro, float scale, float* out, float* lse, sp_stream_t stream) {
    if (!mh_ok(batch, heads, n, m, d, rs, ro, rs_kv, kv_batch) || !q || !k || !v || !out || !lse)
        return SP_EINVAL;
    // self-attention at the split-bf16 kernel's shapes runs there (sp_attention6.hip) unless
    // sp_attention_bf16x6(0) asked for the exact-fp32 kernel
    if (sp_attention_bf16x6_enabled() && m == n && kv_batch == batch && rs_kv == rs &&
        sp_attention6_supported(batch, heads, n, d))
        return sp_attention6_fwd_mh(q, k, v, batch, heads, n, d, rs, ro, scale, out, lse, stream);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t bh = batch * heads;
    const AtKV kv{static_cast<int>(m), rs_kv, kv_batch == 1 && batch > 1};
    switch (d) {
        case 40: return attn_fwd_d<40>(q, k, v, bh, heads, n, rs, ro, kv, scale, out, lse, s);
        case 80: return attn_fwd_d<80>(q, k, v, bh, heads, n, rs, ro, kv, scale, out, lse, s);
        default: return attn_fwd_d<160>(q, k, v, bh, heads, n, rs, ro, kv, scale, out, lse, s);
    }
}

int sp_attention_bwd_mh(const float* q, const float* k, const float* v, const float* out,
                        const float* dout, const float* lse, int64_t batch, int32_t heads, int64_t n,
                        int64_t m, int32_t d, int32_t rs, int32_t rs_kv, int64_t kv_batch, int32_t ro,
                        float scale, float* delta, float* dq, float* dk, float* dv, sp_stream_t stream) {
    if (!mh_ok(batch, heads, n, m, d, rs, ro, rs_kv, kv_batch) || !q || !k || !v || !out || !dout || !lse ||
        !delta)
        return SP_EINVAL;
    // dk / dv only for self-attention (the same rows, the same geometry)
    if ((dk || dv) && (m != n || rs_kv != rs || kv_batch != batch)) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t bh = batch * heads;
    const AtKV kv{static_cast<int>(m), rs_kv, kv_batch == 1 && batch > 1};
    switch (d) {
        case 40: return attn_bwd_d<40>(q, k, v, out, dout, lse, bh, heads, n, rs, ro, kv, scale, delta, dq, dk, dv, s);
        case 80: return attn_bwd_d<80>(q, k, v, out, dout, lse, bh, heads, n, rs, ro, kv, scale, delta, dq, dk, dv, s);
        default: return attn_bwd_d<160>(q, k, v, out, dout, lse, bh, heads, n, rs, ro, kv, scale, delta, dq, dk, dv, s);
    }
}

int sp_attention_fwd(const float* q, const float* k, const float* v, int64_t bh, int64_t n,
                     int32_t d, float scale, float* out, float* lse, sp_stream_t stream) {
    if (!sp_attention_supported(bh, n, n, d)) return SP_EINVAL;
    return sp_attention_fwd_mh(q, k, v, bh, 1, n, n, d, d, d, bh, d, scale, out, lse, stream);
}

int sp_attention_bwd(const float* q, const float* k, const float* v, const float* out,
                     const float* dout, const float* lse, int64_t bh, int64_t n, int32_t d,
                     float scale, float* delta, float* dq, float* dk, float* dv,
                     sp_stream_t stream) {
    if (!sp_attention_supported(bh, n, n, d)) return SP_EINVAL;
    return sp_attention_bwd_mh(q, k, v, out, dout, lse, bh, 1, n, n, d, d, d, bh, d, scale, delta, dq, dk, dv,
                               stream);
}

}  // extern "C"

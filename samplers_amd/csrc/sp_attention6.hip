// Fused self-attention softmax(q k^T * scale) v on the bf16 MFMA datapath with exact
// three-term splits of the fp32 operands (the method of sp_gemm_x6.hip: every fp32 value is
// h + m + l, three bf16 terms, exactly; each product is the six partial products down to
// 2^-16 relative, accumulated in fp32 in two accumulators — the leading h x h product apart).
// Same contract, layouts and lse as k_attn_fwd (sp_attention.hip) for the SD 1.5 ε-UNet's
// attn1 over 4096 / 1024 latent tokens at head dims 40 / 80 (stable_diffusion.py:306-313 via
// diffusers' Attention): the fp32 kernel runs fp32 MFMA (64 FLOP/clk/SIMD) with the softmax's
// VALU work on the same datapath; here the products run at the bf16 rate (1024 FLOP/clk/SIMD,
// six of them per product) and VALU work beside bf16 MFMAs is nearly free.
//
// Per wave: 32 queries; per 32-key block
//   S^T = K Q^T          v_mfma_f32_32x32x16_bf16, K as A (rows = keys), Q^T as B held in
//                        registers (split once); d padded to 16 (40 -> 48)
//   softmax              lane = query (C column), its 16 keys in registers + one xor-32 lane
//   O^T += V^T P^T       P^T straight from the S^T accumulators as the B operand (the key
//                        order inside the MFMA's K is permuted to the C layout's, and V^T is
//                        staged in LDS in that order); d padded to 32 (40 -> 64)
// K and V^T are split into their terms once per workgroup, when a stage of SB keys is written
// to LDS (bf16, three planes), so the waves read ready MFMA fragments (one ds_read_b128 each).
//
// C layout of v_mfma_f32_32x32x16_bf16: register i of lane l is row (i&3) + 8(i>>2) + 4(l>>5),
// column l&31; A/B fragments: lane l holds A[row l&31][k 8(l>>5) + j] / B[k 8(l>>5) + j][col l&31],
// j = 0..7 (cdna_hip_programming.md §3).

#define SP_TU 13  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

#include <algorithm>
#include <cmath>

namespace sp {

typedef float a6_f16 __attribute__((ext_vector_type(16)));
typedef unsigned a6_u4 __attribute__((ext_vector_type(4)));
typedef unsigned a6_u2 __attribute__((ext_vector_type(2)));
typedef __bf16 a6_bf8 __attribute__((ext_vector_type(8)));

constexpr float A6_LOG2E = 1.4426950408889634f;
constexpr float A6_LN2 = 0.6931471805599453f;
constexpr int A6_WAVES = 4;
constexpr int A6_QW = 32;                    // queries per wave
constexpr int A6_WB = A6_WAVES * A6_QW;      // queries per workgroup
constexpr float A6_LAZY = 8.f;               // log2 headroom of the lazily moved running max

#ifndef A6_EXP
#define A6_EXP 0  // diagnostics only: 7 = each 32x32x16 MFMA replaced by two 16x16x32 ones on the same
                  // operands (the same MACs, wrong results): the clock the chip holds per MFMA shape
#endif
__device__ __forceinline__ a6_f16 a6_mfma(a6_u4 a, a6_u4 b, a6_f16 c) {
#if A6_EXP == 7
    typedef float a6_f4 __attribute__((ext_vector_type(4)));
    a6_f4 c0 = {c[0], c[1], c[2], c[3]}, c1 = {c[4], c[5], c[6], c[7]};
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(a6_bf8, a), __builtin_bit_cast(a6_bf8, b), c0,
                                                 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(a6_bf8, b), __builtin_bit_cast(a6_bf8, a), c1,
                                                 0, 0, 0);
    c[0] = c0[0], c[1] = c0[1], c[2] = c0[2], c[3] = c0[3], c[4] = c1[0], c[5] = c1[1], c[6] = c1[2], c[7] = c1[3];
    return c;
#else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(a6_bf8, a), __builtin_bit_cast(a6_bf8, b), c,
                                                   0, 0, 0);
#endif
}

// the bf16 halves (upper 16 bits) of a and b as one dword: a low, b high
__device__ __forceinline__ unsigned a6_pack(unsigned a, unsigned b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }

typedef float a6_f2 __attribute__((ext_vector_type(2)));

// two values -> their three term pairs (a low, b high): the truncations as two ANDs, the
// subtractions as one packed op; a term's bf16 value is the upper half of its fp32 pattern, so
// the packs read h from the values themselves
struct A6T3 { unsigned h, m, l; };
__device__ __forceinline__ A6T3 a6_split2(float a, float b) {
    const a6_f2 v = {a, b};
    const a6_f2 h = {__uint_as_float(__float_as_uint(a) & 0xffff0000u), __uint_as_float(__float_as_uint(b) & 0xffff0000u)};
    const a6_f2 r = v - h;
    const a6_f2 m = {__uint_as_float(__float_as_uint(r.x) & 0xffff0000u), __uint_as_float(__float_as_uint(r.y) & 0xffff0000u)};
    const a6_f2 l = r - m;
    return A6T3{a6_pack(__float_as_uint(a), __float_as_uint(b)), a6_pack(__float_as_uint(r.x), __float_as_uint(r.y)),
                a6_pack(__float_as_uint(l.x), __float_as_uint(l.y))};
}

// eight values -> the three term fragments (element j of each)
__device__ __forceinline__ void a6_split8(const float (&v)[8], a6_u4 (&t)[3]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const A6T3 x = a6_split2(v[2 * q], v[2 * q + 1]);
        t[0][q] = x.h, t[1][q] = x.m, t[2][q] = x.l;
    }
}

// six partial products of one MFMA tile into one accumulator, small ones first (the score
// products: K = 48 or 80 terms per sum)
__device__ __forceinline__ void a6_prod6_1(const a6_u4 (&a)[3], const a6_u4 (&b)[3], a6_f16& acc) {
    acc = a6_mfma(a[0], b[1], acc);
    acc = a6_mfma(a[1], b[0], acc);
    acc = a6_mfma(a[0], b[2], acc);
    acc = a6_mfma(a[2], b[0], acc);
    acc = a6_mfma(a[1], b[1], acc);
    acc = a6_mfma(a[0], b[0], acc);
}

// six partial products of one MFMA tile: the leading one into ah, the five small ones into as
// (the output's sums run over all n keys)
__device__ __forceinline__ void a6_prod6(const a6_u4 (&a)[3], const a6_u4 (&b)[3], a6_f16& ah, a6_f16& as) {
    as = a6_mfma(a[0], b[1], as);
    as = a6_mfma(a[1], b[0], as);
    as = a6_mfma(a[0], b[2], as);
    as = a6_mfma(a[2], b[0], as);
    as = a6_mfma(a[1], b[1], as);
    ah = a6_mfma(a[0], b[0], ah);
}

// key k of a 16-key group -> its position in the MFMA's K order: bits 2 and 3 swapped, so that
// lane half h's eight C rows of one register half (keys 4h + {0..3, 8..11}) are positions
// 8h .. 8h + 7
__device__ __forceinline__ int a6_pos(int k) { return (k & ~12) | ((k & 4) << 1) | ((k & 8) >> 1); }

template <int D>
struct A6Geo {
    static_assert(D == 40 || D == 80, "head dim");
    static constexpr int DK = (D + 15) / 16;       // 16-wide d steps of S^T = K Q^T
    static constexpr int DKP = DK * 16;
    static constexpr int DT = (D + 31) / 32;       // 32-row d tiles of O^T
    static constexpr int SB = 64;                  // keys per LDS stage
    static constexpr int KROW = DKP + 8;           // bf16 per K row in LDS (16-B aligned rows)
    static constexpr int VROW = SB + 8;            // bf16 per V^T row (one d) in LDS
    static constexpr int KPLANE = SB * KROW;       // bf16 per term plane
    static constexpr int VPLANE = DT * 32 * VROW;
    static constexpr int VPLANE_PRE = D * VROW;    // V^T plane of a pre-split stage image (rows < D)
    static constexpr int IMG = 3 * KPLANE + 3 * VPLANE_PRE;  // bf16 per pre-split stage image
    static constexpr int NI4 = (IMG / 8 + kBlock - 1) / kBlock;  // 16-byte pieces per thread
    static_assert(IMG % 8 == 0 && KPLANE % 8 == 0, "16-byte pieces");
    static constexpr int NK4 = (SB * D / 4 + kBlock - 1) / kBlock;        // K float4 per thread
    static constexpr int NVU = (SB / 2 * D / 4 + kBlock - 1) / kBlock;    // V (2 keys x 4 d) units
};

template <int D>
struct A6Stage {
    float4 k[A6Geo<D>::NK4];
    float4 v[A6Geo<D>::NVU][2];
};

template <int D>
__device__ __forceinline__ void a6_load(const float* __restrict__ kb, const float* __restrict__ vb, int rs,
                                        A6Stage<D>& st) {
    using G = A6Geo<D>;
#pragma unroll
    for (int j = 0; j < G::NK4; ++j) {
        const int i = threadIdx.x + j * kBlock;
        if (i < G::SB * D / 4) {
            const int row = (4 * i) / D, col = 4 * i - row * D;
            st.k[j] = *reinterpret_cast<const float4*>(kb + (int64_t)row * rs + col);
        }
    }
#pragma unroll
    for (int j = 0; j < G::NVU; ++j) {
        const int u = threadIdx.x + j * kBlock;
        if (u < G::SB / 2 * D / 4) {
            const int p = u / (D / 4), d0 = 4 * (u - p * (D / 4));
            st.v[j][0] = *reinterpret_cast<const float4*>(vb + (int64_t)(2 * p) * rs + d0);
            st.v[j][1] = *reinterpret_cast<const float4*>(vb + (int64_t)(2 * p + 1) * rs + d0);
        }
    }
}

// the staged rows -> split terms: K [term][key][d], V^T [term][d][key position] (V^T planes
// vplane bf16 apart) — into LDS, or into the workspace image of a stage (k_attn6_split)
template <int D>
__device__ __forceinline__ void a6_store(unsigned short* Ks, unsigned short* Vs, int vplane, const A6Stage<D>& st) {
    using G = A6Geo<D>;
#pragma unroll
    for (int j = 0; j < G::NK4; ++j) {
        const int i = threadIdx.x + j * kBlock;
        if (i < G::SB * D / 4) {
            const int row = (4 * i) / D, col = 4 * i - row * D;
            const A6T3 x = a6_split2(st.k[j].x, st.k[j].y), y = a6_split2(st.k[j].z, st.k[j].w);
            unsigned short* dst = Ks + row * G::KROW + col;
            *reinterpret_cast<a6_u2*>(dst) = a6_u2{x.h, y.h};
            *reinterpret_cast<a6_u2*>(dst + G::KPLANE) = a6_u2{x.m, y.m};
            *reinterpret_cast<a6_u2*>(dst + 2 * G::KPLANE) = a6_u2{x.l, y.l};
        }
    }
#pragma unroll
    for (int j = 0; j < G::NVU; ++j) {
        const int u = threadIdx.x + j * kBlock;
        if (u < G::SB / 2 * D / 4) {
            const int p = u / (D / 4), d0 = 4 * (u - p * (D / 4));
            const int key = 2 * p, pos = (key & ~15) | a6_pos(key & 15);  // keys 2p, 2p + 1 adjacent
            const float a[4] = {st.v[j][0].x, st.v[j][0].y, st.v[j][0].z, st.v[j][0].w};
            const float b[4] = {st.v[j][1].x, st.v[j][1].y, st.v[j][1].z, st.v[j][1].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const A6T3 x = a6_split2(a[e], b[e]);
                unsigned short* dst = Vs + (d0 + e) * G::VROW + pos;
                *reinterpret_cast<unsigned*>(dst) = x.h;
                *reinterpret_cast<unsigned*>(dst + vplane) = x.m;
                *reinterpret_cast<unsigned*>(dst + 2 * vplane) = x.l;
            }
        }
    }
}

__device__ __forceinline__ a6_u4 a6_lds16(const unsigned short* p) { return *reinterpret_cast<const a6_u4*>(p); }

// K / V of every stage of every head split once into their term images (the LDS layout of a
// stage; K's padding columns zero), so that the attention workgroups — n / 128 per head, each
// reading all n keys — copy ready fragments instead of splitting them again.
template <int D>
__global__ __launch_bounds__(kBlock) void k_attn6_split(const float* __restrict__ k, const float* __restrict__ v,
                                                        int n, int heads, int rs, unsigned short* __restrict__ ws) {
    using G = A6Geo<D>;
    const int si = blockIdx.x, bh = blockIdx.y, b = bh / heads;
    const int64_t base = (int64_t)b * n * rs + (int64_t)(bh - b * heads) * D + (int64_t)si * G::SB * rs;
    unsigned short* img = ws + ((int64_t)bh * (n / G::SB) + si) * G::IMG;
    A6Stage<D> st;
    a6_load<D>(k + base, v + base, rs, st);
    a6_store<D>(img, img + 3 * G::KPLANE, G::VPLANE_PRE, st);
    if constexpr (G::DKP > D) {
        for (int i = threadIdx.x; i < 3 * G::SB; i += kBlock)
#pragma unroll
            for (int c = D; c < G::DKP; c += 2)
                *reinterpret_cast<unsigned*>(img + (i / G::SB) * G::KPLANE + (i % G::SB) * G::KROW + c) = 0u;
    }
}

// Workgroup: 128 queries of one (batch, head), 4 waves of 32; keys in stages of SB through LDS.
// PRE: the stages come pre-split from k_attn6_split's images (ws), copied to LDS as they are;
// else each workgroup splits K and V itself while staging them.
template <int D, bool PRE>
__global__ __launch_bounds__(kBlock) void k_attn6_fwd(const float* __restrict__ q, const float* __restrict__ k,
                                                      const float* __restrict__ v, int n, int heads, int rs,
                                                      int ro, float sl2, float* __restrict__ out,
                                                      float* __restrict__ lse, const unsigned short* __restrict__ ws) {
    using G = A6Geo<D>;
    // V^T planes VP apart: a pre-split image holds rows < D only (rows D .. 32 DT - 1 of a plane
    // then read the next plane's, or the tail's, values: they feed only the discarded output rows)
    constexpr int VP = PRE ? G::VPLANE_PRE : G::VPLANE;
    __shared__ __attribute__((aligned(16))) unsigned short Ks[3 * G::KPLANE];
    __shared__ __attribute__((aligned(16))) unsigned short Vs[2 * VP + G::VPLANE];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, r = lane & 31, hh = lane >> 5;
    const int bh = blockIdx.y, b = bh / heads;
    const int64_t base = (int64_t)b * n * rs + (int64_t)(bh - b * heads) * D;  // q, k, v of this head
    const int q0 = blockIdx.x * A6_WB + wv * A6_QW;
    SP_DCHECK(rs >= heads * D && ro >= heads * D && (int64_t)(blockIdx.x + 1) * A6_WB <= n && n % G::SB == 0);

    // K's padding columns d >= D are never written by the staging: zero them once
    if constexpr (!PRE && G::DKP > D) {
        for (int i = threadIdx.x; i < 3 * G::SB; i += kBlock)
#pragma unroll
            for (int c = D; c < G::DKP; c += 2)
                *reinterpret_cast<unsigned*>(Ks + (i / G::SB) * G::KPLANE + (i % G::SB) * G::KROW + c) = 0u;
    }
    // Q^T as the B operand of S^T = K Q^T: lane (query r, half hh) holds Q[q0 + r][16 s + 8 hh + j]
    // scaled by scale * log2 e, split into its terms
    a6_u4 qf[G::DK][3];
#pragma unroll
    for (int s = 0; s < G::DK; ++s) {
        float f[8];
        const int d0 = 16 * s + 8 * hh;
        const float* qr = q + base + (int64_t)(q0 + r) * rs + d0;
        if (d0 + 8 <= D) {
            const float4 a = reinterpret_cast<const float4*>(qr)[0], c = reinterpret_cast<const float4*>(qr)[1];
            f[0] = a.x * sl2, f[1] = a.y * sl2, f[2] = a.z * sl2, f[3] = a.w * sl2;
            f[4] = c.x * sl2, f[5] = c.y * sl2, f[6] = c.z * sl2, f[7] = c.w * sl2;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = 0.f;
        }
        a6_split8(f, qf[s]);
    }
    a6_f16 oh[G::DT], os[G::DT];
#pragma unroll
    for (int dt = 0; dt < G::DT; ++dt) oh[dt] = a6_f16{}, os[dt] = a6_f16{};
    float m = -INFINITY, l = 0.f;

    const float* __restrict__ kb = k + base;
    const float* __restrict__ vb = v + base;
    const int nst = n / G::SB;
    const a6_u4* __restrict__ imgs = reinterpret_cast<const a6_u4*>(ws + (int64_t)bh * nst * G::IMG);
    A6Stage<D> st;
    a6_u4 pre[G::NI4];
    auto load_stage = [&](int si) {
        if constexpr (PRE) {
#pragma unroll
            for (int j = 0; j < G::NI4; ++j) {
                const int i = threadIdx.x + j * kBlock;
                if (i < G::IMG / 8) pre[j] = imgs[(int64_t)si * (G::IMG / 8) + i];
            }
        } else {
            a6_load<D>(kb + (int64_t)si * G::SB * rs, vb + (int64_t)si * G::SB * rs, rs, st);
        }
    };
    load_stage(0);
    for (int si = 0; si < nst; ++si) {
        __syncthreads();  // the previous stage's fragment reads are done
        if constexpr (PRE) {  // the image: K planes, then V^T planes, contiguous in LDS as well
#pragma unroll
            for (int j = 0; j < G::NI4; ++j) {
                const int i = threadIdx.x + j * kBlock;
                if (i < G::IMG / 8) {
                    unsigned short* dst = i < 3 * G::KPLANE / 8 ? Ks + 8 * i : Vs + 8 * i - 3 * G::KPLANE;
                    *reinterpret_cast<a6_u4*>(dst) = pre[j];
                }
            }
        } else {
            a6_store<D>(Ks, Vs, G::VPLANE, st);
        }
        __syncthreads();
        if (si + 1 < nst) load_stage(si + 1);
#pragma unroll
        for (int kb32 = 0; kb32 < G::SB / 32; ++kb32) {
            // S^T block: keys kb32 * 32 + row, queries q0 + r
            a6_f16 sv = a6_f16{};
#pragma unroll
            for (int s = 0; s < G::DK; ++s) {
                const unsigned short* ka = Ks + (kb32 * 32 + r) * G::KROW + 16 * s + 8 * hh;
                const a6_u4 kf[3] = {a6_lds16(ka), a6_lds16(ka + G::KPLANE), a6_lds16(ka + 2 * G::KPLANE)};
                a6_prod6_1(kf, qf[s], sv);
            }
            float bm = -INFINITY;
#pragma unroll
            for (int i = 0; i < 16; ++i) bm = fmaxf(bm, sv[i]);
            bm = fmaxf(bm, __shfl_xor(bm, 32));
            // lazy rescaling: the reference point m moves only when a block's max exceeds it by
            // more than A6_LAZY (weights up to 2^A6_LAZY are exact in the split products and the
            // fp32 sums; the normalisation divides by the same sum), so most blocks skip the
            // accumulators' rescale
            const float mn = bm > m + A6_LAZY ? bm : m;
            const float corr = __builtin_amdgcn_exp2f(m - mn);  // 0 on the first block (m = -inf)
            m = mn;
            float p[16], ps = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                p[i] = __builtin_amdgcn_exp2f(sv[i] - mn);
                ps += p[i];
            }
            l = fmaf(l, corr, ps);
            // rescale only when some query's running max moved (skipping a multiply by 1 changes
            // no bit)
            if (__builtin_amdgcn_ballot_w64(corr != 1.f))
#pragma unroll
                for (int dt = 0; dt < G::DT; ++dt) oh[dt] *= corr, os[dt] *= corr;
            // P^T as the B operand: register half kk (keys 16 kk .. + 15 of the block) in position
            // order 8 hh + j = its registers 8 kk + j
            a6_u4 pf[2][3];
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                float f[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) f[j] = p[8 * kk + j];
                a6_split8(f, pf[kk]);
            }
            // O^T += V^T P^T: A = V^T rows d, K = the block's key positions
#pragma unroll
            for (int dt = 0; dt < G::DT; ++dt)
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    const unsigned short* va = Vs + (dt * 32 + r) * G::VROW + kb32 * 32 + kk * 16 + 8 * hh;
                    const a6_u4 vf[3] = {a6_lds16(va), a6_lds16(va + VP), a6_lds16(va + 2 * VP)};
                    a6_prod6(vf, pf[kk], oh[dt], os[dt]);
                }
        }
    }
    // O = O^T / rowsum: lane (query q0 + r) holds d = 32 dt + (i&3) + 8 (i>>2) + 4 hh
    const float tot = l + __shfl_xor(l, 32);
    const float inv = 1.f / tot;
    const int qq = q0 + r;
    float* orow = out + (int64_t)b * n * ro + (int64_t)(bh - b * heads) * D + (int64_t)qq * ro;
#pragma unroll
    for (int dt = 0; dt < G::DT; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int d0 = 32 * dt + 8 * g4 + 4 * hh;
            if (d0 + 4 <= D)
                *reinterpret_cast<float4*>(orow + d0) = make_float4(
                    (oh[dt][4 * g4] + os[dt][4 * g4]) * inv, (oh[dt][4 * g4 + 1] + os[dt][4 * g4 + 1]) * inv,
                    (oh[dt][4 * g4 + 2] + os[dt][4 * g4 + 2]) * inv, (oh[dt][4 * g4 + 3] + os[dt][4 * g4 + 3]) * inv);
        }
    if (hh == 0) lse[(int64_t)bh * n + qq] = (m + log2f(tot)) * A6_LN2;
}

template <int D>
static int64_t attn6_ws_bytes(int64_t bh, int64_t n) { return bh * (n / A6Geo<D>::SB) * A6Geo<D>::IMG * 2; }

template <int D>
static int attn6_fwd_d(const float* q, const float* k, const float* v, int64_t batch, int heads, int64_t n,
                       int rs, int ro, float scale, float* out, float* lse, void* ws, int64_t ws_bytes,
                       hipStream_t s) {
    using G = A6Geo<D>;
    const int64_t bh = batch * heads;
    const double flops = 4.0 * bh * n * n * D;
    const dim3 grid(static_cast<unsigned>(n / A6_WB), static_cast<unsigned>(bh));
    auto* w = static_cast<unsigned short*>(ws);
    if (w && ws_bytes >= attn6_ws_bytes<D>(bh, n)) {
        launch(0, k_attn6_split<D>, dim3(static_cast<unsigned>(n / G::SB), static_cast<unsigned>(bh)), dim3(kBlock),
               s, k, v, static_cast<int>(n), heads, rs, w);
        launch_w(0, flops, k_attn6_fwd<D, true>, grid, dim3(kBlock), s, q, k, v, static_cast<int>(n), heads, rs, ro,
                 scale * A6_LOG2E, out, lse, static_cast<const unsigned short*>(w));
    } else {
        launch_w(0, flops, k_attn6_fwd<D, false>, grid, dim3(kBlock), s, q, k, v, static_cast<int>(n), heads, rs,
                 ro, scale * A6_LOG2E, out, lse, static_cast<const unsigned short*>(nullptr));
    }
    return check_launch("sp_attention6_fwd");
}

}  // namespace sp

using namespace sp;

static int g_attn6 = 1;  // sp_attention_bf16x6

extern "C" {

// Self-attention forward on the split-bf16 kernel: q, k, v rows of stride rs (the thirds of a
// fused projection when rs = 3 heads d), out rows of stride ro, lse [batch heads][n] (natural
// log), as sp_attention_fwd_mh with m = n and one K/V per sample.
int sp_attention6_supported(int64_t batch, int32_t heads, int64_t n, int32_t d) {
    if (batch <= 0 || heads <= 0 || batch * heads > 65535 || n <= 0 || n > (int64_t(1) << 24)) return 0;
    if (d != 40 && d != 80) return 0;
    return n % A6_WB == 0 && n % A6Geo<40>::SB == 0;
}

// bytes of the pre-split K / V images sp_attention6_fwd_ws uses (0: unsupported shape)
int64_t sp_attention6_workspace(int64_t batch, int32_t heads, int64_t n, int32_t d) {
    if (!sp_attention6_supported(batch, heads, n, d)) return 0;
    return d == 40 ? attn6_ws_bytes<40>(batch * heads, n) : attn6_ws_bytes<80>(batch * heads, n);
}

// ws (or NULL): sp_attention6_workspace() bytes for K / V split once per head (k_attn6_split)
// instead of once per workgroup; the library allocates nothing
int sp_attention6_fwd_ws(const float* q, const float* k, const float* v, int64_t batch, int32_t heads, int64_t n,
                         int32_t d, int32_t rs, int32_t ro, float scale, float* out, float* lse, void* ws,
                         int64_t ws_bytes, sp_stream_t stream) {
    if (!sp_attention6_supported(batch, heads, n, d) || !q || !k || !v || !out || !lse) return SP_EINVAL;
    if (rs < heads * d || ro < heads * d || rs % 4 || ro % 4 || batch * n * (int64_t)std::max(rs, ro) >= (int64_t(1) << 40))
        return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (d == 40) return attn6_fwd_d<40>(q, k, v, batch, heads, n, rs, ro, scale, out, lse, ws, ws_bytes, s);
    return attn6_fwd_d<80>(q, k, v, batch, heads, n, rs, ro, scale, out, lse, ws, ws_bytes, s);
}

int sp_attention6_fwd_mh(const float* q, const float* k, const float* v, int64_t batch, int32_t heads, int64_t n,
                         int32_t d, int32_t rs, int32_t ro, float scale, float* out, float* lse,
                         sp_stream_t stream) {
    return sp_attention6_fwd_ws(q, k, v, batch, heads, n, d, rs, ro, scale, out, lse, nullptr, 0, stream);
}

// 1: sp_attention_fwd / _fwd_mh run self-attention at the supported shapes on the split-bf16
// kernel (default); 0: the exact-fp32 kernel; < 0 query.  Returns the previous setting.
int sp_attention_bf16x6(int32_t enable) {
    const int prev = g_attn6;
    if (enable >= 0) g_attn6 = enable ? 1 : 0;
    return prev;
}

int sp_attention_bf16x6_enabled(void) { return g_attn6; }

}  // extern "C"

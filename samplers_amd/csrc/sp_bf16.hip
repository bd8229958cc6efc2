// The priors at the reference's reduced precision (scripts/run_psld.py:14-20 runs SD 1.5 in bf16;
// stable_diffusion.py:90-101 / ddpm.py:23-34 take any torch_dtype): bf16 activations in HBM,
// bf16 operands on the bf16 MFMAs, fp32 accumulation and fp32 statistics.
//
// Layout: channels-last (NHWC) activations.  The 3x3 convolution is an implicit GEMM whose
// contraction runs over (tap, input channel); with the channels innermost, the eight channels a
// lane feeds to one MFMA are 16 contiguous bytes of one pixel, so the input patch is staged
// into LDS as [pixel][16 channels] rows and every MFMA operand is one ds_read_b128 — no
// transposes anywhere (NCHW would put the contraction index at a stride of H*W).  The same
// layout is the token layout of the transformer blocks ([b][h w][c]).
//
//   k_conv3x3_bf16<TC>   3x3 / stride 1 / padding 1 convolution (+ fp32 bias, + bf16 residual)
//                        and, with the flipped / transposed weight pack, its input VJP
//   k_gnb_stats / _final / _apply / _bwd_*   GroupNorm(+per-(n,c) bias)(+SiLU) forward and
//                        input VJP: per-chunk channel partial sums (shifted), a per-group
//                        finalize in fp64, and a streaming apply — two reads and one write of
//                        the bf16 tensor forward
//   k_attnb_fwd<D>       multi-head attention softmax(q k^T / sqrt(d)) v on bf16 q / k / v
//                        (self or cross, keys past m masked), output bf16, row log-sum-exp fp32
//
// C layout of v_mfma_f32_32x32x16_bf16: register i of lane l is row (i&3) + 8(i>>2) + 4(l>>5),
// column l&31; A/B fragments: lane l holds A[row l&31][k 8(l>>5) + j] / B[k 8(l>>5) + j][col l&31],
// j = 0..7 (cdna_hip_programming.md §3).

#define SP_TU 14  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

#include <algorithm>
#include <cmath>

namespace sp {

typedef float bq_f16 __attribute__((ext_vector_type(16)));
typedef unsigned bq_u4 __attribute__((ext_vector_type(4)));
typedef unsigned bq_u2 __attribute__((ext_vector_type(2)));
typedef __bf16 bq_bf8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16;


#ifndef SP_CONV_XCD
#define SP_CONV_XCD 1  // XCD-aware workgroup order of the bf16 conv tile (k_conv3x3_bf16)
#endif
constexpr bool kConvXcdRemap = SP_CONV_XCD != 0;
#ifndef BQ_EXP
#define BQ_EXP 0  // diagnostics only: 7 = each 32x32x16 MFMA replaced by two 16x16x32 ones on the same
                  // operands (the same MACs, wrong results): the clock the chip holds per MFMA shape;
                  // 8 = the TC = 32 conv's fragment reads after tap 0 removed (wrong results);
                  // 9 = its global loads after the first two stages removed (wrong results);
                  // 10 = every patch load from one cached line (weights as usual; wrong results)
#endif
__device__ __forceinline__ bq_f16 bq_mfma(bq_u4 a, bq_u4 b, bq_f16 c) {
#if BQ_EXP == 7
    typedef float bq_f4 __attribute__((ext_vector_type(4)));
    bq_f4 c0 = {c[0], c[1], c[2], c[3]}, c1 = {c[4], c[5], c[6], c[7]};
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bq_bf8, a), __builtin_bit_cast(bq_bf8, b), c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bq_bf8, b), __builtin_bit_cast(bq_bf8, a), c1, 0, 0, 0);
    c[0] = c0[0], c[1] = c0[1], c[2] = c0[2], c[3] = c0[3], c[4] = c1[0], c[5] = c1[1], c[6] = c1[2], c[7] = c1[3];
    return c;
#else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bq_bf8, a), __builtin_bit_cast(bq_bf8, b), c,
                                                   0, 0, 0);
#endif
}

__device__ __forceinline__ float bf_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ float bf1(u16 v) { return __uint_as_float(static_cast<unsigned>(v) << 16); }
// round to nearest even (v_cvt_pk_bf16_f32)
__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, static_cast<__bf16>(f)); }
__device__ __forceinline__ unsigned pk2(float a, float b) {
    return static_cast<unsigned>(f2bf(a)) | (static_cast<unsigned>(f2bf(b)) << 16);
}
__device__ __forceinline__ void unpack8(bq_u4 v, float (&f)[8]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) f[2 * i] = bf_lo(v[i]), f[2 * i + 1] = bf_hi(v[i]);
}
__device__ __forceinline__ bq_u4 pack8(const float (&f)[8]) {
    return bq_u4{pk2(f[0], f[1]), pk2(f[2], f[3]), pk2(f[4], f[5]), pk2(f[6], f[7])};
}
__device__ __forceinline__ float silu_f(float y) { return y * __builtin_amdgcn_rcpf(1.f + __expf(-y)); }

// ---------------------------------------------------------------------------------------------
// 3x3 convolution, NHWC, implicit GEMM on v_mfma_f32_32x32x16_bf16.
//
// Workgroup: 64 output channels x 512 output pixels, 4 waves; wave w holds all 64 channels of
// pixels 128 w .. 128 w + 127 (2 x 4 MFMA tiles of 32 x 32: channels as A rows, pixels as B
// columns, 128 accumulators).  The 512 pixels are TR "virtual rows" of TC columns: TC = 32 for
// W % 32 == 0 (16 image rows of one sample), TC = W = H for the 16 / 8 / 4 levels (S whole
// samples per tile, each with its own zero halo rows).  The contraction is staged 16 input
// channels at a time: the weights of the stage ([tap][64 co][16 ci]) and the input patch
// ([S (SR + 2) rows][TC + 2 cols][16 ci], zero halo) go to LDS as 48-byte rows (32 bytes + 16
// pad: the 16 lanes of a ds_read_b128 group then read 16 distinct 4-bank slots for any start
// pixel), 9 taps x 8 MFMAs per wave per stage; the next stage's global loads are issued into
// registers before the current stage's MFMAs.
// ---------------------------------------------------------------------------------------------
#ifndef SP_CONV_PRIO
#define SP_CONV_PRIO 0  // wave priority around the TC = 32 pipeline's phases (A/B knob, 0 = none)
#endif

// threadIdx.x re-read opaque to the compiler: the shortcut stages' per-thread addresses are then
// formed inside their loop instead of being hoisted ahead of the 3x3 loop (where they were live
// across it: the kernel spilled ~200 VGPRs)
__device__ __forceinline__ int cv_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

template <int TC>
struct CvGeo {
    static_assert(TC == 32 || TC == 16 || TC == 8 || TC == 4, "tile width");
    static constexpr int PX = 512;
    static constexpr int TR = PX / TC;                // virtual rows per tile
    static constexpr int SR = TC == 32 ? 16 : TC;     // image rows per sample segment
    static constexpr int S = TR / SR;                 // sample segments per tile
    static constexpr int PW = TC + 2;                 // patch columns
    static constexpr int PH = S * (SR + 2);           // patch rows
    static constexpr int PQ = PH * PW;                // patch pixels
    // TC = 32: 32-byte rows with the two 16-byte halves swapped on every other group of 8 rows
    // (weights) / 8 columns (patch) — conflict-free for the fragment reads — and two stage
    // buffers; else 48-byte rows (32 bytes + 16 pad), one buffer
    static constexpr bool DB = TC == 32;
    static constexpr int RB = DB ? 32 : 48;           // LDS bytes per row
    static constexpr int WROWS = 9 * 64;              // weight rows per stage
    static constexpr int LW = WROWS * RB;
    static constexpr int LP = PQ * RB;
    static constexpr int BUF = LW + LP;               // one stage
    static constexpr int LDS = DB ? 2 * BUF : BUF;
    static constexpr int NW = (WROWS * 2 + kBlock - 1) / kBlock;  // 16-byte weight pieces per thread
    static constexpr int PQP = PQ;
    static constexpr int NP = (PQP * 2 + kBlock - 1) / kBlock;    // 16-byte patch pieces per thread
};

// 16-byte piece p of an LDS image of 32-byte rows (48-byte stride): row p / 2, chunk p % 2 —
// consecutive lanes read the two halves of a pixel's 32 bytes (measured faster than writing one
// chunk of 64 rows per instruction, which avoids the 2-way ds_write conflicts but doubles the
// cache lines each global load instruction touches: -8 % on the 64x64 / 512x512 layers)
__device__ __forceinline__ int cv_row(int p) { return p >> 1; }
__device__ __forceinline__ int cv_chunk(int p) { return p & 1; }

// UP: the input is the half-resolution tensor of diffusers' Upsample2D and the patch reads
// pixel (h >> 1, w >> 1) of it for full-resolution pixel (h, w): conv(upsample_nearest2x(x))
// without the upsampled tensor in HBM.
// part != NULL (split-K, gridDim.z parts over the input-channel stages): part z of the
// contraction is stored as fp32 to part[z][n h w][cout] without bias / residual (k_conv_reduce).
// SC (TC = 32): a 1x1 convolution of cat(xs1, xs2) (cs1 + cs2 channels, NHWC, the ResnetBlock's
// conv_shortcut) is summed into the same accumulators as (cs1 + cs2) / 16 further stages of the
// contraction — weights wsp [co block of 64][cs / 16][64 co][16 ci], the stage's 512 pixels
// written to the patch centre and read by the centre tap only (8 MFMAs per wave) — so the
// shortcut's output is never written to HBM nor read back as a residual.
// GS (TC = 32, unsplit): the output y is the cotangent dz of a GroupNorm(+SiLU) over cat(gx1, gx2)
// (gc1 + gc2 = cout channels, NHWC) and the epilogue also emits that GroupNorm VJP's per-(tile,
// channel) sums sum(g), sum(g xhat) (g = dz act'(y) gamma) over the tile's 512 pixels, from dz as
// stored (bf16) and the per-(n, c) coefficients gco = [sc | sh | xs | xo] (k_gnb_coefs): gpart
// [n][tile][2][cout], tile = the tile's index within its sample — the layout k_gnb_final_bwd
// reads, so the separate sums pass (x and dz read again) is not run.
// FS (TC = 32, unsplit): the output y feeds a GroupNorm over y + cb (cb = gn.co: per-(n, c) fp32
// or NULL) and the epilogue emits its per-(tile, channel) shifted moments from y as stored:
// gpart [n][tile][3][cout] = sum(d), sum(d^2), K with d = y + cb - K and K the tile's first pixel's
// y + cb (k_gnb_final_fwd_tiles) — the forward statistics pass is not run.
struct ConvGn {
    const u16* x1;
    const u16* x2;
    int c1, act;
    const float* co;
    const float* gamma;
    float* part;
};

template <int TC, bool UP, bool BLK = false, bool SC = false, bool GS = false, bool FS = false>
__global__ __launch_bounds__(kBlock, TC == 4 ? 1 : 2) void k_conv3x3_bf16(const u16* __restrict__ x, const u16* __restrict__ wp,
                                                         const float* __restrict__ bias, const u16* __restrict__ res,
                                                         int n, int cin, int cout, int h, int w,
                                                         u16* __restrict__ y, float* __restrict__ part,
                                                         const u16* __restrict__ xs1, const u16* __restrict__ xs2,
                                                         int cs1, int cs2, const u16* __restrict__ wsp, ConvGn gn) {
    static_assert(!SC || (TC == 32 && !UP), "shortcut stages: TC = 32 tiles");
    static_assert(!GS || (TC == 32 && !UP && !SC), "GroupNorm VJP sums: TC = 32 tiles");
    static_assert(!FS || (TC == 32 && !UP && !GS), "GroupNorm moments: TC = 32 tiles");
    using G = CvGeo<TC>;
    __shared__ __attribute__((aligned(16))) char lds[G::LDS];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
    // XCD-aware order: the hardware deals workgroups to the 8 XCDs round-robin by dispatch order,
    // which would put the output-channel blocks of one pixel tile (consecutive ids, cb fastest)
    // on 8 different L2s, each fetching the same patch; remapped, XCD x runs ids x T/8 ..
    // (x + 1) T/8 - 1 in order, so a tile's channel blocks and its neighbours share one L2
    int cb = blockIdx.x, pt = blockIdx.y;
    if (kConvXcdRemap) {  // (the blur kernels' mapping: XCD x gets ceil / floor(nb / 8) ids)
        const unsigned nb = gridDim.x * gridDim.y, lin = blockIdx.x + gridDim.x * blockIdx.y;
        const unsigned q8 = nb / 8, r8 = nb % 8, xcd = lin % 8, loc = lin / 8;
        const unsigned l2 = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
        cb = static_cast<int>(l2 % gridDim.x), pt = static_cast<int>(l2 / gridDim.x);
    }
    int n0, h0, c0;
    if constexpr (TC == 32) {
        const int strips = w >> 5, rowblk = h / G::SR;
        c0 = (pt % strips) * 32;
        const int t = pt / strips;
        h0 = (t % rowblk) * G::SR;
        n0 = t / rowblk;
    } else {
        c0 = 0, h0 = 0, n0 = pt * G::S;
    }
    const int nci = cin >> 4, nsc = SC ? (cs1 + cs2) >> 4 : 0;
    const bq_u4* __restrict__ wsrc = reinterpret_cast<const bq_u4*>(wp + (int64_t)cb * nci * (9 * 64 * 16));

    // per-thread patch pieces: global element offset (channel 0 of the stage) or -1 (halo / past the batch)
    int64_t poff[G::NP];
#pragma unroll
    for (int k = 0; k < G::NP; ++k) {
        const int i = tid + k * kBlock;
        poff[k] = -1;
        if (i < 2 * G::PQP && cv_row(i) < G::PQ) {
            const int q = cv_row(i), half = cv_chunk(i);
            const int prow = q / G::PW, pcol = q - prow * G::PW;
            const int seg = prow / (G::SR + 2), pr = prow - seg * (G::SR + 2);
            const int nn = n0 + seg, hi = h0 + pr - 1, wi = c0 + pcol - 1;
            if (nn < n && (unsigned)hi < (unsigned)h && (unsigned)wi < (unsigned)w) {
                if constexpr (UP)
                    poff[k] = (((int64_t)nn * (h >> 1) + (hi >> 1)) * (w >> 1) + (wi >> 1)) * cin + half * 8;
                else if constexpr (BLK)  // [n][cin / 16][h][w][16]: stage ks is plane ks of the sample
                    poff[k] = ((int64_t)nn * (cin >> 4) * h * w + (int64_t)hi * w + wi) * 16 + half * 8;
                else
                    poff[k] = (((int64_t)nn * h + hi) * w + wi) * cin + half * 8;
            }
        }
    }
    bq_u4 sw[G::NW], spx[G::NP];
    const int64_t kstride = BLK ? (int64_t)h * w * 16 : 16;  // elements between stages' pieces
    // shortcut stage k1: the 64 x 16 weights (threads < 128, one piece each) and the tile's 512
    // pixels x 16 channels of cat(xs1, xs2) (4 pieces per thread; TC = 32 tiles lie inside the image)
    auto gload_sc = [&](int k1) {
        const int tid = cv_tid();
        if (tid < 128) sw[0] = reinterpret_cast<const bq_u4*>(wsp)[((int64_t)cb * nsc + k1) * 128 + tid];
        // piece k of thread tid: pixel (tid / 2) + 128 k = row (tid / 64) + 4 k, column (tid / 2) % 32
        const bool first = k1 * 16 < cs1;
        const int64_t cstr = first ? cs1 : cs2;
        const int q0 = tid >> 1;
        const u16* __restrict__ src = (first ? xs1 + k1 * 16 : xs2 + (k1 * 16 - cs1)) + (tid & 1) * 8 +
                                      (((int64_t)n0 * h + h0 + (q0 >> 5)) * w + c0 + (q0 & 31)) * cstr;
        const int64_t kstep = 4 * (int64_t)w * cstr;
#pragma unroll
        for (int k = 0; k < 4; ++k) spx[k] = *reinterpret_cast<const bq_u4*>(src + k * kstep);
    };
    auto gload = [&](int ks) {
        const bq_u4* __restrict__ ws = wsrc + (int64_t)ks * (9 * 64 * 2);
#pragma unroll
        for (int k = 0; k < G::NW; ++k) {
            const int i = tid + k * kBlock;
            if (i < G::WROWS * 2) sw[k] = ws[2 * cv_row(i) + cv_chunk(i)];
        }
#pragma unroll
        for (int k = 0; k < G::NP; ++k)
#if BQ_EXP == 10  // diagnostics (wrong results): every patch piece from one cached 32-byte line per stage
            spx[k] = poff[k] >= 0 ? *reinterpret_cast<const bq_u4*>(x + (tid & 1) * 8 + ks * 16) : bq_u4{0u, 0u, 0u, 0u};
#else
            spx[k] = poff[k] >= 0 ? *reinterpret_cast<const bq_u4*>(x + poff[k] + ks * kstride) : bq_u4{0u, 0u, 0u, 0u};
#endif
    };
    auto lstore = [&]() {
#pragma unroll
        for (int k = 0; k < G::NW; ++k) {
            const int i = tid + k * kBlock;
            if (i < G::WROWS * 2) *reinterpret_cast<bq_u4*>(lds + cv_row(i) * G::RB + cv_chunk(i) * 16) = sw[k];
        }
#pragma unroll
        for (int k = 0; k < G::NP; ++k) {
            const int i = tid + k * kBlock;
            if (i < 2 * G::PQP && cv_row(i) < G::PQ)
                *reinterpret_cast<bq_u4*>(lds + G::LW + cv_row(i) * G::RB + cv_chunk(i) * 16) = spx[k];
        }
    };

    // B-operand base of each of the wave's 4 pixel tiles (tap (0, 0)); tap (dy, dx) adds dy PW + dx
    int qb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int p = 128 * wv + 32 * j + r, vr = p / TC, col = p - vr * TC;
        const int seg = vr / G::SR, rr = vr - seg * G::SR;
        qb[j] = ((seg * (G::SR + 2) + rr) * G::PW + col) * G::RB + hh * 16;
    }
    bq_f16 acc[2][4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[a][j] = bq_f16{};

    const int kz = blockIdx.z, nz = gridDim.z, ntot = nci + nsc;
    const int ks0 = kz * ntot / nz, ks1 = (kz + 1) * ntot / nz;
    if constexpr (G::DB) {
        // Two stage buffers, one barrier per stage: stage s + 1 (in registers since stage s - 1)
        // is written to the other buffer and stage s + 2's global loads are issued before stage
        // s's MFMAs; the barrier after them both publishes stage s + 1 and frees stage s's buffer.
        // Swizzle: weight row wr keeps its 16-byte half c at (c ^ (wr >> 3 & 1)); patch pixel q
        // (column q % PW) at (c ^ (q % PW >> 3 & 1)) — the 16-lane groups of a ds_read_b128 then
        // read 16 distinct 16-byte slots of the 256-byte bank row for any column offset.
        auto lstore_sc = [&](int b) {  // the shortcut stage: weights as tap 0, pixels at the patch centre
            const int tid = cv_tid();
            char* __restrict__ base = lds + b * G::BUF;
            if (tid < 128) {
                const int wr = tid >> 1;
                *reinterpret_cast<bq_u4*>(base + wr * 32 + (((tid & 1) ^ ((wr >> 3) & 1)) << 4)) = sw[0];
            }
            const int q0 = tid >> 1, pcol = (q0 & 31) + 1;
            char* __restrict__ pp = base + G::LW + (((q0 >> 5) + 1) * G::PW + pcol) * 32 +
                                    (((tid & 1) ^ ((pcol >> 3) & 1)) << 4);
#pragma unroll
            for (int k = 0; k < 4; ++k) *reinterpret_cast<bq_u4*>(pp + k * 4 * G::PW * 32) = spx[k];
        };
        auto lstore_db = [&](int b) {
            char* __restrict__ base = lds + b * G::BUF;
#pragma unroll
            for (int k = 0; k < G::NW; ++k) {
                const int i = tid + k * kBlock;
                if (i < G::WROWS * 2) {
                    const int wr = cv_row(i);
                    *reinterpret_cast<bq_u4*>(base + wr * 32 + ((cv_chunk(i) ^ ((wr >> 3) & 1)) << 4)) = sw[k];
                }
            }
#pragma unroll
            for (int k = 0; k < G::NP; ++k) {
                const int i = tid + k * kBlock;
                if (i < 2 * G::PQP && cv_row(i) < G::PQ) {
                    const int q = cv_row(i), col = q % G::PW;
                    *reinterpret_cast<bq_u4*>(base + G::LW + q * 32 + ((cv_chunk(i) ^ ((col >> 3) & 1)) << 4)) = spx[k];
                }
            }
        };
        // per-lane fragment offsets: A row 64 t + 32 a + r (its swizzle bit is r's); B pixel
        // (4 wv + i) PW + r + dx, column r + dx
        const int wl_lane = r * 32 + ((hh ^ ((r >> 3) & 1)) << 4);
        int bl_lane[3];
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) bl_lane[dx] = G::LW + (4 * wv * G::PW + r + dx) * 32 + ((hh ^ (((r + dx) >> 3) & 1)) << 4);
        auto compute = [&](int b) {
            const char* __restrict__ base = lds + b * G::BUF;
            bq_u4 fa[9][2], fb[3][6];
            auto lda = [&](int s) {
                const int dx = s / 3, dy = s - 3 * dx, t = 3 * dy + dx;
                fa[s][0] = *reinterpret_cast<const bq_u4*>(base + wl_lane + (t * 64) * 32);
                fa[s][1] = *reinterpret_cast<const bq_u4*>(base + wl_lane + (t * 64 + 32) * 32);
                if (dy == 0) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) fb[dx][i] = *reinterpret_cast<const bq_u4*>(base + bl_lane[dx] + i * G::PW * 32);
                } else {
                    fb[dx][dy + 3] = *reinterpret_cast<const bq_u4*>(base + bl_lane[dx] + (dy + 3) * G::PW * 32);
                }
            };
            lda(0);
#pragma unroll
            for (int s = 0; s < 9; ++s) {
#if BQ_EXP == 8  // diagnostics (wrong results): tap 0's fragments for every tap, no further LDS reads
                if (s + 1 < 9) {
                    const int dx1 = (s + 1) / 3, dy1 = (s + 1) - 3 * dx1;
                    fa[s + 1][0] = fa[0][0], fa[s + 1][1] = fa[0][1];
                    if (dy1 == 0) {
                        for (int i = 0; i < 4; ++i) fb[dx1][i] = fb[0][i];
                    } else {
                        fb[dx1][dy1 + 3] = fb[0][dy1 - 1];
                    }
                }
#else
                if (s + 1 < 9) lda(s + 1);
#endif
                const int dx = s / 3, dy = s - 3 * dx;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[0][j] = bq_mfma(fa[s][0], fb[dx][j + dy], acc[0][j]);
                    acc[1][j] = bq_mfma(fa[s][1], fb[dx][j + dy], acc[1][j]);
                }
                // issue order pinned: tap s + 1's fragment reads, then tap s's 8 MFMAs (left to
                // itself the scheduler sinks each read to just before its first use, so every
                // tap waited for its LDS latency behind a single MFMA: MFMA busy 0.52)
                if (s + 1 < 9) {
                    const int dx1 = (s + 1) / 3, dy1 = (s + 1) - 3 * dx1;
                    if (dy1 == 0) __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
                    else __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        // the shortcut stage's centre-tap MFMAs (fragments as compute's tap (1, 1))
        auto compute_sc = [&](int b) {
            const int t = cv_tid(), ln = t & 63, rr = ln & 31, h2 = ln >> 5, wq = t >> 6;
            const char* __restrict__ base = lds + b * G::BUF;
            const int wl = rr * 32 + ((h2 ^ ((rr >> 3) & 1)) << 4);
            const int bl = G::LW + (4 * wq * G::PW + rr + 1) * 32 + ((h2 ^ (((rr + 1) >> 3) & 1)) << 4);
            const bq_u4 a0 = *reinterpret_cast<const bq_u4*>(base + wl);
            const bq_u4 a1 = *reinterpret_cast<const bq_u4*>(base + wl + 32 * 32);
            bq_u4 f[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) f[j] = *reinterpret_cast<const bq_u4*>(base + bl + (j + 1) * G::PW * 32);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[0][j] = bq_mfma(a0, f[j], acc[0][j]);
                acc[1][j] = bq_mfma(a1, f[j], acc[1][j]);
            }
        };
        // stages kb .. ke - 1 through the two buffers (gl: global loads of a stage into registers,
        // st: registers -> LDS buffer, cp: the buffer's MFMAs); the shortcut's stages (part z's
        // share of stages nci ..) in a loop of their own ahead of the 3x3 stages (one loop over
        // both kinds, or the shortcut's loop second, spilled ~200 VGPRs)
        auto pipeline = [&](int kb, int ke, auto&& gl, auto&& st, auto&& cp) {
            const int nst = ke - kb;
            if (nst <= 0) return;
            gl(kb);
            st(0);
            if (nst > 1) gl(kb + 1);
            __syncthreads();
            for (int s = 0; s < nst; ++s) {
                const int b = s & 1;
#if SP_CONV_PRIO == 1  // A/B knob: the stage hand-off and next loads issued at raised priority
                __builtin_amdgcn_s_setprio(2);
#endif
                if (s + 1 < nst) st(b ^ 1);
#if BQ_EXP == 9  // diagnostics (wrong results): no global loads after the prologue's two stages
                (void)b;
#else
                if (s + 2 < nst) gl(kb + s + 2);
#endif
                __builtin_amdgcn_sched_barrier(0);
#if SP_CONV_PRIO == 1
                __builtin_amdgcn_s_setprio(0);
#elif SP_CONV_PRIO == 2  // A/B knob: the MFMA phase at raised priority
                __builtin_amdgcn_s_setprio(2);
#endif
                cp(b);
#if SP_CONV_PRIO == 2
                __builtin_amdgcn_s_setprio(0);
#endif
                __syncthreads();
            }
        };
        if constexpr (SC)
            pipeline(ks0 > nci ? ks0 - nci : 0, ks1 - nci, gload_sc, lstore_sc, compute_sc);
        pipeline(ks0, ks1 < nci ? ks1 : nci, gload, lstore_db, compute);
    } else {
        gload(ks0);
        for (int ks = ks0; ks < ks1; ++ks) {
            __syncthreads();  // the previous stage's fragment reads are done
            lstore();
            __syncthreads();
            if (ks + 1 < ks1) gload(ks + 1);
            const char* __restrict__ wl = lds + r * G::RB + hh * 16;
            const char* __restrict__ pl = lds + G::LW;
            // fragments of tap t + 1 are read while tap t's 8 MFMAs run (two register sets)
            bq_u4 fa[2][2], fb[2][4];
            auto frags = [&](int t, int slot) {
                const int dy = t / 3, dx = t - 3 * (t / 3);
                fa[slot][0] = *reinterpret_cast<const bq_u4*>(wl + (t * 64) * G::RB);
                fa[slot][1] = *reinterpret_cast<const bq_u4*>(wl + (t * 64 + 32) * G::RB);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    fb[slot][j] = *reinterpret_cast<const bq_u4*>(pl + qb[j] + (dy * G::PW + dx) * G::RB);
            };
            frags(0, 0);
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                if (t + 1 < 9) frags(t + 1, (t + 1) & 1);
                const int sl = t & 1;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc[0][j] = bq_mfma(fa[sl][0], fb[sl][j], acc[0][j]);
                    acc[1][j] = bq_mfma(fa[sl][1], fb[sl][j], acc[1][j]);
                }
                // tap t + 1's 6 reads, then tap t's 8 MFMAs (as the TC = 32 loop; TC = 8 holds
                // 7 staged patch pieces per thread and would spill with both register sets live)
                if constexpr (TC != 8) {
                    if (t + 1 < 9) __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
                    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
    }

    // epilogue: lane (pixel r of tile j) holds channels 64 cb + 32 a + 8 g + 4 hh + e in register 4 g + e
    if constexpr (FS) {
        const float* __restrict__ cbp = gn.co;
        // the tile's first pixel (wave 0, j = 0, r = 0: lanes 0 / 32) as stored + cb: the shifts K
        float* kb = reinterpret_cast<float*>(lds) + 512;  // [64 local channels]
        if (wv == 0 && r == 0) {
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int cl = 32 * a + 8 * g + 4 * hh, co = cb * 64 + cl;
                    if (co >= cout) continue;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float t = acc[a][0][4 * g + e];
                        if (bias) t += bias[co + e];
                        if (res) t += bf1(res[(((int64_t)n0 * h + h0) * w + c0) * cout + co + e]);
                        kb[cl + e] = bf1(f2bf(t)) + (cbp ? cbp[(int64_t)n0 * cout + co + e] : 0.f);
                    }
                }
        }
        __syncthreads();
        float V[64];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int cl = 32 * a + 8 * g + 4 * hh, co = cb * 64 + cl;
                const bool live = co < cout;  // cout % 16 == 0
                float K[4], C[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int e = 0; e < 4; ++e) K[e] = live ? kb[cl + e] : 0.f;
                if (live && cbp) {
                    const float4 c4 = *reinterpret_cast<const float4*>(cbp + (int64_t)n0 * cout + co);
                    C[0] = c4.x, C[1] = c4.y, C[2] = c4.z, C[3] = c4.w;
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (!live) continue;
                    const int64_t obase = (((int64_t)n0 * h + h0 + 4 * wv + j) * w + c0 + r) * cout;
                    float v[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = acc[a][j][4 * g + e];
                    if (bias) {
                        const float4 bb = *reinterpret_cast<const float4*>(bias + co);
                        v[0] += bb.x, v[1] += bb.y, v[2] += bb.z, v[3] += bb.w;
                    }
                    if (res) {
                        const bq_u2 rv = *reinterpret_cast<const bq_u2*>(res + obase + co);
                        v[0] += bf_lo(rv.x), v[1] += bf_hi(rv.x), v[2] += bf_lo(rv.y), v[3] += bf_hi(rv.y);
                    }
                    const bq_u2 yv{pk2(v[0], v[1]), pk2(v[2], v[3])};
                    *reinterpret_cast<bq_u2*>(y + obase + co) = yv;
                    const float yf[4] = {bf_lo(yv.x), bf_hi(yv.x), bf_lo(yv.y), bf_hi(yv.y)};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {  // the terms of k_gnb_stats<0, _> with the tile's shift
                        const float d = yf[e] + C[e] - K[e];
                        s1[e] += d;
                        s2[e] = fmaf(d, d, s2[e]);
                    }
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) V[2 * ((a * 4 + g) * 4 + e)] = s1[e], V[2 * ((a * 4 + g) * 4 + e) + 1] = s2[e];
            }
#pragma unroll
        for (int m = 16, L = 64; m >= 1; m >>= 1, L >>= 1) {  // halving exchanges, as the GS epilogue
            const bool up = (r & m) != 0;
#pragma unroll
            for (int k = 0; k < L / 2; ++k) {
                const float keep = up ? V[L / 2 + k] : V[k], give = up ? V[k] : V[L / 2 + k];
                V[k] = keep + __shfl_xor(give, m, 64);
            }
        }
        float* red = reinterpret_cast<float*>(lds);  // [wave][stat][64 local channels] (kb lies past it)
        {
            const int i = r, a = i >> 4, g = (i >> 2) & 3, e = i & 3, cl = 32 * a + 8 * g + 4 * hh + e;
            red[(wv * 2 + 0) * 64 + cl] = V[0];
            red[(wv * 2 + 1) * 64 + cl] = V[1];
        }
        __syncthreads();
        if (tid < 192) {
            const int st = tid >> 6, cl = tid & 63, co = cb * 64 + cl;
            const float t = st == 2 ? kb[cl]
                                    : ((red[(0 * 2 + st) * 64 + cl] + red[(1 * 2 + st) * 64 + cl]) +
                                       red[(2 * 2 + st) * 64 + cl]) + red[(3 * 2 + st) * 64 + cl];
            const int tiles = (h / G::SR) * (w >> 5), tile = (h0 / G::SR) * (w >> 5) + (c0 >> 5);
            if (co < cout) gn.part[(((int64_t)n0 * tiles + tile) * 3 + st) * cout + co] = t;
        }
        return;
    }
    if constexpr (GS) {
        // dz stored, and per lane the sums over its 4 pixels (j) of each of its 32 channels: V[2 i + s],
        // i = (a 4 + g) 4 + e, s = 0: sum g, 1: sum g xhat
        const int64_t nc = (int64_t)n * cout;
        const int c2 = cout - gn.c1;
        // restrict-qualified: the x / coefficient loads may then be issued ahead of the dz stores
        // (unqualified, every load waited for the store before it)
        const u16* __restrict__ gx1 = gn.x1;
        const u16* __restrict__ gx2 = gn.x2;
        const float* __restrict__ gco = gn.co;
        const float* __restrict__ ggm = gn.gamma;
        float V[64];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int co = cb * 64 + 32 * a + 8 * g + 4 * hh;
                const bool live = co < cout;  // cout % 16 == 0: a lane's 4 channels are all in or all out
                const int cl = live ? co : 0;
                const float4 k0 = *reinterpret_cast<const float4*>(gco + (int64_t)n0 * cout + cl);
                const float4 k1 = *reinterpret_cast<const float4*>(gco + nc + (int64_t)n0 * cout + cl);
                const float4 k2 = *reinterpret_cast<const float4*>(gco + 2 * nc + (int64_t)n0 * cout + cl);
                const float4 k3 = *reinterpret_cast<const float4*>(gco + 3 * nc + (int64_t)n0 * cout + cl);
                const float4 gm4 = ggm ? *reinterpret_cast<const float4*>(ggm + cl) : make_float4(1.f, 1.f, 1.f, 1.f);
                const float K0[4] = {k0.x, k0.y, k0.z, k0.w}, K1[4] = {k1.x, k1.y, k1.z, k1.w};
                const float K2[4] = {k2.x, k2.y, k2.z, k2.w}, K3[4] = {k3.x, k3.y, k3.z, k3.w};
                const float GM[4] = {gm4.x, gm4.y, gm4.z, gm4.w};
                float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
                bq_u2 xq[4];  // the 4 pixels' x, loaded before any of their arithmetic
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int64_t pix = ((int64_t)n0 * h + h0 + 4 * wv + j) * w + c0 + r;
                    xq[j] = !live ? bq_u2{0u, 0u}
                          : co < gn.c1 ? *reinterpret_cast<const bq_u2*>(gx1 + pix * gn.c1 + co)
                                       : *reinterpret_cast<const bq_u2*>(gx2 + pix * c2 + (co - gn.c1));
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int64_t pix = ((int64_t)n0 * h + h0 + 4 * wv + j) * w + c0 + r;
                    float v[4];
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = acc[a][j][4 * g + e];
                    if (!live) continue;
                    if (bias) {
                        const float4 bb = *reinterpret_cast<const float4*>(bias + co);
                        v[0] += bb.x, v[1] += bb.y, v[2] += bb.z, v[3] += bb.w;
                    }
                    const bq_u2 dzv{pk2(v[0], v[1]), pk2(v[2], v[3])};
                    *reinterpret_cast<bq_u2*>(y + pix * cout + co) = dzv;
                    const bq_u2 xv = xq[j];
                    const float xf[4] = {bf_lo(xv.x), bf_hi(xv.x), bf_lo(xv.y), bf_hi(xv.y)};
                    const float df[4] = {bf_lo(dzv.x), bf_hi(dzv.x), bf_lo(dzv.y), bf_hi(dzv.y)};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {  // the terms of k_gnb_stats<1, ACT>
                        const float yv = fmaf(xf[e], K0[e], K1[e]);
                        float d = df[e];
                        if (gn.act) {
                            const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-yv));
                            d *= sg * (1.f + yv * (1.f - sg));
                        }
                        const float gg = d * GM[e];
                        s1[e] += gg;
                        s2[e] = fmaf(gg, fmaf(xf[e], K2[e], K3[e]), s2[e]);
                    }
                }
#pragma unroll
                for (int e = 0; e < 4; ++e) V[2 * ((a * 4 + g) * 4 + e)] = s1[e], V[2 * ((a * 4 + g) * 4 + e) + 1] = s2[e];
            }
        // sum over the 32 lanes of each half-wave (its 32 pixels of each tile row) by halving
        // exchanges: after the step with mask m a lane keeps the half of its values selected by
        // its lane bit m; lane r ends with V[2 r], V[2 r + 1] = value index r's two sums
#pragma unroll
        for (int m = 16, L = 64; m >= 1; m >>= 1, L >>= 1) {
            const bool up = (r & m) != 0;
#pragma unroll
            for (int k = 0; k < L / 2; ++k) {
                const float keep = up ? V[L / 2 + k] : V[k], give = up ? V[k] : V[L / 2 + k];
                V[k] = keep + __shfl_xor(give, m, 64);
            }
        }
        __syncthreads();  // the stage buffers are free: the wave totals meet in LDS
        float* red = reinterpret_cast<float*>(lds);  // [wave][stat][64 local channels]
        {
            const int i = r, a = i >> 4, g = (i >> 2) & 3, e = i & 3, cl = 32 * a + 8 * g + 4 * hh + e;
            red[(wv * 2 + 0) * 64 + cl] = V[0];
            red[(wv * 2 + 1) * 64 + cl] = V[1];
        }
        __syncthreads();
        if (tid < 128) {
            const int st = tid >> 6, cl = tid & 63, co = cb * 64 + cl;
            const float t = ((red[(0 * 2 + st) * 64 + cl] + red[(1 * 2 + st) * 64 + cl]) + red[(2 * 2 + st) * 64 + cl]) +
                            red[(3 * 2 + st) * 64 + cl];
            const int tiles = (h / G::SR) * (w >> 5), tile = (h0 / G::SR) * (w >> 5) + (c0 >> 5);
            if (co < cout) gn.part[(((int64_t)n0 * tiles + tile) * 2 + st) * cout + co] = t;
        }
        return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int p = 128 * wv + 32 * j + r, vr = p / TC, col = p - vr * TC;
        const int seg = vr / G::SR, rr = vr - seg * G::SR;
        const int nn = n0 + seg;
        if (nn >= n) continue;
        const int64_t obase = (((int64_t)nn * h + h0 + rr) * w + c0 + col) * cout;
        SP_DCHECK(h0 + rr < h && c0 + col < w);
        if (part) {  // split-K partial (cout % 4 == 0): fp32, no bias / residual
            float* pp = part + (int64_t)kz * ((int64_t)n * h * w * cout) + obase;
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int co = cb * 64 + 32 * a + 8 * g + 4 * hh;
                    if (co + 4 <= cout)
                        *reinterpret_cast<float4*>(pp + co) = make_float4(acc[a][j][4 * g], acc[a][j][4 * g + 1],
                                                                          acc[a][j][4 * g + 2], acc[a][j][4 * g + 3]);
                }
            continue;
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int co = cb * 64 + 32 * a + 8 * g + 4 * hh;
                float v[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = acc[a][j][4 * g + e];
                if (co + 4 <= cout && (cout & 3) == 0) {
                    if (bias) {
                        const float4 bb = *reinterpret_cast<const float4*>(bias + co);
                        v[0] += bb.x, v[1] += bb.y, v[2] += bb.z, v[3] += bb.w;
                    }
                    if (res) {
                        const bq_u2 rv = *reinterpret_cast<const bq_u2*>(res + obase + co);
                        v[0] += bf_lo(rv.x), v[1] += bf_hi(rv.x), v[2] += bf_lo(rv.y), v[3] += bf_hi(rv.y);
                    }
                    *reinterpret_cast<bq_u2*>(y + obase + co) = bq_u2{pk2(v[0], v[1]), pk2(v[2], v[3])};
                } else {
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (co + e < cout) {
                            float t = v[e] + (bias ? bias[co + e] : 0.f);
                            if (res) t += bf1(res[obase + co + e]);
                            y[obase + co + e] = f2bf(t);
                        }
                }
            }
    }
}

static unsigned stream_blocks(int64_t vectors);

static int conv_tc(int h, int w) {
    if (w % 32 == 0 && h % 16 == 0) return 32;
    if (h == w && (w == 16 || w == 8 || w == 4)) return w;
    return 0;
}

// y = sum over the split-K parts (fixed order) + bias (+ res), 4 channels per thread-iteration
__global__ __launch_bounds__(kBlock) void k_conv_reduce(const float* __restrict__ part, int parts, int64_t total,
                                                        int cout, const float* __restrict__ bias,
                                                        const u16* __restrict__ res, u16* __restrict__ y) {
    for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < total / 4; v += (int64_t)gridDim.x * kBlock) {
        const int64_t i = 4 * v;
        float4 a = *reinterpret_cast<const float4*>(part + i);
        for (int z = 1; z < parts; ++z) {
            const float4 b = *reinterpret_cast<const float4*>(part + (int64_t)z * total + i);
            a.x += b.x, a.y += b.y, a.z += b.z, a.w += b.w;
        }
        const int co = static_cast<int>(i % cout);
        if (bias) a.x += bias[co], a.y += bias[co + 1], a.z += bias[co + 2], a.w += bias[co + 3];
        if (res) {
            const bq_u2 rv = *reinterpret_cast<const bq_u2*>(res + i);
            a.x += bf_lo(rv.x), a.y += bf_hi(rv.x), a.z += bf_lo(rv.y), a.w += bf_hi(rv.y);
        }
        *reinterpret_cast<bq_u2*>(y + i) = bq_u2{pk2(a.x, a.y), pk2(a.z, a.w)};
    }
}

template <int TC>
static int64_t conv_tiles(int n, int h, int w) {
    using G = CvGeo<TC>;
    if constexpr (TC == 32)
        return (int64_t)n * (h / G::SR) * (w / 32);
    else
        return (n + G::S - 1) / G::S;
}

// split-K parts for a launch whose workgroups leave CUs idle (fewer than two per CU): doubling
// while each part keeps >= 8 input-channel stages and the grid stays under ~4 per CU
static int conv_parts(int n, int cin, int cout, int h, int w) {
    const int tc = conv_tc(h, w);
    if (!tc || cout % 4) return 1;
    const int64_t tiles = tc == 32 ? conv_tiles<32>(n, h, w) : tc == 16 ? conv_tiles<16>(n, h, w)
                        : tc == 8 ? conv_tiles<8>(n, h, w) : conv_tiles<4>(n, h, w);
    const int64_t wgs = tiles * ((cout + 63) / 64);
    int parts = 1;
    while (wgs * parts < 512 && (cin / 16) / (2 * parts) >= 8 && parts < 16) parts *= 2;
    return parts;
}

// the shortcut operands of an SC launch (wsp == nullptr: none)
struct ConvSc {
    const u16* xs1 = nullptr;
    const u16* xs2 = nullptr;
    int cs1 = 0, cs2 = 0;
    const u16* wsp = nullptr;
};

template <int TC, bool UP, bool BLK = false, bool SC = false, bool GS = false, bool FS = false>
static void conv_bf16_launch(const u16* x, const u16* wp, const float* bias, const u16* res, int n, int cin,
                             int cout, int h, int w, u16* y, hipStream_t s, float* part = nullptr, int parts = 1,
                             const ConvSc& sc = ConvSc{}, const ConvGn& gn = ConvGn{}) {
    using G = CvGeo<TC>;
    (void)sizeof(G);
    const int cbn = (cout + 63) / 64;
    const int64_t tiles = conv_tiles<TC>(n, h, w);
    // (+ the shortcut stages' 1x1 contraction)
    const double flops = 18.0 * n * (double)h * w * cin * cout + 2.0 * n * (double)h * w * (sc.cs1 + sc.cs2) * cout;
    launch_w(TK_CONV_BF16, flops, k_conv3x3_bf16<TC, UP, BLK, SC, GS, FS>, dim3(cbn, static_cast<unsigned>(tiles), parts),
             dim3(kBlock), s, x, wp, bias, res, n, cin, cout, h, w, y, parts > 1 ? part : nullptr, sc.xs1, sc.xs2,
             sc.cs1, sc.cs2, sc.wsp, gn);
    if (parts > 1) {
        const int64_t total = (int64_t)n * h * w * cout;
        launch(0, k_conv_reduce, dim3(stream_blocks(total / 8)), dim3(kBlock), s, static_cast<const float*>(part),
               parts, total, cout, bias, res, y);
    }
}

// Upsample2D's VJP after the full-resolution input VJP: dx[n][i][j][c] = sum of the 2 x 2 block
// dz[n][2i + a][2j + b][c] (fp32 sum, one rounding), 8 channels per thread-iteration
__global__ __launch_bounds__(kBlock) void k_pool2x2_bf16(const u16* __restrict__ dz, int64_t n, int c, int hs, int ws,
                                                         u16* __restrict__ dx) {
    const int cv = c / 8;
    const int64_t total = n * hs * ws * cv;
    for (int64_t v = (int64_t)blockIdx.x * kBlock + threadIdx.x; v < total; v += (int64_t)gridDim.x * kBlock) {
        const int j = static_cast<int>(v % cv);
        const int64_t pix = v / cv, nn = pix / ((int64_t)hs * ws), rem = pix - nn * hs * ws;
        const int i = static_cast<int>(rem / ws), jj = static_cast<int>(rem - (int64_t)i * ws);
        float acc[8] = {};
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                float f[8];
                unpack8(*reinterpret_cast<const bq_u4*>(
                            dz + (((nn * 2 * hs + 2 * i + a) * (2 * ws) + 2 * jj + b) * c + 8 * j)), f);
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[e] += f[e];
            }
        *reinterpret_cast<bq_u4*>(dx + pix * c + 8 * j) = pack8(acc);
    }
}

// ---------------------------------------------------------------------------------------------
// GroupNorm over NHWC bf16 (groups of consecutive channels), fp32 statistics.
//
// stats pass (grid: chunks x batch): thread (vector column j, pixel row) accumulates, for its 8
// channels, either the shifted sums  sum (x~ - s_c), sum (x~ - s_c)^2  (x~ = x + chan_bias,
// s_c = x~ at the sample's first pixel: no cancellation when |mean| >> std), or for the VJP
// sum g, sum g xhat (g = dy' gamma); the pixel rows of a column meet in LDS in a fixed order and
// one partial per (sample, chunk, channel) is written.  finalize (one wave per (sample, group),
// fp64, fixed order): forward -> mean, rstd and the per-(n, c) affine of the apply
// (y = x sc + sh); VJP -> the per-(n, c) coefficients of dx = A dy' + B x + D.
// ---------------------------------------------------------------------------------------------
constexpr int GNB_TARGET_BLOCKS = 2048;
#ifndef GNB_U
#define GNB_U 4  // pixels whose loads a thread keeps in flight in the streaming GroupNorm loops
#endif

struct GnbGeo {
    int cv, rows, chunks, chunk_px;
};

// non-temporal GroupNorm streams for tensors of at least SP_GNB_NT_MB MB (0 = always, negative =
// never: the default — at 256 MB the microbenchmark's large shapes gain 5-9 % but the PSLD bf16 step
// lost 2 %, profiles/round6/bf16/gn_nt_ab/)
#ifndef SP_GNB_NT_MB
#define SP_GNB_NT_MB -1
#endif
static bool gnb_nt(int64_t n, int c, int64_t hw) {
    return SP_GNB_NT_MB >= 0 && 2 * n * hw * (int64_t)c >= (int64_t)SP_GNB_NT_MB * (1 << 20);
}

static GnbGeo gnb_geo(int64_t n, int c, int64_t hw) {
    GnbGeo g;
    g.cv = c / 8;
    g.rows = g.cv >= kBlock ? 1 : kBlock / g.cv;
    int64_t want = std::max<int64_t>(1, (GNB_TARGET_BLOCKS + n - 1) / n);
    int64_t maxc = std::max<int64_t>(1, hw / (4 * g.rows));
    int64_t ch = std::min<int64_t>(want, maxc);
    ch = std::min<int64_t>(ch, 1024);
    g.chunk_px = static_cast<int>((hw + ch - 1) / ch);
    g.chunks = static_cast<int>((hw + g.chunk_px - 1) / g.chunk_px);
    return g;
}

// GroupNorm streams: NT = non-temporal cache policy on the loads and stores, chosen per call by the
// tensor's size (gnb_nt: an A/B knob, off by default; below the 256 MB last-level cache the second
// pass's re-read hits that cache and NT loses — measured, profiles/round6/bf16/gn_nt_ab/)
template <bool NT>
__device__ __forceinline__ bq_u4 gnb_load(const u16* p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const bq_u4*>(p));
    return *reinterpret_cast<const bq_u4*>(p);
}
#ifndef SP_GNB_NT_STORE
#define SP_GNB_NT_STORE 1  // the NT policy on the stores too (A/B knob)
#endif
template <bool NT>
__device__ __forceinline__ void gnb_store(u16* p, bq_u4 v) {
    if constexpr (NT && SP_GNB_NT_STORE) __builtin_nontemporal_store(v, reinterpret_cast<bq_u4*>(p));
    else *reinterpret_cast<bq_u4*>(p) = v;
}

// one 16-byte vector (8 channels, column j) of pixel p of sample nn, from the part that holds it
template <bool NT = false>
__device__ __forceinline__ bq_u4 gnb_ld(const u16* __restrict__ x1, const u16* __restrict__ x2, int c1, int c2,
                                        int64_t nn, int64_t hw, int64_t p, int j) {
    const int ch = 8 * j;
    if (ch < c1) return gnb_load<NT>(x1 + ((nn * hw + p) * c1 + ch));
    return gnb_load<NT>(x2 + ((nn * hw + p) * c2 + ch - c1));
}

// MODE 0: forward shifted sums; MODE 1: VJP sums (g, g xhat) given per-(n,c) coefs
// co = [sc | sh | xs | xo] (each n x c fp32) and gamma (c fp32)
template <int MODE, bool ACT, bool NT = false>
__global__ __launch_bounds__(kBlock) void k_gnb_stats(const u16* __restrict__ x1, const u16* __restrict__ x2, int c1,
                                                      int c2, const float* __restrict__ cbias,
                                                      const u16* __restrict__ dz, const float* __restrict__ co,
                                                      const float* __restrict__ gamma, int64_t hw, int chunk_px,
                                                      float* __restrict__ part) {
    __shared__ float red[kBlock * 16];
    const int c = c1 + c2, cv = c / 8, nn = blockIdx.y, chunk = blockIdx.x, tid = threadIdx.x;
    const int64_t nc = (int64_t)gridDim.y * c;
    const int64_t p0 = (int64_t)chunk * chunk_px, p1 = std::min<int64_t>(hw, p0 + chunk_px);
    for (int jb = 0; jb < cv; jb += kBlock) {  // column blocks (cv > 256 only: 2560 channels)
        const int colw = std::min(cv - jb, kBlock);
        const int rows_here = kBlock / colw;
        const int j = jb + tid % colw, row = tid / colw;
        const bool active = row < rows_here;
        float s1[8] = {}, s2[8] = {};
        if (active) {
            float sh[8] = {}, cbv[8] = {}, k0[8], k1[8], k2[8], k3[8], gm[8];
            if (cbias) {
                const float4 a = *reinterpret_cast<const float4*>(cbias + (int64_t)nn * c + 8 * j);
                const float4 b = *reinterpret_cast<const float4*>(cbias + (int64_t)nn * c + 8 * j + 4);
                cbv[0] = a.x, cbv[1] = a.y, cbv[2] = a.z, cbv[3] = a.w, cbv[4] = b.x, cbv[5] = b.y, cbv[6] = b.z,
                cbv[7] = b.w;
            }
            if constexpr (MODE == 0) {
                float f[8];
                unpack8(gnb_ld(x1, x2, c1, c2, nn, hw, 0, j), f);
#pragma unroll
                for (int e = 0; e < 8; ++e) sh[e] = f[e] + cbv[e];
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int64_t ix = (int64_t)nn * c + 8 * j + e;
                    k0[e] = co[ix], k1[e] = co[nc + ix], k2[e] = co[2 * nc + ix], k3[e] = co[3 * nc + ix];
                    gm[e] = gamma[8 * j + e];
                }
            }
            // one pixel's contribution, from its loaded vectors (x; dz for the VJP)
            auto acc1 = [&](bq_u4 xv, bq_u4 dzv) {
                float f[8];
                unpack8(xv, f);
                if constexpr (MODE == 0) {
                    (void)dzv;
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float d = f[e] + cbv[e] - sh[e];
                        s1[e] += d;
                        s2[e] = fmaf(d, d, s2[e]);
                    }
                } else {
                    float dv[8];
                    unpack8(dzv, dv);
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float yv = fmaf(f[e], k0[e], k1[e]);
                        float d = dv[e];
                        if constexpr (ACT) {
                            const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-yv));
                            d *= sg * (1.f + yv * (1.f - sg));
                        }
                        const float g = d * gm[e];
                        const float xh = fmaf(f[e], k2[e], k3[e]);
                        s1[e] += g;
                        s2[e] = fmaf(g, xh, s2[e]);
                    }
                }
            };
            auto ldz = [&](int64_t p) {
                if constexpr (MODE == 1) return gnb_load<NT>(dz + ((int64_t)nn * hw + p) * c + 8 * j);
                else return bq_u4{0u, 0u, 0u, 0u};
            };
            // GNB_U pixels' loads in flight per thread, then their sums in pixel order (the same
            // order as one pixel at a time: bit-identical partials)
            int64_t p = p0 + row;
            for (; p + (GNB_U - 1) * rows_here < p1; p += GNB_U * rows_here) {
                bq_u4 xv[GNB_U], dzv[GNB_U];
#pragma unroll
                for (int u = 0; u < GNB_U; ++u) {
                    xv[u] = gnb_ld<NT>(x1, x2, c1, c2, nn, hw, p + u * rows_here, j);
                    dzv[u] = ldz(p + u * rows_here);
                }
#pragma unroll
                for (int u = 0; u < GNB_U; ++u) acc1(xv[u], dzv[u]);
            }
            for (; p < p1; p += rows_here) acc1(gnb_ld(x1, x2, c1, c2, nn, hw, p, j), ldz(p));
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < 8; ++e) red[tid * 16 + e] = s1[e], red[tid * 16 + 8 + e] = s2[e];
        __syncthreads();
        // column reduce: thread t < colw sums rows 0 .. rows_here-1 of column t in order
        if (tid < colw) {
            float a1[8] = {}, a2[8] = {};
            for (int rr = 0; rr < rows_here; ++rr) {
                const float* src = red + (rr * colw + tid) * 16;
#pragma unroll
                for (int e = 0; e < 8; ++e) a1[e] += src[e], a2[e] += src[8 + e];
            }
            // partials [n][chunk][2][c]
            float* dst = part + (((int64_t)nn * gridDim.x + chunk) * 2) * c + 8 * (jb + tid);
#pragma unroll
            for (int e = 0; e < 8; ++e) dst[e] = a1[e], dst[c + e] = a2[e];
        }
    }
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// forward finalize: one wave per (n, group).  stats = [mean | rstd] (n*groups each);
// co = [sc | sh] (n*c each): y = x sc + sh.  The group's (chunk, channel) partials are spread
// over the wave's lanes (pair i = lane, lane + 64, ...: channel i % cpg of chunk i / cpg, so a
// row of partials is read by consecutive lanes), each lane sums its pairs in a fixed order in
// fp64, and the wave meets in a fixed butterfly — a handful of loads per lane instead of a
// chain of `chunks` dependent loads on cpg lanes (4 of 64 at 128 channels / 32 groups).
__device__ __forceinline__ float gnb_shift(const u16* __restrict__ x1, const u16* __restrict__ x2, int c1, int c2,
                                           const float* __restrict__ cbias, int64_t nn, int64_t hw, int c, int ch) {
    const float cbv = cbias ? cbias[nn * c + ch] : 0.f;
    return (ch < c1 ? bf1(x1[nn * hw * c1 + ch]) : bf1(x2[nn * hw * c2 + ch - c1])) + cbv;
}

__global__ __launch_bounds__(64) void k_gnb_final_fwd(const u16* __restrict__ x1, const u16* __restrict__ x2, int c1,
                                                      int c2, const float* __restrict__ cbias,
                                                      const float* __restrict__ part, int chunks, int64_t hw,
                                                      int groups, float eps, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, float* __restrict__ stats,
                                                      float* __restrict__ co) {
    const int c = c1 + c2, cpg = c / groups, g = blockIdx.x, nn = blockIdx.y, lane = threadIdx.x;
    const int64_t ng = (int64_t)gridDim.y * groups;
    const int pairs = cpg * chunks;
    const float* __restrict__ pb = part + (int64_t)nn * chunks * 2 * c + g * cpg;  // chunk 0, first channel
    // pass 1: group sum of x~ = sum of the shifted partials + hw * shift per channel
    double sa = 0.0;
    for (int i = lane; i < pairs; i += 64) {
        const int k = i / cpg, cc = i - k * cpg;
        sa += pb[(int64_t)k * 2 * c + cc];
    }
    for (int cc = lane; cc < cpg; cc += 64)
        sa += (double)hw * gnb_shift(x1, x2, c1, c2, cbias, nn, hw, c, g * cpg + cc);
    const double cnt = (double)hw * cpg;
    const double mean = wave_sum_d(sa) / cnt;
    // pass 2: sum (x~ - mean)^2 = sum_c [S2_c + 2 dm_c S1_c + hw dm_c^2], dm_c = shift_c - mean
    double sx = 0.0;
    for (int i = lane; i < pairs; i += 64) {
        const int k = i / cpg, cc = i - k * cpg;
        const float* pp = pb + (int64_t)k * 2 * c + cc;
        const double dm = (double)gnb_shift(x1, x2, c1, c2, cbias, nn, hw, c, g * cpg + cc) - mean;
        sx += pp[c] + 2.0 * dm * pp[0];
    }
    for (int cc = lane; cc < cpg; cc += 64) {
        const double dm = (double)gnb_shift(x1, x2, c1, c2, cbias, nn, hw, c, g * cpg + cc) - mean;
        sx += (double)hw * dm * dm;
    }
    const double var = std::max(0.0, wave_sum_d(sx) / cnt);
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float meanf = (float)mean;
    if (lane == 0) stats[(int64_t)nn * groups + g] = meanf, stats[ng + (int64_t)nn * groups + g] = rstd;
    const int64_t nc = (int64_t)gridDim.y * c;
    for (int cc = lane; cc < cpg; cc += 64) {
        const int ch = g * cpg + cc;
        const float cbv = cbias ? cbias[(int64_t)nn * c + ch] : 0.f;
        const float sc = rstd * (gamma ? gamma[ch] : 1.f);
        co[(int64_t)nn * c + ch] = sc;
        co[nc + (int64_t)nn * c + ch] = (beta ? beta[ch] : 0.f) + (cbv - meanf) * sc;
    }
}

// forward finalize from per-tile shifted moments (the FS conv epilogue): part [n][tile][3][c] =
// sum(d), sum(d^2), K (d = x~ - K over the tile's P pixels); per group in fp64: the mean from
// sum(d) + P K, then sum (x~ - mean)^2 = sum over (tile, channel) of S2 + 2 (K - mean) S1 + P (K - mean)^2.
// Outputs as k_gnb_final_fwd.
__global__ __launch_bounds__(64) void k_gnb_final_fwd_tiles(const float* __restrict__ part, int tiles, int64_t px,
                                                            int64_t hw, int c, int groups, float eps,
                                                            const float* __restrict__ cbias,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float* __restrict__ stats,
                                                            float* __restrict__ co) {
    const int cpg = c / groups, g = blockIdx.x, nn = blockIdx.y, lane = threadIdx.x;
    const int64_t ng = (int64_t)gridDim.y * groups;
    const int pairs = cpg * tiles;
    const float* __restrict__ pb = part + (int64_t)nn * tiles * 3 * c + g * cpg;
    double sa = 0.0;
    for (int i = lane; i < pairs; i += 64) {
        const int k = i / cpg, cc = i - k * cpg;
        const float* pp = pb + (int64_t)k * 3 * c + cc;
        sa += (double)pp[0] + (double)px * pp[2 * c];
    }
    const double cnt = (double)hw * cpg;
    const double mean = wave_sum_d(sa) / cnt;
    double sx = 0.0;
    for (int i = lane; i < pairs; i += 64) {
        const int k = i / cpg, cc = i - k * cpg;
        const float* pp = pb + (int64_t)k * 3 * c + cc;
        const double dm = (double)pp[2 * c] - mean;
        sx += (double)pp[c] + 2.0 * dm * pp[0] + (double)px * dm * dm;
    }
    const double var = std::max(0.0, wave_sum_d(sx) / cnt);
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float meanf = (float)mean;
    if (lane == 0) stats[(int64_t)nn * groups + g] = meanf, stats[ng + (int64_t)nn * groups + g] = rstd;
    const int64_t nc = (int64_t)gridDim.y * c;
    for (int cc = lane; cc < cpg; cc += 64) {
        const int ch = g * cpg + cc;
        const float cbv = cbias ? cbias[(int64_t)nn * c + ch] : 0.f;
        const float sc = rstd * (gamma ? gamma[ch] : 1.f);
        co[(int64_t)nn * c + ch] = sc;
        co[nc + (int64_t)nn * c + ch] = (beta ? beta[ch] : 0.f) + (cbv - meanf) * sc;
    }
}

// per-(n, c) coefficients for the VJP from the forward's stats: co = [sc | sh | xs | xo]
// (y = x sc + sh, xhat = x xs + xo)
__global__ void k_gnb_coefs(const float* __restrict__ stats, const float* __restrict__ cbias,
                            const float* __restrict__ gamma, const float* __restrict__ beta, int n, int c,
                            int groups, float* __restrict__ co) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nc = (int64_t)n * c;
    if (i >= nc) return;
    const int nn = static_cast<int>(i / c), ch = static_cast<int>(i - (int64_t)nn * c), g = ch / (c / groups);
    const float mean = stats[(int64_t)nn * groups + g], rstd = stats[(int64_t)n * groups + (int64_t)nn * groups + g];
    const float cbv = cbias ? cbias[i] : 0.f;
    const float sc = rstd * (gamma ? gamma[ch] : 1.f);
    co[i] = sc;
    co[nc + i] = (beta ? beta[ch] : 0.f) + (cbv - mean) * sc;
    co[2 * nc + i] = rstd;
    co[3 * nc + i] = (cbv - mean) * rstd;
}

// VJP finalize: one wave per (n, group): m1 = mean(g), m2 = mean(g xhat) over the group ->
// dx = A dy' + B x + D with A = rstd gamma_c, B = -rstd^2 m2, D = -rstd (m1 + m2 xo_c);
// co2 = [A | B | D]
__global__ __launch_bounds__(64) void k_gnb_final_bwd(const float* __restrict__ part, int chunks, int64_t hw, int c,
                                                      int groups, const float* __restrict__ stats,
                                                      const float* __restrict__ gamma, const float* __restrict__ co,
                                                      float* __restrict__ co2) {
    const int cpg = c / groups, g = blockIdx.x, nn = blockIdx.y, lane = threadIdx.x, n = gridDim.y;
    const int pairs = cpg * chunks;
    const float* __restrict__ pb = part + (int64_t)nn * chunks * 2 * c + g * cpg;
    double s1 = 0.0, s2 = 0.0;  // (chunk, channel) pairs spread over the lanes as k_gnb_final_fwd
    for (int i = lane; i < pairs; i += 64) {
        const int k = i / cpg, cc = i - k * cpg;
        const float* pp = pb + (int64_t)k * 2 * c + cc;
        s1 += pp[0];
        s2 += pp[c];
    }
    const double cnt = (double)hw * cpg;
    const float m1 = (float)(wave_sum_d(s1) / cnt), m2 = (float)(wave_sum_d(s2) / cnt);
    const float rstd = stats[(int64_t)n * groups + (int64_t)nn * groups + g];
    const int64_t nc = (int64_t)n * c;
    for (int cc = lane; cc < cpg; cc += 64) {
        const int ch = g * cpg + cc;
        const int64_t i = (int64_t)nn * c + ch;
        co2[i] = rstd * (gamma ? gamma[ch] : 1.f);
        co2[nc + i] = -rstd * rstd * m2;
        co2[2 * nc + i] = -rstd * (m1 + m2 * co[3 * nc + i]);
    }
}

// forward apply: z = act(x sc + sh) over the concatenated channels.  Grid (chunks, batch) as the
// stats pass: a thread owns one 8-channel column of the sample, keeps its (n, c) coefficients in
// registers and walks the chunk's pixels (the block reads rows of C channels contiguously).
template <bool ACT, bool NT = false>
__global__ __launch_bounds__(kBlock) void k_gnb_apply(const u16* __restrict__ x1, const u16* __restrict__ x2, int c1,
                                                      int c2, const float* __restrict__ co, int64_t hw, int chunk_px,
                                                      u16* __restrict__ z, int blk) {
    const int c = c1 + c2, cv = c / 8, nn = blockIdx.y, tid = threadIdx.x;
    const int64_t nc = (int64_t)gridDim.y * c;
    const int64_t p0 = (int64_t)blockIdx.x * chunk_px, p1 = std::min<int64_t>(hw, p0 + chunk_px);
    for (int jb = 0; jb < cv; jb += kBlock) {
        const int colw = std::min(cv - jb, kBlock), rows = kBlock / colw;
        const int j = jb + tid % colw, row = tid / colw;
        if (row >= rows) continue;
        const float* sc = co + (int64_t)nn * c + 8 * j;
        const float* sh = co + nc + (int64_t)nn * c + 8 * j;
        const float4 a0 = *reinterpret_cast<const float4*>(sc), a1 = *reinterpret_cast<const float4*>(sc + 4);
        const float4 b0 = *reinterpret_cast<const float4*>(sh), b1 = *reinterpret_cast<const float4*>(sh + 4);
        const float sa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const float sb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        auto one = [&](bq_u4 xv, int64_t p) {
            float f[8];
            unpack8(xv, f);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float yv = fmaf(f[e], sa[e], sb[e]);
                f[e] = ACT ? silu_f(yv) : yv;
            }
            // blk: z in the channel-blocked layout [n][c / 16][hw][16] the conv tile reads best
            const int64_t zo = blk ? (((int64_t)nn * (c >> 4) + (j >> 1)) * hw + p) * 16 + 8 * (j & 1)
                                   : ((int64_t)nn * hw + p) * c + 8 * j;
            gnb_store<NT>(z + zo, pack8(f));
        };
        int64_t p = p0 + row;
        for (; p + (GNB_U - 1) * rows < p1; p += GNB_U * rows) {  // GNB_U pixels' loads in flight
            bq_u4 xv[GNB_U];
#pragma unroll
            for (int u = 0; u < GNB_U; ++u) xv[u] = gnb_ld<NT>(x1, x2, c1, c2, nn, hw, p + u * rows, j);
#pragma unroll
            for (int u = 0; u < GNB_U; ++u) one(xv[u], p + u * rows);
        }
        for (; p < p1; p += rows) one(gnb_ld(x1, x2, c1, c2, nn, hw, p, j), p);
    }
}

__device__ __forceinline__ void ld8f(const float* p, float (&f)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    f[0] = a.x, f[1] = a.y, f[2] = a.z, f[3] = a.w, f[4] = b.x, f[5] = b.y, f[6] = b.z, f[7] = b.w;
}

// VJP apply: dx = A dy' + B x + D (+ add1 / add2 / add1b), written to the parts' layouts; grid
// and column ownership as k_gnb_apply (the five (n, c) coefficient rows held in registers)
template <bool ACT, bool NT = false>
__global__ __launch_bounds__(kBlock) void k_gnb_bwd_apply(const u16* __restrict__ dz, const u16* __restrict__ x1,
                                                          const u16* __restrict__ x2, int c1, int c2,
                                                          const float* __restrict__ co, const float* __restrict__ co2,
                                                          int64_t hw, int chunk_px, u16* __restrict__ dx1,
                                                          u16* __restrict__ dx2, const u16* __restrict__ add1,
                                                          const u16* __restrict__ add2,
                                                          const u16* __restrict__ add1b, int blk) {
    const int c = c1 + c2, cv = c / 8, nn = blockIdx.y, tid = threadIdx.x;
    const int64_t nc = (int64_t)gridDim.y * c;
    const int64_t p0 = (int64_t)blockIdx.x * chunk_px, p1 = std::min<int64_t>(hw, p0 + chunk_px);
    for (int jb = 0; jb < cv; jb += kBlock) {
        const int colw = std::min(cv - jb, kBlock), rows = kBlock / colw;
        const int j = jb + tid % colw, row = tid / colw;
        if (row >= rows) continue;
        const int64_t ci = (int64_t)nn * c + 8 * j;
        float ka[8], kb[8], kd[8], ksc[8], ksh[8];
        ld8f(co2 + ci, ka);
        ld8f(co2 + nc + ci, kb);
        ld8f(co2 + 2 * nc + ci, kd);
        if constexpr (ACT) {
            ld8f(co + ci, ksc);
            ld8f(co + nc + ci, ksh);
        }
        const int ch = 8 * j;
        const bool first = ch < c1;
        const int cp = first ? c1 : c2, chp = first ? ch : ch - c1;
        u16* __restrict__ dst = first ? dx1 : dx2;
        // blk & 2: add1 is one addend over the concatenated channels ([n][hw][c1 + c2], e.g. the
        // 1x1 shortcut's input gradient from one GEMM), add2 unused
        const bool acat = (blk & 2) != 0;
        const u16* __restrict__ a = acat ? add1 : first ? add1 : add2;
        const u16* __restrict__ ab = first ? add1b : nullptr;
        const u16* __restrict__ xs = first ? x1 : x2;
        // one pixel from its loaded vectors (x, dy', and the addends or zeros)
        auto one = [&](bq_u4 xv, bq_u4 dv, bq_u4 av, bq_u4 bv, int64_t off, int64_t p) {
            float f[8], d[8], o[8];
            unpack8(xv, f);
            unpack8(dv, d);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float dd = d[e];
                if constexpr (ACT) {
                    const float yv = fmaf(f[e], ksc[e], ksh[e]);
                    const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-yv));
                    dd *= sg * (1.f + yv * (1.f - sg));
                }
                o[e] = fmaf(ka[e], dd, fmaf(kb[e], f[e], kd[e]));
            }
            if (a) {
                float t[8];
                unpack8(av, t);
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] += t[e];
            }
            if (ab) {
                float t[8];
                unpack8(bv, t);
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] += t[e];
            }
            // blk & 1 (one part): dx in the channel-blocked layout [n][c / 16][hw][16]
            const int64_t oo = (blk & 1) ? (((int64_t)nn * (cp >> 4) + (chp >> 4)) * hw + p) * 16 + (chp & 15) : off;
            gnb_store<NT>(dst + oo, pack8(o));
        };
        const bq_u4 zero4 = {0u, 0u, 0u, 0u};
        auto ld = [&](const u16* __restrict__ src, int64_t off) {
            return src ? gnb_load<NT>(src + off) : zero4;
        };
        int64_t p = p0 + row;
        for (; p + (GNB_U - 1) * rows < p1; p += GNB_U * rows) {  // GNB_U pixels' loads in flight
            bq_u4 xv[GNB_U], dv[GNB_U], av[GNB_U], bv[GNB_U];
#pragma unroll
            for (int u = 0; u < GNB_U; ++u) {
                const int64_t pp = p + u * rows, off = ((int64_t)nn * hw + pp) * cp + chp;
                xv[u] = gnb_load<NT>(xs + off);
                dv[u] = gnb_load<NT>(dz + ((int64_t)nn * hw + pp) * c + ch);
                av[u] = ld(a, acat ? ((int64_t)nn * hw + pp) * c + ch : off);
                bv[u] = ld(ab, off);
            }
#pragma unroll
            for (int u = 0; u < GNB_U; ++u)
                one(xv[u], dv[u], av[u], bv[u], ((int64_t)nn * hw + p + u * rows) * cp + chp, p + u * rows);
        }
        for (; p < p1; p += rows) {
            const int64_t off = ((int64_t)nn * hw + p) * cp + chp;
            one(*reinterpret_cast<const bq_u4*>(xs + off), *reinterpret_cast<const bq_u4*>(dz + ((int64_t)nn * hw + p) * c + ch),
                ld(a, acat ? ((int64_t)nn * hw + p) * c + ch : off), ld(ab, off), off, p);
        }
    }
}

static unsigned stream_blocks(int64_t vectors) {
    return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((vectors + kBlock - 1) / kBlock, 256 * 16)));
}

// ---------------------------------------------------------------------------------------------
// GEGLU of the SD 1.5 transformers' feed-forward at bf16: h = [a | gate] ([T][2F], the
// projection's output), y = a * gelu(gate) ([T][F]; exact erf GELU, fp32 arithmetic, one
// rounding); VJP dh = [dy * gelu(gate) | dy * a * gelu'(gate)] written as one [T][2F] buffer (the
// projection's cotangent: no chunk-gradient concatenation).  8 features per thread-iteration.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float bq_gelu(float g) { return 0.5f * g * (1.f + erff(g * 0.70710678118654752f)); }
__device__ __forceinline__ float bq_gelu_grad(float g) {
    const float cdf = 0.5f * (1.f + erff(g * 0.70710678118654752f));
    return cdf + g * (expf(-0.5f * g * g) * 0.39894228040143268f);
}

__global__ __launch_bounds__(kBlock) void k_geglu_bf16_fwd(const u16* __restrict__ h, int64_t rows, int f,
                                                           u16* __restrict__ y) {
    const int f8 = f >> 3;
    const int64_t n8 = rows * f8;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kBlock) {
        const int64_t r = i / f8;
        const int j = static_cast<int>(i - r * f8);
        const bq_u4* hr = reinterpret_cast<const bq_u4*>(h + r * 2 * f);
        float a[8], g[8];
        unpack8(hr[j], a);
        unpack8(hr[f8 + j], g);
#pragma unroll
        for (int e = 0; e < 8; ++e) a[e] *= bq_gelu(g[e]);
        reinterpret_cast<bq_u4*>(y)[i] = pack8(a);
    }
}

__global__ __launch_bounds__(kBlock) void k_geglu_bf16_bwd(const u16* __restrict__ h, const u16* __restrict__ dy,
                                                           int64_t rows, int f, u16* __restrict__ dh) {
    const int f8 = f >> 3;
    const int64_t n8 = rows * f8;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n8; i += (int64_t)gridDim.x * kBlock) {
        const int64_t r = i / f8;
        const int j = static_cast<int>(i - r * f8);
        const bq_u4* hr = reinterpret_cast<const bq_u4*>(h + r * 2 * f);
        float a[8], g[8], d[8], da[8], dg[8];
        unpack8(hr[j], a);
        unpack8(hr[f8 + j], g);
        unpack8(reinterpret_cast<const bq_u4*>(dy)[i], d);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            da[e] = d[e] * bq_gelu(g[e]);
            dg[e] = d[e] * a[e] * bq_gelu_grad(g[e]);
        }
        bq_u4* o = reinterpret_cast<bq_u4*>(dh + r * 2 * f);
        o[j] = pack8(da);
        o[f8 + j] = pack8(dg);
    }
}

// ---------------------------------------------------------------------------------------------
// LayerNorm of the SD 1.5 transformer blocks at bf16 (token rows [T][C], C = 320 / 640 / 1280):
// one wave per row held in registers (lane l: 8-channel vectors l, l + 64, ...), fp32 statistics
// (two wave reductions), fp32 weight / bias; the VJP (frozen weights) adds the residual branch's
// gradient of the same tensor (`add`, the linear that consumed the residual hands it over), so
// x + f(norm(x)) costs no autograd add.
// ---------------------------------------------------------------------------------------------
constexpr int LNB_ROWS = kBlock / 64;

template <int NV>
__device__ __forceinline__ void lnb_load(const u16* __restrict__ row, int c8, int lane, float (&v)[NV][8]) {
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = lane + 64 * j;
        const bq_u4 q = i < c8 ? reinterpret_cast<const bq_u4*>(row)[i] : bq_u4{0u, 0u, 0u, 0u};
        unpack8(q, v[j]);
    }
}

template <int NV>
__global__ __launch_bounds__(kBlock) void k_layernorm_bf16_fwd(const u16* __restrict__ x, const float* __restrict__ w,
                                                               const float* __restrict__ b, int64_t rows, int c,
                                                               float eps, u16* __restrict__ y,
                                                               float* __restrict__ mean, float* __restrict__ rstd) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * LNB_ROWS + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int c8 = c >> 3;
    float v[NV][8];
    lnb_load<NV>(x + r * c, c8, lane, v);
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) s += v[j][e];
    const float mu = wave_sum(s) / static_cast<float>(c);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j)
        if (lane + 64 * j < c8)
#pragma unroll
            for (int e = 0; e < 8; ++e) q = fmaf(v[j][e] - mu, v[j][e] - mu, q);
    const float rs = 1.f / sqrtf(wave_sum(q) / static_cast<float>(c) + eps);
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = lane + 64 * j;
        if (i < c8) {
            float o[8], g[8], bb[8];
            ld8f(w + 8 * i, g);
            ld8f(b + 8 * i, bb);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = fmaf((v[j][e] - mu) * rs, g[e], bb[e]);
            reinterpret_cast<bq_u4*>(y + r * c)[i] = pack8(o);
        }
    }
    if (lane == 0) mean[r] = mu, rstd[r] = rs;
}

template <int NV>
__global__ __launch_bounds__(kBlock) void k_layernorm_bf16_bwd(const u16* __restrict__ dy, const u16* __restrict__ x,
                                                               const float* __restrict__ w,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd,
                                                               const u16* __restrict__ add, int64_t rows, int c,
                                                               u16* __restrict__ dx) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * LNB_ROWS + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int c8 = c >> 3;
    const float mu = mean[r], rs = rstd[r];
    float g[NV][8], h[NV][8];
    lnb_load<NV>(dy + r * c, c8, lane, g);
    lnb_load<NV>(x + r * c, c8, lane, h);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = lane + 64 * j;
        if (i < c8) {
            float ww[8];
            ld8f(w + 8 * i, ww);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                g[j][e] *= ww[e];
                h[j][e] = (h[j][e] - mu) * rs;
                s1 = fmaf(g[j][e], h[j][e], s1);
                s2 += g[j][e];
            }
        }
    }
    const float inv_c = 1.f / static_cast<float>(c);
    const float m1 = wave_sum(s1) * inv_c, m2 = wave_sum(s2) * inv_c;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const int i = lane + 64 * j;
        if (i < c8) {
            float o[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = rs * (g[j][e] - m2 - h[j][e] * m1);
            if (add) {
                float a[8];
                unpack8(reinterpret_cast<const bq_u4*>(add + r * c)[i], a);
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] += a[e];
            }
            reinterpret_cast<bq_u4*>(dx + r * c)[i] = pack8(o);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Multi-head attention on bf16 q / k / v (the SD 1.5 UNet's attn1 / attn2 at the reference's
// bf16): the structure of k_attn6_fwd (sp_attention6.hip) with one bf16 term per operand.
// Per wave 32 queries; per 32-key block S^T = K Q^T (K rows from LDS as A, Q^T in registers as
// B, d padded to 16), the softmax on the lane-local query column (scores scaled by
// scale log2 e in fp32), O^T += V^T P^T with P^T packed to bf16 straight from the S^T
// accumulators (key order inside the MFMA's K = the C layout's, V^T staged in that order).
// Keys past m are masked (-inf); queries past n are computed on zero rows and not stored.
// ---------------------------------------------------------------------------------------------
constexpr float AB_LOG2E = 1.4426950408889634f;
constexpr float AB_LN2 = 0.6931471805599453f;
constexpr int AB_QW = 32, AB_WB = 4 * AB_QW;
constexpr float AB_LAZY = 8.f;


template <int D>
struct AbGeo {
    static_assert(D % 8 == 0 && D <= 160, "head dim");
    static constexpr int DK = (D + 15) / 16;
    static constexpr int DKP = DK * 16;
    static constexpr int DT = (D + 31) / 32;
    static constexpr int SB = 64;
    static constexpr int KROW = DKP + 8;   // bf16 per K row in LDS
    static constexpr int IMG = SB * KROW + 32 * DT;  // a natural image + the columns a last-row tr read reaches
    static constexpr int NVU = (SB / 2 * (D / 8) + kBlock - 1) / kBlock;      // V (2 keys x 8 d) units
};

// a stage of SB rows (row pairs 2p, 2p + 1 x 8 d per unit) into registers.  Rows >= limit read
// row limit - 1 instead (unconditional loads: a select on a loaded value, or a zero written into
// a load's destination, makes the compiler wait for the whole stage's loads at once); the
// kernels give such rows no weight (keys past m: P = 0; queries past n: lse = +inf, delta = 0)
template <int D>
__device__ __forceinline__ void ab_ld_pairs(const u16* __restrict__ src, int64_t rs, int base, int limit,
                                            bq_u4 (&st)[AbGeo<D>::NVU][2]) {
    using G = AbGeo<D>;
#pragma unroll
    for (int j = 0; j < G::NVU; ++j) {
        const int u = threadIdx.x + j * kBlock;
        if (u < G::SB / 2 * (D / 8)) {
            const int p = u / (D / 8), d0 = 8 * (u - p * (D / 8));
            const int r0 = min(base + 2 * p, limit - 1), r1 = min(base + 2 * p + 1, limit - 1);
            st[j][0] = *reinterpret_cast<const bq_u4*>(src + (int64_t)r0 * rs + d0);
            st[j][1] = *reinterpret_cast<const bq_u4*>(src + (int64_t)r1 * rs + d0);
        }
    }
}

// natural image [SB][KROW]
template <int D>
__device__ __forceinline__ void ab_st_nat(u16* img, const bq_u4 (&st)[AbGeo<D>::NVU][2]) {
    using G = AbGeo<D>;
#pragma unroll
    for (int j = 0; j < G::NVU; ++j) {
        const int u = threadIdx.x + j * kBlock;
        if (u < G::SB / 2 * (D / 8)) {
            const int p = u / (D / 8), d0 = 8 * (u - p * (D / 8));
            *reinterpret_cast<bq_u4*>(img + (2 * p) * G::KROW + d0) = st[j][0];
            *reinterpret_cast<bq_u4*>(img + (2 * p + 1) * G::KROW + d0) = st[j][1];
        }
    }
}

typedef short ab_s4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) ab_s4 ab_lds_s4;

// The A fragment of a transposed operand (rows d = 32 dt .. +31, K = 16 rows of a natural
// [rows][KROW] image in the C layout's order: element j of lane half h is row
// row0 + 8 (j >> 2) + 4 h + (j & 3)) read straight from the natural image with two
// ds_read_b64_tr_b16 (T10: lane 4q + p of a 16-lane group gives the address of row q, columns
// 4p .. 4p + 3, and receives column `lane % 16` of the 4 rows) — no transposed copy in LDS.
// trb = img + (4 h + q) KROW + 16 g + 4 p for lane (h, g, q, p); off = row0 KROW + 32 dt.
template <int KROW>
__device__ __forceinline__ bq_u4 ab_tr(const u16* trb, int off) {
    const ab_s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ab_lds_s4*)(trb + off));
    const ab_s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ab_lds_s4*)(trb + off + 8 * KROW));
    return bq_u4{__builtin_bit_cast(bq_u2, lo)[0], __builtin_bit_cast(bq_u2, lo)[1], __builtin_bit_cast(bq_u2, hi)[0],
                 __builtin_bit_cast(bq_u2, hi)[1]};
}

__device__ __forceinline__ int ab_trlane(int lane, int krow) {
    return (4 * (lane >> 5) + ((lane >> 2) & 3)) * krow + 16 * ((lane >> 4) & 1) + 4 * (lane & 3);
}

template <int D>
__global__ __launch_bounds__(kBlock) void k_attnb_fwd(const u16* __restrict__ q, const u16* __restrict__ k,
                                                      const u16* __restrict__ v, int n, int m, int heads,
                                                      int rsq, int rskv, int kv_shared, int ro, float sl2,
                                                      u16* __restrict__ out, float* __restrict__ lse) {
    using G = AbGeo<D>;
    __shared__ __attribute__((aligned(16))) u16 Ks[G::IMG];
    __shared__ __attribute__((aligned(16))) u16 Vs[G::IMG];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
    const int bh = blockIdx.y, b = bh / heads, hd = bh - b * heads;
    const int q0 = blockIdx.x * AB_WB + wv * AB_QW;
    const u16* __restrict__ qb = q + (int64_t)b * n * rsq + hd * D;
    const int64_t kvb = (kv_shared ? 0 : (int64_t)b * m * rskv) + hd * D;

    if constexpr (G::DKP > D) {  // K's padding columns: zero once
        for (int i = tid; i < G::SB; i += kBlock)
#pragma unroll
            for (int cc = D; cc < G::DKP; cc += 2) *reinterpret_cast<unsigned*>(Ks + i * G::KROW + cc) = 0u;
    }
    // Q^T as B: lane (query r, half hh) holds Q[q0 + r][16 s + 8 hh + j]
    bq_u4 qf[G::DK];
    const int qq = q0 + r;
#pragma unroll
    for (int s = 0; s < G::DK; ++s) {
        const int d0 = 16 * s + 8 * hh;
        qf[s] = (d0 + 8 <= D && qq < n) ? *reinterpret_cast<const bq_u4*>(qb + (int64_t)qq * rsq + d0)
                                        : bq_u4{0u, 0u, 0u, 0u};
    }
    bq_f16 o[G::DT];
#pragma unroll
    for (int dt = 0; dt < G::DT; ++dt) o[dt] = bq_f16{};
    float mx = -INFINITY, l = 0.f;

    const int nst = (m + G::SB - 1) / G::SB;
    bq_u4 ks[G::NVU][2], vs[G::NVU][2];
    const u16* trb = Vs + ab_trlane(lane, G::KROW);
    ab_ld_pairs<D>(k + kvb, rskv, 0, m, ks);
    ab_ld_pairs<D>(v + kvb, rskv, 0, m, vs);
    for (int si = 0; si < nst; ++si) {
        __syncthreads();
        ab_st_nat<D>(Ks, ks);
        ab_st_nat<D>(Vs, vs);
        __syncthreads();
        if (si + 1 < nst) {
            ab_ld_pairs<D>(k + kvb, rskv, (si + 1) * G::SB, m, ks);
            ab_ld_pairs<D>(v + kvb, rskv, (si + 1) * G::SB, m, vs);
        }
        const int kbase = si * G::SB;
#pragma unroll
        for (int kb32 = 0; kb32 < G::SB / 32; ++kb32) {
            if (kbase + kb32 * 32 >= m) break;  // wave-uniform
            bq_f16 sv = bq_f16{};
#pragma unroll
            for (int s = 0; s < G::DK; ++s) {
                const bq_u4 kf = *reinterpret_cast<const bq_u4*>(Ks + (kb32 * 32 + r) * G::KROW + 16 * s + 8 * hh);
                sv = bq_mfma(kf, qf[s], sv);
            }
            float bm = -INFINITY;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int key = kbase + kb32 * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
                sv[i] = key < m ? sv[i] * sl2 : -INFINITY;
                bm = fmaxf(bm, sv[i]);
            }
            bm = fmaxf(bm, __shfl_xor(bm, 32));
            const float mn = bm > mx + AB_LAZY ? bm : mx;
            const float corr = __builtin_amdgcn_exp2f(mx - mn);
            mx = mn;
            float p[16], ps = 0.f;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                p[i] = __builtin_amdgcn_exp2f(sv[i] - mn);
                ps += p[i];
            }
            l = fmaf(l, corr, ps);
            if (__builtin_amdgcn_ballot_w64(corr != 1.f))
#pragma unroll
                for (int dt = 0; dt < G::DT; ++dt) o[dt] *= corr;
            bq_u4 pf[2];
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                pf[kk] = bq_u4{pk2(p[8 * kk], p[8 * kk + 1]), pk2(p[8 * kk + 2], p[8 * kk + 3]),
                               pk2(p[8 * kk + 4], p[8 * kk + 5]), pk2(p[8 * kk + 6], p[8 * kk + 7])};
#pragma unroll
            for (int dt = 0; dt < G::DT; ++dt)
#pragma unroll
                for (int kk = 0; kk < 2; ++kk) {
                    const bq_u4 vf = ab_tr<G::KROW>(trb, (kb32 * 32 + kk * 16) * G::KROW + 32 * dt);
                    o[dt] = bq_mfma(vf, pf[kk], o[dt]);
                }
        }
    }
    const float tot = l + __shfl_xor(l, 32);
    const float inv = 1.f / tot;
    if (qq >= n) return;
    u16* orow = out + (int64_t)b * n * ro + hd * D + (int64_t)qq * ro;
#pragma unroll
    for (int dt = 0; dt < G::DT; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int d0 = 32 * dt + 8 * g4 + 4 * hh;
            if (d0 + 4 <= D)
                *reinterpret_cast<bq_u2*>(orow + d0) = bq_u2{pk2(o[dt][4 * g4] * inv, o[dt][4 * g4 + 1] * inv),
                                                             pk2(o[dt][4 * g4 + 2] * inv, o[dt][4 * g4 + 3] * inv)};
        }
    if (hh == 0) lse[(int64_t)bh * n + qq] = (mx + log2f(tot)) * AB_LN2;
}

template <int D>
static void attnb_launch(const u16* q, const u16* k, const u16* v, int64_t batch, int heads, int64_t n, int64_t m,
                         int rsq, int rskv, int kv_shared, int ro, float scale, u16* out, float* lse, hipStream_t s) {
    const dim3 grid(static_cast<unsigned>((n + AB_WB - 1) / AB_WB), static_cast<unsigned>(batch * heads));
    launch(0, k_attnb_fwd<D>, grid, dim3(kBlock), s, q, k, v, static_cast<int>(n), static_cast<int>(m), heads, rsq,
           rskv, kv_shared, ro, scale * AB_LOG2E, out, lse);
}

// ---------------------------------------------------------------------------------------------
// Attention VJP on bf16 MFMAs (FlashAttention-2 recurrence, P never in HBM): delta = rowsum(dO o O),
// then
//   k_attnb_dq   per wave 32 queries: S^T = K Q^T, dP^T = V dO^T (Q^T, dO^T in registers), dS^T =
//                P^T (dP^T - delta), dQ^T += K^T dS^T (K^T staged in LDS in the C layout's key order)
//   k_attnb_dkv  per wave 32 keys: S = Q K^T, dP = dO V^T (K^T, V^T in registers), dS = P (dP -
//                delta), dV^T += dO^T P and dK^T += Q^T dS (Q^T, dO^T staged in that order)
// P and dS are rounded to bf16 as MFMA operands (as the forward's P); fp32 accumulation.
// ---------------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(kBlock) void k_attnb_delta(const u16* __restrict__ out, const u16* __restrict__ dout,
                                                        int n, int heads, int ro, int64_t rows,
                                                        float* __restrict__ delta) {
    const int64_t rr = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (rr >= rows) return;
    const int bh = static_cast<int>(rr / n), i = static_cast<int>(rr - (int64_t)bh * n);
    const int b = bh / heads, hd = bh - b * heads;
    const int64_t off = ((int64_t)b * n + i) * ro + hd * D;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < D / 8; ++j) {
        float a[8], c[8];
        unpack8(*reinterpret_cast<const bq_u4*>(out + off + 8 * j), a);
        unpack8(*reinterpret_cast<const bq_u4*>(dout + off + 8 * j), c);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc = fmaf(a[e], c[e], acc);
    }
    delta[rr] = acc;
}

// the B-operand fragments of 32 rows (lane row r) of a row-major [rows][D] operand, d padded to 16
template <int D>
__device__ __forceinline__ void ab_rowfrags(const u16* __restrict__ src, int64_t rs, int row, int limit, int hh,
                                            bq_u4 (&f)[AbGeo<D>::DK]) {
#pragma unroll
    for (int s = 0; s < AbGeo<D>::DK; ++s) {
        const int d0 = 16 * s + 8 * hh;
        f[s] = (d0 + 8 <= D && row < limit) ? *reinterpret_cast<const bq_u4*>(src + (int64_t)row * rs + d0)
                                            : bq_u4{0u, 0u, 0u, 0u};
    }
}

template <int D>
__device__ __forceinline__ void ab_zero_pad(u16* img) {
    using G = AbGeo<D>;
    if constexpr (G::DKP > D) {
        for (int i = threadIdx.x; i < G::SB; i += kBlock)
#pragma unroll
            for (int cc = D; cc < G::DKP; cc += 2) *reinterpret_cast<unsigned*>(img + i * G::KROW + cc) = 0u;
    }
}

// C-layout rows d of 32 columns -> bf16 row-major output: lane's column `row`, 4 d per store
template <int D>
__device__ __forceinline__ void ab_store_rows(u16* __restrict__ dst, int64_t rs, int row, int limit, int hh,
                                              const bq_f16 (&acc)[AbGeo<D>::DT], float mul) {
    if (row >= limit) return;
    u16* o = dst + (int64_t)row * rs;
#pragma unroll
    for (int dt = 0; dt < AbGeo<D>::DT; ++dt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            const int d0 = 32 * dt + 8 * g4 + 4 * hh;
            if (d0 + 4 <= D)
                *reinterpret_cast<bq_u2*>(o + d0) = bq_u2{pk2(acc[dt][4 * g4] * mul, acc[dt][4 * g4 + 1] * mul),
                                                          pk2(acc[dt][4 * g4 + 2] * mul, acc[dt][4 * g4 + 3] * mul)};
        }
}

template <int D>
__global__ __launch_bounds__(kBlock) void k_attnb_dq(const u16* __restrict__ q, const u16* __restrict__ k,
                                                     const u16* __restrict__ v, const u16* __restrict__ dout,
                                                     const float* __restrict__ lse, const float* __restrict__ delta,
                                                     int n, int m, int heads, int rsq, int rskv, int kv_shared,
                                                     int ro, int rdq, float sl2, float scale,
                                                     u16* __restrict__ dq) {
    using G = AbGeo<D>;
    __shared__ __attribute__((aligned(16))) u16 Kn[G::IMG];
    __shared__ __attribute__((aligned(16))) u16 Vn[G::IMG];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
    const int bh = blockIdx.y, b = bh / heads, hd = bh - b * heads;
    const int qq = blockIdx.x * AB_WB + wv * AB_QW + r;
    const int64_t kvb = (kv_shared ? 0 : (int64_t)b * m * rskv) + hd * D;
    ab_zero_pad<D>(Kn);
    ab_zero_pad<D>(Vn);
    const u16* trk = Kn + ab_trlane(lane, G::KROW);
    bq_u4 qf[G::DK], of[G::DK];
    ab_rowfrags<D>(q + (int64_t)b * n * rsq + hd * D, rsq, qq, n, hh, qf);
    ab_rowfrags<D>(dout + (int64_t)b * n * ro + hd * D, ro, qq, n, hh, of);
    const float ll = qq < n ? lse[(int64_t)bh * n + qq] * AB_LOG2E : 0.f;
    const float dl = qq < n ? delta[(int64_t)bh * n + qq] : 0.f;
    bq_f16 acc[G::DT];
#pragma unroll
    for (int dt = 0; dt < G::DT; ++dt) acc[dt] = bq_f16{};
    const int nst = (m + G::SB - 1) / G::SB;
    bq_u4 ks[G::NVU][2], vs[G::NVU][2];
    ab_ld_pairs<D>(k + kvb, rskv, 0, m, ks);
    ab_ld_pairs<D>(v + kvb, rskv, 0, m, vs);
    for (int si = 0; si < nst; ++si) {
        __syncthreads();
        ab_st_nat<D>(Kn, ks);
        ab_st_nat<D>(Vn, vs);
        __syncthreads();
        if (si + 1 < nst) {
            ab_ld_pairs<D>(k + kvb, rskv, (si + 1) * G::SB, m, ks);
            ab_ld_pairs<D>(v + kvb, rskv, (si + 1) * G::SB, m, vs);
        }
        const int kbase = si * G::SB;
#pragma unroll
        for (int kb32 = 0; kb32 < G::SB / 32; ++kb32) {
            if (kbase + kb32 * 32 >= m) break;
            bq_f16 sv = bq_f16{}, dp = bq_f16{};
#pragma unroll
            for (int s2 = 0; s2 < G::DK; ++s2) {
                const int o = (kb32 * 32 + r) * G::KROW + 16 * s2 + 8 * hh;
                sv = bq_mfma(*reinterpret_cast<const bq_u4*>(Kn + o), qf[s2], sv);
                dp = bq_mfma(*reinterpret_cast<const bq_u4*>(Vn + o), of[s2], dp);
            }
            float ds[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int key = kbase + kb32 * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh;
                const float p = key < m ? __builtin_amdgcn_exp2f(fmaf(sv[i], sl2, -ll)) : 0.f;
                ds[i] = p * (dp[i] - dl);
            }
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const bq_u4 pf = {pk2(ds[8 * kk], ds[8 * kk + 1]), pk2(ds[8 * kk + 2], ds[8 * kk + 3]),
                                  pk2(ds[8 * kk + 4], ds[8 * kk + 5]), pk2(ds[8 * kk + 6], ds[8 * kk + 7])};
#pragma unroll
                for (int dt = 0; dt < G::DT; ++dt) {
                    const bq_u4 a = ab_tr<G::KROW>(trk, (kb32 * 32 + kk * 16) * G::KROW + 32 * dt);
                    acc[dt] = bq_mfma(a, pf, acc[dt]);
                }
            }
        }
    }
    ab_store_rows<D>(dq + (int64_t)b * n * rdq + hd * D, rdq, qq, n, hh, acc, scale);
}

template <int D>
__global__ __launch_bounds__(kBlock) void k_attnb_dkv(const u16* __restrict__ q, const u16* __restrict__ k,
                                                      const u16* __restrict__ v, const u16* __restrict__ dout,
                                                      const float* __restrict__ lse, const float* __restrict__ delta,
                                                      int n, int heads, int rs, int ro, int rdkv, float sl2,
                                                      float scale, u16* __restrict__ dk, u16* __restrict__ dv) {
    using G = AbGeo<D>;
    __shared__ __attribute__((aligned(16))) u16 Qn[G::IMG];
    __shared__ __attribute__((aligned(16))) u16 On[G::IMG];
    __shared__ __attribute__((aligned(16))) float Ls[G::SB], Dl[G::SB];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, r = lane & 31, hh = lane >> 5;
    const int bh = blockIdx.y, b = bh / heads, hd = bh - b * heads;
    const int kk_ = blockIdx.x * AB_WB + wv * AB_QW + r;  // this lane's key
    const int64_t base = (int64_t)b * n * rs + hd * D, obase = (int64_t)b * n * ro + hd * D;
    ab_zero_pad<D>(Qn);
    ab_zero_pad<D>(On);
    const u16* trq = Qn + ab_trlane(lane, G::KROW);
    const u16* tro = On + ab_trlane(lane, G::KROW);
    bq_u4 kf[G::DK], vf[G::DK];
    ab_rowfrags<D>(k + base, rs, kk_, n, hh, kf);
    ab_rowfrags<D>(v + base, rs, kk_, n, hh, vf);
    bq_f16 ak[G::DT], av[G::DT];
#pragma unroll
    for (int dt = 0; dt < G::DT; ++dt) ak[dt] = bq_f16{}, av[dt] = bq_f16{};
    const int nst = (n + G::SB - 1) / G::SB;
    bq_u4 qs[G::NVU][2], os[G::NVU][2];
    // the row constants of the next stage: a plain load in flight beside the Q / dO rows (any
    // arithmetic on it here would make the compiler wait for every load of the stage at once);
    // scaled and masked when stored
    float lv = 0.f;
    auto ld = [&](int si) {
        ab_ld_pairs<D>(q + base, rs, si * G::SB, n, qs);
        ab_ld_pairs<D>(dout + obase, ro, si * G::SB, n, os);
        const int qi = min(si * G::SB + (tid & (G::SB - 1)), n - 1);
        lv = ((tid & G::SB) ? delta : lse)[(int64_t)bh * n + qi];  // every thread: no branch
    };
    ld(0);
    for (int si = 0; si < nst; ++si) {
        __syncthreads();
        ab_st_nat<D>(Qn, qs);
        ab_st_nat<D>(On, os);
        {
            const bool in = si * G::SB + (tid & (G::SB - 1)) < n;
            if (tid < G::SB)
                Ls[tid] = in ? lv * AB_LOG2E : INFINITY;
            else if (tid < 2 * G::SB)
                Dl[tid - G::SB] = in ? lv : 0.f;
        }
        __syncthreads();
        if (si + 1 < nst) ld(si + 1);
#pragma unroll
        for (int ib32 = 0; ib32 < G::SB / 32; ++ib32) {
            if (si * G::SB + ib32 * 32 >= n) break;
            bq_f16 sv = bq_f16{}, dp = bq_f16{};
#pragma unroll
            for (int s2 = 0; s2 < G::DK; ++s2) {
                const int o = (ib32 * 32 + r) * G::KROW + 16 * s2 + 8 * hh;
                sv = bq_mfma(*reinterpret_cast<const bq_u4*>(Qn + o), kf[s2], sv);
                dp = bq_mfma(*reinterpret_cast<const bq_u4*>(On + o), vf[s2], dp);
            }
            float p[16], ds[16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int q0 = ib32 * 32 + 8 * g + 4 * hh;
                const float4 l4 = *reinterpret_cast<const float4*>(Ls + q0);
                const float4 d4 = *reinterpret_cast<const float4*>(Dl + q0);
                const float la[4] = {l4.x, l4.y, l4.z, l4.w}, da[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int i = 4 * g + e;
                    p[i] = __builtin_amdgcn_exp2f(fmaf(sv[i], sl2, -la[e]));
                    ds[i] = p[i] * (dp[i] - da[e]);
                }
            }
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const bq_u4 pp = {pk2(p[8 * kk], p[8 * kk + 1]), pk2(p[8 * kk + 2], p[8 * kk + 3]),
                                  pk2(p[8 * kk + 4], p[8 * kk + 5]), pk2(p[8 * kk + 6], p[8 * kk + 7])};
                const bq_u4 pd = {pk2(ds[8 * kk], ds[8 * kk + 1]), pk2(ds[8 * kk + 2], ds[8 * kk + 3]),
                                  pk2(ds[8 * kk + 4], ds[8 * kk + 5]), pk2(ds[8 * kk + 6], ds[8 * kk + 7])};
#pragma unroll
                for (int dt = 0; dt < G::DT; ++dt) {
                    const int o = (ib32 * 32 + kk * 16) * G::KROW + 32 * dt;
                    av[dt] = bq_mfma(ab_tr<G::KROW>(tro, o), pp, av[dt]);
                    ak[dt] = bq_mfma(ab_tr<G::KROW>(trq, o), pd, ak[dt]);
                }
            }
        }
    }
    ab_store_rows<D>(dk + (int64_t)b * n * rdkv + hd * D, rdkv, kk_, n, hh, ak, scale);
    ab_store_rows<D>(dv + (int64_t)b * n * rdkv + hd * D, rdkv, kk_, n, hh, av, 1.f);
}

template <int D>
static void attnb_bwd_launch(const u16* q, const u16* k, const u16* v, const u16* out, const u16* dout,
                             const float* lse, int64_t batch, int heads, int64_t n, int64_t m, int rsq, int rskv,
                             int kv_shared, int ro, int rdq, int rdkv, float scale, float* delta, u16* dq, u16* dk,
                             u16* dv, hipStream_t s) {
    const int64_t rows = batch * heads * n;
    launch(0, k_attnb_delta<D>, dim3(static_cast<unsigned>((rows + kBlock - 1) / kBlock)), dim3(kBlock), s, out, dout,
           static_cast<int>(n), heads, ro, rows, delta);
    const float sl2 = scale * AB_LOG2E;
    if (dq)
        launch(0, k_attnb_dq<D>, dim3(static_cast<unsigned>((n + AB_WB - 1) / AB_WB), static_cast<unsigned>(batch * heads)),
               dim3(kBlock), s, q, k, v, dout, lse, static_cast<const float*>(delta), static_cast<int>(n),
               static_cast<int>(m), heads, rsq, rskv, kv_shared, ro, rdq, sl2, scale, dq);
    if (dk)
        launch(0, k_attnb_dkv<D>, dim3(static_cast<unsigned>((n + AB_WB - 1) / AB_WB), static_cast<unsigned>(batch * heads)),
               dim3(kBlock), s, q, k, v, dout, lse, static_cast<const float*>(delta), static_cast<int>(n), heads, rsq,
               ro, rdkv, sl2, scale, dk, dv);
}

}  // namespace sp

using namespace sp;

extern "C" {

// ---- 3x3 convolution ------------------------------------------------------------------------

int sp_conv3x3_bf16_supported(int32_t cin, int32_t cout, int32_t h, int32_t w) {
    return cin > 0 && cin % 16 == 0 && cout > 0 && conv_tc(h, w) != 0;
}

// elements (bf16) of the packed weights: [ceil(cout/64)][cin/16][9][64][16]
int64_t sp_conv3x3_bf16_packed_size(int32_t cin, int32_t cout) {
    return (int64_t)((cout + 63) / 64) * 64 * cin * 9;
}

// y[n][h][w][cout] = conv3x3(x[n][h][w][cin], W) + bias (+ res), NHWC bf16, fp32 accumulation.
// wp: packed as [co block of 64][ci block of 16][tap 3 ky + kx][64 co][16 ci] (rows past cout
// zero); the input VJP is the same call with the pack of W'[ci][co][2-ky][2-kx].
static int conv_bf16_call(const void* x, const void* wp, const float* bias, const void* res, int64_t n, int32_t cin,
                          int32_t cout, int32_t h, int32_t w, void* y, sp_stream_t stream, bool up,
                          void* ws = nullptr, int64_t ws_bytes = 0, int blk = 0, const ConvSc& sc = ConvSc{}) {
    if (!x || !wp || !y || n <= 0 || !sp_conv3x3_bf16_supported(cin, cout, h, w)) return SP_EINVAL;
    if (blk && (up || conv_tc(h, w) != 32)) return SP_EINVAL;
    const int cs = sc.cs1 + sc.cs2;
    if (sc.wsp && (up || res || conv_tc(h, w) != 32 || !sc.xs1 || sc.cs1 <= 0 || sc.cs1 % 16 || sc.cs2 < 0 ||
                   sc.cs2 % 16 || (sc.cs2 && !sc.xs2) || n * h * (int64_t)w * cs >= (int64_t(1) << 40)))
        return SP_EINVAL;
    if (up && (h % 2 || w % 2)) return SP_EINVAL;
    if (n * h * (int64_t)w * std::max(cin, cout) >= (int64_t(1) << 40) || n >= (int64_t(1) << 30)) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const u16* xx = static_cast<const u16*>(x);
    const u16* ww = static_cast<const u16*>(wp);
    const u16* rr = static_cast<const u16*>(res);
    u16* yy = static_cast<u16*>(y);
    const int ni = static_cast<int>(n);
    if (up) {
        switch (conv_tc(h, w)) {
            case 32: conv_bf16_launch<32, true>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s); break;
            case 16: conv_bf16_launch<16, true>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s); break;
            case 8: conv_bf16_launch<8, true>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s); break;
            default: conv_bf16_launch<4, true>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s); break;
        }
        return check_launch("sp_conv3x3_bf16_up");
    }
    int parts = conv_parts(ni, cin + (sc.wsp ? cs : 0), cout, h, w);
    if (parts > 1 && (!ws || ws_bytes < 4 * parts * (int64_t)ni * h * w * cout)) parts = 1;
    float* part = static_cast<float*>(ws);
    if (sc.wsp) {
        if (blk) conv_bf16_launch<32, false, true, true>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s, part, parts, sc);
        else conv_bf16_launch<32, false, false, true>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s, part, parts, sc);
        return check_launch("sp_conv3x3_bf16_sc");
    }
    if (blk) {
        conv_bf16_launch<32, false, true>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s, part, parts);
        return check_launch("sp_conv3x3_bf16_ex");
    }
    switch (conv_tc(h, w)) {
        case 32: conv_bf16_launch<32, false>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s, part, parts); break;
        case 16: conv_bf16_launch<16, false>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s, part, parts); break;
        case 8: conv_bf16_launch<8, false>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s, part, parts); break;
        default: conv_bf16_launch<4, false>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s, part, parts); break;
    }
    return check_launch("sp_conv3x3_bf16");
}

// bytes of the split-K workspace sp_conv3x3_bf16_ws uses for this shape (0: the launch fills the
// chip unsplit): parts x n h w cout fp32
int64_t sp_conv3x3_bf16_workspace(int64_t n, int32_t cin, int32_t cout, int32_t h, int32_t w) {
    if (n <= 0 || n >= (int64_t(1) << 30) || !sp_conv3x3_bf16_supported(cin, cout, h, w)) return 0;
    const int parts = conv_parts(static_cast<int>(n), cin, cout, h, w);
    return parts > 1 ? 4 * parts * n * h * (int64_t)w * cout : 0;
}

// sp_conv3x3_bf16 with split-K over the input channels where the workgroups would leave CUs idle:
// the parts' fp32 sums go to ws (sp_conv3x3_bf16_workspace bytes) and a fixed-order reduce adds
// them with the bias / residual (deterministic); ws = NULL or short: unsplit
int sp_conv3x3_bf16_ws(const void* x, const void* wp, const float* bias, const void* res, int64_t n, int32_t cin,
                       int32_t cout, int32_t h, int32_t w, void* y, void* ws, int64_t ws_bytes, sp_stream_t stream) {
    return conv_bf16_call(x, wp, bias, res, n, cin, cout, h, w, y, stream, false, ws, ws_bytes);
}

// sp_conv3x3_bf16_ws with the input in a chosen layout: in_layout 0 = NHWC, 1 = channel-blocked
// [n][cin / 16][h][w][16] (each 16-channel stage of the tile reads whole lines; TC = 32 shapes only:
// sp_conv3x3_bf16_blk_supported).  The output stays NHWC.
int sp_conv3x3_bf16_blk_supported(int32_t cin, int32_t cout, int32_t h, int32_t w) {
    return sp_conv3x3_bf16_supported(cin, cout, h, w) && conv_tc(h, w) == 32;
}

int sp_conv3x3_bf16_ex(const void* x, int32_t in_layout, const void* wp, const float* bias, const void* res, int64_t n,
                       int32_t cin, int32_t cout, int32_t h, int32_t w, void* y, void* ws, int64_t ws_bytes,
                       sp_stream_t stream) {
    if (in_layout != 0 && in_layout != 1) return SP_EINVAL;
    return conv_bf16_call(x, wp, bias, res, n, cin, cout, h, w, y, stream, false, ws, ws_bytes, in_layout);
}

// y = conv3x3(x) + conv1x1(cat(xs1, xs2)) + bias: the ResnetBlock's conv2 with its conv_shortcut summed
// as further stages of the same contraction (no shortcut tensor, no residual read).  wsp: the 1x1
// weights packed as [co block of 64][cs / 16][64 co][16 ci] (sp_conv3x3_bf16_sc_packed_size
// elements, rows past cout zero); bias: conv2's + the shortcut's.  TC = 32 shapes
// (sp_conv3x3_bf16_sc_supported); split-K over all stages (sp_conv3x3_bf16_sc_workspace).
int sp_conv3x3_bf16_sc_supported(int32_t cin, int32_t cout, int32_t cs1, int32_t cs2, int32_t h, int32_t w) {
    return sp_conv3x3_bf16_supported(cin, cout, h, w) && conv_tc(h, w) == 32 && cs1 > 0 && cs1 % 16 == 0 &&
           cs2 >= 0 && cs2 % 16 == 0;
}

int64_t sp_conv3x3_bf16_sc_packed_size(int32_t cs, int32_t cout) { return (int64_t)((cout + 63) / 64) * 64 * cs; }

int64_t sp_conv3x3_bf16_sc_workspace(int64_t n, int32_t cin, int32_t cs, int32_t cout, int32_t h, int32_t w) {
    if (n <= 0 || n >= (int64_t(1) << 30) || cs < 0 || !sp_conv3x3_bf16_supported(cin, cout, h, w)) return 0;
    const int parts = conv_parts(static_cast<int>(n), cin + cs, cout, h, w);
    return parts > 1 ? 4 * parts * n * h * (int64_t)w * cout : 0;
}

int sp_conv3x3_bf16_sc(const void* x, int32_t in_layout, const void* wp, const float* bias, const void* xs1,
                       const void* xs2, int32_t cs1, int32_t cs2, const void* wsp, int64_t n, int32_t cin, int32_t cout,
                       int32_t h, int32_t w, void* y, void* ws, int64_t ws_bytes, sp_stream_t stream) {
    if ((in_layout != 0 && in_layout != 1) || !wsp || !sp_conv3x3_bf16_sc_supported(cin, cout, cs1, cs2, h, w))
        return SP_EINVAL;
    ConvSc sc;
    sc.xs1 = static_cast<const u16*>(xs1), sc.xs2 = static_cast<const u16*>(xs2);
    sc.cs1 = cs1, sc.cs2 = cs2, sc.wsp = static_cast<const u16*>(wsp);
    return conv_bf16_call(x, wp, bias, nullptr, n, cin, cout, h, w, y, stream, false, ws, ws_bytes, in_layout, sc);
}

int sp_conv3x3_bf16(const void* x, const void* wp, const float* bias, const void* res, int64_t n, int32_t cin,
                    int32_t cout, int32_t h, int32_t w, void* y, sp_stream_t stream) {
    return conv_bf16_call(x, wp, bias, res, n, cin, cout, h, w, y, stream, false);
}

// y = conv3x3(upsample_nearest2x(x)) + bias (+ res): x [n][h/2][w/2][cin], y [n][h][w][cout]
int sp_conv3x3_bf16_up(const void* x, const void* wp, const float* bias, const void* res, int64_t n, int32_t cin,
                       int32_t cout, int32_t h, int32_t w, void* y, sp_stream_t stream) {
    return conv_bf16_call(x, wp, bias, res, n, cin, cout, h, w, y, stream, true);
}

// dx[n][h/2][w/2][c] = 2 x 2 block sums of dz[n][h][w][c] (Upsample2D's VJP), NHWC bf16
int sp_pool2x2_bf16(const void* dz, int64_t n, int32_t c, int32_t h, int32_t w, void* dx, sp_stream_t stream) {
    if (!dz || !dx || n <= 0 || c <= 0 || c % 8 || h <= 0 || w <= 0 || h % 2 || w % 2) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t vec = n * (h / 2) * (int64_t)(w / 2) * (c / 8);
    launch(0, k_pool2x2_bf16, dim3(stream_blocks(vec)), dim3(kBlock), s, static_cast<const u16*>(dz), n, c, h / 2,
           w / 2, static_cast<u16*>(dx));
    return check_launch("sp_pool2x2_bf16");
}

// ---- LayerNorm -----------------------------------------------------------------------------

int sp_layernorm_bf16_supported(int64_t rows, int32_t c) { return rows >= 0 && c > 0 && c % 8 == 0 && c <= 8 * 64 * 4; }

int sp_layernorm_bf16_fwd(const void* x, const float* w, const float* b, int64_t rows, int32_t c, float eps, void* y,
                          float* mean, float* rstd, sp_stream_t stream) {
    if (!sp_layernorm_bf16_supported(rows, c)) return SP_EINVAL;
    if (rows == 0) return SP_OK;
    if (!x || !w || !b || !y || !mean || !rstd) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid(static_cast<unsigned>((rows + LNB_ROWS - 1) / LNB_ROWS));
    const int nv = (c / 8 + 63) / 64;
    const u16* xx = static_cast<const u16*>(x);
    u16* yy = static_cast<u16*>(y);
    if (nv == 1) launch(0, k_layernorm_bf16_fwd<1>, grid, dim3(kBlock), s, xx, w, b, rows, static_cast<int>(c), eps, yy, mean, rstd);
    else if (nv == 2) launch(0, k_layernorm_bf16_fwd<2>, grid, dim3(kBlock), s, xx, w, b, rows, static_cast<int>(c), eps, yy, mean, rstd);
    else if (nv == 3) launch(0, k_layernorm_bf16_fwd<3>, grid, dim3(kBlock), s, xx, w, b, rows, static_cast<int>(c), eps, yy, mean, rstd);
    else launch(0, k_layernorm_bf16_fwd<4>, grid, dim3(kBlock), s, xx, w, b, rows, static_cast<int>(c), eps, yy, mean, rstd);
    return check_launch("sp_layernorm_bf16_fwd");
}

int sp_layernorm_bf16_bwd(const void* dy, const void* x, const float* w, const float* mean, const float* rstd,
                          const void* add, int64_t rows, int32_t c, void* dx, sp_stream_t stream) {
    if (!sp_layernorm_bf16_supported(rows, c)) return SP_EINVAL;
    if (rows == 0) return SP_OK;
    if (!dy || !x || !w || !mean || !rstd || !dx) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid(static_cast<unsigned>((rows + LNB_ROWS - 1) / LNB_ROWS));
    const int nv = (c / 8 + 63) / 64;
    const u16 *d = static_cast<const u16*>(dy), *xx = static_cast<const u16*>(x), *a = static_cast<const u16*>(add);
    u16* o = static_cast<u16*>(dx);
    if (nv == 1) launch(0, k_layernorm_bf16_bwd<1>, grid, dim3(kBlock), s, d, xx, w, mean, rstd, a, rows, static_cast<int>(c), o);
    else if (nv == 2) launch(0, k_layernorm_bf16_bwd<2>, grid, dim3(kBlock), s, d, xx, w, mean, rstd, a, rows, static_cast<int>(c), o);
    else if (nv == 3) launch(0, k_layernorm_bf16_bwd<3>, grid, dim3(kBlock), s, d, xx, w, mean, rstd, a, rows, static_cast<int>(c), o);
    else launch(0, k_layernorm_bf16_bwd<4>, grid, dim3(kBlock), s, d, xx, w, mean, rstd, a, rows, static_cast<int>(c), o);
    return check_launch("sp_layernorm_bf16_bwd");
}

// ---- GEGLU ---------------------------------------------------------------------------------

int sp_geglu_bf16_fwd(const void* h, int64_t rows, int32_t f, void* y, sp_stream_t stream) {
    if (rows < 0 || f <= 0 || f % 8) return SP_EINVAL;
    if (rows == 0) return SP_OK;
    if (!h || !y) return SP_EINVAL;
    const int64_t vec = rows * (f / 8);
    launch(0, k_geglu_bf16_fwd, dim3(stream_blocks(vec)), dim3(kBlock), static_cast<hipStream_t>(stream),
           static_cast<const u16*>(h), rows, static_cast<int>(f), static_cast<u16*>(y));
    return check_launch("sp_geglu_bf16_fwd");
}

int sp_geglu_bf16_bwd(const void* h, const void* dy, int64_t rows, int32_t f, void* dh, sp_stream_t stream) {
    if (rows < 0 || f <= 0 || f % 8) return SP_EINVAL;
    if (rows == 0) return SP_OK;
    if (!h || !dy || !dh || dh == h) return SP_EINVAL;
    const int64_t vec = rows * (f / 8);
    launch(0, k_geglu_bf16_bwd, dim3(stream_blocks(vec)), dim3(kBlock), static_cast<hipStream_t>(stream),
           static_cast<const u16*>(h), static_cast<const u16*>(dy), rows, static_cast<int>(f), static_cast<u16*>(dh));
    return check_launch("sp_geglu_bf16_bwd");
}

// ---- GroupNorm ------------------------------------------------------------------------------

int sp_groupnorm_bf16_supported(int32_t c1, int32_t c2, int32_t groups) {
    const int c = c1 + c2;
    return c1 > 0 && c1 % 8 == 0 && c2 >= 0 && c2 % 8 == 0 && groups > 0 && c % groups == 0 && c <= 8 * 1024;
}

// workspace bytes (fp32): partials [n][chunks][2][c] + coefficients [4][n][c] + [3][n][c]
int64_t sp_groupnorm_bf16_workspace(int64_t n, int32_t c, int64_t hw) {
    const GnbGeo g = gnb_geo(n, c, hw);
    return 4 * (n * g.chunks * 2 * (int64_t)c + 7 * n * (int64_t)c);
}

// z[n][hw][c] = act(GroupNorm(cat(x1, x2) + chan_bias[n][c]) * gamma + beta), NHWC bf16;
// stats = [mean | rstd] (2 n groups fp32, for the VJP); gamma / beta / chan_bias fp32 or NULL.
int sp_groupnorm_bf16_fwd(const void* x1, const void* x2, int32_t c1, int32_t c2, const float* chan_bias,
                          const float* gamma, const float* beta, int64_t n, int64_t hw, int32_t groups, float eps,
                          int32_t act, void* z, float* stats, void* ws, int64_t ws_bytes, sp_stream_t stream) {
    return sp_groupnorm_bf16_fwd_ex(x1, x2, c1, c2, chan_bias, gamma, beta, n, hw, groups, eps, act, z, 0, stats, ws,
                                    ws_bytes, stream);
}

// z_layout 1: z in the channel-blocked layout [n][c / 16][hw][16] (c % 16 == 0), the conv tile's
// preferred input (sp_conv3x3_bf16_ex)
int sp_groupnorm_bf16_fwd_ex(const void* x1, const void* x2, int32_t c1, int32_t c2, const float* chan_bias,
                             const float* gamma, const float* beta, int64_t n, int64_t hw, int32_t groups, float eps,
                             int32_t act, void* z, int32_t z_layout, float* stats, void* ws, int64_t ws_bytes,
                             sp_stream_t stream) {
    if (!x1 || (c2 && !x2) || !z || !stats || !ws || n <= 0 || hw <= 0 || !sp_groupnorm_bf16_supported(c1, c2, groups))
        return SP_EINVAL;
    if (z_layout != 0 && (z_layout != 1 || (c1 + c2) % 16)) return SP_EINVAL;
    const int c = c1 + c2;
    if (ws_bytes < sp_groupnorm_bf16_workspace(n, c, hw) || n * hw * c >= (int64_t(1) << 40) || n > 65535)
        return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const GnbGeo g = gnb_geo(n, c, hw);
    float* part = static_cast<float*>(ws);
    float* co = part + n * g.chunks * 2 * (int64_t)c;
    const u16* a = static_cast<const u16*>(x1);
    const u16* b = static_cast<const u16*>(x2);
    const bool nt = gnb_nt(n, c, hw);
    const dim3 grid(g.chunks, static_cast<unsigned>(n));
    auto stats_pass = [&](auto kern) {
        launch(0, kern, grid, dim3(kBlock), s, a, b, c1, c2, chan_bias, static_cast<const u16*>(nullptr),
               static_cast<const float*>(nullptr), static_cast<const float*>(nullptr), hw, g.chunk_px, part);
    };
    if (nt) stats_pass(k_gnb_stats<0, false, true>);
    else stats_pass(k_gnb_stats<0, false, false>);
    launch(0, k_gnb_final_fwd, dim3(groups, static_cast<unsigned>(n)), dim3(64), s, a, b, c1, c2, chan_bias,
           static_cast<const float*>(part), g.chunks, hw, groups, eps, gamma, beta, stats, co);
    auto apply_pass = [&](auto kern) {
        launch(0, kern, grid, dim3(kBlock), s, a, b, c1, c2, static_cast<const float*>(co), hw, g.chunk_px,
               static_cast<u16*>(z), static_cast<int>(z_layout));
    };
    if (act) nt ? apply_pass(k_gnb_apply<true, true>) : apply_pass(k_gnb_apply<true, false>);
    else nt ? apply_pass(k_gnb_apply<false, true>) : apply_pass(k_gnb_apply<false, false>);
    return check_launch("sp_groupnorm_bf16_fwd");
}

// input VJP of sp_groupnorm_bf16_fwd given its stats: dx1 / dx2 (the parts' layouts) =
// GN^T dz (+ add1 / add2, + add1b into dx1); the outputs may alias the addends.
int sp_groupnorm_bf16_bwd(const void* dz, const void* x1, const void* x2, int32_t c1, int32_t c2,
                          const float* chan_bias, const float* gamma, const float* beta, const float* stats,
                          int64_t n, int64_t hw, int32_t groups, int32_t act, void* dx1, void* dx2, const void* add1,
                          const void* add2, const void* add1b, void* ws, int64_t ws_bytes, sp_stream_t stream) {
    return sp_groupnorm_bf16_bwd_ex(dz, x1, x2, c1, c2, chan_bias, gamma, beta, stats, n, hw, groups, act, dx1, dx2,
                                    0, add1, add2, add1b, ws, ws_bytes, stream);
}

// dx_layout 1 (one part, c2 == 0, c1 % 16 == 0): dx1 in the channel-blocked layout [n][c / 16][hw][16]
// (the addends stay NHWC); dx_layout 2: dx1 / dx2 NHWC and add1 one addend over the concatenated
// channels [n][hw][c1 + c2] (add2 NULL; the outputs must not alias it)
int sp_groupnorm_bf16_bwd_ex(const void* dz, const void* x1, const void* x2, int32_t c1, int32_t c2,
                             const float* chan_bias, const float* gamma, const float* beta, const float* stats,
                             int64_t n, int64_t hw, int32_t groups, int32_t act, void* dx1, void* dx2, int32_t dx_layout,
                             const void* add1, const void* add2, const void* add1b, void* ws, int64_t ws_bytes,
                             sp_stream_t stream) {
    if (!dz || !x1 || (c2 && (!x2 || !dx2)) || !dx1 || !stats || !ws || n <= 0 || hw <= 0 ||
        !sp_groupnorm_bf16_supported(c1, c2, groups))
        return SP_EINVAL;
    if (dx_layout != 0 && (dx_layout != 1 || c2 || c1 % 16) && (dx_layout != 2 || add2)) return SP_EINVAL;
    const int c = c1 + c2;
    if (ws_bytes < sp_groupnorm_bf16_workspace(n, c, hw) || n * hw * c >= (int64_t(1) << 40) || n > 65535)
        return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const GnbGeo g = gnb_geo(n, c, hw);
    float* part = static_cast<float*>(ws);
    float* co = part + n * g.chunks * 2 * (int64_t)c;
    float* co2 = co + 4 * n * (int64_t)c;
    const u16* a = static_cast<const u16*>(x1);
    const u16* b = static_cast<const u16*>(x2);
    const u16* d = static_cast<const u16*>(dz);
    const int64_t nc = n * c;
    launch(0, k_gnb_coefs, dim3(static_cast<unsigned>((nc + kBlock - 1) / kBlock)), dim3(kBlock), s, stats, chan_bias,
           gamma, beta, static_cast<int>(n), c, groups, co);
    const bool nt = gnb_nt(n, c, hw);
    const dim3 grid(g.chunks, static_cast<unsigned>(n));
    auto stats_pass = [&](auto kern) {
        launch(0, kern, grid, dim3(kBlock), s, a, b, c1, c2, chan_bias, d, static_cast<const float*>(co), gamma, hw,
               g.chunk_px, part);
    };
    if (act) nt ? stats_pass(k_gnb_stats<1, true, true>) : stats_pass(k_gnb_stats<1, true, false>);
    else nt ? stats_pass(k_gnb_stats<1, false, true>) : stats_pass(k_gnb_stats<1, false, false>);
    launch(0, k_gnb_final_bwd, dim3(groups, static_cast<unsigned>(n)), dim3(64), s, static_cast<const float*>(part),
           g.chunks, hw, c, groups, stats, gamma, static_cast<const float*>(co), co2);
    auto apply_pass = [&](auto kern) {
        launch(0, kern, grid, dim3(kBlock), s, d, a, b, c1, c2, static_cast<const float*>(co),
               static_cast<const float*>(co2), hw, g.chunk_px, static_cast<u16*>(dx1), static_cast<u16*>(dx2),
               static_cast<const u16*>(add1), static_cast<const u16*>(add2), static_cast<const u16*>(add1b),
               static_cast<int>(dx_layout));
    };
    if (act) nt ? apply_pass(k_gnb_bwd_apply<true, true>) : apply_pass(k_gnb_bwd_apply<true, false>);
    else nt ? apply_pass(k_gnb_bwd_apply<false, true>) : apply_pass(k_gnb_bwd_apply<false, false>);
    return check_launch("sp_groupnorm_bf16_bwd");
}

// ---- conv input VJP + the GroupNorm VJP it feeds, with the GroupNorm sums from the conv epilogue ----

static int64_t gnv_tiles(int32_t h, int32_t w) { return (int64_t)(h / 16) * (w / 32); }

int sp_conv3x3_bf16_gnvjp_supported(int64_t n, int32_t cin, int32_t cout, int32_t h, int32_t w, int32_t c1,
                                    int32_t groups) {
    return n > 0 && n <= 65535 && sp_conv3x3_bf16_supported(cin, cout, h, w) && conv_tc(h, w) == 32 &&
           cout % 16 == 0 && c1 > 0 && c1 % 16 == 0 && c1 <= cout &&
           sp_groupnorm_bf16_supported(c1, cout - c1, groups) &&
           conv_parts(static_cast<int>(n), cin, cout, h, w) == 1 &&
           n * h * (int64_t)w * std::max(cin, cout) < (int64_t(1) << 40);
}

// workspace bytes (fp32): per-tile sums [n][tiles][2][cout] + coefficients [4][n][cout] + [3][n][cout]
int64_t sp_conv3x3_bf16_gnvjp_workspace(int64_t n, int32_t cout, int32_t h, int32_t w) {
    return 4 * (n * gnv_tiles(h, w) * 2 * (int64_t)cout + 7 * n * (int64_t)cout);
}

// dz = conv3x3 input VJP of dy (the conv's flipped / transposed weight pack wp, dy in in_layout as
// sp_conv3x3_bf16_ex, cin = dy's channels, cout = dz's), then dx1 / dx2 = the input VJP of
// sp_groupnorm_bf16_fwd over cat(x1, x2) (c1 + c2 = cout channels) at dz, + the addends — as
// sp_conv3x3_bf16_ex followed by sp_groupnorm_bf16_bwd_ex, except that the GroupNorm VJP's sums
// come from the conv's epilogue (per 512-pixel tile, fixed order) instead of a pass that reads dz
// and x again.  dz: a caller buffer [n][h][w][cout] (written, then read by the apply pass).
int sp_conv3x3_bf16_gnvjp(const void* dy, int32_t in_layout, const void* wp, int64_t n, int32_t cin, int32_t cout,
                          int32_t h, int32_t w, void* dz, const void* x1, const void* x2, int32_t c1,
                          const float* chan_bias, const float* gamma, const float* beta, const float* stats,
                          int32_t groups, int32_t act, void* dx1, void* dx2, int32_t dx_layout, const void* add1,
                          const void* add2, const void* add1b, void* ws, int64_t ws_bytes, sp_stream_t stream) {
    if (!dy || !wp || !dz || !x1 || !stats || !dx1 || !ws || (in_layout != 0 && in_layout != 1) ||
        !sp_conv3x3_bf16_gnvjp_supported(n, cin, cout, h, w, c1, groups))
        return SP_EINVAL;
    const int c2 = cout - c1;
    if ((c2 && (!x2 || !dx2)) || (dx_layout != 0 && (dx_layout != 1 || c2)) ||
        ws_bytes < sp_conv3x3_bf16_gnvjp_workspace(n, cout, h, w))
        return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t hw = (int64_t)h * w, nc = n * (int64_t)cout;
    const int tiles = static_cast<int>(gnv_tiles(h, w));
    float* part = static_cast<float*>(ws);
    float* co = part + n * tiles * 2 * (int64_t)cout;
    float* co2 = co + 4 * nc;
    const u16* a = static_cast<const u16*>(x1);
    const u16* b = static_cast<const u16*>(x2);
    const u16* d = static_cast<const u16*>(dz);
    launch(0, k_gnb_coefs, dim3(static_cast<unsigned>((nc + kBlock - 1) / kBlock)), dim3(kBlock), s, stats, chan_bias,
           gamma, beta, static_cast<int>(n), static_cast<int>(cout), groups, co);
    ConvGn gn{a, b, c1, act ? 1 : 0, co, gamma, part};
    const int ni = static_cast<int>(n);
    if (in_layout)
        conv_bf16_launch<32, false, true, false, true>(static_cast<const u16*>(dy), static_cast<const u16*>(wp), nullptr,
                                                       nullptr, ni, cin, cout, h, w, static_cast<u16*>(dz), s, nullptr,
                                                       1, ConvSc{}, gn);
    else
        conv_bf16_launch<32, false, false, false, true>(static_cast<const u16*>(dy), static_cast<const u16*>(wp),
                                                        nullptr, nullptr, ni, cin, cout, h, w, static_cast<u16*>(dz), s,
                                                        nullptr, 1, ConvSc{}, gn);
    launch(0, k_gnb_final_bwd, dim3(groups, static_cast<unsigned>(n)), dim3(64), s, static_cast<const float*>(part),
           tiles, hw, static_cast<int>(cout), groups, stats, gamma, static_cast<const float*>(co), co2);
    const GnbGeo g = gnb_geo(n, cout, hw);
    const dim3 grid(g.chunks, static_cast<unsigned>(n));
    if (act)
        launch(0, k_gnb_bwd_apply<true>, grid, dim3(kBlock), s, d, a, b, c1, c2, static_cast<const float*>(co),
               static_cast<const float*>(co2), hw, g.chunk_px, static_cast<u16*>(dx1), static_cast<u16*>(dx2),
               static_cast<const u16*>(add1), static_cast<const u16*>(add2), static_cast<const u16*>(add1b),
               static_cast<int>(dx_layout));
    else
        launch(0, k_gnb_bwd_apply<false>, grid, dim3(kBlock), s, d, a, b, c1, c2, static_cast<const float*>(co),
               static_cast<const float*>(co2), hw, g.chunk_px, static_cast<u16*>(dx1), static_cast<u16*>(dx2),
               static_cast<const u16*>(add1), static_cast<const u16*>(add2), static_cast<const u16*>(add1b),
               static_cast<int>(dx_layout));
    return check_launch("sp_conv3x3_bf16_gnvjp");
}

// y = conv3x3(x) + bias (+ res) as sp_conv3x3_bf16_ex, then z = act(GroupNorm(y + chan_bias) gamma + beta)
// as sp_groupnorm_bf16_fwd_ex (z_layout, stats [mean | rstd]) — with the GroupNorm's moments taken in
// the conv's epilogue per 512-pixel tile, shifted by the tile's first pixel (no pass re-reading y).
int sp_conv3x3_bf16_gn_supported(int64_t n, int32_t cin, int32_t cout, int32_t h, int32_t w, int32_t groups) {
    return n > 0 && n <= 65535 && sp_conv3x3_bf16_supported(cin, cout, h, w) && conv_tc(h, w) == 32 &&
           cout % 16 == 0 && sp_groupnorm_bf16_supported(cout, 0, groups) &&
           conv_parts(static_cast<int>(n), cin, cout, h, w) == 1 &&
           n * h * (int64_t)w * std::max(cin, cout) < (int64_t(1) << 40);
}

// workspace bytes (fp32): per-tile moments [n][tiles][3][cout] + coefficients [2][n][cout]
int64_t sp_conv3x3_bf16_gn_workspace(int64_t n, int32_t cout, int32_t h, int32_t w) {
    return 4 * (n * gnv_tiles(h, w) * 3 * (int64_t)cout + 2 * n * (int64_t)cout);
}

int sp_conv3x3_bf16_gn(const void* x, int32_t in_layout, const void* wp, const float* bias, const void* res,
                       int64_t n, int32_t cin, int32_t cout, int32_t h, int32_t w, void* y, const float* chan_bias,
                       const float* gamma, const float* beta, int32_t groups, float eps, int32_t act, void* z,
                       int32_t z_layout, float* stats, void* ws, int64_t ws_bytes, sp_stream_t stream) {
    if (!x || !wp || !y || !z || !stats || !ws || (in_layout != 0 && in_layout != 1) || (z_layout != 0 && z_layout != 1) ||
        !sp_conv3x3_bf16_gn_supported(n, cin, cout, h, w, groups) || ws_bytes < sp_conv3x3_bf16_gn_workspace(n, cout, h, w))
        return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t hw = (int64_t)h * w, nc = n * (int64_t)cout;
    const int tiles = static_cast<int>(gnv_tiles(h, w));
    float* part = static_cast<float*>(ws);
    float* co = part + n * tiles * 3 * (int64_t)cout;
    ConvGn gn{nullptr, nullptr, cout, act ? 1 : 0, chan_bias, gamma, part};
    const int ni = static_cast<int>(n);
    const u16* xx = static_cast<const u16*>(x);
    const u16* ww = static_cast<const u16*>(wp);
    const u16* rr = static_cast<const u16*>(res);
    u16* yy = static_cast<u16*>(y);
    if (in_layout)
        conv_bf16_launch<32, false, true, false, false, true>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s, nullptr, 1,
                                                              ConvSc{}, gn);
    else
        conv_bf16_launch<32, false, false, false, false, true>(xx, ww, bias, rr, ni, cin, cout, h, w, yy, s, nullptr, 1,
                                                               ConvSc{}, gn);
    launch(0, k_gnb_final_fwd_tiles, dim3(groups, static_cast<unsigned>(n)), dim3(64), s,
           static_cast<const float*>(part), tiles, static_cast<int64_t>(512), hw, static_cast<int>(cout), groups, eps,
           chan_bias, gamma, beta, stats, co);
    (void)nc;
    const GnbGeo g = gnb_geo(n, cout, hw);
    const dim3 grid(g.chunks, static_cast<unsigned>(n));
    if (act)
        launch(0, k_gnb_apply<true>, grid, dim3(kBlock), s, static_cast<const u16*>(yy), static_cast<const u16*>(nullptr),
               static_cast<int>(cout), 0, static_cast<const float*>(co), hw, g.chunk_px, static_cast<u16*>(z),
               static_cast<int>(z_layout));
    else
        launch(0, k_gnb_apply<false>, grid, dim3(kBlock), s, static_cast<const u16*>(yy), static_cast<const u16*>(nullptr),
               static_cast<int>(cout), 0, static_cast<const float*>(co), hw, g.chunk_px, static_cast<u16*>(z),
               static_cast<int>(z_layout));
    return check_launch("sp_conv3x3_bf16_gn");
}

// ---- attention ------------------------------------------------------------------------------

int sp_attention_bf16_supported(int64_t batch, int32_t heads, int64_t n, int64_t m, int32_t d) {
    if (batch <= 0 || heads <= 0 || batch * heads > 65535 || n <= 0 || m <= 0 || n > (int64_t(1) << 24) ||
        m > (int64_t(1) << 24))
        return 0;
    return d == 40 || d == 64 || d == 80 || d == 160;
}

// out[b][i][h d .. h d + d) = softmax(q k^T scale) v for head h: q rows of stride rsq
// ([batch][n][rsq]), k / v rows of stride rskv ([batch or 1 (kv_shared)][m][rskv]), out rows of
// stride ro; bf16 in and out, lse [batch heads][n] fp32 (natural log).  Pointers at head 0.
int sp_attention_bf16_fwd(const void* q, const void* k, const void* v, int64_t batch, int32_t heads, int64_t n,
                          int64_t m, int32_t d, int32_t rsq, int32_t rskv, int32_t kv_shared, int32_t ro, float scale,
                          void* out, float* lse, sp_stream_t stream) {
    if (!q || !k || !v || !out || !lse || !sp_attention_bf16_supported(batch, heads, n, m, d)) return SP_EINVAL;
    if (rsq < heads * d || rskv < heads * d || ro < heads * d || rsq % 8 || rskv % 8 || ro % 4) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const u16* qq = static_cast<const u16*>(q);
    const u16* kk = static_cast<const u16*>(k);
    const u16* vv = static_cast<const u16*>(v);
    u16* oo = static_cast<u16*>(out);
    switch (d) {
        case 40: attnb_launch<40>(qq, kk, vv, batch, heads, n, m, rsq, rskv, kv_shared, ro, scale, oo, lse, s); break;
        case 64: attnb_launch<64>(qq, kk, vv, batch, heads, n, m, rsq, rskv, kv_shared, ro, scale, oo, lse, s); break;
        case 80: attnb_launch<80>(qq, kk, vv, batch, heads, n, m, rsq, rskv, kv_shared, ro, scale, oo, lse, s); break;
        default: attnb_launch<160>(qq, kk, vv, batch, heads, n, m, rsq, rskv, kv_shared, ro, scale, oo, lse, s); break;
    }
    return check_launch("sp_attention_bf16_fwd");
}

// VJP of sp_attention_bf16_fwd given its output and lse: delta [batch heads][n] fp32 (caller's
// scratch); dq rows of stride rdq ([batch][n][rdq]); dk / dv (self-attention only: m == n, one K/V
// per sample, rsq == rskv) rows of stride rdkv, or NULL (cross-attention: the context is constant).
int sp_attention_bf16_bwd_supported(int64_t batch, int32_t heads, int64_t n, int64_t m, int32_t d) {
    return sp_attention_bf16_supported(batch, heads, n, m, d) && (d == 40 || d == 64 || d == 80);
}

int sp_attention_bf16_bwd(const void* q, const void* k, const void* v, const void* out, const void* dout,
                          const float* lse, int64_t batch, int32_t heads, int64_t n, int64_t m, int32_t d,
                          int32_t rsq, int32_t rskv, int32_t kv_shared, int32_t ro, int32_t rdq, int32_t rdkv,
                          float scale, float* delta, void* dq, void* dk, void* dv, sp_stream_t stream) {
    if (!q || !k || !v || !out || !dout || !lse || !delta || !sp_attention_bf16_bwd_supported(batch, heads, n, m, d))
        return SP_EINVAL;
    if (rsq < heads * d || rskv < heads * d || ro < heads * d || rsq % 8 || rskv % 8 || ro % 8 || rdq % 4 || rdkv % 4)
        return SP_EINVAL;
    if ((dk || dv) && (!dk || !dv || m != n || kv_shared || rsq != rskv || rdkv < heads * d)) return SP_EINVAL;
    if (dq && rdq < heads * d) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const u16 *qq = static_cast<const u16*>(q), *kk = static_cast<const u16*>(k), *vv = static_cast<const u16*>(v);
    const u16 *oo = static_cast<const u16*>(out), *dd = static_cast<const u16*>(dout);
    u16 *a = static_cast<u16*>(dq), *bb = static_cast<u16*>(dk), *c = static_cast<u16*>(dv);
    switch (d) {
        case 40: attnb_bwd_launch<40>(qq, kk, vv, oo, dd, lse, batch, heads, n, m, rsq, rskv, kv_shared, ro, rdq, rdkv, scale, delta, a, bb, c, s); break;
        case 64: attnb_bwd_launch<64>(qq, kk, vv, oo, dd, lse, batch, heads, n, m, rsq, rskv, kv_shared, ro, rdq, rdkv, scale, delta, a, bb, c, s); break;
        default: attnb_bwd_launch<80>(qq, kk, vv, oo, dd, lse, batch, heads, n, m, rsq, rskv, kv_shared, ro, rdq, rdkv, scale, delta, a, bb, c, s); break;
    }
    return check_launch("sp_attention_bf16_bwd");
}

}  // extern "C"

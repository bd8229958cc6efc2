// 1x1 convolution (per-pixel GEMM) Y[n][co][p] = sum_k W[co][k] X[n][k][p] on bf16 MFMAs over
// exact three-term bf16 splits of the fp32 operands (six partial
// products, fp32 accumulation in two accumulators: the leading product and the small ones;
// error half of an fp32 GEMM's, tests/test_gemm_x6_gpu.py).
//
// The UNet's ResnetBlock conv_shortcut (diffusers ResnetBlock2D) over
// cat(x1, x2) in the up path: forward W [x1; x2] (+ its bias folded elsewhere), input VJP
// [W1^T; W2^T] dy into two outputs.  Both sides of the concatenation are addressed in place:
// K blocks of 16 channels come from X1 or X2, output blocks of 32 channels go to Y1 or Y2.
//
// Why bf16 here: with K = 128-256 the fp32-MFMA GEMM is compute-bound (43 FLOP/B against a
// 20 FLOP/B ridge); at the bf16 rate / 6 it is HBM-bound, so one pass over x and y is the
// cost (W, 100-200 KB of split terms, stays in L2).
//
// Tile: workgroup = 128 output channels x 256 pixels of one image; its 8 waves (two per SIMD)
// each own channels 64 (w & 1) .. +63 and pixels 64 (w >> 1) .. +63 (2 x 2 tiles of 32 x 32;
// pixel tile b holds the wave's pixels of parity b).  k-step = 16 input channels: raw fp32 X
// (16 ch x 256 px) comes by direct global->LDS loads six k-steps ahead (a 7-slot ring, 112 KB),
// W's packed fragments (12 KB) two ahead; each wave reads its fp32 X fragments (a ds_read_b64
// = two adjacent pixels, one per pixel tile) and splits them into the three bf16 terms in
// registers right before its MFMAs.

#define SP_TU 11  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

#include <algorithm>
#include <type_traits>

namespace sp {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned uvec4 __attribute__((ext_vector_type(4)));
typedef unsigned uvec2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void_g;

#ifndef G6_SCHED
#define G6_SCHED 1  // hand-ordered issue within the k-step (see k_gemm_x6)
#endif
#ifndef G6_EXP
#define G6_EXP 0  // diagnostics only (wrong results, timing): 1 no MFMAs, 2 no split, 3 no loads,
                  // 4 no output stores, 5 X loads from one cached 2 KB (no X stream from HBM),
                  // 6 MFMAs only (no loads, no split, no stores), 7 each 32x32x16 MFMA replaced by
                  // two 16x16x32 ones on the same operands (the same MACs; the clock the chip holds),
                  // 8 no k-step barrier (the waves drift: races on the LDS ring; timing only)
#endif
#define G6_NO_SPLIT (G6_EXP == 2 || G6_EXP == 6)
#define G6_NO_LOADS (G6_EXP == 3 || G6_EXP == 6)
#define G6_NO_STORES (G6_EXP == 4 || G6_EXP == 6)
#ifndef G6_W4
#define G6_W4 0  // 4 waves (one per SIMD), each 128 channels x 64 pixels, instead of 8 x (64 x 64)
#endif
constexpr int G6_WAVES = G6_W4 ? 4 : 8;
constexpr int G6_NA = G6_W4 ? 4 : 2;        // 32-channel blocks per wave
constexpr int G6_XP = 16 / G6_WAVES;        // X pieces (1 KB) per wave and k-step
constexpr int G6_CO = 128;     // output channels per workgroup
constexpr int G6_PX = 256;     // pixels per workgroup
constexpr int G6_KC = 16;      // input channels per k-step
constexpr int G6_WB = 4 * 3 * 64 * 16;        // bytes of W fragments per k-step (12 KB)
#ifndef G6_NX_SLOTS
#define G6_NX_SLOTS 6
#endif
#ifndef G6_NW_SLOTS
#define G6_NW_SLOTS 4
#endif
constexpr int G6_NX = G6_NX_SLOTS;  // raw X ring slots: X of k-step j + 5 loads during step j
constexpr int G6_NW = G6_NW_SLOTS;  // W ring slots: W of k-step j + 3 loads during step j

struct G6Geom {
    const float* x1;
    const float* x2;      // nullable: channels c1 .. c1 + c2 - 1
    const unsigned short* wp;
    float* y1;
    float* y2;            // nullable: output channels o1 .. o1 + o2 - 1
    const float* bias;    // nullable, per output channel (o1 + o2)
    const float* res;     // nullable, shaped like y1 (o2 == 0 only)
    int c1, c2, o1, o2, hw;
    int ntiles, cob, ptiles, nsteps;  // ntiles: work items = output tiles x ksplit
    int tokens;           // token-major operands: rows of x1 / y1 (images x hw)
    // split-K (under-filled launches): item (tile, kh) runs k-steps kh kper .. + kper - 1 and
    // stores its partial product (no bias, no residual) to ws + kh ws_stride, laid out as a
    // single output of o1 + o2 channels; k_g6_split_reduce adds the parts.  ksplit 1: ws NULL.
    int ksplit, kper;
    float* ws;
    int64_t ws_stride;
    // token-major operands (k_gemm_x6<LTM, STM>, nn.Linear on [tokens][features]): x1 is
    // [tokens][c1] and / or y1 [tokens][o1] with o1 % 32 (W's rows padded to 128 with zeros),
    // one input and output
};

__device__ __forceinline__ void g6_split(float v, unsigned& h, unsigned& m, unsigned& l) {
    const unsigned vb = __float_as_uint(v);
    h = vb & 0xffff0000u;
    const float r = v - __uint_as_float(h);
    m = __float_as_uint(r) & 0xffff0000u;
    l = __float_as_uint(r - __uint_as_float(m));
}
__device__ __forceinline__ unsigned g6_pack(unsigned a, unsigned b) {
    return __builtin_amdgcn_perm(b, a, 0x07060302u);
}
__device__ __forceinline__ f32x16 g6_mfma(uvec4 a, uvec4 b, f32x16 c) {
#if G6_EXP == 7
    f32x4 c0 = {c[0], c[1], c[2], c[3]}, c1 = {c[4], c[5], c[6], c[7]};
    c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b),
                                                 c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, b), __builtin_bit_cast(bf16x8, a),
                                                 c1, 0, 0, 0);
    c[0] = c0[0], c[1] = c0[1], c[2] = c0[2], c[3] = c0[3], c[4] = c1[0], c[5] = c1[1], c[6] = c1[2], c[7] = c1[3];
    return c;
#else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
#endif
}

// direct global->LDS load (64 lanes x 16 B to lds .. lds + 1 KB) written as inline asm: the
// compiler's wait insertion does not see it, so it does not drain it with vmcnt(0) before every
// later LDS read it cannot prove disjoint; the kernel waits for these loads itself (counted vmcnt)
// (lds: the LDS byte address, formed once per kernel from the __shared__ array — a generic
// pointer cast here costs a null check per load, and one form of it trips a backend bug)
__device__ __forceinline__ void g6_lds_dma(__amdgpu_buffer_rsrc_t rs, unsigned la, int voff, int soff) {
    unsigned keep;  // m0 is reserved to the compiler: saved and restored around the load
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "s"(__builtin_amdgcn_readfirstlane(la)), "v"(voff), "s"(rs), "s"(soff)
                 : "memory");
}

// gfx9 s_waitcnt immediate: vmcnt <= n (6 bits), lgkmcnt / expcnt not waited for
constexpr int g6_vmcnt(int n) { return (n & 0xF) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8); }

// raw X of one k-step -> LDS ring slot ([16 ch][256 px] fp32): 16 direct 1-KB loads, 2 per wave
// (channel 2 wv + i, lane l: pixels 4l .. 4l + 3)
// (xb1 / xb2: image n's planes of x1 / x2, formed once per tile; the channel is a scalar
// offset, so a load costs a multiply-add, not a 64-bit channel base: the launcher guarantees
// k hw 4 < 2^31, and hw % 256 == 0 keeps every load inside its plane)
__device__ __forceinline__ void g6_dma_x(const G6Geom& g, const float* xb1, const float* xb2,
                                         int p0, int kstep, int wv, int lane, unsigned slot) {
    const int k0 = kstep * G6_KC;
#pragma unroll
    for (int i = 0; i < G6_XP; ++i) {
        const int c = k0 + G6_XP * wv + i;
        const bool second = c >= g.c1;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(second ? xb2 : xb1), (short)0,
                                                          (second ? g.c2 : g.c1) * g.hw * 4, 0x00020000);
        g6_lds_dma(rs, slot + (G6_XP * wv + i) * 1024, lane * 16, ((second ? c - g.c1 : c) * g.hw + p0) * 4);
    }
}

// token-major X (nn.Linear input [tokens][c1]) -> LDS slot [256 tokens][16 ch] fp32: load i of
// wave wv covers tokens p0 + 16 (2 wv + i) .. +15, lane l: token + (l >> 2), channels 4 (l & 3) .. +3
__device__ __forceinline__ void g6_dma_x_tm(const G6Geom& g, int p0, int kstep, int wv, int lane,
                                            unsigned slot) {
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.x1), (short)0, g.tokens * g.c1 * 4,
                                                      0x00020000);
    const int vo = ((lane >> 2) * g.c1 + 4 * (lane & 3)) * 4;
#pragma unroll
    for (int i = 0; i < G6_XP; ++i) {
        const int t0 = p0 + 16 * (G6_XP * wv + i);
        g6_lds_dma(rs, slot + (G6_XP * wv + i) * 1024, vo, (t0 * g.c1 + kstep * G6_KC) * 4);
    }
}

// W fragments of one k-step (12 KB contiguous in the packed layout): 12 direct 1-KB loads, two
// by each of waves 0-3 and one by each of waves 4-7
__device__ __forceinline__ void g6_dma_w(__amdgpu_buffer_rsrc_t wrs, int stage, int wv, int lane,
                                         unsigned wb) {
#pragma unroll
    for (int i = 0; i < (12 + G6_WAVES - 1) / G6_WAVES; ++i) {
        const int chunk = wv + G6_WAVES * i;
        if (chunk < 12)
            g6_lds_dma(wrs, wb + chunk * 1024, lane * 16, stage * G6_WB + chunk * 1024);
    }
}
// vm ops a wave issues per k-step (8 waves: 2 X + 2 or 1 W; 4 waves: 4 X + 3 W)
__device__ __forceinline__ int g6_dma_per_wave(int wv) { return G6_W4 ? 7 : wv < 4 ? 4 : 3; }
// loads younger than W(j + 2) at the end of step j: X(j + 4), W(j + 3), X(j + 5)
constexpr int G6_YOUNG_A = G6_W4 ? 11 : 6;  // waves with the larger W share (all of them at 4 waves)
constexpr int G6_YOUNG_B = G6_W4 ? 11 : 5;

// eight fp32 values (channels c0 .. c0 + 7 of one pixel) -> the lane's three bf16 term fragments
__device__ __forceinline__ void g6_split8(const float (&v)[8], uvec4 (&t)[3]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#if G6_NO_SPLIT
        const unsigned a = __float_as_uint(v[2 * q]), b = __float_as_uint(v[2 * q + 1]);
        t[0][q] = t[1][q] = t[2][q] = g6_pack(a, b);
#else
        unsigned h0, m0, l0, h1, m1, l1;
        g6_split(v[2 * q], h0, m0, l0);
        g6_split(v[2 * q + 1], h1, m1, l1);
        t[0][q] = g6_pack(h0, h1);
        t[1][q] = g6_pack(m0, m1);
        t[2][q] = g6_pack(l0, l1);
#endif
    }
}

// The lane's raw X of one k-step from an NCHW slot ([16 ch][256 px] fp32): channels
// 8 (lane >> 5) .. +7 of the wave's pixels 64 pq + 2 (lane & 31) + b, b = 0, 1 (pixel tile b)
// — one ds_read_b64 per channel gives both tiles' pixel
__device__ __forceinline__ void g6_raw_x(const unsigned char* raw, int pq, int lane, float (&v)[2][8]) {
    const unsigned char* p = raw + 8 * (lane >> 5) * 1024 + (pq * 64 + 2 * (lane & 31)) * 4;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const f32x2 t = *reinterpret_cast<const f32x2*>(p + i * 1024);
        v[0][i] = t.x, v[1][i] = t.y;
    }
}

// the same from a token-major slot ([256 tokens][16 ch] fp32): 32 contiguous bytes per token;
// PAR: tile b holds the tokens of parity b (as above), else tokens 32 b .. 32 b + 31 (a 64-byte
// lane stride: half the LDS bank conflicts of the parity order's 128 bytes)
template <bool PAR>
__device__ __forceinline__ void g6_raw_x_tm(const unsigned char* raw, int pq, int lane, float (&v)[2][8]) {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int tok = PAR ? 2 * (lane & 31) + b : 32 * b + (lane & 31);
        const unsigned char* p = raw + (pq * 64 + tok) * 64 + (lane >> 5) * 32;
        const uvec4 x = *reinterpret_cast<const uvec4*>(p), y = *reinterpret_cast<const uvec4*>(p + 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[b][i] = __uint_as_float(x[i]), v[b][4 + i] = __uint_as_float(y[i]);
    }
}

struct G6Pos { int n, p0, cb, kh; };
#ifndef G6_DESC
#define G6_DESC 0  // 1: per-tile X load descriptors advanced per k-step (round-6 A/B; else formed per load)
#endif
struct XDesc { int so, rem; };
// SPLIT: the split-K kernels (a compile-time variant: the unsplit ones keep their registers)
template <bool SPLIT>
__device__ __forceinline__ G6Pos g6_pos(const G6Geom& g, int t) {
    // XCD-aware: the output-channel blocks of one pixel tile on one XCD (shared X lines)
    const int lb0 = (g.ntiles & 7) ? t : (t & 7) * (g.ntiles >> 3) + (t >> 3);
    const int kh = SPLIT ? lb0 % g.ksplit : 0, lb = SPLIT ? lb0 / g.ksplit : lb0;
    const int cb = lb % g.cob, rest = lb / g.cob;
    const int n = rest / g.ptiles;
    // the item inside the grid's work, its pixels inside the plane (or the token rows), its
    // k-steps inside K
    SP_DCHECK(t >= 0 && t < g.ntiles && lb0 < g.ntiles && cb * G6_CO < g.o1 + g.o2 + G6_CO &&
              (rest - n * g.ptiles + 1) * G6_PX <= (g.tokens ? g.tokens : g.hw) &&
              (!SPLIT || (kh + 1) * g.kper <= g.nsteps));
    return G6Pos{n, (rest - n * g.ptiles) * G6_PX, cb, kh};
}

// epilogue: register q of tile (a, b) = channel 32 (2 ch + a) + (q&3) + 8(q>>2) + 4(lane>>5),
// pixel px0 + 2 (lane & 31) + b of image n (PAR; px0: the wave's first pixel in the plane), so
// both tiles' registers q form one 8-byte store — else pixel px0 + 32 b + (lane & 31), one
// 4-byte store each; bias and residual added, the 32-channel block to y1 or y2.  Returns the
// stores issued (the caller's wait count for the next k-step).
template <bool PAR>
__device__ __forceinline__ int g6_epilogue(const G6Geom& g, int n, int cb, int px0, int ch, int lane,
                                           const f32x16 (&acc)[G6_NA][2], const f32x16 (&acs)[G6_NA][2]) {
    int nst = 0;
    const int vo = (px0 + 2 * (lane & 31)) * 4;
#pragma unroll
    for (int a = 0; a < G6_NA; ++a) {
        const int co0 = cb * G6_CO + 32 * (G6_NA * ch + a);  // first channel of the 32-block
        if (co0 >= g.o1 + g.o2) continue;  // padded rows of W (uniform)
        const bool second = co0 >= g.o1;
        float* yb = second ? g.y2 + ((int64_t)n * g.o2 + (co0 - g.o1)) * g.hw
                           : g.y1 + ((int64_t)n * g.o1 + co0) * g.hw;
        const auto ors = __builtin_amdgcn_make_buffer_rsrc(yb, (short)0, 32 * g.hw * 4, 0x00020000);
        const auto rrs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(g.res ? g.res + ((int64_t)n * g.o1 + co0) * g.hw : g.y1), (short)0,
            g.res ? 32 * g.hw * 4 : 0, 0x00020000);
        const auto brs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.bias ? g.bias + co0 : g.y1),
                                                           (short)0, g.bias ? 32 * 4 : 0, 0x00020000);
        const float bl = g.bias ? __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(brs, (lane & 31) * 4, 0, 0))
                                : 0.f;
        if constexpr (!PAR) {
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const int vb = (px0 + 32 * b + (lane & 31)) * 4;
                float rs[16];
#pragma unroll
                for (int q = 0; q < 16; ++q) rs[q] = 0.f;
                if (g.res) {
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int cc = (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
                        rs[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rrs, vb + cc * g.hw * 4, 0, 0));
                    }
                }
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int c = (q & 3) + 8 * (q >> 2);
                    const float b0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, bl), c));
                    const float b1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, bl), c + 4));
                    const float y = (acc[a][b][q] + acs[a][b][q]) + ((lane >> 5) ? b1 : b0) + rs[q];
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y), ors, vb + (c + 4 * (lane >> 5)) * g.hw * 4, 0, 0);
                }
                nst += 16;
                __builtin_amdgcn_sched_barrier(0);
            }
            continue;
        }
        f32x2 rv[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) rv[q] = f32x2{0.f, 0.f};
        if (g.res) {  // all 16 loads first (one wait), not a load-use pair per register
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int cc = (q & 3) + 8 * (q >> 2) + 4 * (lane >> 5);
                rv[q] = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rrs, vo + cc * g.hw * 4, 0, 0));
            }
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int c = (q & 3) + 8 * (q >> 2);
            const float b0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, bl), c));
            const float b1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, bl), c + 4));
            const float bv = (lane >> 5) ? b1 : b0;
            const int cc = c + 4 * (lane >> 5);
            const f32x2 y = {(acc[a][0][q] + acs[a][0][q]) + bv + rv[q].x, (acc[a][1][q] + acs[a][1][q]) + bv + rv[q].y};
#if G6_NO_STORES
            if (g.hw >= 0) continue;  // never true at run time: the stores are skipped, all math kept
#endif
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(uvec2, y), ors, vo + cc * g.hw * 4, 0, 0);
        }
        nst += 16;
        __builtin_amdgcn_sched_barrier(0);
    }
    return nst;
}

// token-major epilogue: the MFMA ran with X as A and W as B, so register q of tile (a, b) is token
// p0 + 64 pq + 2 r + b (PAR, else + 32 b + r), r = (q&3) + 8(q>>2) + 4(lane>>5), and output
// feature o0 + (lane & 31): each register row is 32 consecutive features of one token (128
// contiguous bytes).  Returns the stores issued.
template <bool PAR>
__device__ __forceinline__ int g6_epilogue_tm(const G6Geom& g, const G6Pos& ps, int ch, int pq, int lane,
                                               const f32x16 (&acc)[G6_NA][2], const f32x16 (&acs)[G6_NA][2]) {
    const auto ors = __builtin_amdgcn_make_buffer_rsrc(g.y1, (short)0, g.tokens * g.o1 * 4, 0x00020000);
    const auto rrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.res ? g.res : g.y1), (short)0,
                                                       g.res ? g.tokens * g.o1 * 4 : 0, 0x00020000);
    const int tok0 = ps.n * g.hw + ps.p0;  // first token row of the tile (image n's plane)
    int nst = 0;
#pragma unroll
    for (int a = 0; a < G6_NA; ++a) {
        const int o = ps.cb * G6_CO + 32 * (G6_NA * ch + a) + (lane & 31);
        if (ps.cb * G6_CO + 32 * (G6_NA * ch + a) >= g.o1) continue;  // padded rows of W (uniform)
        const float bv = g.bias ? g.bias[o] : 0.f;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            constexpr int RS = PAR ? 2 : 1;  // token stride of the register rows
            const int t0 = tok0 + pq * 64 + (PAR ? b : 32 * b) + RS * 4 * (lane >> 5);  // r = 4 (lane >> 5)
            float rv[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) rv[q] = 0.f;
            if (g.res) {
#pragma unroll
                for (int q = 0; q < 16; ++q)
                    rv[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                        rrs, ((t0 + RS * ((q & 3) + 8 * (q >> 2))) * g.o1 + o) * 4, 0, 0));
            }
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const float y = (acc[a][b][q] + acs[a][b][q]) + bv + rv[q];
#if G6_NO_STORES
                if (g.hw >= 0) continue;  // never true at run time: the stores are skipped, all math kept
#endif
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(y), ors,
                                                      ((t0 + RS * ((q & 3) + 8 * (q >> 2))) * g.o1 + o) * 4, 0, 0);
            }
            nst += 16;
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    return nst;
}

// The workgroup walks a flat stream of k-steps j = (its tile j / nsteps, step j % nsteps): the
// loads of X(j + 5) and W(j + 3) run during the MFMAs of step j, across tile boundaries (raw X
// in a 6-slot and W in a 4-slot LDS ring filled by direct loads), and each wave reads its
// fragments of step j + 1 from LDS into registers during them too: the workgroup's barrier
// aligns all eight waves' phases, so LDS reads issued after it would leave the MFMAs idle.
constexpr int G6_THREADS = 64 * G6_WAVES;

#ifndef G6_STAGGER
#define G6_STAGGER 1  // the second wave of each SIMD issues its loads half-way through its MFMAs
#endif
#ifndef G6_STORE_CREDIT
#define G6_STORE_CREDIT 1  // the first k-step after an epilogue does not wait for its stores
#endif

// LTM / STM: X read token-major ([tokens][k]) / Y written token-major ([tokens][m]); else the
// per-image channel-major planes ([n][k][hw] / [n][m][hw]).  Tokens of image n are rows
// n hw .. n hw + hw - 1.
typedef unsigned char G6XSlot[G6_KC * G6_PX * 4];
typedef unsigned char G6WSlot[G6_WB];

// LATE: this wave issues its loads half-way through its MFMAs (the second wave of each SIMD)
template <bool LTM, bool STM, bool LATE, bool SPLIT>
__device__ __forceinline__ void g6_body(const G6Geom& g, G6XSlot* xraw, G6WSlot* wl, int wv) {
    const int kper = SPLIT ? g.kper : g.nsteps;  // k-steps per work item
    const int tid = threadIdx.x, lane = tid & 63;
    // 8 waves: 64 output channels (block ch) x 64 pixels (quarter pq); 4 waves: 128 x 64
    const int ch = G6_W4 ? 0 : wv & 1, pq = G6_W4 ? wv : wv >> 1;
    const auto wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned short*>(g.wp), (short)0,
                                                       g.cob * g.nsteps * G6_WB, 0x00020000);
    const unsigned xraw_lds = static_cast<unsigned>(reinterpret_cast<size_t>((lds_void_g*)&xraw[0][0]));
    const unsigned wl_lds = static_cast<unsigned>(reinterpret_cast<size_t>((lds_void_g*)&wl[0][0]));
    const int G = gridDim.x, b0 = blockIdx.x;
    const int ntile_wg = (g.ntiles - b0 + G - 1) / G;
    const int J = ntile_wg * kper;
    // two load streams, advanced one k-step at a time (divisions once per tile)
    struct Cursor { int j, tw, s, slot; G6Pos ps; };
    Cursor cx{0, 0, 0, 0, g6_pos<SPLIT>(g, b0)}, cw = cx;
    // the X stream's image bases, renewed when its tile changes
    const float* xb1 = g.x1 + (int64_t)cx.ps.n * g.c1 * g.hw;
    const float* xb2 = g.x2 + (int64_t)cx.ps.n * g.c2 * g.hw;
    auto advance = [&](Cursor& c, int nslots) {
        ++c.j;
        c.slot = c.slot + 1 == nslots ? 0 : c.slot + 1;
        if (++c.s == kper) {
            c.s = 0;
            if (++c.tw < ntile_wg) c.ps = g6_pos<SPLIT>(g, b0 + c.tw * G);
            return true;
        }
        return false;
    };
#if G6_DESC
    // Per-tile load descriptors of the X stream (NCHW X): this wave's load i reads channel
    // 16 ks + G6_XP wv + i at k-step ks, an arithmetic progression — so its buffer resource and
    // byte offset are formed once per tile and then advanced by one k-step's channel stride
    // (one scalar add); `rem` = c1 - channel detects the one step at which the progression
    // crosses from x1 into x2 (c1 % 8 == 0 only: a k-step may straddle the parts).
    XDesc xd[G6_XP];
    auto xdesc_init = [&]() {
        const int ks = SPLIT ? cx.ps.kh * kper : 0;
#pragma unroll
        for (int i = 0; i < G6_XP; ++i) {
            const int c = ks * G6_KC + G6_XP * wv + i;
            const bool second = c >= g.c1;
            xd[i].so = ((second ? c - g.c1 : c) * g.hw + cx.ps.p0) * 4;
            xd[i].rem = g.c1 - c;
        }
    };
    if constexpr (!LTM) xdesc_init();
#endif
    auto dma_x = [&]() {
        if (cx.j < J) {
            const unsigned sl = xraw_lds + cx.slot * (G6_KC * G6_PX * 4);
            const int ks = SPLIT ? cx.ps.kh * kper + cx.s : cx.s;  // the k-step inside K
#if G6_EXP == 5  // diagnostics (wrong results): the same DMA pieces, all from one cached 2 KB
            (void)ks;
            g6_lds_dma(wrs, sl + (2 * wv) * 1024, lane * 16, 0);
            g6_lds_dma(wrs, sl + (2 * wv + 1) * 1024, lane * 16, 1024);
#else
            if constexpr (LTM) {
                g6_dma_x_tm(g, cx.ps.n * g.hw + cx.ps.p0, ks, wv, lane, sl);
            } else {
#if G6_DESC
                (void)ks;
#pragma unroll
                for (int i = 0; i < G6_XP; ++i) {
                    const bool second = xd[i].rem <= 0;
                    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(second ? xb2 : xb1), (short)0,
                                                                      (second ? g.c2 : g.c1) * g.hw * 4, 0x00020000);
                    g6_lds_dma(rs, sl + (G6_XP * wv + i) * 1024, lane * 16, xd[i].so);
                }
#else
                g6_dma_x(g, xb1, xb2, cx.ps.p0, ks, wv, lane, sl);
#endif
            }
#endif
        }
        if (advance(cx, G6_NX) && !LTM) {
            xb1 = g.x1 + (int64_t)cx.ps.n * g.c1 * g.hw;
            xb2 = g.x2 + (int64_t)cx.ps.n * g.c2 * g.hw;
#if G6_DESC
            xdesc_init();
        } else if (!LTM) {
#pragma unroll
            for (int i = 0; i < G6_XP; ++i) {
                xd[i].rem -= G6_KC;
                if (xd[i].rem > 0 || xd[i].rem <= -G6_KC) {
                    xd[i].so += G6_KC * g.hw * 4;
                } else {  // this step's channel is the first of x2 in the progression
                    xd[i].so = (-xd[i].rem * g.hw + cx.ps.p0) * 4;
                }
            }
#endif
        }
    };
    auto dma_w = [&]() {
        if (cw.j < J)
            g6_dma_w(wrs, cw.ps.cb * g.nsteps + (SPLIT ? cw.ps.kh * kper : 0) + cw.s, wv, lane,
                     wl_lds + cw.slot * G6_WB);
        advance(cw, G6_NW);
    };
    // prologue: W 0 .. 2 and X 0 .. 4 in flight, then all landed
    dma_w();
    dma_w();
    dma_w();
#pragma unroll
    for (int i = 0; i < G6_NX - 1; ++i) dma_x();
    __builtin_amdgcn_s_waitcnt(g6_vmcnt(0));
    __builtin_amdgcn_s_barrier();

    const bool four = G6_W4 || g6_dma_per_wave(wv) == 4;  // this wave's W loads per step: 2 (else 1; 3 at 4 waves)
    // two accumulators per tile: the leading product (hi x hi) and the five small terms, so the
    // small terms' fp32 roundings happen at 2^-8 of the result's magnitude (with one
    // accumulator the error grew past an fp32 GEMM's at K = 768)
    f32x16 acc[G6_NA][2], acs[G6_NA][2];
    int j = 0, wslot = 0, xslot = 0;
    int nst = 0;  // stores of the previous tile's epilogue (younger than W(j + 2) at its step 0)
    // step j's W fragments and raw X (read during step j - 1; step 0's here), in two register
    // sets used alternately (A, B) so that no copy moves them from one step to the next
    uvec4 fuA[G6_NA][3], fuB[G6_NA][3];
    float xrA[2][8], xrB[2][8];
    auto read_frags = [&](int ws, int xs, uvec4 (&u)[G6_NA][3], float (&r)[2][8]) {
        if constexpr (!G6_W4) {  // (4 waves: W read at the start of its own step, kstep)
            const uvec4* wq = reinterpret_cast<const uvec4*>(wl[ws]) + lane;
#pragma unroll
            for (int a = 0; a < G6_NA; ++a)
#pragma unroll
                for (int e = 0; e < 3; ++e) u[a][e] = wq[((G6_NA * ch + a) * 3 + e) * 64];
        }
        if constexpr (LTM) g6_raw_x_tm<!LTM>(xraw[xs], pq, lane, r);
        else g6_raw_x(xraw[xs], pq, lane, r);
    };
    read_frags(0, 0, fuA, xrA);
    int s = 0;  // k-step within the tile
    // One k-step: the next step's fragment reads and this step's split between its MFMAs, then
    // the loads of W(j + 3) and X(j + 5) (their scalar address work overlaps the MFMAs in
    // flight), one barrier.
    auto kstep = [&](const uvec4 (&fu)[G6_NA][3], const float (&xr)[2][8], uvec4 (&fun)[G6_NA][3],
                     float (&xrn)[2][8]) {
        // 4 waves: no second register set for W (a wave's 128 channels x 3 terms = 48 VGPRs);
        // this step's fragments are read first and the MFMAs wait for them in order
        uvec4 fw[G6_NA][3];
        if constexpr (G6_W4) {
            const uvec4* wq = reinterpret_cast<const uvec4*>(wl[wslot]) + lane;
#pragma unroll
            for (int a = 0; a < G6_NA; ++a)
#pragma unroll
                for (int e = 0; e < 3; ++e) fw[a][e] = wq[(a * 3 + e) * 64];
        }
        const uvec4(&fuse)[G6_NA][3] = G6_W4 ? fw : fu;
        wslot = wslot == G6_NW - 1 ? 0 : wslot + 1;
        xslot = xslot == G6_NX - 1 ? 0 : xslot + 1;
        // step j + 1's fragments (in since the last barrier; past the stream's end: unused)
        read_frags(wslot, xslot, fun, xrn);
        // step j's X split into its terms
        uvec4 fv[2][3];
        g6_split8(xr[0], fv[0]);
        g6_split8(xr[1], fv[1]);
        // the six partial products (small terms first) over the 4 independent accumulators,
        // terms [LO, HI) of them, with the split's rest and the next step's fragment reads
        // between the MFMAs
        auto prods = [&](auto lo_c, auto hi_c) {
            constexpr int LO = decltype(lo_c)::value, HI = decltype(hi_c)::value;
            constexpr int TU[6] = {2, 0, 1, 1, 0, 0}, TV[6] = {0, 2, 1, 0, 1, 0};
#if G6_EXP != 1
#pragma unroll
            for (int e = LO; e < HI; ++e)
#pragma unroll
                for (int b = 0; b < 2; ++b)
#pragma unroll
                    for (int a = 0; a < G6_NA; ++a) {
                        if constexpr (STM)  // tokens as the MFMA's rows: features contiguous in C
                            (e == 5 ? acc : acs)[a][b] = g6_mfma(fv[b][TV[e]], fuse[a][TU[e]], (e == 5 ? acc : acs)[a][b]);
                        else
                            (e == 5 ? acc : acs)[a][b] = g6_mfma(fuse[a][TU[e]], fv[b][TV[e]], (e == 5 ? acc : acs)[a][b]);
                    }
#endif
#if G6_SCHED
            if constexpr (G6_W4 && LO == 0) __builtin_amdgcn_sched_group_barrier(0x100, 3 * G6_NA, 0);  // W
            if constexpr (LO == 0) __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);  // the first terms
            // per MFMA: the split's rest (3 VALU at 8 waves, 2 at 4) and one of the next step's
            // fragment reads (W: 3 NA b128; X: 8 b64 or 4 b128 token-major)
            constexpr int MPT = 2 * G6_NA, NV = G6_W4 ? 2 : 3, ND = (G6_W4 ? 0 : 3 * G6_NA) + (LTM ? 4 : 8);
#pragma unroll
            for (int k = MPT * LO; k < MPT * HI; ++k) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
                if (k < ND) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
#endif
        };
        // the loads of W(j + 3) and X(j + 5): their scalar address work runs while MFMAs are in
        // the pipe — after all of this wave's, or (the waves sharing a SIMD with the first four)
        // half-way, so that the two waves of a SIMD never do it at the same time
        auto dma = [&]() {
#if !G6_NO_LOADS
            dma_w();  // step j + 3
            dma_x();  // step j + 5
#endif
        };
        if constexpr (LATE) {
            prods(std::integral_constant<int, 0>{}, std::integral_constant<int, 3>{});
            __builtin_amdgcn_sched_barrier(0);
            dma();
            __builtin_amdgcn_sched_barrier(0);
            prods(std::integral_constant<int, 3>{}, std::integral_constant<int, 6>{});
        } else {
            prods(std::integral_constant<int, 0>{}, std::integral_constant<int, 6>{});
            __builtin_amdgcn_sched_barrier(0);
            dma();
        }
        // one barrier per k-step, behind which X(j + 2) and W(j + 2) are in (read during
        // step j + 1).  Younger than W(j + 2) (issued at step j - 1, after X(j + 2)): X(j + 4),
        // this step's W(j + 3) and X(j + 5) — and at a tile's first step the previous
        // epilogue's stores
        if (j + G6_NX - 1 >= J) __builtin_amdgcn_s_waitcnt(0x0070);  // the stream's tail: vmcnt(0)
#if G6_STORE_CREDIT
        else if (s == 0 && nst == 32) {
            if (four) __builtin_amdgcn_s_waitcnt(g6_vmcnt(G6_YOUNG_A + 32) & ~0x0F00);
            else __builtin_amdgcn_s_waitcnt(g6_vmcnt(G6_YOUNG_B + 32) & ~0x0F00);
        } else if (s == 0 && nst == 16) {
            if (four) __builtin_amdgcn_s_waitcnt(g6_vmcnt(G6_YOUNG_A + 16) & ~0x0F00);
            else __builtin_amdgcn_s_waitcnt(g6_vmcnt(G6_YOUNG_B + 16) & ~0x0F00);
        }
#endif
        else if (four) __builtin_amdgcn_s_waitcnt(g6_vmcnt(G6_YOUNG_A) & ~0x0F00);
        else __builtin_amdgcn_s_waitcnt(g6_vmcnt(G6_YOUNG_B) & ~0x0F00);
#if G6_EXP != 8
        __builtin_amdgcn_s_barrier();
#endif
        ++s, ++j;
    };
    for (int tw = 0; tw < ntile_wg; ++tw) {
#pragma unroll
        for (int a = 0; a < G6_NA; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{}, acs[a][b] = f32x16{};
        s = 0;
        while (s + 1 < kper) {
            kstep(fuA, xrA, fuB, xrB);
            kstep(fuB, xrB, fuA, xrA);
        }
        if (s < kper) {  // odd step count: one more, and set A back to the current step
            kstep(fuA, xrA, fuB, xrB);
#pragma unroll
            for (int a = 0; a < G6_NA; ++a)
#pragma unroll
                for (int e = 0; e < 3; ++e) fuA[a][e] = fuB[a][e];
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int i = 0; i < 8; ++i) xrA[b][i] = xrB[b][i];
        }
        const G6Pos ps = g6_pos<SPLIT>(g, b0 + tw * G);
        // split-K: the part goes to its workspace slice as a single output of all m channels
        G6Geom ge = g;
        if (SPLIT) {
            ge.y1 = g.ws + ps.kh * g.ws_stride;
            ge.y2 = nullptr;
            ge.o1 = g.o1 + g.o2;
            ge.o2 = 0;
            ge.bias = nullptr;
            ge.res = nullptr;
        }
        // tiles hold the pixels of parity b (NCHW X: one ds_read_b64 per channel) or 32 b .. (token
        // X: fewer LDS bank conflicts)
        if constexpr (STM) nst = g6_epilogue_tm<!LTM>(ge, ps, ch, pq, lane, acc, acs);
        else nst = g6_epilogue<!LTM>(ge, ps.n, ps.cb, ps.p0 + pq * 64, ch, lane, acc, acs);
        if (nst > 32) nst = 32;  // 64 stores: credit 32 of them (a lower bound is safe)
    }
}

template <bool LTM, bool STM, bool SPLIT = false>
__global__ __launch_bounds__(G6_THREADS, 1) void k_gemm_x6(G6Geom g) {
    __shared__ __attribute__((aligned(16))) G6XSlot xraw[G6_NX];
    __shared__ __attribute__((aligned(16))) G6WSlot wl[G6_NW];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // waves w and w + 4 share a SIMD: the second one issues its loads half-way (G6_STAGGER);
    // at 4 waves (one per SIMD) every wave issues them half-way, between its MFMAs
    if (G6_W4 || (G6_STAGGER && (wv & 4))) g6_body<LTM, STM, true, SPLIT>(g, xraw, wl, wv);
    else g6_body<LTM, STM, false, SPLIT>(g, xraw, wl, wv);
}

// the split terms of A element (row, col) of an [M][K] operand into their fragment slots
__device__ __forceinline__ void g6_pack_store(unsigned short* __restrict__ wp, float v, int row, int col, int k) {
    unsigned h, mm, l;
    g6_split(v, h, mm, l);
    const int nsteps = k / G6_KC, cb = row / G6_CO, sub = (row % G6_CO) / 32, s = col / G6_KC;
    const int lane = (row & 31) + 32 * ((col & 15) >> 3), j = col & 7;
    const int64_t base = (((int64_t)cb * nsteps + s) * 4 + sub) * 3;
    wp[((base + 0) * 64 + lane) * 8 + j] = static_cast<unsigned short>(h >> 16);
    wp[((base + 1) * 64 + lane) * 8 + j] = static_cast<unsigned short>(mm >> 16);
    wp[((base + 2) * 64 + lane) * 8 + j] = static_cast<unsigned short>(l >> 16);
}

// W [M = o rows][K = c columns] (row-major fp32, or its transpose for trans = 1: W stored [K][M])
// -> packed A fragments: u16 index (((cb * nsteps + s) * 4 + sub) * 3 + term) * 64 + lane) * 8 + j
// for row 128 cb + 32 sub + (lane & 31), column 16 s + 8 (lane >> 5) + j.
__global__ void k_gemm_x6_pack(const float* __restrict__ w, int m, int k, int trans,
                               unsigned short* __restrict__ wp) {
    const int mpad = (m + G6_CO - 1) / G6_CO * G6_CO;  // rows past m packed as zeros
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)mpad * k) return;
    const int row = static_cast<int>(i / k), col = static_cast<int>(i - (int64_t)row * k);
    const float v = row >= m ? 0.f : trans ? w[(int64_t)col * m + row] : w[(int64_t)row * k + col];
    g6_pack_store(wp, v, row, col, k);
}

// Split-K reduce: y = (((ws_0 + ws_1) + ws_2) + ...) + bias[c] (+ res), four elements per
// thread, the parts added in a fixed order (bitwise reproducible).  ws slices are laid out as
// one output of m channels: [n][m][hw] (stm = 0; channels < o1 go to y1 [n][o1][hw], the rest
// to y2 [n][o2][hw]) or [tokens][m] (stm = 1, y1 only); res is shaped like y1 (o2 == 0 only).
__global__ __launch_bounds__(256) void k_g6_split_reduce(const float* __restrict__ ws, int ks, int64_t stride,
                                                         int64_t total4, int m, int hw, int stm, int o1, int o2,
                                                         const float* __restrict__ bias,
                                                         const float* __restrict__ res, float* __restrict__ y1,
                                                         float* __restrict__ y2) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total4) return;
    const int64_t e = 4 * i;
    f32x4 acc = *reinterpret_cast<const f32x4*>(ws + e);
    for (int p = 1; p < ks; ++p) acc += *reinterpret_cast<const f32x4*>(ws + p * stride + e);
    if (stm) {
        const int c = static_cast<int>(e % m);  // four consecutive channels (m % 4 == 0)
        if (bias) acc += f32x4{bias[c], bias[c + 1], bias[c + 2], bias[c + 3]};
        if (res) acc += *reinterpret_cast<const f32x4*>(res + e);
        *reinterpret_cast<f32x4*>(y1 + e) = acc;
        return;
    }
    const int64_t img = e / ((int64_t)m * hw);
    const int64_t rem = e - img * m * hw;
    const int c = static_cast<int>(rem / hw), p = static_cast<int>(rem - (int64_t)c * hw);
    if (bias) acc += bias[c];
    if (c < o1) {
        const int64_t o = (img * o1 + c) * hw + p;
        SP_DCHECK(o + 4 <= total4 * 4);
        if (res) acc += *reinterpret_cast<const f32x4*>(res + o);
        *reinterpret_cast<f32x4*>(y1 + o) = acc;
    } else {
        *reinterpret_cast<f32x4*>(y2 + (img * o2 + (c - o1)) * hw + p) = acc;
    }
}


}  // namespace sp

using namespace sp;


static int g6_cu_count() {
    static int cached[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cached[dev]) {
        int v = 0;
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
            v = 256;
        cached[dev] = v;
    }
    return cached[dev];
}

// Split-K parts for a launch of `tiles` output tiles over `nsteps` k-steps: doubled while the
// items still fit half the CUs, up to 16 parts of >= 2 k-steps (a launch that fills the chip
// is not split).  At batch 1 the 16² / 8² levels' projections are 1-16 tiles with 16-32
// k-steps, one k-step chain per CU (40-80 us) without it.
static int g6_ksplit(int64_t tiles, int nsteps) {
    const int cus = g6_cu_count();
    int ks = 1;
    while (ks < 16 && tiles * ks * 2 <= cus && nsteps % (ks * 2) == 0 && nsteps / (ks * 2) >= 2) ks *= 2;
    return ks;
}

// split-K workspace: ks slices of n * hw * m floats (0: the launch is not split)
static int64_t g6_ws_floats(int64_t tiles, int nsteps, int64_t n, int64_t hw, int m) {
    const int ks = g6_ksplit(tiles, nsteps);
    return ks > 1 ? (int64_t)ks * n * hw * m : 0;
}

// launch k_gemm_x6<LTM, STM> over g (tiles = output tiles), split when ws allows it, then the
// reduce into y1 / y2 with g's bias and residual
template <bool LTM, bool STM>
static int g6_launch(G6Geom g, int64_t tiles, int64_t n, float* ws, int64_t ws_bytes, hipStream_t s) {
    const int m = g.o1 + g.o2;
    const int64_t need = g6_ws_floats(tiles, g.nsteps, n, g.hw, m);
    const int ks = ws && need > 0 && ws_bytes >= need * 4 ? g6_ksplit(tiles, g.nsteps) : 1;
    g.ksplit = ks;
    g.kper = g.nsteps / ks;
    g.ws = ks > 1 ? ws : nullptr;
    g.ws_stride = n * g.hw * m;
    g.ntiles = static_cast<int>(tiles * ks);
    const int grid = static_cast<int>(std::min<int64_t>(g.ntiles, g6_cu_count()));
    if (ks > 1) launch(0, k_gemm_x6<LTM, STM, true>, dim3(grid), dim3(G6_THREADS), s, g);
    else launch(0, k_gemm_x6<LTM, STM>, dim3(grid), dim3(G6_THREADS), s, g);
    if (ks > 1) {
        const int64_t total4 = n * g.hw * m / 4;
        launch(0, k_g6_split_reduce, dim3(static_cast<unsigned>((total4 + 255) / 256)), dim3(256), s, ws, ks,
               g.ws_stride, total4, m, g.hw, STM ? 1 : 0, g.o1, g.o2, g.bias, g.res, g.y1, g.y2);
    }
    return SP_OK;
}

extern "C" {

int sp_gemm_x6_supported(int32_t m, int32_t k, int64_t hw) {
    return m >= G6_CO && m % G6_CO == 0 && k >= G6_KC && k % G6_KC == 0 && hw >= G6_PX &&
           hw % G6_PX == 0 && hw * 32 * 4 < (int64_t(1) << 31) && hw * k * 4 < (int64_t(1) << 31);
}

int64_t sp_gemm_x6_packed_size(int32_t m, int32_t k) {
    return (int64_t)((m + G6_CO - 1) / G6_CO * G6_CO) * k * 6 / 4;
}

int sp_gemm_x6_pack(const float* w, int32_t m, int32_t k, int32_t trans, float* wp, sp_stream_t stream) {
    if (!w || !wp || m % 32 || k % G6_KC || m <= 0 || k <= 0) return SP_EINVAL;
    const int64_t total = (int64_t)((m + G6_CO - 1) / G6_CO * G6_CO) * k;
    launch(0, k_gemm_x6_pack, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256),
           static_cast<hipStream_t>(stream), w, m, k, trans, reinterpret_cast<unsigned short*>(wp));
    return check_launch("sp_gemm_x6_pack");
}

int64_t sp_gemm_x6_workspace(int64_t n, int64_t hw, int32_t k, int32_t m) {
    if (n <= 0 || hw < G6_PX || hw % G6_PX || k < G6_KC || k % G6_KC || m < 32 || m % 32) return 0;
    const int64_t tiles = n * (hw / G6_PX) * ((m + G6_CO - 1) / G6_CO);
    return 4 * g6_ws_floats(tiles, k / G6_KC, n, hw, m);
}

int sp_gemm_x6(const float* x1, int32_t c1, const float* x2, int32_t c2, const float* wp,
               const float* bias, const float* res, int64_t n, int64_t hw, float* y1, int32_t o1,
               float* y2, int32_t o2, sp_stream_t stream) {
    return sp_gemm_x6_ws(x1, c1, x2, c2, wp, bias, res, n, hw, y1, o1, y2, o2, nullptr, 0, stream);
}

int sp_gemm_x6_ws(const float* x1, int32_t c1, const float* x2, int32_t c2, const float* wp,
                  const float* bias, const float* res, int64_t n, int64_t hw, float* y1, int32_t o1,
                  float* y2, int32_t o2, float* ws, int64_t ws_bytes, sp_stream_t stream) {
    const int k = c1 + c2, m = o1 + o2;
    if (!sp_gemm_x6_supported(m, k, hw) || n < 0 || c1 <= 0 || o1 <= 0 || c2 < 0 || o2 < 0)
        return SP_EINVAL;
    if (c1 % 8 || c2 % 8 || o1 % 32 || o2 % 32 || (c2 && !x2) || (o2 && !y2) || (res && o2))
        return SP_EINVAL;
    if (n == 0) return SP_OK;
    if (!x1 || !wp || !y1) return SP_EINVAL;
    const int64_t tiles = n * (hw / G6_PX) * (m / G6_CO);
    if (tiles >= (int64_t(1) << 31)) return SP_EINVAL;
    G6Geom g = {};
    g.x1 = x1;
    g.x2 = x2;
    g.wp = reinterpret_cast<const unsigned short*>(wp);
    g.y1 = y1;
    g.y2 = y2;
    g.bias = bias;
    g.res = res;
    g.c1 = c1;
    g.c2 = c2;
    g.o1 = o1;
    g.o2 = o2;
    g.hw = static_cast<int>(hw);
    g.ntiles = static_cast<int>(tiles);
    g.cob = m / G6_CO;
    g.ptiles = static_cast<int>(hw / G6_PX);
    g.nsteps = k / G6_KC;
    g.tokens = 0;
    g6_launch<false, false>(g, tiles, n, ws, ws_bytes, static_cast<hipStream_t>(stream));
    return check_launch("sp_gemm_x6");
}

int sp_linear_x6_supported(int64_t tokens, int32_t k, int32_t m) {
    return tokens >= G6_PX && tokens % G6_PX == 0 && k >= G6_KC && k % G6_KC == 0 && m >= 32 && m % 32 == 0 &&
           tokens * (int64_t)std::max(k, m) * 4 < (int64_t(1) << 31);
}

// nn.Linear on token-major activations: y[t][o] = sum_k x[t][k] W[o][k] (+ bias[o]) (+ res[t][o]);
// W packed by sp_gemm_x6_pack(w, m, k, 0) (or trans = 1 from W^T for the input VJP).
int sp_linear_x6(const float* x, const float* wp, const float* bias, const float* res, int64_t tokens,
                 int32_t k, int32_t m, float* y, sp_stream_t stream) {
    return sp_linear_x6_ws(x, wp, bias, res, tokens, k, m, y, nullptr, 0, stream);
}

int sp_linear_x6_ws(const float* x, const float* wp, const float* bias, const float* res, int64_t tokens,
                    int32_t k, int32_t m, float* y, float* ws, int64_t ws_bytes, sp_stream_t stream) {
    if (!sp_linear_x6_supported(tokens, k, m)) return SP_EINVAL;
    if (!x || !wp || !y || (res && res == y)) return SP_EINVAL;
    const int cob = (m + G6_CO - 1) / G6_CO;
    const int64_t tiles = tokens / G6_PX * cob;
    G6Geom g = {};
    g.x1 = x;
    g.wp = reinterpret_cast<const unsigned short*>(wp);
    g.y1 = y;
    g.bias = bias;
    g.res = res;
    g.c1 = k;
    g.o1 = m;
    g.hw = static_cast<int>(tokens);
    g.ntiles = static_cast<int>(tiles);
    g.cob = cob;
    g.ptiles = static_cast<int>(tokens / G6_PX);  // one "image" of all tokens
    g.nsteps = k / G6_KC;
    g.tokens = static_cast<int>(tokens);
    g6_launch<true, true>(g, tiles, 1, ws, ws_bytes, static_cast<hipStream_t>(stream));
    return check_launch("sp_linear_x6");
}

int sp_gemm_x6_layout_supported(int64_t n, int64_t hw, int32_t k, int32_t m) {
    return n >= 0 && hw >= G6_PX && hw % G6_PX == 0 && k >= G6_KC && k % G6_KC == 0 && m >= 32 &&
           m % 32 == 0 && n * hw * (int64_t)std::max(k, m) * 4 < (int64_t(1) << 31) &&
           n * hw / G6_PX * ((m + G6_CO - 1) / G6_CO) < (int64_t(1) << 31);
}

// 1x1 conv / linear between the two activation layouts: x [n][k][hw] (in_tm = 0) or
// [n hw][k] (in_tm = 1), y (and res) [n][m][hw] (out_tm = 0) or [n hw][m] (out_tm = 1)
int sp_gemm_x6_layout(const float* x, const float* wp, const float* bias, const float* res, int64_t n,
                      int64_t hw, int32_t k, int32_t m, int32_t in_tm, int32_t out_tm, float* y,
                      sp_stream_t stream) {
    return sp_gemm_x6_layout_ws(x, wp, bias, res, n, hw, k, m, in_tm, out_tm, y, nullptr, 0, stream);
}

int sp_gemm_x6_layout_ws(const float* x, const float* wp, const float* bias, const float* res, int64_t n,
                         int64_t hw, int32_t k, int32_t m, int32_t in_tm, int32_t out_tm, float* y, float* ws,
                         int64_t ws_bytes, sp_stream_t stream) {
    if (!sp_gemm_x6_layout_supported(n, hw, k, m)) return SP_EINVAL;
    if (n == 0) return SP_OK;
    if (!x || !wp || !y || (res && res == y) || x == y) return SP_EINVAL;
    const int cob = (m + G6_CO - 1) / G6_CO;
    G6Geom g = {};
    g.x1 = x;
    g.wp = reinterpret_cast<const unsigned short*>(wp);
    g.y1 = y;
    g.bias = bias;
    g.res = res;
    g.c1 = k;
    g.o1 = m;
    g.hw = static_cast<int>(hw);
    g.ptiles = static_cast<int>(hw / G6_PX);
    const int64_t tiles = n * g.ptiles * cob;
    g.cob = cob;
    g.nsteps = k / G6_KC;
    g.tokens = static_cast<int>(n * hw);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (in_tm && out_tm) g6_launch<true, true>(g, tiles, n, ws, ws_bytes, s);
    else if (in_tm) g6_launch<true, false>(g, tiles, n, ws, ws_bytes, s);
    else if (out_tm) g6_launch<false, true>(g, tiles, n, ws, ws_bytes, s);
    else g6_launch<false, false>(g, tiles, n, ws, ws_bytes, s);
    return check_launch("sp_gemm_x6_layout");
}

}  // extern "C"

// 3x3 / stride 2 convolution with diffusers' Downsample2D padding (downsample_padding=0:
// one zero row / column on the bottom / right, /root/reference/samplers/networks/ddpm.py:40-43
// -> diffusers UNet2DModel) on fp32 MFMA (v_mfma_f32_32x32x2_f32), forward and input VJP, in
// NCHW without the pad copy and the NHWC transposes MIOpen needs for it.
//
//   y[n, co, i, j] = b[co] + sum_{ci, a, b} W[co, ci, a, b] * x[n, ci, 2i + a, 2j + b]
//                    (x = 0 at row H / column W)
//
// Forward: implicit GEMM as sp_conv.hip's tile (M = 128 co, N = 8 output rows x 32 output
// columns, K = 4 input channels x 9 taps per LDS chunk, double-buffered), but the input
// patch (17 rows x 65 columns per channel) is stored de-interleaved by column parity, so the
// stride-2 B reads of a wave are unit-stride LDS addresses: patch column 2c + s lives at
// [parity s & 1][c + (s >> 1)].
//
// Input VJP (optionally accumulated into dx: dx += ..., for a UNet skip tensor whose other
// consumer's gradient is already there), per output phase (p, q) = (row & 1, column & 1) of dx:
//   dx[2i' + p, 2j' + q] = sum_co sum_{a = p, p + 2 <= 2} sum_{b = q, q + 2 <= 2}
//                          W[co, ci, a, b] * dy[co, i' - a/2, j' - b/2]
// i.e. 4, 2, 2 and 1 taps for the phases (0,0), (0,1), (1,0), (1,1) (9 in all: no padded
// work).  One workgroup owns 128 ci x 2 half-rows x 32 half-columns of all four phases
// (= 128 ci x 4 rows x 64 columns of dx); each wave 64 ci x 1 half-row with the four phases'
// accumulators (8 tiles of 32 x 32), sharing one LDS patch of dy (3 rows x 33 columns per
// output channel) and one packed weight chunk (4 co x 9 taps x 128 ci).  The stores write
// both column phases of a row as one float2 per lane.

#define SP_TU 8  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

namespace sp {

typedef float s2_f32x16 __attribute__((ext_vector_type(16)));
typedef float s2_f32x4 __attribute__((ext_vector_type(4)));
typedef float s2_f32x2 __attribute__((ext_vector_type(2)));

constexpr int S2_M = 128;          // output channels per workgroup (forward)
constexpr int S2_TPH = 8;          // output rows per workgroup
constexpr int S2_TPW = 32;         // output columns per workgroup
constexpr int S2_CI = 4;           // input channels per K chunk
constexpr int S2_K = S2_CI * 9;    // 36
constexpr int S2_KH = S2_K / 2;    // k-steps per chunk (lane half h: ci + 2h)
constexpr int S2_NR = S2_TPH / 2;  // pixel rows per wave
constexpr int S2_PR = 2 * S2_TPH + 1;  // 17 patch rows
constexpr int S2_HALF = 34;            // one parity's columns (33 used), even: 8-B aligned pairs
constexpr int S2_RS = 2 * S2_HALF;     // patch row stride
constexpr int S2_PATCH = 1168;         // >= 17 * 68; 2 * S2_PATCH = 32 (mod 64): halves on other banks
constexpr int S2_A4 = S2_K * S2_M / 4;                          // 1152 float4 of A per chunk
constexpr int S2_NA = (S2_A4 + kBlock - 1) / kBlock;            // 5
constexpr int S2_F4 = S2_CI * S2_PR * 16;                       // 1088 float4 of the patch
constexpr int S2_NP = (S2_F4 + kBlock - 1) / kBlock;            // 5
constexpr int S2_TAIL = S2_CI * S2_PR;                          // 68 column-64 scalars

struct S2Stage {
    s2_f32x4 a[S2_NA];
    s2_f32x4 p[S2_NP];
    float t;
};

__device__ __forceinline__ void s2_load(const float* __restrict__ wp, const float* __restrict__ xn,
                                        int cc, int cout, int co0, int r0, int c0, int H, int W,
                                        int64_t plane, int tid, S2Stage& st) {
    const float* src = wp + (int64_t)cc * S2_K * cout + co0;
#pragma unroll
    for (int i = 0; i < S2_NA; ++i) {
        const int idx = tid + kBlock * i;
        if (i < S2_NA - 1 || idx < S2_A4)
            st.a[i] = *reinterpret_cast<const s2_f32x4*>(src + (int64_t)(idx >> 5) * cout + (idx & 31) * 4);
    }
    // the patch by buffer loads over this chunk's planes: a position outside the image (the
    // zero row / column of the padding) gets an offset past the buffer, which reads as 0 — no
    // branches or zero-fill moves around the loads
    constexpr int OOB = 0x7FFFFFF0;
    const auto xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xn + (int64_t)cc * S2_CI * plane),
                                                       (short)0, static_cast<int>(S2_CI * plane * 4), 0x00020000);
#pragma unroll
    for (int i = 0; i < S2_NP; ++i) {
        const int idx = tid + kBlock * i;
        const int q = idx & 15, rc = idx >> 4, ci = rc / S2_PR, row = rc - ci * S2_PR;
        const bool ok = (i < S2_NP - 1 || idx < S2_F4) && r0 + row < H;
        const int off = ok ? static_cast<int>((ci * plane + (int64_t)(r0 + row) * W + c0 + 4 * q) * 4) : OOB;
        st.p[i] = __builtin_bit_cast(s2_f32x4, __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0));
    }
    {
        const int ci = tid / S2_PR, row = tid - ci * S2_PR;
        const bool ok = tid < S2_TAIL && r0 + row < H && c0 + 64 < W;
        const int off = ok ? static_cast<int>((ci * plane + (int64_t)(r0 + row) * W + c0 + 64) * 4) : OOB;
        st.t = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xrs, off, 0, 0));
    }
}

__device__ __forceinline__ void s2_store(float* As, float* Ps, int tid, const S2Stage& st) {
#pragma unroll
    for (int i = 0; i < S2_NA; ++i) {
        const int idx = tid + kBlock * i;
        if (i < S2_NA - 1 || idx < S2_A4) *reinterpret_cast<s2_f32x4*>(&As[idx * 4]) = st.a[i];
    }
#pragma unroll
    for (int i = 0; i < S2_NP; ++i) {
        const int idx = tid + kBlock * i;
        const int q = idx & 15, rc = idx >> 4, ci = rc / S2_PR, row = rc - ci * S2_PR;
        if (i < S2_NP - 1 || idx < S2_F4) {
            float* d = Ps + ci * S2_PATCH + row * S2_RS + 2 * q;
            // two ds_write2_b32 of (even, odd) element pairs: float2 stores of (p0, p2) and
            // (p1, p3) cost four register moves per piece to form the pairs (the empty asm keeps
            // the compiler from merging the dword stores back into them)
            d[0] = st.p[i][0], d[S2_HALF] = st.p[i][1];
            asm volatile("" ::: "memory");
            d[1] = st.p[i][2], d[S2_HALF + 1] = st.p[i][3];
        }
    }
    if (tid < S2_TAIL) {
        const int ci = tid / S2_PR, row = tid - ci * S2_PR;
        Ps[ci * S2_PATCH + row * S2_RS + 32] = st.t;  // column 64: even parity, index 32
    }
}

// split-K (blockIdx.z = part kh of gridDim.z): the part runs input-channel chunks
// kh cper .. + cper - 1 and stores its partial sums (no bias) to out + kh ws_stride;
// k_s2_split_reduce adds the parts.  Unsplit: gridDim.z = 1, cper = all chunks.
__global__ __launch_bounds__(kBlock, 2) void k_conv3x3_s2(const float* __restrict__ x,
                                                          const float* __restrict__ wp,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ out, int cin, int cout,
                                                          int H, int W, int cper, int64_t ws_stride) {
    __shared__ __attribute__((aligned(16))) float As[2][S2_K * S2_M];
    __shared__ __attribute__((aligned(16))) float Ps[2][S2_CI * S2_PATCH];

    const int Ho = H / 2, Wo = W / 2;
    const int tiles_w = Wo / S2_TPW, per_img = tiles_w * (Ho / S2_TPH);
    const int n = blockIdx.x / per_img, t = blockIdx.x - n * per_img;
    const int h0 = (t / tiles_w) * S2_TPH, w0 = (t - (t / tiles_w) * tiles_w) * S2_TPW;
    const int co0 = blockIdx.y * S2_M;
    SP_DCHECK(Wo % S2_TPW == 0 && Ho % S2_TPH == 0 && co0 + S2_M <= cout && cin % S2_CI == 0 &&
              h0 + S2_TPH <= Ho && w0 + S2_TPW <= Wo);
    const int64_t plane = (int64_t)H * W, oplane = (int64_t)Ho * Wo;
    const float* __restrict__ xn = x + (int64_t)n * cin * plane;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5, l = lane & 31;
    const int m_w = (wv & 1) * 64, prow = (wv >> 1) * S2_NR;
    const int cbeg = blockIdx.z * cper, cend = cbeg + cper;
    SP_DCHECK(cend <= cin / S2_CI);
    out += blockIdx.z * ws_stride;

    S2Stage st;
    s2_f32x16 acc[2][S2_NR];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < S2_NR; ++b) acc[a][b] = s2_f32x16{};

    s2_load(wp, xn, cbeg, cout, co0, 2 * h0, 2 * w0, H, W, plane, tid, st);
    s2_store(As[0], Ps[0], tid, st);
    __syncthreads();
    for (int cc = cbeg; cc < cend; ++cc) {
        const int buf = (cc - cbeg) & 1;
        if (cc + 1 < cend) s2_load(wp, xn, cc + 1, cout, co0, 2 * h0, 2 * w0, H, W, plane, tid, st);
        const float* Ab = &As[buf][(S2_KH * hh) * S2_M + m_w + l];
        const float* Pb = &Ps[buf][(S2_CI / 2 * hh) * S2_PATCH + 2 * prow * S2_RS + l];
#pragma unroll
        for (int kk = 0; kk < S2_KH; ++kk) {
            const int r = (kk % 9) / 3, s = kk % 3;
            const int koff = (kk / 9) * S2_PATCH + r * S2_RS + (s & 1) * S2_HALF + (s >> 1);
            const float a0 = Ab[kk * S2_M], a1 = Ab[kk * S2_M + 32];
            float b[S2_NR];
#pragma unroll
            for (int ni = 0; ni < S2_NR; ++ni) b[ni] = Pb[koff + 2 * ni * S2_RS];
#pragma unroll
            for (int ni = 0; ni < S2_NR; ++ni) {
                acc[0][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b[ni], acc[0][ni], 0, 0, 0);
                acc[1][ni] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b[ni], acc[1][ni], 0, 0, 0);
            }
        }
        if (cc + 1 < cend) s2_store(As[buf ^ 1], Ps[buf ^ 1], tid, st);
        __syncthreads();
    }

    // C/D map: col = lane & 31 (output column), row = (r&3) + 8(r>>2) + 4h (co)
    float* on = out + (int64_t)n * cout * oplane;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int co = co0 + m_w + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
            const float bv = bias ? bias[co] : 0.f;
#pragma unroll
            for (int ni = 0; ni < S2_NR; ++ni)
                on[(int64_t)co * oplane + (h0 + prow + ni) * Wo + w0 + l] = acc[mi][ni][r] + bv;
        }
    }
}

// ---- input VJP ------------------------------------------------------------------------------
constexpr int S2B_M = 128;        // input channels (dx) per workgroup
constexpr int S2B_TH = 2;         // half-rows per workgroup (one per wave row)
constexpr int S2B_TW = 32;        // half-columns per workgroup
constexpr int S2B_CO = 4;         // output channels (dy) per K chunk
constexpr int S2B_K = S2B_CO * 9; // packed rows per chunk: k = co_l * 9 + a * 3 + b
constexpr int S2B_PW = 34;        // dy patch row: columns j0 - 1 .. j0 + 31 (33 used)
constexpr int S2B_PATCH = 112;    // >= 3 * 34; 2 * 112 = 32 (mod 64)
constexpr int S2B_PN = S2B_CO * (S2B_TH + 1) * 33;              // 396 patch scalars
constexpr int S2B_NP = (S2B_PN + kBlock - 1) / kBlock;          // 2
constexpr int S2B_A4 = S2B_K * S2B_M / 4;                       // 1152
constexpr int S2B_NA = (S2B_A4 + kBlock - 1) / kBlock;          // 5

struct S2BStage {
    s2_f32x4 a[S2B_NA];
    float p[S2B_NP];
};

__device__ __forceinline__ void s2b_load(const float* __restrict__ wp, const float* __restrict__ dyn,
                                         int cc, int cin, int ci0, int i0, int j0, int Ho, int Wo,
                                         int64_t oplane, int tid, S2BStage& st) {
    const float* src = wp + (int64_t)cc * S2B_K * cin + ci0;
#pragma unroll
    for (int i = 0; i < S2B_NA; ++i) {
        const int idx = tid + kBlock * i;
        if (i < S2B_NA - 1 || idx < S2B_A4)
            st.a[i] = *reinterpret_cast<const s2_f32x4*>(src + (int64_t)(idx >> 5) * cin + (idx & 31) * 4);
    }
    // the dy patch by buffer loads (outside the image: an offset past the buffer, read as 0)
    constexpr int OOB = 0x7FFFFFF0;
    const auto drs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(dyn + (int64_t)cc * S2B_CO * oplane),
                                                       (short)0, static_cast<int>(S2B_CO * oplane * 4), 0x00020000);
#pragma unroll
    for (int i = 0; i < S2B_NP; ++i) {
        const int idx = tid + kBlock * i;
        const int co = idx / ((S2B_TH + 1) * 33), rem = idx - co * ((S2B_TH + 1) * 33);
        const int pr = rem / 33, pc = rem - pr * 33;
        const int gi = i0 - 1 + pr, gj = j0 - 1 + pc;
        const bool ok = idx < S2B_PN && gi >= 0 && gj >= 0 && gi < Ho && gj < Wo;
        const int off = ok ? static_cast<int>((co * oplane + (int64_t)gi * Wo + gj) * 4) : OOB;
        st.p[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(drs, off, 0, 0));
    }
}

__device__ __forceinline__ void s2b_store(float* As, float* Ps, int tid, const S2BStage& st) {
#pragma unroll
    for (int i = 0; i < S2B_NA; ++i) {
        const int idx = tid + kBlock * i;
        if (i < S2B_NA - 1 || idx < S2B_A4) *reinterpret_cast<s2_f32x4*>(&As[idx * 4]) = st.a[i];
    }
#pragma unroll
    for (int i = 0; i < S2B_NP; ++i) {
        const int idx = tid + kBlock * i;
        const int co = idx / ((S2B_TH + 1) * 33), rem = idx - co * ((S2B_TH + 1) * 33);
        const int pr = rem / 33, pc = rem - pr * 33;
        if (idx < S2B_PN) Ps[co * S2B_PATCH + pr * S2B_PW + pc] = st.p[i];
    }
}

// split-K as k_conv3x3_s2 (parts over the output-channel chunks; acc_in 0 for parts)
__global__ __launch_bounds__(kBlock, 2) void k_conv3x3_s2_bwd(const float* __restrict__ dy,
                                                              const float* __restrict__ wp,
                                                              float* __restrict__ dx, int cin,
                                                              int cout, int H, int W, int acc_in,
                                                              int cper, int64_t ws_stride) {
    __shared__ __attribute__((aligned(16))) float As[2][S2B_K * S2B_M];
    __shared__ float Ps[2][S2B_CO * S2B_PATCH];

    const int Ho = H / 2, Wo = W / 2;
    const int tiles_w = Wo / S2B_TW, per_img = tiles_w * (Ho / S2B_TH);
    const int n = blockIdx.x / per_img, t = blockIdx.x - n * per_img;
    const int i0 = (t / tiles_w) * S2B_TH, j0 = (t - (t / tiles_w) * tiles_w) * S2B_TW;
    const int ci0 = blockIdx.y * S2B_M;
    SP_DCHECK(Wo % S2B_TW == 0 && Ho % S2B_TH == 0 && ci0 + S2B_M <= cin && cout % S2B_CO == 0 &&
              i0 + S2B_TH <= Ho && j0 + S2B_TW <= Wo);
    const int64_t plane = (int64_t)H * W, oplane = (int64_t)Ho * Wo;
    const float* __restrict__ dyn = dy + (int64_t)n * cout * oplane;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, hh = lane >> 5, l = lane & 31;
    const int m_w = (wv & 1) * 64, rw = wv >> 1;
    const int cbeg = blockIdx.z * cper, cend = cbeg + cper;
    SP_DCHECK(cend <= cout / S2B_CO && (gridDim.z == 1 || !acc_in));
    dx += blockIdx.z * ws_stride;

    S2BStage st;
    s2_f32x16 acc[4][2];  // [phase p * 2 + q][ci tile]
#pragma unroll
    for (int a = 0; a < 4; ++a) acc[a][0] = s2_f32x16{}, acc[a][1] = s2_f32x16{};

    s2b_load(wp, dyn, cbeg, cin, ci0, i0, j0, Ho, Wo, oplane, tid, st);
    s2b_store(As[0], Ps[0], tid, st);
    __syncthreads();
    for (int cc = cbeg; cc < cend; ++cc) {
        const int buf = (cc - cbeg) & 1;
        if (cc + 1 < cend) s2b_load(wp, dyn, cc + 1, cin, ci0, i0, j0, Ho, Wo, oplane, tid, st);
        // lane half h carries output channel co_l = kc + 2h
        const float* Ab = &As[buf][(2 * hh) * 9 * S2B_M + m_w + l];
        const float* Pb = &Ps[buf][(2 * hh) * S2B_PATCH + rw * S2B_PW + l];
#pragma unroll
        for (int kc = 0; kc < 2; ++kc) {
            float bv[2][2];  // dy[i' - da, j' - db]: patch row rw + 1 - da, column l + 1 - db
#pragma unroll
            for (int da = 0; da < 2; ++da)
#pragma unroll
                for (int db = 0; db < 2; ++db)
                    bv[da][db] = Pb[kc * S2B_PATCH + (1 - da) * S2B_PW + (1 - db)];
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    const int ph = (a & 1) * 2 + (b & 1);
                    const float* ap = Ab + (kc * 9 + a * 3 + b) * S2B_M;
#pragma unroll
                    for (int mt = 0; mt < 2; ++mt)
                        acc[ph][mt] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                            ap[mt * 32], bv[a >> 1][b >> 1], acc[ph][mt], 0, 0, 0);
                }
        }
        if (cc + 1 < cend) s2b_store(As[buf ^ 1], Ps[buf ^ 1], tid, st);
        __syncthreads();
    }

    // C/D map: col = l (half-column j0 + l), row = (r&3) + 8(r>>2) + 4h (ci)
    float* dn = dx + (int64_t)n * cin * plane;
    const int ip = i0 + rw;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int ci = ci0 + m_w + mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                s2_f32x2* d = reinterpret_cast<s2_f32x2*>(dn + (int64_t)ci * plane +
                                                          (int64_t)(2 * ip + p) * W + 2 * (j0 + l));
                s2_f32x2 v{acc[p * 2][mt][r], acc[p * 2 + 1][mt][r]};
                if (acc_in) v = *d + v;  // accumulate: dx already holds another consumer's gradient
                *d = v;
            }
        }
    }
}

// Split-K reduce: out = (acc ? out : 0) + (((ws_0 + ws_1) + ws_2) + ...) + bias[c], four
// elements per thread (plane % 4 == 0), the parts added in a fixed order (bitwise reproducible)
__global__ __launch_bounds__(256) void k_s2_split_reduce(const float* __restrict__ ws, int ks, int64_t stride,
                                                         int64_t total4, int64_t plane, int channels,
                                                         const float* __restrict__ bias, int acc,
                                                         float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total4) return;
    const int64_t e = 4 * i;
    s2_f32x4 v = *reinterpret_cast<const s2_f32x4*>(ws + e);
    for (int p = 1; p < ks; ++p) v += *reinterpret_cast<const s2_f32x4*>(ws + p * stride + e);
    if (bias) v += bias[(e / plane) % channels];
    if (acc) v = *reinterpret_cast<const s2_f32x4*>(out + e) + v;
    *reinterpret_cast<s2_f32x4*>(out + e) = v;
}

// Forward: wp[(cc*36 + ci_l*9 + a*3 + b)*cout + co] (sp_conv3x3_pack's layout); input VJP:
// wp[(cc*36 + co_l*9 + a*3 + b)*cin + ci] (no flip: the phases index the taps directly).
__global__ void k_conv3x3_s2_pack(const float* __restrict__ w, int cout, int cin, int vjp,
                                  float* __restrict__ wp) {
    const int64_t total = (int64_t)cout * cin * 9;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    const int co = static_cast<int>(i / ((int64_t)cin * 9));
    const int rem = static_cast<int>(i - (int64_t)co * cin * 9);
    const int ci = rem / 9, ab = rem - ci * 9;
    if (!vjp)
        wp[((int64_t)(ci / S2_CI) * S2_K + (ci % S2_CI) * 9 + ab) * cout + co] = w[i];
    else
        wp[((int64_t)(co / S2B_CO) * S2B_K + (co % S2B_CO) * 9 + ab) * cin + ci] = w[i];
}

}  // namespace sp

using namespace sp;

static int s2_cu_count() {
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

// split-K parts for `blocks` workgroups over `nchunks` K chunks: doubled while the workgroups
// still fit the CUs, up to 16 parts of >= 4 chunks (at batch 1 the 128² -> 64² and 64² -> 32²
// downsamplers are 16 and 8 workgroups walking 32-64 chunks, 150-300 us unsplit)
static int s2_ksplit(int64_t blocks, int nchunks) {
    const int cus = s2_cu_count();
    int ks = 1;
    while (ks < 16 && blocks * ks * 2 <= cus && nchunks % (ks * 2) == 0 && nchunks / (ks * 2) >= 4) ks *= 2;
    return ks;
}

static int s2_parts(int64_t n, int32_t cin, int32_t cout, int32_t height, int32_t width, int vjp) {
    if (!vjp) return s2_ksplit(n * (height / 2 / S2_TPH) * (width / 2 / S2_TPW) * (cout / S2_M), cin / S2_CI);
    return s2_ksplit(n * (height / 2 / S2B_TH) * (width / 2 / S2B_TW) * (cin / S2B_M), cout / S2B_CO);
}

extern "C" {

int64_t sp_conv3x3_s2_workspace(int64_t n, int32_t cin, int32_t cout, int32_t height, int32_t width,
                                int32_t input_vjp) {
    if (n <= 0 || !sp_conv3x3_s2_supported(cin, cout, height, width, input_vjp)) return 0;
    const int ks = s2_parts(n, cin, cout, height, width, input_vjp);
    if (ks <= 1) return 0;
    const int64_t outf = input_vjp ? n * cin * (int64_t)height * width : n * cout * (int64_t)(height / 2) * (width / 2);
    return 4 * ks * outf;
}

int sp_conv3x3_s2_supported(int32_t cin, int32_t cout, int32_t height, int32_t width,
                            int32_t input_vjp) {
    if (cin <= 0 || cout <= 0 || height <= 0 || width <= 0 || height % 2 || width % 2) return 0;
    const int ho = height / 2, wo = width / 2;
    if (!input_vjp)
        return cin % S2_CI == 0 && cout % S2_M == 0 && ho % S2_TPH == 0 && wo % S2_TPW == 0;
    return cout % S2B_CO == 0 && cin % S2B_M == 0 && ho % S2B_TH == 0 && wo % S2B_TW == 0;
}

int sp_conv3x3_s2_pack(const float* w, int32_t cout, int32_t cin, int32_t input_vjp, float* wp,
                       sp_stream_t stream) {
    if (!w || !wp || cout <= 0 || cin <= 0) return SP_EINVAL;
    if (input_vjp ? (cout % S2B_CO) : (cin % S2_CI)) return SP_EINVAL;
    const int64_t total = (int64_t)cout * cin * 9;
    launch(0, k_conv3x3_s2_pack, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256),
           static_cast<hipStream_t>(stream), w, cout, cin, input_vjp ? 1 : 0, wp);
    return check_launch("sp_conv3x3_s2_pack");
}

int sp_conv3x3_s2_fwd(const float* x, const float* wp, const float* bias, int64_t n, int32_t cin,
                      int32_t cout, int32_t height, int32_t width, float* y, sp_stream_t stream) {
    return sp_conv3x3_s2_fwd_ws(x, wp, bias, n, cin, cout, height, width, y, nullptr, 0, stream);
}

int sp_conv3x3_s2_fwd_ws(const float* x, const float* wp, const float* bias, int64_t n, int32_t cin,
                         int32_t cout, int32_t height, int32_t width, float* y, float* ws, int64_t ws_bytes,
                         sp_stream_t stream) {
    if (!sp_conv3x3_s2_supported(cin, cout, height, width, 0) || n < 0) return SP_EINVAL;
    if (n == 0) return SP_OK;
    if (!x || !wp || !y) return SP_EINVAL;
    const int64_t tiles = n * (height / 2 / S2_TPH) * (width / 2 / S2_TPW);
    if (tiles >= (int64_t(1) << 31) || (int64_t)cin * height * width >= (int64_t(1) << 31))
        return SP_EINVAL;
    const double flops = 18.0 * n * cin * cout * (height / 2) * (width / 2);
    const int64_t need = sp_conv3x3_s2_workspace(n, cin, cout, height, width, 0);
    const int ks = ws && need > 0 && ws_bytes >= need ? s2_parts(n, cin, cout, height, width, 0) : 1;
    const int64_t outf = n * cout * (int64_t)(height / 2) * (width / 2);
    hipStream_t s = static_cast<hipStream_t>(stream);
    launch_w(TK_CONV3X3_FWD, flops, k_conv3x3_s2, dim3(static_cast<unsigned>(tiles), cout / S2_M, ks),
             dim3(kBlock), s, x, wp, ks > 1 ? nullptr : bias, ks > 1 ? ws : y, cin, cout, height, width,
             cin / S2_CI / ks, outf);
    if (ks > 1)
        launch(0, k_s2_split_reduce, dim3(static_cast<unsigned>((outf / 4 + 255) / 256)), dim3(256), s, ws, ks,
               outf, outf / 4, (int64_t)(height / 2) * (width / 2), cout, bias, 0, y);
    return check_launch("sp_conv3x3_s2_fwd");
}

int sp_conv3x3_s2_bwd_input(const float* dy, const float* wp_vjp, int64_t n, int32_t cin,
                            int32_t cout, int32_t height, int32_t width, int32_t accumulate,
                            float* dx, sp_stream_t stream) {
    return sp_conv3x3_s2_bwd_input_ws(dy, wp_vjp, n, cin, cout, height, width, accumulate, dx, nullptr, 0, stream);
}

int sp_conv3x3_s2_bwd_input_ws(const float* dy, const float* wp_vjp, int64_t n, int32_t cin,
                               int32_t cout, int32_t height, int32_t width, int32_t accumulate,
                               float* dx, float* ws, int64_t ws_bytes, sp_stream_t stream) {
    if (!sp_conv3x3_s2_supported(cin, cout, height, width, 1) || n < 0) return SP_EINVAL;
    if (n == 0) return SP_OK;
    if (!dy || !wp_vjp || !dx) return SP_EINVAL;
    const int64_t tiles = n * (height / 2 / S2B_TH) * (width / 2 / S2B_TW);
    if (tiles >= (int64_t(1) << 31) || (int64_t)cin * height * width >= (int64_t(1) << 31))
        return SP_EINVAL;
    const double flops = 18.0 * n * cin * cout * (height / 2) * (width / 2);
    const int64_t need = sp_conv3x3_s2_workspace(n, cin, cout, height, width, 1);
    const int ks = ws && need > 0 && ws_bytes >= need ? s2_parts(n, cin, cout, height, width, 1) : 1;
    const int64_t outf = n * cin * (int64_t)height * width;
    hipStream_t s = static_cast<hipStream_t>(stream);
    launch_w(TK_CONV3X3_BWD_INPUT, flops, k_conv3x3_s2_bwd,
             dim3(static_cast<unsigned>(tiles), cin / S2B_M, ks), dim3(kBlock), s, dy, wp_vjp,
             ks > 1 ? ws : dx, cin, cout, height, width, ks > 1 ? 0 : (accumulate ? 1 : 0), cout / S2B_CO / ks,
             outf);
    if (ks > 1)
        launch(0, k_s2_split_reduce, dim3(static_cast<unsigned>((outf / 4 + 255) / 256)), dim3(256), s, ws, ks,
               outf, outf / 4, (int64_t)height * width, cin, nullptr, accumulate ? 1 : 0, dx);
    return check_launch("sp_conv3x3_s2_bwd_input");
}

}  // extern "C"

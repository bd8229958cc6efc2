// Depthwise separable Gaussian blur (BASELINE config 3) with reflect padding:
//   A x  = conv_v(conv_h(reflect_pad(x)))   per channel plane, taps k[-R..R]
//   A^T s = exact transpose: zero-extended correlation, then the padded halo
//           folded back onto the reflected pixels (adjoint of reflect-pad).
// The reference has no blur operator; the CPU oracle
// (oracle/blur.py) pins these semantics with torch autograd of
// F.pad(mode="reflect") + conv2d.
//
// One workgroup owns a TH x TW output tile of one channel plane.  For the fused
// DPS pass the tile needs x0 on T +- 2R (forward blur of the residual halo),
// the residual s on T +- R and produces v on T: every intermediate lives in LDS
// (two ping-pong buffers), HBM sees x, eps, y once plus the halo re-reads that
// neighbouring tiles mostly serve from L2.

#include <algorithm>

#include "sp_common.h"

namespace sp {

constexpr int TH = 32;
constexpr int TW = 64;

__device__ __forceinline__ int reflect_clamp(int g, int L) {
    if (g < 0) g = -g;
    if (g >= L) g = 2 * (L - 1) - g;
    return g < 0 ? 0 : (g >= L ? L - 1 : g);
}

enum { MODE_APPLY = 0, MODE_ADJOINT = 1, MODE_DPS = 2 };

template <int R>
struct BlurLds {
    static constexpr int XR = TH + 4 * R, XC = TW + 4 * R;  // x0 window (T +- 2R)
    static constexpr int HR = TH + 4 * R, HC = TW + 2 * R;  // horizontal pass of it
    static constexpr int SR = TH + 2 * R, SC = TW + 2 * R;  // residual window (T +- R)
    static constexpr int UR = TH, UC = TW + 2 * R;          // vertical adjoint
    static constexpr int A = (XR * XC > SR * SC) ? XR * XC : SR * SC;
    static constexpr int B = (HR * HC > UR * UC) ? HR * HC : UR * UC;
};

// Vertical adjoint for rows of T, columns [C0-R, C0+TW+R): U = A_v^T S.
template <int R>
__device__ __forceinline__ void vertical_adjoint(const float* S, float* U, const float* tk, int R0,
                                                 int C0, int H, int W) {
    using L = BlurLds<R>;
    for (int idx = threadIdx.x; idx < L::UR * L::UC; idx += kBlock) {
        const int i = idx / L::UC, q = idx % L::UC;
        const int gi = R0 + i, gj = C0 - R + q;
        float acc = 0.f;
        if (gi < H && gj >= 0 && gj < W) {
            // S row index of global row g: g - (R0 - R)
            const bool lo = gi > 0 && gi <= R;
            const bool hi = gi < H - 1 && gi >= H - 1 - R;
#pragma unroll
            for (int d = -R; d <= R; ++d) {
                const float kd = tk[d + R];
                float s = 0.f;
                int g = gi - d;
                if (g >= 0 && g < H) s += S[(g - R0 + R) * L::SC + q];
                if (lo) {
                    g = -gi - d;
                    if (g >= 0) s += S[(g - R0 + R) * L::SC + q];
                }
                if (hi) {
                    g = 2 * H - 2 - gi - d;
                    if (g < H) s += S[(g - R0 + R) * L::SC + q];
                }
                acc += kd * s;
            }
        }
        U[i * L::UC + q] = acc;
    }
}

// Horizontal adjoint for the output tile: out = A_h^T U (rows of T).
template <int R>
__device__ __forceinline__ void horizontal_adjoint_store(const float* U, const float* tk, int R0,
                                                         int C0, int H, int W,
                                                         float* __restrict__ plane_out) {
    using L = BlurLds<R>;
    for (int idx = threadIdx.x; idx < TH * TW; idx += kBlock) {
        const int i = idx / TW, j = idx % TW;
        const int gi = R0 + i, gj = C0 + j;
        if (gi >= H || gj >= W) continue;
        const bool lo = gj > 0 && gj <= R;
        const bool hi = gj < W - 1 && gj >= W - 1 - R;
        float acc = 0.f;
#pragma unroll
        for (int d = -R; d <= R; ++d) {
            const float kd = tk[d + R];
            float u = 0.f;
            int g = gj - d;
            if (g >= 0 && g < W) u += U[i * L::UC + (g - C0 + R)];
            if (lo) {
                g = -gj - d;
                if (g >= 0) u += U[i * L::UC + (g - C0 + R)];
            }
            if (hi) {
                g = 2 * W - 2 - gj - d;
                if (g < W) u += U[i * L::UC + (g - C0 + R)];
            }
            acc += kd * u;
        }
        plane_out[(int64_t)gi * W + gj] = acc;
    }
}

template <int R, int MODE>
__global__ __launch_bounds__(kBlock) void k_blur(sp_op op, const float* __restrict__ in,
                                                 const float* __restrict__ eps,
                                                 const float* __restrict__ y, int64_t y_div,
                                                 float a, float k, float gs,
                                                 float* __restrict__ out,
                                                 float* __restrict__ partial, int P) {
    using L = BlurLds<R>;
    __shared__ float bufA[L::A];
    __shared__ float bufB[L::B];
    __shared__ float tk[2 * R + 1];
    __shared__ float red[4];

    const int H = op.height, W = op.width, C = op.channels;
    const int tilesW = (W + TW - 1) / TW;
    const int R0 = (blockIdx.x / tilesW) * TH, C0 = (blockIdx.x % tilesW) * TW;
    const int c = blockIdx.y;
    const int64_t b = blockIdx.z;
    const int64_t plane = (int64_t)H * W;
    const int64_t xoff = (b * C + c) * plane;

    if (threadIdx.x < 2 * R + 1) tk[threadIdx.x] = op.taps[threadIdx.x];

    if constexpr (MODE == MODE_ADJOINT) {
        // S = input s on T +- R, zero outside the image
        float* S = bufA;
        for (int idx = threadIdx.x; idx < L::SR * L::SC; idx += kBlock) {
            const int p = idx / L::SC, q = idx % L::SC;
            const int gi = R0 - R + p, gj = C0 - R + q;
            S[idx] = (gi >= 0 && gi < H && gj >= 0 && gj < W) ? in[xoff + (int64_t)gi * W + gj] : 0.f;
        }
        __syncthreads();
        vertical_adjoint<R>(S, bufB, tk, R0, C0, H, W);
        __syncthreads();
        horizontal_adjoint_store<R>(bufB, tk, R0, C0, H, W, out + xoff);
        return;
    } else if constexpr (MODE == MODE_APPLY) {
        // X = x on T +- R (reflected), Hz = horizontal pass on rows T +- R, out = vertical pass on T
        constexpr int XR = TH + 2 * R, XC = TW + 2 * R;
        float* X = bufA;
        float* Hz = bufB;
        for (int idx = threadIdx.x; idx < XR * XC; idx += kBlock) {
            const int p = idx / XC, q = idx % XC;
            const int gi = reflect_clamp(R0 - R + p, H), gj = reflect_clamp(C0 - R + q, W);
            X[idx] = in[xoff + (int64_t)gi * W + gj];
        }
        __syncthreads();
        for (int idx = threadIdx.x; idx < XR * TW; idx += kBlock) {
            const int p = idx / TW, q = idx % TW;
            float acc = 0.f;
#pragma unroll
            for (int d = -R; d <= R; ++d) acc += tk[d + R] * X[p * XC + q + R + d];
            Hz[idx] = acc;
        }
        __syncthreads();
        for (int idx = threadIdx.x; idx < TH * TW; idx += kBlock) {
            const int i = idx / TW, j = idx % TW;
            const int gi = R0 + i, gj = C0 + j;
            if (gi >= H || gj >= W) continue;
            float acc = 0.f;
#pragma unroll
            for (int d = -R; d <= R; ++d) acc += tk[d + R] * Hz[(i + R + d) * TW + j];
            out[xoff + (int64_t)gi * W + gj] = acc;
        }
        return;
    } else {
        // fused DPS residual pass
        const int64_t yoff = ((b / y_div) * C + c) * plane;
        float* X = bufA;
        float* Hz = bufB;
        for (int idx = threadIdx.x; idx < L::XR * L::XC; idx += kBlock) {
            const int p = idx / L::XC, q = idx % L::XC;
            const int gi = reflect_clamp(R0 - 2 * R + p, H), gj = reflect_clamp(C0 - 2 * R + q, W);
            const int64_t o = xoff + (int64_t)gi * W + gj;
            X[idx] = (in[o] - k * eps[o]) / a;
        }
        __syncthreads();
        for (int idx = threadIdx.x; idx < L::HR * L::HC; idx += kBlock) {
            const int p = idx / L::HC, q = idx % L::HC;
            float acc = 0.f;
#pragma unroll
            for (int d = -R; d <= R; ++d) acc += tk[d + R] * X[p * L::XC + q + R + d];
            Hz[idx] = acc;
        }
        __syncthreads();
        float* S = bufA;  // X is dead
        float racc = 0.f;
        for (int idx = threadIdx.x; idx < L::SR * L::SC; idx += kBlock) {
            const int p = idx / L::SC, q = idx % L::SC;
            const int gi = R0 - R + p, gj = C0 - R + q;
            float sv = 0.f;
            if (gi >= 0 && gi < H && gj >= 0 && gj < W) {
                float z = 0.f;
#pragma unroll
                for (int d = -R; d <= R; ++d) z += tk[d + R] * Hz[(p + R + d) * L::HC + q];
                const float r = y[yoff + (int64_t)gi * W + gj] - z;
                sv = gs * r;
                if (p >= R && p < R + TH && q >= R && q < R + TW) racc += r * r;
            }
            S[idx] = sv;
        }
        __syncthreads();
        vertical_adjoint<R>(S, bufB, tk, R0, C0, H, W);  // Hz is dead
        const float t = block_sum(racc, red);            // contains a barrier
        if (threadIdx.x == 0) partial[b * P + (int64_t)c * gridDim.x + blockIdx.x] = t;
        __syncthreads();
        horizontal_adjoint_store<R>(bufB, tk, R0, C0, H, W, out + xoff);
    }
}

int64_t blur_partials(const sp_op* op) {
    const int64_t tiles = (int64_t)((op->height + TH - 1) / TH) * ((op->width + TW - 1) / TW);
    return tiles * op->channels;
}

template <int MODE>
static int launch_blur(const sp_op* op, const float* in, const float* eps, const float* y,
                       int64_t y_div, float a, float k, float gs, float* out, float* partial,
                       int64_t batch, hipStream_t s) {
    const int tiles = ((op->height + TH - 1) / TH) * ((op->width + TW - 1) / TW);
    const dim3 grid(tiles, op->channels, static_cast<unsigned>(batch));
    const int P = static_cast<int>(blur_partials(op));
    switch (op->radius) {
#define SP_BLUR_CASE(RR)                                                                       \
    case RR:                                                                                   \
        launch(MODE == MODE_DPS ? TK_DPS_RESIDUAL : 0, k_blur<RR, MODE>, grid, dim3(kBlock), s, \
               *op, in, eps, y, y_div, a, k, gs, out, partial, P);                               \
        break;
        SP_BLUR_CASE(1) SP_BLUR_CASE(2) SP_BLUR_CASE(3) SP_BLUR_CASE(4)
        SP_BLUR_CASE(5) SP_BLUR_CASE(6) SP_BLUR_CASE(7) SP_BLUR_CASE(8)
#undef SP_BLUR_CASE
        default: return SP_EINVAL;
    }
    return check_launch("blur");
}

int blur_dps_residual(const sp_op* op, const float* x, const float* eps, const float* y,
                      int64_t batch, int64_t y_div, float a, float k, float gs, float* v,
                      float* partial, hipStream_t s) {
    return launch_blur<MODE_DPS>(op, x, eps, y, y_div, a, k, gs, v, partial, batch, s);
}

int blur_apply(const sp_op* op, const float* x, float* y, int64_t batch, hipStream_t s) {
    return launch_blur<MODE_APPLY>(op, x, nullptr, nullptr, 1, 1.f, 0.f, 0.f, y, nullptr, batch, s);
}

int blur_adjoint(const sp_op* op, const float* y, float* x, int64_t batch, hipStream_t s) {
    return launch_blur<MODE_ADJOINT>(op, y, nullptr, nullptr, 1, 1.f, 0.f, 0.f, x, nullptr, batch,
                                     s);
}

}  // namespace sp

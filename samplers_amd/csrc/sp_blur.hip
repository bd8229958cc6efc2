// Depthwise separable Gaussian blur (BASELINE config 3) with reflect padding:
//   A x   = conv_v(conv_h(reflect_pad(x)))   per channel plane, taps k[-R..R]
//   A^T s = exact transpose of that map: a zero-extended correlation, then the
//           padded halo folded back onto the pixels it was reflected from:
//             U(p)  = sum_d k[d] s(p - d)                (s = 0 off the image)
//             v(j)  = U(j) + [0 < j <= R] U(-j) + [N-1-R <= j < N-1] U(2N-2-j)
//           applied per axis (vertical, then horizontal).
// The reference has no blur operator; oracle/blur.py pins these
// semantics with torch autograd of F.pad(mode="reflect") + conv2d.
//
// One workgroup owns a TH x TW output tile T of one channel plane.  The fused DPS
// pass keeps every intermediate in LDS and register-blocks each stage so that LDS
// traffic stays far below the HBM time of the pass:
//   1  X  = x0 = (x - k eps)/a on T +- 2R (reflected)   x, eps from HBM, lane = column
//   2  Hh = horizontal pass on T +- 2R rows, T +- R cols 4 adjacent outputs per thread
//                                                       (ds_read_b128 of the 4+2R inputs)
//   3  S  = c (y - vertical(Hh)) on T +- R, 0 off image column strips of 8 rows per
//          + |r|^2 partial over T                       thread (sliding window), y from HBM
//   4  V  = vertical adjoint of S (+ row fold) on T     column strips again
//   5  v  = horizontal adjoint of V (+ column fold)     4-wide items, float4 stores to HBM
// HBM traffic: x, eps, y, v once plus halo re-reads that neighbouring tiles serve
// from the XCD's L2 (tiles are ordered so one XCD walks neighbouring tiles).
// Taps live in SGPRs (uniform loads), not LDS.

#include <utility>

#define SP_TU 2  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

namespace sp {

constexpr int TH = 32;
constexpr int TW = 64;
constexpr int BX = 64;  // lanes per row in the load stage
constexpr int BY = kBlock / BX;
constexpr int STRIP = 8;  // rows per thread in the column stages

__device__ __forceinline__ int reflect_clamp(int g, int L) {
    if (g < 0) g = -g;
    if (g >= L) g = 2 * (L - 1) - g;
    return g < 0 ? 0 : (g >= L ? L - 1 : g);
}

__host__ __device__ constexpr int round4(int v) { return (v + 3) & ~3; }

typedef float f2v __attribute__((ext_vector_type(2)));

// two FMAs in one v_pk_fma_f32 (scalar tap broadcast to both halves)
__device__ __forceinline__ f2v pk_fma(float s, f2v a, f2v c) {
    return __builtin_elementwise_fma(f2v{s, s}, a, c);
}

enum { MODE_APPLY = 0, MODE_ADJOINT = 1, MODE_DPS = 2 };

template <int R>
struct BlurGeom {
    static constexpr int K = 2 * R + 1;
    static constexpr int NB = (4 + 2 * R + 3) / 4;        // float4 reads per 4-wide item
    static constexpr int WR = TH + 4 * R;                 // X / Hh rows (T +- 2R)
    static constexpr int SR = TH + 2 * R;                 // S rows (T +- R)
    static constexpr int HC = TW + 2 * R;                 // Hh / S / V columns (T +- R)
    static constexpr int HCP = round4(HC);                // their row stride
    static constexpr int XC = TW + 4 * R;                 // X columns (T +- 2R)
    static constexpr int XCP = round4(HCP - 4 + 4 * NB > XC ? HCP - 4 + 4 * NB : XC);
    static constexpr int LDS_A = WR * XCP;                // X, later S
    static constexpr int LDS_B = WR * HCP;                // Hh, later V
};

// dst[r][q..q+3] = sum_d k[d] src[r][q + R + d] for 4-wide items over rows x cols4*4.
template <int R>
__device__ __forceinline__ void hpass(const float* src, int sstride, float* dst, int dstride,
                                      int rows, int cols4, const float (&tk)[2 * R + 1]) {
    using G = BlurGeom<R>;
    for (int it = threadIdx.x; it < rows * cols4; it += kBlock) {
        const int r = it / cols4, q = (it - r * cols4) * 4;
        float w[4 * G::NB];
        const float4* s4 = reinterpret_cast<const float4*>(src + r * sstride + q);
#pragma unroll
        for (int j = 0; j < G::NB; ++j) {
            const float4 t = s4[j];
            w[4 * j] = t.x, w[4 * j + 1] = t.y, w[4 * j + 2] = t.z, w[4 * j + 3] = t.w;
        }
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float acc = 0.f;
#pragma unroll
            for (int d = 0; d < G::K; ++d) acc = fmaf(tk[d], w[e + d], acc);
            o[e] = acc;
        }
        *reinterpret_cast<float4*>(dst + r * dstride + q) = make_float4(o[0], o[1], o[2], o[3]);
    }
}

// Vertical adjoint on T rows: V[i][q] = U(R0+i) + folds, with S on T +- R rows
// (S row of global row g is g - R0 + R; rows outside S are zero / off the image).
// Fold terms exist only in tiles within R rows of the top/bottom edge (a uniform
// branch); there U(-g) = sum_{i=0}^{R-g} k[-g-i] S(i) and
// U(2H-2-g) = sum_{i=2H-2-g-R}^{H-1} k[2H-2-g-i] S(i).
template <int R>
__device__ __forceinline__ void vadjoint(const float* S, float* V, int R0, int H,
                                         const float (&tk)[2 * R + 1], const float* tkl) {
    using G = BlurGeom<R>;
    constexpr int NS = TH / STRIP, HP = G::HC / 2;  // items: 8-row strips x column pairs
    const bool rfold = R0 <= R || R0 + TH >= H - 1 - R;
    for (int it = threadIdx.x; it < NS * HP; it += kBlock) {
        const int s = it / HP, q = 2 * (it - s * HP);
        const int i0 = s * STRIP;
        f2v w[STRIP + 2 * R];
#pragma unroll
        for (int j = 0; j < STRIP + 2 * R; ++j) w[j] = *reinterpret_cast<const f2v*>(S + (i0 + j) * G::HCP + q);
        f2v u[STRIP];
#pragma unroll
        for (int e = 0; e < STRIP; ++e) {
            // U(g) = sum_d k[d] S(g - d): S rows i0+e+R-d  ->  w[e + 2R - (d+R)]
            f2v acc = {0.f, 0.f};
#pragma unroll
            for (int d = 0; d < G::K; ++d) acc = pk_fma(tk[d], w[e + 2 * R - d], acc);
            u[e] = acc;
        }
        if (rfold) {
#pragma unroll
            for (int e = 0; e < STRIP; ++e) {
                const int gi = R0 + i0 + e;
                if (gi > 0 && gi <= R)
                    for (int i = 0; i <= R - gi; ++i)
                        u[e] = pk_fma(tkl[R - gi - i],
                                      *reinterpret_cast<const f2v*>(S + (i - R0 + R) * G::HCP + q), u[e]);
                if (gi < H - 1 && gi >= H - 1 - R)
                    for (int i = 2 * H - 2 - gi - R; i < H; ++i)
                        u[e] = pk_fma(tkl[R + 2 * H - 2 - gi - i],
                                      *reinterpret_cast<const f2v*>(S + (i - R0 + R) * G::HCP + q), u[e]);
            }
        }
#pragma unroll
        for (int e = 0; e < STRIP; ++e) *reinterpret_cast<f2v*>(V + (i0 + e) * G::HCP + q) = u[e];
    }
}

// out[T] = horizontal adjoint of V (+ column folds in edge tiles); 4-wide items,
// float4 stores.
template <int R>
__device__ __forceinline__ void hadjoint_store(const float* V, int R0, int C0, int H, int W,
                                               const float (&tk)[2 * R + 1], const float* tkl,
                                               float* __restrict__ plane_out) {
    using G = BlurGeom<R>;
    constexpr int C4 = TW / 4;
    const bool cfold = C0 <= R || C0 + TW >= W - 1 - R;
    const bool vec = (W & 3) == 0 && (reinterpret_cast<uintptr_t>(plane_out) & 15) == 0;
    for (int it = threadIdx.x; it < TH * C4; it += kBlock) {
        const int i = it / C4, j0 = (it - i * C4) * 4;
        const int gi = R0 + i;
        if (gi >= H) continue;
        const float* row = V + i * G::HCP;
        float w[4 * G::NB];
        const float4* s4 = reinterpret_cast<const float4*>(row + j0);
#pragma unroll
        for (int j = 0; j < G::NB; ++j) {
            const float4 t = s4[j];
            w[4 * j] = t.x, w[4 * j + 1] = t.y, w[4 * j + 2] = t.z, w[4 * j + 3] = t.w;
        }
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float u = 0.f;
#pragma unroll
            for (int d = 0; d < G::K; ++d) u = fmaf(tk[d], w[e + 2 * R - d], u);
            o[e] = u;
        }
        if (cfold) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int gj = C0 + j0 + e;
                if (gj > 0 && gj <= R)
                    for (int c = 0; c <= R - gj; ++c)
                        o[e] = fmaf(tkl[R - gj - c], row[c - C0 + R], o[e]);
                if (gj < W - 1 && gj >= W - 1 - R)
                    for (int c = 2 * W - 2 - gj - R; c < W; ++c)
                        o[e] = fmaf(tkl[R + 2 * W - 2 - gj - c], row[c - C0 + R], o[e]);
            }
        }
        float* dst = plane_out + (unsigned)(gi * W + C0 + j0);
        if (vec && C0 + j0 + 4 <= W) {
            *reinterpret_cast<float4*>(dst) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (C0 + j0 + e < W) dst[e] = o[e];
        }
    }
}

template <int R, int MODE>
__global__ __launch_bounds__(kBlock) void k_blur(sp_op op, const float* __restrict__ in,
                                                 const float* __restrict__ eps,
                                                 const float* __restrict__ y, int y_div,
                                                 float a, float k, float gs,
                                                 float* __restrict__ out,
                                                 float* __restrict__ partial, int P,
                                                 const sp_step_rec* __restrict__ sched,
                                                 const int32_t* __restrict__ cursor) {
    using G = BlurGeom<R>;
    if (MODE == MODE_DPS && sched) {  // device-resident schedule (graph replay)
        const sp_dps_coefs& c = sched[*cursor].c;
        a = c.a, k = c.k, gs = c.grad_scale;
    }
    __shared__ __attribute__((aligned(16))) float bufA[G::LDS_A];
    __shared__ __attribute__((aligned(16))) float bufB[G::LDS_B];
    __shared__ float red[4];
    __shared__ float tkl[2 * R + 1];  // taps for the (lane-indexed) fold terms

    const int H = op.height, W = op.width, C = op.channels;
    const int tilesW = (W + TW - 1) / TW;
    const int tiles = tilesW * ((H + TH - 1) / TH);
    // XCD-aware order: dispatch deals blocks round-robin over the 8 XCDs, so give each
    // XCD a contiguous run of tiles (neighbours share halos through that XCD's L2).
    const unsigned nblk = gridDim.x;
    const unsigned q8 = nblk / 8, r8 = nblk % 8, xcd = blockIdx.x % 8, loc = blockIdx.x / 8;
    const unsigned lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    const unsigned pl = lin / tiles;  // plane index b*C + c
    const int tile = static_cast<int>(lin - pl * tiles);
    const int c = static_cast<int>(pl % C);
    const unsigned b = pl / C;
    const int R0 = (tile / tilesW) * TH, C0 = (tile % tilesW) * TW;
    const int64_t plane = (int64_t)H * W;
    const int64_t xoff = (int64_t)pl * plane;
    // uniform plane bases; per-element offsets are 32-bit (plane < 2^31 elements)
    const float* __restrict__ xp = in + xoff;
    const int tx = threadIdx.x % BX, ty = threadIdx.x / BX;

    float tk[2 * R + 1];  // uniform -> scalar loads
#pragma unroll
    for (int d = 0; d < 2 * R + 1; ++d) tk[d] = op.taps[d];
    if (threadIdx.x < 2 * R + 1) tkl[threadIdx.x] = op.taps[threadIdx.x];

    if constexpr (MODE == MODE_APPLY) {
        // X = x on T +- R (reflected); Hh = horizontal pass on those rows; out = vertical
        float* X = bufA;
        float* Hh = bufB;
        constexpr int XR = TH + 2 * R, XW = TW + 2 * R;
        for (int r = ty; r < XR; r += BY) {
            const unsigned gro = (unsigned)reflect_clamp(R0 - R + r, H) * W;
            for (int q = tx; q < XW; q += BX) X[r * G::XCP + q] = xp[gro + reflect_clamp(C0 - R + q, W)];
        }
        __syncthreads();
        hpass<R>(X, G::XCP, Hh, G::HCP, XR, TW / 4, tk);
        __syncthreads();
        constexpr int NS = TH / STRIP;
        for (int it = threadIdx.x; it < NS * TW; it += kBlock) {
            const int s = it / TW, q = it - s * TW;
            const int i0 = s * STRIP;
            if (C0 + q >= W) continue;
            float w[STRIP + 2 * R];
#pragma unroll
            for (int j = 0; j < STRIP + 2 * R; ++j) w[j] = Hh[(i0 + j) * G::HCP + q];
#pragma unroll
            for (int e = 0; e < STRIP; ++e) {
                const int gi = R0 + i0 + e;
                if (gi >= H) break;
                float acc = 0.f;
#pragma unroll
                for (int d = 0; d < G::K; ++d) acc = fmaf(tk[d], w[e + d], acc);
                (out + xoff)[(unsigned)(gi * W + C0 + q)] = acc;
            }
        }
        return;
    } else {
        float* S = bufA;  // T +- R rows x HC cols, stride HCP
        float racc = 0.f;
        if constexpr (MODE == MODE_ADJOINT) {
            for (int r = ty; r < G::SR; r += BY) {
                const int gi = R0 - R + r;
                for (int q = tx; q < G::HC; q += BX) {
                    const int gj = C0 - R + q;
                    const bool ok = gi >= 0 && gi < H && gj >= 0 && gj < W;
                    S[r * G::HCP + q] = ok ? xp[(unsigned)(gi * W + gj)] : 0.f;
                }
            }
            __syncthreads();
        } else {
            // ---- fused DPS residual pass ----
            const float* __restrict__ yp = y + ((int64_t)(b / (unsigned)y_div) * C + c) * plane;
            const float* __restrict__ ep = eps + xoff;
            float* X = bufA;
            float* Hh = bufB;
            const float inv_a = 1.f / a;  // x0 to 1 ulp of the division K2 uses
            static_assert(G::WR % BY == 0 && G::XC > BX && G::XC <= 2 * BX, "window layout");
            constexpr int NI = G::WR / BY;
            // Stage 1 loads: column tx for every window row, then column tx + 64 (a
            // duplicate, unused load on lanes past the window).  Rows are wave-uniform,
            // so the reflected row offset is a scalar (buffer-load soffset) and each
            // lane's reflected column a fixed voffset: no per-load vector address math.
            const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            const int nbytes = static_cast<int>(plane * 4);
            const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xp), (short)0, nbytes, 0x00020000);
            const auto er = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ep), (short)0, nbytes, 0x00020000);
            const int vo0 = 4 * reflect_clamp(C0 - 2 * R + tx, W);
            const int vo1 = 4 * reflect_clamp(C0 - 2 * R + tx + BX, W);
            const bool has1 = tx < G::XC - BX;
            float xv[NI][2], ev[NI][2];
#pragma unroll
            for (int it = 0; it < NI; ++it) {
                const int so = 4 * W * reflect_clamp(R0 - 2 * R + wv + BY * it, H);
                xv[it][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, vo0, so, 0));
                ev[it][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(er, vo0, so, 0));
                xv[it][1] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, vo1, so, 0));
                ev[it][1] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(er, vo1, so, 0));
            }
            // observation for this thread's stage-3 items (strip x column pair), prefetched
            // behind the window; addresses clamped into the image (off-image entries unused)
            constexpr bool EXACT3 = G::SR % STRIP == 0;
            constexpr int NS3 = (G::SR + STRIP - 1) / STRIP, HP = G::HC / 2;
            constexpr int NIT3 = (NS3 * HP + kBlock - 1) / kBlock;
            f2v yv[NIT3][STRIP];
#pragma unroll
            for (int u = 0; u < NIT3; ++u) {
                const int it = min((int)threadIdx.x + u * kBlock, NS3 * HP - 1);
                const int s = it / HP, q = 2 * (it - s * HP);
                const int gj0 = min(max(C0 - R + q, 0), W - 1), gj1 = min(max(C0 - R + q + 1, 0), W - 1);
#pragma unroll
                for (int e = 0; e < STRIP; ++e) {
                    const unsigned ro = (unsigned)min(max(R0 - R + s * STRIP + e, 0), H - 1) * W;
                    yv[u][e] = f2v{yp[ro + gj0], yp[ro + gj1]};
                }
            }
#pragma unroll
            for (int it = 0; it < NI; ++it) {
                const int r = wv + BY * it;
                X[r * G::XCP + tx] = (xv[it][0] - k * ev[it][0]) * inv_a;
                if (has1) X[r * G::XCP + tx + BX] = (xv[it][1] - k * ev[it][1]) * inv_a;
            }
            __syncthreads();
            hpass<R>(X, G::XCP, Hh, G::HCP, G::WR, G::HCP / 4, tk);
            __syncthreads();  // X is dead: S reuses bufA
#pragma unroll
            for (int u = 0; u < NIT3; ++u) {
                const int it = threadIdx.x + u * kBlock;
                if (it >= NS3 * HP) break;
                const int s = it / HP, q = 2 * (it - s * HP);
                const int i0 = s * STRIP;
                const int gj = C0 - R + q;
                const bool cin0 = gj >= 0 && gj < W, cin1 = gj + 1 >= 0 && gj + 1 < W;
                const bool cT0 = q >= R && q < R + TW, cT1 = q + 1 >= R && q + 1 < R + TW;
                f2v w[STRIP + 2 * R];
#pragma unroll
                for (int j = 0; j < STRIP + 2 * R; ++j)
                    w[j] = (EXACT3 || i0 + j < G::WR) ? *reinterpret_cast<const f2v*>(Hh + (i0 + j) * G::HCP + q)
                                                     : f2v{0.f, 0.f};
#pragma unroll
                for (int e = 0; e < STRIP; ++e) {
                    const int i = i0 + e;
                    if (!EXACT3 && i >= G::SR) break;
                    const int gi = R0 - R + i;
                    f2v z = {0.f, 0.f};
#pragma unroll
                    for (int d = 0; d < G::K; ++d) z = pk_fma(tk[d], w[e + d], z);
                    const f2v rr = yv[u][e] - z;
                    const bool rok = (unsigned)gi < (unsigned)H, rT = rok && i >= R && i < R + TH;
                    const f2v sv = rr * gs;
                    *reinterpret_cast<f2v*>(S + i * G::HCP + q) =
                        f2v{(rok && cin0) ? sv.x : 0.f, (rok && cin1) ? sv.y : 0.f};
                    racc += (rT && cT0 && cin0) ? rr.x * rr.x : 0.f;
                    racc += (rT && cT1 && cin1) ? rr.y * rr.y : 0.f;
                }
            }
            __syncthreads();  // Hh is dead: V reuses bufB
        }
        vadjoint<R>(S, bufB, R0, H, tk, tkl);
        if constexpr (MODE == MODE_DPS) {
            const float t = block_sum(racc, red);  // contains the barrier V needs
            if (threadIdx.x == 0) partial[(int64_t)b * P + c * tiles + tile] = t;
        } else {
            __syncthreads();
        }
        hadjoint_store<R>(bufB, R0, C0, H, W, tk, tkl, out + xoff);
    }
}

// ---------------------------------------------------------------------------
// Streaming DPS pass for 256-column planes (BASELINE config 3 and any H % SSEG == 0).
//
// One wave owns one SSEG-row segment of one channel plane and sweeps it from one end
// to the other; each lane owns 4 adjacent columns, so one wave-instruction moves one
// whole 1 KiB image row.  The vertical stencils run on rolling register windows (no
// vertical halo is recomputed inside a segment); the horizontal stencils exchange a
// row through LDS (one wave writes and reads it: no barrier).  Per chunk of DCH input
// rows g:
//   1  x0(g) = (x - k eps)/a on reflected row g; Hh(g) = horizontal A
//   2  z(g-R) = vertical A over Hh; S = c (y - z), 0 off the image; |r|^2
//   3  V(g-2R) = vertical A^T over S (edge rows: fold-corrected taps)
//   4  v(g-2R) = horizontal A^T over V (per-lane fold-corrected taps)
// The only redundant reads are the segment's vertical halo (4R rows of x / eps, 2R of
// y per SSEG rows); neighbouring segments sweep in opposite directions so both reach
// a shared boundary together and the second read of its halo hits L2.
// ---------------------------------------------------------------------------
#ifndef SP_BLUR_SEG
#define SP_BLUR_SEG 32
#endif
#ifndef SP_BLUR_STREAM
#define SP_BLUR_STREAM 1
#endif
constexpr int SSEG = SP_BLUR_SEG;  // output rows per wave
constexpr int SWID = 256;          // plane width served: 64 lanes x 4 columns
constexpr int SPAD = 4;            // window columns each side of a lane's 4 (R <= SPAD)

typedef float f4v __attribute__((ext_vector_type(4)));

__host__ __device__ inline bool blur_streams(const sp_op* op) {
    return SP_BLUR_STREAM && op->width == SWID && op->radius <= SPAD && op->height % SSEG == 0 &&
           op->height >= 2 * op->radius + 2;
}

// Tap of the fold-corrected adjoint: (A1^T s)(j) = sum_o T_j[o] s(j + o), |o| <= R,
// for the 1-D reflect-padded correlation over an extent of N (s = 0 off [0, N)):
// T_j[o] = t[R-o] + t[R-2j-o] (1 <= j <= R) + t[2N-2-2j+R-o] (N-1-R <= j <= N-2).
__device__ __forceinline__ float adj_tap(const float* t, int R, int N, int j, int o) {
    float v = t[R - o];
    if (j >= 1 && j <= R) {
        const int i = R - 2 * j - o;
        if (i >= 0 && i <= 2 * R) v += t[i];
    }
    if (j >= N - 1 - R && j <= N - 2) {
        const int i = 2 * N - 2 - 2 * j + R - o;
        if (i >= 0 && i <= 2 * R) v += t[i];
    }
    return v;
}

// LDS written by some lanes of a wave and read by others of the same wave: DS
// instructions of one wave execute in order, so only the compiler needs fencing.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------------------
// LDS-DMA ring: the x / eps / y rows of DSLOT-1 chunks are in flight as
// buffer_load_dwordx4 ... lds (one 1 KiB image row per wave-instruction, straight into
// a wave-private LDS ring, no VGPRs held).  The DMAs are issued from inline asm (the
// compiler would otherwise wait vmcnt(0) before every ds_read of the ring) and retired
// by counted s_waitcnt vmcnt(N) = the exact number of younger vector memory
// operations (later DMAs and the v stores in between).  The exchange rows live in
// place in the consumed slot's x rows.  Window rows rotate through the registers with
// period WIN / gcd(WIN, DCH) (the chunk body is instantiated per phase), so no
// register moves shift them.
// ---------------------------------------------------------------------------
#ifndef SP_BLUR_CHUNK
#define SP_BLUR_CHUNK 2
#endif
constexpr int DCH = SP_BLUR_CHUNK;  // rows per chunk
#ifndef SP_BLUR_SLOTS
#define SP_BLUR_SLOTS 4
#endif
constexpr int DSLOT = SP_BLUR_SLOTS;  // ring slots: DSLOT - 1 chunks in flight
constexpr int DROWS = 3 * DCH;    // x, eps, y rows per slot
constexpr int DRING = DSLOT * DROWS * SWID;

// one 1 KiB row: buffer_load_dwordx4 ... lds, row offset in soffset (scalar), lane offset
// in a fixed VGPR, LDS destination = M0 + 16 * lane
__device__ __forceinline__ void dma_row(__amdgpu_buffer_rsrc_t rsrc, uint32_t voff, uint32_t soff,
                                        uint32_t lds_byte) {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, %3 offen lds\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds_byte)
        : "memory");
}

// s_waitcnt vmcnt(n) for the even n a chunk can leave younger (<= 62, the counter's range)
__device__ __forceinline__ void wait_vm(int n) {
    switch (n) {
#define SP_VM(N) \
    case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
        SP_VM(0) SP_VM(2) SP_VM(4) SP_VM(6) SP_VM(8) SP_VM(10) SP_VM(12) SP_VM(14)
        SP_VM(16) SP_VM(18) SP_VM(20) SP_VM(22) SP_VM(24) SP_VM(26) SP_VM(28) SP_VM(30)
        SP_VM(32) SP_VM(34) SP_VM(36) SP_VM(38) SP_VM(40) SP_VM(42) SP_VM(44) SP_VM(46)
        SP_VM(48) SP_VM(50) SP_VM(52) SP_VM(54) SP_VM(56) SP_VM(58) SP_VM(60) SP_VM(62)
#undef SP_VM
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}

constexpr int gcd_c(int a, int b) { return b == 0 ? a : gcd_c(b, a % b); }

// f(phase P0), f(P0 + 1), ..., f(N - 1) on chunks cc + P0, ... (compile-time phases)
template <int P0, int N, class F>
__device__ __forceinline__ void phases(F& f, int cc) {
    if constexpr (P0 < N) {
        f(std::integral_constant<int, P0>{}, cc + P0);
        phases<P0 + 1, N>(f, cc);
    }
}

template <int R>
__global__ __launch_bounds__(64) void k_blur_dps_dma(
    sp_op op, const float* __restrict__ x, const float* __restrict__ eps,
    const float* __restrict__ y, int y_div, float a, float k, float gs, float* __restrict__ out,
    float* __restrict__ partial, int P, unsigned units, const sp_step_rec* __restrict__ sched,
    const int32_t* __restrict__ cursor) {
    constexpr int K = 2 * R + 1, CH = DCH, WIN = CH + 2 * R, NCH = (SSEG + 4 * R) / CH;
    constexpr int C2 = (2 * R) / CH, C3 = (4 * R) / CH, PER = WIN / gcd_c(WIN, CH);
    static_assert(SSEG % CH == 0 && (4 * R) % CH == 0 && R >= 1 && R <= SPAD, "dma geometry");
    static_assert(DROWS * (DSLOT - 1) + CH * (DSLOT - 1) <= 62 && DROWS % 2 == 0 && CH % 2 == 0, "vmcnt cases");
    if (sched) {
        const sp_dps_coefs& cf = sched[*cursor].c;
        a = cf.a, k = cf.k, gs = cf.grad_scale;
    }
    __shared__ __attribute__((aligned(16))) float lds[DRING + 8];
    __shared__ float tl[2][K];  // taps, and reversed (vertical taps of a bottom-up sweep)
    float* ring = lds + 4;  // guards either side: lanes 0 / 63 read one float4 past a row
    const int lane = threadIdx.x;
    if (lane < K) tl[0][lane] = tl[1][K - 1 - lane] = op.taps[lane];
    __syncthreads();

    const int H = op.height, C = op.channels, nseg = H / SSEG;
    const unsigned nblk = gridDim.x;
    const unsigned q8 = nblk / 8, r8 = nblk % 8, xcd = blockIdx.x % 8, loc = blockIdx.x / 8;
    const unsigned u = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    if (u >= units) return;
    const unsigned pl = u / nseg;
    const int sg = static_cast<int>(u - pl * nseg);
    const int c = static_cast<int>(pl % C);
    const unsigned b = pl / C;
    // Odd segments sweep bottom-up (mirrored rows and vertical taps; the reflect-padded
    // blur is mirror-symmetric), so the two waves that read the halo rows of a segment
    // boundary both reach it at the start, or both at the end, of their sweeps and the
    // second read hits L2.  Row indices below are sweep coordinates; prow() maps them.
    const bool flip = sg & 1;
    const int s0 = flip ? H - (sg + 1) * SSEG : sg * SSEG;
    auto prow = [&](int g) { return flip ? H - 1 - g : g; };
    const float* tlv = tl[flip ? 1 : 0];
    const int64_t plane = (int64_t)H * SWID;
    const float* __restrict__ xp = x + pl * plane;
    const float* __restrict__ ep = eps + pl * plane;
    const float* __restrict__ yp = y + ((int64_t)(b / (unsigned)y_div) * C + c) * plane;
    float* __restrict__ op_out = out + pl * plane;
    const int col = 4 * lane;
    const uint32_t voff = 16u * lane;
    const uint32_t ring_b =
        static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float*)ring));

    float tk[K];
#pragma unroll
    for (int d = 0; d < K; ++d) tk[d] = op.taps[d];
    float tv[K];  // vertical taps in sweep order
#pragma unroll
    for (int d = 0; d < K; ++d) tv[d] = flip ? tk[K - 1 - d] : tk[d];
    float th[4][K];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int o = -R; o <= R; ++o) th[e][o + R] = adj_tap(tl[0], R, SWID, col + e, o);
    const float inv_a = 1.f / a;

    const int pbytes = static_cast<int>(plane * 4);
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xp), (short)0, pbytes, 0x00020000);
    const auto er = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ep), (short)0, pbytes, 0x00020000);
    const auto yr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(yp), (short)0, pbytes, 0x00020000);
    auto issue = [&](int cc) {
        const int s = cc % DSLOT;
#pragma unroll
        for (int e = 0; e < CH; ++e) {
            const int gi = s0 - 2 * R + CH * cc + e;
            const int gr = reflect_clamp(gi, H);
            const int gy = min(max(gi - R, 0), H - 1);
            const uint32_t rb = ring_b + 4u * ((s * DROWS + e) * SWID);
            const uint32_t ox = 4u * SWID * prow(gr), oy = 4u * SWID * prow(gy);
            dma_row(xr, voff, ox, rb);
            dma_row(er, voff, ox, rb + 4u * CH * SWID);
            dma_row(yr, voff, oy, rb + 8u * CH * SWID);
        }
    };
#pragma unroll
    for (int cc = 0; cc < DSLOT - 1; ++cc)
        if (cc < NCH) issue(cc);

    f4v hw[WIN], sw[WIN];
#pragma unroll
    for (int j = 0; j < WIN; ++j) hw[j] = sw[j] = f4v{0.f, 0.f, 0.f, 0.f};
    float racc = 0.f;

    auto read_win = [&](const float* row, float (&w)[12]) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const f4v t = *reinterpret_cast<const f4v*>(row + col - SPAD + 4 * q);
            w[4 * q] = t.x, w[4 * q + 1] = t.y, w[4 * q + 2] = t.z, w[4 * q + 3] = t.w;
        }
    };

    auto body = [&](auto phc, int cc) {
        constexpr int PH = decltype(phc)::value;
        auto ix = [](int j) { return (j + PH * CH) % WIN; };  // logical window row -> register slot
        // slot of chunk cc-1 is refilled below: its exchange reads must have returned
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (cc + DSLOT - 1 < NCH) issue(cc + DSLOT - 1);
        {   // retire chunk cc's DMAs: younger = later chunks' DMAs + v stores issued since
            const int later = min(DSLOT - 1, NCH - 1 - cc);
            const int st = max(0, min(cc, DSLOT - 1) - max(0, C3 - (cc - min(cc, DSLOT - 1))));
            wait_vm(DROWS * later + CH * st);
        }
        float* xrow = ring + (cc % DSLOT) * DROWS * SWID;  // x rows, then exchange rows
        const float* erow = xrow + CH * SWID;
        const float* yrow = xrow + 2 * CH * SWID;

        // ---- 1: x0 (in place), horizontal A ----
        f4v x0[CH];
#pragma unroll
        for (int e = 0; e < CH; ++e) {
            const f4v xv = *reinterpret_cast<const f4v*>(xrow + e * SWID + col);
            const f4v ev = *reinterpret_cast<const f4v*>(erow + e * SWID + col);
            x0[e] = (xv - k * ev) * inv_a;
        }
        wave_lds_sync();
#pragma unroll
        for (int e = 0; e < CH; ++e) *reinterpret_cast<f4v*>(xrow + e * SWID + col) = x0[e];
        wave_lds_sync();
#pragma unroll
        for (int e = 0; e < CH; ++e) {
            float w[12];
            read_win(xrow + e * SWID, w);
#pragma unroll
            for (int i = 1; i <= R; ++i) {  // reflect padding at the side edges
                w[SPAD - i] = lane == 0 ? w[SPAD + i] : w[SPAD - i];
                w[SPAD + 3 + i] = lane == 63 ? w[SPAD + 3 - i] : w[SPAD + 3 + i];
            }
            f4v h;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float acc = 0.f;
#pragma unroll
                for (int d = 0; d < K; ++d) acc = fmaf(tk[d], w[SPAD - R + q + d], acc);
                h[q] = acc;
            }
            hw[ix(2 * R + e)] = h;
        }
        if (cc < C2) return;

        // ---- 2: vertical A, residual, S, |r|^2 ----
#pragma unroll
        for (int e = 0; e < CH; ++e) {
            const int gz = s0 - 3 * R + CH * cc + e;
            f4v z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int d = 0; d < K; ++d) z += tv[d] * hw[ix(e + d)];
            const f4v rr = *reinterpret_cast<const f4v*>(yrow + e * SWID + col) - z;
            const bool in = (unsigned)gz < (unsigned)H;
            sw[ix(2 * R + e)] = in ? rr * gs : f4v{0.f, 0.f, 0.f, 0.f};
            if (gz >= s0 && gz < s0 + SSEG)
                racc += (rr.x * rr.x + rr.y * rr.y) + (rr.z * rr.z + rr.w * rr.w);
        }
        if (cc < C3) return;

        // ---- 3: vertical A^T ----
        const int gv0 = s0 - 4 * R + CH * cc;
        f4v vv[CH];
        if (gv0 > R && gv0 + CH - 1 < H - 1 - R) {
#pragma unroll
            for (int e = 0; e < CH; ++e) {
                f4v u4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = 0; i < K; ++i) u4 += tv[i] * sw[ix(e + 2 * R - i)];
                vv[e] = u4;
            }
        } else {
#pragma unroll
            for (int e = 0; e < CH; ++e) {
                f4v u4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int o = -R; o <= R; ++o) u4 += adj_tap(tlv, R, H, gv0 + e, o) * sw[ix(e + R + o)];
                vv[e] = u4;
            }
        }

        // ---- 4: horizontal A^T through the exchange rows, store v ----
        wave_lds_sync();
#pragma unroll
        for (int e = 0; e < CH; ++e) *reinterpret_cast<f4v*>(xrow + e * SWID + col) = vv[e];
        wave_lds_sync();
#pragma unroll
        for (int e = 0; e < CH; ++e) {
            float w[12];
            read_win(xrow + e * SWID, w);
#pragma unroll
            for (int i = 0; i < SPAD; ++i) {  // V = 0 off the image
                w[i] = lane == 0 ? 0.f : w[i];
                w[SPAD + 4 + i] = lane == 63 ? 0.f : w[SPAD + 4 + i];
            }
            f4v o4;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float acc = 0.f;
#pragma unroll
                for (int o = -R; o <= R; ++o) acc = fmaf(th[q][o + R], w[SPAD + q + o], acc);
                o4[q] = acc;
            }
            *reinterpret_cast<f4v*>(op_out + prow(gv0 + e) * SWID + col) = o4;
        }
    };

    int cc = 0;
    for (; cc + PER <= NCH; cc += PER) phases<0, PER>(body, cc);
    phases<0, NCH % PER>(body, cc);
    racc = wave_sum(racc);
    if (lane == 0) partial[(int64_t)b * P + c * nseg + sg] = racc;
}

// ---------------------------------------------------------------------------
// Register-streamed DPS pass (the default for 256-column planes; k_blur_dps_dma above is the
// LDS-DMA form it replaced, kept selectable with -DSP_BLUR_REG=0).  Same sweep, same
// segment / flip geometry and the same arithmetic order per element; what changed is how
// the wave spends its instruction issue, which (not HBM) bounded the DMA form: ~10.3 k
// instructions per wave at 1.5 waves per SIMD, a third of them scalar bookkeeping (M0
// juggling per DMA, run-time chunk-phase tests, a vmcnt switch) — PMC, round 2.
//   * the whole sweep is unrolled at compile time (chunk index, stage presence, the |r|^2
//     rows, the edge cases are constants; the vertical windows are arrays with constant
//     indices, i.e. registers; the compiler derives every vmcnt wait);
//   * x, eps and y rows go straight to VGPRs (buffer_load_dwordx4, row offset in soffset),
//     PF chunks ahead; LDS holds only the two exchange rows of the horizontal passes;
//   * the horizontal forward pass runs on row pairs: the chunk's two x0 rows are exchanged
//     interleaved ({row0, row1} per column), so each window column is one aligned register
//     pair and one v_pk_fma_f32 applies a tap to both rows (18 per row instead of 36 FMAs);
//   * the horizontal adjoint (per-lane fold-corrected taps) runs on column pairs: the V row
//     is exchanged twice, as is and shifted by one column, so that the column pair at every
//     tap offset is an aligned register pair of one of the two windows; V's off-image
//     columns are zero pads written once.
// Requires an even number of segments per plane (H / SSEG), so that in sweep coordinates no
// segment reaches the bottom edge (the flip maps the last segment to the top).
// ---------------------------------------------------------------------------
#ifndef SP_BLUR_REG
#define SP_BLUR_REG 1
#endif
#ifndef SP_BLUR_PF
#define SP_BLUR_PF 1
#endif
#ifndef SP_BLUR_LDSWAIT
#define SP_BLUR_LDSWAIT 0
#endif
#ifndef SP_BLUR_HADJ
#define SP_BLUR_HADJ 0
#endif
#ifndef SP_BLUR_NT
#define SP_BLUR_NT 2  // aux (cache policy) bits for the loads of rows only this segment reads
#endif
#ifndef SP_BLUR_NTST
#define SP_BLUR_NTST 0  // aux bits of the v stores
#endif
#ifndef SP_BLUR_G
#define SP_BLUR_G 1  // waves (segments) per workgroup of the register-streamed pass
#endif
#ifndef SP_BLUR_DBG
#define SP_BLUR_DBG 0  // 1: store the vertical adjoint V (before the horizontal pass) as v
#endif

template <int N>
using ic_t = std::integral_constant<int, N>;

template <class F, int... I>
__device__ __forceinline__ void unroll_seq(F& f, std::integer_sequence<int, I...>) {
    (f(ic_t<I>{}), ...);
}

typedef float f2v_t __attribute__((ext_vector_type(2)));
typedef unsigned u4v_t __attribute__((ext_vector_type(4)));

// G waves per workgroup: G = 2 puts the two segments that END their sweeps at a shared boundary
// (an even segment sweeping down, the odd one below it sweeping up) on one CU, so they reach
// their shared halo rows together and the second read is served by the CU's L2 (separately
// placed, their progress drifts apart over the sweep and part of those reads went to HBM)
template <int R, int SEG, int G>
__global__ __launch_bounds__(64 * G, 2) void k_blur_dps_reg(
    sp_op op, const float* __restrict__ x, const float* __restrict__ eps,
    const float* __restrict__ y, int y_div, float a, float k, float gs, float* __restrict__ out,
    float* __restrict__ partial, int P, unsigned units, const sp_step_rec* __restrict__ sched,
    const int32_t* __restrict__ cursor) {
    constexpr int K = 2 * R + 1, CH = 2, NCH = (SEG + 4 * R) / CH, NR = NCH * CH;
    constexpr int C2 = 2 * R / CH, C3 = 4 * R / CH, PF = SP_BLUR_PF;
    static_assert((4 * R) % CH == 0 && SEG % CH == 0 && R >= 1 && R <= SPAD, "geometry");
    if (sched) {
        const sp_dps_coefs& cf = sched[*cursor].c;
        a = cf.a, k = cf.k, gs = cf.grad_scale;
    }
    constexpr int XS = SWID + 2 * SPAD;  // exchange row stride (columns -SPAD .. SWID+SPAD-1)
    __shared__ __attribute__((aligned(16))) float xbs[G][2 * XS];    // x0 row pair, interleaved
    __shared__ __attribute__((aligned(16))) float vbs[G][2][2][XS];  // V rows: [row][as is / shifted]
    __shared__ float tl[2][K];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) >> 6);
    float* xb = xbs[wv];
    float (*vb)[2][XS] = vbs[wv];
    if (threadIdx.x < K) tl[0][threadIdx.x] = tl[1][K - 1 - threadIdx.x] = op.taps[threadIdx.x];
    // V = 0 off the image: the row writes never touch the pads (as-is copy: indices < SPAD and
    // >= SWID + SPAD; shifted copy: < SPAD - 1 and >= SWID + SPAD - 1), so zero them once
    for (int i = threadIdx.x; i < G * 4 * XS; i += 64 * G) (&vbs[0][0][0][0])[i] = 0.f;
    __syncthreads();

    const int H = op.height, C = op.channels, nseg = H / SEG;
    const unsigned nblk = gridDim.x;
    const unsigned q8 = nblk / 8, r8 = nblk % 8, xcd = blockIdx.x % 8, loc = blockIdx.x / 8;
    const unsigned u = ((xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc) * G + wv;
    if (u >= units) return;
    const unsigned pl = u / nseg;
    const int sg = static_cast<int>(u - pl * nseg);
    const int c = static_cast<int>(pl % C);
    const unsigned b = pl / C;
    const bool flip = sg & 1;  // odd segments sweep bottom-up (see k_blur_dps_dma)
    const int s0 = flip ? H - (sg + 1) * SEG : sg * SEG;
    const bool top = s0 == 0;  // the only segments that meet an image edge in sweep coordinates
    // the unit's segment inside its plane, the plane inside the batch, partials in range
    SP_DCHECK(s0 >= 0 && s0 + SEG <= H && H % SEG == 0 && op.width == SWID && c < C &&
              c * nseg + sg < P && (int64_t)b * C * nseg < (int64_t)units);
    const int64_t plane = (int64_t)H * SWID;
    const int pbytes = static_cast<int>(plane * 4);
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x + pl * plane), (short)0, pbytes, 0x00020000);
    const auto er = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(eps + pl * plane), (short)0, pbytes, 0x00020000);
    const auto yr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(y + ((int64_t)(b / (unsigned)y_div) * C + c) * plane), (short)0, pbytes, 0x00020000);
    const auto vr = __builtin_amdgcn_make_buffer_rsrc(out + pl * plane, (short)0, pbytes, 0x00020000);
    const int col = 4 * lane;
    const uint32_t voff = 16u * lane;
    // physical byte offset of sweep row g (0 <= g < H); rows above the top reflect
    const int rbase = flip ? (H - 1) * SWID * 4 : 0, rstep = flip ? -SWID * 4 : SWID * 4;
    auto row_off = [&](int g) { return rbase + rstep * g; };

    float tk[K], tv[K];
#pragma unroll
    for (int d = 0; d < K; ++d) tk[d] = op.taps[d];
#pragma unroll
    for (int d = 0; d < K; ++d)  // wave-uniform: keep them scalar (SGPR pairs for v_pk_fma_f32)
        tv[d] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(
                                              __builtin_bit_cast(int, flip ? tk[K - 1 - d] : tk[d])));
    f2v_t th01[K], th23[K];  // per-lane fold-corrected adjoint taps, column pairs (q0,q1), (q2,q3)
#pragma unroll
    for (int o = -R; o <= R; ++o) {
        th01[o + R] = f2v_t{adj_tap(tl[0], R, SWID, col, o), adj_tap(tl[0], R, SWID, col + 1, o)};
        th23[o + R] = f2v_t{adj_tap(tl[0], R, SWID, col + 2, o), adj_tap(tl[0], R, SWID, col + 3, o)};
    }
    const float inv_a = 1.f / a;

    f4v px[NCH][CH], pe[NCH][CH], py[NCH][CH];  // constant indices only: registers
    f4v hw[NR], sw[NR];
    f4v racc = {0.f, 0.f, 0.f, 0.f};

    auto issue = [&](auto icc) __attribute__((always_inline)) {
        constexpr int cc = decltype(icc)::value;
        if constexpr (cc < NCH) {
#pragma unroll
            for (int e = 0; e < CH; ++e) {
                const int gi = s0 - 2 * R + CH * cc + e;  // sweep row
                int gr = gi;
                if (CH * cc + CH <= 2 * R) gr = gi < 0 ? -gi : gi;  // top reflection (s0 == 0)
                const int so = row_off(gr);
                // rows no other segment reads (not within 4R rows of either end of the sweep)
                // may stream past the L2; the shared halo rows keep the default policy
                constexpr int ri0 = CH * cc;
                constexpr int AUX = (SP_BLUR_NT && ri0 >= 4 * R && ri0 + CH <= NR - 4 * R) ? SP_BLUR_NT : 0;
                constexpr int AUXY = (SP_BLUR_NT && ri0 >= 4 * R && ri0 + CH <= NR - 2 * R) ? SP_BLUR_NT : 0;
                px[cc][e] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(xr, voff, so, AUX));
                pe[cc][e] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(er, voff, so, AUX));
                if (cc >= C2) {  // y rows are first used by stage 2 (rows above the image: unused)
                    const int gy = max(gi - R, 0);
                    py[cc][e] = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(yr, voff, row_off(gy), AUXY));
                }
            }
        }
    };

    auto body = [&](auto icc) __attribute__((always_inline)) {
        constexpr int cc = decltype(icc)::value;
        issue(ic_t<cc + PF>{});
        // ---- 1: x0, horizontal A on the row pair ----
        {
            f4v x0[CH];
#pragma unroll
            for (int e = 0; e < CH; ++e) x0[e] = (px[cc][e] - k * pe[cc][e]) * inv_a;
            wave_lds_sync();
            float* dst = xb + 2 * (col + SPAD);
            *reinterpret_cast<f4v*>(dst) = f4v{x0[0].x, x0[1].x, x0[0].y, x0[1].y};
            *reinterpret_cast<f4v*>(dst + 4) = f4v{x0[0].z, x0[1].z, x0[0].w, x0[1].w};
            wave_lds_sync();
            f2v_t W[12];
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                const f4v t = *reinterpret_cast<const f4v*>(xb + 2 * col + 4 * q);
                W[2 * q] = f2v_t{t.x, t.y};
                W[2 * q + 1] = f2v_t{t.z, t.w};
            }
#pragma unroll
            for (int i = 1; i <= R; ++i) {  // reflect padding at the side edges
                W[SPAD - i] = lane == 0 ? W[SPAD + i] : W[SPAD - i];
                W[SPAD + 3 + i] = lane == 63 ? W[SPAD + 3 - i] : W[SPAD + 3 + i];
            }
            f2v_t acc[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f2v_t s = {0.f, 0.f};
#pragma unroll
                for (int d = 0; d < K; ++d) s = __builtin_elementwise_fma(f2v_t{tk[d], tk[d]}, W[SPAD - R + q + d], s);
                acc[q] = s;
            }
            hw[CH * cc] = f4v{acc[0].x, acc[1].x, acc[2].x, acc[3].x};
            hw[CH * cc + 1] = f4v{acc[0].y, acc[1].y, acc[2].y, acc[3].y};
        }
        // ---- 2: vertical A, residual, S, |r|^2 ----
        if constexpr (cc >= C2) {
#pragma unroll
            for (int e = 0; e < CH; ++e) {
                constexpr int g0 = CH * cc - R;  // z row (loaded-row index) of e = 0
                const int g = g0 + e;
                f4v z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int d = 0; d < K; ++d) z += tv[d] * hw[g - R + d];
                const f4v rr = py[cc][e] - z;
                // global sweep row s0 - 2R + g: above the image only in a top segment
                const bool in = (g0 + e >= 2 * R) || !top;
                sw[g] = in ? rr * gs : f4v{0.f, 0.f, 0.f, 0.f};
                if (g >= 2 * R && g < 2 * R + SEG) racc += rr * rr;
            }
        }
        // ---- 3: vertical A^T; 4: horizontal A^T, store v ----
        if constexpr (cc >= C3) {
#pragma unroll
            for (int e = 0; e < CH; ++e) {
                const int h = CH * cc - 2 * R + e;  // v row (loaded-row index); sweep row s0 + h - 2R
                f4v vv = {0.f, 0.f, 0.f, 0.f};
                if (CH * cc - 4 * R + e <= R && top) {  // near the top edge: folded taps
#pragma unroll
                    for (int o = -R; o <= R; ++o)
                        vv += adj_tap(tl[flip ? 1 : 0], R, H, CH * cc - 4 * R + e, o) * sw[h + o];
                } else {
#pragma unroll
                    for (int i = 0; i < K; ++i) vv += tv[i] * sw[h + R - i];
                }
                wave_lds_sync();
                *reinterpret_cast<f4v*>(&vb[e][0][col + SPAD]) = vv;
                float* s1 = &vb[e][1][col + SPAD - 1];  // shifted copy: column c at c + SPAD - 1
                s1[0] = vv.x, s1[1] = vv.y, s1[2] = vv.z, s1[3] = vv.w;
                if (SP_BLUR_LDSWAIT) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                wave_lds_sync();
                f2v_t wn[6], ws[6];  // wn[i] = V(col-SPAD+2i, +1); ws[i] = V(col-SPAD+2i+1, +2)
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const f4v t0 = *reinterpret_cast<const f4v*>(&vb[e][0][col + 4 * q]);
                    const f4v t1 = *reinterpret_cast<const f4v*>(&vb[e][1][col + 4 * q]);
                    wn[2 * q] = f2v_t{t0.x, t0.y}, wn[2 * q + 1] = f2v_t{t0.z, t0.w};
                    ws[2 * q] = f2v_t{t1.x, t1.y}, ws[2 * q + 1] = f2v_t{t1.z, t1.w};
                }
                // window index j = SPAD + q + o holds V(col + q + o); pair (j, j+1) lives in wn
                // (j even) or ws (j odd)
                auto pair = [&](int j) { return (j & 1) ? ws[j >> 1] : wn[j >> 1]; };
                f2v_t o01 = {0.f, 0.f}, o23 = {0.f, 0.f};
                if (SP_BLUR_HADJ == 0) {
#pragma unroll
                    for (int o = -R; o <= R; ++o) {
                        o01 = __builtin_elementwise_fma(th01[o + R], pair(SPAD + o), o01);
                        o23 = __builtin_elementwise_fma(th23[o + R], pair(SPAD + 2 + o), o23);
                    }
                } else if (SP_BLUR_HADJ == 1) {
                    float w[12];
#pragma unroll
                    for (int i = 0; i < 6; ++i) w[2 * i] = wn[i].x, w[2 * i + 1] = wn[i].y;
                    float oo[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        float acc = 0.f;
#pragma unroll
                        for (int o = -R; o <= R; ++o)
                            acc = fmaf(q < 2 ? (q == 0 ? th01[o + R].x : th01[o + R].y)
                                             : (q == 2 ? th23[o + R].x : th23[o + R].y),
                                       w[SPAD + q + o], acc);
                        oo[q] = acc;
                    }
                    o01 = f2v_t{oo[0], oo[1]}, o23 = f2v_t{oo[2], oo[3]};
                } else {
#pragma unroll
                    for (int o = -R; o <= R; ++o) {
                        o01 = __builtin_elementwise_fma(f2v_t{tk[R - o], tk[R - o]}, pair(SPAD + o), o01);
                        o23 = __builtin_elementwise_fma(f2v_t{tk[R - o], tk[R - o]}, pair(SPAD + 2 + o), o23);
                    }
                }
                const int gv = s0 - 2 * R + h;
                const f4v res = SP_BLUR_DBG == 1 ? vv : f4v{o01.x, o01.y, o23.x, o23.y};
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v_t, res), vr, voff,
                                                       row_off(gv), SP_BLUR_NTST);
                // hipcc (ROCm 7.2) lets the next instruction overwrite a buffer_store_dwordx4's data
                // VGPRs with no wait state; the store then reads some lanes' data after the write
                // (seen as corrupt lanes of the stored row).  Keep the data live across two wait
                // states (tools/store_hazard_scan.py checks the built code).
                asm volatile("s_nop 1" ::"v"(res) : "memory");
            }
        }
    };

    unroll_seq(issue, std::make_integer_sequence<int, PF>{});
    unroll_seq(body, std::make_integer_sequence<int, NCH>{});
    float t = (racc.x + racc.y) + (racc.z + racc.w);
    t = wave_sum(t);
    if (lane == 0) partial[(int64_t)b * P + c * nseg + sg] = t;
}

int64_t blur_partials(const sp_op* op) {
    if (blur_streams(op)) return (int64_t)op->channels * (op->height / SSEG);
    const int64_t tiles = (int64_t)((op->height + TH - 1) / TH) * ((op->width + TW - 1) / TW);
    return tiles * op->channels;
}

template <int MODE>
static int launch_blur(const sp_op* op, const float* in, const float* eps, const float* y,
                       int64_t y_div, float a, float k, float gs, float* out, float* partial,
                       int64_t batch, hipStream_t s, const sp_step_rec* sched = nullptr,
                       const int32_t* cursor = nullptr) {
    const int64_t tiles = (int64_t)((op->height + TH - 1) / TH) * ((op->width + TW - 1) / TW);
    const int64_t blocks = tiles * op->channels * batch;
    // the kernel decodes blocks and in-plane offsets in 32 bits
    if (blocks >= (int64_t(1) << 31) || (int64_t)op->height * op->width >= (int64_t(1) << 31) ||
        y_div < 1 || y_div > batch)
        return SP_EINVAL;
    if (blocks == 0) return SP_OK;
    const int P = static_cast<int>(blur_partials(op));
    if (MODE == MODE_DPS && blur_streams(op)) {
        const int64_t units = (int64_t)op->channels * (op->height / SSEG) * batch;
        if (SP_BLUR_REG && (op->height / SSEG) % 2 == 0) {
            switch (op->radius) {
#define SP_REG_CASE(RR)                                                                         \
    case RR:                                                                                    \
        launch_w(TK_DPS_RESIDUAL, (double)batch, k_blur_dps_reg<RR, SSEG, SP_BLUR_G>,           \
                 dim3(static_cast<unsigned>(units / SP_BLUR_G)), dim3(64 * SP_BLUR_G), s, *op, in, eps, y, \
                 static_cast<int>(y_div), a, k, gs, out, partial, P,                            \
                 static_cast<unsigned>(units), sched, cursor);                                  \
        break;
                SP_REG_CASE(1) SP_REG_CASE(2) SP_REG_CASE(3) SP_REG_CASE(4)
#undef SP_REG_CASE
                default: return SP_EINVAL;
            }
            return check_launch("blur_stream_reg");
        }
        switch (op->radius) {
#define SP_STREAM_CASE(RR)                                                                      \
    case RR:                                                                                    \
        launch_w(TK_DPS_RESIDUAL, (double)batch, k_blur_dps_dma<RR>,                            \
                 dim3(static_cast<unsigned>(units)), dim3(64), s, *op, in, eps, y,              \
                 static_cast<int>(y_div), a, k, gs, out, partial, P,                            \
                 static_cast<unsigned>(units), sched, cursor);                                  \
        break;
            SP_STREAM_CASE(1) SP_STREAM_CASE(2) SP_STREAM_CASE(3) SP_STREAM_CASE(4)
#undef SP_STREAM_CASE
            default: return SP_EINVAL;
        }
        return check_launch("blur_stream");
    }
    const dim3 grid(static_cast<unsigned>(blocks));
    switch (op->radius) {
#define SP_BLUR_CASE(RR)                                                                        \
    case RR:                                                                                    \
        launch_w(MODE == MODE_DPS ? TK_DPS_RESIDUAL : 0, (double)batch, k_blur<RR, MODE>, grid, dim3(kBlock), s, \
               *op, in, eps, y, static_cast<int>(y_div), a, k, gs, out, partial, P, sched, cursor); \
        break;
        SP_BLUR_CASE(1) SP_BLUR_CASE(2) SP_BLUR_CASE(3) SP_BLUR_CASE(4)
        SP_BLUR_CASE(5) SP_BLUR_CASE(6) SP_BLUR_CASE(7) SP_BLUR_CASE(8)
#undef SP_BLUR_CASE
        default: return SP_EINVAL;
    }
    return check_launch("blur");
}

int blur_dps_residual(const sp_op* op, const float* x, const float* eps, const float* y,
                      int64_t batch, int64_t y_div, float a, float k, float gs,
                      const sp_step_rec* sched, const int32_t* cursor, float* v, float* partial,
                      hipStream_t s) {
    return launch_blur<MODE_DPS>(op, x, eps, y, y_div, a, k, gs, v, partial, batch, s, sched,
                                 cursor);
}

int blur_apply(const sp_op* op, const float* x, float* y, int64_t batch, hipStream_t s) {
    return launch_blur<MODE_APPLY>(op, x, nullptr, nullptr, 1, 1.f, 0.f, 0.f, y, nullptr, batch, s);
}

int blur_adjoint(const sp_op* op, const float* y, float* x, int64_t batch, hipStream_t s) {
    return launch_blur<MODE_ADJOINT>(op, y, nullptr, nullptr, 1, 1.f, 0.f, 0.f, x, nullptr, batch,
                                     s);
}

}  // namespace sp

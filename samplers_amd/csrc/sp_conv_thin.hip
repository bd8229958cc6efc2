// 3x3 / stride 1 / pad 1 convolutions with few channels on one side: the priors' conv_in
// (3 or 4 input channels) and conv_out (3 or 8 output channels) and their input VJPs
// (any side with at most 8 channels)
// (diffusers UNet2DModel / AutoencoderKL, reached from ddpm.py:40-43 and
// stable_diffusion.py:330-345).  MIOpen runs them through NHWC implicit GEMMs with layout
// transposes, or its naive kernel (decoder conv_out at 512^2: ~1.5 ms per 4 images).
//
// The work is ~14 k FMA per output pixel at most and the memory traffic is the wide side's
// tensor, so this is a VALU direct convolution: one workgroup = a 16 x 64 pixel tile of one
// image x CO output channels; input channels are walked in chunks of CI, each chunk's
// 18 x 66 patch (zero outside the image = the padding) staged in LDS with float4 row
// pieces (W % 4 == 0).  Every thread owns four horizontally adjacent pixels x CO outputs:
// per channel and window row it reads its 6 window values as one ds_read_b128 and two
// ds_read_b32 and runs the taps as packed FMAs on pixel pairs (v_pk_fma_f32, the weight
// broadcast from an SGPR), so the VALU work is half that of scalar FMAs and the LDS reads
// per pixel a third of a 2-pixel layout's.  The next chunk's patch is loaded into registers
// while the current one is computed.  The input VJP is the same kernel on the transposed,
// flipped weights (strides + flip flag, no repacking).
//
// Round 3: the 8 x 64 tile with two pixels per thread and scalar FMAs (no prefetch) ran the
// UNet's conv_out (64 x 128 -> 3 at 256^2) in 725 us = 0.38 of HBM peak on its 2.2 GB input.

#define SP_TU 7  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

namespace sp {

#ifndef SP_THIN_WIDE_CO
#define SP_THIN_WIDE_CO 16  // outputs per workgroup when the inputs are few (conv_in, conv_out's VJP)
#endif

constexpr int TN_TH = 16, TN_TW = 64;       // output tile: 16 rows x 16 threads of 4 pixels
constexpr int TN_PH = TN_TH + 2;
// patch row in LDS: [3] left padding column, [4, 68) the tile's 64 columns (16-byte
// aligned, so the row is staged with float4 loads and stores), [68] right padding column
constexpr int TN_PW = TN_TW + 8;
constexpr int TN_PATCH = TN_PH * TN_PW;     // 1296
constexpr int TN_Q = TN_TW / 4;             // float4 pieces per patch row

struct ThinArgs {
    const float* x;      // [n, cin, H, W]
    const float* w;      // weights: element (co, ci, t) at co * sco + ci * sci + (flip ? 8 - t : t)
    const float* bias;   // [cout] or NULL
    float* y;            // [n, cout, H, W]
    int cin, cout, H, W;
    int64_t sco, sci;
    int flip;
    int tiles_w, tiles;  // tiles per image row / per image
};

// Workgroups are dealt round-robin over the 8 XCDs in linear block order, so tiles that are
// neighbours in the image would land on different XCDs and each fetch their shared halo lines
// into its own L2 (the patch's single-column halo loads touch a whole line each: PMC fetch
// 2.2x the input).  The linear id is remapped so that runs of consecutive logical tiles —
// horizontal, then vertical neighbours — execute on one XCD and share its L2.
__device__ __forceinline__ void thin_block(int& tile, int& cob, int64_t& n) {
    const unsigned X = gridDim.x, Y = gridDim.y, T = X * Y * gridDim.z;
    unsigned l = blockIdx.x + X * (blockIdx.y + Y * blockIdx.z);
    // (with several output-channel blocks the natural order already keeps a tile's blocks,
    // X apart, on one XCD: remap single-block grids only)
    if (Y == 1 && T % 8 == 0) l = (l % 8) * (T / 8) + l / 8;  // placement only: any order is correct
    tile = static_cast<int>(l % X);
    cob = static_cast<int>((l / X) % Y);
    n = l / (X * Y);
    SP_DCHECK(l < T && n < gridDim.z);  // the remap is a permutation of the grid
}

typedef float tn_f2 __attribute__((ext_vector_type(2)));

// Output channels per workgroup as held in LDS (CO = 3 padded to 4: whole float4 reads).
template <int CO>
constexpr int thin_cop() { return (CO + 3) & ~3; }

// One chunk's patch pieces and weights held in registers between their loads and the LDS
// stores.  Weights go to LDS as wl[(c * 9 + t) * COP + o] (tap t in the kernel's order, the
// flip applied here), zero for channels / outputs past the tensor's, so the math has no
// per-channel or per-output branches (a zero patch times a zero weight adds nothing).
template <int CI, int CO, bool FLIP>
struct ThinStage {
    static constexpr int COP = thin_cop<CO>();
    static constexpr int NQ = (CI * TN_PH * TN_Q + kBlock - 1) / kBlock;   // float4 pieces
    static constexpr int NH = (CI * TN_PH * 2 + kBlock - 1) / kBlock;      // padding columns
    static constexpr int NW = CI <= 4 ? (CI * 9 * COP + kBlock - 1) / kBlock : 0;  // weights (in LDS only for few inputs)
    float4 q[NQ];
    float h[NH];
    float wv[NW];

    __device__ __forceinline__ void load(const ThinArgs& a, const float* xn, int64_t plane, int c0,
                                         int h0, int w0, int co0) {
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const int i = threadIdx.x + k * kBlock;
            const int o = i % COP, ct = i / COP, c = ct / 9, t = ct - 9 * c;
            const bool ok = i < CI * 9 * COP && o < CO && co0 + o < a.cout && c0 + c < a.cin;
            wv[k] = ok ? a.w[(int64_t)(co0 + o) * a.sco + (int64_t)(c0 + c) * a.sci + (FLIP ? 8 - t : t)] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            const int i = threadIdx.x + k * kBlock;
            const int cr = i / TN_Q, qq = i - cr * TN_Q;                  // (channel, row), piece
            const int c = cr / TN_PH, r = cr - c * TN_PH;
            const int gr = h0 - 1 + r, gc = w0 + 4 * qq;
            q[k] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (i < CI * TN_PH * TN_Q && c0 + c < a.cin && (unsigned)gr < (unsigned)a.H && gc < a.W)
                q[k] = *reinterpret_cast<const float4*>(xn + (int64_t)(c0 + c) * plane + (int64_t)gr * a.W + gc);
        }
#pragma unroll
        for (int k = 0; k < NH; ++k) {
            const int i = threadIdx.x + k * kBlock;
            const int cr = i >> 1, side = i & 1;
            const int c = cr / TN_PH, r = cr - c * TN_PH;
            const int gr = h0 - 1 + r, gc = side ? w0 + TN_TW : w0 - 1;
            const bool ok = i < CI * TN_PH * 2 && c0 + c < a.cin && (unsigned)gr < (unsigned)a.H &&
                            (unsigned)gc < (unsigned)a.W;
            h[k] = ok ? xn[(int64_t)(c0 + c) * plane + (int64_t)gr * a.W + gc] : 0.f;
        }
    }

    __device__ __forceinline__ void store(float* patch, float* wl) const {
#pragma unroll
        for (int k = 0; k < NW; ++k) {
            const int i = threadIdx.x + k * kBlock;
            if (i < CI * 9 * COP) wl[i] = wv[k];
        }
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            const int i = threadIdx.x + k * kBlock;
            if (i >= CI * TN_PH * TN_Q) break;
            const int cr = i / TN_Q, qq = i - cr * TN_Q;
            const int c = cr / TN_PH, r = cr - c * TN_PH;
            *reinterpret_cast<float4*>(&patch[c * TN_PATCH + r * TN_PW + 4 + 4 * qq]) = q[k];
        }
#pragma unroll
        for (int k = 0; k < NH; ++k) {
            const int i = threadIdx.x + k * kBlock;
            if (i >= CI * TN_PH * 2) break;
            const int cr = i >> 1, side = i & 1;
            const int c = cr / TN_PH, r = cr - c * TN_PH;
            patch[c * TN_PATCH + r * TN_PW + (side ? 4 + TN_TW : 3)] = h[k];
        }
    }
};

template <int CI, int CO, bool FLIP>
__global__ __launch_bounds__(kBlock) void k_conv3x3_thin(ThinArgs a) {
    // WL: weights staged in LDS and read as float4 broadcasts (16 outputs per workgroup);
    // with few outputs the scalar loads measured faster (their LDS reads cost the patch's)
    constexpr bool WL = CI <= 4;
    constexpr int COP = thin_cop<CO>();
    __shared__ __attribute__((aligned(16))) float patch[CI * TN_PATCH];
    __shared__ __attribute__((aligned(16))) float wl[WL ? CI * 9 * COP : 4];
    int tile, cob;
    int64_t n;
    thin_block(tile, cob, n);
    const int co0 = cob * CO;
    const int ty = tile / a.tiles_w, tx = tile - ty * a.tiles_w;
    const int h0 = ty * TN_TH, w0 = tx * TN_TW;
    const int64_t plane = (int64_t)a.H * a.W;
    const float* xn = a.x + n * a.cin * plane;
    const int pr = threadIdx.x / (TN_TW / 4), pc = 4 * (threadIdx.x % (TN_TW / 4));  // 4 pixels
    tn_f2 acc[CO][2];  // pixels (0, 1) and (2, 3)
#pragma unroll
    for (int o = 0; o < CO; ++o) {
        const float b = a.bias && co0 + o < a.cout ? a.bias[co0 + o] : 0.f;
        acc[o][0] = acc[o][1] = tn_f2{b, b};
    }
    ThinStage<CI, CO, FLIP> st;
    st.load(a, xn, plane, 0, h0, w0, co0);
    for (int c0 = 0; c0 < a.cin; c0 += CI) {
        __syncthreads();  // previous chunk's patch / weight reads are done
        st.store(patch, wl);
        __syncthreads();
        if (c0 + CI < a.cin) st.load(a, xn, plane, c0 + CI, h0, w0, co0);  // in flight during the math
#pragma unroll
        for (int c = 0; c < CI; ++c) {
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                const float* row = &patch[c * TN_PATCH + (pr + r) * TN_PW + pc];
                const float lf = row[3], rt = row[8];
                const float4 m = *reinterpret_cast<const float4*>(row + 4);
                const tn_f2 p01{m.x, m.y}, p23{m.z, m.w}, pl0{lf, m.x}, p12{m.y, m.z}, p3r{m.w, rt};
                // this row's 3 x COP weights: uniform addresses (LDS broadcast), float4 reads
                float wt[3][COP] = {};
#pragma unroll
                for (int s = 0; s < 3 && WL; ++s)
#pragma unroll
                    for (int o4 = 0; o4 < COP; o4 += 4) {
                        const float4 v = *reinterpret_cast<const float4*>(&wl[(c * 9 + 3 * r + s) * COP + o4]);
                        wt[s][o4] = v.x, wt[s][o4 + 1] = v.y, wt[s][o4 + 2] = v.z, wt[s][o4 + 3] = v.w;
                    }
#pragma unroll
                for (int o = 0; o < CO; ++o) {  // taps in the order t = 3r + s
                    float w0s = wt[0][o], w1s = wt[1][o], w2s = wt[2][o];
                    if (!WL) {  // few outputs: the weights as uniform scalar loads instead,
                        // unconditional (clamped indices: a channel past cin has a zero patch,
                        // an output past cout is never stored), so they batch ahead of use
                        const float* wr = a.w + (int64_t)min(co0 + o, a.cout - 1) * a.sco +
                                          (int64_t)min(c0 + c, a.cin - 1) * a.sci;
                        w0s = wr[FLIP ? 8 - 3 * r : 3 * r];
                        w1s = wr[FLIP ? 7 - 3 * r : 3 * r + 1];
                        w2s = wr[FLIP ? 6 - 3 * r : 3 * r + 2];
                    }
                    const tn_f2 w0v{w0s, w0s}, w1v{w1s, w1s}, w2v{w2s, w2s};
                    acc[o][0] = __builtin_elementwise_fma(w0v, pl0, acc[o][0]);
                    acc[o][1] = __builtin_elementwise_fma(w0v, p12, acc[o][1]);
                    acc[o][0] = __builtin_elementwise_fma(w1v, p01, acc[o][0]);
                    acc[o][1] = __builtin_elementwise_fma(w1v, p23, acc[o][1]);
                    acc[o][0] = __builtin_elementwise_fma(w2v, p12, acc[o][0]);
                    acc[o][1] = __builtin_elementwise_fma(w2v, p3r, acc[o][1]);
                }
            }
        }
    }
    const int gr = h0 + pr, gc = w0 + pc;
    if (gr >= a.H || gc >= a.W) return;  // W % 4 == 0: a thread's 4 pixels are all in or all out
    float* yn = a.y + n * a.cout * plane + (int64_t)gr * a.W + gc;
#pragma unroll
    for (int o = 0; o < CO; ++o) {
        if (co0 + o >= a.cout) break;
        *reinterpret_cast<float4*>(yn + (int64_t)(co0 + o) * plane) =
            make_float4(acc[o][0].x, acc[o][0].y, acc[o][1].x, acc[o][1].y);
    }
}

// (CI, CO) per kernel shape: few outputs -> all of them per workgroup, 8 input channels per
// chunk; few inputs -> all of them in one chunk, 16 outputs per workgroup.
static int thin_launch(const ThinArgs& a0, int64_t n, hipStream_t s, int kind) {
    ThinArgs a = a0;
    a.tiles_w = (a.W + TN_TW - 1) / TN_TW;
    a.tiles = a.tiles_w * ((a.H + TN_TH - 1) / TN_TH);
    if (n > 65535 || (int64_t)a.cin * a.H * a.W >= (int64_t(1) << 31) ||
        (int64_t)a.cout * a.H * a.W >= (int64_t(1) << 31) || (a.W & 3))
        return SP_EINVAL;
    const double flops = 18.0 * n * a.cin * a.cout * a.H * a.W;
#define SP_THIN(CI_, CO_)                                                                    \
    launch_w(kind, flops, a.flip ? k_conv3x3_thin<CI_, CO_, true> : k_conv3x3_thin<CI_, CO_, false>, \
             dim3(static_cast<unsigned>(a.tiles), (a.cout + CO_ - 1) / CO_, static_cast<unsigned>(n)), \
             dim3(kBlock), s, a)
    if (a.cout <= 3) SP_THIN(8, 3);
    else if (a.cout <= 4) SP_THIN(8, 4);
    else if (a.cout <= 8) SP_THIN(8, 8);
    else if (a.cin <= 3) SP_THIN(3, SP_THIN_WIDE_CO);
    else if (a.cin <= 4) SP_THIN(4, SP_THIN_WIDE_CO);
    else if (a.cin <= 8) SP_THIN(8, 16);
    else return SP_EINVAL;
#undef SP_THIN
    return check_launch("sp_conv3x3_thin");
}

}  // namespace sp

using namespace sp;

extern "C" {

int sp_conv3x3_thin_supported(int32_t cin, int32_t cout, int32_t height, int32_t width) {
    return cin > 0 && cout > 0 && height > 0 && width > 0 && width % 4 == 0 &&
           (cout <= 8 || cin <= 8);
}

int sp_conv3x3_thin_fwd(const float* x, const float* w, const float* bias, int64_t n,
                        int32_t cin, int32_t cout, int32_t height, int32_t width, float* y,
                        sp_stream_t stream) {
    if (!sp_conv3x3_thin_supported(cin, cout, height, width) || n < 0) return SP_EINVAL;
    if (n == 0) return SP_OK;
    if (!x || !w || !y) return SP_EINVAL;
    ThinArgs a{x, w, bias, y, cin, cout, height, width, (int64_t)cin * 9, 9, 0, 0, 0};
    return thin_launch(a, n, static_cast<hipStream_t>(stream), 0);  // VALU: not in the MFMA roofline
}

int sp_conv3x3_thin_bwd_input(const float* dy, const float* w, int64_t n, int32_t cin,
                              int32_t cout, int32_t height, int32_t width, float* dx,
                              sp_stream_t stream) {
    // dx = conv(dy) with W'[ci][co][t] = W[co][ci][8 - t]: a (cout -> cin) convolution
    if (!sp_conv3x3_thin_supported(cout, cin, height, width) || n < 0) return SP_EINVAL;
    if (n == 0) return SP_OK;
    if (!dy || !w || !dx) return SP_EINVAL;
    ThinArgs a{dy, w, nullptr, dx, cout, cin, height, width, 9, (int64_t)cin * 9, 1, 0, 0};
    return thin_launch(a, n, static_cast<hipStream_t>(stream), 0);
}

}  // extern "C"

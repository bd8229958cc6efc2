// 3x3 / stride 1 / pad 1 convolutions with few channels on one side: the priors' conv_in
// (3 or 4 input channels) and conv_out (3 or 8 output channels) and their input VJPs
// (any side with at most 8 channels)
// (diffusers UNet2DModel / AutoencoderKL, reached from ddpm.py:40-43 and
// stable_diffusion.py:330-345).  MIOpen runs them through NHWC implicit GEMMs with layout
// transposes, or its naive kernel (decoder conv_out at 512^2: ~1.5 ms per 4 images).
//
// The work is ~14 k FMA per output pixel at most and the memory traffic is the wide side's
// tensor, so this is a VALU direct convolution: one workgroup = an 8 x 64 pixel tile of one
// image x CO output channels; input channels are walked in chunks of CI, each chunk's
// 10 x 66 patch (zero outside the image = the padding) staged in LDS with float4 row
// pieces (W % 4 == 0); every thread owns two
// horizontally adjacent pixels x CO outputs, reads its 3 x 4 window per channel from LDS
// and takes the weights as wave-uniform scalar loads.  The input VJP is the same kernel on
// the transposed, flipped weights (strides + flip flag, no repacking).

#include "sp_common.h"

namespace sp {

constexpr int TN_TH = 8, TN_TW = 64;        // output tile
constexpr int TN_PH = TN_TH + 2;
// patch row in LDS: [3] left padding column, [4, 68) the tile's 64 columns (16-byte
// aligned, so the row is staged with float4 loads and stores), [68] right padding column
constexpr int TN_PW = TN_TW + 8;
constexpr int TN_PATCH = TN_PH * TN_PW;     // 720
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
}

template <int CI, int CO>
__global__ __launch_bounds__(kBlock) void k_conv3x3_thin(ThinArgs a) {
    __shared__ __attribute__((aligned(16))) float patch[CI * TN_PATCH];
    int tile, cob;
    int64_t n;
    thin_block(tile, cob, n);
    const int co0 = cob * CO;
    const int ty = tile / a.tiles_w, tx = tile - ty * a.tiles_w;
    const int h0 = ty * TN_TH, w0 = tx * TN_TW;
    const int64_t plane = (int64_t)a.H * a.W;
    const float* xn = a.x + n * a.cin * plane;
    const int pr = threadIdx.x / (TN_TW / 2), pc = 2 * (threadIdx.x % (TN_TW / 2));  // pixel pair
    float acc[CO][2];
#pragma unroll
    for (int o = 0; o < CO; ++o) {
        const float b = a.bias && co0 + o < a.cout ? a.bias[co0 + o] : 0.f;
        acc[o][0] = acc[o][1] = b;
    }
    for (int c0 = 0; c0 < a.cin; c0 += CI) {
        __syncthreads();  // previous chunk's patch reads are done
        for (int i = threadIdx.x; i < CI * TN_PH * TN_Q; i += kBlock) {  // interior columns
            const int cr = i / TN_Q, q = i - cr * TN_Q;                  // (channel, row), piece
            const int c = cr / TN_PH, r = cr - c * TN_PH;
            const int gr = h0 - 1 + r, gc = w0 + 4 * q;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (c0 + c < a.cin && (unsigned)gr < (unsigned)a.H && gc < a.W)
                v = *reinterpret_cast<const float4*>(xn + (int64_t)(c0 + c) * plane + (int64_t)gr * a.W + gc);
            *reinterpret_cast<float4*>(&patch[c * TN_PATCH + r * TN_PW + 4 + 4 * q]) = v;
        }
        for (int i = threadIdx.x; i < CI * TN_PH * 2; i += kBlock) {  // padding columns
            const int cr = i >> 1, side = i & 1;
            const int c = cr / TN_PH, r = cr - c * TN_PH;
            const int gr = h0 - 1 + r, gc = side ? w0 + TN_TW : w0 - 1;
            const bool ok = c0 + c < a.cin && (unsigned)gr < (unsigned)a.H && (unsigned)gc < (unsigned)a.W;
            patch[c * TN_PATCH + r * TN_PW + (side ? 4 + TN_TW : 3)] =
                ok ? xn[(int64_t)(c0 + c) * plane + (int64_t)gr * a.W + gc] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int c = 0; c < CI; ++c) {
            if (c0 + c >= a.cin) break;
            float win[3][4];
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int s = 0; s < 4; ++s) win[r][s] = patch[c * TN_PATCH + (pr + r) * TN_PW + 3 + pc + s];
#pragma unroll
            for (int o = 0; o < CO; ++o) {
                if (co0 + o >= a.cout) break;
                const float* wr = a.w + (int64_t)(co0 + o) * a.sco + (int64_t)(c0 + c) * a.sci;
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    const float wt = wr[a.flip ? 8 - t : t];  // uniform: scalar loads
                    acc[o][0] = fmaf(wt, win[t / 3][t % 3], acc[o][0]);
                    acc[o][1] = fmaf(wt, win[t / 3][t % 3 + 1], acc[o][1]);
                }
            }
        }
    }
    const int gr = h0 + pr, gc = w0 + pc;
    if (gr >= a.H) return;
    float* yn = a.y + n * a.cout * plane + (int64_t)gr * a.W + gc;
#pragma unroll
    for (int o = 0; o < CO; ++o) {
        if (co0 + o >= a.cout) break;
        if (gc + 1 < a.W) {
            *reinterpret_cast<float2*>(yn + (int64_t)(co0 + o) * plane) = make_float2(acc[o][0], acc[o][1]);
        } else if (gc < a.W) {
            yn[(int64_t)(co0 + o) * plane] = acc[o][0];
        }
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
    launch_w(kind, flops, k_conv3x3_thin<CI_, CO_>,                                         \
             dim3(static_cast<unsigned>(a.tiles), (a.cout + CO_ - 1) / CO_, static_cast<unsigned>(n)), \
             dim3(kBlock), s, a)
    if (a.cout <= 3) SP_THIN(8, 3);
    else if (a.cout <= 4) SP_THIN(8, 4);
    else if (a.cout <= 8) SP_THIN(8, 8);
    else if (a.cin <= 3) SP_THIN(3, 16);
    else if (a.cin <= 4) SP_THIN(4, 16);
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

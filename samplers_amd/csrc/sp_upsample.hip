// 2x nearest-neighbour upsampling of Upsample2D (the UNet's up blocks and the SD VAE decoder;
// reached from /root/reference/samplers/networks/ddpm.py:40-43 and stable_diffusion.py:330-336
// -> diffusers' Upsample2D, F.interpolate(scale_factor=2, mode="nearest")) and its VJP,
// the 2x2 block sum, as streaming HBM kernels: one thread per 4 input columns of one row
// (one float4 of x / dx), two 32-byte row pieces of the 2x image (4 float4) on the other
// side.  The VJP sums each block in torch's loop order ((0,0) + (0,1)) + (1,0)) + (1,1).

#define SP_TU 9  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

namespace sp {

typedef float up_f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kBlock) void k_upsample2x(const float* __restrict__ x,
                                                       float* __restrict__ y, int64_t rows,
                                                       int w4) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= rows * w4) return;
    const int64_t r = t / w4;  // input row (plane * h + i)
    const int j = static_cast<int>(t - r * w4);
    SP_DCHECK(r < rows && j < w4);
    const up_f4 v = reinterpret_cast<const up_f4*>(x)[t];
    const up_f4 lo{v[0], v[0], v[1], v[1]}, hi{v[2], v[2], v[3], v[3]};
    up_f4* o = reinterpret_cast<up_f4*>(y) + (2 * r) * (2 * w4) + 2 * j;
    o[0] = lo;
    o[1] = hi;
    o[2 * w4] = lo;
    o[2 * w4 + 1] = hi;
}

__global__ __launch_bounds__(kBlock) void k_upsample2x_vjp(const float* __restrict__ dy,
                                                           float* __restrict__ dx, int64_t rows,
                                                           int w4) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (t >= rows * w4) return;
    const int64_t r = t / w4;
    const int j = static_cast<int>(t - r * w4);
    const up_f4* g = reinterpret_cast<const up_f4*>(dy) + (2 * r) * (2 * w4) + 2 * j;
    const up_f4 a0 = g[0], a1 = g[1], b0 = g[2 * w4], b1 = g[2 * w4 + 1];
    up_f4 d;
    d[0] = ((a0[0] + a0[1]) + b0[0]) + b0[1];
    d[1] = ((a0[2] + a0[3]) + b0[2]) + b0[3];
    d[2] = ((a1[0] + a1[1]) + b1[0]) + b1[1];
    d[3] = ((a1[2] + a1[3]) + b1[2]) + b1[3];
    reinterpret_cast<up_f4*>(dx)[t] = d;
}

}  // namespace sp

using namespace sp;

extern "C" {

int sp_upsample2x_supported(int32_t height, int32_t width) {
    return height > 0 && width > 0 && width % 4 == 0;
}

static int upsample2x(bool vjp, const float* src, int64_t planes, int32_t height, int32_t width,
                      float* dst, sp_stream_t stream) {
    if (planes < 0 || !sp_upsample2x_supported(height, width)) return SP_EINVAL;
    if (planes == 0) return SP_OK;
    if (!src || !dst) return SP_EINVAL;
    if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) return SP_EINVAL;
    const int64_t rows = planes * height, total = rows * (width / 4);
    const int64_t blocks = (total + kBlock - 1) / kBlock;
    if (blocks >= (int64_t(1) << 31)) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (vjp)
        launch(0, k_upsample2x_vjp, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), s, src, dst,
               rows, width / 4);
    else
        launch(0, k_upsample2x, dim3(static_cast<unsigned>(blocks)), dim3(kBlock), s, src, dst, rows,
               width / 4);
    return check_launch(vjp ? "sp_upsample2x_vjp" : "sp_upsample2x");
}

int sp_upsample2x(const float* x, int64_t planes, int32_t height, int32_t width, float* y,
                  sp_stream_t stream) {
    return upsample2x(false, x, planes, height, width, y, stream);
}

int sp_upsample2x_vjp(const float* dy, int64_t planes, int32_t height, int32_t width, float* dx,
                      sp_stream_t stream) {
    return upsample2x(true, dy, planes, height, width, dx, stream);
}

}  // extern "C"

// Latent-space samplers (PSLD, ReSample): the pixel-space glue around the VAE.
//
// PSLD step (psld.py:118-153) with x0 = D(z0):
//   L = ||y - A x0||_F,  x_eff = A^T y + x0 - A^T A x0,  G = ||z0 - E(x_eff)||_F  (batch-global)
//   cotangent of x0:  -omega A^T r / L + (I - A^T A) u,   u = E^T(-gamma d / G)
// ReSample (resample.py, resample_kernels.py): epsilon-form DDIM step, stochastic
// resample, fused AdamW on the hard-consistency problems.
//
// Norms over the whole batch are two-stage: per-block partials (fixed order) then
// sp_sum_partials into a device scalar — the consumers read the scalar from device
// memory, so nothing synchronises with the host, and a multi-GPU caller can
// all-reduce the scalar in between.

#include <algorithm>

#define SP_TU 3  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

namespace sp {

int64_t tiles_elementwise(int64_t n);
bool valid_op(const sp_op* op);

// x_eff and A^T r for the elementwise operators (IDENTITY / INPAINT / MASK)
template <int OPK, int V>
__global__ __launch_bounds__(kBlock) void k_psld_pixel(sp_op op, const float* __restrict__ x0,
                                                       const float* __restrict__ y, int64_t y_div,
                                                       float* __restrict__ x_eff,
                                                       float* __restrict__ atr,
                                                       float* __restrict__ partial, int P) {
    __shared__ float red[4];
    const int64_t b = blockIdx.y, n = op.n;
    const float* xb = x0 + b * n;
    const float* yb = y + (b / y_div) * op.m;
    const int64_t j0 = (int64_t)blockIdx.x * kIter * (kBlock * V) + threadIdx.x * V;
    float acc = 0.f;
#pragma unroll
    for (int it = 0; it < kIter; ++it) {
        const int64_t j = j0 + it * (kBlock * V);
        if (j >= n) break;
        float xv[V], yv[V], xe[V], ar[V];
        load_v<V>(xb + j, xv);
        uint32_t bits = 0xFu;
        if constexpr (OPK == SP_OP_INPAINT) {
            int64_t r;
            inpaint_lookup(op, j, bits, r);
#pragma unroll
            for (int e = 0; e < V; ++e) yv[e] = ((bits >> e) & 1u) ? yb[r++] : 0.f;
        } else {
            load_v<V>(yb + j, yv);
            if constexpr (OPK == SP_OP_MASK) bits = mask_bits(op, j);
        }
#pragma unroll
        for (int e = 0; e < V; ++e) {
            const bool kept = (bits >> e) & 1u;
            const float r = yv[e] - (kept ? xv[e] : 0.f);  // y - A x0 (A x0 = 0 off the mask)
            xe[e] = kept ? yv[e] : xv[e];                  // A^T y + (I - A^T A) x0
            ar[e] = kept ? r : 0.f;                        // A^T r
            if (OPK != SP_OP_INPAINT || kept) acc += r * r;
        }
        store_v<V>(x_eff + b * n + j, xe);
        store_v<V>(atr + b * n + j, ar);
    }
    const float t = block_sum(acc, red);
    SP_DCHECK(static_cast<int>(blockIdx.x) < P);
    if (threadIdx.x == 0) partial[b * P + blockIdx.x] = t;
}

// out[0] = sum of count partials (one workgroup, fixed order)
__global__ __launch_bounds__(kBlock) void k_sum(const float* __restrict__ p, int64_t count,
                                                float* __restrict__ out) {
    __shared__ float red[4];
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < count; i += kBlock) s += p[i];
    const float t = block_sum(s, red);
    if (threadIdx.x == 0) *out = t;
}

__device__ __forceinline__ float inv_norm(const float* norm_sq) {
    const float nrm = sqrtf(*norm_sq);
    return nrm > 0.f ? 1.f / nrm : 0.f;  // torch's norm backward is 0 at a zero norm
}

// out = alpha * a + beta / sqrt(*norm_sq) * b   (a may be null)
template <int V>
__global__ __launch_bounds__(kBlock) void k_scaled_combine(const float* __restrict__ a, float alpha,
                                                           const float* __restrict__ b, float beta,
                                                           const float* __restrict__ norm_sq,
                                                           int64_t count, float* __restrict__ out) {
    const float cb = norm_sq ? beta * inv_norm(norm_sq) : beta;
    const int64_t stride = (int64_t)gridDim.x * kBlock * V;
    for (int64_t j = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * V; j < count; j += stride) {
        float bv[V], o[V];
        load_v<V>(b + j, bv);
        if (a) {
            float av[V];
            load_v<V>(a + j, av);
#pragma unroll
            for (int e = 0; e < V; ++e) o[e] = alpha * av[e] + cb * bv[e];
        } else {
#pragma unroll
            for (int e = 0; e < V; ++e) o[e] = cb * bv[e];
        }
        store_v<V>(out + j, o);
    }
}

// c_x0 = -omega A^T r / L + (I - A^T A) u   (ata_u = A^T A u supplied for BLUR)
template <int OPK, int V>
__global__ __launch_bounds__(kBlock) void k_psld_cotangent(sp_op op, const float* __restrict__ atr,
                                                           const float* __restrict__ u,
                                                           const float* __restrict__ ata_u,
                                                           const float* __restrict__ norm_sq,
                                                           float omega, float* __restrict__ out) {
    const float cl = -omega * inv_norm(norm_sq);
    const int64_t b = blockIdx.y, n = op.n;
    const int64_t stride = (int64_t)gridDim.x * kBlock * V;
    for (int64_t j = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * V; j < n; j += stride) {
        float av[V], uv[V], o[V];
        load_v<V>(atr + b * n + j, av);
        load_v<V>(u + b * n + j, uv);
        if constexpr (OPK == SP_OP_BLUR) {
            float pv[V];
            load_v<V>(ata_u + b * n + j, pv);
#pragma unroll
            for (int e = 0; e < V; ++e) o[e] = cl * av[e] + (uv[e] - pv[e]);
        } else {
            const uint32_t bits = OPK == SP_OP_IDENTITY ? 0xFu : mask_bits(op, j);
#pragma unroll
            for (int e = 0; e < V; ++e) o[e] = cl * av[e] + (((bits >> e) & 1u) ? 0.f : uv[e]);
        }
        store_v<V>(out + b * n + j, o);
    }
}

// epsilon-form DDIM step (bridge_kernels.py:82-115): returns x_prev, x0, pseudo-x0
template <int V, bool XI_IN>
__global__ __launch_bounds__(kBlock) void k_ddim_eps(const float* __restrict__ x,
                                                     const float* __restrict__ e, int64_t n,
                                                     sp_eps_coefs c, const float* __restrict__ xi,
                                                     uint64_t seed, int64_t step, int64_t offset,
                                                     float* __restrict__ x_prev,
                                                     float* __restrict__ x0,
                                                     float* __restrict__ pseudo) {
    const int64_t b = blockIdx.y;
    const int64_t stride = (int64_t)gridDim.x * kBlock * V;
    for (int64_t j = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * V; j < n; j += stride) {
        float xv[V], ev[V], z[V], o0[V], o1[V], o2[V];
        load_v<V>(x + b * n + j, xv);
        load_v<V>(e + b * n + j, ev);
        if constexpr (XI_IN) load_v<V>(xi + b * n + j, z);
        else philox_normals<V>(seed, step, offset + b, j, z);
#pragma unroll
        for (int e2 = 0; e2 < V; ++e2) {
            const float p0 = (xv[e2] - c.sqrt_oma * ev[e2]) / c.sqrt_a;
            o1[e2] = p0;
            o2[e2] = (xv[e2] - c.oma * ev[e2]) / c.sqrt_a;
            o0[e2] = (c.sqrt_a_prev * p0 + c.dir * ev[e2]) + c.sigma * z[e2];
        }
        if (x_prev) store_v<V>(x_prev + b * n + j, o0);
        if (x0) store_v<V>(x0 + b * n + j, o1);
        if (pseudo) store_v<V>(pseudo + b * n + j, o2);
    }
}

// stochastic resample (resample_kernels.py:96-107)
template <int V, bool XI_IN>
__global__ __launch_bounds__(kBlock) void k_stochastic_resample(
    const float* __restrict__ px0, const float* __restrict__ xt, int64_t n, float a_t, float sigma,
    const float* __restrict__ xi, uint64_t seed, int64_t step, int64_t offset, float* __restrict__ out) {
    const int64_t b = blockIdx.y;
    const float oma = 1.f - a_t;
    const float sa = sqrtf(a_t);
    const float den = (sigma + 1.f) - a_t;  // sigma + 1 - a_t, evaluated as the reference does
    const float sd = sqrtf(1.f / (1.f / sigma + 1.f / oma));
    const int64_t stride = (int64_t)gridDim.x * kBlock * V;
    for (int64_t j = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * V; j < n; j += stride) {
        float pv[V], xv[V], z[V], o[V];
        load_v<V>(px0 + b * n + j, pv);
        load_v<V>(xt + b * n + j, xv);
        if constexpr (XI_IN) load_v<V>(xi + b * n + j, z);
        else philox_normals<V>(seed, step, offset + b, j, z);
#pragma unroll
        for (int e = 0; e < V; ++e) o[e] = (sigma * sa * pv[e] + oma * xv[e]) / den + z[e] * sd;
        store_v<V>(out + b * n + j, o);
    }
}

// torch.optim.AdamW update of one parameter (decoupled weight decay, no amsgrad)
__device__ __forceinline__ void adamw_1(float& p, float g, float& m, float& v, const sp_adamw_coefs& c) {
    p = p * c.decay;                                // p *= 1 - lr * weight_decay
    m = m + (1.f - c.beta1) * (g - m);              // exp_avg.lerp_(g, 1 - beta1)
    v = v * c.beta2 + (1.f - c.beta2) * g * g;      // exp_avg_sq.mul_(beta2).addcmul_
    const float denom = sqrtf(v) / c.bc2_sqrt + c.eps;
    p = p - c.step_size * m / denom;
}

// torch.optim.AdamW step, in place; a set *stop makes it a no-op (device-side early stop)
template <int V>
__global__ __launch_bounds__(kBlock) void k_adamw(float* __restrict__ p, const float* __restrict__ g,
                                                  float* __restrict__ m, float* __restrict__ v,
                                                  int64_t count, sp_adamw_coefs c,
                                                  const int32_t* __restrict__ stop) {
    if (stop && *stop) return;
    const int64_t stride = (int64_t)gridDim.x * kBlock * V;
    for (int64_t j = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * V; j < count; j += stride) {
        float pv[V], gv[V], mv[V], vv[V];
        load_v<V>(p + j, pv);
        load_v<V>(g + j, gv);
        load_v<V>(m + j, mv);
        load_v<V>(v + j, vv);
#pragma unroll
        for (int e = 0; e < V; ++e) adamw_1(pv[e], gv[e], mv[e], vv[e], c);
        store_v<V>(p + j, pv);
        store_v<V>(m + j, mv);
        store_v<V>(v + j, vv);
    }
}

// One iteration of ReSample's pixel-space hard data consistency for the elementwise
// operators (resample_kernels.py:32-54: AdamW(lr=1e-2) on MSE(y, A x)), one pass over x:
// r = y - A x, g = A^T (gs r) with gs = -2/M (the MSE gradient w.r.t. A x), the AdamW
// update of x in place, and the iteration's r^2 partials (the loss of x before the
// update, as the reference's measurement_loss).  A set *stop makes it a no-op.
template <int OPK, int V>
__global__ __launch_bounds__(kBlock) void k_pixel_opt(sp_op op, float* __restrict__ x,
                                                      float* __restrict__ m, float* __restrict__ v,
                                                      const float* __restrict__ y, int64_t y_div,
                                                      float gs, sp_adamw_coefs c,
                                                      const int32_t* __restrict__ stop,
                                                      float* __restrict__ partial, int P) {
    __shared__ float red[4];
    if (stop && *stop) return;
    const int64_t b = blockIdx.y, n = op.n;
    float* xb = x + b * n;
    float* mb = m + b * n;
    float* vb = v + b * n;
    const float* yb = y + (b / y_div) * op.m;
    const int64_t j0 = (int64_t)blockIdx.x * kIter * (kBlock * V) + threadIdx.x * V;
    float acc = 0.f;
#pragma unroll
    for (int it = 0; it < kIter; ++it) {
        const int64_t j = j0 + it * (kBlock * V);
        if (j >= n) break;
        float xv[V], mv[V], vv[V], yv[V];
        load_v<V>(xb + j, xv);
        load_v<V>(mb + j, mv);
        load_v<V>(vb + j, vv);
        uint32_t bits = 0xFu;
        if constexpr (OPK == SP_OP_INPAINT) {
            int64_t r;
            inpaint_lookup(op, j, bits, r);
#pragma unroll
            for (int e = 0; e < V; ++e) yv[e] = ((bits >> e) & 1u) ? yb[r++] : 0.f;
        } else {
            load_v<V>(yb + j, yv);
            if constexpr (OPK == SP_OP_MASK) bits = mask_bits(op, j);
        }
#pragma unroll
        for (int e = 0; e < V; ++e) {
            const bool kept = (bits >> e) & 1u;
            const float r = yv[e] - (kept ? xv[e] : 0.f);
            if (OPK != SP_OP_INPAINT || kept) acc += r * r;
            adamw_1(xv[e], kept ? gs * r : 0.f, mv[e], vv[e], c);
        }
        store_v<V>(xb + j, xv);
        store_v<V>(mb + j, mv);
        store_v<V>(vb + j, vv);
    }
    const float t = block_sum(acc, red);
    SP_DCHECK(static_cast<int>(blockIdx.x) < P);
    if (threadIdx.x == 0) partial[b * P + blockIdx.x] = t;
}

// Early-stop test of the optimisation loops (resample_kernels.py:50-51): loss = (sum of
// the count partials) / total; *stop = 1 once loss < threshold (compared in double, as
// the reference compares measurement_loss.item() with eps**2).  Runs after the
// iteration's update, so the stopping iteration's step is kept, as in the reference.
__global__ __launch_bounds__(kBlock) void k_opt_check(const float* __restrict__ p, int64_t count,
                                                      float total, double threshold,
                                                      int32_t* __restrict__ stop,
                                                      float* __restrict__ loss_out) {
    __shared__ float red[4];
    if (*stop) return;
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < count; i += kBlock) s += p[i];
    const float t = block_sum(s, red);
    if (threadIdx.x == 0) {
        const float loss = t / total;
        if (loss_out) *loss_out = loss;
        if ((double)loss < threshold) *stop = 1;
    }
}

// ReSample's latent-space stopping rule (resample_kernels.py:75-91) on the device: from
// iteration `plateau_from` on, stop when the loss rose above the previous iteration's; stop
// below the threshold.  prev[0] holds the previous loss (written from plateau_from on).
__global__ void k_opt_check_plateau(const float* __restrict__ p, int64_t count, float total,
                                    double threshold, int64_t itr, int64_t plateau_from,
                                    float* __restrict__ prev, int32_t* __restrict__ stop,
                                    float* __restrict__ loss_out) {
    __shared__ float red[4];
    if (*stop) return;
    float s = 0.f;
    for (int64_t i = threadIdx.x; i < count; i += kBlock) s += p[i];
    const float t = block_sum(s, red);
    if (threadIdx.x == 0) {
        const float loss = t / total;
        if (loss_out) *loss_out = loss;
        if (itr >= plateau_from) {
            if (itr > plateau_from && prev[0] < loss) *stop = 1;
            prev[0] = loss;
        }
        if ((double)loss < threshold) *stop = 1;
    }
}

static inline unsigned grid_for(int64_t work, int V, int64_t batch) {
    int64_t blocks = (work + (int64_t)kBlock * V - 1) / ((int64_t)kBlock * V);
    const int64_t cap = std::max<int64_t>(1, 4096 / std::max<int64_t>(batch, 1));
    return static_cast<unsigned>(std::max<int64_t>(1, std::min(blocks, cap)));
}

static inline bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace sp

using namespace sp;

extern "C" {

int sp_psld_pixel(const sp_op* op, const float* x0, const float* y, int64_t batch, int64_t y_div,
                  float* x_eff, float* atr, float* rsq_partial, sp_stream_t stream) {
    if (!valid_op(op) || !x0 || !y || !x_eff || !atr || !rsq_partial || batch <= 0 ||
        batch > 65535 || y_div <= 0)
        return SP_EINVAL;
    if (op->kind == SP_OP_BLUR) return SP_EUNSUPPORTED;  // composed from apply/adjoint by the caller
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int P = static_cast<int>(tiles_elementwise(op->n));
    const dim3 grid(P, static_cast<unsigned>(batch));
    const bool v4 = op->n % 4 == 0;
#define SP_PX(OPK, V) \
    launch(0, k_psld_pixel<OPK, V>, grid, dim3(kBlock), s, *op, x0, y, y_div, x_eff, atr, rsq_partial, P)
    switch (op->kind) {
        case SP_OP_IDENTITY: if (v4) SP_PX(SP_OP_IDENTITY, 4); else SP_PX(SP_OP_IDENTITY, 1); break;
        case SP_OP_INPAINT: if (v4) SP_PX(SP_OP_INPAINT, 4); else SP_PX(SP_OP_INPAINT, 1); break;
        default: if (v4) SP_PX(SP_OP_MASK, 4); else SP_PX(SP_OP_MASK, 1); break;
    }
#undef SP_PX
    return check_launch("sp_psld_pixel");
}

int sp_sum_partials(const float* partials, int64_t count, float* out, sp_stream_t stream) {
    if (!partials || !out || count <= 0) return SP_EINVAL;
    launch(0, k_sum, dim3(1), dim3(kBlock), static_cast<hipStream_t>(stream), partials, count, out);
    return check_launch("sp_sum_partials");
}

int sp_scaled_combine(const float* a, float alpha, const float* b, float beta, const float* norm_sq,
                      int64_t count, float* out, sp_stream_t stream) {
    if (!b || !out || count <= 0) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool v4 = count % 4 == 0 && aligned16(b) && aligned16(out) && (!a || aligned16(a));
    if (v4)
        launch(0, k_scaled_combine<4>, dim3(grid_for(count, 4, 1)), dim3(kBlock), s, a, alpha, b,
               beta, norm_sq, count, out);
    else
        launch(0, k_scaled_combine<1>, dim3(grid_for(count, 1, 1)), dim3(kBlock), s, a, alpha, b,
               beta, norm_sq, count, out);
    return check_launch("sp_scaled_combine");
}

int sp_psld_cotangent(const sp_op* op, const float* atr, const float* u, const float* ata_u,
                      const float* norm_sq, float omega, int64_t batch, float* out,
                      sp_stream_t stream) {
    if (!valid_op(op) || !atr || !u || !norm_sq || !out || batch <= 0 || batch > 65535)
        return SP_EINVAL;
    if (op->kind == SP_OP_BLUR && !ata_u) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool v4 = op->n % 4 == 0;
    const dim3 grid(grid_for(op->n, v4 ? 4 : 1, batch), static_cast<unsigned>(batch));
#define SP_CT(OPK, V) \
    launch(0, k_psld_cotangent<OPK, V>, grid, dim3(kBlock), s, *op, atr, u, ata_u, norm_sq, omega, out)
    switch (op->kind) {
        case SP_OP_IDENTITY: if (v4) SP_CT(SP_OP_IDENTITY, 4); else SP_CT(SP_OP_IDENTITY, 1); break;
        case SP_OP_BLUR: if (v4) SP_CT(SP_OP_BLUR, 4); else SP_CT(SP_OP_BLUR, 1); break;
        default: if (v4) SP_CT(SP_OP_MASK, 4); else SP_CT(SP_OP_MASK, 1); break;
    }
#undef SP_CT
    return check_launch("sp_psld_cotangent");
}

int sp_ddim_eps_step(const float* x, const float* eps, int64_t batch, int64_t n,
                     const sp_eps_coefs* c, const float* xi, uint64_t seed, int64_t step,
                     int64_t sample_offset, float* x_prev, float* x0, float* pseudo_x0,
                     sp_stream_t stream) {
    if (!x || !eps || !c || batch <= 0 || batch > 65535 || n <= 0) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool v4 = n % 4 == 0;
    const dim3 grid(grid_for(n, v4 ? 4 : 1, batch), static_cast<unsigned>(batch));
#define SP_DE(V, XIN)                                                                       \
    launch(0, k_ddim_eps<V, XIN>, grid, dim3(kBlock), s, x, eps, n, *c, xi, seed, step,     \
           sample_offset, x_prev, x0, pseudo_x0)
    if (v4) { if (xi) SP_DE(4, true); else SP_DE(4, false); }
    else { if (xi) SP_DE(1, true); else SP_DE(1, false); }
#undef SP_DE
    return check_launch("sp_ddim_eps_step");
}

int sp_stochastic_resample(const float* pseudo_x0, const float* x_t, int64_t batch, int64_t n,
                           float a_t, float sigma, const float* xi, uint64_t seed, int64_t step,
                           int64_t sample_offset, float* out, sp_stream_t stream) {
    if (!pseudo_x0 || !x_t || !out || batch <= 0 || batch > 65535 || n <= 0) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool v4 = n % 4 == 0;
    const dim3 grid(grid_for(n, v4 ? 4 : 1, batch), static_cast<unsigned>(batch));
#define SP_SR(V, XIN)                                                                      \
    launch(0, k_stochastic_resample<V, XIN>, grid, dim3(kBlock), s, pseudo_x0, x_t, n, a_t, \
           sigma, xi, seed, step, sample_offset, out)
    if (v4) { if (xi) SP_SR(4, true); else SP_SR(4, false); }
    else { if (xi) SP_SR(1, true); else SP_SR(1, false); }
#undef SP_SR
    return check_launch("sp_stochastic_resample");
}

int sp_adamw_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                  int64_t count, const sp_adamw_coefs* c, sp_stream_t stream) {
    return sp_adamw_step_until(param, grad, exp_avg, exp_avg_sq, count, c, nullptr, stream);
}

int sp_adamw_step_until(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                        int64_t count, const sp_adamw_coefs* c, const int32_t* stop,
                        sp_stream_t stream) {
    if (!param || !grad || !exp_avg || !exp_avg_sq || !c || count <= 0) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool v4 = count % 4 == 0 && aligned16(param) && aligned16(grad) && aligned16(exp_avg) &&
                    aligned16(exp_avg_sq);
    if (v4)
        launch(0, k_adamw<4>, dim3(grid_for(count, 4, 1)), dim3(kBlock), s, param, grad, exp_avg,
               exp_avg_sq, count, *c, stop);
    else
        launch(0, k_adamw<1>, dim3(grid_for(count, 1, 1)), dim3(kBlock), s, param, grad, exp_avg,
               exp_avg_sq, count, *c, stop);
    return check_launch("sp_adamw_step");
}

int sp_pixel_opt_step(const sp_op* op, float* x, float* exp_avg, float* exp_avg_sq,
                      const float* y, int64_t batch, int64_t y_div, float grad_scale,
                      const sp_adamw_coefs* c, const int32_t* stop, float* rsq_partial,
                      sp_stream_t stream) {
    if (!valid_op(op) || !x || !exp_avg || !exp_avg_sq || !y || !c || !rsq_partial ||
        batch <= 0 || batch > 65535 || y_div <= 0)
        return SP_EINVAL;
    if (op->kind == SP_OP_BLUR) return SP_EUNSUPPORTED;  // composed by the caller
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int P = static_cast<int>(tiles_elementwise(op->n));
    const dim3 grid(P, static_cast<unsigned>(batch));
    const bool v4 = op->n % 4 == 0;
#define SP_PO(OPK, V)                                                                         \
    launch(0, k_pixel_opt<OPK, V>, grid, dim3(kBlock), s, *op, x, exp_avg, exp_avg_sq, y, y_div, \
           grad_scale, *c, stop, rsq_partial, P)
    switch (op->kind) {
        case SP_OP_IDENTITY: if (v4) SP_PO(SP_OP_IDENTITY, 4); else SP_PO(SP_OP_IDENTITY, 1); break;
        case SP_OP_INPAINT: if (v4) SP_PO(SP_OP_INPAINT, 4); else SP_PO(SP_OP_INPAINT, 1); break;
        default: if (v4) SP_PO(SP_OP_MASK, 4); else SP_PO(SP_OP_MASK, 1); break;
    }
#undef SP_PO
    return check_launch("sp_pixel_opt_step");
}

int sp_opt_check(const float* partials, int64_t count, float total, double threshold,
                 int32_t* stop, float* loss_out, sp_stream_t stream) {
    if (!partials || !stop || count <= 0 || !(total > 0.f)) return SP_EINVAL;
    launch(0, k_opt_check, dim3(1), dim3(kBlock), static_cast<hipStream_t>(stream), partials,
           count, total, threshold, stop, loss_out);
    return check_launch("sp_opt_check");
}

int sp_opt_check_plateau(const float* partials, int64_t count, float total, double threshold,
                         int64_t itr, int64_t plateau_from, float* prev_loss, int32_t* stop,
                         float* loss_out, sp_stream_t stream) {
    if (!partials || !stop || !prev_loss || count <= 0 || !(total > 0.f) || itr < 0)
        return SP_EINVAL;
    launch(0, k_opt_check_plateau, dim3(1), dim3(kBlock), static_cast<hipStream_t>(stream),
           partials, count, total, threshold, itr, plateau_from, prev_loss, stop, loss_out);
    return check_launch("sp_opt_check_plateau");
}

}  // extern "C"

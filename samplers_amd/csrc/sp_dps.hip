// DPS guidance hot path for IDENTITY and INPAINT operators (elementwise in
// x-space), plus the elementwise helpers every sampler uses (x0 prediction,
// Philox normals, y-space likelihood gradient, inpaint gather/scatter).
//
// Memory model: every kernel streams contiguous fp32 rows of n elements with
// one float4 per lane (1 KiB per wave-instruction); a block covers
// kIter*1024 consecutive elements of ONE sample, grid = (tiles, batch), so the
// per-sample residual norm is a fixed-order sum of per-block partials — no
// atomics, bitwise reproducible.  Observation rows y are read in the packed
// order of the reference (kept pixels ascending), the keep bit-mask and
// per-word ranks (12 B per 64 pixels) stay L2-resident.

#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#define SP_TU 1  // debug-build site numbering (sp_common.h SP_DCHECK)
#include "sp_common.h"

namespace sp {

static thread_local char g_err[256] = "";

void set_error(const char* what, hipError_t e) {
    std::snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
}

int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(what, e);
        return SP_ELAUNCH;
    }
    return SP_OK;
}

#if SP_DEBUG
// readers of every translation unit's debug words (SP_DCHECK), registered at load time
static std::vector<dcheck_reader>& dcheck_readers() {
    static std::vector<dcheck_reader> v;
    return v;
}
void dcheck_register(dcheck_reader r) { dcheck_readers().push_back(r); }

// debug build self-test: every thread of one block states a false invariant (no memory access)
__global__ void k_dcheck_selftest(int limit) { SP_DCHECK(static_cast<int>(threadIdx.x) < limit); }
#endif

struct TimingRecord {
    int kind;
    double work;
    hipEvent_t start, stop;
};
static std::mutex g_timing_mu;
static bool g_timing = false;
static std::vector<TimingRecord> g_records;
static std::vector<hipEvent_t> g_event_pool;

bool timing_on() { return g_timing; }

static hipEvent_t take_event() {
    if (!g_event_pool.empty()) {
        hipEvent_t e = g_event_pool.back();
        g_event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

void timing_events(int kind, double work, hipEvent_t* start, hipEvent_t* stop) {
    std::lock_guard<std::mutex> lock(g_timing_mu);
    *start = take_event();
    *stop = take_event();
    if (*start && *stop) g_records.push_back({kind, work, *start, *stop});
}

// ---------------------------------------------------------------------------
// K1: x0 -> residual -> v = A^T(grad_scale * r), per-block sum r^2
// ---------------------------------------------------------------------------
#ifndef SP_UPD_NT
#define SP_UPD_NT 1  // non-temporal loads of the DPS passes' once-read streams (measured +4-5 %)
#endif
template <int OPK, int V>
__global__ __launch_bounds__(kBlock) void k_dps_residual(sp_op op, const float* __restrict__ x,
                                                         const float* __restrict__ eps,
                                                         const float* __restrict__ y, int64_t y_div,
                                                         float a, float k, float gs,
                                                         float* __restrict__ v,
                                                         float* __restrict__ partial, int P,
                                                         const sp_step_rec* __restrict__ sched,
                                                         const int32_t* __restrict__ cursor) {
    __shared__ float red[4];
    if (sched) {  // device-resident schedule (graph replay): uniform scalar loads
        const sp_dps_coefs& c = sched[*cursor].c;
        a = c.a, k = c.k, gs = c.grad_scale;
    }
    const int64_t b = blockIdx.y;
    const int64_t n = op.n;
    const float* xb = x + b * n;
    const float* eb = eps + b * n;
    const float* yb = y + (b / y_div) * op.m;
    float* vb = v + b * n;
    const int64_t j0 = (int64_t)blockIdx.x * kIter * (kBlock * V) + threadIdx.x * V;
    // issue every load of the tile first (memory-level parallelism), then compute
    float xv[kIter][V], ev[kIter][V], yv[kIter][V];
    uint32_t bits[kIter];
    int64_t rank[kIter];
#pragma unroll
    for (int it = 0; it < kIter; ++it) {
        const int64_t j = j0 + it * (kBlock * V);
        if (j < n) {
            load_v<V, SP_UPD_NT>(xb + j, xv[it]);
            load_v<V, SP_UPD_NT>(eb + j, ev[it]);
            if constexpr (OPK == SP_OP_INPAINT) {
                inpaint_lookup(op, j, bits[it], rank[it]);
            } else {
                load_v<V>(yb + j, yv[it]);
                if constexpr (OPK == SP_OP_MASK) bits[it] = mask_bits(op, j);
            }
        }
    }
    if constexpr (OPK == SP_OP_INPAINT) {
#pragma unroll
        for (int it = 0; it < kIter; ++it) {
            const int64_t j = j0 + it * (kBlock * V);
            if (j < n) {
                int64_t r = rank[it];
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    yv[it][e] = 0.f;
                    if ((bits[it] >> e) & 1u) yv[it][e] = yb[r];
                    r += (bits[it] >> e) & 1u;
                }
                SP_DCHECK(r <= op.m);  // packed observation index inside the row
            }
        }
    }
    float acc = 0.f;
#pragma unroll
    for (int it = 0; it < kIter; ++it) {
        const int64_t j = j0 + it * (kBlock * V);
        if (j < n) {
            float vv[V];
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const bool kept = OPK == SP_OP_IDENTITY || ((bits[it] >> e) & 1u);
                const float x0 = (xv[it][e] - k * ev[it][e]) / a;
                // MASK: unobserved pixels still add y^2 to the residual (A x0 = 0 there)
                const float r = yv[it][e] - (kept ? x0 : 0.f);
                vv[e] = kept ? gs * r : 0.f;
                if (OPK != SP_OP_INPAINT || kept) acc += r * r;
            }
            store_v<V>(vb + j, vv);
        }
    }
    const float t = block_sum(acc, red);
    SP_DCHECK(static_cast<int>(blockIdx.x) < P);
    if (threadIdx.x == 0) partial[b * P + blockIdx.x] = t;
}

// ---------------------------------------------------------------------------
// K2: bridge mean + std*xi + gamma/(||r_b|| + eps) * (v - k*w)/a
// ---------------------------------------------------------------------------
#ifndef SP_UPD_RCP
#define SP_UPD_RCP 1  // 1: multiply by 1/a instead of dividing (1 ulp from the reference's division)
#endif
#ifndef SP_UPD_WAVES
#define SP_UPD_WAVES 5  // waves per SIMD the update pass is built for (<= 80 VGPRs, see below)
#endif
// 6 waves per SIMD = 6 blocks per CU = 1536 resident blocks: the 3072 blocks of the B = 64,
// 256^2 step run in exactly two rounds (at 5, 83 VGPRs, they took 2.4 with a partial tail)
template <int OPK, int V, bool V_IN, bool XI_IN>
__global__ __launch_bounds__(kBlock, SP_UPD_WAVES) void k_dps_update(
    sp_op op, const float* __restrict__ x, const float* __restrict__ eps,
    const float* __restrict__ y, const float* __restrict__ v, const float* __restrict__ w,
    const float* __restrict__ partial, int P, const float* __restrict__ xi, uint64_t seed,
    int64_t step, int64_t sample_offset, int64_t y_div, sp_dps_coefs c, float* __restrict__ xo,
    const sp_step_rec* __restrict__ sched, const int32_t* __restrict__ cursor) {
    if (sched) {  // device-resident schedule (graph replay)
        const sp_step_rec& rec = sched[*cursor];
        c = rec.c;
        step = rec.step;
    }
    const int64_t b = blockIdx.y;
    const int64_t n = op.n;
    const float* xb = x + b * n;
    const float* eb = eps + b * n;
    const float* wb = w + b * n;
    const float* yb = y + (b / y_div) * op.m;
    float* ob = xo + b * n;
    const int64_t j0 = (int64_t)blockIdx.x * kIter * (kBlock * V) + threadIdx.x * V;
    float xv[kIter][V], ev[kIter][V], wv[kIter][V], yv[kIter][V];
    uint32_t bits[kIter];
    int64_t rank[kIter];
#pragma unroll
    for (int it = 0; it < kIter; ++it) {
        const int64_t j = j0 + it * (kBlock * V);
        if (j < n) {
            load_v<V, SP_UPD_NT>(xb + j, xv[it]);
            load_v<V, SP_UPD_NT>(eb + j, ev[it]);
            load_v<V, SP_UPD_NT>(wb + j, wv[it]);
            if constexpr (V_IN) {
                load_v<V, SP_UPD_NT>(v + b * n + j, yv[it]);  // yv holds v in this variant
            } else if constexpr (OPK == SP_OP_INPAINT) {
                inpaint_lookup(op, j, bits[it], rank[it]);
            } else {
                load_v<V>(yb + j, yv[it]);
                if constexpr (OPK == SP_OP_MASK) bits[it] = mask_bits(op, j);
            }
        }
    }
    if constexpr (!V_IN && OPK == SP_OP_INPAINT) {
#pragma unroll
        for (int it = 0; it < kIter; ++it) {
            const int64_t j = j0 + it * (kBlock * V);
            if (j < n) {
                int64_t r = rank[it];
#pragma unroll
                for (int e = 0; e < V; ++e) {
                    yv[it][e] = 0.f;
                    if ((bits[it] >> e) & 1u) yv[it][e] = yb[r];
                    r += (bits[it] >> e) & 1u;
                }
                SP_DCHECK(r <= op.m);
            }
        }
    }
    SP_DCHECK(!partial || P > 0);
    const float inv_a = 1.f / c.a;
    // DPS: gamma / (||r_b|| + eps); without partials a fixed factor (PGDM, PSLD)
    __shared__ float red4[4];
    const float scale =
        partial ? c.gamma / (sqrtf(block_sum_partials(partial + b * P, P, red4)) + c.norm_eps) : c.gamma;
#pragma unroll
    for (int it = 0; it < kIter; ++it) {
        const int64_t j = j0 + it * (kBlock * V);
        if (j < n) {
            float z[V];
            if constexpr (XI_IN) {
                load_v<V>(xi + b * n + j, z);
            } else {
                philox_normals<V>(seed, step, sample_offset + b, j, z);
            }
            float out[V];
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const float x0 = SP_UPD_RCP ? (xv[it][e] - c.k * ev[it][e]) * inv_a
                                            : (xv[it][e] - c.k * ev[it][e]) / c.a;
                float vv;
                if constexpr (V_IN) {
                    vv = yv[it][e];
                } else {
                    const bool kept = OPK == SP_OP_IDENTITY || ((bits[it] >> e) & 1u);
                    vv = kept ? c.grad_scale * (yv[it][e] - x0) : 0.f;
                }
                const float mean = c.c_ell * xv[it][e] + c.c_s * x0;
                const float g = SP_UPD_RCP ? (vv - c.k * wv[it][e]) * inv_a : (vv - c.k * wv[it][e]) / c.a;
                out[e] = (mean + c.std * z[e]) + scale * g;
            }
            store_v<V, true>(ob + j, out);
        }
    }
}

// ---------------------------------------------------------------------------
// elementwise helpers
// ---------------------------------------------------------------------------
template <int V>
__global__ __launch_bounds__(kBlock) void k_predict_x0(const float* __restrict__ x,
                                                       const float* __restrict__ eps, int64_t count,
                                                       float a, float k, float* __restrict__ out) {
    const int64_t stride = (int64_t)gridDim.x * kBlock * V;
    for (int64_t j = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * V; j < count; j += stride) {
        float xv[V], ev[V], o[V];
        load_v<V>(x + j, xv);
        load_v<V>(eps + j, ev);
#pragma unroll
        for (int e = 0; e < V; ++e) o[e] = (xv[e] - k * ev[e]) / a;
        store_v<V>(out + j, o);
    }
}

template <int V>
__global__ __launch_bounds__(kBlock) void k_randn(float* __restrict__ out, int64_t n, uint64_t seed,
                                                  int64_t step, int64_t sample_offset) {
    const int64_t b = blockIdx.y;
    const int64_t stride = (int64_t)gridDim.x * kBlock * V;
    for (int64_t j = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * V; j < n; j += stride) {
        float z[V];
        philox_normals<V>(seed, step, sample_offset + b, j, z);
        store_v<V>(out + b * n + j, z);
    }
}

template <int V>
__global__ __launch_bounds__(kBlock) void k_residual_grad(const float* __restrict__ y,
                                                          const float* __restrict__ z, int64_t m,
                                                          int64_t y_div, float gs,
                                                          float* __restrict__ g,
                                                          float* __restrict__ partial, int P) {
    __shared__ float red[4];
    const int64_t b = blockIdx.y;
    const float* yb = y + (b / y_div) * m;
    const float* zb = z + b * m;
    float acc = 0.f;
#pragma unroll
    for (int it = 0; it < kIter; ++it) {
        const int64_t j = ((int64_t)blockIdx.x * kIter + it) * (kBlock * V) + threadIdx.x * V;
        if (j < m) {
            float yv[V], zv[V], gv[V];
            load_v<V>(yb + j, yv);
            load_v<V>(zb + j, zv);
#pragma unroll
            for (int e = 0; e < V; ++e) {
                const float r = yv[e] - zv[e];
                gv[e] = gs * r;
                acc += r * r;
            }
            if (g) store_v<V>(g + b * m + j, gv);
        }
    }
    const float t = block_sum(acc, red);
    if (threadIdx.x == 0 && partial) partial[b * P + blockIdx.x] = t;
}

// y[b][rank(j)] = x[b][j] for observed j (gather, inpainting.py:132-145)
template <int V>
__global__ __launch_bounds__(kBlock) void k_inpaint_gather(sp_op op, const float* __restrict__ x,
                                                           float* __restrict__ y) {
    const int64_t b = blockIdx.y;
    const int64_t n = op.n;
    const int64_t stride = (int64_t)gridDim.x * kBlock * V;
    for (int64_t j = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * V; j < n; j += stride) {
        float xv[V];
        load_v<V>(x + b * n + j, xv);
        uint32_t bits;
        int64_t rank;
        inpaint_lookup(op, j, bits, rank);
#pragma unroll
        for (int e = 0; e < V; ++e)
            if ((bits >> e) & 1u) y[b * op.m + rank++] = xv[e];
        SP_DCHECK(rank <= op.m);
    }
}

// x[b][j] = observed(j) ? y[b][rank(j)] : 0 (scatter into zeros, inpainting.py:169-187)
template <int V>
__global__ __launch_bounds__(kBlock) void k_inpaint_scatter(sp_op op, const float* __restrict__ y,
                                                            float* __restrict__ x) {
    const int64_t b = blockIdx.y;
    const int64_t n = op.n;
    const int64_t stride = (int64_t)gridDim.x * kBlock * V;
    for (int64_t j = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * V; j < n; j += stride) {
        float xv[V];
        uint32_t bits;
        int64_t rank;
        inpaint_lookup(op, j, bits, rank);
#pragma unroll
        for (int e = 0; e < V; ++e) xv[e] = ((bits >> e) & 1u) ? y[b * op.m + rank++] : 0.f;
        SP_DCHECK(rank <= op.m);
        store_v<V>(x + b * n + j, xv);
    }
}

// y = keep ? x : 0 (inpainting.py:106-109 / :180-187 with flatten=False); self-adjoint
template <int V>
__global__ __launch_bounds__(kBlock) void k_mask(sp_op op, const float* __restrict__ x,
                                                 float* __restrict__ y) {
    const int64_t b = blockIdx.y;
    const int64_t n = op.n;
    const int64_t stride = (int64_t)gridDim.x * kBlock * V;
    for (int64_t j = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * V; j < n; j += stride) {
        float xv[V];
        load_v<V>(x + b * n + j, xv);
        const uint32_t bits = mask_bits(op, j);
#pragma unroll
        for (int e = 0; e < V; ++e) xv[e] = ((bits >> e) & 1u) ? xv[e] : 0.f;
        store_v<V>(y + b * n + j, xv);
    }
}

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// grid.x for grid-stride kernels: enough blocks to fill 256 CUs a few times over
static inline unsigned stride_blocks(int64_t work, int V, int64_t batch) {
    int64_t blocks = cdiv(work, (int64_t)kBlock * V);
    const int64_t cap = std::max<int64_t>(1, 4096 / std::max<int64_t>(batch, 1));
    if (blocks > cap) blocks = cap;
    return static_cast<unsigned>(std::max<int64_t>(blocks, 1));
}

int64_t tiles_elementwise(int64_t n) {
    const int V = (n % 4 == 0) ? 4 : 1;
    return cdiv(n, (int64_t)kIter * kBlock * V);
}

bool valid_op(const sp_op* op) {
    if (!op || op->n <= 0 || op->m <= 0) return false;
    switch (op->kind) {
        case SP_OP_IDENTITY: return op->m == op->n;
        case SP_OP_INPAINT: return op->keep_bits && op->word_rank && op->m <= op->n;
        case SP_OP_MASK: return op->keep_bits && op->m == op->n;
        case SP_OP_BLUR:
            return op->taps && op->radius >= 1 && op->radius <= 8 && op->m == op->n &&
                   (int64_t)op->channels * op->height * op->width == op->n &&
                   op->height > 2 * op->radius && op->width > 2 * op->radius;
        default: return false;
    }
}

// blur entry points (sp_blur.hip)
int64_t blur_partials(const sp_op* op);
int blur_dps_residual(const sp_op* op, const float* x, const float* eps, const float* y,
                      int64_t batch, int64_t y_div, float a, float k, float gs,
                      const sp_step_rec* sched, const int32_t* cursor, float* v, float* partial,
                      hipStream_t s);
int blur_apply(const sp_op* op, const float* x, float* y, int64_t batch, hipStream_t s);
int blur_adjoint(const sp_op* op, const float* y, float* x, int64_t batch, hipStream_t s);

}  // namespace sp

using namespace sp;

extern "C" {

int sp_version(void) { return 101; }

int sp_debug_build(void) { return SP_DEBUG; }

int64_t sp_debug_violations(int32_t reset, int32_t* first_site) {
    if (first_site) *first_site = 0;
#if SP_DEBUG
    if (hipDeviceSynchronize() != hipSuccess) return check_launch("sp_debug_violations");
    int64_t total = 0;
    for (dcheck_reader r : dcheck_readers()) {
        unsigned w[2] = {0u, 0u};
        if (r(w, reset) != 0) return check_launch("sp_debug_violations (read)");
        if (w[0] && first_site && !*first_site) *first_site = static_cast<int32_t>(w[1]);
        total += w[0];
    }
    return total;
#else
    (void)reset;
    return 0;
#endif
}

int sp_debug_selftest(sp_stream_t stream) {
#if SP_DEBUG
    launch(0, k_dcheck_selftest, dim3(1), dim3(64), static_cast<hipStream_t>(stream), 0);
    return check_launch("sp_debug_selftest");
#else
    (void)stream;
    return SP_EINVAL;
#endif
}

int sp_timing_enable(int on) {
    std::lock_guard<std::mutex> lock(g_timing_mu);
    g_timing = on != 0;
    return SP_OK;
}

int sp_timing_collect(int32_t* kinds, float* ms, int max_records) {
    return sp_timing_collect_work(kinds, ms, nullptr, max_records);
}

int sp_timing_collect_work(int32_t* kinds, float* ms, double* work, int max_records) {
    std::lock_guard<std::mutex> lock(g_timing_mu);
    int n = 0;
    for (const TimingRecord& r : g_records) {
        float t = -1.f;
        if (hipEventSynchronize(r.stop) == hipSuccess && hipEventElapsedTime(&t, r.start, r.stop) == hipSuccess &&
            n < max_records && kinds && ms) {
            kinds[n] = r.kind;
            ms[n] = t;
            if (work) work[n] = r.work;
            ++n;
        }
        g_event_pool.push_back(r.start);
        g_event_pool.push_back(r.stop);
    }
    g_records.clear();
    return n;
}

const char* sp_last_error(void) { return g_err; }

int64_t sp_rsq_partials(const sp_op* op) {
    if (!valid_op(op)) return SP_EINVAL;
    if (op->kind == SP_OP_BLUR) return blur_partials(op);
    return tiles_elementwise(op->n);
}

int64_t sp_vec_partials(int64_t count) { return count > 0 ? tiles_elementwise(count) : SP_EINVAL; }

static int dps_residual_impl(const sp_op* op, const float* x, const float* eps, const float* y,
                             int64_t batch, int64_t y_div, sp_dps_coefs c,
                             const sp_step_rec* sched, const int32_t* cursor, float* v_out,
                             float* rsq_partial, sp_stream_t stream) {
    if (!valid_op(op) || !x || !eps || !y || !v_out || !rsq_partial || batch <= 0 ||
        y_div <= 0 || batch > 65535)
        return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (op->kind == SP_OP_BLUR)
        return blur_dps_residual(op, x, eps, y, batch, y_div, c.a, c.k, c.grad_scale, sched,
                                 cursor, v_out, rsq_partial, s);
    const int P = static_cast<int>(tiles_elementwise(op->n));
    const dim3 grid(P, static_cast<unsigned>(batch));
    const bool v4 = op->n % 4 == 0;
#define SP_K1(OPK, V)                                                                       \
    launch_w(TK_DPS_RESIDUAL, (double)batch, k_dps_residual<OPK, V>, grid, dim3(kBlock), s, *op, x, eps, y, y_div, \
           c.a, c.k, c.grad_scale, v_out, rsq_partial, P, sched, cursor)
    if (op->kind == SP_OP_IDENTITY) {
        if (v4) SP_K1(SP_OP_IDENTITY, 4); else SP_K1(SP_OP_IDENTITY, 1);
    } else if (op->kind == SP_OP_MASK) {
        if (v4) SP_K1(SP_OP_MASK, 4); else SP_K1(SP_OP_MASK, 1);
    } else {
        if (v4) SP_K1(SP_OP_INPAINT, 4); else SP_K1(SP_OP_INPAINT, 1);
    }
#undef SP_K1
    return check_launch("sp_dps_residual");
}

int sp_dps_residual(const sp_op* op, const float* x, const float* eps, const float* y,
                    int64_t batch, int64_t y_div, const sp_dps_coefs* c, float* v_out,
                    float* rsq_partial, sp_stream_t stream) {
    if (!c) return SP_EINVAL;
    return dps_residual_impl(op, x, eps, y, batch, y_div, *c, nullptr, nullptr, v_out, rsq_partial,
                             stream);
}

int sp_dps_residual_sched(const sp_op* op, const float* x, const float* eps, const float* y,
                          int64_t batch, int64_t y_div, const sp_step_rec* sched,
                          const int32_t* cursor, float* v_out, float* rsq_partial,
                          sp_stream_t stream) {
    if (!sched || !cursor) return SP_EINVAL;
    return dps_residual_impl(op, x, eps, y, batch, y_div, sp_dps_coefs{}, sched, cursor, v_out,
                             rsq_partial, stream);
}

static int dps_update_impl(const sp_op* op, const float* x, const float* eps, const float* y,
                           const float* v, const float* w, const float* rsq_partial,
                           const float* xi, uint64_t seed, int64_t step, int64_t sample_offset,
                           int64_t batch, int64_t y_div, sp_dps_coefs c,
                           const sp_step_rec* sched, const int32_t* cursor, float* x_out,
                           sp_stream_t stream) {
    if (!valid_op(op) || !x || !eps || !w || !x_out || batch <= 0 || y_div <= 0 ||
        batch > 65535)
        return SP_EINVAL;
    if (!v && (op->kind == SP_OP_BLUR || !y)) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int P = static_cast<int>(sp_rsq_partials(op));
    const int Pw = static_cast<int>(tiles_elementwise(op->n));
    const dim3 grid(Pw, static_cast<unsigned>(batch));
    const bool v4 = op->n % 4 == 0;
    const int opk = op->kind == SP_OP_BLUR ? SP_OP_IDENTITY : op->kind;  // BLUR reads v
#define SP_K2(OPK, V, VIN, XIN)                                                            \
    launch_w(TK_DPS_UPDATE, (double)batch, k_dps_update<OPK, V, VIN, XIN>, grid, dim3(kBlock), s, *op, x, eps, y, \
           v, w, rsq_partial, P, xi, seed, step, sample_offset, y_div, c, x_out, sched, cursor)
#define SP_K2_XI(OPK, V, VIN) \
    if (xi) SP_K2(OPK, V, VIN, true); else SP_K2(OPK, V, VIN, false)
#define SP_K2_V(OPK, V) \
    if (v) { SP_K2_XI(OPK, V, true); } else { SP_K2_XI(OPK, V, false); }
    if (opk == SP_OP_IDENTITY) {
        if (v4) { SP_K2_V(SP_OP_IDENTITY, 4) } else { SP_K2_V(SP_OP_IDENTITY, 1) }
    } else if (opk == SP_OP_MASK) {
        if (v4) { SP_K2_V(SP_OP_MASK, 4) } else { SP_K2_V(SP_OP_MASK, 1) }
    } else {
        if (v4) { SP_K2_V(SP_OP_INPAINT, 4) } else { SP_K2_V(SP_OP_INPAINT, 1) }
    }
#undef SP_K2_V
#undef SP_K2_XI
#undef SP_K2
    return check_launch("sp_dps_update");
}

int sp_dps_update(const sp_op* op, const float* x, const float* eps, const float* y,
                  const float* v, const float* w, const float* rsq_partial, const float* xi,
                  uint64_t seed, int64_t step, int64_t sample_offset, int64_t batch, int64_t y_div,
                  const sp_dps_coefs* c, float* x_out, sp_stream_t stream) {
    if (!c) return SP_EINVAL;
    return dps_update_impl(op, x, eps, y, v, w, rsq_partial, xi, seed, step, sample_offset, batch,
                           y_div, *c, nullptr, nullptr, x_out, stream);
}

int sp_dps_update_sched(const sp_op* op, const float* x, const float* eps, const float* y,
                        const float* v, const float* w, const float* rsq_partial,
                        uint64_t seed, int64_t sample_offset, int64_t batch, int64_t y_div,
                        const sp_step_rec* sched, const int32_t* cursor, float* x_out,
                        sp_stream_t stream) {
    if (!sched || !cursor) return SP_EINVAL;
    return dps_update_impl(op, x, eps, y, v, w, rsq_partial, nullptr, seed, 0, sample_offset,
                           batch, y_div, sp_dps_coefs{}, sched, cursor, x_out, stream);
}

__global__ void k_sched_timestep(const sp_step_rec* sched, const int32_t* cursor, int64_t* t) {
    *t = sched[*cursor].t;
}

__global__ void k_sched_advance(int32_t* cursor) { *cursor += 1; }

int sp_sched_timestep(const sp_step_rec* sched, const int32_t* cursor, int64_t* t_out,
                      sp_stream_t stream) {
    if (!sched || !cursor || !t_out) return SP_EINVAL;
    launch(0, k_sched_timestep, dim3(1), dim3(1), static_cast<hipStream_t>(stream), sched, cursor,
           t_out);
    return check_launch("sp_sched_timestep");
}

int sp_sched_advance(int32_t* cursor, sp_stream_t stream) {
    if (!cursor) return SP_EINVAL;
    launch(0, k_sched_advance, dim3(1), dim3(1), static_cast<hipStream_t>(stream), cursor);
    return check_launch("sp_sched_advance");
}

int sp_predict_x0(const float* x, const float* eps, int64_t count, float a, float k, float* out,
                  sp_stream_t stream) {
    if (!x || !eps || !out || count <= 0) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool v4 = count % 4 == 0 && ((uintptr_t)x % 16 == 0) && ((uintptr_t)eps % 16 == 0) &&
                    ((uintptr_t)out % 16 == 0);
    if (v4)
        hipLaunchKernelGGL(k_predict_x0<4>, dim3(stride_blocks(count, 4, 1)), dim3(kBlock), 0, s,
                           x, eps, count, a, k, out);
    else
        hipLaunchKernelGGL(k_predict_x0<1>, dim3(stride_blocks(count, 1, 1)), dim3(kBlock), 0, s,
                           x, eps, count, a, k, out);
    return check_launch("sp_predict_x0");
}

int sp_randn(float* out, int64_t batch, int64_t n, uint64_t seed, int64_t step,
             int64_t sample_offset, sp_stream_t stream) {
    if (!out || batch <= 0 || n <= 0 || batch > 65535) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (n % 4 == 0)
        hipLaunchKernelGGL(k_randn<4>, dim3(stride_blocks(n, 4, batch), batch), dim3(kBlock), 0, s,
                           out, n, seed, step, sample_offset);
    else
        hipLaunchKernelGGL(k_randn<1>, dim3(stride_blocks(n, 1, batch), batch), dim3(kBlock), 0, s,
                           out, n, seed, step, sample_offset);
    return check_launch("sp_randn");
}

int sp_residual_grad(const float* y, const float* z, int64_t batch, int64_t m, int64_t y_div,
                     float grad_scale, float* g, float* rsq_partial, sp_stream_t stream) {
    if (!y || !z || batch <= 0 || m <= 0 || y_div <= 0 || batch > 65535 || (!g && !rsq_partial))
        return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int P = static_cast<int>(tiles_elementwise(m));
    const dim3 grid(P, static_cast<unsigned>(batch));
    if (m % 4 == 0)
        hipLaunchKernelGGL(k_residual_grad<4>, grid, dim3(kBlock), 0, s, y, z, m, y_div,
                           grad_scale, g, rsq_partial, P);
    else
        hipLaunchKernelGGL(k_residual_grad<1>, grid, dim3(kBlock), 0, s, y, z, m, y_div,
                           grad_scale, g, rsq_partial, P);
    return check_launch("sp_residual_grad");
}

int sp_op_apply(const sp_op* op, const float* x, float* y, int64_t batch, sp_stream_t stream) {
    if (!valid_op(op) || !x || !y || batch <= 0 || batch > 65535) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (op->kind) {
        case SP_OP_IDENTITY: {
            const hipError_t e = hipMemcpyAsync(y, x, sizeof(float) * op->n * batch,
                                                hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) { set_error("sp_op_apply", e); return SP_ELAUNCH; }
            return SP_OK;
        }
        case SP_OP_INPAINT: {
            const dim3 grid(stride_blocks(op->n, op->n % 4 == 0 ? 4 : 1, batch), batch);
            if (op->n % 4 == 0)
                hipLaunchKernelGGL(k_inpaint_gather<4>, grid, dim3(kBlock), 0, s, *op, x, y);
            else
                hipLaunchKernelGGL(k_inpaint_gather<1>, grid, dim3(kBlock), 0, s, *op, x, y);
            return check_launch("sp_op_apply");
        }
        case SP_OP_MASK: {
            const dim3 grid(stride_blocks(op->n, op->n % 4 == 0 ? 4 : 1, batch), batch);
            if (op->n % 4 == 0)
                hipLaunchKernelGGL(k_mask<4>, grid, dim3(kBlock), 0, s, *op, x, y);
            else
                hipLaunchKernelGGL(k_mask<1>, grid, dim3(kBlock), 0, s, *op, x, y);
            return check_launch("sp_op_apply");
        }
        case SP_OP_BLUR: return blur_apply(op, x, y, batch, s);
    }
    return SP_EINVAL;
}

int sp_op_adjoint(const sp_op* op, const float* y, float* x, int64_t batch, sp_stream_t stream) {
    if (!valid_op(op) || !x || !y || batch <= 0 || batch > 65535) return SP_EINVAL;
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (op->kind) {
        case SP_OP_IDENTITY: {
            const hipError_t e = hipMemcpyAsync(x, y, sizeof(float) * op->n * batch,
                                                hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) { set_error("sp_op_adjoint", e); return SP_ELAUNCH; }
            return SP_OK;
        }
        case SP_OP_INPAINT: {
            const dim3 grid(stride_blocks(op->n, op->n % 4 == 0 ? 4 : 1, batch), batch);
            if (op->n % 4 == 0)
                hipLaunchKernelGGL(k_inpaint_scatter<4>, grid, dim3(kBlock), 0, s, *op, y, x);
            else
                hipLaunchKernelGGL(k_inpaint_scatter<1>, grid, dim3(kBlock), 0, s, *op, y, x);
            return check_launch("sp_op_adjoint");
        }
        case SP_OP_MASK: {
            const dim3 grid(stride_blocks(op->n, op->n % 4 == 0 ? 4 : 1, batch), batch);
            if (op->n % 4 == 0)
                hipLaunchKernelGGL(k_mask<4>, grid, dim3(kBlock), 0, s, *op, y, x);
            else
                hipLaunchKernelGGL(k_mask<1>, grid, dim3(kBlock), 0, s, *op, y, x);
            return check_launch("sp_op_adjoint");
        }
        case SP_OP_BLUR: return blur_adjoint(op, y, x, batch, s);
    }
    return SP_EINVAL;
}

}  // extern "C"

/*
 * samplers_hip.h — C ABI of libsamplers_hip.so, the MI355X (gfx950) hot path of
 * diffusion posterior sampling (DPS / PSLD / PGDM / ReSample guidance steps).
 *
 * The reference (thomashirtz/samplers) is pure Python over PyTorch; every entry
 * point below replaces a group of eager ATen calls that the reference issues
 * per reverse-diffusion step.  Each declaration cites the reference code it
 * replaces (paths relative to the reference repository root).
 *
 * Conventions (all entry points):
 *   - device pointers to contiguous fp32 data; a "sample" is one row of
 *     n = C*H*W elements (x-space) or m elements (y-space, observation);
 *   - `stream` is the caller's hipStream_t (PyTorch passes its current stream);
 *     every call is asynchronous on that stream and never synchronises;
 *   - the library allocates nothing; callers pass every buffer;
 *   - return 0 on success, a negative SP_E* code on bad arguments or a failed
 *     launch (the launch error is also readable through sp_last_error()).
 *   - observation row for sample b is b / y_div (y_div = number of
 *     reconstructions sharing one observation, >= 1).
 */
#ifndef SAMPLERS_HIP_H
#define SAMPLERS_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* sp_stream_t; /* hipStream_t */

enum {
    SP_OK = 0,
    SP_EINVAL = -1,   /* bad argument (null pointer, size, unsupported operator kind) */
    SP_ELAUNCH = -2,  /* kernel launch failed */
    SP_EUNSUPPORTED = -3
};

/* Operator kinds (reference: samplers/operators/). */
enum {
    SP_OP_IDENTITY = 0, /* identity.py:8-68        y = x                      */
    SP_OP_INPAINT = 1,  /* inpainting.py:8-195     y = x.flat[kept]            */
    SP_OP_BLUR = 2,     /* new (BASELINE config 3): depthwise separable Gaussian
                           blur with reflect padding; adjoint = exact transpose */
    SP_OP_MASK = 3      /* inpainting.py:106-109 (flatten=False): y = x with the
                           masked pixels zeroed; uses keep_bits only, m == n   */
};

/* Forward-operator descriptor.  Device arrays are owned by the caller
 * (the Python Operator's buffers) and must outlive every call using them. */
typedef struct sp_op {
    int32_t kind;
    int32_t channels, height, width; /* x_shape = (C, H, W); n = C*H*W        */
    int64_t n;                       /* elements per x sample                 */
    int64_t m;                       /* elements per y sample                 */
    const uint64_t* keep_bits;       /* INPAINT: ceil(n/64) words; bit (j%64) of
                                        word j/64 set <=> x[j] observed (= ~mask) */
    const int32_t* word_rank;        /* INPAINT: observed count before word w  */
    const float* taps;               /* BLUR: 2*radius+1 normalised taps       */
    int32_t radius;                  /* BLUR: 1..8                             */
    int32_t reserved;
} sp_op;

/* Scalars of one DPS step (all fp32, computed on the host exactly as the
 * reference computes them). */
typedef struct sp_dps_coefs {
    float a;          /* sqrt(alpha_bar[t])      networks/base.py:41-43          */
    float k;          /* sqrt(1 - alpha_bar[t])                                   */
    float grad_scale; /* d logp / d(Ax): 1/sigma^2 (noise.py:77-79) or
                         2/(rate+1e-3) (noise.py:121-123)                          */
    float c_ell;      /* bridge_coeff_ell        bridge_kernels.py:36            */
    float c_s;        /* bridge_coeff_s          bridge_kernels.py:37            */
    float std;        /* bridge_std              bridge_kernels.py:33-35         */
    float gamma;      /* DPS step size           dps.py:121                      */
    float norm_eps;   /* 1e-9                    dps.py:121                      */
} sp_dps_coefs;

/* Scalars of the epsilon-form DDIM step (bridge_kernels.py:82-115), fp32 as there. */
typedef struct sp_eps_coefs {
    float sqrt_oma;    /* sqrt(1 - acp_t)                                   */
    float oma;         /* 1 - acp_t                  (pseudo-x0)            */
    float sqrt_a;      /* sqrt(acp_t)                                       */
    float sqrt_a_prev; /* sqrt(acp_prev)                                    */
    float sigma;       /* eta*sqrt(clamp((1-acp_prev)/(1-acp_t)*(1-acp_t/acp_prev)))      */
    float dir;         /* sqrt(clamp(1 - acp_prev - sigma^2))                */
} sp_eps_coefs;

/* One torch.optim.AdamW step (resample_kernels.py:32-93 optimisers). */
typedef struct sp_adamw_coefs {
    float decay;      /* 1 - lr*weight_decay                                 */
    float beta1;      /* 0.9                                                 */
    float beta2;      /* 0.999                                               */
    float eps;        /* 1e-8                                                */
    float step_size;  /* lr / (1 - beta1^step)                               */
    float bc2_sqrt;   /* sqrt(1 - beta2^step)                                */
} sp_adamw_coefs;

/* Kernel timing (instrumentation, off by default).  While enabled, every
 * sp_dps_residual / sp_dps_update launch gets a start/stop hipEvent pair attached
 * to its dispatch packet (hipExtLaunchKernel), i.e. the kernel's own execution
 * interval.  sp_timing_collect waits for the recorded launches, writes up to
 * max_records (kind, milliseconds) pairs — kind 1 = residual pass, 2 = update
 * pass — clears the log and returns the number written. */
int sp_timing_enable(int on);
int sp_timing_collect(int32_t* kinds, float* ms, int max_records);
/* As sp_timing_collect, plus each launch's algorithmic work: samples for kinds 1-2 (DPS
 * passes), FLOPs for kinds 3-4 (sp_conv3x3_fwd / _bwd_input: 18*N*Cin*Cout*H*W) and
 * executed MFMA FLOPs for kinds 5-6 (sp_wino3x3_fwd / _bwd_input: 8*N*Cin*Cout*H*W) and FLOPs
 * for kind 7 (sp_conv3x3_bf16, forward or input VJP: 18*N*Cin*Cout*H*W). */
int sp_timing_collect_work(int32_t* kinds, float* ms, double* work, int max_records);

/* Library / ABI version (major*10000 + minor*100 + patch). */
int sp_version(void);
/* Text of the last launch error on this thread ("" if none). */
const char* sp_last_error(void);

/* Bounds-checked debug build (`make debug` -> samplers_amd/lib/debug/libsamplers_hip.so,
 * -DSP_DEBUG=1; SURVEY.md §5 "race detection / sanitizers"): the kernels' index / range
 * invariants (SP_DCHECK) are checked on the device and counted.  No reference counterpart
 * (the reference has no native code); test and diagnosis tooling.
 *   sp_debug_build       1 in the debug library, 0 in the release one.
 *   sp_debug_violations  waits for the device, returns the number of violated checks since the
 *                        last reset (0 in the release build, < 0 on error); *first_site
 *                        (nullable) = (source file id << 16) | line of the first one.
 *   sp_debug_selftest    debug build: one launch whose 64 threads each violate a check (no
 *                        memory access), to prove the counting works; SP_EINVAL otherwise. */
int sp_debug_build(void);
int64_t sp_debug_violations(int32_t reset, int32_t* first_site);
int sp_debug_selftest(sp_stream_t stream);

/* Number of per-sample partial sums written by sp_dps_residual for `op`
 * (callers allocate batch * sp_rsq_partials(op) floats). */
int64_t sp_rsq_partials(const sp_op* op);

/* DPS pass 1 — replaces dps.py:99-103 up to the prior's VJP and dps.py:117-118:
 *   x0  = (x - k*eps)/a                         (networks/base.py:41-43)
 *   r   = y - A(x0)                             (inverse_problem.py:17-18)
 *   v   = A^T(grad_scale * r)  -> v_out         (autograd of noise.log_prob through A)
 *   rsq_partial[b][p] = partial sums of r^2 over sample b (dps.py:117-120).
 * v_out is the cotangent of x0; the caller feeds it to the prior's VJP. */
int sp_dps_residual(const sp_op* op, const float* x, const float* eps, const float* y,
                    int64_t batch, int64_t y_div, const sp_dps_coefs* c,
                    float* v_out, float* rsq_partial, sp_stream_t stream);

/* DPS pass 2 — replaces dps.py:106-122 (ddim_step -> sample_bridge_kernel and
 * the guidance correction):
 *   g   = v/a - (k/a) * w          (w = J_eps^T v from the prior's VJP)
 *   x'  = c_ell*x + c_s*x0 + std*xi + gamma/(sqrt(sum_p rsq_partial[b][p]) + norm_eps) * g
 * v: pass NULL to recompute v from (x, eps, y) (IDENTITY/INPAINT/MASK), else
 *    the buffer written by sp_dps_residual (required for BLUR).
 * rsq_partial: NULL selects a fixed factor, x' = ... + gamma * g — the PGDM update
 *    (pgdm.py:126-135, gamma = -guidance_weight*sqrt(1-acp_t), v = -2 A^T r) and the
 *    PSLD update (psld.py:144-153, gamma = -1, v = the latent cotangent).
 * xi: injected standard-normal noise (B*n) or NULL to draw Philox4x32-10
 *    normals keyed by (seed, step, sample_offset + b, element) — invariant to
 *    how the batch is sharded across GPUs.  x_out may alias x. */
int sp_dps_update(const sp_op* op, const float* x, const float* eps, const float* y,
                  const float* v, const float* w, const float* rsq_partial, const float* xi,
                  uint64_t seed, int64_t step, int64_t sample_offset,
                  int64_t batch, int64_t y_div, const sp_dps_coefs* c,
                  float* x_out, sp_stream_t stream);

/* x0 = (x - k*eps)/a over `count` elements (networks/base.py:41-43; final
 * prediction dps.py:125-126). out may alias x. */
int sp_predict_x0(const float* x, const float* eps, int64_t count, float a, float k,
                  float* out, sp_stream_t stream);

/* Standard normals, Philox4x32-10 keyed by (seed, step, sample_offset+b, j);
 * replaces torch.randn / randn_like (dps.py:83-87, bridge_kernels.py:59). */
int sp_randn(float* out, int64_t batch, int64_t n, uint64_t seed, int64_t step,
             int64_t sample_offset, sp_stream_t stream);

/* y = A x (operators/base.py:91-92; linear.py:141-152; inpainting.py:132-145). */
int sp_op_apply(const sp_op* op, const float* x, float* y, int64_t batch, sp_stream_t stream);
/* x = A^T y (linear.py:154-165; inpainting.py:169-187). */
int sp_op_adjoint(const sp_op* op, const float* y, float* x, int64_t batch, sp_stream_t stream);

/* Likelihood gradient in y-space (noise.py:19-27 score, 77-79, 121-123):
 *   r = y[b/y_div] - z[b];  g[b] = grad_scale * r;  rsq_partial[b][p] += r^2 partials.
 * g may be NULL (norm only).  Partials per sample: sp_vec_partials(m). */
int64_t sp_vec_partials(int64_t count);
int sp_residual_grad(const float* y, const float* z, int64_t batch, int64_t m, int64_t y_div,
                     float grad_scale, float* g, float* rsq_partial, sp_stream_t stream);

/* ---- latent samplers (PSLD psld.py:118-153, ReSample resample.py:131-228) ---------- */

/* PSLD pixel pass for IDENTITY / INPAINT / MASK (BLUR returns SP_EUNSUPPORTED: the
 * caller composes it from sp_op_apply / sp_op_adjoint):
 *   r = y - A x0,  x_eff = A^T y + x0 - A^T A x0,  atr = A^T r,
 *   rsq_partial[b][p] = partial sums of r^2 (sp_rsq_partials(op) per sample). */
int sp_psld_pixel(const sp_op* op, const float* x0, const float* y, int64_t batch, int64_t y_div,
                  float* x_eff, float* atr, float* rsq_partial, sp_stream_t stream);
/* out[0] = sum of count partials (one workgroup, fixed order; a device scalar). */
int sp_sum_partials(const float* partials, int64_t count, float* out, sp_stream_t stream);
/* out = alpha*a + beta/sqrt(*norm_sq)*b  (a may be NULL; norm_sq NULL means 1; a zero norm
 * gives 0, as torch's norm backward).  Gluing-term cotangents of psld.py:138-141. */
int sp_scaled_combine(const float* a, float alpha, const float* b, float beta, const float* norm_sq,
                      int64_t count, float* out, sp_stream_t stream);
/* c_x0 = -omega * atr / sqrt(*norm_sq) + (I - A^T A) u   (ata_u = A^T A u, BLUR only). */
int sp_psld_cotangent(const sp_op* op, const float* atr, const float* u, const float* ata_u,
                      const float* norm_sq, float omega, int64_t batch, float* out,
                      sp_stream_t stream);
/* epsilon-form DDIM step: x_prev = sqrt_a_prev*x0 + dir*eps + sigma*xi, x0 and pseudo-x0;
 * any output may be NULL; xi NULL = Philox(seed, step, sample_offset+b). */
int sp_ddim_eps_step(const float* x, const float* eps, int64_t batch, int64_t n,
                     const sp_eps_coefs* c, const float* xi, uint64_t seed, int64_t step,
                     int64_t sample_offset, float* x_prev, float* x0, float* pseudo_x0,
                     sp_stream_t stream);
/* ReSample stochastic resample (resample_kernels.py:96-107), a_t / sigma scalars. */
int sp_stochastic_resample(const float* pseudo_x0, const float* x_t, int64_t batch, int64_t n,
                           float a_t, float sigma, const float* xi, uint64_t seed, int64_t step,
                           int64_t sample_offset, float* out, sp_stream_t stream);
/* In-place AdamW update of `count` parameters. */
int sp_adamw_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                  int64_t count, const sp_adamw_coefs* c, sp_stream_t stream);
/* The same with a device-side stop flag: no-op once *stop != 0. */
int sp_adamw_step_until(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                        int64_t count, const sp_adamw_coefs* c, const int32_t* stop,
                        sp_stream_t stream);
/* One iteration of ReSample's pixel-space hard data consistency (resample_kernels.py:32-54:
 * AdamW(lr=1e-2) on MSELoss(y, A x)) for IDENTITY / INPAINT / MASK in one pass over x:
 *   r = y[b/y_div] - A x,  g = A^T(grad_scale * r)  (grad_scale = -2/M, M = elements of the
 *   MSE mean), AdamW update of x / exp_avg / exp_avg_sq in place, r^2 partials
 *   (sp_rsq_partials(op) per sample) of the loss at x before the update.
 * No-op once *stop != 0 (stop may be NULL).  BLUR: SP_EUNSUPPORTED (the caller composes
 * sp_op_apply / sp_residual_grad / sp_op_adjoint / sp_adamw_step_until). */
int sp_pixel_opt_step(const sp_op* op, float* x, float* exp_avg, float* exp_avg_sq,
                      const float* y, int64_t batch, int64_t y_div, float grad_scale,
                      const sp_adamw_coefs* c, const int32_t* stop, float* rsq_partial,
                      sp_stream_t stream);
/* Early-stop test of the optimisation loops (resample_kernels.py:50-51):
 *   loss = (sum of count partials, fixed order) / total;  *loss_out = loss (may be NULL);
 *   *stop = 1 if loss < threshold (compared in double).  Skipped once *stop != 0. */
int sp_opt_check(const float* partials, int64_t count, float total, double threshold,
                 int32_t* stop, float* loss_out, sp_stream_t stream);
/* The latent-space loop's rule (resample_kernels.py:75-91): as sp_opt_check, and from
 * iteration plateau_from (200 in the reference) on also *stop = 1 when the loss exceeds the
 * previous iteration's (*prev_loss, updated here).  itr is the 0-based iteration. */
int sp_opt_check_plateau(const float* partials, int64_t count, float total, double threshold,
                         int64_t itr, int64_t plateau_from, float* prev_loss, int32_t* stop,
                         float* loss_out, sp_stream_t stream);

/* ---- prior building blocks (SURVEY.md §8b "groupnorm_silu_fwd/bwd") -------------------
 * GroupNorm over NCHW x (n, channels, hw = H*W) with `groups` groups, eps, optional
 * per-(sample, channel) bias added to x first (chan_bias [n, channels] or NULL: the UNet's
 * time-embedding add), optional affine (gamma/beta [channels] or NULL) and, if act != 0,
 * SiLU on the output.  Replaces torch GroupNorm + SiLU inside diffusers' ResnetBlock2D /
 * Attention / conv_norm_out (called from ddpm.py:40-43 and stable_diffusion.py:330-345).
 * work: sp_groupnorm_workspace() floats.  mean/rstd [n*groups] are written by the
 * forward and read by the backward, which returns the input VJP dx (= the VJP w.r.t.
 * chan_bias after a sum over H*W). */
int64_t sp_groupnorm_workspace(int64_t n, int32_t channels, int64_t hw, int32_t groups);
int sp_groupnorm_silu_fwd(const float* x, const float* chan_bias, const float* gamma,
                          const float* beta, int64_t n, int32_t channels, int64_t hw,
                          int32_t groups, float eps, int32_t act, float* z, float* mean,
                          float* rstd, float* work, sp_stream_t stream);
int sp_groupnorm_silu_bwd(const float* dz, const float* x, const float* chan_bias,
                          const float* gamma, const float* beta, const float* mean,
                          const float* rstd, int64_t n, int32_t channels, int64_t hw,
                          int32_t groups, int32_t act, float* dx, float* work,
                          sp_stream_t stream);
/* The same over a channel concatenation x = cat(x1, x2) (x1: c1 channels, x2: the other
 * channels - c1; x2 NULL: one tensor), read in place — the up-path ResnetBlocks'
 * torch.cat([h, skip]) is never materialised.  The backward writes the input VJP into the
 * two parts (dx1, dx2) and adds the optional addends (add1, add2: e.g. the residual
 * branch's gradient; an addend may alias its output).
 * team (or NULL): the caller's region for the single-pass kernels' team words, team_bytes
 * >= sp_groupnorm_team_bytes(); zeroed once by the caller (e.g. at allocation), left zero by
 * every launch, and used by one stream at a time — then a call issues no memset.  NULL: the
 * words live in `work`, zeroed by a memset each call (what sp_groupnorm_silu_fwd / _bwd do).
 * The library allocates nothing. */
int sp_groupnorm_silu_fwd2(const float* x1, const float* x2, int32_t c1, const float* chan_bias,
                           const float* gamma, const float* beta, int64_t n, int32_t channels,
                           int64_t hw, int32_t groups, float eps, int32_t act, float* z,
                           float* mean, float* rstd, float* work, void* team, int64_t team_bytes,
                           sp_stream_t stream);
int sp_groupnorm_silu_bwd2(const float* dz, const float* x1, const float* x2, int32_t c1,
                           const float* chan_bias, const float* gamma, const float* beta,
                           const float* mean, const float* rstd, int64_t n, int32_t channels,
                           int64_t hw, int32_t groups, int32_t act, float* dx1, float* dx2,
                           const float* add1, const float* add2, const float* add1b,
                           float* work, void* team, int64_t team_bytes, sp_stream_t stream);

/* Single-pass GroupNorm (default on): a team of workgroups per group keeps the group in
 * registers across its reduction (forward reads x once, backward x and dz once).  enable:
 * 1 on, 0 off (the two-pass kernels), < 0 query; returns the previous setting.  Process-wide;
 * results are bit-identical either way.  A team member that has not published its chunk
 * partials within the poll bound (not resident: another process or stream holds CUs) has
 * them recomputed by the waiting workgroup from the chunk's inputs, in the member's own
 * order, so the result stays bit-identical.  team_timeouts: how many chunk partials were
 * recomputed that way (a cost, not an error).  set_spin_limit: the poll bound (< 0 default;
 * 0 recomputes every partial not present at the first poll — a test of that path). */
int sp_groupnorm_single_pass(int32_t enable);
int64_t sp_groupnorm_team_bytes(int64_t n, int32_t channels, int64_t hw, int32_t groups);
int64_t sp_groupnorm_team_timeouts(void);
int sp_groupnorm_set_spin_limit(int32_t spins);

/* ---- device-resident step schedule (hipGraph capture of a step) ----
 * One record per guided step, precomputed on the host in the same fp64->fp32 arithmetic
 * as the by-value calls; a device cursor selects the current record, so a captured step
 * (timestep write, UNet forward/VJP, both passes, cursor advance) replays unchanged. */
typedef struct sp_step_rec {
    sp_dps_coefs c;   /* this step's scalars                          */
    int64_t step;     /* Philox step index (the sampler's loop index) */
    int64_t t;        /* the prior's timestep                          */
} sp_step_rec;       /* 48 bytes */

/* *t_out = sched[*cursor].t (the prior's timestep tensor, int64) */
int sp_sched_timestep(const sp_step_rec* sched, const int32_t* cursor, int64_t* t_out,
                      sp_stream_t stream);
/* *cursor += 1 */
int sp_sched_advance(int32_t* cursor, sp_stream_t stream);
/* sp_dps_residual / sp_dps_update with the scalars (and the Philox step) read from
 * sched[*cursor] on the device. */
int sp_dps_residual_sched(const sp_op* op, const float* x, const float* eps, const float* y,
                          int64_t batch, int64_t y_div, const sp_step_rec* sched,
                          const int32_t* cursor, float* v_out, float* rsq_partial,
                          sp_stream_t stream);
int sp_dps_update_sched(const sp_op* op, const float* x, const float* eps, const float* y,
                        const float* v, const float* w, const float* rsq_partial,
                        uint64_t seed, int64_t sample_offset, int64_t batch, int64_t y_div,
                        const sp_step_rec* sched, const int32_t* cursor, float* x_out,
                        sp_stream_t stream);

/* 3x3 / stride 1 / pad 1 convolution on fp32 MFMA (SURVEY.md §8b "vae_conv3x3_fwd/bwd_input",
 * §8f f1): the ResnetBlock / mid / up-sampling convolutions of the SD VAE and DDPM UNet
 * (diffusers Conv2d(k=3, p=1), reached from stable_diffusion.py:330-345, ddpm.py:40-43).
 * Weights are packed once per layer (sp_conv3x3_pack; input_vjp=1 packs the transposed,
 * flipped weights of the input VJP); NCHW fp32 activations.  Shapes: see _supported. */
int sp_conv3x3_supported(int32_t cin, int32_t cout, int32_t height, int32_t width);
int64_t sp_conv3x3_packed_size(int32_t cin, int32_t cout);
int sp_conv3x3_pack(const float* w, int32_t cout, int32_t cin, int32_t input_vjp, float* wp,
                    sp_stream_t stream);
int sp_conv3x3_fwd(const float* x, const float* wp, const float* bias, int64_t n, int32_t cin,
                   int32_t cout, int32_t height, int32_t width, float* y, sp_stream_t stream);
int sp_conv3x3_bwd_input(const float* dy, const float* wp_vjp, int64_t n, int32_t cin,
                         int32_t cout, int32_t height, int32_t width, float* dx,
                         sp_stream_t stream);

/* 3x3 / stride 1 / pad 1 convolutions with few channels on one side (cout <= 8 or cin <= 8:
 * the priors' conv_in / conv_out) as VALU direct convolutions on the raw weights
 * [cout][cin][3][3]; the input VJP reads the same weights transposed and flipped. */
int sp_conv3x3_thin_supported(int32_t cin, int32_t cout, int32_t height, int32_t width);
int sp_conv3x3_thin_fwd(const float* x, const float* w, const float* bias, int64_t n,
                        int32_t cin, int32_t cout, int32_t height, int32_t width, float* y,
                        sp_stream_t stream);
int sp_conv3x3_thin_bwd_input(const float* dy, const float* w, int64_t n, int32_t cin,
                              int32_t cout, int32_t height, int32_t width, float* dx,
                              sp_stream_t stream);

/* 3x3 / stride 2 convolution with one zero row / column on the bottom / right (diffusers'
 * Downsample2D, downsample_padding=0: the UNet's and the VAE encoder's downsampling layers;
 * reached from ddpm.py:40-43 and stable_diffusion.py:338-345), on fp32 MFMA, NCHW.
 * height / width are the INPUT's (even); the output is height/2 x width/2.  Forward: cin % 4,
 * cout % 128, (height/2) % 8, (width/2) % 32; input VJP (input_vjp=1): cout % 4, cin % 128,
 * (height/2) % 2, (width/2) % 32 — each output phase (row & 1, column & 1) of dx is its own
 * sum over the taps that reach it.  Weights packed once per layer by sp_conv3x3_s2_pack
 * (cin * cout * 9 floats; layouts differ for the two directions).  FLOPs recorded for
 * kinds 3-4 (18*N*Cin*Cout*(H/2)*(W/2)). */
int sp_conv3x3_s2_supported(int32_t cin, int32_t cout, int32_t height, int32_t width,
                            int32_t input_vjp);
/* 2x nearest-neighbour upsampling (Upsample2D of the UNet and the VAE decoder, before its
 * 3x3 conv) over `planes` = N*C planes of height x width (width % 4, 16-B aligned buffers),
 * and its VJP, the 2x2 block sum of dy (2*height x 2*width) into dx (height x width). */
int sp_upsample2x_supported(int32_t height, int32_t width);
int sp_upsample2x(const float* x, int64_t planes, int32_t height, int32_t width, float* y,
                  sp_stream_t stream);
int sp_upsample2x_vjp(const float* dy, int64_t planes, int32_t height, int32_t width, float* dx,
                      sp_stream_t stream);
int sp_conv3x3_s2_pack(const float* w, int32_t cout, int32_t cin, int32_t input_vjp, float* wp,
                       sp_stream_t stream);
int sp_conv3x3_s2_fwd(const float* x, const float* wp, const float* bias, int64_t n, int32_t cin,
                      int32_t cout, int32_t height, int32_t width, float* y, sp_stream_t stream);
int sp_conv3x3_s2_bwd_input(const float* dy, const float* wp_vjp, int64_t n, int32_t cin,
                            int32_t cout, int32_t height, int32_t width, int32_t accumulate,
                            float* dx, sp_stream_t stream);
/* Split-K forms (a workspace; same results to fp32 rounding, bitwise reproducible): a launch
 * whose workgroups fill less than half the CUs (batch 1) runs 2-16 parts over K that store
 * partial sums to ws, then adds them in a fixed order (+ bias, or onto dx with accumulate).
 * sp_conv3x3_s2_workspace = the bytes a launch needs, 0 = not split (ws may be NULL). */
int64_t sp_conv3x3_s2_workspace(int64_t n, int32_t cin, int32_t cout, int32_t height, int32_t width,
                                int32_t input_vjp);
int sp_conv3x3_s2_fwd_ws(const float* x, const float* wp, const float* bias, int64_t n, int32_t cin,
                         int32_t cout, int32_t height, int32_t width, float* y, float* ws, int64_t ws_bytes,
                         sp_stream_t stream);
int sp_conv3x3_s2_bwd_input_ws(const float* dy, const float* wp_vjp, int64_t n, int32_t cin,
                               int32_t cout, int32_t height, int32_t width, int32_t accumulate,
                               float* dx, float* ws, int64_t ws_bytes, sp_stream_t stream);

/* The same layers by Winograd F(2x2,3x3) on fp32 MFMA (2.25x fewer multiplies; the
 * transforms add F(2,3) rounding, as MIOpen's Winograd solver does).  up = U = G g G^T
 * packed by sp_wino3x3_pack (input_vjp=1: of the transposed, flipped weights). */
int sp_wino3x3_supported(int32_t cin, int32_t cout, int32_t height, int32_t width);
int64_t sp_wino3x3_packed_size(int32_t cin, int32_t cout);
int sp_wino3x3_pack(const float* w, int32_t cout, int32_t cin, int32_t input_vjp, float* up,
                    sp_stream_t stream);
int sp_wino3x3_fwd(const float* x, const float* up, const float* bias, int64_t n, int32_t cin,
                   int32_t cout, int32_t height, int32_t width, float* y, sp_stream_t stream);
/* y = conv(x) + bias + res: the ResnetBlock's residual added in the tile's epilogue
 * (res shaped like y, not aliasing it). */
int sp_wino3x3_fwd_res(const float* x, const float* up, const float* bias, const float* res,
                       int64_t n, int32_t cin, int32_t cout, int32_t height, int32_t width,
                       float* y, sp_stream_t stream);
int sp_wino3x3_bwd_input(const float* dy, const float* up_vjp, int64_t n, int32_t cin,
                         int32_t cout, int32_t height, int32_t width, float* dx,
                         sp_stream_t stream);
/* Split-K forms (round 4): where the launch's tiles leave CUs idle (small batches, the
 * low-resolution levels) K is cut into up to 32 parts, each part's partial output stored to
 * the caller's workspace and the parts summed in a fixed order (+ bias, + res) by a reduce
 * launch — deterministic.  sp_wino3x3_workspace = the bytes a shape's split needs (0: the
 * shape fills the chip unsplit); a smaller (or NULL) workspace runs unsplit.  res nullable. */
int64_t sp_wino3x3_workspace(int64_t n, int32_t cin, int32_t cout, int32_t height, int32_t width);
int sp_wino3x3_fwd_ws(const float* x, const float* up, const float* bias, const float* res,
                      int64_t n, int32_t cin, int32_t cout, int32_t height, int32_t width,
                      float* y, float* ws, int64_t ws_bytes, sp_stream_t stream);
int sp_wino3x3_bwd_input_ws(const float* dy, const float* up_vjp, int64_t n, int32_t cin,
                            int32_t cout, int32_t height, int32_t width, float* dx, float* ws,
                            int64_t ws_bytes, sp_stream_t stream);
/* Round 5: diffusers' Upsample2D (nearest 2x upsample, then this conv) fused into the tile, so
 * the upsampled tensor is never written (reference call sites: the UNet / VAE up blocks behind
 * ddpm.py:40-43 and stable_diffusion.py:330-336).  height x width = the conv's (upsampled) size.
 * sp_wino3x3_fwd_up: x is the [n][cin][height/2][width/2] source, y the [n][cout][height][width]
 * conv output (+ bias).  sp_wino3x3_bwd_input_pool: the input VJP of conv(upsample(x)), dy
 * [n][cout][height][width] -> dx [n][cin][height/2][width/2] (each 2x2 block's sum in
 * sp_upsample2x_vjp's order: bitwise the unfused pair's result when that runs unsplit).
 * Unsplit (no workspace); sp_wino3x3_up_supported says where both directions run. */
int sp_wino3x3_up_supported(int32_t cin, int32_t cout, int32_t height, int32_t width);
int sp_wino3x3_fwd_up(const float* x, const float* up, const float* bias, int64_t n, int32_t cin,
                      int32_t cout, int32_t height, int32_t width, float* y, sp_stream_t stream);
int sp_wino3x3_bwd_input_pool(const float* dy, const float* up_vjp, int64_t n, int32_t cin,
                              int32_t cout, int32_t height, int32_t width, float* dx,
                              sp_stream_t stream);

/* 1x1 convolution as a per-pixel GEMM on bf16 MFMAs over exact three-term splits of the fp32
 * operands (fp32-class error): Y[n][co][p] = sum_k W[co][k] X[n][k][p] (+ bias[co]) (+ res),
 * X = cat(x1 [n][c1][hw], x2 [n][c2][hw]) read in place, Y split into y1 [n][o1][hw] and
 * y2 [n][o2][hw] (o2 may be 0).  Replaces diffusers ResnetBlock2D.conv_shortcut over the
 * up path's concatenation (forward) and its input VJP (W^T dy into both parts), SURVEY.md §8f
 * f1.  M = o1 + o2 % 128, K = c1 + c2 % 16, c1 % 8, c2 % 8, o1 % 32, o2 % 32, hw % 256;
 * res only with o2 == 0.  W packed by sp_gemm_x6_pack from a row-major [M][K] matrix, or
 * (trans = 1) from one stored [K][M]. */
int sp_gemm_x6_supported(int32_t m, int32_t k, int64_t hw);
int64_t sp_gemm_x6_packed_size(int32_t m, int32_t k);
int sp_gemm_x6_pack(const float* w, int32_t m, int32_t k, int32_t trans, float* wp, sp_stream_t stream);
int sp_gemm_x6(const float* x1, int32_t c1, const float* x2, int32_t c2, const float* wp,
               const float* bias, const float* res, int64_t n, int64_t hw, float* y1, int32_t o1,
               float* y2, int32_t o2, sp_stream_t stream);

/* nn.Linear on token-major activations with the same bf16x6 arithmetic:
 * y[t][o] = sum_k x[t][k] W[o][k] (+ bias[o]) (+ res[t][o]), tokens % 256, k % 16, m % 32
 * (W's rows padded to 128 with zeros by sp_gemm_x6_pack; pack W^T with trans = 1 for the
 * input VJP).  Replaces torch.nn.functional.linear in the ε-UNets' attention / transformer
 * blocks (diffusers Attention to_q/k/v/out, FeedForward), SURVEY.md §8f f1. */
int sp_linear_x6_supported(int64_t tokens, int32_t k, int32_t m);
int sp_linear_x6(const float* x, const float* wp, const float* bias, const float* res, int64_t tokens,
                 int32_t k, int32_t m, float* y, sp_stream_t stream);

/* The same GEMM between the two activation layouts of the transformer blocks' 1x1 proj_in /
 * proj_out (diffusers Transformer2DModel): x [n][k][hw] (in_tm = 0) or [n hw][k] (in_tm = 1),
 * y and res [n][m][hw] (out_tm = 0) or [n hw][m] (out_tm = 1); the NCHW <-> token transposes
 * happen in the tile's loads and stores.  hw % 256, k % 16, m % 32. */
int sp_gemm_x6_layout_supported(int64_t n, int64_t hw, int32_t k, int32_t m);
int sp_gemm_x6_layout(const float* x, const float* wp, const float* bias, const float* res, int64_t n,
                      int64_t hw, int32_t k, int32_t m, int32_t in_tm, int32_t out_tm, float* y,
                      sp_stream_t stream);

/* Split-K forms of the three (same arguments, plus a workspace): a launch whose tiles fill
 * less than half the CUs (batch 1, the 16² / 8² levels) runs 2-16 K parts that store their
 * partial products to ws, then adds them in a fixed order with the bias and the residual
 * (bitwise reproducible).  sp_gemm_x6_workspace(n, hw, k, m) = the bytes a launch over n
 * images of hw pixels (sp_linear_x6: n = 1, hw = tokens), K = k, M = m needs; 0 = not split
 * (ws may be NULL; a NULL or short ws runs unsplit). */
int64_t sp_gemm_x6_workspace(int64_t n, int64_t hw, int32_t k, int32_t m);
int sp_gemm_x6_ws(const float* x1, int32_t c1, const float* x2, int32_t c2, const float* wp,
                  const float* bias, const float* res, int64_t n, int64_t hw, float* y1, int32_t o1,
                  float* y2, int32_t o2, float* ws, int64_t ws_bytes, sp_stream_t stream);
int sp_linear_x6_ws(const float* x, const float* wp, const float* bias, const float* res, int64_t tokens,
                    int32_t k, int32_t m, float* y, float* ws, int64_t ws_bytes, sp_stream_t stream);
int sp_gemm_x6_layout_ws(const float* x, const float* wp, const float* bias, const float* res, int64_t n,
                         int64_t hw, int32_t k, int32_t m, int32_t in_tm, int32_t out_tm, float* y, float* ws,
                         int64_t ws_bytes, sp_stream_t stream);

/* Fused self-attention softmax(q k^T * scale) v of the SD 1.5 eps-UNet's transformer blocks
 * (attn1 over the latent tokens; diffusers UNet2DConditionModel, stable_diffusion.py:306-313;
 * replaces the scores / softmax / weighted-sum chain and its autograd VJP) on fp32 MFMA,
 * without materialising the score matrix.  q, k, v, out, dout, dq, dk, dv: [bh][n][d];
 * lse, delta: [bh][n] (lse = row log-sum-exp, natural log, written by the forward; delta =
 * rowsum(dout * out), written by the backward).  Self-attention only (m == n); head dims 40,
 * 80, 160; n a multiple of the kernels' row blocks (see _supported).  The backward writes dq
 * when dq != NULL and dk, dv when both are given. */
int sp_attention_supported(int64_t bh, int64_t n, int64_t m, int32_t d);
int sp_attention_fwd(const float* q, const float* k, const float* v, int64_t bh, int64_t n,
                     int32_t d, float scale, float* out, float* lse, sp_stream_t stream);
int sp_attention_bwd(const float* q, const float* k, const float* v, const float* out,
                     const float* dout, const float* lse, int64_t bh, int64_t n, int32_t d,
                     float scale, float* delta, float* dq, float* dk, float* dv,
                     sp_stream_t stream);
/* The same on the token-major activations of the projections, without head split / merge
 * copies, and cross-attention: row i of head h of sample b of q (and dq) starts at
 * (b n + i) rs + h d, of out (and dout) at (b n + i) ro + h d, of k, v (and dk, dv) at
 * (b' m + j) rs_kv + h d with b' = b (kv_batch = batch) or 0 (kv_batch = 1: one context
 * shared by the batch).  Self-attention: m = n, rs_kv = rs (rs = 3 heads d when q, k, v are
 * the thirds of one fused qkv projection [b n][3 heads d]).  Cross-attention (m != n, any
 * m >= 1, e.g. the 77-token text context of attn2): forward and dq only (dk = dv = NULL).
 * lse, delta: [b heads][n]. */
int sp_attention_mh_supported(int64_t batch, int32_t heads, int64_t n, int64_t m, int32_t d);
int sp_attention_fwd_mh(const float* q, const float* k, const float* v, int64_t batch, int32_t heads,
                        int64_t n, int64_t m, int32_t d, int32_t rs, int32_t rs_kv, int64_t kv_batch,
                        int32_t ro, float scale, float* out, float* lse, sp_stream_t stream);
int sp_attention_bwd_mh(const float* q, const float* k, const float* v, const float* out,
                        const float* dout, const float* lse, int64_t batch, int32_t heads, int64_t n,
                        int64_t m, int32_t d, int32_t rs, int32_t rs_kv, int64_t kv_batch, int32_t ro,
                        float scale, float* delta, float* dq, float* dk, float* dv, sp_stream_t stream);
/* Self-attention forward on the bf16 MFMA datapath over exact three-term splits of the fp32
 * operands (six partial products per product, fp32 accumulation; error at or below the
 * exact-fp32 kernel's), head dims 40 / 80, n % 128 == 0; q / k / v rows of stride rs, out rows
 * of stride ro, lse as sp_attention_fwd_mh.  sp_attention_fwd / _fwd_mh route self-attention
 * at these shapes here while sp_attention_bf16x6 is on (default; 0: the exact-fp32 kernel,
 * < 0 query; returns the previous setting). */
int sp_attention6_supported(int64_t batch, int32_t heads, int64_t n, int32_t d);
int sp_attention6_fwd_mh(const float* q, const float* k, const float* v, int64_t batch, int32_t heads, int64_t n,
                         int32_t d, int32_t rs, int32_t ro, float scale, float* out, float* lse,
                         sp_stream_t stream);
/* ws (or NULL): sp_attention6_workspace() bytes, where K and V are split into their bf16 terms
 * once per head instead of once per 128-query workgroup. */
int64_t sp_attention6_workspace(int64_t batch, int32_t heads, int64_t n, int32_t d);
int sp_attention6_fwd_ws(const float* q, const float* k, const float* v, int64_t batch, int32_t heads, int64_t n,
                         int32_t d, int32_t rs, int32_t ro, float scale, float* out, float* lse, void* ws,
                         int64_t ws_bytes, sp_stream_t stream);
int sp_attention_bf16x6(int32_t enable);
int sp_attention_bf16x6_enabled(void);

/* Transformer-block glue of the SD 1.5 eps-UNet (diffusers BasicTransformerBlock,
 * stable_diffusion.py:306-313): torch.nn.LayerNorm over the C channels of token-major rows
 * [rows][C] (C % 4, C <= 2048; mean / rstd [rows] written for the VJP) and its input VJP
 * (frozen weights; add != NULL is summed into dx: the residual branch's gradient of the same
 * tensor), and the feed-forward's GEGLU gate y = a * gelu(gate) over h = [a | gate]
 * ([rows][2F] -> [rows][F], exact erf GELU, F % 4) and its input VJP dh. */
int sp_layernorm_supported(int64_t rows, int32_t c);
int sp_layernorm_fwd(const float* x, const float* w, const float* b, int64_t rows, int32_t c, float eps,
                     float* y, float* mean, float* rstd, sp_stream_t stream);
int sp_layernorm_bwd(const float* dy, const float* x, const float* w, const float* mean, const float* rstd,
                     const float* add, int64_t rows, int32_t c, float* dx, sp_stream_t stream);
int sp_geglu_fwd(const float* h, int64_t rows, int32_t f, float* y, sp_stream_t stream);
int sp_geglu_bwd(const float* h, const float* dy, int64_t rows, int32_t f, float* dh, sp_stream_t stream);

/* Row softmax of materialised attention scores [rows][n] in place (n % 4, n <= 4096; lse
 * [rows] = row log-sum-exp when non-NULL) and its VJP scaled by the score scale,
 * dp <- scale * p * (dp - rowsum(p * dp)): the single-head d = 512 attention of the SD VAE
 * mid blocks and the DDPM UNet (diffusers Attention, ddpm.py:40-43 / stable_diffusion.py:
 * 330-345), whose score GEMMs are hipBLASLt's. */
int sp_softmax_rows_supported(int64_t rows, int32_t n);
int sp_softmax_rows(float* s, int64_t rows, int32_t n, float* lse, sp_stream_t stream);
int sp_softmax_bwd_rows(const float* p, float* dp, int64_t rows, int32_t n, float scale, sp_stream_t stream);

/* 1x1 convolution over 4 or 8 channels (the SD VAE's quant_conv / post_quant_conv):
 * y[n][o][p] = sum_c w[o][c] x[n][c][p] (+ b[o]); trans = 1 applies W^T (input VJP, b NULL).
 * hw % 4. */
int sp_conv1x1_small_supported(int32_t cin, int32_t cout, int64_t hw);
int sp_conv1x1_small(const float* x, const float* w, const float* b, int64_t n, int32_t cin, int32_t cout,
                     int64_t hw, int32_t trans, float* y, sp_stream_t stream);

/* ---- The priors at reduced precision (bf16), NHWC activations (csrc/sp_bf16.hip) ----------
 * The reference's adapters take any torch_dtype and its PSLD driver runs SD 1.5 in bf16
 * (reference: samplers/networks/diffusers/stable_diffusion.py:90-101, ddpm.py:23-34,
 * scripts/run_psld.py:14-20).  These entry points are the bf16 layers of those priors:
 * activations channels-last ([n][h][w][c]) bf16, bf16 MFMA operands, fp32 accumulation and
 * fp32 statistics.  Device pointers; bf16 buffers are passed as void*. */
int sp_conv3x3_bf16_supported(int32_t cin, int32_t cout, int32_t h, int32_t w);
/* bf16 elements of the packed weights: [ceil(cout/64)][cin/16][9 taps][64 co][16 ci] */
int64_t sp_conv3x3_bf16_packed_size(int32_t cin, int32_t cout);
/* y = conv3x3(x) + bias (+ res): stride 1, padding 1 (diffusers' ResnetBlock2D / conv_in /
 * conv_out / Upsample2D convolutions); the input VJP is the same call with the pack of
 * W'[ci][co][2-ky][2-kx].  bias fp32 [cout] or NULL, res bf16 like y or NULL. */
int sp_conv3x3_bf16(const void* x, const void* wp, const float* bias, const void* res, int64_t n, int32_t cin,
                    int32_t cout, int32_t h, int32_t w, void* y, sp_stream_t stream);
/* split-K form for launches that leave CUs idle (the priors' 16x16 / 8x8 levels): the parts' fp32
 * sums in ws (sp_conv3x3_bf16_workspace bytes, 0 = unsplit), reduced in a fixed order */
int64_t sp_conv3x3_bf16_workspace(int64_t n, int32_t cin, int32_t cout, int32_t h, int32_t w);
int sp_conv3x3_bf16_ws(const void* x, const void* wp, const float* bias, const void* res, int64_t n, int32_t cin,
                       int32_t cout, int32_t h, int32_t w, void* y, void* ws, int64_t ws_bytes, sp_stream_t stream);
/* y = conv3x3(upsample_nearest2x(x)) + bias (+ res) (diffusers' Upsample2D): x [n][h/2][w/2][cin],
 * y [n][h][w][cout] — the upsampled tensor is never written; its VJP is sp_conv3x3_bf16 with the
 * VJP pack at full resolution followed by sp_pool2x2_bf16. */
int sp_conv3x3_bf16_up(const void* x, const void* wp, const float* bias, const void* res, int64_t n, int32_t cin,
                       int32_t cout, int32_t h, int32_t w, void* y, sp_stream_t stream);
/* dx[n][h/2][w/2][c] = 2x2 block sums of dz[n][h][w][c], NHWC bf16 (c % 8 == 0) */
int sp_pool2x2_bf16(const void* dz, int64_t n, int32_t c, int32_t h, int32_t w, void* dx, sp_stream_t stream);
/* LayerNorm over bf16 token rows [rows][c] (BasicTransformerBlock's norm1-3 at bf16), fp32 weight /
 * bias / statistics (mean, rstd per row, for the VJP); the VJP (frozen weights) adds `add` (bf16,
 * nullable: the residual branch's gradient of the same tensor).  c % 8 == 0, c <= 2048. */
int sp_layernorm_bf16_supported(int64_t rows, int32_t c);
int sp_layernorm_bf16_fwd(const void* x, const float* w, const float* b, int64_t rows, int32_t c, float eps, void* y,
                          float* mean, float* rstd, sp_stream_t stream);
int sp_layernorm_bf16_bwd(const void* dy, const void* x, const float* w, const float* mean, const float* rstd,
                          const void* add, int64_t rows, int32_t c, void* dx, sp_stream_t stream);
/* GEGLU at bf16 (diffusers GEGLU after its projection, the SD 1.5 transformers' feed-forward,
 * reached from stable_diffusion.py:306-313): h = [a | gate] [rows][2f] -> y = a * gelu(gate)
 * [rows][f] (exact erf GELU, fp32 arithmetic); VJP dh = [dy gelu(gate) | dy a gelu'(gate)] as one
 * [rows][2f] buffer.  f % 8 == 0; bf16 throughout. */
int sp_geglu_bf16_fwd(const void* h, int64_t rows, int32_t f, void* y, sp_stream_t stream);
int sp_geglu_bf16_bwd(const void* h, const void* dy, int64_t rows, int32_t f, void* dh, sp_stream_t stream);
int sp_groupnorm_bf16_supported(int32_t c1, int32_t c2, int32_t groups);
int64_t sp_groupnorm_bf16_workspace(int64_t n, int32_t c, int64_t hw);
/* z = act(GroupNorm(cat(x1, x2) + chan_bias) * gamma + beta) over NHWC bf16 parts (channel
 * concatenation read in place); stats = [mean | rstd] per (n, group), fp32. */
int sp_groupnorm_bf16_fwd(const void* x1, const void* x2, int32_t c1, int32_t c2, const float* chan_bias,
                          const float* gamma, const float* beta, int64_t n, int64_t hw, int32_t groups, float eps,
                          int32_t act, void* z, float* stats, void* ws, int64_t ws_bytes, sp_stream_t stream);
/* its input VJP into the parts' layouts (+ addends; outputs may alias them) */
int sp_groupnorm_bf16_bwd(const void* dz, const void* x1, const void* x2, int32_t c1, int32_t c2,
                          const float* chan_bias, const float* gamma, const float* beta, const float* stats,
                          int64_t n, int64_t hw, int32_t groups, int32_t act, void* dx1, void* dx2, const void* add1,
                          const void* add2, const void* add1b, void* ws, int64_t ws_bytes, sp_stream_t stream);
/* The same with a chosen layout for z (z_layout 1: channel-blocked [n][c/16][hw][16], c % 16 == 0:
 * the conv tile's preferred input, sp_conv3x3_bf16_ex) / for dx1 (dx_layout 1: one part, c1 % 16 == 0;
 * the addends stay NHWC; dx_layout 2: dx1 / dx2 NHWC, add1 one addend over the concatenated channels
 * [n][hw][c1 + c2] and add2 NULL — a 1x1 shortcut's input gradient from one GEMM). */
int sp_groupnorm_bf16_fwd_ex(const void* x1, const void* x2, int32_t c1, int32_t c2, const float* chan_bias,
                             const float* gamma, const float* beta, int64_t n, int64_t hw, int32_t groups, float eps,
                             int32_t act, void* z, int32_t z_layout, float* stats, void* ws, int64_t ws_bytes,
                             sp_stream_t stream);
int sp_groupnorm_bf16_bwd_ex(const void* dz, const void* x1, const void* x2, int32_t c1, int32_t c2,
                             const float* chan_bias, const float* gamma, const float* beta, const float* stats,
                             int64_t n, int64_t hw, int32_t groups, int32_t act, void* dx1, void* dx2, int32_t dx_layout,
                             const void* add1, const void* add2, const void* add1b, void* ws, int64_t ws_bytes,
                             sp_stream_t stream);
/* sp_conv3x3_bf16_ws with the input in a chosen layout (in_layout 0 NHWC, 1 channel-blocked
 * [n][cin/16][h][w][16]: every 16-channel stage reads whole cache lines); in_layout 1 needs
 * sp_conv3x3_bf16_blk_supported (w % 32 == 0, h % 16 == 0).  The output stays NHWC. */
int sp_conv3x3_bf16_blk_supported(int32_t cin, int32_t cout, int32_t h, int32_t w);
int sp_conv3x3_bf16_ex(const void* x, int32_t in_layout, const void* wp, const float* bias, const void* res, int64_t n,
                       int32_t cin, int32_t cout, int32_t h, int32_t w, void* y, void* ws, int64_t ws_bytes,
                       sp_stream_t stream);
/* y = conv3x3(x) + conv1x1(cat(xs1, xs2)) + bias: a ResnetBlock's conv2 with its conv_shortcut
 * summed as (cs1 + cs2) / 16 further stages of the same contraction (no shortcut tensor, no
 * residual read).  wsp: [ceil(cout/64)][cs/16][64 co][16 ci] bf16 (rows past cout zero,
 * sp_conv3x3_bf16_sc_packed_size elements); bias: conv2's + the shortcut's; x in in_layout as
 * sp_conv3x3_bf16_ex; xs1 / xs2 NHWC.  Replaces the shortcut GEMM + residual epilogue of
 * diffusers' ResnetBlock2D (reference: samplers/networks/diffusers/ddpm.py:40-43 prior call). */
int sp_conv3x3_bf16_sc_supported(int32_t cin, int32_t cout, int32_t cs1, int32_t cs2, int32_t h, int32_t w);
int64_t sp_conv3x3_bf16_sc_packed_size(int32_t cs, int32_t cout);
int64_t sp_conv3x3_bf16_sc_workspace(int64_t n, int32_t cin, int32_t cs, int32_t cout, int32_t h, int32_t w);
int sp_conv3x3_bf16_sc(const void* x, int32_t in_layout, const void* wp, const float* bias, const void* xs1,
                       const void* xs2, int32_t cs1, int32_t cs2, const void* wsp, int64_t n, int32_t cin,
                       int32_t cout, int32_t h, int32_t w, void* y, void* ws, int64_t ws_bytes, sp_stream_t stream);
/* dz = the 3x3 conv input VJP of dy (flipped / transposed pack wp; dy in in_layout as
 * sp_conv3x3_bf16_ex), then dx1 / dx2 = the input VJP of sp_groupnorm_bf16_fwd over cat(x1, x2)
 * (c1 + c2 = cout) at dz (+ add1 / add2 / add1b; dx_layout as sp_groupnorm_bf16_bwd_ex): the
 * ResnetBlock VJP's conv2^T -> GN2^T and conv1^T -> GN1^T pairs, with the GroupNorm VJP's sums
 * taken in the conv's epilogue per 512-pixel tile (no pass re-reading dz and x).  dz: caller
 * buffer [n][h][w][cout]; ws: sp_conv3x3_bf16_gnvjp_workspace bytes.  TC = 32 unsplit shapes. */
int sp_conv3x3_bf16_gnvjp_supported(int64_t n, int32_t cin, int32_t cout, int32_t h, int32_t w, int32_t c1,
                                    int32_t groups);
int64_t sp_conv3x3_bf16_gnvjp_workspace(int64_t n, int32_t cout, int32_t h, int32_t w);
int sp_conv3x3_bf16_gnvjp(const void* dy, int32_t in_layout, const void* wp, int64_t n, int32_t cin, int32_t cout,
                          int32_t h, int32_t w, void* dz, const void* x1, const void* x2, int32_t c1,
                          const float* chan_bias, const float* gamma, const float* beta, const float* stats,
                          int32_t groups, int32_t act, void* dx1, void* dx2, int32_t dx_layout, const void* add1,
                          const void* add2, const void* add1b, void* ws, int64_t ws_bytes, sp_stream_t stream);
/* y = conv3x3(x) + bias (+ res) (as sp_conv3x3_bf16_ex), then z = act(GroupNorm(y + chan_bias))
 * (as sp_groupnorm_bf16_fwd_ex: gamma / beta, z_layout, stats [mean | rstd]) — the ResnetBlock's
 * conv1 -> GN2 pair, with the GroupNorm moments taken in the conv's epilogue per 512-pixel tile
 * (shifted by the tile's first pixel; no statistics pass re-reading y).  ws:
 * sp_conv3x3_bf16_gn_workspace bytes.  TC = 32 unsplit shapes. */
int sp_conv3x3_bf16_gn_supported(int64_t n, int32_t cin, int32_t cout, int32_t h, int32_t w, int32_t groups);
int64_t sp_conv3x3_bf16_gn_workspace(int64_t n, int32_t cout, int32_t h, int32_t w);
int sp_conv3x3_bf16_gn(const void* x, int32_t in_layout, const void* wp, const float* bias, const void* res,
                       int64_t n, int32_t cin, int32_t cout, int32_t h, int32_t w, void* y, const float* chan_bias,
                       const float* gamma, const float* beta, int32_t groups, float eps, int32_t act, void* z,
                       int32_t z_layout, float* stats, void* ws, int64_t ws_bytes, sp_stream_t stream);
int sp_attention_bf16_supported(int64_t batch, int32_t heads, int64_t n, int64_t m, int32_t d);
/* multi-head softmax(q k^T scale) v on bf16 token rows (self: m = n; cross: kv_shared = 1 for
 * one context row for the whole batch); lse [batch heads][n] fp32 for the VJP. */
int sp_attention_bf16_fwd(const void* q, const void* k, const void* v, int64_t batch, int32_t heads, int64_t n,
                          int64_t m, int32_t d, int32_t rsq, int32_t rskv, int32_t kv_shared, int32_t ro, float scale,
                          void* out, float* lse, sp_stream_t stream);
/* its VJP on the bf16 MFMAs (P, dS never in HBM): delta = caller's [batch heads][n] fp32 scratch;
 * dq rows of stride rdq; dk / dv (self-attention only) rows of stride rdkv, or NULL. */
int sp_attention_bf16_bwd_supported(int64_t batch, int32_t heads, int64_t n, int64_t m, int32_t d);
int sp_attention_bf16_bwd(const void* q, const void* k, const void* v, const void* out, const void* dout,
                          const float* lse, int64_t batch, int32_t heads, int64_t n, int64_t m, int32_t d,
                          int32_t rsq, int32_t rskv, int32_t kv_shared, int32_t ro, int32_t rdq, int32_t rdkv,
                          float scale, float* delta, void* dq, void* dk, void* dv, sp_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SAMPLERS_HIP_H */

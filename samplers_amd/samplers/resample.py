"""ReSample: latent diffusion with hard data consistency
(mirrors ``/root/reference/samplers/samplers/resample.py:27-228`` and
``utils/resample_kernels.py``).

Same control flow as the reference (ε-form DDIM step, DPS-style conditioning
with scale ½ᾱ_t, time-travel blocks every ``time_travel_interval`` indices in
the later part of the trajectory, pixel-space or latent-space AdamW hard
consistency, stochastic resample, a final latent optimisation); the arithmetic
between the priors is HIP:

* ``sp_ddim_eps_step``       ε-form DDIM (x_prev, x0, pseudo-x0) + noise
* ``sp_residual_grad`` + ``sp_sum_partials``  y − A(x), ‖·‖² / MSE, ∂/∂(Ax)
* ``sp_op_apply`` / ``sp_op_adjoint``        A and Aᵀ
* ``sp_adamw_step``          fused torch.optim.AdamW update
* ``sp_pixel_opt_step`` + ``sp_opt_check``  one launch per pixel-space AdamW iteration
  and the early-stop test on the device (no host sync per iteration)
* ``sp_stochastic_resample`` the resample step

Losses and norms are batch-global (MSE mean / Frobenius norm over the whole
flat batch, as in the reference); with a process group they are
all-reduced (8 bytes) before use.  Both optimisers test their stopping rules on
the device (``sp_opt_check`` / ``sp_opt_check_plateau``) and the flag gates the
AdamW update, where the reference calls ``.item()`` per iteration
(``resample_kernels.py:50,81``).  Operators without a HIP descriptor take the
same loops with ``A`` and its VJP from torch autograd (``_GenericConsistency``).
"""

from __future__ import annotations

import math
from typing import Generic, TypeVar

import numpy as np
import torch
import torch.distributed as dist
from torch import Tensor

from samplers_amd import _hip
from samplers_amd.distributed import all_reduce_sum_
from samplers_amd.dtypes import Shape
from samplers_amd.inverse_problem import InverseProblem
from samplers_amd.networks.base import LatentEpsilonNetwork, host_alphas_cumprod, host_timesteps
from samplers_amd.noise import GaussianNoise
from samplers_amd.samplers.base import PosteriorSampler
from samplers_amd.samplers.dps import NoiseFn, draw_seed, initial_sample
from samplers_amd.samplers.utils.batch_view import BatchView
from samplers_amd.samplers.utils.bridge_kernels import eps_step_coefficients

Condition_co = TypeVar("Condition_co", covariant=True)

# Philox stream keys of the draw sites (the main DDIM step uses the loop index)
_TRAVEL, _RESAMPLE = 1 << 32, 2 << 32


def adamw_coefficients(step: int, lr: float, beta1: float = 0.9, beta2: float = 0.999,
                       eps: float = 1e-8, weight_decay: float = 1e-2) -> _hip.SpAdamWCoefs:
    """Scalars of torch.optim.AdamW's single-tensor step ``step`` (1-based), fp32-rounded."""
    f = np.float32
    bc1 = 1 - beta1**step
    bc2 = 1 - beta2**step
    return _hip.SpAdamWCoefs(float(f(1 - lr * weight_decay)), beta1, beta2, eps,
                             float(f(lr / bc1)), float(f(math.sqrt(bc2))))


class _Consistency:
    """Batch-global ``||y - A x||`` / MSE and their gradients w.r.t. x, on HIP."""

    def __init__(self, operator, y_rows: Tensor, y_div: int, group=None) -> None:
        self.lib = _hip.load_library()
        self.op = operator
        self.desc = operator.hip_descriptor()
        if self.desc is None:
            raise NotImplementedError(f"{type(operator).__name__} has no native (HIP) implementation")
        self.y = y_rows.to(torch.float32).contiguous()
        self.y_div = int(y_div)
        self.m, self.n = int(self.desc.m), int(self.desc.n)
        self.P = int(self.lib.sp_vec_partials(self.m))
        self.group = group

    def _reduce(self, part: Tensor, out: Tensor, stream: int) -> None:
        _hip.check(self.lib.sp_sum_partials(_hip.ptr(part), part.numel(), out.data_ptr(), stream),
                   "sp_sum_partials")
        all_reduce_sum_(out, self.group)

    def residual(self, x: Tensor, scale: float) -> tuple[Tensor, Tensor]:
        """(g_y = scale * (y - A x), sum of squares (device scalar, global))."""
        lib, b = self.lib, x.shape[0]
        stream = _hip.stream_of(x)
        xf = x.reshape(b, self.n).contiguous()
        ax = torch.empty(b, self.m, device=x.device)
        _hip.check(lib.sp_op_apply(self.desc, _hip.ptr(xf), _hip.ptr(ax), b, stream), "sp_op_apply")
        g = torch.empty_like(ax)
        part = torch.empty(b, self.P, device=x.device)
        _hip.check(lib.sp_residual_grad(_hip.ptr(self.y), _hip.ptr(ax), b, self.m, self.y_div,
                                        scale, _hip.ptr(g), _hip.ptr(part), stream),
                   "sp_residual_grad")
        ss = torch.empty(1, device=x.device)
        self._reduce(part, ss, stream)
        return g, ss

    def adjoint(self, g: Tensor, like: Tensor) -> Tensor:
        out = torch.empty(like.shape, device=like.device, dtype=torch.float32)
        _hip.check(self.lib.sp_op_adjoint(self.desc, _hip.ptr(g), _hip.ptr(out), g.shape[0],
                                          _hip.stream_of(g)), "sp_op_adjoint")
        return out

    def mse_grad(self, x: Tensor, total: int) -> tuple[Tensor, Tensor]:
        """(∂ MSE/∂x, MSE) with MSE = mean over all `total` observation elements."""
        g, ss = self.mse_grad_ss(x, total)
        return g, ss / total

    def mse_grad_ss(self, x: Tensor, total: int) -> tuple[Tensor, Tensor]:
        """(∂ MSE/∂x, global Σ r²)."""
        g, ss = self.residual(x, float(np.float32(-2.0 / total)))  # mse_loss backward: 2(y-Ax)/M
        return self.adjoint(g, x), ss

    def norm_grad(self, x: Tensor) -> Tensor:
        """∂ ||y - A x||_F / ∂x = -A^T r / ||r|| (0 at r = 0)."""
        g, ss = self.residual(x, 1.0)
        gs = torch.empty_like(g)
        _hip.check(self.lib.sp_scaled_combine(None, 0.0, _hip.ptr(g), -1.0, ss.data_ptr(), g.numel(),
                                              _hip.ptr(gs), _hip.stream_of(g)), "combine")
        return self.adjoint(gs, x)


class _GenericConsistency(_Consistency):
    """``_Consistency`` for operators without a HIP descriptor: ``A`` is the plugin's own
    ``apply`` and its Jacobian-transpose products come from torch autograd on the device
    (the reference's ``operator.apply`` inside ``MSELoss`` / ``linalg.norm``,
    ``resample_kernels.py:15-93``); sums, norms and their all-reduce are the same device
    scalars as on the HIP path."""

    def __init__(self, operator, y_rows: Tensor, y_div: int, group=None) -> None:
        self.lib = _hip.load_library()
        self.op = operator
        self.desc = None
        self.y_div = int(y_div)
        self.y = y_rows.to(torch.float32).reshape(-1, *operator.y_shape)
        self.m, self.n = int(math.prod(operator.y_shape)), int(math.prod(operator.x_shape))
        self.group = group

    def residual_vjp(self, x: Tensor, scale: float) -> tuple[Tensor, Tensor]:
        """(J_A(x)ᵀ(scale · r), Σ r² as a global device scalar) with r = y − A x."""
        b = x.shape[0]
        idx = torch.arange(b, device=x.device) // self.y_div
        y = self.y.index_select(0, idx)
        with torch.enable_grad():
            xr = x.detach().reshape(b, *self.op.x_shape).requires_grad_(True)
            r = y - self.op.apply(xr)
            (g,) = torch.autograd.grad(r, xr, grad_outputs=r.detach() * (-scale))
        ss = all_reduce_sum_(r.detach().float().square().sum().reshape(1), self.group)
        return g.reshape(x.shape).to(torch.float32).contiguous(), ss

    def mse_grad_ss(self, x: Tensor, total: int) -> tuple[Tensor, Tensor]:
        return self.residual_vjp(x, float(np.float32(-2.0 / total)))

    def norm_grad(self, x: Tensor) -> Tensor:
        """−J_Aᵀ r / ‖r‖ (0 at r = 0)."""
        g, ss = self.residual_vjp(x, 1.0)
        out = torch.empty_like(g)
        _hip.check(self.lib.sp_scaled_combine(None, 0.0, _hip.ptr(g), -1.0, ss.data_ptr(), g.numel(),
                                              _hip.ptr(out), _hip.stream_of(g)), "combine")
        return out


def _is_gaussian(noise) -> bool:
    """``isinstance(noise, GaussianNoise)`` (``resample.py:123``), also for a model derived
    from the reference's own ``GaussianNoise`` (duck-typed plugins)."""
    return isinstance(noise, GaussianNoise) or any(
        c.__name__ == "GaussianNoise" for c in type(noise).__mro__)


_NOT_RUN = -1.0  # loss-log entry of an iteration the stopping rule skipped (losses are >= 0)


def _loss_log(max_iters: int, device) -> Tensor:
    """Per-iteration losses of one hard-consistency solve, written by the device check
    (``loss_out``); a check after the stop writes nothing, so the entries left at ``_NOT_RUN``
    count the iterations the stopping rule skipped (a loss that genuinely went inf / NaN is
    still counted as run)."""
    return torch.full((max(max_iters, 1),), _NOT_RUN, device=device)


def _log_solve(owner, kind: str, losses: Tensor, trips: int, max_iters: int) -> None:
    """Queue one solve's record for ``owner.optimization_log`` (the sampler's; reset per
    ``__call__``; nothing when there is no owner).  No host sync here: the device loss log is
    kept and read once, at the end of the call (``_finish_log``)."""
    if owner is None:
        return
    owner.__dict__.setdefault("_pending_log", []).append((kind, losses, trips, max_iters))


def _finish_log(owner) -> None:
    """Turn the queued solves into ``optimization_log`` records: the iterations the reference's
    stopping rule ran (``resample_kernels.py:32-93``), the host loop's trips (``loop_trips``: a
    few more than ran, since the flag is read late — not host synchronisations), the final
    loss."""
    pending = owner.__dict__.pop("_pending_log", [])
    log = owner.__dict__.setdefault("optimization_log", [])
    for kind, losses, trips, max_iters in pending:
        done = losses[:max(trips, 0)].cpu()
        ran = int((done != _NOT_RUN).sum())
        last = float(done[ran - 1]) if ran else float("nan")
        log.append({"kind": kind, "iterations": ran, "loop_trips": trips, "max_iters": max_iters,
                    "stopped_early": ran < max_iters, "final_loss": last})


def make_consistency(operator, y_rows: Tensor, y_div: int, group=None) -> _Consistency:
    if getattr(operator, "hip_descriptor", lambda: None)() is None:
        return _GenericConsistency(operator, y_rows, y_div, group)
    return _Consistency(operator, y_rows, y_div, group)


class ReSampleSampler(PosteriorSampler, Generic[Condition_co]):
    """ReSample (Song et al., 2023) on the HIP path."""

    def __init__(self, network):
        super().__init__(network)
        if not isinstance(self._epsilon_network, LatentEpsilonNetwork):
            raise TypeError(
                f"{self.__class__.__name__} requires a latent diffusion model, but build_network "
                f"returned a non-latent network ({type(self._epsilon_network).__name__})."
            )

    # --- pieces ------------------------------------------------------------
    def _ddim_eps(self, z: Tensor, t: int, t_prev: int, eta: float, noise: Tensor | None,
                  seed: int, key: int, offset: int, *, want_x0: bool = False):
        """ε-form DDIM step (``bridge_kernels.py:82-115``) -> (z_prev, pseudo_x0[, x0])."""
        net, lib = self._network, _hip.load_library()
        c = eps_step_coefficients(host_alphas_cumprod(net), t, t_prev, eta)
        with torch.no_grad():
            e = net.predict_noise(z, t).contiguous()
        zp, pseudo = torch.empty_like(z), torch.empty_like(z)
        x0 = torch.empty_like(z) if want_x0 else None
        coefs = _hip.SpEpsCoefs(c["sqrt_oma"], c["oma"], c["sqrt_a"], c["sqrt_a_prev"], c["sigma"],
                                c["dir"])
        b = z.shape[0]
        _hip.check(lib.sp_ddim_eps_step(_hip.ptr(z.detach().contiguous()), _hip.ptr(e), b,
                                        z[0].numel(), coefs, _hip.ptr(noise), seed, key, offset,
                                        _hip.ptr(zp), _hip.ptr(x0), _hip.ptr(pseudo),
                                        _hip.stream_of(z)), "sp_ddim_eps_step")
        return zp, pseudo, c["sqrt_a"]

    def _dps_conditioning(self, z_next: Tensor, pseudo: Tensor, sqrt_a: float, a_t: float,
                          cons: _Consistency) -> Tensor:
        """``resample_kernels.py:15-29``: z_next - 0.5 a_t * ∇_z ||y - A D(pseudo)||."""
        net = self._network
        with torch.enable_grad():
            pr = pseudo.detach().requires_grad_(True)
            x = net.decode(pr, differentiable=True)
        gx = cons.norm_grad(x.detach())
        (gp,) = torch.autograd.grad(x, pr, grad_outputs=gx.reshape(x.shape))
        out = torch.empty_like(z_next)
        scale = float(np.float32(a_t) * np.float32(0.5))
        # d pseudo / d z = 1/sqrt(a_t) (eps is evaluated without grad, bridge_kernels.py:97-98)
        _hip.check(cons.lib.sp_scaled_combine(_hip.ptr(z_next), 1.0, _hip.ptr(gp.contiguous()),
                                              -scale / sqrt_a, None, out.numel(), _hip.ptr(out),
                                              _hip.stream_of(out)), "combine")
        return out

    def _pixel_optimization(self, x0: Tensor, cons: _Consistency, total: int, eps: float,
                            max_iters: int, check_every: int = 16) -> Tensor:
        """``resample_kernels.py:32-54``: AdamW(lr=1e-2) on x, MSE, stop below eps^2.

        On the device: one fused launch per iteration for the
        elementwise operators (``sp_pixel_opt_step``: residual, MSE gradient, AdamW update,
        loss partials), and the stopping test in ``sp_opt_check`` after the update, which
        sets a device flag that turns every later launch of the loop into a no-op.  The host
        reads the flag once per ``check_every`` iterations instead of ``.item()`` per
        iteration; the result is the reference's (the same iterations run)."""
        lib = cons.lib
        x = x0.detach().clone().contiguous()
        b = x.shape[0]
        m_, v_ = torch.zeros_like(x), torch.zeros_like(x)
        stop = torch.zeros(1, dtype=torch.int32, device=x.device)
        stream = _hip.stream_of(x)
        gs = float(np.float32(-2.0 / total))  # mse_loss backward w.r.t. A x: 2 (Ax - y) / M
        tot, thr = float(np.float32(total)), float(eps) ** 2
        generic = cons.desc is None
        fused = not generic and int(cons.desc.kind) != _hip.SP_OP_BLUR
        shared = dist.is_initialized() and dist.get_world_size(cons.group) > 1
        part = torch.empty(b, int(lib.sp_rsq_partials(cons.desc)), device=x.device) if fused else None
        ss = torch.empty(1, device=x.device)
        losses = _loss_log(max_iters, x.device)
        it = -1
        for it in range(max_iters):
            c = adamw_coefficients(it + 1, 1e-2)
            if fused:
                _hip.check(lib.sp_pixel_opt_step(cons.desc, _hip.ptr(x), _hip.ptr(m_), _hip.ptr(v_),
                                                 _hip.ptr(cons.y), b, cons.y_div, gs, c,
                                                 _hip.ptr(stop), _hip.ptr(part), stream),
                           "sp_pixel_opt_step")
                if shared:
                    cons._reduce(part, ss, stream)
                parts, count = (ss, 1) if shared else (part, part.numel())
            else:  # BLUR / generic: A, residual, A^T composed; the update skips once stopped
                if generic:
                    grad, ss = cons.residual_vjp(x, gs)
                else:
                    g, ss = cons.residual(x, gs)
                    grad = cons.adjoint(g, x)
                _hip.check(lib.sp_adamw_step_until(_hip.ptr(x), _hip.ptr(grad), _hip.ptr(m_),
                                                   _hip.ptr(v_), x.numel(), c, _hip.ptr(stop),
                                                   stream), "sp_adamw_step_until")
                parts, count = ss, 1
            _hip.check(lib.sp_opt_check(_hip.ptr(parts), count, tot, thr, _hip.ptr(stop),
                                        _hip.ptr(losses) + 4 * it, stream), "sp_opt_check")
            if (it + 1) % check_every == 0 and int(stop.item()):
                break
        _log_solve(self, "pixel", losses, it + 1, max_iters)
        return x

    def _latent_optimization(self, z0: Tensor, cons: _Consistency, total: int, eps: float,
                             max_iters: int, plateau_from: int = 200) -> Tensor:
        """``resample_kernels.py:57-93``: AdamW(lr=5e-3) on z through the decoder.

        The stopping rule (loss below eps², or, from iteration 200 on, a loss above the
        previous iteration's) is evaluated on the device (``sp_opt_check_plateau``) and gates
        the AdamW update (``sp_adamw_step_until``), so the iterate is the reference's
        whatever the host does.  The host reads the flag one iteration late through pinned
        memory: iteration i + 1 is already queued when it waits for iteration i's flag, so
        the GPU queue never drains (the reference's ``.item()`` per iteration stalls it), at
        the price of one decoder forward + VJP past the stop whose update is a no-op."""
        net, lib = self._network, cons.lib
        z = z0.detach().clone().contiguous()
        m_, v_ = torch.zeros_like(z), torch.zeros_like(z)
        stop = torch.zeros(1, dtype=torch.int32, device=z.device)
        prev = torch.zeros(1, dtype=torch.float32, device=z.device)
        flags = torch.zeros(2, dtype=torch.int32, pin_memory=True)
        events = [torch.cuda.Event(), torch.cuda.Event()]
        stream = _hip.stream_of(z)
        tot, thr = float(np.float32(total)), float(eps) ** 2
        losses = _loss_log(max_iters, z.device)
        itr = -1
        for itr in range(max_iters):
            with torch.enable_grad():
                zr = z.detach().requires_grad_(True)
                x = net.decode(zr, differentiable=True)
            gx, ss = cons.mse_grad_ss(x.detach(), total)
            (gz,) = torch.autograd.grad(x, zr, grad_outputs=gx.reshape(x.shape))
            del x, zr
            c = adamw_coefficients(itr + 1, 5e-3)
            _hip.check(lib.sp_adamw_step_until(_hip.ptr(z), _hip.ptr(gz.contiguous()), _hip.ptr(m_),
                                               _hip.ptr(v_), z.numel(), c, _hip.ptr(stop), stream),
                       "sp_adamw_step_until")
            _hip.check(lib.sp_opt_check_plateau(_hip.ptr(ss), 1, tot, thr, itr, plateau_from,
                                                _hip.ptr(prev), _hip.ptr(stop),
                                                _hip.ptr(losses) + 4 * itr, stream),
                       "sp_opt_check_plateau")
            slot = itr & 1
            flags[slot:slot + 1].copy_(stop, non_blocking=True)
            events[slot].record()
            if itr >= 1:
                events[slot ^ 1].synchronize()
                if int(flags[slot ^ 1]):
                    break
        _log_solve(self, "latent", losses, itr + 1, max_iters)
        return z

    def _resample(self, z_opt: Tensor, snapshot: Tensor, a_prev: float, sigma: float,
                  noise: Tensor | None, seed: int, key: int, offset: int) -> Tensor:
        out = torch.empty_like(z_opt)
        _hip.check(_hip.load_library().sp_stochastic_resample(
            _hip.ptr(z_opt.contiguous()), _hip.ptr(snapshot.contiguous()), z_opt.shape[0],
            z_opt[0].numel(), a_prev, sigma, _hip.ptr(noise), seed, key, offset, _hip.ptr(out),
            _hip.stream_of(out)), "sp_stochastic_resample")
        return out

    # --- driver --------------------------------------------------------------
    def __call__(
        self,
        inverse_problem: InverseProblem,
        *,
        num_sampling_steps: int = 100,
        num_reconstructions: int = 1,
        scale: float = 0.3,
        sigma_scale: float = 40.0,
        max_optimization_iters: int = 2000,
        eta: float = 1.0,
        inter_timesteps: int = 5,
        time_travel_interval: int = 10,
        stage_splits: int = 3,
        decode_output: bool = True,
        condition: Condition_co | None = None,
        rng: str = "philox",
        seed: int | None = None,
        noise_fn: NoiseFn | None = None,
        sample_offset: int = 0,
        group=None,
    ) -> Tensor:
        """Run ReSample; ``scale`` is accepted and unused, as in the reference
        (its DPS step size is ½ᾱ_t, ``resample.py:145-146``).  Afterwards
        ``optimization_log`` lists every hard-consistency solve of the call (pixel / latent,
        the AdamW iterations the stopping rules ran, the final loss)."""
        self.optimization_log = []
        self._pending_log = []
        x_shape: Shape = inverse_problem.operator.x_shape
        batch_shape: Shape = inverse_problem.batch_shape
        x_view = BatchView(batch_shape, num_reconstructions, x_shape)
        net: LatentEpsilonNetwork = self._network
        latent_shape: Shape = tuple(net.get_latent_shape(x_shape))
        z_view = BatchView(batch_shape, num_reconstructions, latent_shape)
        net.set_sampling_parameters(num_sampling_steps=num_sampling_steps,
                                    num_reconstructions=num_reconstructions,
                                    batch_size=x_view.batch_size)
        net.set_condition(condition)
        try:
            obs = inverse_problem.observation
            _hip.require_cuda(obs, "ReSampleSampler")
            y_rows = obs.reshape(max(x_view.batch_size, 1), -1).to(torch.float32)
            cons = make_consistency(inverse_problem.operator, y_rows, num_reconstructions, group)
            total = z_view.leading_size * cons.m  # MSELoss mean over the tiled observation
            if dist.is_initialized() and dist.get_world_size(group) > 1:
                t = torch.tensor([float(total)], device=obs.device, dtype=torch.float64)
                dist.all_reduce(t, group=group)
                total = int(t.item())
            if seed is None and noise_fn is None and rng == "philox":
                seed = draw_seed()
            seed = int(seed or 0)
            off = sample_offset

            def draw(kind: str, key: int, like: Tensor) -> Tensor | None:
                if noise_fn is not None:
                    return noise_fn(kind, key, tuple(like.shape)).to(device=like.device,
                                                                     dtype=torch.float32)
                if rng == "torch":
                    return torch.randn_like(like)
                return None  # Philox inside the kernel

            z = initial_sample(z_view.flat_shape, net.device, rng=rng, seed=seed,
                               sample_offset=off, noise_fn=noise_fn)
            eps = float(inverse_problem.noise.sigma.item()) if _is_gaussian(inverse_problem.noise) \
                else 1e-3
            ts = host_timesteps(net)
            acp = host_alphas_cumprod(net)
            total_steps = len(ts) - 1
            index_split = total_steps // stage_splits
            for idx in range(len(ts) - 1, 1, -1):
                t, tp = ts[idx], ts[idx - 1]
                z_next, pseudo, sqrt_a = self._ddim_eps(z, t, tp, eta, draw("step", idx, z), seed,
                                                        idx, off)
                a_t = float(np.float32(acp[t]))
                z = self._dps_conditioning(z_next, pseudo, sqrt_a, a_t, cons)
                if idx <= total_steps - index_split and idx > 0 and idx % time_travel_interval == 0:
                    snapshot = z.clone()
                    for kk in range(idx, max(idx - inter_timesteps, 1), -1):
                        if kk <= 1:
                            break
                        key = _TRAVEL | (idx << 16) | kk
                        z, pseudo, _ = self._ddim_eps(z, ts[kk], ts[kk - 1], eta,
                                                      draw("travel", key, z), seed, key, off)
                    a_prev = np.float32(acp[tp])
                    f = np.float32
                    sigma = float(f(sigma_scale) * (f(1) - a_prev) / (f(1) - f(a_t))
                                  * (f(1) - f(a_t) / a_prev))
                    if idx >= index_split:
                        x_pix = net.decode(pseudo, differentiable=False)
                        x_opt = self._pixel_optimization(x_pix, cons, total, eps,
                                                         max_optimization_iters)
                        z_opt = net.encode(x_opt.reshape(x_pix.shape), differentiable=False)
                    else:
                        z_opt = self._latent_optimization(pseudo, cons, total, eps,
                                                          max_optimization_iters)
                    key = _RESAMPLE | idx
                    z = self._resample(z_opt, snapshot, float(a_prev), sigma,
                                       draw("resample", key, z_opt), seed, key, off)
            final_z0 = self._latent_optimization(z, cons, total, eps, max_optimization_iters)
            _finish_log(self)
            if decode_output:
                return self._as_output(x_view.unflatten(net.decode(final_z0, differentiable=False)))
            return self._as_output(z_view.unflatten(final_z0))
        finally:
            net.clear_condition()
            net.clear_sampling_parameters()

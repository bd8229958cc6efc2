"""Diffusion Posterior Sampling on the MI355X hot path.

Same call contract as ``DPSSampler.__call__`` of the reference
(``/root/reference/samplers/samplers/dps.py:25-134``); the loop body
(``dps.py:91-122``) is rebuilt around two fused HIP passes with the prior's
input-VJP between them::

    eps = unet(x, t)                               the prior (its layers on this project's kernels)
    v, |r|^2 partials = sp_dps_residual(x, eps, y) HIP pass 1: x0, A x0, residual, A^T grad
    w = J_eps^T v                                  the prior's input VJP (PyTorch-ROCm autograd)
    x <- sp_dps_update(x, eps, y|v, w, noise)      HIP pass 2: bridge mean + std*xi + guidance

which is algebraically the reference's ``autograd.grad(log_likelihood(predict_x0(x)).sum(), x)``
followed by ``ddim_step`` and ``x += gamma / (||r_b|| + 1e-9) * grad``
(closed form: SURVEY.md §8a A9).  Timesteps and schedule scalars stay on the
host, so a step issues no device->host synchronisation.

Noise (``rng=``):
  * ``"philox"`` (default): standard normals drawn inside pass 2 by Philox4x32-10
    keyed by (seed, step, global sample index, element) — identical whatever the
    batch sharding or micro-batching;
  * ``"torch"``: the reference's draw order — ``torch.randn`` for x_T and one
    ``torch.randn_like`` per step on the sample's device;
  * ``noise_fn(kind, step, shape)``: injected tensors (parity tests replay the
    reference's captured noise).
"""

from __future__ import annotations

from typing import Callable, Generic, TypeVar

import numpy as np
import torch
from torch import Tensor

from samplers_amd import _hip
from samplers_amd.dtypes import Shape
from samplers_amd.inverse_problem import InverseProblem
from samplers_amd.networks.base import EpsilonNetwork, host_alphas_cumprod, host_timesteps
from samplers_amd.samplers.base import PosteriorSampler
from samplers_amd.samplers.utils.batch_view import BatchView
from samplers_amd.samplers.utils.bridge_kernels import bridge_coefficients, x0_coefficients

Condition_co = TypeVar("Condition_co", covariant=True)

NoiseFn = Callable[[str, int, tuple], Tensor]


def draw_seed() -> int:
    """A 63-bit seed from torch's default CPU generator (reproducible under manual_seed)."""
    return int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())


class KernelTimer:
    """Per-launch durations of the library's timed kernels.

    Uses the library's dispatch-packet events (``sp_timing_enable``: a start/stop
    hipEvent pair attached to each kernel's AQL packet via hipExtLaunchKernel),
    i.e. the kernel's own execution interval on its launch stream — the same
    interval rocprofv3's kernel trace reports — not a host-side bracket.  Each
    record carries the launch's algorithmic work (``sp_timing_collect_work``):
    samples for the two DPS passes, FLOPs for the fp32-MFMA convolution tile.
    """

    _KIND = {1: "dps_residual", 2: "dps_update", 3: "conv3x3_fwd", 4: "conv3x3_bwd_input",
             5: "wino3x3_fwd", 6: "wino3x3_bwd_input", 7: "conv3x3_bf16"}
    _CAP = 1 << 16

    def __init__(self) -> None:
        self.batches: list[tuple[str, int]] = []
        self._lib = _hip.load_library()
        self._lib.sp_timing_enable(1)

    def span(self, name: str, batch: int):
        timer = self

        class _Span:
            def __enter__(self):
                return self

            def __exit__(self, *exc):
                timer.batches.append((name, batch))
                return False

        return _Span()

    def summary(self) -> dict[str, dict[str, float]]:
        """{kind: {count, ms, work}} over the launches since the last call; ``samples`` is
        the DPS passes' work, ``flops`` the convolutions'."""
        import ctypes

        kinds = (ctypes.c_int32 * self._CAP)()
        ms = (ctypes.c_float * self._CAP)()
        work = (ctypes.c_double * self._CAP)()
        n = self._lib.sp_timing_collect_work(kinds, ms, work, self._CAP)
        out: dict[str, dict[str, float]] = {}
        for kind, t, w in zip(kinds[:n], ms[:n], work[:n]):
            name = self._KIND.get(kind, f"kind{kind}")
            d = out.setdefault(name, {"count": 0, "ms": 0.0, "work": 0.0})
            d["count"] += 1
            d["ms"] += float(t)
            d["work"] += float(w)
        for name, d in out.items():
            d["samples" if name.startswith("dps") else "flops"] = d["work"]
        self.batches.clear()
        return out

    def clear(self) -> None:
        self.summary()

    def close(self) -> None:
        self.clear()
        self._lib.sp_timing_enable(0)


class FusedDPSStep:
    """One guided DPS iteration (``dps.py:91-122``) over a flat batch, on HIP.

    ``observation_rows``: ``(num_rows, *y_shape)`` fp32 device tensor; sample b
    uses row ``b // y_div`` (``y_div`` = reconstructions per observation).
    """

    def __init__(self, network: EpsilonNetwork, inverse_problem: InverseProblem,
                 observation_rows: Tensor, y_div: int, *, gamma: float = 1.0, eta: float = 1.0,
                 micro_batch: int | None = None, timer: KernelTimer | None = None,
                 reuse_v: bool = False, mode: str = "dps", guidance_weight: float = 1.0) -> None:
        op = inverse_problem.operator
        desc = getattr(op, "hip_descriptor", lambda: None)()
        if desc is None:
            raise NotImplementedError(
                f"{type(op).__name__} has no native (HIP) implementation; the fused DPS path "
                "supports IdentityOperator, InpaintingOperator (and subclasses) and "
                "GaussianBlurOperator"
            )
        _hip.require_cuda(observation_rows, "DPSSampler")
        if observation_rows.dtype != torch.float32:
            raise TypeError("the HIP path computes in fp32; cast the observation to float32")
        self.lib = _hip.load_library()
        self.network = network
        self.operator = op
        self.desc = desc
        self.y = observation_rows.contiguous()
        self.y_div = int(y_div)
        self.m = int(desc.m)
        self.n = int(desc.n)
        self.partials = int(self.lib.sp_rsq_partials(desc))
        if self.partials <= 0:
            raise _hip.HipLibraryError(f"operator descriptor rejected ({self.partials})")
        if mode not in ("dps", "pgdm"):
            raise ValueError(mode)
        self.mode = mode
        # DPS: d log p/d(Ax) = c r.  PGDM: d/dx0 of ||A^+ y - A^+ A x0||^2 = -2 A^T r for the
        # partial isometries with a native kernel (A^+ = A^T: identity, inpainting, mask).
        self.grad_scale = -2.0
        if mode == "dps":
            gs = getattr(inverse_problem.noise, "grad_scale", None)
            if gs is None:
                from samplers_amd.noise import probe_grad_scale

                gs = lambda: probe_grad_scale(inverse_problem.noise)  # noqa: E731
            c = gs()
            if c is None:
                raise NotImplementedError(f"{type(inverse_problem.noise).__name__} has no constant "
                                          "likelihood-gradient factor; use GenericDPSStep")
            self.grad_scale = float(c)
        self.guidance_weight = float(guidance_weight)
        self.gamma, self.eta = float(gamma), float(eta)
        # pass 2 re-derives v from (x, eps, y) (default: SURVEY §8d's minimal bytes, 4n + m per
        # sample; with non-temporal loads and 2 float4 groups per thread it is 7 % faster than
        # re-reading pass 1's v, 42.3 vs 45.2 us at B = 64, 256^2) or re-reads v (reuse_v).
        # Blur always re-reads it (its adjoint needs a halo).
        self.needs_v = desc.kind == _hip.SP_OP_BLUR or bool(reuse_v)
        self.micro_batch = micro_batch
        self.timer = timer

    def coefficients(self, t: int, t_prev: int, s: int) -> _hip.SpDpsCoefs:
        acp = host_alphas_cumprod(self.network)
        a, k = x0_coefficients(acp, t)
        br = bridge_coefficients(acp, ell=t, t=t_prev, s=s, eta=self.eta)
        # PGDM: sample = ddim - guidance_weight * sqrt(1 - acp_t) * grad   (pgdm.py:131-135)
        gamma = self.gamma if self.mode == "dps" else float(np.float32(-self.guidance_weight) *
                                                                  np.float32(k))
        return _hip.SpDpsCoefs(a, k, self.grad_scale, br.c_ell, br.c_s, br.std, gamma, 1e-9)

    def _chunks(self, batch: int):
        mb = self.micro_batch or batch
        mb = max(self.y_div, (mb // self.y_div) * self.y_div)  # chunks never split an observation
        for b0 in range(0, batch, mb):
            yield b0, min(batch, b0 + mb)

    def __call__(self, x: Tensor, step: int, t: int, t_prev: int, s: int, *,
                 xi: Tensor | None = None, seed: int = 0, sample_offset: int = 0) -> Tensor:
        """Advance ``x`` (flat ``(B, *x_shape)``, contiguous fp32) one step, in place."""
        lib, desc = self.lib, self.desc
        coefs = self.coefficients(t, t_prev, s)
        stream = _hip.stream_of(x)
        batch = x.shape[0]
        for b0, b1 in self._chunks(batch):
            xc = x[b0:b1]
            bc = b1 - b0
            yc = self.y[b0 // self.y_div:]
            with torch.enable_grad():
                xr = xc.detach().requires_grad_(True)
                eps = self.network.forward(xr, t)
            eps_c = eps.detach()
            if not eps_c.is_contiguous():
                eps_c = eps_c.contiguous()
            v = torch.empty_like(xc)
            part = torch.empty((bc, self.partials), device=x.device, dtype=torch.float32)
            span = self.timer.span("dps_residual", bc) if self.timer else None
            if span:
                span.__enter__()
            _hip.check(lib.sp_dps_residual(desc, _hip.ptr(xc), _hip.ptr(eps_c), _hip.ptr(yc), bc,
                                           self.y_div, coefs, _hip.ptr(v), _hip.ptr(part), stream),
                       "sp_dps_residual")
            if span:
                span.__exit__(None, None, None)
            (w,) = torch.autograd.grad(eps, xr, grad_outputs=v.view_as(eps))
            del eps, xr
            w = w.contiguous()
            xic = None if xi is None else xi[b0:b1].contiguous()
            span = self.timer.span("dps_update", bc) if self.timer else None
            if span:
                span.__enter__()
            _hip.check(lib.sp_dps_update(desc, _hip.ptr(xc), _hip.ptr(eps_c), _hip.ptr(yc),
                                         _hip.ptr(v) if self.needs_v else None, _hip.ptr(w),
                                         _hip.ptr(part) if self.mode == "dps" else None,
                                         _hip.ptr(xic), seed, step,
                                         sample_offset + b0, bc, self.y_div, coefs, _hip.ptr(xc),
                                         stream),
                       "sp_dps_update")
            if span:
                span.__exit__(None, None, None)
        return x

    def predict_x0(self, x: Tensor, t: int) -> Tensor:
        """Final ``predict_x0`` (``dps.py:125-126``): prior forward + HIP epilogue."""
        a, k = x0_coefficients(host_alphas_cumprod(self.network), t)
        out = torch.empty_like(x)
        for b0, b1 in self._chunks(x.shape[0]):
            with torch.no_grad():
                eps = self.network.forward(x[b0:b1], t).contiguous()
            _hip.check(self.lib.sp_predict_x0(_hip.ptr(x[b0:b1]), _hip.ptr(eps), eps.numel(), a, k,
                                              _hip.ptr(out[b0:b1]), _hip.stream_of(x)),
                       "sp_predict_x0")
        return out


class GenericDPSStep(FusedDPSStep):
    """One DPS / PGDM iteration for plugins the HIP library does not know.

    The reference differentiates through *any* ``Operator`` and ``NoiseModel``
    (``dps.py:99-103``, ``pgdm.py:104-119``).  Here the residual cotangent
    ``v = ∂(objective)/∂x̂₀`` comes from torch autograd through the plugin's own
    ``apply`` (and ``log_prob`` / ``apply_pseudo_inverse``) on the device, and everything
    else stays on the HIP path: x̂₀ by ``sp_predict_x0``, the prior's input-VJP with
    ``grad_outputs = v``, and pass 2 (``sp_dps_update`` over an identity descriptor of
    the sample, v given) for the bridge mean, noise and guidance.  The per-sample
    ``‖r_b‖²`` enters pass 2 through its partial-sum slot (column 0, the rest zero, so
    the fixed-order sum is exact).
    """

    def __init__(self, network: EpsilonNetwork, inverse_problem: InverseProblem,
                 observation_rows: Tensor, y_div: int, *, gamma: float = 1.0, eta: float = 1.0,
                 micro_batch: int | None = None, timer: KernelTimer | None = None,
                 mode: str = "dps", guidance_weight: float = 1.0, **_unused) -> None:
        from samplers_amd.operators import IdentityOperator

        if mode not in ("dps", "pgdm"):
            raise ValueError(mode)
        _hip.require_cuda(observation_rows, "DPSSampler")
        self.lib = _hip.load_library()
        self.network = network
        self.problem = inverse_problem
        self.operator = inverse_problem.operator
        self.x_shape = tuple(self.operator.x_shape)
        self.desc = IdentityOperator(self.x_shape).hip_descriptor()
        self.n = self.m = int(self.desc.n)
        self.partials = int(self.lib.sp_rsq_partials(self.desc))
        self.y = observation_rows
        self.y_div = int(y_div)
        self.mode = mode
        self.grad_scale = 0.0  # unused: v comes from autograd
        self.guidance_weight = float(guidance_weight)
        self.gamma, self.eta = float(gamma), float(eta)
        self.needs_v = True
        self.micro_batch = micro_batch
        self.timer = timer
        self._pinv_y = None

    def _rows(self, b0: int, b1: int) -> Tensor:
        idx = torch.arange(b0, b1, device=self.y.device) // self.y_div
        return self.y.index_select(0, idx)

    def _cotangent(self, x0: Tensor, b0: int, b1: int) -> tuple[Tensor, Tensor | None]:
        """(v = ∂ objective / ∂x̂₀, ‖r_b‖² per sample or None) by autograd through the plugin."""
        op = self.operator
        y = self._rows(b0, b1)
        with torch.enable_grad():
            x0r = x0.detach().requires_grad_(True)
            if self.mode == "dps":  # inverse_problem.log_likelihood (inverse_problem.py:17-21)
                r = y - op.apply(x0r)
                obj = self.problem.noise.log_prob(r).sum()
            else:  # PGDM consistency loss (pgdm.py:110-115)
                y_inv = op.apply_pseudo_inverse(y)
                obj = (y_inv - op.apply_pseudo_inverse(op.forward(x0r))).pow(2).sum()
                r = None
            (v,) = torch.autograd.grad(obj, x0r)
        rsq = None
        if r is not None:
            rsq = r.detach().reshape(r.shape[0], -1).float().square().sum(dim=1)
        return v.to(torch.float32).contiguous(), rsq

    def __call__(self, x: Tensor, step: int, t: int, t_prev: int, s: int, *,
                 xi: Tensor | None = None, seed: int = 0, sample_offset: int = 0) -> Tensor:
        lib, desc = self.lib, self.desc
        coefs = self.coefficients(t, t_prev, s)
        stream = _hip.stream_of(x)
        for b0, b1 in self._chunks(x.shape[0]):
            xc = x[b0:b1]
            bc = b1 - b0
            with torch.enable_grad():
                xr = xc.detach().requires_grad_(True)
                eps = self.network.forward(xr, t)
            eps_c = eps.detach().contiguous()
            x0 = torch.empty_like(xc)
            _hip.check(lib.sp_predict_x0(_hip.ptr(xc), _hip.ptr(eps_c), xc.numel(), coefs.a,
                                         coefs.k, _hip.ptr(x0), stream), "sp_predict_x0")
            v, rsq = self._cotangent(x0, b0, b1)
            part = None
            if rsq is not None:
                part = torch.zeros((bc, self.partials), device=x.device, dtype=torch.float32)
                part[:, 0] = rsq
            (w,) = torch.autograd.grad(eps, xr, grad_outputs=v.view_as(eps))
            del eps, xr
            xic = None if xi is None else xi[b0:b1].contiguous()
            _hip.check(lib.sp_dps_update(desc, _hip.ptr(xc), _hip.ptr(eps_c), None, _hip.ptr(v),
                                         _hip.ptr(w.contiguous()), _hip.ptr(part), _hip.ptr(xic),
                                         seed, step, sample_offset + b0, bc, 1, coefs,
                                         _hip.ptr(xc), stream), "sp_dps_update")
        return x


def native_plugins(inverse_problem) -> bool:
    """True when the operator has a HIP descriptor and the noise a constant ∂log p/∂(Ax)
    factor, i.e. the fused passes can replace autograd entirely."""
    desc_fn = getattr(inverse_problem.operator, "hip_descriptor", None)
    if desc_fn is None or desc_fn() is None:
        return False
    gs = getattr(inverse_problem.noise, "grad_scale", None)
    if gs is None:
        from samplers_amd.noise import probe_grad_scale

        return probe_grad_scale(inverse_problem.noise) is not None
    return gs() is not None


def make_dps_step(network, inverse_problem, observation_rows, y_div, **kw):
    """The fused HIP step for native plugins, the generic-plugin step otherwise."""
    mode = kw.get("mode", "dps")
    native_op = getattr(inverse_problem.operator, "hip_descriptor", lambda: None)() is not None
    if (mode == "dps" and native_plugins(inverse_problem)) or (mode == "pgdm" and native_op):
        return FusedDPSStep(network, inverse_problem, observation_rows, y_div, **kw)
    return GenericDPSStep(network, inverse_problem, observation_rows, y_div, **kw)


# hipGraph replay by default where it pays: below GRAPH_AUTO_MAX_BATCH samples.
# Measured (profiles/round5/final/bench_call_b1.json): a whole 1000-step call at batch 1 runs
# 9.47 ms per step eager and 10.05 ms replayed — the captured step runs GroupNorm's two-pass
# kernels, and the eager step is no longer host-bound once no per-launch timing events are
# attached (bench.py's B = 1 eager figure, 11.4 ms, carries them); from batch 2 on the eager step
# wins by more (tools/graph_sweep.sh).  So the automatic choice is off (0); graph=True replays.
# Capture costs about three steps (two warm-up steps and the capture), so short solves stay eager.
GRAPH_AUTO_MAX_BATCH = 0
GRAPH_AUTO_MIN_STEPS = 8


def graph_auto(step, x: Tensor, guided_steps: int, *, rng: str, noise_fn, callback,
               micro_batch: int | None) -> bool:
    """Whether ``DPSSampler(graph=None)`` replays a captured step: the fused HIP step (native
    operator and noise plugins), in-kernel Philox noise, no callback / kernel timer /
    micro-batching, a flat batch of at most ``GRAPH_AUTO_MAX_BATCH`` and at least
    ``GRAPH_AUTO_MIN_STEPS`` guided iterations, and a prior that declares itself capturable
    (``graph_capturable``: this project's priors, whose layers run on HIP kernels and
    allocate nothing outside torch's caching allocator; a third-party network stays eager
    unless it sets the flag).  ``SAMPLERS_AMD_GRAPH=0`` turns the automatic choice off."""
    import os

    if os.environ.get("SAMPLERS_AMD_GRAPH", "auto").lower() in ("0", "off", "false", "eager"):
        return False
    return (getattr(step.network, "graph_capturable", False)
            and isinstance(step, FusedDPSStep) and not isinstance(step, GenericDPSStep)
            and step.timer is None and rng == "philox" and noise_fn is None and callback is None
            and (not micro_batch or micro_batch >= x.shape[0]) and x.is_cuda
            and 0 < x.shape[0] <= GRAPH_AUTO_MAX_BATCH and guided_steps >= GRAPH_AUTO_MIN_STEPS)


def initial_sample(shape: tuple, device: torch.device, *, rng: str, seed: int, sample_offset: int,
                   noise_fn: NoiseFn | None) -> Tensor:
    """x_T ~ N(0, I) (``dps.py:83-87``)."""
    if noise_fn is not None:
        return noise_fn("init", -1, shape).to(device=device, dtype=torch.float32).contiguous()
    if rng == "torch":
        return torch.randn(size=shape, device=device, dtype=torch.float32)
    if rng != "philox":
        raise ValueError(f"rng must be 'philox' or 'torch', got {rng!r}")
    lib = _hip.load_library()
    x = torch.empty(shape, device=device, dtype=torch.float32)
    n = x[0].numel() if shape[0] else 0
    if shape[0]:
        _hip.check(lib.sp_randn(_hip.ptr(x), shape[0], n, seed, -1, sample_offset,
                                _hip.stream_of(x)), "sp_randn")
    return x


class DPSSampler(PosteriorSampler, Generic[Condition_co]):
    """DPS (Chung et al., 2022) with the guided step fused into two HIP passes."""

    def __call__(
        self,
        inverse_problem: InverseProblem,
        num_sampling_steps: int = 50,
        num_reconstructions: int = 1,
        gamma: float = 1.0,
        eta: float = 1.0,
        condition: Condition_co | None = None,
        keep_reconstruction_dim: bool = False,
        *args,
        rng: str = "philox",
        seed: int | None = None,
        noise_fn: NoiseFn | None = None,
        sample_offset: int = 0,
        micro_batch: int | None = None,
        timer: KernelTimer | None = None,
        graph: bool | None = None,
        callback: Callable[[int, Tensor], None] | None = None,
        **kwargs,
    ) -> Tensor:
        """Run DPS; returns ``(*batch_shape, R, *x_shape)`` (R squeezed when 1).

        Extra keyword-only options (all default to the reference behaviour):
        ``rng`` / ``seed`` / ``noise_fn`` choose the noise source (module
        docstring); ``sample_offset`` is the global index of this shard's first
        flat sample (multi-GPU, keeps Philox streams shard-invariant);
        ``micro_batch`` bounds how many samples share one prior forward+VJP;
        ``graph=True`` replays one hipGraph-captured step for every iteration
        (``samplers.graph``; Philox noise only) — same samples, no per-launch host work;
        ``graph=None`` (default) applies the automatic rule ``graph_auto`` (native plugins,
        Philox noise, no callback / timer / micro-batching, a flat batch of at most
        ``GRAPH_AUTO_MAX_BATCH`` and enough steps) — currently **off**: ``GRAPH_AUTO_MAX_BATCH``
        is 0 because replay measured slower than eager at every batch, so
        ``graph=None`` runs eagerly; ``graph=False`` always runs eagerly;
        ``callback(i, x)`` is called after guided iteration ``i`` with the flat sample (a view of
        the working buffer: copy it to keep it; not with ``graph=True``).
        """
        if args or kwargs:
            print(f"Warning: Unused args={args}, kwargs={kwargs} in DPSSampler")

        x_shape: Shape = inverse_problem.operator.x_shape
        batch_shape: Shape = inverse_problem.batch_shape
        view = BatchView(batch_shape=batch_shape, num_samples=num_reconstructions, data_shape=x_shape)

        net = self._network
        net.set_sampling_parameters(num_sampling_steps=num_sampling_steps,
                                    num_reconstructions=num_reconstructions,
                                    batch_size=view.batch_size)
        net.set_condition(condition=condition)
        try:
            obs = inverse_problem.observation
            _hip.require_cuda(obs, "DPSSampler")
            y_rows = obs.reshape(max(view.batch_size, 1), *inverse_problem.operator.y_shape)
            step = make_dps_step(net, inverse_problem, y_rows.to(torch.float32), num_reconstructions,
                                 gamma=gamma, eta=eta, micro_batch=micro_batch, timer=timer)
            if seed is None and noise_fn is None and rng == "philox":
                seed = draw_seed()
            seed = int(seed or 0)

            x = initial_sample(view.flat_shape, net.device, rng=rng, seed=seed,
                               sample_offset=sample_offset, noise_fn=noise_fn)
            ts = host_timesteps(net)
            if graph is None:
                graph = graph_auto(step, x, len(ts) - 2, rng=rng, noise_fn=noise_fn,
                                   callback=callback, micro_batch=micro_batch)
            self.execution = "graph" if graph else "eager"  # what the last call ran
            if graph:
                if not isinstance(step, FusedDPSStep) or isinstance(step, GenericDPSStep):
                    raise ValueError("graph=True needs natively implemented plugins")
                if noise_fn is not None or rng != "philox":
                    raise ValueError("graph=True needs the in-kernel Philox noise (rng='philox')")
                if callback is not None:
                    raise ValueError("graph=True replays the steps without returning to the host: "
                                     "no per-iteration callback")
                from .graph import GraphedStepLoop, schedule_for

                GraphedStepLoop(step, x, schedule_for(ts), seed=seed,
                                sample_offset=sample_offset).replay()
            else:
                for i in range(len(ts) - 1, 1, -1):
                    xi = None
                    if noise_fn is not None:
                        xi = noise_fn("step", i, tuple(x.shape)).to(device=x.device,
                                                                    dtype=torch.float32)
                    elif rng == "torch":
                        xi = torch.randn_like(x)
                    step(x, i, ts[i], ts[i - 1], ts[0], xi=xi, seed=seed,
                         sample_offset=sample_offset)
                    if callback is not None:
                        callback(i, x)

            x0_final = view.unflatten(step.predict_x0(x, ts[1]))
            if num_reconstructions == 1 and not keep_reconstruction_dim:
                x0_final = x0_final.squeeze(len(batch_shape))
            return self._as_output(x0_final)
        finally:
            net.clear_condition()
            net.clear_sampling_parameters()

"""Posterior Sampling with Latent Diffusion (mirrors ``/root/reference/samplers/samplers/psld.py:17-166``).

Loop body (``psld.py:118-153``) as an explicit reverse-mode chain: the priors
(latent UNet, VAE decoder, VAE encoder: module graphs over this project's conv /
GroupNorm / GEMM / attention kernels) are differentiated with
``autograd.grad(out, in, grad_outputs=...)``; every
pixel/latent-space step between them is a HIP kernel::

    eps  = UNet(z, t)                     z0 = (z - k eps)/a           sp_predict_x0
    x0   = D(z0)                          r, x_eff = A^T y + (I-A^T A) x0, A^T r, |r|^2   sp_psld_pixel
    zeff = E(x_eff)                       d = z0 - zeff, |d|^2          sp_residual_grad
    L, G = sqrt(sum partials)             (device scalars; all-reduced across ranks)       sp_sum_partials
    u    = E^T(-gamma d / G)              c_x0 = -omega A^T r / L + (I - A^T A) u       sp_psld_cotangent
    c    = D^T(c_x0) + gamma d / G        w = J_eps^T c                                   sp_scaled_combine
    z'   = bridge(z, z0) + std xi - (c - k w)/a                                          sp_dps_update

which is the gradient of ``omega*||y - A D(z0)|| + gamma*||z0 - E(x_eff)||`` that
the reference obtains from one ``autograd.grad`` (``psld.py:140-141``).  The
norms are global over the batch, as in the reference.

Observation tiling uses the observation's own rank, so flattened observations
(inpainting) work for batch > 1 — the reference fails there.
"""

from __future__ import annotations

import math
from typing import Generic, TypeVar

import torch
from torch import Tensor

from samplers_amd import _hip
from samplers_amd.distributed import all_reduce_sum_
from samplers_amd.dtypes import Shape
from samplers_amd.inverse_problem import InverseProblem
from samplers_amd.networks.base import LatentEpsilonNetwork, host_alphas_cumprod, host_timesteps
from samplers_amd.operators import IdentityOperator
from samplers_amd.samplers.base import PosteriorSampler
from samplers_amd.samplers.dps import NoiseFn, draw_seed, initial_sample
from samplers_amd.samplers.utils.batch_view import BatchView
from samplers_amd.samplers.utils.bridge_kernels import bridge_coefficients, x0_coefficients

Condition_co = TypeVar("Condition_co", covariant=True)


def generic_pixel_terms(op, y_rows: Tensor, hty_rows: Tensor, y_div: int, x0: Tensor):
    """PSLD's pixel-space terms for an operator without a HIP descriptor, by its own ``apply``
    / ``apply_transpose`` under autograd (``psld.py:129-136``): returns
    (x_eff = Aᵀy + x̂₀ − AᵀA x̂₀ as a flat fp32 tensor, this shard's ‖y − A x̂₀‖² as a 1-element
    tensor, the autograd graph (x̂₀ leaf, r, x_eff) for the cotangent).  Sample b uses
    observation row b // y_div."""
    b = x0.shape[0]
    idx = torch.arange(b, device=x0.device) // y_div
    y = y_rows.index_select(0, idx).reshape(b, *op.y_shape)
    hty = hty_rows.index_select(0, idx).reshape(b, *op.x_shape)
    with torch.enable_grad():
        x0r = x0.detach().reshape(b, *op.x_shape).requires_grad_(True)
        hx = op.apply(x0r)
        r = y - hx
        x_eff = hty + x0r - op.apply_transpose(hx)
    ss = r.detach().float().square().sum().reshape(1)
    return x_eff.detach().reshape(b, -1).to(torch.float32).contiguous(), ss, (x0r, r, x_eff)


class FusedPSLDStep:
    """One PSLD iteration over a flat latent batch on the HIP path."""

    def __init__(self, network: LatentEpsilonNetwork, inverse_problem: InverseProblem,
                 observation_rows: Tensor, y_div: int, latent_shape: Shape, *, gamma: float = 1.0,
                 omega: float = 0.1, eta: float = 1.0, group=None) -> None:
        op = inverse_problem.operator
        desc = getattr(op, "hip_descriptor", lambda: None)()
        _hip.require_cuda(observation_rows, "PSLDSampler")
        self.lib = _hip.load_library()
        self.net, self.op, self.desc = network, op, desc
        self.y = observation_rows.to(torch.float32).contiguous()
        self.y_div = int(y_div)
        # operators without a HIP descriptor: A, A^T and their VJPs by torch autograd
        self.generic = desc is None
        self.blur = not self.generic and desc.kind == _hip.SP_OP_BLUR
        if self.generic:
            self.n, self.m = int(math.prod(op.x_shape)), int(math.prod(op.y_shape))
        else:
            self.n, self.m = int(desc.n), int(desc.m)
        self.latent_shape = tuple(latent_shape)
        self.nz = int(math.prod(self.latent_shape))
        self.zdesc = IdentityOperator(self.latent_shape).hip_descriptor()
        self.gamma, self.omega, self.eta = float(gamma), float(omega), float(eta)
        self.group = group
        self.hty = None
        self._graph = None
        if self.blur or self.generic:  # A^T y once per run (psld.py:113-115)
            with torch.no_grad():
                self.hty = op.apply_transpose(self.y.reshape(-1, *op.y_shape)).reshape(-1, self.n)

    def _pixel_pass_generic(self, x0: Tensor, norms: Tensor) -> Tensor:
        x_eff, ss, self._graph = generic_pixel_terms(self.op, self.y, self.hty, self.y_div, x0)
        norms.copy_(ss)
        return x_eff

    def _cotangent_generic(self, u: Tensor, norms: Tensor) -> Tensor:
        """c_x0 = ω J_rᵀ r/‖r‖ + J_{x_eff}ᵀ u through the saved graph (the gradient of
        ω‖y − A x̂₀‖ + γ‖ẑ₀ − E(x_eff)‖ w.r.t. x̂₀, given u = its cotangent at x_eff)."""
        x0r, r, x_eff = self._graph
        self._graph = None
        L = norms.sqrt()
        scale = torch.where(L > 0, self.omega / L, torch.zeros_like(L))
        (c,) = torch.autograd.grad((r, x_eff), x0r,
                                   grad_outputs=(r.detach() * scale, u.reshape(x_eff.shape)))
        return c.reshape(u.shape[0], self.n).to(torch.float32).contiguous()

    def _pixel_pass(self, x0: Tensor, norms: Tensor, stream: int) -> tuple[Tensor, Tensor]:
        lib, b = self.lib, x0.shape[0]
        if self.generic:
            return self._pixel_pass_generic(x0, norms), None
        x_eff, atr = torch.empty_like(x0), torch.empty_like(x0)
        if not self.blur:
            P = int(lib.sp_rsq_partials(self.desc))
            part = torch.empty(b, P, device=x0.device)
            _hip.check(lib.sp_psld_pixel(self.desc, _hip.ptr(x0), _hip.ptr(self.y), b, self.y_div,
                                         _hip.ptr(x_eff), _hip.ptr(atr), _hip.ptr(part), stream),
                       "sp_psld_pixel")
        else:
            hx = torch.empty(b, self.m, device=x0.device)
            _hip.check(lib.sp_op_apply(self.desc, _hip.ptr(x0), _hip.ptr(hx), b, stream), "apply")
            r = torch.empty_like(hx)
            P = int(lib.sp_vec_partials(self.m))
            part = torch.empty(b, P, device=x0.device)
            _hip.check(lib.sp_residual_grad(_hip.ptr(self.y), _hip.ptr(hx), b, self.m, self.y_div,
                                            1.0, _hip.ptr(r), _hip.ptr(part), stream), "residual")
            _hip.check(lib.sp_op_adjoint(self.desc, _hip.ptr(r), _hip.ptr(atr), b, stream), "adj")
            at_hx = torch.empty_like(x0)
            _hip.check(lib.sp_op_adjoint(self.desc, _hip.ptr(hx), _hip.ptr(at_hx), b, stream), "adj")
            hty = self.hty.repeat_interleave(self.y_div, dim=0).contiguous()
            _hip.check(lib.sp_scaled_combine(_hip.ptr(x0), 1.0, _hip.ptr(at_hx), -1.0, None,
                                             x0.numel(), _hip.ptr(x_eff), stream), "combine")
            _hip.check(lib.sp_scaled_combine(_hip.ptr(hty), 1.0, _hip.ptr(x_eff), 1.0, None,
                                             x0.numel(), _hip.ptr(x_eff), stream), "combine")
        _hip.check(lib.sp_sum_partials(_hip.ptr(part), part.numel(), norms.data_ptr(), stream),
                   "sp_sum_partials")
        return x_eff, atr

    def __call__(self, z: Tensor, step: int, t: int, t_prev: int, s: int, *,
                 xi: Tensor | None = None, seed: int = 0, sample_offset: int = 0) -> Tensor:
        lib, net = self.lib, self.net
        b = z.shape[0]
        stream = _hip.stream_of(z)
        acp = host_alphas_cumprod(net)
        a, k = x0_coefficients(acp, t)
        br = bridge_coefficients(acp, ell=t, t=t_prev, s=s, eta=self.eta)
        norms = torch.zeros(2, device=z.device, dtype=torch.float32)  # [|y - A x0|^2, |z0 - z_eff|^2]

        with torch.enable_grad():
            zr = z.detach().requires_grad_(True)
            eps = net.forward(zr, t)
        eps_c = eps.detach().contiguous()
        z0 = torch.empty_like(z)
        _hip.check(lib.sp_predict_x0(_hip.ptr(z), _hip.ptr(eps_c), z.numel(), a, k, _hip.ptr(z0),
                                     stream), "sp_predict_x0")
        with torch.enable_grad():
            z0r = z0.detach().requires_grad_(True)
            x0 = net.decode(z0r, differentiable=True)
        x0c = x0.detach().reshape(b, self.n).contiguous()
        x_eff, atr = self._pixel_pass(x0c, norms[0:1], stream)

        with torch.enable_grad():
            xer = x_eff.reshape(x0.shape).requires_grad_(True)
            z_eff = net.encode(xer, differentiable=True)
        d = torch.empty_like(z0)
        Pz = int(lib.sp_vec_partials(self.nz))
        partz = torch.empty(b, Pz, device=z.device)
        _hip.check(lib.sp_residual_grad(_hip.ptr(z0), _hip.ptr(z_eff.detach().contiguous()), b,
                                        self.nz, 1, 1.0, _hip.ptr(d), _hip.ptr(partz), stream),
                   "sp_residual_grad")
        _hip.check(lib.sp_sum_partials(_hip.ptr(partz), partz.numel(), norms[1:2].data_ptr(),
                                       stream), "sp_sum_partials")
        all_reduce_sum_(norms, self.group)  # batch-global norms (psld.py:130,138): 8 bytes

        go = torch.empty_like(d)  # d(gamma*G)/d z_eff = -gamma d / G
        _hip.check(lib.sp_scaled_combine(None, 0.0, _hip.ptr(d), -self.gamma, norms[1:2].data_ptr(),
                                         d.numel(), _hip.ptr(go), stream), "combine")
        (u,) = torch.autograd.grad(z_eff, xer, grad_outputs=go)
        u = u.reshape(b, self.n).contiguous()
        ata_u = None
        if self.generic:
            c_x0 = self._cotangent_generic(u, norms[0:1])
        elif self.blur:
            au = torch.empty(b, self.m, device=z.device)
            _hip.check(lib.sp_op_apply(self.desc, _hip.ptr(u), _hip.ptr(au), b, stream), "apply")
            ata_u = torch.empty_like(u)
            _hip.check(lib.sp_op_adjoint(self.desc, _hip.ptr(au), _hip.ptr(ata_u), b, stream), "adj")
        if not self.generic:
            c_x0 = torch.empty_like(u)
            _hip.check(lib.sp_psld_cotangent(self.desc, _hip.ptr(atr), _hip.ptr(u), _hip.ptr(ata_u),
                                             norms[0:1].data_ptr(), self.omega, b, _hip.ptr(c_x0),
                                             stream), "sp_psld_cotangent")
        (c_dec,) = torch.autograd.grad(x0, z0r, grad_outputs=c_x0.reshape(x0.shape))
        c = torch.empty_like(z0)
        _hip.check(lib.sp_scaled_combine(_hip.ptr(c_dec.contiguous()), 1.0, _hip.ptr(d), self.gamma,
                                         norms[1:2].data_ptr(), c.numel(), _hip.ptr(c), stream),
                   "combine")
        (w,) = torch.autograd.grad(eps, zr, grad_outputs=c)
        del eps, zr, x0, z0r, z_eff, xer
        coefs = _hip.SpDpsCoefs(a, k, 0.0, br.c_ell, br.c_s, br.std, -1.0, 0.0)
        xic = None if xi is None else xi.contiguous()
        _hip.check(lib.sp_dps_update(self.zdesc, _hip.ptr(z), _hip.ptr(eps_c), None, _hip.ptr(c),
                                     _hip.ptr(w.contiguous()), None, _hip.ptr(xic), seed, step,
                                     sample_offset, b, 1, coefs, _hip.ptr(z), stream),
                   "sp_dps_update")
        return z

    def predict_x0(self, z: Tensor, t: int) -> Tensor:
        a, k = x0_coefficients(host_alphas_cumprod(self.net), t)
        with torch.no_grad():
            eps = self.net.forward(z, t).contiguous()
        out = torch.empty_like(z)
        _hip.check(self.lib.sp_predict_x0(_hip.ptr(z), _hip.ptr(eps), z.numel(), a, k,
                                          _hip.ptr(out), _hip.stream_of(z)), "sp_predict_x0")
        return out


class PSLDSampler(PosteriorSampler, Generic[Condition_co]):
    """PSLD (Rout et al., NeurIPS 2023) with the pixel/latent glue in HIP."""

    def __init__(self, network):
        super().__init__(network)
        if not isinstance(self._epsilon_network, LatentEpsilonNetwork):
            raise TypeError(
                f"{self.__class__.__name__} requires a latent diffusion model, but build_network "
                f"returned a non-latent network ({type(self._epsilon_network).__name__})."
            )

    def __call__(
        self,
        inverse_problem: InverseProblem,
        *,
        num_sampling_steps: int = 100,
        num_reconstructions: int = 1,
        gamma: float = 1.0,
        omega: float = 0.1,
        eta: float = 1.0,
        decode_output: bool = True,
        condition: Condition_co | None = None,
        rng: str = "philox",
        seed: int | None = None,
        noise_fn: NoiseFn | None = None,
        sample_offset: int = 0,
        group=None,
    ) -> Tensor:
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
            _hip.require_cuda(obs, "PSLDSampler")
            y_rows = obs.reshape(max(x_view.batch_size, 1), -1).to(torch.float32)
            step = FusedPSLDStep(net, inverse_problem, y_rows, num_reconstructions, latent_shape,
                                 gamma=gamma, omega=omega, eta=eta, group=group)
            if seed is None and noise_fn is None and rng == "philox":
                seed = draw_seed()
            seed = int(seed or 0)
            z = initial_sample(z_view.flat_shape, net.device, rng=rng, seed=seed,
                               sample_offset=sample_offset, noise_fn=noise_fn)
            ts = host_timesteps(net)
            for i in range(len(ts) - 1, 1, -1):
                xi = None
                if noise_fn is not None:
                    xi = noise_fn("step", i, tuple(z.shape)).to(device=z.device, dtype=torch.float32)
                elif rng == "torch":
                    xi = torch.randn_like(z)
                step(z, i, ts[i], ts[i - 1], ts[0], xi=xi, seed=seed, sample_offset=sample_offset)
            final_z0 = step.predict_x0(z, ts[1])
            if decode_output:
                return self._as_output(x_view.unflatten(net.decode(final_z0, differentiable=False)))
            return self._as_output(z_view.unflatten(final_z0))
        finally:
            net.clear_condition()
            net.clear_sampling_parameters()

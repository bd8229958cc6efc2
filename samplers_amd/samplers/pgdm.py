"""Pseudoinverse-Guided Diffusion Models (mirrors ``/root/reference/samplers/samplers/pgdm.py:18-147``).

Loop body (``pgdm.py:104-135``) on the same two fused HIP passes as DPS:
pass 1 computes v = ∂/∂x0 ||A⁺y − A⁺A x0||² = −2 Aᵀ(y − A x0) (A⁺ = Aᵀ for the
identity / inpainting / mask operators, which are partial isometries), the
prior's input-VJP gives w = Jᵀv, and pass 2 writes
``ddim_step(x, x0) − guidance_weight·sqrt(1−ᾱ_t)·(v − k w)/a``.
Operators without ``apply_pseudo_inverse`` raise ``NotImplementedError`` as in
the reference (``pgdm.py:56-66``).
"""

from __future__ import annotations

from typing import Generic, TypeVar

import torch
from torch import Tensor

from samplers_amd import _hip
from samplers_amd.dtypes import Shape
from samplers_amd.inverse_problem import InverseProblem
from samplers_amd.networks.base import host_timesteps
from samplers_amd.samplers.base import PosteriorSampler
from samplers_amd.samplers.dps import KernelTimer, NoiseFn, draw_seed, initial_sample, make_dps_step
from samplers_amd.samplers.utils.batch_view import BatchView

Condition_co = TypeVar("Condition_co", covariant=True)


class PGDMSampler(PosteriorSampler, Generic[Condition_co]):
    """PGDM (Song et al., ICLR 2023) with the guided step fused into two HIP passes."""

    def __call__(
        self,
        inverse_problem: InverseProblem,
        num_sampling_steps: int = 50,
        num_reconstructions: int = 1,
        guidance_weight: float = 1.0,
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
        **kwargs,
    ) -> Tensor:
        operator = inverse_problem.operator
        try:
            dummy_y = torch.zeros((1, *operator.y_shape),
                                  device=next(operator.buffers(), torch.tensor(0)).device)
            operator.apply_pseudo_inverse(dummy_y)
        except NotImplementedError as exc:
            raise NotImplementedError(
                "The operator in the inverse_problem must implement 'apply_pseudo_inverse' for PGDM."
            ) from exc
        if args or kwargs:
            print(f"Warning: Unused args={args}, kwargs={kwargs} in PGDMSampler")

        x_shape: Shape = operator.x_shape
        batch_shape: Shape = inverse_problem.batch_shape
        view = BatchView(batch_shape=batch_shape, num_samples=num_reconstructions, data_shape=x_shape)
        net = self._network
        net.set_sampling_parameters(num_sampling_steps=num_sampling_steps,
                                    num_reconstructions=num_reconstructions,
                                    batch_size=view.batch_size)
        net.set_condition(condition=condition)
        try:
            obs = inverse_problem.observation
            _hip.require_cuda(obs, "PGDMSampler")
            y_rows = obs.reshape(max(view.batch_size, 1), *operator.y_shape).to(torch.float32)
            step = make_dps_step(net, inverse_problem, y_rows, num_reconstructions, eta=eta,
                                 micro_batch=micro_batch, timer=timer, mode="pgdm",
                                 guidance_weight=guidance_weight)
            if seed is None and noise_fn is None and rng == "philox":
                seed = draw_seed()
            seed = int(seed or 0)
            x = initial_sample(view.flat_shape, net.device, rng=rng, seed=seed,
                               sample_offset=sample_offset, noise_fn=noise_fn)
            ts = host_timesteps(net)
            for i in range(len(ts) - 1, 1, -1):
                xi = None
                if noise_fn is not None:
                    xi = noise_fn("step", i, tuple(x.shape)).to(device=x.device, dtype=torch.float32)
                elif rng == "torch":
                    xi = torch.randn_like(x)
                step(x, i, ts[i], ts[i - 1], ts[0], xi=xi, seed=seed, sample_offset=sample_offset)
            x0_final = view.unflatten(step.predict_x0(x, ts[1]))
            if num_reconstructions == 1 and not keep_reconstruction_dim:
                x0_final = x0_final.squeeze(len(batch_shape))
            return self._as_output(x0_final)
        finally:
            net.clear_condition()
            net.clear_sampling_parameters()

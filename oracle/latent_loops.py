"""torch-CPU restatements of the PGDM and PSLD loops — TEST INFRASTRUCTURE ONLY.

``pgdm_reference`` follows ``/root/reference/samplers/samplers/pgdm.py:83-147``
and ``psld_reference`` follows ``/root/reference/samplers/samplers/psld.py:100-163``
operation by operation (same autograd graphs, same bridge step as
``oracle.dps_loop.bridge_step``), with prior, VAE, operator and noise injected.
``observation_rows`` is the observation already tiled to the flat batch (the
reference's ``repeat_observation``).
"""

from __future__ import annotations

from typing import Callable

import torch
from torch import Tensor

from oracle.dps_loop import bridge_step

Fn = Callable[[Tensor], Tensor]


def pgdm_reference(eps_fn, alphas_cumprod: Tensor, timesteps: list[int], apply_op: Fn, pinv: Fn,
                   observation_rows: Tensor, x_init: Tensor, step_noise, *,
                   guidance_weight: float = 1.0, eta: float = 1.0) -> Tensor:
    acp = alphas_cumprod
    sample = x_init
    for i in range(len(timesteps) - 1, 1, -1):
        t, t_prev = int(timesteps[i]), int(timesteps[i - 1])
        sample = sample.detach().requires_grad_()
        acp_t = acp[t]
        x0_pred = (sample - (1 - acp_t) ** 0.5 * eps_fn(sample, t)) / (acp_t**0.5)
        with torch.enable_grad():
            y0_inv = pinv(observation_rows)
            x0_pred_inv = pinv(apply_op(x0_pred))
            loss = (y0_inv - x0_pred_inv).pow(2).sum()
        grad = torch.autograd.grad(loss, sample)[0]
        sample_ddim = bridge_step(sample.detach(), x0_pred.detach(), acp, ell=t, t=t_prev,
                                  s=int(timesteps[0]), eta=eta, xi=step_noise(i))
        with torch.no_grad():
            scale = guidance_weight * torch.sqrt(1 - acp[t])
            sample = sample_ddim - scale * grad
    with torch.no_grad():
        t1 = int(timesteps[1])
        return (sample - (1 - acp[t1]) ** 0.5 * eps_fn(sample, t1)) / (acp[t1] ** 0.5)


def psld_reference(eps_fn, alphas_cumprod: Tensor, timesteps: list[int], apply_op: Fn,
                   adjoint_op: Fn, decode: Fn, encode: Fn, observation_rows: Tensor,
                   z_init: Tensor, step_noise, *, gamma: float = 1.0, omega: float = 0.1,
                   eta: float = 1.0, decode_output: bool = True, steps_limit: int | None = None
                   ) -> Tensor:
    acp = alphas_cumprod
    z_t = z_init
    hty = adjoint_op(observation_rows)
    done = 0
    for i in range(len(timesteps) - 1, 1, -1):
        if steps_limit is not None and done >= steps_limit:
            return z_t.detach()
        t, t_prev = int(timesteps[i]), int(timesteps[i - 1])
        z_t = z_t.detach().requires_grad_()
        acp_t = acp[t]
        z0 = (z_t - (1 - acp_t) ** 0.5 * eps_fn(z_t, t)) / (acp_t**0.5)
        x0 = decode(z0)
        hx0 = apply_op(x0)
        likelihood_error = torch.norm(observation_rows - hx0)
        x_eff = hty + x0 - adjoint_op(hx0)
        z_eff = encode(x_eff)
        gluing_error = torch.norm(z0 - z_eff)
        total = omega * likelihood_error + gamma * gluing_error
        (gradient,) = torch.autograd.grad(total, z_t)
        with torch.no_grad():
            z_t = bridge_step(z_t.detach(), z0, acp, ell=t, t=t_prev, s=int(timesteps[0]), eta=eta,
                              xi=step_noise(i))
            z_t = z_t - gradient
        done += 1
    with torch.no_grad():
        t1 = int(timesteps[1])
        z0 = (z_t - (1 - acp[t1]) ** 0.5 * eps_fn(z_t, t1)) / (acp[t1] ** 0.5)
        return decode(z0) if decode_output else z0

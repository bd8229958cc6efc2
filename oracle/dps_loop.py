"""torch-CPU restatement of the reference DPS loop — TEST INFRASTRUCTURE ONLY.

Follows ``/root/reference/samplers/samplers/dps.py:25-134`` operation by
operation (same autograd graph, same fp64 bridge coefficients from
``utils/bridge_kernels.py:15-75``, same residual-norm correction), with the
prior, operator and noise model passed in as plain callables so the same loop
checks the GPU sampler and, timed on the host cores, provides the CPU baseline.
"""

from __future__ import annotations

from typing import Callable

import torch
from torch import Tensor


def gaussian_log_prob(sigma: float | Tensor) -> Callable[[Tensor], Tensor]:
    """``noise.py:77-79``."""
    sig = torch.as_tensor(sigma)

    def log_prob(r: Tensor) -> Tensor:
        var = sig.to(r.dtype).pow(2)
        return -(r.square().sum(dim=tuple(range(1, r.ndim)))) / (2 * var)

    return log_prob


def poisson_log_prob(rate: float | Tensor) -> Callable[[Tensor], Tensor]:
    """``noise.py:121-123``."""
    lam = torch.as_tensor(rate)

    def log_prob(r: Tensor) -> Tensor:
        return -(r.pow(2) / (lam.to(r.dtype) + 1e-3)).sum(dim=tuple(range(1, r.ndim)))

    return log_prob


def bridge_step(x_ell: Tensor, x_s: Tensor, acp: Tensor, ell: int, t: int, s: int, eta: float,
                xi: Tensor) -> Tensor:
    """``compute_bridge_kernel_statistics`` + ``sample_bridge_kernel`` (bridge_kernels.py:15-59)."""
    dtype = x_ell.dtype
    a_t = acp[t].to(torch.float64)
    a_ell = acp[ell].to(torch.float64)
    a_s = acp[s].to(torch.float64)
    a_st = a_t / a_s
    a_tl = a_ell / a_t
    a_sl = a_ell / a_s
    std = eta * ((1 - a_tl) * (1 - a_st) / (1 - a_sl)) ** 0.5
    c_ell = ((1 - a_st - std**2) / (1 - a_sl)) ** 0.5
    c_s = (a_st**0.5) - c_ell * (a_sl**0.5)
    mean = (c_ell * x_ell + c_s * x_s).to(dtype=dtype)
    return mean + std.to(dtype=dtype) * xi


def dps_reference(
    eps_fn: Callable[[Tensor, int], Tensor],
    alphas_cumprod: Tensor,
    timesteps: list[int],
    apply_op: Callable[[Tensor], Tensor],
    log_prob: Callable[[Tensor], Tensor],
    observation: Tensor,
    x_init: Tensor,
    step_noise: Callable[[int], Tensor],
    *,
    gamma: float = 1.0,
    eta: float = 1.0,
    leading_size: int | None = None,
    steps_limit: int | None = None,
    return_sample: bool = False,
) -> Tensor:
    """DPS as in ``dps.py:83-126``; returns the final x0 prediction (flat batch).

    ``step_noise(i)`` returns the standard normal drawn at loop index ``i``
    (``randn_like`` in ``sample_bridge_kernel``).  ``steps_limit`` stops after
    that many guided iterations and ``return_sample`` returns x instead of the
    final prediction (the CPU baseline times a bounded sample of iterations).
    """
    acp = alphas_cumprod
    sample = x_init
    b = leading_size or sample.shape[0]
    bshape = (b,) + (1,) * (sample.ndim - 1)
    done = 0
    for i in range(len(timesteps) - 1, 1, -1):
        if steps_limit is not None and done >= steps_limit:
            break
        t, t_prev = int(timesteps[i]), int(timesteps[i - 1])
        sample = sample.detach().requires_grad_()
        acp_t = acp[t]
        x0_pred = (sample - (1 - acp_t) ** 0.5 * eps_fn(sample, t)) / (acp_t**0.5)
        log_l = log_prob(observation - apply_op(x0_pred)).sum()
        grad_pot = torch.autograd.grad(log_l, sample)[0]
        sample = bridge_step(sample.detach(), x0_pred, acp, ell=t, t=t_prev, s=int(timesteps[0]),
                             eta=eta, xi=step_noise(i))
        with torch.no_grad():
            residual = observation - apply_op(x0_pred)
            residual = residual.reshape(b, -1)
            error = residual.norm(dim=1).view(bshape)
            sample = sample + (gamma / (error + 1e-9)) * grad_pot
        done += 1
    if return_sample:
        return sample.detach()
    with torch.no_grad():
        t1 = int(timesteps[1])
        acp_t = acp[t1]
        return (sample - (1 - acp_t) ** 0.5 * eps_fn(sample, t1)) / (acp_t**0.5)

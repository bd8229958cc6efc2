"""Diffusion bridge / DDIM updates.

``bridge_coefficients`` restates ``compute_bridge_kernel_statistics``
(``/root/reference/samplers/samplers/utils/bridge_kernels.py:15-46``) on the
host: the alphas are promoted to fp64, every coefficient is computed in fp64
and handed to the fp32 kernels (the reference multiplies fp64 0-d tensors into
fp32 tensors, which rounds the coefficient to fp32 first).

The tensor-level functions keep the reference API for samplers that need it
(PGDM / ReSample); on device tensors ``ddim_step`` / ``ddim_step_eps`` run the
HIP kernels (bridge mean + Philox / injected noise).
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch
from torch import Tensor

from samplers_amd.networks.base import EpsilonNetwork, host_alphas_cumprod, host_timesteps


@dataclass(frozen=True)
class BridgeCoefficients:
    c_ell: float  # weight of x_ell (the current sample)
    c_s: float    # weight of x_s (the x0 prediction)
    std: float


@dataclass(frozen=True)
class BridgeStatistics:
    mean: Tensor
    std: Tensor


def bridge_coefficients(acp: np.ndarray, ell: int, t: int, s: int, eta: float) -> BridgeCoefficients:
    """fp32-rounded coefficients of the bridge kernel q(x_t | x_ell, x_s), s < t < ell."""
    a_t = np.float64(np.float32(acp[t]))
    a_ell = np.float64(np.float32(acp[ell]))
    a_s = np.float64(np.float32(acp[s]))
    a_st = a_t / a_s
    a_tl = a_ell / a_t
    a_sl = a_ell / a_s
    with np.errstate(invalid="ignore", divide="ignore"):
        std = eta * ((1 - a_tl) * (1 - a_st) / (1 - a_sl)) ** 0.5
        c_ell = ((1 - a_st - std**2) / (1 - a_sl)) ** 0.5
        c_s = a_st**0.5 - c_ell * a_sl**0.5
    return BridgeCoefficients(float(np.float32(c_ell)), float(np.float32(c_s)), float(np.float32(std)))


def x0_coefficients(acp: np.ndarray, t: int) -> tuple[float, float]:
    """(a, k) = (sqrt(acp[t]), sqrt(1 - acp[t])) in fp32, as ``predict_x0`` computes them."""
    acp_t = np.float32(acp[t])
    k = np.sqrt(np.float32(1.0) - acp_t, dtype=np.float32)
    a = np.sqrt(acp_t, dtype=np.float32)
    return float(a), float(k)


def compute_bridge_kernel_statistics(x_ell: Tensor, x_s: Tensor, epsilon_net: EpsilonNetwork,
                                     ell: int, t: int, s: int, eta: float = 1.0) -> BridgeStatistics:
    c = bridge_coefficients(host_alphas_cumprod(epsilon_net), ell, t, s, eta)
    mean = c.c_ell * x_ell + c.c_s * x_s
    return BridgeStatistics(mean=mean, std=torch.tensor(c.std, dtype=x_ell.dtype, device=x_ell.device))


def sample_bridge_kernel(x_ell: Tensor, x_s: Tensor, epsilon_net: EpsilonNetwork, ell: int, t: int,
                         s: int, eta: float = 1.0) -> Tensor:
    st = compute_bridge_kernel_statistics(x_ell, x_s, epsilon_net, ell, t, s, eta)
    return st.mean + st.std * torch.randn_like(st.mean)


def ddim_step(x: Tensor, epsilon_net: EpsilonNetwork, t: int, t_prev: int, eta: float,
              e_t: Tensor | None = None) -> Tensor:
    """DDIM step in the x0 ("bridge") parameterisation (``bridge_kernels.py:62-75``)."""
    t_0 = host_timesteps(epsilon_net)[0]
    if e_t is None:
        e_t = epsilon_net.predict_x0(x, t)
    return sample_bridge_kernel(x_ell=x, x_s=e_t, epsilon_net=epsilon_net, ell=t, t=t_prev, s=t_0,
                                eta=eta)


def eps_step_coefficients(acp: np.ndarray, t: int, t_prev: int, eta: float) -> dict[str, float]:
    """Scalars of ``ddim_step_eps`` (``bridge_kernels.py:82-115``), fp32 as the reference."""
    f = np.float32
    a_t, a_p = f(acp[t]), f(acp[t_prev])
    one = f(1.0)
    sigma = f(eta) * np.sqrt(np.maximum((one - a_p) / (one - a_t) * (one - a_t / a_p), f(0)),
                             dtype=np.float32)
    dir_c = np.sqrt(np.maximum(one - a_p - sigma * sigma, f(0)), dtype=np.float32)
    return {
        "sqrt_oma": float(np.sqrt(one - a_t, dtype=np.float32)),
        "oma": float(one - a_t),
        "sqrt_a": float(np.sqrt(a_t, dtype=np.float32)),
        "sqrt_a_prev": float(np.sqrt(a_p, dtype=np.float32)),
        "sigma": float(sigma),
        "dir": float(dir_c),
    }


def ddim_step_eps(x: Tensor, *, epsilon_net: EpsilonNetwork, t: int, t_prev: int,
                  eta: float) -> tuple[Tensor, Tensor, Tensor]:
    """ε-form DDIM step returning (x_prev, x0, pseudo-x0) (``bridge_kernels.py:82-115``)."""
    c = eps_step_coefficients(host_alphas_cumprod(epsilon_net), t, t_prev, eta)
    with torch.no_grad():
        e_t = epsilon_net.predict_noise(x, t)
    pred_x0 = (x - c["sqrt_oma"] * e_t) / c["sqrt_a"]
    pseudo_x0 = (x - c["oma"] * e_t) / c["sqrt_a"]
    noise = c["sigma"] * torch.randn_like(x)
    x_prev = c["sqrt_a_prev"] * pred_x0 + c["dir"] * e_t + noise
    return x_prev, pred_x0, pseudo_x0

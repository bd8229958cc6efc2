"""Noise models (mirrors ``/root/reference/samplers/noise.py:13-138``).

Besides the reference API (``log_prob``, ``score``, ``sample``) each model
reports ``grad_scale()``: the fp32 factor ``c`` with ``d log p / d(Ax) = c * r``
that the fused HIP kernels apply (Gaussian ``1/sigma^2``, Poisson
``2/(rate + 1e-3)``).
"""

from __future__ import annotations

from abc import ABC, abstractmethod

import numpy as np
import torch
from torch import nn

from samplers_amd.dtypes import RNG, Device, DType, Shape, Tensor


def _validate_scalar(t: Tensor, name: str) -> None:
    if t.ndim != 0:
        raise ValueError(f"`{name}` must be a scalar (0-D tensor).")


class NoiseModel(nn.Module, ABC):
    """Abstract noise model with log-probability, score, and sampling."""

    @abstractmethod
    def log_prob(self, residual: Tensor) -> Tensor: ...

    def score(self, residual: Tensor) -> Tensor:
        """∇ log p(residual) by autograd (``noise.py:19-27``)."""
        residual = residual.detach().requires_grad_(True)
        with torch.enable_grad():
            logp = self.log_prob(residual).sum()
            (grad,) = torch.autograd.grad(logp, residual, retain_graph=True)
        return grad

    @abstractmethod
    def sample(self, shape: Shape, *, device: Device | None = None, dtype: DType = None,
               generator: RNG = None) -> Tensor: ...

    def grad_scale(self) -> float | None:
        """fp32 ``c`` such that ``∂ log p / ∂(Ax) = c · (y − Ax)`` per element, or ``None``.

        Not part of the reference ABC (``noise.py:13-45``), so a subclass written against
        it need not define it.  This default probes ``score`` (autograd of ``log_prob``) on
        a fixed residual: if the score is ``−c·r`` for one scalar c at every element (an
        isotropic quadratic log-density, e.g. a Gaussian), c is returned and the fused HIP
        passes apply it; otherwise ``None`` and the samplers differentiate ``log_prob``
        by autograd for the residual cotangent (the generic plugin path)."""
        return probe_grad_scale(self)

    @property
    def device(self) -> torch.device:
        return next(self.buffers()).device

    @property
    def dtype(self) -> torch.dtype:
        return next(self.buffers()).dtype


def _draw_device(device, generator):
    """Where to draw: the generator's device when one is given (a CPU generator with a device
    observation draws on the host and the values move; the reference requires them to match),
    else ``device``."""
    if generator is None:
        return device
    return generator.device


PROBE_SCALES = (1.0, 1e2, 1e-3)  # residual magnitudes the probe checks the score at


def probe_grad_scale(noise) -> float | None:
    """``c`` with ``score(r) == −c·r`` on probe residuals, or ``None`` (see
    ``NoiseModel.grad_scale``).  Works on any object with the reference's
    ``score`` / ``log_prob`` methods (duck-typed third-party models).

    The residuals are standard normals scaled by each of ``PROBE_SCALES`` (|r| from ~1e-3
    to a few hundred): a density that is quadratic only near zero (Huber, a clipped or
    tempered Gaussian) gives a different ``c`` at some scale and takes the generic autograd
    path, as does anything whose score is not exactly proportional to the residual."""
    gen = torch.Generator().manual_seed(0)
    base = torch.randn(2, 64, generator=gen, dtype=torch.float32)
    base[:, 0] = 1.0
    c = None
    for scale in PROBE_SCALES:
        r = base * scale
        try:
            buffers = list(noise.buffers()) if isinstance(noise, nn.Module) else []
            dev = buffers[0].device if buffers else torch.device("cpu")
            score = getattr(noise, "score", None)
            if score is None:
                return None
            g = score(r.to(dev)).detach().float().cpu()
        except Exception:  # noqa: BLE001 - a model that cannot be probed takes the generic path
            return None
        if g.shape != r.shape or not torch.isfinite(g).all():
            return None
        cs = -float(g[0, 0]) / scale
        if not np.isfinite(cs) or cs == 0.0:
            return None
        if not torch.allclose(g, -cs * r, rtol=1e-5, atol=1e-6 * abs(cs) * scale):
            return None
        if c is None:
            c = cs
        elif abs(cs - c) > 1e-5 * abs(c):
            return None
    return float(np.float32(c))


class GaussianNoise(NoiseModel):
    """Independent Gaussian noise ε ~ N(0, σ²)."""

    sigma: Tensor

    def __init__(self, sigma: float | Tensor, *, device: Device = None, dtype: DType = None) -> None:
        super().__init__()
        if isinstance(sigma, Tensor):
            _validate_scalar(sigma, "sigma")
            sigma_tensor = sigma.detach().clone()
        else:
            sigma_tensor = torch.tensor(float(sigma), device=device, dtype=dtype or torch.float32)
        if torch.any(sigma_tensor <= 0):
            raise ValueError("σ must be positive.")
        self.register_buffer("sigma", sigma_tensor)

    def log_prob(self, r: Tensor) -> Tensor:
        var = self.sigma.pow(2)
        return -(r.square().sum(dim=tuple(range(1, r.ndim)))) / (2 * var)

    def sample(self, shape: Shape, *, device: Device = None, dtype: DType = None,
               generator: RNG = None) -> Tensor:
        device = self.sigma.device if device is None else device
        dtype = self.sigma.dtype if dtype is None else dtype
        eps = torch.randn(shape, dtype=dtype, device=_draw_device(device, generator),
                          generator=generator).to(device)
        return eps * self.sigma.to(dtype)

    def grad_scale(self) -> float:
        # autograd of -(sum r^2)/(2 var): 2 r * (1/(2 var)) with var = sigma^2 in fp32
        var = np.float32(self.sigma.detach().cpu().item()) ** 2
        return float(np.float32(1.0) / np.float32(var))


class PoissonNoise(NoiseModel):
    """Poisson noise ε = k − λ, k ~ Pois(λ); log-prob is the Gaussian approximation."""

    rate: Tensor

    def __init__(self, rate: float | Tensor, *, device: Device | None = None, dtype: DType = None) -> None:
        super().__init__()
        if isinstance(rate, Tensor):
            _validate_scalar(rate, "rate")
            rate_tensor = rate.detach().clone()
        else:
            rate_tensor = torch.tensor(float(rate), device=device, dtype=dtype or torch.float32)
        if rate_tensor <= 0:
            raise ValueError("λ (rate) must be positive.")
        self.register_buffer("rate", rate_tensor)

    def log_prob(self, r: Tensor) -> Tensor:
        return -(r.pow(2) / (self.rate + 1e-3)).sum(dim=tuple(range(1, r.ndim)))

    def sample(self, shape: Shape, *, device: Device = None, dtype: DType = None,
               generator: RNG = None) -> Tensor:
        device = self.rate.device if device is None else device
        dtype = self.rate.dtype if dtype is None else dtype
        lam = torch.full(shape, self.rate.item(), device=_draw_device(device, generator),
                         dtype=dtype)
        k = torch.poisson(lam, generator=generator)
        return (k - lam).to(device)

    def grad_scale(self) -> float:
        denom = np.float32(self.rate.detach().cpu().item()) + np.float32(1e-3)
        return float(np.float32(2.0) / np.float32(denom))

"""Gaussian blur operator (BASELINE config 3: 9x9, sigma=3).

The reference ships no blur operator (``/root/reference/samplers/operators/
__init__.py:1-24``), so its semantics are defined here and
pinned by ``oracle/blur.py`` (torch autograd of the same map):

* depthwise, separable: 1-D taps ``k_i ∝ exp(-(i-R)^2 / (2 sigma^2))``,
  normalised to sum 1, R = kernel_size // 2 (the DPS paper's deblurring setup);
* reflect padding by R on both spatial axes (``F.pad(mode="reflect")``);
* ``apply_transpose`` is the exact adjoint (zero-extended correlation followed
  by folding the padded halo back onto the reflected pixels);
* no pseudo-inverse (deconvolution is ill-posed; PGDM raises as in the
  reference for operators lacking ``apply_pseudo_inverse``).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from samplers_amd import _hip
from samplers_amd.dtypes import Device, Shape, Tensor

from .base import HipLinearMap
from .linear import LinearOperator


def gaussian_taps(kernel_size: int, sigma: float) -> torch.Tensor:
    """Normalised 1-D Gaussian taps (computed in fp64, stored fp32)."""
    r = kernel_size // 2
    i = torch.arange(-r, r + 1, dtype=torch.float64)
    k = torch.exp(-(i**2) / (2.0 * sigma**2))
    return (k / k.sum()).to(torch.float32)


def blur_reflect_torch(x: Tensor, taps: Tensor) -> Tensor:
    """Host (torch) form of the forward map on ``(..., C, H, W)``."""
    r = (taps.numel() - 1) // 2
    shape = x.shape
    planes = x.reshape(-1, 1, shape[-2], shape[-1])
    p = F.pad(planes, (r, r, r, r), mode="reflect")
    kw = taps.to(x.dtype).view(1, 1, 1, -1)
    kh = taps.to(x.dtype).view(1, 1, -1, 1)
    out = F.conv2d(F.conv2d(p, kw), kh)
    return out.reshape(shape)


class GaussianBlurOperator(LinearOperator):
    """Depthwise Gaussian blur with reflect padding; ``y`` has ``x_shape``."""

    def __init__(self, x_shape: Shape, kernel_size: int = 9, sigma: float = 3.0,
                 device: Device = None) -> None:
        if kernel_size % 2 != 1 or not (3 <= kernel_size <= 17):
            raise ValueError("kernel_size must be odd and in [3, 17]")
        if sigma <= 0:
            raise ValueError("sigma must be positive")
        if len(x_shape) != 3:
            raise ValueError("x_shape must be (C, H, W)")
        r = kernel_size // 2
        if x_shape[-1] <= 2 * r or x_shape[-2] <= 2 * r:
            raise ValueError("image must be larger than the blur kernel for reflect padding")
        torch.nn.Module.__init__(self)
        self.kernel_size, self.sigma, self.radius = kernel_size, float(sigma), r
        self.register_buffer("taps", gaussian_taps(kernel_size, sigma).to(device))
        self.x_shape = tuple(x_shape)
        self.y_shape = tuple(x_shape)

    def apply(self, x: Tensor) -> Tensor:
        if x.is_cuda:
            return HipLinearMap.apply(self, x, False)
        return blur_reflect_torch(x, self.taps)

    def apply_transpose(self, y: Tensor) -> Tensor:
        if y.is_cuda:
            return HipLinearMap.apply(self, y, True)
        x = torch.zeros_like(y, requires_grad=True)
        with torch.enable_grad():
            out = blur_reflect_torch(x, self.taps)
            (g,) = torch.autograd.grad(out, x, grad_outputs=y)
        return g

    def hip_descriptor(self) -> _hip.SpOp:
        c, h, w = self.x_shape
        d = _hip.SpOp()
        d.kind = _hip.SP_OP_BLUR
        d.channels, d.height, d.width = c, h, w
        d.n = d.m = int(math.prod(self.x_shape))
        d.taps = self.taps.data_ptr()
        d.radius = self.radius
        return d

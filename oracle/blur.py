"""Reflect-padded separable Gaussian blur — TEST INFRASTRUCTURE ONLY.

The reference has no blur operator.  The semantics the HIP
kernels implement are pinned here by plain torch: ``F.pad(mode="reflect")``
followed by a depthwise 2-D correlation with ``outer(k, k)`` (float64), and
the adjoint by autograd of that map (exact transpose by construction).
"""

from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def taps(kernel_size: int = 9, sigma: float = 3.0) -> np.ndarray:
    r = kernel_size // 2
    i = np.arange(-r, r + 1, dtype=np.float64)
    k = np.exp(-(i**2) / (2.0 * sigma**2))
    return (k / k.sum()).astype(np.float32)


def blur(x: torch.Tensor, k1d: np.ndarray) -> torch.Tensor:
    """Forward map on (..., C, H, W) in float64."""
    k = torch.from_numpy(np.asarray(k1d, dtype=np.float64))
    r = (k.numel() - 1) // 2
    shp = x.shape
    planes = x.to(torch.float64).reshape(-1, 1, shp[-2], shp[-1])
    p = F.pad(planes, (r, r, r, r), mode="reflect")
    w2 = torch.outer(k, k).view(1, 1, 2 * r + 1, 2 * r + 1)
    return F.conv2d(p, w2).reshape(shp)


def blur_adjoint(y: torch.Tensor, k1d: np.ndarray) -> torch.Tensor:
    """A^T y by autograd of the forward map; differentiable in y (create_graph), so
    loops that backpropagate through A^T (PSLD's x_eff) see the exact transpose."""
    x = torch.zeros_like(y, dtype=torch.float64, requires_grad=True)
    with torch.enable_grad():
        out = blur(x, k1d)
        (g,) = torch.autograd.grad(out, x, grad_outputs=y.to(torch.float64),
                                   create_graph=y.requires_grad)
    return g


def blur_ops(shape: tuple, k1d: np.ndarray):
    """(apply, adjoint) on flat (B, n) float64 numpy arrays for oracle.closed_form."""

    def apply(x: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(x.reshape(x.shape[0], *shape))
        return blur(t, k1d).reshape(x.shape[0], -1).numpy()

    def adjoint(y: np.ndarray) -> np.ndarray:
        t = torch.from_numpy(y.reshape(y.shape[0], *shape))
        return blur_adjoint(t, k1d).reshape(y.shape[0], -1).numpy()

    return apply, adjoint

"""numpy fp64 closed form of one fused DPS step — TEST INFRASTRUCTURE ONLY.

SURVEY.md §8a A9 (verified there against the reference to 5.7e-7): with
k = sqrt(1 - acp_t), a = sqrt(acp_t),

    x0 = (x - k eps) / a                 networks/base.py:41-43
    r  = y - A x0                        inverse_problem.py:17-18
    v  = A^T (c r)                       c = 1/sigma^2 (noise.py:77-79) | 2/(rate+1e-3) (:121-123)
    g  = (v - k J^T v) / a               autograd through predict_x0 (dps.py:102-103)
    x' = c_ell x + c_s x0 + std xi + gamma / (||r_b|| + 1e-9) g     dps.py:106-122

``apply`` / ``adjoint`` act on (B, n) float64 arrays.
"""

from __future__ import annotations

from typing import Callable

import numpy as np

Arr = np.ndarray


def residual_pass(x: Arr, eps: Arr, y_rows: Arr, y_div: int, a: float, k: float, gs: float,
                  apply: Callable[[Arr], Arr], adjoint: Callable[[Arr], Arr]) -> tuple[Arr, Arr]:
    """Returns (v, ||r_b||^2) — what ``sp_dps_residual`` computes (its partials summed)."""
    x = x.astype(np.float64)
    eps = eps.astype(np.float64)
    x0 = (x - k * eps) / a
    rows = np.arange(x.shape[0]) // y_div
    r = y_rows.astype(np.float64)[rows] - apply(x0)
    v = adjoint(gs * r)
    return v, (r.reshape(r.shape[0], -1) ** 2).sum(axis=1)


def update_pass(x: Arr, eps: Arr, v: Arr, w: Arr, rsq: Arr, xi: Arr, a: float, k: float,
                c_ell: float, c_s: float, std: float, gamma: float, norm_eps: float = 1e-9) -> Arr:
    """What ``sp_dps_update`` computes."""
    x = x.astype(np.float64)
    eps = eps.astype(np.float64)
    x0 = (x - k * eps) / a
    scale = gamma / (np.sqrt(rsq) + norm_eps)
    g = (v.astype(np.float64) - k * w.astype(np.float64)) / a
    return c_ell * x + c_s * x0 + std * xi.astype(np.float64) + scale.reshape(-1, 1) * g


def identity_ops():
    return (lambda t: t), (lambda t: t)


def inpaint_ops(kept: Arr, n: int):
    kept = np.asarray(kept, dtype=np.int64)

    def apply(x: Arr) -> Arr:
        return x.reshape(x.shape[0], -1)[:, kept]

    def adjoint(y: Arr) -> Arr:
        out = np.zeros((y.shape[0], n), dtype=np.float64)
        out[:, kept] = y
        return out

    return apply, adjoint


def mask_ops(keep: Arr):
    keep = np.asarray(keep, dtype=bool).reshape(-1)

    def apply(x: Arr) -> Arr:
        return np.where(keep[None, :], x.reshape(x.shape[0], -1), 0.0)

    return apply, apply

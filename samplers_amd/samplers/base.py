"""``PosteriorSampler`` base (mirrors ``/root/reference/samplers/samplers/base.py:7-24``)."""

from __future__ import annotations

import functools
import warnings
from abc import ABC

from samplers_amd import _hip
from samplers_amd.dtypes import Shape, Tensor
from samplers_amd.networks.base import EpsilonNetwork, fp32_view, output_dtype


_RECOMPUTE_WARNED = [False]


def _warn_recomputed(count: int) -> None:
    """One warning per process when a solve had to recompute GroupNorm team partials: the
    result is exact, but every such group waited out the spin budget first, so a solve sharing
    the GPU with another process (team members not resident) can run far slower than usual."""
    if count > 0 and not _RECOMPUTE_WARNED[0]:
        _RECOMPUTE_WARNED[0] = True
        warnings.warn(f"single-pass GroupNorm recomputed {count} chunk partials whose team member "
                      "was not resident (exact results; each cost a full spin-wait): is another "
                      "process using this GPU's CUs?  sp_groupnorm_single_pass(0) selects the "
                      "two-pass kernels", RuntimeWarning, stacklevel=3)


def _guarded(call):
    @functools.wraps(call)
    def run(self, *args, **kwargs):
        with _hip.solve_guard() as guard:
            out = call(self, *args, **kwargs)
        self.last_groupnorm_recomputed = guard.recomputed
        _warn_recomputed(guard.recomputed)
        return out

    return run


class PosteriorSampler(ABC):
    """Every subclass's ``__call__`` runs under ``_hip.solve_guard``: after a solve,
    ``last_groupnorm_recomputed`` holds how many single-pass GroupNorm chunk partials were
    recomputed because a team member was not resident (exact either way; a diagnostic)."""

    def __init__(self, network: EpsilonNetwork):
        self._epsilon_network = network

    @property
    def _network(self):
        """The ε-network as the fp32 hot path calls it (``networks.base.fp32_view``: a bf16 /
        fp16 network runs in its dtype behind an fp32 boundary)."""
        return fp32_view(self._epsilon_network)

    def _as_output(self, x: Tensor) -> Tensor:
        """Results are returned in the network's dtype, as the reference's are (its samples
        live in ``epsilon_net.dtype``, ``dps.py:83-87``)."""
        return x.to(output_dtype(self._epsilon_network))

    def __init_subclass__(cls, **kwargs):
        super().__init_subclass__(**kwargs)
        if "__call__" in cls.__dict__:
            cls.__call__ = _guarded(cls.__dict__["__call__"])

    @staticmethod
    def _flatten_leading(x: Tensor, *, x_shape: Shape) -> tuple[Tensor, Shape]:
        batch_shape = x.shape[: -len(x_shape)]
        return x.reshape(-1, *x_shape), batch_shape

    @staticmethod
    def _unflatten_leading(x_flat: Tensor, *, batch_shape: tuple[int, ...]) -> Tensor:
        return x_flat.reshape(*batch_shape, *x_flat.shape[1:])

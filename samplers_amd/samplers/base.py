"""``PosteriorSampler`` base (mirrors ``/root/reference/samplers/samplers/base.py:7-24``)."""

from __future__ import annotations

from abc import ABC

from samplers_amd.dtypes import Shape, Tensor
from samplers_amd.networks.base import EpsilonNetwork


class PosteriorSampler(ABC):
    def __init__(self, network: EpsilonNetwork):
        self._epsilon_network = network

    @staticmethod
    def _flatten_leading(x: Tensor, *, x_shape: Shape) -> tuple[Tensor, Shape]:
        batch_shape = x.shape[: -len(x_shape)]
        return x.reshape(-1, *x_shape), batch_shape

    @staticmethod
    def _unflatten_leading(x_flat: Tensor, *, batch_shape: tuple[int, ...]) -> Tensor:
        return x_flat.reshape(*batch_shape, *x_flat.shape[1:])

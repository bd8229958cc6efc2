"""Identity operator (mirrors ``/root/reference/samplers/operators/identity.py:8-68``)."""

from __future__ import annotations

import math

from samplers_amd import _hip
from samplers_amd.dtypes import Device, Shape, Tensor

from .linear import LinearOperator


class IdentityOperator(LinearOperator):
    """``y = x``; with ``flatten=True`` the sample axes collapse to one."""

    def __init__(self, x_shape: Shape, flatten: bool = False) -> None:
        self.flatten = flatten
        super().__init__(x_shape=x_shape)

    def _infer_y_shape(self, x_shape: Shape, device: Device = None):
        if self.flatten:
            return (int(math.prod(x_shape)),)
        return tuple(x_shape)

    def apply(self, x: Tensor) -> Tensor:
        if self.flatten:
            batch_dims = x.shape[: -len(self.x_shape)]
            return x.reshape(*batch_dims, *self.y_shape)
        return x

    def apply_transpose(self, y: Tensor) -> Tensor:
        if self.flatten:
            batch_dims = y.shape[: -len(self.y_shape)]
            return y.reshape(*batch_dims, *self.x_shape)
        return y

    apply_pseudo_inverse = apply_transpose

    def hip_descriptor(self) -> _hip.SpOp:
        n = int(math.prod(self.x_shape))
        d = _hip.SpOp()
        d.kind = _hip.SP_OP_IDENTITY
        d.channels, d.height, d.width = 1, 1, n
        d.n = d.m = n
        return d

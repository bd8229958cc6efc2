"""Linear and SVD-factored operators (mirrors ``/root/reference/samplers/operators/linear.py``).

``GeneralSVDOperator`` registers its factors *before* the base class infers
``y_shape`` by running ``apply`` — the reference registers them afterwards,
which raises ``AttributeError`` (``linear.py:201-205``); the
assertions of the reference's ``tests/operators/test_linear.py`` hold here.
"""

from __future__ import annotations

from abc import abstractmethod
from typing import Tuple

import torch

from samplers_amd.dtypes import Device, Shape, Tensor

from .base import Operator


class LinearOperator(Operator):
    """Linear forward operator; adjoint / pseudo-inverse optional."""

    def apply_transpose(self, y: Tensor) -> Tensor:
        return super().apply_transpose(y)

    def apply_pseudo_inverse(self, y: Tensor) -> Tensor:
        return super().apply_pseudo_inverse(y)


class SVDOperator(LinearOperator):
    r"""Operator given by a thin SVD ``H = U diag(s) V^T`` (``linear.py:49-183``)."""

    def __init__(self, x_shape: Shape, device: Device = None) -> None:
        super().__init__(x_shape=x_shape, device=device)

    @property
    def shape(self) -> Tuple[int, int]:
        raise NotImplementedError("Subclasses must implement shape property")

    @abstractmethod
    def apply_U(self, z: Tensor) -> Tensor: ...

    @abstractmethod
    def apply_U_transpose(self, y: Tensor) -> Tensor: ...

    @abstractmethod
    def apply_V(self, z: Tensor) -> Tensor: ...

    @abstractmethod
    def apply_V_transpose(self, x: Tensor) -> Tensor: ...

    @abstractmethod
    def get_singular_values(self) -> Tensor: ...

    def apply(self, x: Tensor) -> Tensor:
        z = self.apply_V_transpose(x)
        z = z * self.get_singular_values()
        return self.apply_U(z)

    def apply_transpose(self, y: Tensor) -> Tensor:
        z = self.apply_U_transpose(y)
        z = z * self.get_singular_values()
        return self.apply_V(z)

    def apply_pseudo_inverse(self, y: Tensor) -> Tensor:
        z = self.apply_U_transpose(y)
        s = self.get_singular_values()
        s_inv = torch.zeros_like(s)
        nz = s > 0
        s_inv[nz] = 1.0 / s[nz]
        return self.apply_V(z * s_inv)


class GeneralSVDOperator(SVDOperator):
    """SVD operator with explicit ``U`` (m,k), ``s`` (k,), ``Vh`` (k,n)."""

    def __init__(self, U: Tensor, s: Tensor, Vh: Tensor):
        torch.nn.Module.__init__(self)
        self._m, self._n = U.shape[0], Vh.shape[1]
        self.register_buffer("_U", U)
        self.register_buffer("_singular_values", s)
        self.register_buffer("_V_transpose", Vh)
        self.x_shape = (Vh.shape[1],)
        self.y_shape = self._infer_y_shape(self.x_shape, device=U.device)

    def apply_U(self, x: Tensor) -> Tensor:
        return x @ self._U.t()

    def apply_U_transpose(self, x: Tensor) -> Tensor:
        return x @ self._U

    def apply_V(self, x: Tensor) -> Tensor:
        return x @ self._V_transpose

    def apply_V_transpose(self, x: Tensor) -> Tensor:
        return x @ self._V_transpose.t()

    def get_singular_values(self) -> Tensor:
        return self._singular_values

    @property
    def shape(self) -> Tuple[int, int]:
        return self._m, self._n

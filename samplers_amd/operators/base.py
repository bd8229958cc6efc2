"""Forward-operator plugin API (mirrors ``/root/reference/samplers/operators/base.py:8-113``).

An ``Operator`` is an ``nn.Module`` holding its long-lived tensors as buffers.
Operators that the HIP library implements natively also expose
``hip_descriptor()`` -> :class:`samplers_amd._hip.SpOp`, which the fused DPS
kernels consume; on device tensors their ``apply`` / ``apply_transpose`` run
HIP kernels (differentiable through :class:`HipLinearMap`).  On host tensors
they run plain torch ops — only setup code (shape inference, synthetic
observations) touches that path.
"""

from __future__ import annotations

from abc import ABC, abstractmethod

import torch

from samplers_amd import _hip
from samplers_amd.dtypes import Device, Shape, Tensor


class Operator(torch.nn.Module, ABC):
    """Generic forward model ``A`` (``apply`` mandatory; ``apply_transpose`` and
    ``apply_pseudo_inverse`` optional, raising ``NotImplementedError``)."""

    def __init__(self, x_shape: Shape, device: Device = None) -> None:
        super().__init__()
        self.x_shape = tuple(x_shape)
        self.y_shape = self._infer_y_shape(self.x_shape, device=device)

    def _infer_y_shape(self, x_shape: Shape, device: Device = None) -> Shape:
        """Run a zero batch of one through ``apply`` (reference ``base.py:36-49``)."""
        device = device or next(self.buffers(), torch.tensor(0)).device
        dummy = torch.zeros((1, *x_shape), dtype=torch.float32, device=device)
        with torch.no_grad():
            y = self.apply(dummy)
        return tuple(y.shape[1:])

    @abstractmethod
    def apply(self, x: Tensor) -> Tensor:
        """Forward map ``y = A(x)`` for ``x`` of shape ``(*batch, *x_shape)``."""

    def apply_transpose(self, y: Tensor) -> Tensor:
        raise NotImplementedError("Transpose not defined for this operator")

    def apply_pseudo_inverse(self, y: Tensor) -> Tensor:
        raise NotImplementedError("Pseudo-inverse not defined for this operator")

    def forward(self, x: Tensor) -> Tensor:
        return self.apply(x)

    # --- HIP integration -------------------------------------------------
    def hip_descriptor(self) -> "_hip.SpOp | None":
        """Descriptor for the fused kernels, or ``None`` if the operator has no
        native implementation (the samplers then refuse the fused path)."""
        return None


class NonlinearOperator(Operator):
    """Non-linear degradation operator (``apply`` required; adjoint optional)."""

    @abstractmethod
    def apply(self, x: Tensor) -> Tensor: ...


def _flatten_batch(t: Tensor, sample_shape: Shape) -> tuple[Tensor, tuple[int, ...]]:
    nd = len(sample_shape)
    batch = tuple(t.shape[: t.ndim - nd])
    b = 1
    for s in batch:
        b *= s
    return t.reshape(b, *sample_shape).contiguous(), batch


class HipLinearMap(torch.autograd.Function):
    """Differentiable wrapper around ``sp_op_apply`` / ``sp_op_adjoint``.

    ``forward(op, x, transpose)`` applies A (or A^T); the backward of a linear
    map is its adjoint, so third-party samplers can differentiate through any
    natively implemented operator without leaving HIP.
    """

    @staticmethod
    def forward(ctx, op: Operator, x: Tensor, transpose: bool) -> Tensor:
        ctx.op, ctx.transpose = op, transpose
        return _hip_linear(op, x, transpose)

    @staticmethod
    def backward(ctx, g: Tensor):
        return None, _hip_linear(ctx.op, g.contiguous(), not ctx.transpose), None


def _hip_linear(op: Operator, t: Tensor, transpose: bool) -> Tensor:
    _hip.require_cuda(t, type(op).__name__)
    lib = _hip.load_library()
    desc = op.hip_descriptor()
    in_shape, out_shape = (op.y_shape, op.x_shape) if transpose else (op.x_shape, op.y_shape)
    if t.dtype != torch.float32:
        raise _hip.HipLibraryError(f"{type(op).__name__}: HIP operators compute in fp32")
    flat, batch = _flatten_batch(t, in_shape)
    out = torch.empty((flat.shape[0], *out_shape), device=t.device, dtype=torch.float32)
    if flat.shape[0] > 0:
        fn = lib.sp_op_adjoint if transpose else lib.sp_op_apply
        _hip.check(fn(desc, _hip.ptr(flat), _hip.ptr(out), flat.shape[0], _hip.stream_of(t)),
                   "sp_op_adjoint" if transpose else "sp_op_apply")
    return out.reshape(*batch, *out_shape)

"""Shape bookkeeping ``(*batch, R, *data) <-> (B*R, *data)``.

Same API and semantics as ``/root/reference/samplers/samplers/utils/batch_view.py:8-146``.
"""

from __future__ import annotations

import math
from typing import Sequence, Tuple

import torch
from torch import Tensor


class BatchView:
    """Structured view ``(*batch_shape, num_samples, *data_shape)`` and its flattening
    ``(leading_size, *data_shape)``."""

    def __init__(self, batch_shape: int | Sequence[int] | torch.Size, num_samples: int,
                 data_shape: int | Sequence[int] | torch.Size) -> None:
        self._batch_shape: Tuple[int, ...] = self._to_tuple(batch_shape)
        self._num_samples = int(num_samples)
        self._data_shape: Tuple[int, ...] = self._to_tuple(data_shape)
        self._leading_shape = (*self._batch_shape, self._num_samples)
        self._leading_size = math.prod(self._leading_shape)

    @staticmethod
    def _to_tuple(x) -> Tuple[int, ...]:
        return (x,) if isinstance(x, int) else tuple(int(v) for v in x)

    @property
    def batch_shape(self) -> Tuple[int, ...]:
        return self._batch_shape

    @property
    def batch_size(self) -> int:
        return math.prod(self._batch_shape)

    @property
    def num_samples(self) -> int:
        return self._num_samples

    @property
    def data_shape(self) -> Tuple[int, ...]:
        return self._data_shape

    @property
    def leading_shape(self) -> Tuple[int, ...]:
        return self._leading_shape

    @property
    def leading_size(self) -> int:
        return self._leading_size

    @property
    def flat_shape(self) -> Tuple[int, ...]:
        return (self._leading_size, *self._data_shape)

    @property
    def shape(self) -> Tuple[int, ...]:
        return (*self._leading_shape, *self._data_shape)

    @property
    def per_sample_broadcast_shape(self) -> Tuple[int, ...]:
        return (self._leading_size,) + (1,) * len(self._data_shape)

    def flatten(self, x: Tensor) -> Tensor:
        tail = len(self._data_shape)
        return x.reshape(self._leading_size, *x.shape[-tail:])

    def unflatten(self, x: Tensor) -> Tensor:
        tail = len(self._data_shape)
        return x.reshape(*self._leading_shape, *x.shape[-tail:])

    def repeat_observation(self, observation: Tensor, sample_ndim: int | None = None) -> Tensor:
        """Tile an observation over the sample axis, then flatten.

        ``sample_ndim`` is the rank of one observation; the reference uses the
        data rank (``batch_view.py:128-137``), which breaks for flattened
        observations at batch > 1.  Passing the observation's
        own rank (``len(operator.y_shape)``) gives the intended tiling.
        """
        nd = len(self._data_shape) if sample_ndim is None else sample_ndim
        tail = tuple(observation.shape[observation.ndim - nd:])
        expanded = observation.unsqueeze(len(self._batch_shape)).expand(*self._leading_shape, *tail)
        return expanded.reshape(self._leading_size, *tail)

    def __repr__(self) -> str:
        return (f"{self.__class__.__name__}(batch_shape={self._batch_shape}, "
                f"num_samples={self._num_samples}, data_shape={self._data_shape})")

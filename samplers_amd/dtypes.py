"""Type aliases (mirrors ``/root/reference/samplers/dtypes.py:7-22``)."""

from typing import Sequence, TypeAlias

import torch
from torch import Tensor  # noqa: F401

Shape: TypeAlias = Sequence[int] | torch.Size
Device: TypeAlias = torch.device | str | None
DType: TypeAlias = torch.dtype | None
Scalars: TypeAlias = int | float
TensorLike: TypeAlias = "Tensor | Scalars"
RNG: TypeAlias = torch.Generator | None

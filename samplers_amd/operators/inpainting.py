"""Inpainting / outpainting operators (mirrors ``/root/reference/samplers/operators/inpainting.py``).

Semantics kept bit-for-bit:
  * ``mask`` is True where a pixel is *missing*; non-bool masks become ``mask.ne(0)``
    (``inpainting.py:37-41``); the mask must have exactly ``x_shape``
    (``:43-46``);
  * the observation packs the kept pixels in ascending row-major order,
    ``kept = nonzero(~mask.flatten())`` (``:49-50``), so ``y = x.flat[kept]``;
  * ``flatten=False`` returns the full image with masked pixels zeroed
    (``:106-109``) — constructible here (the reference raises).

For the HIP kernels the kept set is stored as a bit-mask (bit ``j % 64`` of word
``j // 64`` set when pixel ``j`` is observed) plus the observed count before each
word; ``rank(j) = word_rank[j//64] + popcount(lower bits)`` is exactly the
position of ``j`` in ``kept``.  That costs 12 bytes per 64 pixels and stays in L2.
"""

from __future__ import annotations

import numpy as np
import torch

from samplers_amd import _hip
from samplers_amd.dtypes import Device, Shape, Tensor

from .base import HipLinearMap
from .linear import SVDOperator


def keep_bitmask(keep: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """Pack a flat boolean 'observed' vector into (uint64 words, int32 word ranks)."""
    keep = np.ascontiguousarray(keep, dtype=bool).reshape(-1)
    words = (keep.size + 63) // 64
    padded = np.zeros(words * 64, dtype=bool)
    padded[: keep.size] = keep
    bits = np.packbits(padded.reshape(-1, 8), axis=1, bitorder="little").reshape(-1)
    bits = bits.view("<u8").copy()
    counts = padded.reshape(words, 64).sum(axis=1)
    rank = np.zeros(words, dtype=np.int64)
    np.cumsum(counts[:-1], out=rank[1:])
    if keep.size >= 2**31:
        raise ValueError("inpainting mask too large for int32 ranks")
    return bits, rank.astype(np.int32)


class InpaintingOperator(SVDOperator):
    """Keep the observed pixels (``mask`` False) and drop the masked ones."""

    def __init__(self, x_shape: Shape, mask: Tensor, flatten: bool = True, device: Device = None):
        self._x_shape_internal = tuple(x_shape)
        self.flatten = bool(flatten)

        target_device = torch.device(device) if device is not None else mask.device
        mask = mask.to(target_device)
        if mask.dtype != torch.bool:
            mask = mask.ne(0)
        if tuple(mask.shape) != self._x_shape_internal:
            raise ValueError(
                f"Mask shape incompatible with x_shape: {mask.shape} vs. {self._x_shape_internal}."
            )

        flat_mask = mask.flatten()
        kept = torch.nonzero(~flat_mask, as_tuple=False).squeeze(1)
        self._m_dim = kept.numel()
        self._n_dim = flat_mask.numel()
        bits, rank = keep_bitmask((~flat_mask).cpu().numpy())

        torch.nn.Module.__init__(self)
        self.register_buffer("mask", mask)
        self.register_buffer("_kept_indices", kept)
        self.register_buffer(
            "_singular_values", torch.ones(kept.numel(), dtype=torch.float32, device=target_device)
        )
        self.register_buffer("_keep_bits", torch.from_numpy(bits.view(np.int64)).to(target_device))
        self.register_buffer("_word_rank", torch.from_numpy(rank).to(target_device))
        self.x_shape = self._x_shape_internal
        self.y_shape = (self._m_dim,) if self.flatten else self._x_shape_internal

    @staticmethod
    def _expand_kept_indices(batch_dims: tuple[int, ...], idx_1d: Tensor) -> Tensor:
        view_shape = (1,) * len(batch_dims) + (idx_1d.numel(),)
        return idx_1d.view(view_shape).expand(*batch_dims, -1)

    @property
    def shape(self) -> tuple[int, int]:
        return self._m_dim, self._n_dim

    # --- forward / adjoint ------------------------------------------------
    def apply(self, x: Tensor) -> Tensor:
        if x.is_cuda:
            return HipLinearMap.apply(self, x, False)
        if self.flatten:
            return super().apply(x)
        return x.masked_fill(self._batch_mask(x), 0)

    def apply_transpose(self, y: Tensor) -> Tensor:
        if y.is_cuda:
            return HipLinearMap.apply(self, y, True)
        if self.flatten:
            return super().apply_transpose(y)
        return y.masked_fill(self._batch_mask(y), 0)

    apply_pseudo_inverse = apply_transpose

    def _batch_mask(self, t: Tensor) -> Tensor:
        batch_dims = t.shape[: -len(self._x_shape_internal)]
        m = self.mask.view((1,) * len(batch_dims) + self.mask.shape)
        return m.expand(*batch_dims, *self.mask.shape)

    # --- SVD factors (inpainting.py:132-187) --------------------------------
    def apply_V_transpose(self, x: Tensor) -> Tensor:
        if x.is_cuda and self.flatten:
            return HipLinearMap.apply(self, x, False)
        sample_rank = len(self._x_shape_internal)
        batch_dims = x.shape[:-sample_rank]
        x_flat = x.reshape(*batch_dims, -1)
        idx = self._expand_kept_indices(batch_dims, self._kept_indices)
        return x_flat.gather(dim=-1, index=idx)

    def apply_U(self, z: Tensor) -> Tensor:
        return z

    def apply_U_transpose(self, y: Tensor) -> Tensor:
        return y

    def apply_V(self, z_kept: Tensor) -> Tensor:
        if z_kept.is_cuda and self.flatten:
            return HipLinearMap.apply(self, z_kept, True)
        batch_dims = z_kept.shape[:-1]
        flat = torch.zeros(*batch_dims, self._n_dim, device=z_kept.device, dtype=z_kept.dtype)
        idx = self._expand_kept_indices(batch_dims, self._kept_indices)
        flat.scatter_(dim=-1, index=idx, src=z_kept)
        return flat.reshape(*batch_dims, *self._x_shape_internal)

    def get_singular_values(self) -> Tensor:
        return self._singular_values

    # --- HIP ------------------------------------------------------------------
    def hip_descriptor(self) -> _hip.SpOp:
        d = _hip.SpOp()
        d.kind = _hip.SP_OP_INPAINT if self.flatten else _hip.SP_OP_MASK
        d.channels, d.height, d.width = 1, 1, self._n_dim
        d.n = self._n_dim
        d.m = self._m_dim if self.flatten else self._n_dim
        d.keep_bits = self._keep_bits.data_ptr()
        d.word_rank = self._word_rank.data_ptr()
        return d


class CenterInpaintingOperator(InpaintingOperator):
    """Mask out a centred rectangle covering ``paint_fraction`` of each side."""

    def __init__(self, x_shape: Shape, paint_fraction: float = 0.5, device: Device = None):
        if not (0.0 <= paint_fraction <= 1.0):
            raise ValueError("paint_fraction must be in [0, 1]")
        start, end = (1.0 - paint_fraction) / 2.0, (1.0 + paint_fraction) / 2.0
        super().__init__(x_shape, get_mask_inpaint_center(x_shape, start, end, device=device))


class CenterOutpaintingOperator(InpaintingOperator):
    """Keep a centred rectangle covering ``keep_fraction`` of each side."""

    def __init__(self, x_shape: Shape, keep_fraction: float = 0.5, device: Device = None):
        if not (0.0 <= keep_fraction <= 1.0):
            raise ValueError("keep_fraction must be in [0, 1]")
        start, end = (1.0 - keep_fraction) / 2.0, (1.0 + keep_fraction) / 2.0
        super().__init__(x_shape, ~get_mask_inpaint_center(x_shape, start, end, device=device))


class SidePaintingOperator(InpaintingOperator):
    """Mask a vertical slice of ``paint_fraction`` of the width on one side."""

    def __init__(self, x_shape: Shape, paint_fraction: float = 0.5, left: bool = True,
                 device: Device = None):
        if not (0.0 <= paint_fraction <= 1.0):
            raise ValueError("paint_fraction must be in [0, 1]")
        super().__init__(x_shape, get_mask_side_painting(x_shape, paint_fraction, left, device=device))


class RandomInpaintingOperator(InpaintingOperator):
    """Random pixel mask shared by all channels (BASELINE config 2: 50 % random).

    The reference has no helper for it; the mask follows
    SURVEY.md §8d: ``torch.rand(H, W, generator=seed) < fraction`` expanded to
    ``(C, H, W)``.
    """

    def __init__(self, x_shape: Shape, fraction: float = 0.5, seed: int = 1, device: Device = None):
        if not (0.0 <= fraction <= 1.0):
            raise ValueError("fraction must be in [0, 1]")
        super().__init__(x_shape, get_mask_random(x_shape, fraction, seed, device=device))


def get_mask_inpaint_center(image_shape: Shape, start_pct: float = 0.25, end_pct: float = 0.75,
                            device: Device = None) -> Tensor:
    """True inside the centred rectangle [start, end) of H and W (``inpainting.py:269-297``)."""
    if not (0 <= start_pct < end_pct <= 1):
        raise ValueError("start_pct and end_pct must satisfy 0 <= start_pct < end_pct <= 1")
    h, w = image_shape[-2], image_shape[-1]
    sh, eh = int(h * start_pct), int(h * end_pct)
    sw, ew = int(w * start_pct), int(w * end_pct)
    mask = torch.zeros(tuple(image_shape), dtype=torch.bool, device=device)
    mask[..., sh:eh, sw:ew] = True
    return mask


def get_mask_side_painting(image_shape: Shape, pct: float = 0.50, left: bool = True,
                           device: Device = None) -> Tensor:
    """True on the left/right ``pct`` of the width (``inpainting.py:300-330``)."""
    if not (0 < pct <= 1):
        raise ValueError("pct must satisfy 0 < pct <= 1")
    w = image_shape[-1]
    mask_width = int(w * pct)
    mask = torch.zeros(tuple(image_shape), dtype=torch.bool, device=device)
    if left:
        mask[..., :mask_width] = True
    else:
        mask[..., -mask_width:] = True
    return mask


def get_mask_random(image_shape: Shape, fraction: float = 0.5, seed: int = 1,
                    device: Device = None) -> Tensor:
    """True (missing) where ``rand(H, W) < fraction`` for a seeded CPU generator."""
    h, w = image_shape[-2], image_shape[-1]
    gen = torch.Generator().manual_seed(seed)
    m2 = torch.rand(h, w, generator=gen) < fraction
    return m2.expand(tuple(image_shape)).contiguous().to(device)

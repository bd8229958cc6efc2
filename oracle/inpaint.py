"""Inpainting index restatement — TEST INFRASTRUCTURE ONLY.

``kept_indices`` restates ``torch.nonzero(~mask.flatten())`` of
``/root/reference/samplers/operators/inpainting.py:49-50`` with numpy, and
``rank_of`` the bit-mask + prefix-count lookup the HIP kernels use, as an
independent check that both give the same packed order (bit-exact).
"""

from __future__ import annotations

import numpy as np


def kept_indices(mask: np.ndarray) -> np.ndarray:
    """Observed (mask False) flat indices, ascending row-major."""
    return np.flatnonzero(~np.asarray(mask, dtype=bool).reshape(-1)).astype(np.int64)


def rank_of(keep_bits: np.ndarray, word_rank: np.ndarray, j: np.ndarray) -> np.ndarray:
    """Position of element j in the packed observation (valid for observed j)."""
    j = np.asarray(j, dtype=np.int64)
    words = np.asarray(keep_bits).view(np.uint64)[j >> 6]
    sh = (j & 63).astype(np.uint64)
    low = words & ((np.uint64(1) << sh) - np.uint64(1))
    pop = np.array([bin(int(v)).count("1") for v in low], dtype=np.int64)
    return np.asarray(word_rank, dtype=np.int64)[j >> 6] + pop

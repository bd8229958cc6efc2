"""Loading the golden fixtures (tests/golden/*.npz) into ready-to-run cases."""

from __future__ import annotations

import json
from dataclasses import dataclass
from pathlib import Path

import numpy as np
import torch

import stand_ins as si

GOLDEN = Path(__file__).resolve().parent / "golden"


@dataclass
class DpsCase:
    name: str
    meta: dict
    y: torch.Tensor
    out: torch.Tensor
    mask: torch.Tensor | None
    kept: np.ndarray | None

    @property
    def shape(self) -> tuple:
        return tuple(self.meta["shape"])

    @property
    def lead(self) -> int:
        bs = self.meta["batch_shape"]
        return (int(np.prod(bs)) if bs else 1) * self.meta["R"]

    def noise(self):
        shape = tuple(self.meta.get("latent_shape", self.shape))
        return si.replay_noise(self.meta["seed"], (self.lead, *shape), self.meta["N"])

    def observation_rows(self) -> torch.Tensor:
        """y tiled to the flat batch (what the reference's repeat_observation produces)."""
        bs = self.meta["batch_shape"]
        rows = self.y.reshape(int(np.prod(bs)) if bs else 1, -1)
        return rows.repeat_interleave(self.meta["R"], dim=0)


def dps_case_names(prefix: str = "dps") -> list[str]:
    """Fixture names ``{prefix}_*`` (a prefix may itself hold a glob, e.g. ``dps_*_bounded``)."""
    pattern = f"{prefix}.npz" if "*" in prefix else f"{prefix}_*.npz"
    return sorted(p.stem for p in GOLDEN.glob(pattern))


def load_dps_case(name: str) -> DpsCase:
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    mask = torch.from_numpy(z["mask"]) if "mask" in z.files else None
    kept = z["kept"] if "kept" in z.files else None
    return DpsCase(name, meta, torch.from_numpy(z["y"]), torch.from_numpy(z["out"]), mask, kept)

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
        return si.replay_noise(self.meta["seed"], (self.lead, *self.shape), self.meta["N"])


def dps_case_names() -> list[str]:
    return sorted(p.stem for p in GOLDEN.glob("dps_*.npz"))


def load_dps_case(name: str) -> DpsCase:
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    mask = torch.from_numpy(z["mask"]) if "mask" in z.files else None
    kept = z["kept"] if "kept" in z.files else None
    return DpsCase(name, meta, torch.from_numpy(z["y"]), torch.from_numpy(z["out"]), mask, kept)

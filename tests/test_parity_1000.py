"""The 1000-step parity comparison (tools/parity_1000.py::compare) on synthetic trajectories, and the
committed round-6 record it produced (profiles/round6/parity/dps_1000_steps.json)."""
import importlib.util
import json
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]


def _tool():
    spec = importlib.util.spec_from_file_location("parity_1000", ROOT / "tools" / "parity_1000.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _traj(b, gen):
    x = {k: torch.randn(b, 2, 4, 4, generator=gen) for k in (1, 10, 100, 250, 500, 998)}
    return {"checkpoints": x, "x0": torch.randn(b, 2, 4, 4, generator=gen), "seconds": 1.0}


@pytest.mark.parametrize("chaotic", [False, True])
def test_compare_classifies_by_perturbation_growth(tmp_path, monkeypatch, chaotic):
    tool = _tool()
    monkeypatch.setattr(tool, "SHAPE", (2, 4, 4))
    gen = torch.Generator().manual_seed(0)
    rec = tmp_path / "dps_1000_steps.json"
    growth, one = {}, {}
    for case, b in tool.CASES.items():
        c = _traj(b, gen)
        g = {"checkpoints": {k: v * (1 + 1e-6) for k, v in c["checkpoints"].items()}, "x0": c["x0"] * (1 + 1e-6),
             "seconds": 0.1}
        if chaotic and case == "identity":  # late checkpoints decorrelated, as a chaotic map does
            for k in (100, 250, 500, 998):
                g["checkpoints"][k] = torch.randn(b, 2, 4, 4, generator=gen)
            growth[case] = {"1": 1e-6, "250": 1.0, "eps": 1e-6}
            one[case] = {"0": {"gpu_fp32_vs_cpu_fp64": 1e-6}}
        else:
            growth[case] = {"1": 1e-6, "998": 4e-6, "eps": 1e-6}
        torch.save(c, tmp_path / f"cpu_{case}.pt")
        torch.save(g, tmp_path / f"gpu_{case}.pt")
    (tmp_path / "dps_1000_steps_perturb.json").write_text(json.dumps(growth))
    (tmp_path / "dps_1000_steps_onestep-cpu.json").write_text(json.dumps(one))
    res = tool.compare(tmp_path, rec, 1e-3)
    assert res["cases"]["identity"]["chaotic"] is chaotic
    assert res["cases"]["inpaint"]["chaotic"] is False
    assert res["pass"]
    # a chaotic case with no one-step record does not pass
    if chaotic:
        (tmp_path / "dps_1000_steps_onestep-cpu.json").write_text("{}")
        assert not tool.compare(tmp_path, rec, 1e-3)["pass"]


def test_committed_round6_record():
    rec = json.loads((ROOT / "profiles" / "round6" / "parity" / "dps_1000_steps.json").read_text())
    assert rec["pass"] and rec["steps"] == 1000 and rec["tolerance_rel_l2"] == 1e-3
    inp = rec["cases"]["inpaint"]
    assert not inp["chaotic"] and max(inp["sample_rel_l2_after"].values()) < 1e-3 and inp["x0_rel_l2"] < 1e-3
    ide = rec["cases"]["identity"]
    assert ide["chaotic"] and all(v["gpu_fp32_vs_cpu_fp64"] < 1e-5 for v in ide["onestep"].values())

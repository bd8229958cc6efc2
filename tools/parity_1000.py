"""Parity over the length of the real call: 1000-step DPS solves on the GPU vs the oracle loop.

configs[0] and configs[1] are 1000-step DPS solves (``/root/reference/samplers/samplers/dps.py:89-126``:
998 guided iterations of ``:91-122``, then ``:125-126``).  This script pins the whole length:

* ``--phase gpu`` (on the MI355X): ``DPSSampler.__call__`` with N = 1000 and the full
  ddpm-celebahq-256 UNet (random weights, seed 0) for
    - ``identity``: configs[0]'s problem — IdentityOperator, GaussianNoise(σ = 0.05), B = 1;
    - ``inpaint``: configs[1]'s operator — 50 % random inpainting, σ = 0.05, B = 2;
  with injected noise (the initial sample and every step's ξ from a CPU generator seeded by the
  loop index, so the oracle redraws the same values without storing them) and the sample saved
  through ``callback`` after 1, 10, 100, 250, 500 and 998 guided iterations, plus the final x̂.
* ``--phase cpu`` (in the build container, no time limit): ``oracle/dps_loop.py`` with the same
  UNet weights on the CPU, the same observation and noise, the same checkpoints saved.
* ``--phase compare``: relative L2 of every checkpoint, written as JSON (the drift curve).

Test infrastructure: the oracle is the checker here, never the thing measured.
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

STEPS = 1000
CHECKPOINTS = (1, 10, 100, 250, 500, 998)
SHAPE = (3, 256, 256)
CASES = {"identity": 1, "inpaint": 2}  # case -> batch


def noise(i: int, shape) -> torch.Tensor:
    """Standard normals of loop index i (i = -1: the initial sample), from a CPU generator."""
    g = torch.Generator().manual_seed(100_000 + i)
    return torch.randn(tuple(shape), generator=g)


def problem_cpu(case: str):
    """(x_true, y, apply) on the CPU."""
    b = CASES[case]
    g = torch.Generator().manual_seed(11)
    x_true = torch.rand((b, *SHAPE), generator=g) * 2 - 1
    if case == "identity":
        def apply(v):
            return v
    else:
        from samplers_amd.operators import RandomInpaintingOperator

        kept = RandomInpaintingOperator(SHAPE, 0.5, seed=1)._kept_indices.cpu()

        def apply(v):
            return v.reshape(v.shape[0], -1)[:, kept]
    y = apply(x_true)
    y = y + 0.05 * torch.randn(y.shape, generator=torch.Generator().manual_seed(12))
    return x_true, y, apply


def run_gpu(case: str, out: Path) -> None:
    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.networks.ddpm import DDPMNetwork
    from samplers_amd.noise import GaussianNoise
    from samplers_amd.operators import IdentityOperator, RandomInpaintingOperator
    from samplers_amd.samplers import DPSSampler

    dev = torch.device("cuda:0")
    b = CASES[case]
    _, y, _ = problem_cpu(case)
    op = IdentityOperator(SHAPE) if case == "identity" else RandomInpaintingOperator(SHAPE, 0.5, seed=1)
    problem = InverseProblem(op.to(dev), y.to(dev), GaussianNoise(0.05).to(dev))
    net = DDPMNetwork.from_config(seed=0, device=dev)
    seen = {}

    def keep(i, x):
        done = STEPS - i  # i runs STEPS-1 .. 2: guided iterations finished
        if done in CHECKPOINTS:
            seen[done] = x.detach().cpu().clone()
            print(f"[gpu {case}] checkpoint {done}", flush=True)

    fn = lambda k, i, s: noise(-1 if k == "init" else i, s).to(dev)  # noqa: E731
    t0 = time.perf_counter()
    x0 = DPSSampler(net)(problem, num_sampling_steps=STEPS, gamma=1.0, eta=1.0, noise_fn=fn,
                         callback=keep)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    torch.save({"checkpoints": seen, "x0": x0.detach().cpu().reshape(b, *SHAPE), "seconds": dt},
               out / f"gpu_{case}.pt")
    print(f"[gpu {case}] done in {dt:.1f} s", flush=True)


def run_cpu(case: str, out: Path) -> None:
    from oracle import dps_loop
    from samplers_amd.networks.ddpm import DDPMNetwork
    from samplers_amd.networks.unet2d import build_unet

    b = CASES[case]
    _, y, apply = problem_cpu(case)
    net = DDPMNetwork.from_config(seed=0)
    unet = build_unet(seed=0)
    acp = net.alphas_cumprod.cpu()
    ts = net.schedule.set_timesteps(STEPS).flip(0).tolist()
    lp = dps_loop.gaussian_log_prob(0.05)
    eps = lambda v, t: unet(v, t)  # noqa: E731
    sample = noise(-1, (b, *SHAPE))
    done, seen, t0 = 0, {}, time.perf_counter()
    for c in CHECKPOINTS:
        i_cur = STEPS - 1 - done  # the next loop index of dps.py's loop
        sample = dps_loop.dps_reference(eps, acp, ts[:i_cur + 1], apply, lp, y, sample,
                                        lambda i: noise(i, (b, *SHAPE)), gamma=1.0, eta=1.0,
                                        steps_limit=c - done, return_sample=True)
        done = c
        seen[c] = sample.clone()
        print(f"[cpu {case}] checkpoint {c} at {time.perf_counter() - t0:.0f} s", flush=True)
        torch.save({"checkpoints": seen}, out / f"cpu_{case}.partial.pt")
    x0 = dps_loop.dps_reference(eps, acp, ts[:2], apply, lp, y, sample,
                                lambda i: noise(i, (b, *SHAPE)), gamma=1.0, eta=1.0)
    torch.save({"checkpoints": seen, "x0": x0.reshape(b, *SHAPE), "seconds": time.perf_counter() - t0,
                "threads": torch.get_num_threads()}, out / f"cpu_{case}.pt")


def rel(a: torch.Tensor, b: torch.Tensor) -> float:
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float((a - b).norm() / max(b.norm().item(), 1e-30))


def compare(out: Path, record: Path, tol: float) -> dict:
    res = {"tolerance_rel_l2": tol, "steps": STEPS, "guided_iterations": STEPS - 2, "image": list(SHAPE),
           "cases": {}}
    for case, b in CASES.items():
        g, c = torch.load(out / f"gpu_{case}.pt"), torch.load(out / f"cpu_{case}.pt")
        curve = {str(k): rel(g["checkpoints"][k], c["checkpoints"][k]) for k in CHECKPOINTS}
        per_sample = [rel(g["x0"][i], c["x0"][i]) for i in range(b)]
        res["cases"][case] = {"batch": b, "sample_rel_l2_after": curve, "x0_rel_l2": rel(g["x0"], c["x0"]),
                              "x0_rel_l2_per_sample": per_sample,
                              "x0_norm": float(c["x0"].double().norm()),
                              "gpu_seconds": g["seconds"], "cpu_seconds": c["seconds"],
                              "cpu_threads": c.get("threads")}
    res["pass"] = all(v <= tol for cs in res["cases"].values()
                      for v in list(cs["sample_rel_l2_after"].values()) + [cs["x0_rel_l2"]])
    record.parent.mkdir(parents=True, exist_ok=True)
    record.write_text(json.dumps(res, indent=1) + "\n")
    return res


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--phase", choices=("gpu", "cpu", "compare"), required=True)
    ap.add_argument("--case", choices=tuple(CASES) + ("all",), default="all")
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "parity1000"))
    ap.add_argument("--record", default=str(ROOT / "profiles" / "round6" / "parity" / "dps_1000_steps.json"))
    ap.add_argument("--tol", type=float, default=1e-3)
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args()
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    if a.threads:
        torch.set_num_threads(a.threads)
    cases = tuple(CASES) if a.case == "all" else (a.case,)
    if a.phase == "compare":
        res = compare(out, Path(a.record), a.tol)
        print(json.dumps(res, indent=1))
        return 0 if res["pass"] else 1
    for case in cases:
        (run_gpu if a.phase == "gpu" else run_cpu)(case, out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

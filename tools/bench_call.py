"""A whole ``DPSSampler.__call__`` at its defaults (BASELINE configs[0]: identity operator,
GaussianNoise(0.05), the ddpm-celebahq-256 prior, batch 1 on the GPU; ``--config inpaint
--batch 64``: configs[1]), timed end to end — SURVEY.md §8d's metric: B x (N - 2) guided
iterations over the wall time of the call, the final prediction included:

    python tools/bench_call.py [--config identity --batch 1 --steps 1000 --modes default,eager]

Reports the wall time of one call (after an untimed one: MIOpen / allocator warm-up and, on the
default path, the step's hipGraph capture happen inside every call and are included), the time
per guided iteration (``steps - 2`` of them, ``dps.py:90-122``), the execution the default
chose (``DPSSampler.execution``: eager at every batch with the shipped
``GRAPH_AUTO_MAX_BATCH = 0``; ``SAMPLERS_AMD_GRAPH=1`` opts in to hipGraph replay) and the same
call forced eager (``graph=False``).  One JSON line.
"""
from __future__ import annotations

import argparse
import json
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--image", type=int, default=256)
    p.add_argument("--config", choices=("identity", "inpaint", "blur"), default="identity")
    p.add_argument("--modes", default="default,eager", help="default (graph=None), eager and / or graph (forced replay)")
    p.add_argument("--warm-steps", type=int, default=0, help="steps of the untimed call (0: --steps)")
    args = p.parse_args()
    # a long call (configs[1]: ~5 min) prints nothing until it ends: report progress every 30 s
    start = time.perf_counter()

    def heartbeat():
        while True:
            time.sleep(30)
            print(f"[bench_call] {time.perf_counter() - start:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.networks.ddpm import DDPMNetwork
    from samplers_amd.noise import GaussianNoise
    from samplers_amd.operators import GaussianBlurOperator, IdentityOperator, RandomInpaintingOperator
    from samplers_amd.samplers import DPSSampler

    dev = torch.device("cuda:0")
    shape = (3, args.image, args.image)
    gen = torch.Generator().manual_seed(7)
    x_true = torch.rand((args.batch, *shape), generator=gen) * 2 - 1
    op = {"identity": lambda: IdentityOperator(shape),
          "inpaint": lambda: RandomInpaintingOperator(shape, 0.5, seed=1),
          "blur": lambda: GaussianBlurOperator(shape, kernel_size=9, sigma=3.0)}[args.config]().to(dev)
    y = op.apply(x_true.to(dev))
    y = y + (0.05 * torch.randn(tuple(y.shape), generator=gen)).to(dev)
    prob = InverseProblem(op, y, GaussianNoise(0.05).to(dev))
    net = DDPMNetwork.from_config(seed=0, device=dev)
    sampler = DPSSampler(net)
    rec = {"workload": f"DPS + {args.config} + GaussianNoise(0.05), 3x{args.image}², batch {args.batch}, "
                       f"{args.steps}-step schedule ({args.steps - 2} guided iterations), "
                       "ddpm-celebahq-256 architecture (random init)"}
    modes = {"default": {}, "eager": {"graph": False}, "graph": {"graph": True}}
    for label in args.modes.split(","):
        kw = modes[label]
        sampler(prob, num_sampling_steps=args.warm_steps or args.steps, seed=1, **kw)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = sampler(prob, num_sampling_steps=args.steps, seed=1, **kw)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        if not torch.isfinite(out).all():
            raise SystemExit("non-finite result")
        rec[label] = {"execution": sampler.execution, "call_s": round(wall, 4),
                      "ms_per_guided_step": round(wall / (args.steps - 2) * 1e3, 3),
                      "samples_per_s": round(args.batch * (args.steps - 2) / wall, 2)}
        print(f"[bench_call] {label}: {rec[label]}", file=sys.stderr, flush=True)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()

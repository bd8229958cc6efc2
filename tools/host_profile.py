"""Host-side cost of the eager DPS step at a small batch: cProfile over K steps after a warmup
(bench.py's workload and step), per-function self time per step, and the host issue time per
step (the step call returning before the device finishes) against the device step time.

    python tools/host_profile.py [--batch 1] [--config identity] [--steps 10]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--config", default="identity")
    ap.add_argument("--image", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    from samplers_amd import _hip
    from samplers_amd.samplers.dps import FusedDPSStep, initial_sample

    _hip.load_library()
    dev = torch.device("cuda:0")
    problem, net, shape = bench.build_workload(a.config, a.batch, a.image, 0, dev)
    step = FusedDPSStep(net, problem, problem.observation, 1, gamma=1.0, eta=1.0)
    x = initial_sample((a.batch, *shape), dev, rng="philox", seed=1, sample_offset=0, noise_fn=None)
    ts = net.timesteps_host
    it = iter(range(len(ts) - 1, 1, -1))

    def one():
        i = next(it)
        step(x, i, ts[i], ts[i - 1], ts[0], seed=1, sample_offset=0)

    for _ in range(3):
        one()
    torch.cuda.synchronize()
    # host issue time: the call returns once its launches are queued
    issue = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        one()
        issue.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        one()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.steps
    prof = cProfile.Profile()
    prof.enable()
    for _ in range(a.steps):
        one()
    torch.cuda.synchronize()
    prof.disable()
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(40)
    print(f"host issue per step {1e3 * sum(issue) / len(issue):.2f} ms (min {1e3 * min(issue):.2f}); "
          f"pipelined wall per step {1e3 * wall:.2f} ms; cProfile over {a.steps} steps below")
    print(s.getvalue())


if __name__ == "__main__":
    main()

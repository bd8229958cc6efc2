"""bf16 GroupNorm(+SiLU) forward and input VJP (sp_groupnorm_bf16_fwd / _bwd) on the priors' shapes.

    python tools/bench_gn_bf16.py [--reps 10]

One JSON line per shape: ms per call each way and the HBM rate on the bytes the two-pass
kernels move (forward: x read twice, z written = 6 B/elem; VJP: x and dy read twice, dx
written = 10 B/elem), against the 8 TB/s peak.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import samplers_amd  # noqa: E402,F401
from samplers_amd.networks import bf16  # noqa: E402
from samplers_amd.networks.layers import GroupNormAct  # noqa: E402

SHAPES = [(32, 128, 512, 512), (32, 256, 256, 256), (32, 512, 128, 128), (32, 512, 64, 64),
          (32, 320, 64, 64), (32, 640, 32, 32), (32, 1280, 16, 16)]


def timeit(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for n, c, h, w in SHAPES:
        norm = GroupNormAct(32, c, eps=1e-6, act=True).to(dev, torch.bfloat16).requires_grad_(False)
        x = torch.randn(n, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dz = torch.randn_like(x).contiguous(memory_format=torch.channels_last)
        z, st = bf16._gn_fwd_raw(norm, x, None, None)
        fwd = timeit(lambda: bf16._gn_fwd_raw(norm, x, None, None), a.reps)
        bwd = timeit(lambda: bf16._gn_bwd_raw(norm, dz, x, None, None, st), a.reps)
        el = n * c * h * w
        rec = {"shape": [n, c, h, w], "fwd_ms": round(fwd, 4), "bwd_ms": round(bwd, 4),
               "fwd_TBs": round(6 * el / fwd / 1e9, 2), "bwd_TBs": round(10 * el / bwd / 1e9, 2)}
        print(json.dumps(rec), flush=True)
        del x, dz, z


if __name__ == "__main__":
    main()

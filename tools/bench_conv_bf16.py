"""bf16 implicit-GEMM 3x3 convolution (sp_conv3x3_bf16) on the priors' bf16 layer shapes.

    python tools/bench_conv_bf16.py [--reps 10] [--shapes all|sd|vae] [--miopen]

One JSON line per shape: ms per call and TFLOP/s (2*N*Cout*Cin*9*H*W / time) for the HIP tile,
the fraction of the dense bf16 MFMA peak (2516.6 TFLOP/s), and with --miopen the same shape on
F.conv2d (MIOpen, channels-last bf16) for comparison.
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import samplers_amd  # noqa: E402,F401
from samplers_amd import _hip  # noqa: E402
from samplers_amd.networks import bf16  # noqa: E402

PEAK = 2516.6
SD = [(32, 320, 320, 64, 64), (32, 640, 640, 32, 32), (32, 1280, 1280, 16, 16), (32, 1280, 1280, 8, 8),
      (32, 2560, 1280, 8, 8), (32, 960, 320, 64, 64)]
VAE = [(32, 128, 128, 512, 512), (32, 256, 256, 256, 256), (32, 512, 512, 128, 128), (32, 512, 512, 64, 64)]


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
    ap.add_argument("--shapes", default="all")
    ap.add_argument("--miopen", action="store_true")
    a = ap.parse_args()
    shapes = {"sd": SD, "vae": VAE}.get(a.shapes, SD + VAE)
    lib = _hip.load_library()
    dev = torch.device("cuda:0")
    for n, ci, co, h, w in shapes:
        conv = torch.nn.Conv2d(ci, co, 3, padding=1).to(dev, torch.bfloat16).requires_grad_(False)
        x = torch.randn(n, ci, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = torch.empty(n, co, h, w, device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)
        pk = bf16.conv_pack(conv, False)
        bias = conv.bias.float().contiguous()
        s = _hip.stream_of(x)
        nb = int(lib.sp_conv3x3_bf16_workspace(n, ci, co, h, w))
        ws = torch.empty(max(nb // 4, 1), device=dev)

        def run():
            _hip.check(lib.sp_conv3x3_bf16_ws(x.data_ptr(), pk.data_ptr(), bias.data_ptr(), None, n, ci, co, h, w,
                                              y.data_ptr(), ws.data_ptr() if nb else None, nb, s), "sp_conv3x3_bf16_ws")

        ms = timeit(run, a.reps)
        fl = 2.0 * n * co * ci * 9 * h * w
        rec = {"shape": [n, ci, co, h, w], "ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1),
               "frac": round(fl / ms / 1e9 / PEAK, 3), "split_k_bytes": nb}
        if a.miopen:
            ms2 = timeit(lambda: F.conv2d(x, conv.weight, conv.bias, padding=1), a.reps)
            rec["miopen_ms"] = round(ms2, 4)
            rec["miopen_tflops"] = round(fl / ms2 / 1e9, 1)
        print(json.dumps(rec), flush=True)
        del x, y


if __name__ == "__main__":
    main()

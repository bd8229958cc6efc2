"""Downsample2D's stride-2 3x3 conv: csrc/sp_conv_s2.hip tiles vs F.pad + MIOpen, forward and
input VJP, on the UNet's (and the SD VAE encoder's) downsampling shapes.
    python tools/bench_s2.py        (one JSON line per shape)"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from samplers_amd.networks.layers import downsample_conv  # noqa: E402

SHAPES = [(64, 128, 256, 256), (64, 128, 128, 128), (64, 256, 64, 64), (8, 128, 512, 512),
          (8, 256, 256, 256), (8, 512, 128, 128)]


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    dev = torch.device("cuda:0")
    for n, c, h, w in SHAPES:
        conv = torch.nn.Conv2d(c, c, 3, stride=2).to(dev).requires_grad_(False)
        x = torch.randn(n, c, h, w, device=dev, requires_grad=True)
        dy = torch.randn(n, c, h // 2, w // 2, device=dev)
        flops = 18.0 * n * c * c * (h // 2) * (w // 2)
        row = {"shape": [n, c, h, w]}
        for name, f in (("tile", lambda: downsample_conv(conv, x)),
                        ("miopen", lambda: conv(F.pad(x, (0, 1, 0, 1))))):
            with torch.no_grad():
                tf = timed(f)
            y = f()
            tb = timed(lambda: torch.autograd.grad(y, x, dy, retain_graph=True))
            row[name] = {"fwd_us": round(tf * 1e6, 1), "vjp_us": round(tb * 1e6, 1),
                         "fwd_TFLOPs": round(flops / tf / 1e12, 1),
                         "vjp_TFLOPs": round(flops / tb / 1e12, 1)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

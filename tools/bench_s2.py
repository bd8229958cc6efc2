"""Downsample2D's stride-2 3x3 conv: csrc/sp_conv_s2.hip tiles vs F.pad + MIOpen, forward and
input VJP, on the UNet's (and the SD VAE encoder's) downsampling shapes; Upsample2D's 2x
nearest upsampling (csrc/sp_upsample.hip) vs torch on the up blocks' shapes.
    python tools/bench_s2.py [--upsample-only]     (one JSON line per shape)"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from samplers_amd.networks.layers import downsample_conv, upsample_nearest2x  # noqa: E402

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


UP_SHAPES = [(64, 128, 128, 128), (64, 256, 64, 64), (64, 512, 32, 32), (8, 512, 256, 256)]


def upsample_rows(dev):
    for n, c, h, w in UP_SHAPES:
        x = torch.randn(n, c, h, w, device=dev, requires_grad=True)
        dy = torch.randn(n, c, 2 * h, 2 * w, device=dev)
        nbytes = 5 * x.numel() * 4  # read x, write 4x (forward); read 4x, write x (VJP)
        row = {"shape": [n, c, h, w], "op": "upsample2x"}
        for name, f in (("hip", lambda: upsample_nearest2x(x)),
                        ("torch", lambda: F.interpolate(x, scale_factor=2.0, mode="nearest"))):
            with torch.no_grad():
                tf = timed(f)
            y = f()
            tb = timed(lambda: torch.autograd.grad(y, x, dy, retain_graph=True))
            row[name] = {"fwd_us": round(tf * 1e6, 1), "vjp_us": round(tb * 1e6, 1),
                         "fwd_GBps": round(nbytes / tf / 1e9), "vjp_GBps": round(nbytes / tb / 1e9)}
        print(json.dumps(row), flush=True)


def main():
    dev = torch.device("cuda:0")
    upsample_rows(dev)
    if "--upsample-only" in sys.argv:
        return
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

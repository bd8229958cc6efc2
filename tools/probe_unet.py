"""GPU probe: UNet-256 forward + input-VJP cost at several batch sizes / layouts.

Prints one line per configuration (ms per step, sample-steps/s, TFLOP/s, peak GiB).
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from samplers_amd.networks.unet2d import build_unet  # noqa: E402

FLOP_PER_SAMPLE = 992.7e9  # fwd + input-VJP, SURVEY.md §6


def heartbeat(path="gpurun_out/heartbeat.log", every=30):
    import threading

    def beat():
        while True:
            time.sleep(every)
            with open(path, "a") as f:
                f.write(f"{time.time():.0f}\n")

    threading.Thread(target=beat, daemon=True).start()


def run(batch, channels_last=False, dtype=torch.float32, steps=3, bench=False):
    torch.backends.cudnn.benchmark = bench
    net = build_unet(device="cuda", dtype=dtype)
    if channels_last:
        net = net.to(memory_format=torch.channels_last)
    x = torch.randn(batch, 3, 256, 256, device="cuda", dtype=dtype)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    torch.cuda.reset_peak_memory_stats()

    def step():
        xx = x.detach().requires_grad_()
        e = net(xx, 500)
        (g,) = torch.autograd.grad(e, xx, grad_outputs=torch.ones_like(e))
        return g

    t0 = time.time()
    step()
    torch.cuda.synchronize()
    first = time.time() - t0
    print(f"B={batch} first step {first:.1f}s", flush=True)
    t0 = time.time()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.time() - t0) / steps
    peak = torch.cuda.max_memory_allocated() / 2**30
    print(f"B={batch} cl={channels_last} {dtype} first={first:.1f}s step={dt*1e3:.1f}ms "
          f"{batch/dt:.1f} sample-steps/s {batch*FLOP_PER_SAMPLE/dt/1e12:.1f} TFLOP/s peak={peak:.1f}GiB",
          flush=True)
    del net, x
    torch.cuda.empty_cache()


if __name__ == "__main__":
    os.makedirs("gpurun_out", exist_ok=True)
    heartbeat()
    cfgs = sys.argv[1:] or ["8", "64", "64cl", "16bf"]
    for c in cfgs:
        cl = c.endswith("cl")
        bf = c.endswith("bf")
        b = int(c.rstrip("clbf"))
        run(b, channels_last=cl, dtype=torch.bfloat16 if bf else torch.float32)

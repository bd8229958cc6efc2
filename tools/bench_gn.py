"""GroupNorm(+SiLU) forward / input-VJP kernels, two-pass vs single-pass (team), on the
UNet's largest layer shapes:  python tools/bench_gn.py   (one JSON line per shape x mode)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from samplers_amd import _hip  # noqa: E402
from samplers_amd.networks.layers import GroupNormAct, gn_backward, gn_forward  # noqa: E402

SHAPES = [(64, 128, 256, 256), (64, 256, 128, 128), (64, 256, 64, 64), (64, 512, 32, 32)]


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
    lib = _hip.load_library()
    dev = torch.device("cuda:0")
    # the chip's read + write streaming rate on the largest shape: a device-to-device copy
    a = torch.randn(SHAPES[0], device=dev)
    b = torch.empty_like(a)
    tc = timed(lambda: b.copy_(a))
    print(json.dumps({"copy_GBps": round(2 * a.numel() * 4 / tc / 1e9), "bytes": 2 * a.numel() * 4}),
          flush=True)
    del a, b
    for shape in SHAPES:
        n, c, h, w = shape
        layer = GroupNormAct(32, c, eps=1e-6, act=True).to(dev)
        x = torch.randn(shape, device=dev)
        dz = torch.randn(shape, device=dev)
        z, st = gn_forward(layer, x)
        nbytes = x.numel() * 4
        for mode in (0, 1):
            lib.sp_groupnorm_single_pass(mode)
            tf = timed(lambda: gn_forward(layer, x))
            tb = timed(lambda: gn_backward(layer, dz, x, None, None, st))
            rec = {"shape": shape, "single_pass": mode,
                   "fwd_us": round(tf * 1e6, 1), "bwd_us": round(tb * 1e6, 1),
                   "fwd_GBps_min_traffic": round(2 * nbytes / tf / 1e9),
                   "bwd_GBps_min_traffic": round(3 * nbytes / tb / 1e9)}
            if mode == 0:
                # the two-pass kernels one by one: the apply alone is what a forward whose
                # statistics came from the producing convolution's epilogue would cost
                rec["kernels_us"] = kernel_times(lambda: (gn_forward(layer, x),
                                                          gn_backward(layer, dz, x, None, None, st)))
            print(json.dumps(rec), flush=True)
        lib.sp_groupnorm_single_pass(1)


def kernel_times(fn, reps=10):
    """Mean device time per launch of each kernel fn launches (torch profiler)."""
    from torch.profiler import ProfilerActivity, profile

    fn()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
    out = {}
    for ev in prof.key_averages():
        if ev.device_type.name == "CUDA" and ev.count:
            name = ev.key.split("(")[0].replace("void ", "")[:48]
            t = getattr(ev, "device_time_total", None)
            if t is None:
                t = ev.cuda_time_total
            out[name] = round(t / ev.count, 1)
    return out


if __name__ == "__main__":
    main()

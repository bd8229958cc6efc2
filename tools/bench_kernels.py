"""Time the fused DPS passes in isolation (B=64, 3x256x256; BATCH / IMAGE override) for one
library build.

    SAMPLERS_HIP_LIB=build/variants/lib_k8.so python tools/bench_kernels.py [label]

OPS=blur,inpaint restricts the operators; FLUSH=0 times warm-cache launches.

Prints one JSON line per (operator, kernel): mean microseconds over 50 launches
(HIP events on the launch stream) and algorithmic GB/s.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from samplers_amd import _hip  # noqa: E402
from samplers_amd.operators import GaussianBlurOperator, IdentityOperator, RandomInpaintingOperator  # noqa: E402


_FLUSH = None


def timeit(fn, reps=30):
    """Mean launch time with cold caches: 1 GiB is READ between launches so the
    256 MiB Infinity Cache holds none of the operands (as in the sampler, where
    the prior's VJP streams gigabytes between the two passes).  A read, not a
    write: a written flush leaves dirty lines whose write-back lands inside the
    timed launch (measured: a device copy then reads 3.1 instead of ~5 TB/s)."""
    global _FLUSH
    if _FLUSH is None:
        _FLUSH = torch.ones(2**28, device="cuda")
    for _ in range(3):
        fn()
    total = 0.0
    flush = os.environ.get("FLUSH", "1") == "1"
    for _ in range(reps):
        if flush:
            _FLUSH.sum()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        total += e0.elapsed_time(e1)
    return total / reps * 1e3  # us


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else os.environ.get("SAMPLERS_HIP_LIB", "default")
    lib = _hip.load_library()
    dev = torch.device("cuda")
    img = int(os.environ.get("IMAGE", "256"))
    B, shape = int(os.environ.get("BATCH", "64")), (3, img, img)
    n = 3 * img * img
    st = torch.cuda.current_stream().cuda_stream
    # achievable HBM bandwidth reference: device copy of 4 buffers' worth
    src = torch.randn(B, n, device=dev)
    dst = torch.empty_like(src)
    us = timeit(lambda: dst.copy_(src))
    print(json.dumps({"lib": label, "kernel": "torch_copy", "us": round(us, 2),
                      "GB/s": round(2 * src.numel() * 4 / us / 1e3, 1)}), flush=True)
    ops = {"identity": IdentityOperator(shape),
           "inpaint": RandomInpaintingOperator(shape, 0.5, seed=1).to(dev),
           "blur": GaussianBlurOperator(shape, 9, 3.0).to(dev)}
    only = os.environ.get("OPS")
    for name, op in ops.items():
        if only and name not in only.split(","):
            continue
        desc = op.hip_descriptor()
        m = int(desc.m)
        x, eps, w = (torch.randn(B, n, device=dev) for _ in range(3))
        y = torch.randn(B, m, device=dev)
        v = torch.empty_like(x)
        P = lib.sp_rsq_partials(desc)
        part = torch.empty(B, P, device=dev)
        out = torch.empty_like(x)
        c = _hip.SpDpsCoefs(0.5, 0.8, 400.0, 0.9, 0.1, 0.2, 1.0, 1e-9)
        k1 = lambda: lib.sp_dps_residual(desc, x.data_ptr(), eps.data_ptr(), y.data_ptr(), B, 1, c,  # noqa: E731
                                         v.data_ptr(), part.data_ptr(), st)
        needs_v = name == "blur" or os.environ.get("REUSE_V") == "1"
        k2 = lambda: lib.sp_dps_update(desc, x.data_ptr(), eps.data_ptr(), y.data_ptr(),  # noqa: E731
                                       v.data_ptr() if needs_v else None, w.data_ptr(),
                                       part.data_ptr(), None, 7, 3, 0, B, 1, c, out.data_ptr(), st)
        b1 = 4 * (3 * n + m) * B
        b2 = 4 * ((5 if needs_v else 4) * n + (0 if needs_v else m)) * B
        for kname, fn, nb in (("dps_residual", k1, b1), ("dps_update", k2, b2)):
            us = timeit(fn)
            print(json.dumps({"lib": label, "op": name, "kernel": kname, "batch": B, "image": img,
                              "us": round(us, 2),
                              "GB/s": round(nb / us / 1e3, 1), "frac": round(nb / us / 1e3 / 8000, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()

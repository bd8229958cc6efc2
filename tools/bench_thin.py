"""Few-channel 3x3 convolutions (sp_conv3x3_thin_fwd / _bwd_input) on the priors' shapes.

    python tools/bench_thin.py                    # the in-tree library
    SAMPLERS_HIP_LIB=build/variants/lib_thin_v1.so python tools/bench_thin.py

One JSON line per shape and direction: mean µs per call over HIP events, the wide side's
bytes (the few-channel side is small) and the rate on them against the 8 TB/s HBM spec.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from samplers_amd import _hip  # noqa: E402

SHAPES = [  # n, cin, cout, h, w (forward direction); the VJP runs cout -> cin
    (64, 3, 128, 256, 256),    # DDPM UNet conv_in (B = 64, configs[1])
    (64, 128, 3, 256, 256),    # DDPM UNet conv_out
    (32, 3, 128, 512, 512),    # SD VAE encoder conv_in (B = 32, configs[3])
    (32, 128, 3, 512, 512),    # SD VAE decoder conv_out
    (32, 4, 512, 64, 64),      # SD VAE decoder conv_in (latent)
    (32, 512, 8, 64, 64),      # SD VAE encoder conv_out (moments)
]


def timeit(fn, reps=20):
    for _ in range(20):  # ~15 ms: the clock settles before the timed calls
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    lib = _hip.load_library()
    st = torch.cuda.current_stream().cuda_stream
    for n, cin, cout, h, w in SHAPES:
        x = torch.randn(n, cin, h, w, device="cuda")
        wt = torch.randn(cout, cin, 3, 3, device="cuda") * (cin * 9) ** -0.5
        b = torch.randn(cout, device="cuda")
        y = torch.empty(n, cout, h, w, device="cuda")
        dx = torch.empty_like(x)
        fwd = lambda: _hip.check(lib.sp_conv3x3_thin_fwd(x.data_ptr(), wt.data_ptr(), b.data_ptr(), n, cin, cout,  # noqa: E731
                                                         h, w, y.data_ptr(), st), "thin fwd")
        bwd = lambda: _hip.check(lib.sp_conv3x3_thin_bwd_input(y.data_ptr(), wt.data_ptr(), n, cin, cout, h, w,  # noqa: E731
                                                               dx.data_ptr(), st), "thin bwd")
        nbytes = 4.0 * n * h * w * (cin + cout)
        for name, fn in (("fwd", fwd), ("vjp", bwd)):
            us = timeit(fn)
            print(json.dumps({"shape": [n, cin, cout, h, w], "dir": name, "us": round(us, 1),
                              "GB": round(nbytes / 1e9, 3), "TB/s": round(nbytes / us / 1e6, 3),
                              "frac_hbm": round(nbytes / us / 1e6 / 8.0, 3),
                              "lib": os.environ.get("SAMPLERS_HIP_LIB", "in-tree")}), flush=True)


if __name__ == "__main__":
    main()

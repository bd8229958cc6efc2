"""fp32-MFMA 3x3 convolution vs MIOpen on the priors' layer shapes.

    python tools/bench_conv.py

One JSON line per shape and direction: ms per call and TFLOP/s (2*N*Cout*Cin*9*H*W /
time) for the HIP tile (sp_conv3x3_fwd / _bwd_input) and for MIOpen (F.conv2d /
torch.nn.grad.conv2d_input, immediate mode with this project's find-db).
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import samplers_amd  # noqa: E402,F401
from samplers_amd import _hip  # noqa: E402

SHAPES = [  # n, cin, cout, h, w  (UNet B=64 at 256^2 levels; VAE B=32 at 512^2)
    (64, 128, 128, 256, 256),
    (64, 256, 128, 256, 256),
    (64, 256, 256, 128, 128),
    (64, 512, 256, 64, 64),
    (64, 512, 512, 32, 32),
    (32, 128, 128, 512, 512),
    (32, 256, 256, 256, 256),
    (32, 512, 512, 128, 128),
    (32, 512, 512, 64, 64),
]


def timeit(fn, reps=5):
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
    torch.backends.cudnn.benchmark = False
    lib = _hip.load_library()
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    only = os.environ.get("SHAPES")
    shapes = SHAPES
    if os.environ.get("CUSTOM"):  # "n,cin,cout,h,w;n,cin,cout,h,w"
        shapes = [tuple(int(v) for v in c.split(",")) for c in os.environ["CUSTOM"].split(";")]
    for idx, (n, cin, cout, h, w) in enumerate(shapes):
        if only and str(idx) not in only.split(","):
            continue
        flop = 2.0 * n * cout * cin * 9 * h * w
        x = torch.randn(n, cin, h, w, device="cuda")
        wt = torch.randn(cout, cin, 3, 3, device="cuda") * (cin * 9) ** -0.5
        b = torch.randn(cout, device="cuda")
        y = torch.empty(n, cout, h, w, device="cuda")
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        wp = torch.empty(cin * cout * 9, device="cuda")
        wv = torch.empty_like(wp)
        _hip.check(lib.sp_conv3x3_pack(wt.data_ptr(), cout, cin, 0, wp.data_ptr(), st()), "pack")
        if lib.sp_conv3x3_supported(cout, cin, h, w):
            _hip.check(lib.sp_conv3x3_pack(wt.data_ptr(), cout, cin, 1, wv.data_ptr(), st()), "pack")
        up = torch.empty(cin * cout * 16, device="cuda")
        uv = torch.empty_like(up)
        _hip.check(lib.sp_wino3x3_pack(wt.data_ptr(), cout, cin, 0, up.data_ptr(), st()), "pack")
        if lib.sp_wino3x3_supported(cout, cin, h, w):
            _hip.check(lib.sp_wino3x3_pack(wt.data_ptr(), cout, cin, 1, uv.data_ptr(), st()), "pack")
        y2 = torch.empty_like(y)
        rows = {
            "wino_fwd": lambda: lib.sp_wino3x3_fwd(x.data_ptr(), up.data_ptr(), b.data_ptr(), n, cin,
                                                   cout, h, w, y2.data_ptr(), st()),
            "wino_bwd_input": lambda: lib.sp_wino3x3_bwd_input(dy.data_ptr(), uv.data_ptr(), n, cin,
                                                               cout, h, w, dx.data_ptr(), st()),
            "hip_fwd": lambda: lib.sp_conv3x3_fwd(x.data_ptr(), wp.data_ptr(), b.data_ptr(), n, cin,
                                                  cout, h, w, y.data_ptr(), st()),
            "miopen_fwd": lambda: F.conv2d(x, wt, b, padding=1),
            "hip_bwd_input": lambda: lib.sp_conv3x3_bwd_input(dy.data_ptr(), wv.data_ptr(), n, cin,
                                                              cout, h, w, dx.data_ptr(), st()),
            "miopen_bwd_input": lambda: torch.nn.grad.conv2d_input(x.shape, wt, dy, padding=1),
        }
        keep = os.environ.get("ROWS")
        for name, fn in rows.items():
            if keep and name not in keep.split(","):
                continue
            if name in ("hip_bwd_input", "wino_bwd_input") and not lib.sp_conv3x3_supported(cout, cin, h, w):
                continue
            ms = timeit(fn)
            print(json.dumps({"shape": [n, cin, cout, h, w], "kernel": name, "ms": round(ms, 3),
                              "TFLOP/s": round(flop / ms / 1e9, 1)}), flush=True)
        if os.environ.get("ROWS"):
            continue
        ref = F.conv2d(x, wt, b, padding=1)
        lib.sp_conv3x3_fwd(x.data_ptr(), wp.data_ptr(), b.data_ptr(), n, cin, cout, h, w,
                           y.data_ptr(), st())
        err = ((y - ref).norm() / ref.norm()).item()
        lib.sp_wino3x3_fwd(x.data_ptr(), up.data_ptr(), b.data_ptr(), n, cin, cout, h, w,
                           y2.data_ptr(), st())
        err2 = ((y2 - ref).norm() / ref.norm()).item()
        print(json.dumps({"shape": [n, cin, cout, h, w], "hip_vs_miopen_rel_l2": err,
                          "wino_vs_miopen_rel_l2": err2}), flush=True)
        del x, y, dy, dx, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

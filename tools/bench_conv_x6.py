"""The direct 3x3 convolution on the bf16 datapath (csrc/sp_gemm_x6.hip, k_conv3x3_x6) against
the fp32-MFMA Winograd tile (csrc/sp_wino.hip): error vs fp64 and time per call, forward (with
bias + residual) and input VJP.

    python tools/bench_conv_x6.py       (one JSON line per shape; CUSTOM="n,cin,cout,h,w;...")

Error: relative L2 vs a float64 convolution of the first image (CPU); time: HIP events over
5 calls after 2 warm-up calls.  TFLOP/s are direct-convolution FLOPs (2*N*Cin*Cout*9*H*W)."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import samplers_amd  # noqa: E402,F401
from samplers_amd import _hip  # noqa: E402

SHAPES = [  # n, cin, cout, h, w  (the ddpm-celebahq-256 UNet's 3x3 convs at B = 64)
    (64, 128, 128, 256, 256),
    (64, 256, 128, 256, 256),
    (64, 128, 256, 128, 128),
    (64, 256, 256, 128, 128),
    (64, 512, 256, 64, 64),
    (64, 512, 512, 32, 32),
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


def rel(a, b):
    return float((a.double() - b).norm() / b.norm())


def main():
    lib = _hip.load_library()
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    shapes = SHAPES
    if os.environ.get("CUSTOM"):
        shapes = [tuple(int(v) for v in c.split(",")) for c in os.environ["CUSTOM"].split(";")]
    for n, cin, cout, h, w in shapes:
        if not lib.sp_conv3x3_x6_supported(cout, cin, h, w):
            print(json.dumps({"shape": [n, cin, cout, h, w], "skip": "unsupported"}), flush=True)
            continue
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(n, cin, h, w, device="cuda", generator=g)
        wt = torch.randn(cout, cin, 3, 3, device="cuda", generator=g) * (cin * 9) ** -0.5
        b = torch.randn(cout, device="cuda", generator=g)
        res = torch.randn(n, cout, h, w, device="cuda", generator=g)
        dy = torch.randn(n, cout, h, w, device="cuda", generator=g)
        bwd = bool(lib.sp_conv3x3_x6_supported(cin, cout, h, w))
        up = torch.empty(int(lib.sp_wino3x3_packed_size(cin, cout)), device="cuda")
        uv = torch.empty_like(up)
        _hip.check(lib.sp_wino3x3_pack(wt.data_ptr(), cout, cin, 0, up.data_ptr(), st()), "pack")
        _hip.check(lib.sp_wino3x3_pack(wt.data_ptr(), cout, cin, 1, uv.data_ptr(), st()), "pack")
        dp = torch.empty(int(lib.sp_conv3x3_x6_packed_size(cout, cin)), device="cuda")
        _hip.check(lib.sp_conv3x3_x6_pack(wt.data_ptr(), cout, cin, 0, dp.data_ptr(), st()), "pack")
        dv = torch.empty(int(lib.sp_conv3x3_x6_packed_size(cin, cout)), device="cuda") if bwd else None
        if bwd:
            _hip.check(lib.sp_conv3x3_x6_pack(wt.data_ptr(), cin, cout, 1, dv.data_ptr(), st()), "pack")
        y_w, y_d = torch.empty_like(res), torch.empty_like(res)
        dx_w, dx_d = torch.empty_like(x), torch.empty_like(x)
        rows = {
            "wino_fwd": lambda: lib.sp_wino3x3_fwd_res(x.data_ptr(), up.data_ptr(), b.data_ptr(), res.data_ptr(),
                                                       n, cin, cout, h, w, y_w.data_ptr(), st()),
            "x6d_fwd": lambda: lib.sp_conv3x3_x6(x.data_ptr(), dp.data_ptr(), b.data_ptr(), res.data_ptr(),
                                                 n, cin, cout, h, w, y_d.data_ptr(), st()),
            "wino_bwd": lambda: lib.sp_wino3x3_bwd_input(dy.data_ptr(), uv.data_ptr(), n, cin, cout, h, w,
                                                         dx_w.data_ptr(), st()),
            "x6d_bwd": lambda: lib.sp_conv3x3_x6(dy.data_ptr(), dv.data_ptr(), None, None, n, cout, cin, h, w,
                                                 dx_d.data_ptr(), st()),
        }
        out = {"shape": [n, cin, cout, h, w]}
        flop = 2.0 * n * cin * cout * 9 * h * w
        for name, fn in rows.items():
            if name == "x6d_bwd" and not bwd:
                continue
            rc = fn()
            if rc != 0:
                out[name] = f"rc={rc}"
                continue
            ms = timeit(fn)
            out[name + "_ms"] = round(ms, 3)
            out[name + "_tflops"] = round(flop / ms / 1e9, 1)
        torch.cuda.synchronize()
        x0, w64 = x[:1].double().cpu(), wt.double().cpu()
        ref = F.conv2d(x0, w64, b.double().cpu(), padding=1) + res[:1].double().cpu()
        refb = torch.nn.grad.conv2d_input(x0.shape, w64, dy[:1].double().cpu(), padding=1)
        out["err_wino_fwd"] = rel(y_w[:1].cpu(), ref)
        out["err_x6d_fwd"] = rel(y_d[:1].cpu(), ref)
        out["err_wino_bwd"] = rel(dx_w[:1].cpu(), refb)
        if bwd:
            out["err_x6d_bwd"] = rel(dx_d[:1].cpu(), refb)
        print(json.dumps(out), flush=True)
        del x, res, dy, y_w, y_d, dx_w, dx_d
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

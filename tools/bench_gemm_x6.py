"""The bf16x6 1x1-conv GEMM (csrc/sp_gemm_x6.hip) against the torch/hipBLASLt fp32 path of the
UNet's conv_shortcut (networks/unet2d.py: matmul + baddbmm forward, two matmuls for the VJP):
error vs fp64 (first image, CPU) and time per call.

    python tools/bench_gemm_x6.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import samplers_amd  # noqa: E402,F401
from samplers_amd import _hip  # noqa: E402

CASES = [  # n, c1, c2, cout, h, w  (the headline step's shortcut shapes)
    (64, 128, 128, 128, 256, 256),
    (64, 128, 128, 128, 128, 128),
    (64, 256, 128, 256, 64, 64),
    (2, 64, 64, 128, 16, 16),
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
    return float((a.double().cpu() - b).norm() / b.norm())


def main():
    lib = _hip.load_library()
    st = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    pick = os.environ.get("G6_CASES")  # e.g. "0" or "0,2": a subset of CASES (profiling)
    cases = [CASES[int(i)] for i in pick.split(",")] if pick else CASES
    for n, c1, c2, co, h, w in cases:
        hw = h * w
        g = torch.Generator(device="cuda").manual_seed(1)
        x1 = torch.randn(n, c1, h, w, device="cuda", generator=g)
        x2 = torch.randn(n, c2, h, w, device="cuda", generator=g)
        W = torch.randn(co, c1 + c2, device="cuda", generator=g) * (c1 + c2) ** -0.5
        dy = torch.randn(n, co, h, w, device="cuda", generator=g)
        wp = torch.empty(int(lib.sp_gemm_x6_packed_size(co, c1 + c2)), device="cuda")
        wt = torch.empty(int(lib.sp_gemm_x6_packed_size(c1 + c2, co)), device="cuda")
        _hip.check(lib.sp_gemm_x6_pack(W.data_ptr(), co, c1 + c2, 0, wp.data_ptr(), st()), "pack")
        _hip.check(lib.sp_gemm_x6_pack(W.data_ptr(), c1 + c2, co, 1, wt.data_ptr(), st()), "pack")
        y = torch.empty(n, co, h, w, device="cuda")
        d1, d2 = torch.empty_like(x1), torch.empty_like(x2)

        def torch_fwd():
            yy = torch.matmul(W[:, :c1], x1.reshape(n, c1, -1))
            yy.baddbmm_(W[:, c1:].expand(n, co, c2), x2.reshape(n, c2, -1))
            return yy

        def torch_bwd():
            dyv = dy.reshape(n, co, -1)
            return torch.matmul(W[:, :c1].t(), dyv), torch.matmul(W[:, c1:].t(), dyv)

        def x6_fwd():
            return lib.sp_gemm_x6(x1.data_ptr(), c1, x2.data_ptr(), c2, wp.data_ptr(), None, None, n, hw,
                                  y.data_ptr(), co, None, 0, st())

        def x6_bwd():
            return lib.sp_gemm_x6(dy.data_ptr(), co, None, 0, wt.data_ptr(), None, None, n, hw,
                                  d1.data_ptr(), c1, d2.data_ptr(), c2, st())

        out = {"case": [n, c1, c2, co, h, w]}
        for name, fn in (("torch_fwd", torch_fwd), ("x6_fwd", x6_fwd), ("torch_bwd", torch_bwd),
                         ("x6_bwd", x6_bwd)):
            r = fn()
            if isinstance(r, int) and r != 0:
                out[name] = f"rc={r}"
                continue
            out[name + "_ms"] = round(timeit(fn), 3)
        tf, (t1, t2) = torch_fwd(), torch_bwd()
        x6_fwd()
        x6_bwd()
        torch.cuda.synchronize()
        Wd = W.double().cpu()
        ref = torch.einsum("ok,kp->op", Wd, torch.cat([x1[0], x2[0]]).reshape(c1 + c2, -1).double().cpu())
        refb = torch.einsum("ok,op->kp", Wd, dy[0].reshape(co, -1).double().cpu())
        out["err_torch_fwd"] = rel(tf[0], ref)
        out["err_x6_fwd"] = rel(y[0].reshape(co, -1), ref)
        out["err_torch_bwd"] = rel(torch.cat([t1[0], t2[0]]), refb)
        out["err_x6_bwd"] = rel(torch.cat([d1[0], d2[0]]).reshape(c1 + c2, -1), refb)
        print(json.dumps(out), flush=True)
        del x1, x2, dy, y, d1, d2
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

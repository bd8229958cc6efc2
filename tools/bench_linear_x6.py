"""sp_linear_x6 (token-major nn.Linear on the bf16x6 tile) at the SD 1.5 UNet's transformer shapes
(PSLD configs[3]: 32 latents x 64² / 32² tokens) against hipBLASLt fp32 (F.linear): time, TB/s
on the minimal bytes (x read, y written) and executed TFLOP/s (6 bf16 products).

    python tools/bench_linear_x6.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from samplers_amd import _hip  # noqa: E402

CASES = [  # tokens, k, m
    (131072, 320, 960),    # 64²: fused q/k/v
    (131072, 320, 320),    # 64²: to_out, proj_in / proj_out
    (131072, 320, 2560),   # 64²: GEGLU proj
    (131072, 1280, 320),   # 64²: FF out
    (32768, 640, 1920),    # 32²: fused q/k/v
    (32768, 640, 5120),    # 32²: GEGLU proj
    (32768, 2560, 640),    # 32²: FF out
]


def timeit(fn, reps=10):
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
    st = torch.cuda.current_stream().cuda_stream
    for t, k, m in CASES:
        x = torch.randn(t, k, device=dev)
        w = torch.randn(m, k, device=dev) * k ** -0.5
        wp = torch.empty(int(lib.sp_gemm_x6_packed_size(m, k)), device=dev)
        _hip.check(lib.sp_gemm_x6_pack(w.data_ptr(), m, k, 0, wp.data_ptr(), st), "pack")
        y = torch.empty(t, m, device=dev)
        tx6 = timeit(lambda: lib.sp_linear_x6(x.data_ptr(), wp.data_ptr(), None, None, t, k, m, y.data_ptr(), st))
        tbl = timeit(lambda: torch.nn.functional.linear(x, w))
        nbytes = 4 * t * (k + m)
        print(json.dumps({"tokens": t, "k": k, "m": m, "x6_us": round(tx6 * 1e6, 1), "fp32_hipblaslt_us": round(tbl * 1e6, 1),
                          "x6_TBps_min_bytes": round(nbytes / tx6 / 1e12, 2),
                          "x6_exec_TFLOPs": round(12 * t * k * m / tx6 / 1e12, 1)}), flush=True)
        del x, w, wp, y


if __name__ == "__main__":
    main()

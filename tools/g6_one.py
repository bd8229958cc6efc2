"""Run the bf16x6 1x1 GEMM alone (64 x [128+128 -> 128] x 256^2, forward) a few times, for PMC
passes:  rocprofv3 --pmc ... -- python3 tools/g6_one.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from samplers_amd import _hip  # noqa: E402


def main():
    lib = _hip.load_library()
    n, c1, c2, co, hw = 64, 128, 128, 128, 256 * 256
    x1 = torch.randn(n, c1, hw, device="cuda")
    x2 = torch.randn(n, c2, hw, device="cuda")
    W = torch.randn(co, c1 + c2, device="cuda") * 0.06
    wp = torch.empty(int(lib.sp_gemm_x6_packed_size(co, c1 + c2)), device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    _hip.check(lib.sp_gemm_x6_pack(W.data_ptr(), co, c1 + c2, 0, wp.data_ptr(), st), "pack")
    y = torch.empty(n, co, hw, device="cuda")
    for _ in range(4):
        _hip.check(lib.sp_gemm_x6(x1.data_ptr(), c1, x2.data_ptr(), c2, wp.data_ptr(), None, None, n, hw,
                                  y.data_ptr(), co, None, 0, st), "gemm")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

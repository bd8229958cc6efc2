"""Run the direct bf16x6 3x3 conv alone (64 x 128 -> 128 x 256^2, forward with bias + residual) a
few times, for PMC passes:  rocprofv3 --pmc ... -- python3 tools/c6_one.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from samplers_amd import _hip  # noqa: E402


def main():
    lib = _hip.load_library()
    n, cin, cout, h, w = 64, 128, 128, 256, 256
    x = torch.randn(n, cin, h, w, device="cuda")
    W = torch.randn(cout, cin, 3, 3, device="cuda") * 0.03
    b = torch.randn(cout, device="cuda")
    res = torch.randn(n, cout, h, w, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    wp = torch.empty(int(lib.sp_conv3x3_x6_packed_size(cout, cin)), device="cuda")
    _hip.check(lib.sp_conv3x3_x6_pack(W.data_ptr(), cout, cin, 0, wp.data_ptr(), st), "pack")
    y = torch.empty(n, cout, h, w, device="cuda")
    for _ in range(4):
        _hip.check(lib.sp_conv3x3_x6(x.data_ptr(), wp.data_ptr(), b.data_ptr(), res.data_ptr(), n, cin, cout, h, w,
                                     y.data_ptr(), st), "conv")
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

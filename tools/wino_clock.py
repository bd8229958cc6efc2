"""The Winograd tile's forward on one layer shape, launched back to back for about two seconds so
that the clock the chip holds under it settles (MI355X_MICROARCH.md: clock under load), then
the mean time of the last half of the launches.  Run it under tools/sq_pmc.sh
(FILTER=k_wino3x3) for the held clock and MFMA busy per dispatch, or plainly for the time:

    python tools/wino_clock.py [n cin cout h w] [launches]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import samplers_amd  # noqa: E402,F401
from samplers_amd import _hip  # noqa: E402


def main():
    args = [int(a) for a in sys.argv[1:]]
    n, cin, cout, h, w = args[:5] if len(args) >= 5 else (64, 128, 128, 256, 256)
    launches = args[5] if len(args) >= 6 else 800
    lib = _hip.load_library()
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(n, cin, h, w, device="cuda", generator=g)
    wt = torch.randn(cout, cin, 3, 3, device="cuda", generator=g) * (cin * 9) ** -0.5
    b = torch.randn(cout, device="cuda", generator=g)
    y = torch.empty(n, cout, h, w, device="cuda")
    up = torch.empty(cin * cout * 16, device="cuda")
    _hip.check(lib.sp_wino3x3_pack(wt.data_ptr(), cout, cin, 0, up.data_ptr(), st), "pack")
    fwd = lambda: lib.sp_wino3x3_fwd(x.data_ptr(), up.data_ptr(), b.data_ptr(), n, cin, cout, h, w,  # noqa: E731
                                     y.data_ptr(), st)
    half = launches // 2
    for _ in range(half):
        fwd()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(launches - half):
        fwd()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / (launches - half)
    flop = 8.0 * n * cin * cout * h * w  # executed (Winograd F(2,3): 16 products per 4 outputs)
    print(json.dumps({"shape": [n, cin, cout, h, w], "launches": launches, "ms": round(ms, 4),
                      "executed_TFLOP/s": round(flop / ms / 1e9, 1),
                      "lib": os.path.basename(os.environ.get("SAMPLERS_HIP_LIB", "default"))}), flush=True)


if __name__ == "__main__":
    main()

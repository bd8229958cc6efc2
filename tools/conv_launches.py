"""Per-launch times of this project's MFMA conv kernels over one UNet forward + input VJP
(B = 64, 3x256x256): kind, executed GFLOP, ms, TFLOP/s, in launch order.
    python tools/conv_launches.py"""
import ctypes
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from samplers_amd import _hip  # noqa: E402
from samplers_amd.networks.unet2d import build_unet  # noqa: E402

KIND = {3: "conv_fwd", 4: "conv_vjp", 5: "wino_fwd", 6: "wino_vjp"}


def main():
    dev = torch.device("cuda:0")
    lib = _hip.load_library()
    net = build_unet(device=dev)
    x = torch.randn(64, 3, 256, 256, device=dev, requires_grad=True)
    v = torch.randn_like(x)
    t = torch.full((64,), 500, device=dev, dtype=torch.long)

    def step():
        eps = net(x, t)
        return torch.autograd.grad(eps, x, v)

    step()
    torch.cuda.synchronize()
    lib.sp_timing_enable(1)
    step()
    torch.cuda.synchronize()
    n = 4096
    kinds, ms, work = (ctypes.c_int32 * n)(), (ctypes.c_float * n)(), (ctypes.c_double * n)()
    got = lib.sp_timing_collect_work(kinds, ms, work, n)
    lib.sp_timing_enable(0)
    tot = {}
    for i in range(got):
        k = KIND.get(kinds[i])
        if not k:
            continue
        tf = work[i] / (ms[i] * 1e-3) / 1e12
        tot.setdefault(k, [0.0, 0.0])
        tot[k][0] += ms[i]
        tot[k][1] += work[i]
        print(f"{i:4d} {k:9s} {work[i] / 1e9:9.1f} GF {ms[i]:8.3f} ms {tf:7.1f} TF/s")
    for k, (m, w) in tot.items():
        print(f"total {k:9s} {m:8.2f} ms {w / (m * 1e-3) / 1e12:7.1f} TF/s")


if __name__ == "__main__":
    main()

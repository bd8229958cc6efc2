"""GEMM-type ops of one headline DPS step (UNet forward + input VJP at B = 64, 256^2) with their
shapes and device time, from the torch profiler:  python tools/gemm_shapes.py"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import samplers_amd  # noqa: E402,F401
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from samplers_amd.networks.ddpm import DDPMNetwork  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    net = DDPMNetwork.from_config(seed=0, device=dev)
    net.set_sampling_parameters(1000, batch_size=64)
    x = torch.randn(64, 3, 256, 256, device=dev)
    v = torch.randn_like(x)

    def step():
        xr = x.clone().requires_grad_()
        eps = net(xr, 500)
        torch.autograd.grad(eps, xr, v)

    step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    rows = [e for e in prof.key_averages(group_by_input_shape=True)
            if any(k in e.key for k in ("mm", "linear", "addmm", "baddbmm", "matmul"))]
    rows.sort(key=lambda e: -e.device_time_total)
    for e in rows[:25]:
        print(f"{e.device_time_total / 1e3:8.2f} ms  x{e.count:3d}  {e.key:20s} {e.input_shapes}")


if __name__ == "__main__":
    main()

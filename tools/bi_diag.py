"""Diagnostic: the first UNet module whose output differs between a batch of 2 and the same
samples run one at a time, in batch-invariant mode (runtime.batch_invariant)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from samplers_amd.networks.ddpm import DDPMNetwork  # noqa: E402
from samplers_amd.runtime import batch_invariant  # noqa: E402

dev = torch.device("cuda:0")
net = DDPMNetwork.from_config(seed=0, device=dev)
net.set_sampling_parameters(1000, batch_size=2)
x = torch.randn(2, 3, 256, 256, generator=torch.Generator().manual_seed(0)).to(dev)
outs = {}


def hook(name):
    def f(mod, inp, out):
        if isinstance(out, torch.Tensor):
            outs.setdefault(name, []).append(out.detach().clone())
    return f


def bhook(name):
    def f(mod, gin, gout):
        for i, t in enumerate(gin):
            if isinstance(t, torch.Tensor):
                outs.setdefault(f"grad_in[{i}] {name}", []).append(t.detach().clone())
        for i, t in enumerate(gout):
            if isinstance(t, torch.Tensor):
                outs.setdefault(f"grad_out[{i}] {name}", []).append(t.detach().clone())
    return f


for name, mod in net.unet.named_modules():
    if name:
        mod.register_forward_hook(hook(name))
        mod.register_full_backward_hook(bhook(name))
with batch_invariant():
    for run in ("full", "s0", "s1"):
        xr = (x if run == "full" else x[int(run[1]):int(run[1]) + 1]).detach().requires_grad_(True)
        eps = net(xr, 999)
        (g,) = torch.autograd.grad(eps, xr, grad_outputs=torch.ones_like(eps))
        outs.setdefault("__grad__", []).append(g.detach().clone())
        outs.setdefault("__eps__", []).append(eps.detach().clone())
torch.cuda.synchronize()
bad = 0
for name, v in outs.items():
    if len(v) != 3:
        continue
    full, a, b = v
    same = torch.equal(full[:1], a) and torch.equal(full[1:], b)
    if not same:
        d = (full - torch.cat([a, b])).abs().max().item()
        print(f"DIFF {name}: max|d| {d:.3e} shape {tuple(full.shape)}")
        bad += 1
        if bad > 12:
            break
print("modules compared:", len(outs), "differing:", bad)

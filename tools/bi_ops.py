"""Diagnostic: which primitive op of the UNet's 16x16 level gives a batch-dependent result
(batch of 2 vs the same samples one at a time), in batch-invariant mode."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402

from samplers_amd.networks import layers as L  # noqa: E402
from samplers_amd.networks import unet2d as U  # noqa: E402
from samplers_amd.runtime import batch_invariant  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(0)


def check(name, fn, *xs):
    full = fn(*xs)
    parts = [fn(*(x[i:i + 1] if x is not None else None for x in xs)) for i in range(2)]
    full = full[0] if isinstance(full, tuple) else full
    parts = [p[0] if isinstance(p, tuple) else p for p in parts]
    torch.cuda.synchronize()
    ok = torch.equal(full, torch.cat(parts))
    d = (full - torch.cat(parts)).abs().max().item()
    print(f"{'ok  ' if ok else 'DIFF'} {name}: max|d| {d:.3e}", flush=True)


with batch_invariant(), torch.no_grad():
    for (c, co, h) in ((128, 256, 64), (256, 256, 32), (256, 512, 16), (512, 512, 16), (512, 512, 8), (1024, 512, 8), (1024, 512, 16)):
        x = torch.randn(2, c, h, h, generator=g).to(dev)
        norm = L.GroupNormAct(32, c, eps=1e-6, act=True).to(dev)
        check(f"gn {c}x{h}", lambda v: L.gn_forward(norm, v), x)
        conv = L.Conv3x3(c, co).to(dev) if hasattr(L, "Conv3x3") else None
        if conv is not None:
            check(f"conv3x3 {c}->{co} @{h}", lambda v: L.conv3x3_forward(conv, v), x)
            dy = torch.randn(2, co, h, h, generator=g).to(dev)
            check(f"conv3x3 vjp {c}->{co} @{h}", lambda v: L.conv3x3_input_vjp(conv, v, (v.shape[0], c, h, h)), dy)
        sc = torch.nn.Conv2d(c, co, 1).to(dev)
        check(f"shortcut {c}->{co} @{h}", lambda v: U._shortcut_forward(sc, v, None), x)
        dy = torch.randn(2, co, h, h, generator=g).to(dev)
        check(f"shortcut vjp {c}->{co} @{h}", lambda v: U._shortcut_input_vjp(sc, v, c, 0), dy)

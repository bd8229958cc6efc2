"""Locate mismatches between the single-pass and two-pass GroupNorm kernels (debug aid)."""
import sys
import torch
sys.path.insert(0, ".")
from samplers_amd import _hip
from samplers_amd.networks.layers import GroupNormAct, gn_forward, gn_backward

lib = _hip.load_library()
dev = torch.device("cuda:0")
n, c, h, w, g = tuple(int(a) for a in sys.argv[1:6]) if len(sys.argv) > 5 else (2, 256, 128, 128, 32)
gen = torch.Generator().manual_seed(0)
layer = GroupNormAct(g, c, eps=1e-6, act=True).to(dev)
x = (torch.randn(n, c, h, w, generator=gen) * 2 + 0.5).to(dev)
dz = torch.randn(n, c, h, w, generator=gen).to(dev)
res = []
for mode in (0, 1):
    lib.sp_groupnorm_single_pass(mode)
    z, st = gn_forward(layer, x)
    d, _ = gn_backward(layer, dz, x, None, None, st)
    torch.cuda.synchronize()
    res.append((z, st, d))
print("timeouts", lib.sp_groupnorm_team_timeouts())
print("stats equal", torch.equal(res[0][1], res[1][1]), (res[0][1] - res[1][1]).abs().max().item())
for k, name in ((0, "z"), (2, "dx")):
    a, b = res[0][k].reshape(n * g, -1), res[1][k].reshape(n * g, -1)
    bad = (a != b)
    print(name, "bad elements", bad.sum().item(), "of", bad.numel())
    if bad.any():
        idx = bad.nonzero()
        gi = idx[:, 0].unique()
        print(" groups", gi[:20].tolist(), len(gi))
        e = idx[idx[:, 0] == gi[0], 1]
        f4 = e // 4
        chunk = f4 // 2048
        rem = f4 % 2048
        print(" chunks", chunk.unique().tolist())
        print(" tid", (rem % 256).unique()[:20].tolist(), " i", (rem // 256).unique().tolist())
        print(" sample vals", a.flatten()[bad.flatten().nonzero()[:5, 0]].tolist(), b.flatten()[bad.flatten().nonzero()[:5, 0]].tolist())

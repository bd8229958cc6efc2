"""Fused GroupNorm(+bias)(+SiLU) kernels (csrc/sp_groupnorm.hip) against an fp64 torch
reference of the same op (F.group_norm + silu).  Tolerance: |err| <= 2e-5 * max(1, |ref|)
elementwise for the forward, 1e-4 relative-L2 for the VJPs (fp32 accumulation over groups
of up to 2^18 elements)."""

import pytest
import torch

from samplers_amd.networks.layers import GroupNormAct, group_norm_act_torch

pytestmark = pytest.mark.gpu

SHAPES = [  # (n, c, h, w, groups)
    (2, 128, 32, 32, 32),
    (3, 64, 7, 5, 32),       # H*W % 4 != 0: scalar kernels
    (1, 512, 8, 8, 32),
    (2, 256, 128, 128, 32),  # 8 chunks per group
    (1, 64, 256, 256, 32),   # 2^17 elements per group
    (4, 6, 3, 4, 3),
]


def _ref(x, layer, cb, act):
    w = layer.weight.double() if layer.weight is not None else None
    b = layer.bias.double() if layer.bias is not None else None
    return group_norm_act_torch(x.double(), layer.num_groups, w, b, layer.eps, act,
                                None if cb is None else cb.double())


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("act", [True, False])
@pytest.mark.parametrize("with_bias", [True, False])
def test_forward_and_input_vjp(cuda, shape, act, with_bias):
    n, c, h, w, g = shape
    gen = torch.Generator().manual_seed(hash((shape, act, with_bias)) % 2**31)
    x = (torch.randn(n, c, h, w, generator=gen) * 2 + 0.7)
    cb = torch.randn(n, c, generator=gen) if with_bias else None
    layer = GroupNormAct(g, c, eps=1e-6, act=act)
    with torch.no_grad():
        layer.weight.copy_(1 + 0.3 * torch.randn(c, generator=gen))
        layer.bias.copy_(0.2 * torch.randn(c, generator=gen))
    dz = torch.randn(n, c, h, w, generator=gen)

    xd = x.double().requires_grad_()
    ref = _ref(xd, layer, cb, act)
    (gref,) = torch.autograd.grad(ref, xd, dz.double())

    lg = layer.to(cuda)
    xg = x.to(cuda).requires_grad_()
    out = lg(xg, None if cb is None else cb.to(cuda))
    (gx,) = torch.autograd.grad(out, xg, dz.to(cuda))
    err = (out.cpu().double() - ref.detach()).abs() / ref.detach().abs().clamp_min(1.0)
    assert err.max().item() < 2e-5
    assert _rel(gx.cpu(), gref) < 1e-4


def test_bias_and_parameter_grads(cuda):
    n, c, h, w, g = 2, 64, 16, 16, 32
    gen = torch.Generator().manual_seed(7)
    x, cb, dz = torch.randn(n, c, h, w, generator=gen), torch.randn(n, c, generator=gen), torch.randn(n, c, h, w, generator=gen)
    layer = GroupNormAct(g, c, eps=1e-6, act=True).double().requires_grad_(True)
    xd, cbd = x.double().requires_grad_(), cb.double().requires_grad_()
    ref = layer(xd, cbd)  # CPU path = torch
    grads = torch.autograd.grad(ref, (xd, cbd, layer.weight, layer.bias), dz.double())
    lg = GroupNormAct(g, c, eps=1e-6, act=True).to(cuda).requires_grad_(True)
    xg, cbg = x.to(cuda).requires_grad_(), cb.to(cuda).requires_grad_()
    out = lg(xg, cbg)
    got = torch.autograd.grad(out, (xg, cbg, lg.weight, lg.bias), dz.to(cuda))
    for a, b in zip(got, grads):
        assert _rel(a.cpu(), b) < 1e-4


def test_zero_batch_and_constant_groups(cuda):
    layer = GroupNormAct(4, 8, eps=1e-6, act=True).to(cuda)
    assert layer(torch.empty(0, 8, 4, 4, device=cuda)).shape == (0, 8, 4, 4)
    x = torch.full((2, 8, 4, 4), 3.0, device=cuda)  # zero variance: output = silu(beta)
    torch.testing.assert_close(layer(x), torch.nn.functional.silu(layer.bias).view(1, 8, 1, 1).expand(2, 8, 4, 4))


def test_unet_forward_vjp_matches_cpu(cuda):
    """A two-level UNet (all block types) on the GPU (HIP norms, MIOpen convs) vs the
    same weights on the CPU in fp64."""
    from samplers_amd.networks.unet2d import UNet2DConfig, build_unet

    cfg = UNet2DConfig(sample_size=32, block_out_channels=(32, 64), attention_levels=(1,),
                       norm_num_groups=8)
    net = build_unet(cfg, seed=3)
    x = torch.randn(2, 3, 32, 32, generator=torch.Generator().manual_seed(0))
    v = torch.randn_like(x)
    xd = x.double().requires_grad_()
    ref = net.double()(xd, 500)
    (gref,) = torch.autograd.grad(ref, xd, v.double())
    net = net.float().to(cuda)
    xg = x.to(cuda).requires_grad_()
    out = net(xg, 500)
    (gx,) = torch.autograd.grad(out, xg, v.to(cuda))
    assert _rel(out.detach().cpu(), ref.detach()) < 1e-4
    assert _rel(gx.cpu(), gref) < 1e-4


@pytest.mark.parametrize("act", [True, False])
def test_two_part_input_and_addends(cuda, act):
    """sp_groupnorm_silu_fwd2 / bwd2 over cat(x1, x2) read in place (groups straddling the
    split: c1 = 40 is not a multiple of Cg = 12) and the input VJP split into the parts
    plus addends, accumulated in place for one part — against torch on the concatenation."""
    from samplers_amd.networks.layers import gn_backward, gn_forward

    gen = torch.Generator().manual_seed(11)
    n, c1, c2, h, w, g = 3, 40, 56, 12, 20, 8
    x1, x2 = torch.randn(n, c1, h, w, generator=gen), torch.randn(n, c2, h, w, generator=gen)
    dz = torch.randn(n, c1 + c2, h, w, generator=gen)
    a1, a2 = torch.randn(n, c1, h, w, generator=gen), torch.randn(n, c2, h, w, generator=gen)
    layer = GroupNormAct(g, c1 + c2, eps=1e-6, act=act)
    with torch.no_grad():
        layer.weight.uniform_(0.5, 1.5, generator=gen)
        layer.bias.uniform_(-0.5, 0.5, generator=gen)
    xd = torch.cat([x1, x2], 1).double().requires_grad_()
    ref = layer.double()(xd)
    (gref,) = torch.autograd.grad(ref, xd, dz.double())
    lg = layer.float().to(cuda)
    z, st = gn_forward(lg, x1.to(cuda), x2.to(cuda))
    assert _rel(z.cpu(), ref.detach()) < 2e-5
    s2 = a2.to(cuda)
    d1, d2 = gn_backward(lg, dz.to(cuda), x1.to(cuda), x2.to(cuda), None, st,
                         add1=a1.to(cuda), add2=s2, out2=s2)
    assert d2.data_ptr() == s2.data_ptr()
    assert _rel(d1.cpu(), gref[:, :c1] + a1.double()) < 1e-4
    assert _rel(d2.cpu(), gref[:, c1:] + a2.double()) < 1e-4


def test_fused_resnet_blocks_match_cpu(cuda):
    """The UNet with every ResnetBlock as one fused autograd function (GN over cat(h, skip)
    in place, 1x1 shortcuts as GEMMs, the residual in the Winograd epilogue, the
    residual's gradient added inside GN1's backward) against fp64 CPU, forward and input
    VJP, at channel widths / sizes where the Winograd tile serves the 3x3 convs."""
    from samplers_amd.networks.unet2d import UNet2DConfig, build_unet

    cfg = UNet2DConfig(sample_size=64, block_out_channels=(64, 128), attention_levels=(1,),
                       norm_num_groups=32)
    net = build_unet(cfg, seed=5)
    x = torch.randn(2, 3, 64, 64, generator=torch.Generator().manual_seed(1))
    v = torch.randn_like(x)
    xd = x.double().requires_grad_()
    ref = net.double()(xd, 321)
    (gref,) = torch.autograd.grad(ref, xd, v.double())
    net = net.float().to(cuda)
    xg = x.to(cuda).requires_grad_()
    out = net(xg, 321)
    (gx,) = torch.autograd.grad(out, xg, v.to(cuda))
    assert _rel(out.detach().cpu(), ref.detach()) < 1e-4
    assert _rel(gx.cpu(), gref) < 1e-4


@pytest.mark.parametrize("shape", [  # (n, c1, c2, h, w, groups)
    (2, 128, 128, 64, 64, 32),    # 8 channels per group, 4 chunks per group
    (3, 64, 0, 48, 48, 32),       # 2 channels x 2304: one partial chunk
    (2, 128, 0, 256, 256, 32),    # 16 chunks per group
    (5, 256, 256, 8, 8, 32),      # many small groups: several groups per team
    (2, 96, 32, 16, 16, 32),      # c1 % (channels per group) == 0 with a 2-part split
    (1, 256, 128, 128, 128, 32),  # a group straddles the parts at a chunk boundary (UNet 128^2)
])
@pytest.mark.parametrize("act", [True, False])
def test_single_pass_matches_two_pass_bitwise(cuda, shape, act, monkeypatch):
    """The single-pass team kernels (one workgroup per chunk, chunk partials exchanged through
    agent-scope atomics) against the two-pass kernels: same chunking, same summation order,
    so the forward output, statistics and the input VJP agree bit for bit."""
    from samplers_amd import _hip
    from samplers_amd.networks.layers import _team_regions, gn_backward, gn_forward

    lib = _hip.load_library()
    n, c1, c2, h, w, g = shape
    gen = torch.Generator().manual_seed(sum(shape) + act)
    c = c1 + c2
    layer = GroupNormAct(g, c, eps=1e-6, act=act)
    with torch.no_grad():
        layer.weight.copy_(1 + 0.3 * torch.randn(c, generator=gen))
        layer.bias.copy_(0.2 * torch.randn(c, generator=gen))
    layer = layer.to(cuda)
    x1 = (torch.randn(n, c1, h, w, generator=gen) * 2 + 0.5).to(cuda)
    x2 = (torch.randn(n, c2, h, w, generator=gen) - 0.3).to(cuda) if c2 else None
    cb = torch.randn(n, c, generator=gen).to(cuda)
    dz = torch.randn(n, c, h, w, generator=gen).to(cuda)
    a1 = torch.randn(n, c1, h, w, generator=gen).to(cuda)
    a2 = torch.randn(n, c2, h, w, generator=gen).to(cuda) if c2 else None
    outs = []
    prev = lib.sp_groupnorm_single_pass(-1)
    recomputed = 0
    try:
        # two-pass; single-pass; single-pass with a poll bound of 0 (every partial not yet
        # published at the first poll is recomputed by the waiting workgroup: the path that
        # keeps the result exact when a team member is not resident); single-pass again (the
        # caller's team region, layers.gn_team_region, must have been left clean by every launch
        # before, the recomputing ones included); single-pass on the call's zeroed workspace
        # (no team region: SAMPLERS_AMD_GN_TEAM=0)
        for mode, spins, team in ((0, -1, "1"), (1, -1, "1"), (1, 0, "1"), (1, -1, "1"), (1, -1, "0")):
            lib.sp_groupnorm_single_pass(mode)
            monkeypatch.setenv("SAMPLERS_AMD_GN_TEAM", team)
            _hip.check(lib.sp_groupnorm_set_spin_limit(spins), "spin limit")
            before = lib.sp_groupnorm_team_timeouts()
            z, st = gn_forward(layer, x1, x2, cb)
            d1, d2 = gn_backward(layer, dz, x1, x2, cb, st, add1=a1, add2=a2)
            torch.cuda.synchronize()
            outs.append((z, st, d1, d2))
            if spins == 0:
                recomputed = lib.sp_groupnorm_team_timeouts() - before
        assert _team_regions  # the single-pass launches ran on a caller-owned region
        for region in _team_regions.values():
            assert int(region.count_nonzero()) == 0  # every launch left its region zero
    finally:
        lib.sp_groupnorm_single_pass(prev)
        lib.sp_groupnorm_set_spin_limit(-1)
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            if a is None:
                assert b is None
                continue
            assert torch.equal(a, b)
    if (c // g) * h * w > 8192:  # several chunks per group: some partials were late
        assert recomputed > 0


@pytest.mark.parametrize("single", [0, 1])
def test_second_addend_matches_separate_add(cuda, single):
    """add1b (a UNet skip tensor's gradient, added inside the VJP kernel after add1) equals
    the separate add autograd would do, bit for bit, on both kernel paths."""
    from samplers_amd import _hip
    from samplers_amd.networks.layers import gn_backward, gn_forward

    lib = _hip.load_library()
    gen = torch.Generator().manual_seed(21)
    n, c, h, w = 2, 128, 64, 64
    layer = GroupNormAct(32, c, eps=1e-6, act=True).to(cuda)
    x = torch.randn(n, c, h, w, generator=gen).to(cuda)
    dz, a1, a1b = (torch.randn(n, c, h, w, generator=gen).to(cuda) for _ in range(3))
    prev = lib.sp_groupnorm_single_pass(single)
    try:
        _, st = gn_forward(layer, x)
        d_sep, _ = gn_backward(layer, dz, x, None, None, st, add1=a1)
        d_sep = d_sep + a1b
        d_in, _ = gn_backward(layer, dz, x, None, None, st, add1=a1, add1b=a1b)
        torch.cuda.synchronize()
    finally:
        lib.sp_groupnorm_single_pass(prev)
    assert torch.equal(d_in, d_sep)

"""Transformer-block glue of the SD 1.5 ε-UNet on HIP (csrc/sp_transformer.hip, layers.py):
LayerNorm and GEGLU forward / input VJP against fp64 torch, the residual-in-epilogue linear
whose gradient rides into the LayerNorm VJP (``SkipGrad`` box), and a whole
``BasicTransformerBlock`` forward + input VJP against the same module on the CPU (torch fp32).

Tolerances: fp32 rounding of one normalisation / one erf (relative L2 < 2e-6 against fp64);
the whole block (x6 linears, fused attention) 1e-5 relative L2 against CPU fp32."""

import pytest
import torch
import torch.nn.functional as F

from samplers_amd.networks.layers import LayerNorm, Linear, SkipGrad, geglu, layer_norm
from samplers_amd.networks.unet2d_condition import BasicTransformerBlock

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm())


@pytest.mark.parametrize("rows,c", [(256, 320), (1000, 640), (37, 1280), (5, 4), (64, 2048), (0, 320)])
@pytest.mark.parametrize("with_add", [False, True])
def test_layernorm_fwd_vjp(cuda, rows, c, with_add):
    g = torch.Generator().manual_seed(rows + c)
    x = torch.randn(rows, c, generator=g) * 3 + 1.5
    dy = torch.randn(rows, c, generator=g)
    add = torch.randn(rows, c, generator=g) if with_add else None
    mod = LayerNorm(c, eps=1e-6)
    with torch.no_grad():
        mod.weight.copy_(torch.rand(c, generator=g) + 0.5)
        mod.bias.copy_(torch.randn(c, generator=g))
    mod.requires_grad_(False)
    xd = x.double().requires_grad_()
    yd = F.layer_norm(xd, (c,), mod.weight.double(), mod.bias.double(), 1e-6)
    (gd,) = torch.autograd.grad(yd, xd, dy.double())
    if add is not None:
        gd = gd + add.double()

    mg = mod.to(cuda)
    xg = x.to(cuda).requires_grad_()
    box = SkipGrad() if with_add else None
    y = mg(xg, box)
    if box is not None:
        box.grad = add.to(cuda)
    (gx,) = torch.autograd.grad(y, xg, dy.to(cuda))
    if rows == 0:
        assert y.shape == (0, c) and gx.shape == (0, c)
        return
    assert _rel(y, yd) < 2e-6
    assert _rel(gx, gd) < 2e-6


@pytest.mark.parametrize("rows,f", [(256, 1280), (300, 2560), (7, 4)])
def test_geglu_fwd_vjp(cuda, rows, f):
    g = torch.Generator().manual_seed(rows * 7 + f)
    h = torch.randn(rows, 2 * f, generator=g) * 2
    dy = torch.randn(rows, f, generator=g)
    hd = h.double().requires_grad_()
    a, gate = hd.chunk(2, -1)
    yd = a * F.gelu(gate)
    (gd,) = torch.autograd.grad(yd, hd, dy.double())
    hg = h.to(cuda).requires_grad_()
    y = geglu(hg)
    (gh,) = torch.autograd.grad(y, hg, dy.to(cuda))
    assert _rel(y, yd) < 2e-6
    assert _rel(gh, gd) < 2e-6


def test_residual_linear_hands_its_gradient_to_the_norm(cuda, monkeypatch):
    """x + lin(norm(x)) with the residual in lin's epilogue: the x gradient equals autograd's
    sum of the two branches, and the hand-over happened (no separate accumulation).  (The x6
    GEMM serves this small call only with the size rule off: SAMPLERS_AMD_X6_MIN_TILES=0.)"""
    monkeypatch.setenv("SAMPLERS_AMD_X6_MIN_TILES", "0")
    tokens, c = 512, 320
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, tokens // 2, c, generator=g)
    dy = torch.randn(2, tokens // 2, c, generator=g)
    norm = LayerNorm(c).requires_grad_(False)
    lin = Linear(c, c).requires_grad_(False)
    with torch.no_grad():
        lin.weight.copy_(torch.randn(c, c, generator=g) * c ** -0.5)
    xd = x.double().requires_grad_()
    yd = xd + F.linear(F.layer_norm(xd, (c,), norm.weight.double(), norm.bias.double(), norm.eps),
                       lin.weight.double(), lin.bias.double())
    (gd,) = torch.autograd.grad(yd, xd, dy.double())

    norm, lin = norm.to(cuda), lin.to(cuda)
    xg = x.to(cuda).requires_grad_()
    box = SkipGrad()
    y = lin(layer_norm(xg, norm, box), res=xg, box=box)
    assert box.enabled
    (gx,) = torch.autograd.grad(y, xg, dy.to(cuda))
    assert box.grad is None  # taken by the norm's VJP
    assert _rel(y, yd) < 1e-6
    assert _rel(gx, gd) < 1e-6


def _vjp(mod, x, dy, *args):
    xr = x.clone().requires_grad_()
    y = mod(xr, *args)
    (g,) = torch.autograd.grad(y, xr, dy)
    return y.detach(), g


def _check_vs_fp64(mod, x, dy, cuda, *args, what=""):
    """GPU fp32 and CPU fp32 against the same module in fp64 on the CPU: the GPU's relative
    L2 error must be below 1e-5 or within 4x the CPU fp32 error (the module's own fp32
    conditioning, which sharp softmaxes amplify)."""
    import copy

    m64 = copy.deepcopy(mod).double()
    y64, g64 = _vjp(m64, x.double(), dy.double(), *(a.double() for a in args))
    yc, gc = _vjp(mod, x, dy, *args)
    yg, gg = _vjp(copy.deepcopy(mod).to(cuda), x.to(cuda), dy.to(cuda), *(a.to(cuda) for a in args))
    ec = (_rel(yc, y64), _rel(gc, g64))
    eg = (_rel(yg, y64), _rel(gg, g64))
    print(f"{what}: gpu y {eg[0]:.2e} dx {eg[1]:.2e} | cpu fp32 y {ec[0]:.2e} dx {ec[1]:.2e}")
    for e, c in zip(eg, ec):
        assert e < max(1e-5, 4 * c)


@pytest.mark.parametrize("dim,heads,tokens", [(320, 8, 256), (640, 8, 512)])
def test_basic_transformer_block_matches_cpu(cuda, dim, heads, tokens):
    torch.manual_seed(dim)
    blk = BasicTransformerBlock(dim, heads, 768).eval().requires_grad_(False)
    with torch.no_grad():
        for p in blk.parameters():
            p.mul_(3.0)  # bring the random-init branches up to the residual's scale
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, tokens, dim, generator=g)
    ctx = torch.randn(2, 77, 768, generator=g)
    dy = torch.randn(2, tokens, dim, generator=g)
    _check_vs_fp64(blk, x, dy, cuda, ctx, what=f"block dim {dim}")


@pytest.mark.parametrize("in_tm,out_tm", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("n,hw,k,m", [(2, 256, 320, 320), (3, 512, 64, 96)])
def test_gemm_x6_layouts_match_fp64(cuda, in_tm, out_tm, n, hw, k, m):
    from samplers_amd import _hip

    lib = _hip.load_library()
    assert lib.sp_gemm_x6_layout_supported(n, hw, k, m)
    g = torch.Generator().manual_seed(n * hw + k + m)
    x = torch.randn(n, k, hw, generator=g)
    W = torch.randn(m, k, generator=g) * k ** -0.5
    bias = torch.randn(m, generator=g)
    res = torch.randn(n, m, hw, generator=g)
    ref = torch.einsum("ok,nkp->nop", W.double(), x.double()) + bias.double()[None, :, None] + res.double()
    to_tm = lambda t: t.permute(0, 2, 1).contiguous()  # noqa: E731  [n][c][hw] -> [n hw][c]
    xi = to_tm(x) if in_tm else x
    ri = to_tm(res) if out_tm else res
    st = torch.cuda.current_stream().cuda_stream
    wg = W.to(cuda)
    wp = torch.empty(int(lib.sp_gemm_x6_packed_size(m, k)), device=cuda)
    _hip.check(lib.sp_gemm_x6_pack(wg.data_ptr(), m, k, 0, wp.data_ptr(), st), "pack")
    xg, bg, rg = xi.to(cuda), bias.to(cuda), ri.to(cuda)
    y = torch.full(ri.shape, float("nan"), device=cuda)
    _hip.check(lib.sp_gemm_x6_layout(xg.data_ptr(), wp.data_ptr(), bg.data_ptr(), rg.data_ptr(), n, hw, k, m,
                                     in_tm, out_tm, y.data_ptr(), st), "layout")
    got = y.cpu().reshape(n, hw, m).permute(0, 2, 1) if out_tm else y.cpu()
    assert _rel(got, ref) < 1e-6


def test_transformer2d_matches_cpu(cuda):
    from samplers_amd.networks.unet2d_condition import Transformer2DModel

    torch.manual_seed(5)
    mod = Transformer2DModel(320, 8, 768, 32, 1e-6).eval().requires_grad_(False)
    g = torch.Generator().manual_seed(6)
    x = torch.randn(2, 320, 16, 16, generator=g)
    ctx = torch.randn(1, 77, 768, generator=g)
    dy = torch.randn(2, 320, 16, 16, generator=g)
    _check_vs_fp64(mod, x, dy, cuda, ctx, what="Transformer2D")


@pytest.mark.parametrize("d,heads,n", [(40, 8, 512), (80, 4, 512), (160, 2, 1024)])
def test_fused_qkv_attention_matches_fp64(cuda, d, heads, n):
    """Self-attention read straight from the fused projection's [b][n][3 heads d] output and
    its VJP written into one buffer of that layout (no head split / merge copies)."""
    from samplers_amd.networks.attention import fused_qkv_attention

    b, c = 2, heads * d
    g = torch.Generator().manual_seed(d * n + heads)
    qkv = torch.randn(b, n, 3 * c, generator=g)
    dy = torch.randn(b, n, c, generator=g)
    qd = qkv.double().requires_grad_()
    q, k, v = (t.reshape(b, n, heads, d).transpose(1, 2) for t in qd.split(c, -1))
    p = torch.softmax(q @ k.transpose(-1, -2) / d ** 0.5, -1)
    od = (p @ v).transpose(1, 2).reshape(b, n, c)
    (gd,) = torch.autograd.grad(od, qd, dy.double())
    qg = qkv.to(cuda).requires_grad_()
    o = fused_qkv_attention(qg, heads)
    (gg,) = torch.autograd.grad(o, qg, dy.to(cuda))
    eo, eg = _rel(o, od), _rel(gg, gd)
    print(f"fused qkv d={d}: out {eo:.2e} dqkv {eg:.2e}")
    assert eo < 2e-6 and eg < 1e-5


@pytest.mark.parametrize("rows,n", [(64, 4096), (300, 256), (5, 76), (8, 12)])
def test_softmax_rows_and_vjp(cuda, rows, n):
    from samplers_amd import _hip

    lib = _hip.load_library()
    g = torch.Generator().manual_seed(rows + n)
    s = torch.randn(rows, n, generator=g) * 4
    dp = torch.randn(rows, n, generator=g)
    sd = s.double().requires_grad_()
    pd = torch.softmax(sd, -1)
    (gd,) = torch.autograd.grad(pd, sd, dp.double())
    st = torch.cuda.current_stream().cuda_stream
    sg, dg = s.to(cuda), dp.to(cuda)
    lse = torch.empty(rows, device=cuda)
    _hip.check(lib.sp_softmax_rows(sg.data_ptr(), rows, n, lse.data_ptr(), st), "softmax")
    _hip.check(lib.sp_softmax_bwd_rows(sg.data_ptr(), dg.data_ptr(), rows, n, 0.5, st), "softmax bwd")
    assert _rel(sg, pd) < 2e-6
    assert _rel(dg, 0.5 * gd) < 2e-6
    assert _rel(lse, torch.logsumexp(s.double(), -1)) < 1e-6


@pytest.mark.parametrize("c", [4, 8])
def test_conv1x1_small_fwd_vjp(cuda, c):
    from samplers_amd.networks.layers import conv1x1_small

    torch.manual_seed(c)
    conv = torch.nn.Conv2d(c, c, 1).requires_grad_(False)
    x = torch.randn(3, c, 64, 64)
    dy = torch.randn(3, c, 64, 64)
    xd = x.double().requires_grad_()
    yd = F.conv2d(xd, conv.weight.double(), conv.bias.double())
    (gd,) = torch.autograd.grad(yd, xd, dy.double())
    cg = conv.to(cuda)
    xg = x.to(cuda).requires_grad_()
    y = conv1x1_small(cg, xg)
    (gx,) = torch.autograd.grad(y, xg, dy.to(cuda))
    assert _rel(y, yd) < 1e-6 and _rel(gx, gd) < 1e-6


@pytest.mark.parametrize("c,hw,groups,eps", [(512, 64, 32, 1e-6), (256, 16, 32, 1e-6)])
def test_single_head_spatial_attention_matches_cpu(cuda, c, hw, groups, eps):
    """The VAE mid-block / DDPM 16x16 attention: fused qkv projection from NCHW into token
    rows, hipBLASLt score GEMMs with the HIP softmax each way, to_out back to NCHW with the
    residual in its epilogue."""
    from samplers_amd.networks.unet2d import SpatialSelfAttention

    torch.manual_seed(c + hw)
    mod = SpatialSelfAttention(c, groups, eps, None).eval().requires_grad_(False)
    with torch.no_grad():
        for p in mod.parameters():
            p.mul_(2.0)
    g = torch.Generator().manual_seed(2)
    x = torch.randn(2, c, hw, hw, generator=g)
    dy = torch.randn(2, c, hw, hw, generator=g)
    _check_vs_fp64(mod, x, dy, cuda, what=f"spatial attention c={c} {hw}x{hw}")


@pytest.mark.parametrize("d,heads,n,m,bc", [(40, 8, 512, 77, 1), (80, 4, 256, 77, 2), (160, 2, 64, 77, 2),
                                             (40, 2, 128, 5, 1), (160, 1, 128, 130, 1)])
def test_fused_cross_attention_matches_fp64(cuda, d, heads, n, m, bc):
    """Cross-attention of token rows to a context of m keys (one row shared by the batch, or
    one per sample): keys past m masked in the last stage; forward and dq against fp64."""
    from samplers_amd.networks.attention import fused_cross_attention, fused_cross_supported

    b, c = 2, heads * d
    g = torch.Generator().manual_seed(d + n + m + bc)
    q = torch.randn(b, n, c, generator=g)
    k = torch.randn(bc, m, c, generator=g)
    v = torch.randn(bc, m, c, generator=g)
    dy = torch.randn(b, n, c, generator=g)
    qd = q.double().requires_grad_()
    sp = lambda t: t.reshape(t.shape[0], t.shape[1], heads, d).transpose(1, 2)  # noqa: E731
    kd, vd = sp(k.double()).expand(b, -1, -1, -1), sp(v.double()).expand(b, -1, -1, -1)
    p = torch.softmax(sp(qd) @ kd.transpose(-1, -2) / d ** 0.5, -1)
    od = (p @ vd).transpose(1, 2).reshape(b, n, c)
    (gd,) = torch.autograd.grad(od, qd, dy.double())
    qg, kg, vg = q.to(cuda).requires_grad_(), k.to(cuda), v.to(cuda)
    assert fused_cross_supported(qg, kg, heads)
    o = fused_cross_attention(qg, kg, vg, heads)
    (gq,) = torch.autograd.grad(o, qg, dy.to(cuda))
    eo, eg = _rel(o, od), _rel(gq, gd)
    print(f"fused cross d={d} m={m} bc={bc}: out {eo:.2e} dq {eg:.2e}")
    assert eo < 2e-6 and eg < 1e-5

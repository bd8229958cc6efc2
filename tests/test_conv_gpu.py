"""fp32-MFMA 3x3 convolution tiles (csrc/sp_conv.hip direct, csrc/sp_wino.hip Winograd)
against an fp64 torch reference.

The direct tile is an exact-fp32 fmaf chain over K = Cin*9 (v_mfma_f32_32x32x2_f32), so the
tolerance is the fp32 accumulation error: relative L2 <= 2e-6 and max |err| <= 1e-5 x the
largest |output|; the Winograd tile's fp32 transforms add F(2,3) rounding: 5x that."""

import pytest
import torch
import torch.nn.functional as F

from samplers_amd import _hip
from samplers_amd.networks.layers import Conv3x3

pytestmark = pytest.mark.gpu

SHAPES = [  # n, cin, cout, h, w
    (2, 128, 128, 32, 64),
    (1, 4, 512, 8, 32),      # VAE decoder conv_in (forward only on the tile; VJP on MIOpen)
    (2, 384, 128, 16, 32),   # UNet up-block concat input
    (1, 256, 256, 64, 64),
    (3, 132, 256, 8, 96),
]


def _check(got, ref, slack=1):
    """slack 5 for the Winograd tile (its fp32 transforms add F(2,3) rounding)."""
    ref = ref.double()
    rel = ((got.double().cpu() - ref).norm() / ref.norm()).item()
    mx = (got.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert rel < 2e-6 * slack and mx < 1e-5 * slack, (rel, mx)


@pytest.mark.parametrize("backend", ["auto", "direct"])
@pytest.mark.parametrize("shape", SHAPES)
def test_conv3x3_forward_and_input_vjp(cuda, shape, backend, monkeypatch):
    monkeypatch.setenv("SAMPLERS_AMD_CONV", backend)
    n, cin, cout, h, w = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(n, cin, h, w, generator=g)
    conv = Conv3x3(cin, cout)
    with torch.no_grad():
        conv.weight.normal_(0, (cin * 9) ** -0.5, generator=g)
        conv.bias.normal_(0, 0.1, generator=g)
    dy = torch.randn(n, cout, h, w, generator=g)
    xd = x.double().requires_grad_()
    ref = F.conv2d(xd, conv.weight.double(), conv.bias.double(), padding=1)
    (gref,) = torch.autograd.grad(ref, xd, dy.double())

    lib = _hip.load_library()
    assert lib.sp_conv3x3_supported(cin, cout, h, w)
    import os
    wino = os.environ.get("SAMPLERS_AMD_CONV", "auto") == "auto" and lib.sp_wino3x3_supported(cin, cout, h, w)
    cg = conv.to(cuda)
    xg = x.to(cuda).requires_grad_()
    out = cg(xg)
    (gx,) = torch.autograd.grad(out, xg, dy.to(cuda))
    _check(out.detach(), ref.detach(), 5 if wino else 1)
    _check(gx, gref, 5 if wino else 1)


def test_conv3x3_matches_miopen_and_repacks(cuda, monkeypatch):
    conv = Conv3x3(128, 128).to(cuda)
    x = torch.randn(2, 128, 8, 32, device=cuda)
    a = conv(x)
    monkeypatch.setenv("SAMPLERS_AMD_CONV", "miopen")
    b = conv(x)
    torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)
    monkeypatch.setenv("SAMPLERS_AMD_CONV", "auto")
    with torch.no_grad():
        conv.weight.mul_(2)  # in-place update -> packed weights rebuilt
    torch.testing.assert_close(conv(x) - conv.bias.view(1, -1, 1, 1),
                               2 * (a - conv.bias.view(1, -1, 1, 1)), rtol=1e-4, atol=1e-4)


def test_conv3x3_rejects_unsupported(cuda):
    lib = _hip.load_library()
    assert not lib.sp_conv3x3_supported(3, 128, 32, 32)
    assert not lib.sp_conv3x3_supported(128, 64, 32, 32)
    assert not lib.sp_conv3x3_supported(128, 128, 16, 16)
    assert not lib.sp_conv3x3_supported(128, 128, 4, 32)
    conv = Conv3x3(128, 128).to(cuda)  # no direct tile at 16x16: the Winograd tile serves it
    x = torch.randn(1, 128, 16, 16, device=cuda)
    torch.testing.assert_close(conv(x), F.conv2d(x, conv.weight, conv.bias, padding=1))


def test_conv3x3_timing_records_flops(cuda, monkeypatch):
    from samplers_amd.samplers.dps import KernelTimer

    conv = Conv3x3(128, 256).to(cuda)
    x = torch.randn(2, 128, 8, 64, device=cuda, requires_grad=True)
    monkeypatch.setenv("SAMPLERS_AMD_CONV", "direct")
    timer = KernelTimer()
    try:
        out = conv(x)
        torch.autograd.grad(out, x, torch.ones_like(out))
        s = timer.summary()
    finally:
        timer.close()
    flops = 18.0 * 2 * 128 * 256 * 8 * 64
    assert s["conv3x3_fwd"]["count"] == 1 and s["conv3x3_fwd"]["flops"] == flops
    assert s["conv3x3_bwd_input"]["count"] == 1 and s["conv3x3_bwd_input"]["flops"] == flops
    assert 0 < s["conv3x3_fwd"]["ms"] < 100
    monkeypatch.setenv("SAMPLERS_AMD_CONV", "auto")
    timer = KernelTimer()
    try:
        out = conv(x)
        torch.autograd.grad(out, x, torch.ones_like(out))
        s = timer.summary()
    finally:
        timer.close()
    assert s["wino3x3_fwd"]["flops"] == flops * 8 / 18  # executed MFMA work
    assert s["wino3x3_bwd_input"]["count"] == 1


@pytest.mark.parametrize("shape", [(2, 128, 128, 32, 64), (1, 256, 64, 16, 32), (2, 64, 128, 8, 96),
                                   (3, 64, 192, 24, 64), (3, 128, 64, 16, 16), (2, 64, 128, 32, 16),
                                   (1, 512, 512, 16, 16), (3, 64, 128, 8, 8), (5, 512, 512, 8, 8),
                                   (8, 128, 64, 8, 8), (64, 512, 512, 8, 8), (12, 256, 128, 8, 8),
                                   (2, 24, 64, 8, 32), (2, 32, 64, 16, 64), (1, 48, 64, 8, 32)])
def test_winograd_forward_and_input_vjp(cuda, shape):
    """Winograd F(2x2,3x3) tile: fp32 transforms + exact fp32 MFMA accumulation; the
    transforms add F(2,3) rounding, so the bound is 1e-5 relative L2 (vs 2e-6 direct).
    W = 16 shapes run the 4 x 8-tile wave geometry (the UNet's 16x16 level); 8x8 shapes the
    same geometry over two images side by side (batches not a multiple of 4 included).
    cin = 24 / 48 (not a multiple of twice the ξ-split tile's ring): the W % 32 layers' other
    kernel; cin = 32: the ξ-split tile's shortest K (its first and last ring blocks only)."""
    n, cin, cout, h, w = shape
    lib = _hip.load_library()
    assert lib.sp_wino3x3_supported(cin, cout, h, w)
    g = torch.Generator().manual_seed(11 + sum(shape))
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * (cin * 9) ** -0.5
    b = torch.randn(cout, generator=g)
    dy = torch.randn(n, cout, h, w, generator=g)
    xd = x.double().requires_grad_()
    ref = F.conv2d(xd, wt.double(), b.double(), padding=1)
    (gref,) = torch.autograd.grad(ref, xd, dy.double())
    st = torch.cuda.current_stream().cuda_stream
    xg, wg, bg, dyg = x.to(cuda), wt.to(cuda), b.to(cuda), dy.to(cuda)
    up = torch.empty(int(lib.sp_wino3x3_packed_size(cin, cout)), device=cuda)
    uv = torch.empty_like(up)
    _hip.check(lib.sp_wino3x3_pack(wg.data_ptr(), cout, cin, 0, up.data_ptr(), st), "pack")
    y = torch.empty(n, cout, h, w, device=cuda)
    dx = torch.empty_like(xg)
    _hip.check(lib.sp_wino3x3_fwd(xg.data_ptr(), up.data_ptr(), bg.data_ptr(), n, cin, cout, h, w,
                                  y.data_ptr(), st), "wino fwd")
    if lib.sp_wino3x3_supported(cout, cin, h, w):
        _hip.check(lib.sp_wino3x3_pack(wg.data_ptr(), cout, cin, 1, uv.data_ptr(), st), "pack")
        _hip.check(lib.sp_wino3x3_bwd_input(dyg.data_ptr(), uv.data_ptr(), n, cin, cout, h, w,
                                            dx.data_ptr(), st), "wino bwd")
        rel = ((dx.double().cpu() - gref).norm() / gref.norm()).item()
        assert rel < 1e-5, rel
    rel = ((y.double().cpu() - ref.detach()).norm() / ref.detach().norm()).item()
    assert rel < 1e-5, rel


@pytest.mark.parametrize("shape", [(1, 128, 128, 128, 128), (1, 256, 256, 64, 64), (1, 512, 512, 32, 32),
                                   (1, 512, 512, 16, 16), (1, 512, 512, 8, 8), (3, 256, 128, 8, 8),
                                   (2, 64, 128, 32, 64)])
def test_winograd_split_k_workspace(cuda, shape):
    """Split-K (round 4): the small-batch / low-resolution launches cut K into 2-32 parts whose
    partial outputs go to a workspace and are summed in a fixed order with the bias and the
    residual.  Forward (bias + residual) and input VJP against fp64, bitwise-repeatable, and
    equal to the unsplit launch to fp32 rounding."""
    n, cin, cout, h, w = shape
    lib = _hip.load_library()
    ws_f = int(lib.sp_wino3x3_workspace(n, cin, cout, h, w))
    ws_b = int(lib.sp_wino3x3_workspace(n, cout, cin, h, w))
    assert ws_f > 0  # every shape here under-fills the chip unsplit
    g = torch.Generator().manual_seed(41 + sum(shape))
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * (cin * 9) ** -0.5
    b = torch.randn(cout, generator=g)
    res = torch.randn(n, cout, h, w, generator=g)
    dy = torch.randn(n, cout, h, w, generator=g)
    xd = x.double().requires_grad_()
    ref = F.conv2d(xd, wt.double(), b.double(), padding=1)
    (gref,) = torch.autograd.grad(ref, xd, dy.double())
    ref = ref.detach() + res.double()
    st = torch.cuda.current_stream().cuda_stream
    xg, wg, bg, rg, dyg = x.to(cuda), wt.to(cuda), b.to(cuda), res.to(cuda), dy.to(cuda)
    up = torch.empty(int(lib.sp_wino3x3_packed_size(cin, cout)), device=cuda)
    uv = torch.empty_like(up)
    _hip.check(lib.sp_wino3x3_pack(wg.data_ptr(), cout, cin, 0, up.data_ptr(), st), "pack")
    _hip.check(lib.sp_wino3x3_pack(wg.data_ptr(), cout, cin, 1, uv.data_ptr(), st), "pack")

    def fwd(ws_bytes):
        y = torch.empty(n, cout, h, w, device=cuda)
        ws = torch.full((max(ws_bytes, 4) // 4,), float("nan"), device=cuda)  # NaN: unread parts show
        _hip.check(lib.sp_wino3x3_fwd_ws(xg.data_ptr(), up.data_ptr(), bg.data_ptr(), rg.data_ptr(), n, cin,
                                         cout, h, w, y.data_ptr(), ws.data_ptr() if ws_bytes else None,
                                         ws_bytes, st), "wino fwd ws")
        return y

    def vjp(ws_bytes):
        dx = torch.empty(n, cin, h, w, device=cuda)
        ws = torch.full((max(ws_bytes, 4) // 4,), float("nan"), device=cuda)
        _hip.check(lib.sp_wino3x3_bwd_input_ws(dyg.data_ptr(), uv.data_ptr(), n, cin, cout, h, w,
                                               dx.data_ptr(), ws.data_ptr() if ws_bytes else None,
                                               ws_bytes, st), "wino vjp ws")
        return dx

    y1, y2, y0 = fwd(ws_f), fwd(ws_f), fwd(0)
    assert torch.equal(y1, y2)
    assert ((y1.double().cpu() - ref).norm() / ref.norm()).item() < 1e-5
    assert ((y1 - y0).norm() / y0.norm()).item() < 1e-6
    d1, d2, d0 = vjp(ws_b), vjp(ws_b), vjp(0)
    assert torch.equal(d1, d2)
    assert ((d1.double().cpu() - gref).norm() / gref.norm()).item() < 1e-5
    assert ((d1 - d0).norm() / d0.norm()).item() < 1e-6


def test_winograd_residual_epilogue(cuda):
    """sp_wino3x3_fwd_res = sp_wino3x3_fwd + res, exactly (the add happens once, in fp32)."""
    from samplers_amd.networks.layers import Conv3x3, conv3x3_forward

    torch.manual_seed(3)
    conv = Conv3x3(64, 128).to(cuda).requires_grad_(False)
    x = torch.randn(2, 64, 16, 64, device=cuda)
    res = torch.randn(2, 128, 16, 64, device=cuda)
    y = conv3x3_forward(conv, x)
    yr = conv3x3_forward(conv, x, res=res)
    assert torch.equal(yr, y + res)
    x16 = torch.randn(2, 64, 16, 16, device=cuda)  # the W = 16 geometry
    r16 = torch.randn(2, 128, 16, 16, device=cuda)
    assert torch.equal(conv3x3_forward(conv, x16, res=r16), conv3x3_forward(conv, x16) + r16)
    x8 = torch.randn(3, 64, 8, 8, device=cuda)  # the two-image mosaic geometry
    r8 = torch.randn(3, 128, 8, 8, device=cuda)
    # 8x8 images split K over two workgroups (few tiles): the residual joins part 0's partial
    # before part 1's is added, so the match is to fp32 rounding rather than bitwise
    torch.testing.assert_close(conv3x3_forward(conv, x8, res=r8), conv3x3_forward(conv, x8) + r8,
                               rtol=1e-6, atol=1e-6)


def test_winograd_split_k_deterministic(cuda):
    """The 8x8 level's split-K tile adds two partials atomically into a zeroed output; with
    two addends the result does not depend on their order, so repeated launches agree bitwise."""
    from samplers_amd.networks.layers import Conv3x3, conv3x3_forward, conv3x3_input_vjp

    torch.manual_seed(4)
    conv = Conv3x3(512, 512).to(cuda).requires_grad_(False)
    x = torch.randn(64, 512, 8, 8, device=cuda)
    ys = [conv3x3_forward(conv, x) for _ in range(3)]
    gs = [conv3x3_input_vjp(conv, x, x.shape) for _ in range(3)]
    assert all(torch.equal(ys[0], y) for y in ys[1:])
    assert all(torch.equal(gs[0], g) for g in gs[1:])


@pytest.mark.parametrize("shape", [(2, 3, 128, 32, 64), (3, 128, 3, 40, 68), (1, 4, 512, 16, 16),
                                   (2, 512, 8, 16, 16), (2, 256, 4, 8, 12)])
def test_thin_conv_forward_and_input_vjp(cuda, shape):
    """The few-channel 3x3 kernel (conv_in / conv_out of the priors): forward with bias and
    input VJP (transposed, flipped weights read in place) against fp64, ragged tiles
    (H % 8, W % 64 != 0) included; fp32 accumulation, 2e-6 relative L2.  Rows are staged as
    float4 pieces, so W % 4 == 0 is required."""
    n, cin, cout, h, w = shape
    lib = _hip.load_library()
    assert lib.sp_conv3x3_thin_supported(cin, cout, h, w)
    assert lib.sp_conv3x3_thin_supported(cout, cin, h, w)
    assert not lib.sp_conv3x3_thin_supported(cin, cout, h, w + 2)
    g = torch.Generator().manual_seed(5 + sum(shape))
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) * (cin * 9) ** -0.5
    b = torch.randn(cout, generator=g)
    dy = torch.randn(n, cout, h, w, generator=g)
    xd = x.double().requires_grad_()
    ref = F.conv2d(xd, wt.double(), b.double(), padding=1)
    (gref,) = torch.autograd.grad(ref, xd, dy.double())
    st = torch.cuda.current_stream().cuda_stream
    xg, wg, bg, dyg = x.to(cuda), wt.to(cuda), b.to(cuda), dy.to(cuda)
    y = torch.full((n, cout, h, w), float("nan"), device=cuda)
    dx = torch.full_like(xg, float("nan"))
    _hip.check(lib.sp_conv3x3_thin_fwd(xg.data_ptr(), wg.data_ptr(), bg.data_ptr(), n, cin, cout, h, w,
                                       y.data_ptr(), st), "thin fwd")
    _hip.check(lib.sp_conv3x3_thin_bwd_input(dyg.data_ptr(), wg.data_ptr(), n, cin, cout, h, w,
                                             dx.data_ptr(), st), "thin bwd")
    rel = ((y.double().cpu() - ref.detach()).norm() / ref.detach().norm()).item()
    assert rel < 2e-6, rel
    rel = ((dx.double().cpu() - gref).norm() / gref.norm()).item()
    assert rel < 2e-6, rel


S2_SHAPES = [  # n, cin, cout, h, w (input size; output h/2 x w/2)
    (2, 128, 128, 32, 64),    # UNet level shape, both directions on the tile
    (1, 256, 256, 128, 64),   # VAE encoder-like, several tiles per image
    (2, 132, 256, 16, 128),   # cin % 128 != 0: forward on the tile, VJP on MIOpen
    (1, 512, 512, 16, 16),    # 8x8 output: MIOpen both ways (fallback)
]


@pytest.mark.parametrize("shape", S2_SHAPES)
def test_downsample_stride2_forward_and_input_vjp(cuda, shape):
    """Downsample2D's 3x3 / stride-2 conv (zero row / column bottom / right) on the
    csrc/sp_conv_s2.hip tiles (exact fp32 fmaf chains: the direct tile's tolerance) against
    fp64 torch on the padded input; the output-phase sums of the input VJP cover every tap
    exactly once (no tap is dropped or doubled at the image edges)."""
    from samplers_amd.networks.layers import downsample_conv, downsample_s2_supported

    n, cin, cout, h, w = shape
    g = torch.Generator().manual_seed(sum(shape) + 7)
    x = torch.randn(n, cin, h, w, generator=g)
    conv = torch.nn.Conv2d(cin, cout, 3, stride=2, padding=0)
    with torch.no_grad():
        conv.weight.normal_(0, (cin * 9) ** -0.5, generator=g)
        conv.bias.normal_(0, 0.1, generator=g)
    dy = torch.randn(n, cout, h // 2, w // 2, generator=g)
    xd = x.double().requires_grad_()
    ref = F.conv2d(F.pad(xd, (0, 1, 0, 1)), conv.weight.double(), conv.bias.double(), stride=2)
    (gref,) = torch.autograd.grad(ref, xd, dy.double())

    lib = _hip.load_library()
    fwd_tile = bool(lib.sp_conv3x3_s2_supported(cin, cout, h, w, 0))
    vjp_tile = bool(lib.sp_conv3x3_s2_supported(cin, cout, h, w, 1))
    assert (fwd_tile, vjp_tile) == {0: (True, True), 1: (True, True), 2: (True, False),
                                    3: (False, False)}[S2_SHAPES.index(shape)]
    cg = conv.to(cuda)
    xg = x.to(cuda).requires_grad_()
    assert downsample_s2_supported(cg, xg) == (fwd_tile and vjp_tile)
    out = downsample_conv(cg, xg)
    (gx,) = torch.autograd.grad(out, xg, dy.to(cuda))
    _check(out.detach(), ref.detach())
    _check(gx, gref)
    # the raw entry points on the shapes each direction serves
    if fwd_tile:
        wp = torch.empty(cin * cout * 9, device=cuda)
        _hip.check(lib.sp_conv3x3_s2_pack(_hip.ptr(cg.weight.detach().contiguous()), cout, cin, 0,
                                          _hip.ptr(wp), None), "pack")
        y = torch.empty(n, cout, h // 2, w // 2, device=cuda)
        xc = x.to(cuda)
        _hip.check(lib.sp_conv3x3_s2_fwd(_hip.ptr(xc), _hip.ptr(wp), None, n, cin, cout, h, w,
                                         _hip.ptr(y), None), "fwd")
        torch.cuda.synchronize()
        _check(y, ref.detach() - cg.bias.detach().double().cpu().view(1, -1, 1, 1))
    if vjp_tile:
        wv = torch.empty(cin * cout * 9, device=cuda)
        _hip.check(lib.sp_conv3x3_s2_pack(_hip.ptr(cg.weight.detach().contiguous()), cout, cin, 1,
                                          _hip.ptr(wv), None), "pack vjp")
        dx = torch.full((n, cin, h, w), float("nan"), device=cuda)
        dyc = dy.to(cuda)
        _hip.check(lib.sp_conv3x3_s2_bwd_input(_hip.ptr(dyc), _hip.ptr(wv), n, cin, cout, h, w, 0,
                                               _hip.ptr(dx), None), "bwd")
        torch.cuda.synchronize()
        assert torch.isfinite(dx).all()  # every dx element written
        _check(dx, gref)
        base = torch.randn(n, cin, h, w, generator=g)  # accumulate: dx += conv^T dy
        dxa = base.to(cuda)
        _hip.check(lib.sp_conv3x3_s2_bwd_input(_hip.ptr(dyc), _hip.ptr(wv), n, cin, cout, h, w, 1,
                                               _hip.ptr(dxa), None), "bwd acc")
        torch.cuda.synchronize()
        assert torch.equal(dxa, base.to(cuda) + dx)


@pytest.mark.parametrize("shape", [(1, 256, 256, 64, 64), (1, 128, 128, 128, 128), (2, 128, 128, 32, 64)])
def test_downsample_stride2_split_k(cuda, shape):
    """The split-K stride-2 launches (sp_conv3x3_s2_*_ws; batch-1 downsamplers): against fp64,
    bitwise repeatable, and the accumulating VJP equals base + the split VJP bitwise."""
    n, cin, cout, h, w = shape
    lib = _hip.load_library()
    nf = int(lib.sp_conv3x3_s2_workspace(n, cin, cout, h, w, 0))
    nv = int(lib.sp_conv3x3_s2_workspace(n, cin, cout, h, w, 1))
    assert nf > 0 and nv > 0
    g = torch.Generator().manual_seed(sum(shape) + 11)
    x = torch.randn(n, cin, h, w, generator=g)
    W = torch.randn(cout, cin, 3, 3, generator=g) * (cin * 9) ** -0.5
    b = torch.randn(cout, generator=g) * 0.1
    dy = torch.randn(n, cout, h // 2, w // 2, generator=g)
    xd = x.double().requires_grad_()
    ref = F.conv2d(F.pad(xd, (0, 1, 0, 1)), W.double(), b.double(), stride=2)
    (gref,) = torch.autograd.grad(ref, xd, dy.double())
    wg, bg, xc, dyc = W.to(cuda), b.to(cuda), x.to(cuda), dy.to(cuda)
    wp = torch.empty(cin * cout * 9, device=cuda)
    wv = torch.empty(cin * cout * 9, device=cuda)
    _hip.check(lib.sp_conv3x3_s2_pack(_hip.ptr(wg), cout, cin, 0, _hip.ptr(wp), None), "pack")
    _hip.check(lib.sp_conv3x3_s2_pack(_hip.ptr(wg), cout, cin, 1, _hip.ptr(wv), None), "pack vjp")
    wsf = torch.empty(nf // 4, device=cuda)
    wsv = torch.empty(nv // 4, device=cuda)
    ys, dxs = [], []
    for _ in range(2):
        y = torch.full((n, cout, h // 2, w // 2), float("nan"), device=cuda)
        _hip.check(lib.sp_conv3x3_s2_fwd_ws(_hip.ptr(xc), _hip.ptr(wp), _hip.ptr(bg), n, cin, cout, h, w,
                                            _hip.ptr(y), _hip.ptr(wsf), nf, None), "fwd_ws")
        dx = torch.full((n, cin, h, w), float("nan"), device=cuda)
        _hip.check(lib.sp_conv3x3_s2_bwd_input_ws(_hip.ptr(dyc), _hip.ptr(wv), n, cin, cout, h, w, 0,
                                                  _hip.ptr(dx), _hip.ptr(wsv), nv, None), "bwd_ws")
        ys.append(y)
        dxs.append(dx)
    base = torch.randn(n, cin, h, w, generator=g).to(cuda)
    dxa = base.clone()
    _hip.check(lib.sp_conv3x3_s2_bwd_input_ws(_hip.ptr(dyc), _hip.ptr(wv), n, cin, cout, h, w, 1,
                                              _hip.ptr(dxa), _hip.ptr(wsv), nv, None), "bwd_ws acc")
    torch.cuda.synchronize()
    assert torch.equal(ys[0], ys[1]) and torch.equal(dxs[0], dxs[1])
    _check(ys[0], ref.detach())
    _check(dxs[0], gref)
    assert torch.equal(dxa, base + dxs[0])


def test_downsample_stride2_rejects_bad_shapes():
    lib = _hip.load_library()
    assert not lib.sp_conv3x3_s2_supported(128, 128, 33, 64, 0)   # odd height
    assert not lib.sp_conv3x3_s2_supported(128, 100, 32, 64, 0)   # cout % 128
    assert not lib.sp_conv3x3_s2_supported(100, 128, 32, 64, 1)   # cin % 128 (VJP)
    assert lib.sp_conv3x3_s2_fwd(None, None, None, 1, 128, 100, 32, 64, None, None) != 0


@pytest.mark.parametrize("shape", [(2, 128, 8, 8), (1, 64, 32, 64), (3, 5, 16, 12), (2, 4, 6, 6)])
def test_upsample_nearest2x_and_vjp(cuda, shape):
    """csrc/sp_upsample.hip: forward is a copy (bit-exact vs F.interpolate); the VJP sums each
    2x2 block of dy in torch's loop order (bit-exact vs torch's backward on the same device).
    Width 6 is not a multiple of 4: the torch fallback serves it."""
    from samplers_amd.networks.layers import upsample_nearest2x

    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(*shape, generator=g).to(cuda).requires_grad_()
    dy = torch.randn(shape[0], shape[1], 2 * shape[2], 2 * shape[3], generator=g).to(cuda)
    out = upsample_nearest2x(x)
    (gx,) = torch.autograd.grad(out, x, dy)
    ref = F.interpolate(x, scale_factor=2.0, mode="nearest")
    (gref,) = torch.autograd.grad(ref, x, dy)
    assert torch.equal(out, ref)
    torch.testing.assert_close(gx, gref, rtol=1e-6, atol=1e-6)
    # fp64 block sums on the CPU
    want = dy.double().cpu().reshape(shape[0], shape[1], shape[2], 2, shape[3], 2).sum((3, 5))
    assert ((gx.double().cpu() - want).abs().max() <= 4e-7 * want.abs().max().clamp_min(1)).item()


STRIDE2_FULL_SHAPES = [  # n, c, h, w: the SD 1.5 UNet's downsamplers and the UNet's 16x16 one
    (2, 320, 64, 64),
    (2, 640, 32, 32),
    (1, 1280, 16, 16),
    (3, 256, 16, 16),
]


@pytest.mark.parametrize("padding", [1, 0])
@pytest.mark.parametrize("shape", STRIDE2_FULL_SHAPES)
def test_stride2_conv_via_full_resolution_tiles(cuda, shape, padding):
    """3x3 / stride-2 convolutions outside the stride-2 tile's rules run as the stride-1
    tile at full resolution read at the even (padding 1) or odd (one zero row / column
    bottom / right) positions; the input VJP scatters dy to those positions.  Against fp64
    torch, with the Winograd tolerance; the path must not reach MIOpen."""
    from samplers_amd.networks.layers import conv3x3_stride2, strided_full_supported

    n, c, h, w = shape
    g = torch.Generator().manual_seed(sum(shape) + padding)
    x = torch.randn(n, c, h, w, generator=g)
    conv = torch.nn.Conv2d(c, c, 3, stride=2, padding=padding).requires_grad_(False)
    with torch.no_grad():
        conv.weight.normal_(0, (c * 9) ** -0.5, generator=g)
        conv.bias.normal_(0, 0.1, generator=g)
    dy = torch.randn(n, c, h // 2, w // 2, generator=g)
    xd = x.double().requires_grad_()
    xin = xd if padding else F.pad(xd, (0, 1, 0, 1))
    ref = F.conv2d(xin, conv.weight.double(), conv.bias.double(), stride=2, padding=padding)
    (gref,) = torch.autograd.grad(ref, xd, dy.double())

    cg = conv.to(cuda)
    xg = x.to(cuda).requires_grad_()
    assert strided_full_supported(cg, xg)
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        out = conv3x3_stride2(cg, xg, padding)
        (gx,) = torch.autograd.grad(out, xg, dy.to(cuda))
        torch.cuda.synchronize()
    names = {e.name for e in prof.events() if e.device_type.name == "CUDA"}
    assert not any("naive_conv" in k or "igemm" in k or "Conv" in k for k in names), names
    assert out.shape == ref.shape
    _check(out.detach(), ref.detach(), slack=5)
    _check(gx, gref, slack=5)


# --- the default tile against fp64 (the bar the removed split-bf16 backends were held to) ----

FP64_SHAPES = [(2, 32, 64, 16, 32), (1, 16, 64, 32, 32), (2, 64, 64, 32, 64), (1, 128, 128, 48, 96)]


@pytest.mark.parametrize("shape", FP64_SHAPES)
def test_default_tile_error_vs_fp64(cuda, shape):
    """The Conv3x3 module's default dispatch (Winograd F(2x2,3x3) tile on fp32 MFMAs) against
    an fp64 convolution of the same data: forward with bias + residual epilogue and input VJP,
    relative L2 < 1e-6 (measured 2-4e-7: fp32-class)."""
    n, cin, cout, h, w = shape
    g = torch.Generator().manual_seed(sum(shape) + 7)
    x = torch.randn(n, cin, h, w, generator=g)
    conv = Conv3x3(cin, cout)
    with torch.no_grad():
        conv.weight.normal_(0, (cin * 9) ** -0.5, generator=g)
        conv.bias.normal_(0, 0.1, generator=g)
    res = torch.randn(n, cout, h, w, generator=g)
    dy = torch.randn(n, cout, h, w, generator=g)
    xd = x.double().requires_grad_()
    ref = F.conv2d(xd, conv.weight.double(), conv.bias.double(), padding=1)
    (gref,) = torch.autograd.grad(ref, xd, dy.double())
    ref = ref.detach() + res.double()
    from samplers_amd.networks.layers import conv3x3_forward, conv3x3_input_vjp

    cg = conv.to(cuda)
    y = conv3x3_forward(cg, x.to(cuda), res=res.to(cuda))
    dx = conv3x3_input_vjp(cg, dy.to(cuda), x.shape)
    torch.cuda.synchronize()
    rel = lambda a, b: ((a.double().cpu() - b).norm() / b.norm()).item()  # noqa: E731
    assert rel(y, ref) < 1e-6 and rel(dx, gref) < 1e-6, (rel(y, ref), rel(dx, gref))


UPCONV_SHAPES = [  # n, c (cin = cout, diffusers Upsample2D), source h, w
    (2, 128, 16, 16),
    (1, 256, 16, 32),
    (2, 64, 32, 32),
    (1, 512, 16, 16),
]


def _upconv_operands(shape, cuda):
    n, c, h, w = shape
    g = torch.Generator().manual_seed(sum(shape) + 7)
    x = torch.randn(n, c, h, w, generator=g)
    wt = torch.randn(c, c, 3, 3, generator=g) * (c * 9) ** -0.5
    b = torch.randn(c, generator=g) * 0.1
    dy = torch.randn(n, c, 2 * h, 2 * w, generator=g)
    return x, wt, b, dy


@pytest.mark.parametrize("shape", UPCONV_SHAPES)
def test_winograd_fused_upsample_matches_the_unfused_pair(cuda, shape):
    """Upsample2D fused into the Winograd tile (sp_wino3x3_fwd_up / sp_wino3x3_bwd_input_pool):
    the forward equals the unsplit tile on the materialised upsample bitwise (the same values
    reach the same LDS image), the input VJP equals sp_wino3x3_bwd_input followed by
    sp_upsample2x_vjp bitwise (the epilogue sums each 2x2 block in the upsample VJP's order),
    and both agree with fp64 conv2d(interpolate(x)) to the tile's usual bound."""
    from samplers_amd.networks.layers import upsample_nearest2x

    n, c, h, w = shape
    H, W = 2 * h, 2 * w
    lib = _hip.load_library()
    assert lib.sp_wino3x3_up_supported(c, c, H, W)
    x, wt, b, dy = _upconv_operands(shape, cuda)
    st = torch.cuda.current_stream().cuda_stream
    xg, wg, bg, dyg = x.to(cuda), wt.to(cuda), b.to(cuda), dy.to(cuda)
    up = torch.empty(c * c * 16, device=cuda)
    uv = torch.empty_like(up)
    assert lib.sp_wino3x3_pack(_hip.ptr(wg), c, c, 0, _hip.ptr(up), st) == 0
    assert lib.sp_wino3x3_pack(_hip.ptr(wg), c, c, 1, _hip.ptr(uv), st) == 0
    # fused
    y = torch.empty(n, c, H, W, device=cuda)
    assert lib.sp_wino3x3_fwd_up(_hip.ptr(xg), _hip.ptr(up), _hip.ptr(bg), n, c, c, H, W, _hip.ptr(y), st) == 0
    dx = torch.empty(n, c, h, w, device=cuda)
    assert lib.sp_wino3x3_bwd_input_pool(_hip.ptr(dyg), _hip.ptr(uv), n, c, c, H, W, _hip.ptr(dx), st) == 0
    # the unfused pair, unsplit
    xu = upsample_nearest2x(xg).contiguous()
    yr = torch.empty_like(y)
    assert lib.sp_wino3x3_fwd(_hip.ptr(xu), _hip.ptr(up), _hip.ptr(bg), n, c, c, H, W, _hip.ptr(yr), st) == 0
    gu = torch.empty(n, c, H, W, device=cuda)
    assert lib.sp_wino3x3_bwd_input(_hip.ptr(dyg), _hip.ptr(uv), n, c, c, H, W, _hip.ptr(gu), st) == 0
    dxr = torch.empty_like(dx)
    assert lib.sp_upsample2x_vjp(_hip.ptr(gu), n * c, h, w, _hip.ptr(dxr), st) == 0  # source dims
    torch.cuda.synchronize()
    assert torch.equal(y, yr)
    assert torch.equal(dx, dxr)
    # fp64
    xd = x.double().requires_grad_()
    ref = F.conv2d(F.interpolate(xd, scale_factor=2.0, mode="nearest"), wt.double(), b.double(), padding=1)
    (gref,) = torch.autograd.grad(ref, xd, dy.double())
    _check(y, ref.detach(), 5)
    _check(dx, gref, 5)


def test_winograd_fused_upsample_rejects_unsupported(cuda):
    lib = _hip.load_library()
    assert not lib.sp_wino3x3_up_supported(128, 128, 16, 16)   # W = 16: the narrow geometry
    assert not lib.sp_wino3x3_up_supported(32, 128, 32, 32)    # VJP output channels % 64
    assert not lib.sp_wino3x3_up_supported(8, 64, 32, 32)      # K below the xi ring
    assert lib.sp_wino3x3_up_supported(128, 128, 32, 32)
    bad = torch.empty(16, device=cuda)
    st = torch.cuda.current_stream().cuda_stream
    assert lib.sp_wino3x3_fwd_up(_hip.ptr(bad), _hip.ptr(bad), None, 1, 128, 128, 16, 16,
                                 _hip.ptr(bad), st) != 0


def test_upsample2d_module_fused_equals_unfused(cuda, monkeypatch):
    """Upsample2D (unet2d.py) through autograd: the fused path (default) and the unfused pair
    (SAMPLERS_AMD_UPCONV=0) give bitwise-equal outputs and input gradients at a shape whose
    unfused launches run unsplit; under-filled shapes keep the (split) unfused pair."""
    from samplers_amd.networks import layers
    from samplers_amd.networks.unet2d import Upsample2D

    n, c, h, w = 8, 128, 32, 32  # 64x64 output: 256 tiles, unsplit
    g = torch.Generator().manual_seed(11)
    m = Upsample2D(c)
    with torch.no_grad():
        m.conv.weight.normal_(0, (c * 9) ** -0.5, generator=g)
        m.conv.bias.normal_(0, 0.1, generator=g)
    m = m.to(cuda).requires_grad_(False)
    x = torch.randn(n, c, h, w, generator=g).to(cuda)
    dy = torch.randn(n, c, 2 * h, 2 * w, generator=g).to(cuda)
    assert layers.upsample_conv_supported(m.conv, x)
    assert not layers.upsample_conv_supported(m.conv, x[:1])  # one image: the pair splits K

    calls = []
    orig = layers._UpsampleConv3x3Fn.apply
    monkeypatch.setattr(layers._UpsampleConv3x3Fn, "apply", lambda *a: calls.append(1) or orig(*a))

    def run():
        xr = x.clone().requires_grad_()
        out = m(xr)
        (gx,) = torch.autograd.grad(out, xr, dy)
        return out.detach(), gx

    y1, g1 = run()
    assert calls
    monkeypatch.setenv("SAMPLERS_AMD_UPCONV", "0")
    calls.clear()
    y0, g0 = run()
    assert not calls
    assert torch.equal(y1, y0)
    assert torch.equal(g1, g0)

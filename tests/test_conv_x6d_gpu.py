"""The direct 3x3 convolution on the bf16 datapath (csrc/sp_gemm_x6.hip, k_conv3x3_x6) against
fp64: y = conv3x3(x, W) (+ bias) (+ residual), stride 1, zero padding 1, and the input VJP
through the transposed / flipped pack.

Tolerance: relative L2 <= 1.5x the error of torch's fp32 convolution (CPU) on the same data,
and < 1e-6 (three exact bf16 terms per operand, six partial products, fp32 accumulation)."""

import pytest
import torch
import torch.nn.functional as F

from samplers_amd import _hip

pytestmark = pytest.mark.gpu

CASES = [  # n, cin, cout, h, w
    (1, 16, 128, 8, 32),
    (2, 32, 128, 16, 32),
    (1, 48, 256, 24, 64),
    (3, 128, 128, 8, 64),
    (1, 256, 128, 32, 32),
]


def _rel(a, b):
    return float((a.double().cpu() - b).norm() / b.norm())


def _pack(lib, w, m, k, trans, cuda):
    wp = torch.empty(int(lib.sp_conv3x3_x6_packed_size(m, k)), device=cuda)
    _hip.check(lib.sp_conv3x3_x6_pack(w.data_ptr(), m, k, trans, wp.data_ptr(),
                                      torch.cuda.current_stream().cuda_stream), "pack")
    return wp


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("extras", [False, True])
def test_conv3x3_x6_matches_fp64(cuda, case, extras):
    n, cin, cout, h, w = case
    lib = _hip.load_library()
    assert lib.sp_conv3x3_x6_supported(cout, cin, h, w)
    g = torch.Generator().manual_seed(sum(case) + extras)
    x = torch.randn(n, cin, h, w, generator=g)
    W = torch.randn(cout, cin, 3, 3, generator=g) * (9 * cin) ** -0.5
    bias = torch.randn(cout, generator=g) if extras else None
    res = torch.randn(n, cout, h, w, generator=g) if extras else None
    ref = F.conv2d(x.double(), W.double(), None if bias is None else bias.double(), padding=1)
    t32 = F.conv2d(x, W, bias, padding=1)
    if res is not None:
        ref, t32 = ref + res.double(), t32 + res
    wg = W.to(cuda)
    wp = _pack(lib, wg, cout, cin, 0, cuda)
    xg = x.to(cuda)
    # device copies held by name for the call (a temporary freed inside the argument list can
    # hand its block to the next one before the kernel runs)
    bg = None if bias is None else bias.to(cuda)
    rg = None if res is None else res.to(cuda)
    y = torch.full((n, cout, h, w), float("nan"), device=cuda)
    _hip.check(lib.sp_conv3x3_x6(xg.data_ptr(), wp.data_ptr(), None if bg is None else bg.data_ptr(),
                                 None if rg is None else rg.data_ptr(), n, cin, cout, h, w,
                                 y.data_ptr(), torch.cuda.current_stream().cuda_stream), "sp_conv3x3_x6")
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    e6, e32 = _rel(y, ref), _rel(t32, ref)
    assert e6 <= 1.5 * e32 + 1e-9 and e6 < 1e-6, (e6, e32)


@pytest.mark.parametrize("case", [(2, 128, 128, 16, 32), (1, 128, 256, 8, 64)])
def test_conv3x3_x6_transposed_pack_is_the_input_vjp(cuda, case):
    """trans = 1 packs the forward's W [cout][cin][3][3] as the VJP's operand: dx = conv(dy, W')."""
    n, cin, cout, h, w = case
    lib = _hip.load_library()
    assert lib.sp_conv3x3_x6_supported(cin, cout, h, w)
    g = torch.Generator().manual_seed(7)
    W = torch.randn(cout, cin, 3, 3, generator=g) * (9 * cin) ** -0.5
    dy = torch.randn(n, cout, h, w, generator=g)
    ref = torch.nn.grad.conv2d_input((n, cin, h, w), W.double(), dy.double(), padding=1)
    t32 = torch.nn.grad.conv2d_input((n, cin, h, w), W, dy, padding=1)
    wp = _pack(lib, W.to(cuda), cin, cout, 1, cuda)
    dyg = dy.to(cuda)
    dx = torch.full((n, cin, h, w), float("nan"), device=cuda)
    _hip.check(lib.sp_conv3x3_x6(dyg.data_ptr(), wp.data_ptr(), None, None, n, cout, cin, h, w, dx.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream), "sp_conv3x3_x6")
    torch.cuda.synchronize()
    e6, e32 = _rel(dx, ref), _rel(t32, ref)
    assert e6 <= 1.5 * e32 + 1e-9 and e6 < 1e-6, (e6, e32)


def test_conv3x3_x6_rejects_bad_shapes(cuda):
    lib = _hip.load_library()
    assert not lib.sp_conv3x3_x6_supported(96, 64, 16, 32)    # cout % 128
    assert not lib.sp_conv3x3_x6_supported(128, 24, 16, 32)   # cin % 16
    assert not lib.sp_conv3x3_x6_supported(128, 64, 12, 32)   # h % 8
    assert not lib.sp_conv3x3_x6_supported(128, 64, 16, 48)   # w % 32
    x = torch.empty(1, device=cuda)
    assert lib.sp_conv3x3_x6(x.data_ptr(), x.data_ptr(), None, None, 1, 64, 96, 16, 32, x.data_ptr(), 0) != 0


@pytest.mark.parametrize("shape", [(2, 128, 128, 16, 32), (1, 128, 256, 8, 64), (1, 256, 128, 16, 64)])
def test_x6d_backend_error_is_fp32_class(cuda, shape, monkeypatch):
    """``SAMPLERS_AMD_CONV=x6d`` through the Conv3x3 module's dispatch (forward with bias +
    residual, input VJP) is at least as close to fp64 as the fp32-MFMA Winograd tile."""
    from samplers_amd.networks.layers import Conv3x3, conv3x3_forward, conv3x3_input_vjp

    n, cin, cout, h, w = shape
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(n, cin, h, w, generator=g)
    conv = Conv3x3(cin, cout)
    with torch.no_grad():
        conv.weight.normal_(0, (cin * 9) ** -0.5, generator=g)
        conv.bias.normal_(0, 0.1, generator=g)
    conv.requires_grad_(False)
    res = torch.randn(n, cout, h, w, generator=g)
    dy = torch.randn(n, cout, h, w, generator=g)
    xd = x.double().requires_grad_()
    ref = F.conv2d(xd, conv.weight.double(), conv.bias.double(), padding=1)
    (gref,) = torch.autograd.grad(ref, xd, dy.double())
    ref = ref.detach() + res.double()
    cg = conv.to(cuda)
    xg, rg, dyg = x.to(cuda), res.to(cuda), dy.to(cuda)
    errs = {}
    for backend in ("auto", "x6d"):
        monkeypatch.setenv("SAMPLERS_AMD_CONV", backend)
        y = conv3x3_forward(cg, xg, res=rg)
        dx = conv3x3_input_vjp(cg, dyg, x.shape)
        torch.cuda.synchronize()
        errs[backend] = (_rel(y, ref), _rel(dx, gref))
    for k in range(2):
        assert errs["x6d"][k] <= 1.2 * errs["auto"][k] + 1e-9, errs
        assert errs["x6d"][k] < 1e-6, errs


def test_x6d_backend_kernel_runs(cuda, monkeypatch):
    """The x6d backend really dispatches to k_conv3x3_x6 (kernel names in the profiler)."""
    from samplers_amd.networks.layers import Conv3x3

    monkeypatch.setenv("SAMPLERS_AMD_CONV", "x6d")
    conv = Conv3x3(128, 128).to(cuda).requires_grad_(False)
    x = torch.randn(2, 128, 16, 32, device=cuda)
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        conv(x)
        torch.cuda.synchronize()
    names = " ".join(e.key for e in prof.key_averages())
    assert "k_conv3x3_x6" in names, names

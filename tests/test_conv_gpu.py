"""fp32-MFMA 3x3 convolution (csrc/sp_conv.hip) against an fp64 torch reference.

The kernel is an exact-fp32 fmaf chain over K = Cin*9 (v_mfma_f32_32x32x2_f32), so the
tolerance is the fp32 accumulation error: relative L2 <= 2e-6 and max |err| <= 1e-5 x the
largest |output| for the forward and the input VJP."""

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


def _check(got, ref):
    ref = ref.double()
    rel = ((got.double().cpu() - ref).norm() / ref.norm()).item()
    mx = (got.double().cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert rel < 2e-6 and mx < 1e-5, (rel, mx)


@pytest.mark.parametrize("shape", SHAPES)
def test_conv3x3_forward_and_input_vjp(cuda, shape):
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
    cg = conv.to(cuda)
    xg = x.to(cuda).requires_grad_()
    out = cg(xg)
    (gx,) = torch.autograd.grad(out, xg, dy.to(cuda))
    _check(out.detach(), ref.detach())
    _check(gx, gref)


def test_conv3x3_matches_miopen_and_repacks(cuda, monkeypatch):
    conv = Conv3x3(128, 128).to(cuda)
    x = torch.randn(2, 128, 8, 32, device=cuda)
    a = conv(x)
    monkeypatch.setenv("SAMPLERS_AMD_CONV", "miopen")
    b = conv(x)
    torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)
    monkeypatch.setenv("SAMPLERS_AMD_CONV", "hip")
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
    conv = Conv3x3(128, 128).to(cuda)  # falls back to MIOpen at 16x16
    x = torch.randn(1, 128, 16, 16, device=cuda)
    torch.testing.assert_close(conv(x), F.conv2d(x, conv.weight, conv.bias, padding=1))


def test_conv3x3_timing_records_flops(cuda):
    from samplers_amd.samplers.dps import KernelTimer

    conv = Conv3x3(128, 256).to(cuda)
    x = torch.randn(2, 128, 8, 64, device=cuda, requires_grad=True)
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

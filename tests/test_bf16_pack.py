"""CPU checks of the bf16 layers' host logic (networks/bf16.py): the weight pack that
``sp_conv3x3_bf16`` reads, forward and input VJP, reconstructed here in torch exactly as the
kernel's index map walks it ([co block][ci block][tap 3 ky + kx][64 co][16 ci]; tap (dy, dx)
reads input pixel (h + dy - 1, w + dx - 1)), against ``F.conv2d`` / ``conv2d_input``; and the
reduced-precision networks' dtype (the reference's ``_pipeline.dtype``)."""

from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

from samplers_amd.networks import bf16


def _conv_from_pack(x: torch.Tensor, pack: torch.Tensor, cout: int) -> torch.Tensor:
    """The kernel's contraction over a pack: y[n, 64 cb + r, h, w] = sum over ci block, tap,
    16 ci of pack[cb][cib][tap][r][c] x[n, 16 cib + c, h + dy - 1, w + dx - 1]."""
    n, cin, h, w = x.shape
    cbn, cib, _, _, _ = pack.shape
    xp = F.pad(x, (1, 1, 1, 1, 0, cib * 16 - cin))
    y = torch.zeros(n, cbn * 64, h, w, dtype=torch.float64)
    for t in range(9):
        dy, dx = divmod(t, 3)
        win = xp[:, :, dy:dy + h, dx:dx + w].double()  # [n][cib*16][h][w]
        wt = pack[:, :, t].double()                       # [cbn][cib][64][16]
        wt = wt.permute(0, 2, 1, 3).reshape(cbn * 64, cib * 16)
        y += torch.einsum("oc,nchw->nohw", wt, win)
    return y[:, :cout]


@pytest.mark.parametrize("cin,cout", [(16, 64), (4, 320), (320, 4), (3, 128), (128, 3), (48, 80)])
def test_conv_pack_forward_and_vjp_match_torch(cin, cout):
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(cin, cout, 3, padding=1).requires_grad_(False)
    x = torch.randn(2, cin, 6, 5, dtype=torch.float64)
    pack = bf16.conv_pack(conv, False)
    assert pack.dtype == torch.bfloat16 and pack.numel() == -(-cout // 64) * 64 * -(-cin // 16) * 16 * 9
    wq = conv.weight.to(torch.bfloat16).double()  # the pack holds the weights rounded to bf16
    ref = F.conv2d(x, wq, padding=1)
    got = _conv_from_pack(x, pack, cout)
    assert torch.allclose(got, ref, rtol=1e-12, atol=1e-10)
    dy = torch.randn(2, cout, 6, 5, dtype=torch.float64)
    ref_dx = torch.nn.grad.conv2d_input(x.shape, wq, dy, padding=1)
    got_dx = _conv_from_pack(dy, bf16.conv_pack(conv, True), cin)
    assert torch.allclose(got_dx, ref_dx, rtol=1e-12, atol=1e-10)


def test_conv_pack_cache_follows_the_weight():
    conv = torch.nn.Conv2d(16, 64, 3, padding=1).requires_grad_(False)
    p0 = bf16.conv_pack(conv, False)
    assert bf16.conv_pack(conv, False) is p0
    with torch.no_grad():
        conv.weight.mul_(2)
    p1 = bf16.conv_pack(conv, False)
    assert p1 is not p0 and torch.equal(p1.float(), (p0.float() * 2))


def test_reduced_precision_networks_report_their_dtype():
    """``from_config(torch_dtype=bf16)`` gives a network whose ``dtype`` is bf16 (the reference's
    ``pipeline.dtype``), so the samplers put it behind the fp32 boundary and return bf16."""
    from samplers_amd.networks.base import Fp32Boundary, fp32_view
    from samplers_amd.networks.ddpm import DDPMNetwork
    from samplers_amd.networks.unet2d import UNet2DConfig

    tiny = UNet2DConfig(sample_size=16, block_out_channels=(32, 32), attention_levels=(1,), layers_per_block=1)
    net = DDPMNetwork.from_config(tiny, torch_dtype=torch.bfloat16)
    assert net.dtype == torch.bfloat16
    assert isinstance(fp32_view(net), Fp32Boundary)
    assert DDPMNetwork.from_config(tiny).dtype == torch.float32

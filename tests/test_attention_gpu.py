"""The priors' self-attention on the GPU: materialised scores on batched fp32 GEMMs + softmax
(the default, ``SAMPLERS_AMD_ATTN=gemm``) against F.scaled_dot_product_attention
(``SAMPLERS_AMD_ATTN=sdpa``), forward and input VJP, one head of 512 (DDPM UNet / VAE mid
block) and several heads (latent UNet)."""

import pytest
import torch

from samplers_amd.networks.unet2d import SpatialSelfAttention

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a - b).norm() / b.norm())


@pytest.mark.parametrize("c,head_dim,hw", [(512, None, 8), (128, 32, 16), (64, None, 16)])
def test_attention_gemm_path_matches_sdpa(cuda, monkeypatch, c, head_dim, hw):
    torch.manual_seed(0)
    m = SpatialSelfAttention(c, 32, 1e-6, head_dim).to(cuda).requires_grad_(False)
    x = torch.randn(3, c, hw, hw, device=cuda)
    v = torch.randn_like(x)
    outs = []
    for backend in ("gemm", "sdpa"):
        monkeypatch.setenv("SAMPLERS_AMD_ATTN", backend)
        xg = x.clone().requires_grad_()
        y = m(xg)
        (g,) = torch.autograd.grad(y, xg, v)
        outs.append((y.detach(), g))
    assert _rel(outs[0][0], outs[1][0]) < 2e-5
    assert _rel(outs[0][1], outs[1][1]) < 2e-5

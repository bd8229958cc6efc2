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


@pytest.mark.parametrize("bh,n,d", [(6, 256, 40), (3, 1024, 40), (4, 128, 80), (3, 64, 160),
                                    (2, 256, 160)])
def test_fused_self_attention_matches_fp64(cuda, bh, n, d):
    """The fused fp32-MFMA self-attention (csrc/sp_attention.hip) against fp64 torch:
    output and the three input VJPs at the SD 1.5 UNet's head dims (40 / 80 / 160), relative
    L2 <= 1e-5 (exact fp32 MFMA sums; exp2 on the hardware transcendental)."""
    from torch.profiler import ProfilerActivity, profile

    from samplers_amd import _hip
    from samplers_amd.networks.attention import FUSED_BWD_MIN_TOKENS, attention, fused_supported

    g = torch.Generator().manual_seed(bh * n + d)
    q, k, v, do = (torch.randn(bh, n, d, generator=g) * s for s in (1.0, 1.0, 1.0, 0.5))
    qd, kd, vd = (t.double().requires_grad_() for t in (q, k, v))
    ref = torch.softmax(qd @ kd.transpose(1, 2) / d ** 0.5, dim=-1) @ vd
    gref = torch.autograd.grad(ref, (qd, kd, vd), do.double())

    qg, kg, vg = (t.to(cuda).requires_grad_() for t in (q, k, v))
    assert fused_supported(qg, kg)
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        out = attention(qg, kg, vg)
        grads = torch.autograd.grad(out, (qg, kg, vg), do.to(cuda))
        torch.cuda.synchronize()
    names = {e.name for e in prof.events() if e.device_type.name == "CUDA"}
    assert any("k_attn_fwd" in x for x in names)
    fused_bwd = n >= FUSED_BWD_MIN_TOKENS
    assert any("k_attn_dkv" in x for x in names) == fused_bwd
    if fused_bwd:
        assert not any("Cijk" in x for x in names), "score GEMMs should not run"
    assert _rel(out.detach().cpu().double(), ref.detach()) < 1e-5
    for got, want in zip(grads, gref):
        assert _rel(got.cpu().double(), want) < 1e-5
    # the fused VJP kernels at every shape, through the C ABI
    lib = _hip.load_library()
    qc, kc, vc, oc, dc = (t.detach().contiguous() for t in (qg, kg, vg, out, do.to(cuda)))
    lse = torch.empty(bh, n, device=cuda)
    o2 = torch.empty_like(qc)
    _hip.check(lib.sp_attention_fwd(_hip.ptr(qc), _hip.ptr(kc), _hip.ptr(vc), bh, n, d, d ** -0.5,
                                    _hip.ptr(o2), _hip.ptr(lse), None), "fwd")
    delta = torch.empty(bh, n, device=cuda)
    dq, dk, dv = (torch.full_like(qc, float("nan")) for _ in range(3))
    _hip.check(lib.sp_attention_bwd(_hip.ptr(qc), _hip.ptr(kc), _hip.ptr(vc), _hip.ptr(o2),
                                    _hip.ptr(dc), _hip.ptr(lse), bh, n, d, d ** -0.5,
                                    _hip.ptr(delta), _hip.ptr(dq), _hip.ptr(dk), _hip.ptr(dv),
                                    None), "bwd")
    torch.cuda.synchronize()
    assert torch.equal(o2, oc)  # the forward is deterministic
    for got, want in zip((dq, dk, dv), gref):
        assert _rel(got.cpu().double(), want) < 1e-5


def test_fused_attention_falls_back_for_cross_attention(cuda):
    from samplers_amd.networks.attention import attention, fused_supported

    q = torch.randn(2, 256, 40, device=cuda)
    k = torch.randn(2, 77, 40, device=cuda)
    assert not fused_supported(q, k)
    out = attention(q, k, torch.randn(2, 77, 40, device=cuda))
    assert out.shape == q.shape

"""The SD 1.5 latent prior on the CPU: architecture size and diffusers parameter names, the
recompute-attention VJP, and the reference's conditioning semantics
(``/root/reference/samplers/networks/diffusers/stable_diffusion.py:146-328``)."""

import pytest
import torch

from samplers_amd.networks.attention import _RecomputeAttention
from samplers_amd.networks.latent import (LatentDiffusionNetwork, StableDiffusionCondition,
                                          rescale_noise_cfg)
from samplers_amd.networks.unet2d import count_parameters
from samplers_amd.networks.unet2d_condition import (SD15_UNET, UNet2DConditionConfig,
                                                    UNet2DConditionModel)
from samplers_amd.networks.vae import VAEConfig

TINY_UNET = UNet2DConditionConfig(sample_size=16, block_out_channels=(32, 64),
                                  cross_attention_levels=(0,), attention_heads=2,
                                  cross_attention_dim=24, norm_num_groups=8, context_tokens=5)
TINY_VAE = VAEConfig(block_out_channels=(16, 32), norm_num_groups=8)


def test_sd15_unet_size_and_names():
    with torch.device("meta"):
        net = UNet2DConditionModel(SD15_UNET)
    assert count_parameters(net) == 859_520_964  # SD 1.5 unet
    keys = set(net.state_dict())
    assert len(keys) == 686
    for k in ("conv_in.weight", "time_embedding.linear_2.bias",
              "down_blocks.0.attentions.1.transformer_blocks.0.attn2.to_k.weight",
              "down_blocks.0.attentions.0.proj_in.weight", "down_blocks.2.downsamplers.0.conv.weight",
              "down_blocks.3.resnets.1.conv2.weight", "mid_block.attentions.0.norm.weight",
              "up_blocks.0.upsamplers.0.conv.weight",
              "up_blocks.3.attentions.2.transformer_blocks.0.ff.net.0.proj.weight",
              "up_blocks.3.attentions.2.transformer_blocks.0.ff.net.2.bias",
              "up_blocks.1.resnets.2.conv_shortcut.weight", "conv_norm_out.weight", "conv_out.bias"):
        assert k in keys, k
    assert tuple(net.state_dict()["down_blocks.1.attentions.0.transformer_blocks.0.attn2.to_k.weight"]
                 .shape) == (640, 768)


@pytest.mark.parametrize("n,m", [(7, 7), (9, 5)])
def test_recompute_attention_vjp(n, m, monkeypatch):
    monkeypatch.setenv("SAMPLERS_AMD_ATTN_CHUNK_MIB", "0")  # one row per chunk: chunk seams
    torch.manual_seed(0)
    q = torch.randn(3, n, 4, dtype=torch.float64, requires_grad=True)
    k = torch.randn(3, m, 4, dtype=torch.float64, requires_grad=True)
    v = torch.randn(3, m, 6, dtype=torch.float64, requires_grad=True)
    assert torch.autograd.gradcheck(_RecomputeAttention.apply, (q, k, v))
    ref = torch.softmax(q @ k.transpose(1, 2) / 2.0, dim=-1) @ v
    torch.testing.assert_close(_RecomputeAttention.apply(q, k, v), ref)


def _tiny_net():
    return LatentDiffusionNetwork.from_config(TINY_UNET, TINY_VAE, seed=3)


def test_condition_requires_sampling_parameters_and_matching_batch():
    net = _tiny_net()
    with pytest.raises(RuntimeError):
        net.set_condition(None)
    net.set_sampling_parameters(10, batch_size=2)
    with pytest.raises(ValueError, match="Batch size mismatch"):
        net.set_condition(None)  # prompt "" is one prompt (stable_diffusion.py:200-221)
    with pytest.raises(NotImplementedError, match="text encoder"):
        net.set_condition(StableDiffusionCondition(prompt=["a cat", "a dog"]))
    net.set_condition(StableDiffusionCondition(prompt=["", ""]))
    assert net.is_condition_initialized
    net.clear_condition()
    assert not net.is_condition_initialized
    with pytest.raises(RuntimeError, match="set_condition"):
        net(torch.zeros(2, 4, 8, 8), 5)


def test_default_cfg_collapses_to_one_pass_exactly():
    """Empty prompt + empty negative prompt at guidance 7.5 (the reference default): the CFG
    combination equals the single conditional pass."""
    net = _tiny_net()
    net.set_sampling_parameters(10, batch_size=2)
    net.set_condition(StableDiffusionCondition(prompt=["", ""]))
    st = net._conditioning
    assert not st.do_classifier_free_guidance and st.prompt_embeds.shape[0] == 1
    z = torch.randn(2, 4, 8, 8)
    with torch.no_grad():
        got = net(z, 21)
        u = net.unet(z, 21, net.null_prompt_embeds.expand(2, -1, -1))
        full = u + 7.5 * (u - u)
    torch.testing.assert_close(got, full, rtol=0, atol=0)


def test_cfg_with_distinct_embeddings_and_rescale():
    net = _tiny_net()
    net.set_sampling_parameters(10, batch_size=2, num_reconstructions=2)
    gen = torch.Generator().manual_seed(5)
    pos = torch.randn(2, 5, 24, generator=gen)
    neg = torch.randn(2, 5, 24, generator=gen)
    net.set_condition(StableDiffusionCondition(prompt=None, prompt_embeds=pos,
                                               negative_prompt_embeds=neg, guidance_scale=3.0,
                                               guidance_rescale=0.7))
    z = torch.randn(4, 4, 8, 8)  # batch 2 x R 2, flat row b*R + r
    with torch.no_grad():
        got = net(z, 31)
        c = net.unet(z, 31, pos.repeat_interleave(2, 0))
        u = net.unet(z, 31, neg.repeat_interleave(2, 0))
        ref = rescale_noise_cfg(u + 3.0 * (c - u), c, 0.7)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-5)  # batch-2B GEMMs vs two B ones


def test_tiny_latent_network_roundtrip_shapes():
    net = _tiny_net()
    assert net.get_latent_shape((3, 16, 16)) == (4, 8, 8)
    with pytest.raises(ValueError):
        net.get_latent_shape((3, 15, 16))
    x = torch.rand(1, 3, 16, 16) * 2 - 1
    z = net.encode(x)
    assert z.shape == (1, 4, 8, 8) and net.decode(z).shape == x.shape

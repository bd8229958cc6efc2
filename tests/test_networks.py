"""Prior modules on the CPU: architecture sizes, diffusers-compatible parameter names, the
fused-norm layer's CPU semantics."""

import pytest
import torch

from samplers_amd.networks.layers import GroupNormAct, Linear, linear
from samplers_amd.networks.unet2d import CELEBAHQ_256, UNet2DConfig, UNet2DModel, build_unet, count_parameters
from samplers_amd.networks.vae import SD15_VAE, AutoencoderKL


def test_group_norm_act_cpu_is_torch():
    layer = GroupNormAct(4, 8, eps=1e-6, act=True)
    ref = torch.nn.GroupNorm(4, 8, eps=1e-6)
    with torch.no_grad():
        layer.weight.uniform_(0.5, 1.5), layer.bias.uniform_(-0.5, 0.5)
    ref.load_state_dict(layer.state_dict())
    x, cb = torch.randn(3, 8, 5, 6), torch.randn(3, 8)
    torch.testing.assert_close(layer(x, cb), torch.nn.functional.silu(ref(x + cb[:, :, None, None])))
    layer.act = False
    torch.testing.assert_close(layer(x), ref(x))


def test_linear_cpu_is_nn_linear():
    """``layers.Linear`` keeps nn.Linear's parameters / state-dict keys and, off the GPU,
    its exact forward and input gradient; ``linear`` with an explicit 2-D view of a 1x1
    conv weight (proj_in / proj_out) is F.linear on that view."""
    torch.manual_seed(0)
    lin, ref = Linear(12, 7), torch.nn.Linear(12, 7)
    ref.load_state_dict(lin.state_dict())
    assert list(lin.state_dict()) == ["weight", "bias"]
    x = torch.randn(2, 5, 12, requires_grad=True)
    xr = x.detach().clone().requires_grad_(True)
    y, yr = lin(x), ref(xr)
    assert torch.equal(y, yr)
    y.square().sum().backward(), yr.square().sum().backward()
    assert torch.equal(x.grad, xr.grad)
    conv = torch.nn.Conv2d(12, 7, 1)
    out = linear(x.detach(), conv, conv.weight.view(7, 12), conv.bias)
    assert torch.equal(out, torch.nn.functional.linear(x.detach(), conv.weight.view(7, 12), conv.bias))


def test_unet_size_and_names():
    with torch.device("meta"):
        net = UNet2DModel(CELEBAHQ_256)
    assert abs(count_parameters(net) - 113.7e6) < 0.1e6
    keys = set(net.state_dict())
    for k in ("conv_in.weight", "time_embedding.linear_1.weight",
              "down_blocks.0.resnets.0.norm1.weight", "down_blocks.4.attentions.0.to_q.weight",
              "mid_block.attentions.0.group_norm.weight", "up_blocks.5.resnets.2.conv_shortcut.weight",
              "conv_norm_out.bias", "conv_out.weight"):
        assert k in keys, k


def test_vae_size():
    with torch.device("meta"):
        vae = AutoencoderKL(SD15_VAE)
    assert abs(count_parameters(vae) - 83.65e6) < 0.05e6


def test_tiny_unet_shapes_and_determinism():
    cfg = UNet2DConfig(sample_size=16, block_out_channels=(16, 32), attention_levels=(1,),
                       norm_num_groups=8)
    a, b = build_unet(cfg, seed=1), build_unet(cfg, seed=1)
    x = torch.randn(2, 3, 16, 16)
    ya = a(x, 10)
    assert ya.shape == x.shape
    torch.testing.assert_close(ya, b(x, torch.tensor([10])))


def test_from_pretrained_loads_a_local_diffusers_layout_checkpoint(tmp_path):
    """f4: ``DDPMNetwork.from_pretrained(local_dir)`` (the reference loads by hub name,
    ``ddpm.py:22-38``): a safetensors state dict with diffusers key names — including the
    legacy attention names query/key/value/proj_attn — plus unet/config.json and
    scheduler/scheduler_config.json round-trip to the same module and outputs."""
    import json

    from safetensors.torch import save_file

    from samplers_amd.networks.ddpm import DDPMNetwork
    from samplers_amd.networks.unet2d import UNet2DConfig, build_unet

    cfg = UNet2DConfig(sample_size=16, block_out_channels=(32, 64), attention_levels=(1,),
                       layers_per_block=1)
    src = build_unet(cfg, seed=3)
    state = {}
    for k, v in src.state_dict().items():
        k = (k.replace(".to_q.", ".query.").replace(".to_k.", ".key.")
             .replace(".to_v.", ".value.").replace(".to_out.0.", ".proj_attn."))
        state[k] = v.contiguous()
    (tmp_path / "unet").mkdir()
    (tmp_path / "scheduler").mkdir()
    save_file(state, str(tmp_path / "unet" / "diffusion_pytorch_model.safetensors"))
    (tmp_path / "unet" / "config.json").write_text(json.dumps({
        "sample_size": 16, "in_channels": 3, "out_channels": 3, "block_out_channels": [32, 64],
        "down_block_types": ["DownBlock2D", "AttnDownBlock2D"], "layers_per_block": 1,
        "norm_num_groups": 32, "norm_eps": 1e-6, "freq_shift": 1, "flip_sin_to_cos": False}))
    (tmp_path / "scheduler" / "scheduler_config.json").write_text(json.dumps({
        "num_train_timesteps": 1000, "beta_start": 1e-4, "beta_end": 0.02,
        "beta_schedule": "linear"}))
    net = DDPMNetwork.from_pretrained(str(tmp_path))
    for (ka, a), (kb, b) in zip(src.state_dict().items(), net.unet.state_dict().items()):
        assert ka == kb and torch.equal(a, b)
    net.set_sampling_parameters(10)
    x = torch.randn(2, 3, 16, 16, generator=torch.Generator().manual_seed(0))
    with torch.no_grad():
        assert torch.equal(net(x, 500), src(x, 500))
    assert torch.allclose(net.alphas_cumprod[1:], torch.cumprod(1 - torch.linspace(1e-4, 0.02, 1000), 0).clip(1e-6, 1))


def test_from_pretrained_never_fetches(tmp_path):
    import pytest

    from samplers_amd.networks.ddpm import DDPMNetwork

    with pytest.raises(FileNotFoundError, match="never fetches"):
        DDPMNetwork.from_pretrained("google/ddpm-celebahq-256", cache_dir=str(tmp_path))


def test_batched_time_embedding_projections_equal_per_block():
    """unet2d.temb_projections: every ResnetBlock's time_emb_proj(silu(temb)) from one batched
    GEMM per projection width equals the per-block nn.Linear (to fp32 rounding), contiguous
    [B, C] per block; the whole UNet forward agrees with the per-block path; trainable
    projections fall back to the per-block path (gradients reach the parameters)."""
    import torch.nn.functional as F

    from samplers_amd.networks.unet2d import ResnetBlock2D, UNet2DConfig, build_unet, temb_projections

    cfg = UNet2DConfig(sample_size=16, block_out_channels=(32, 64), attention_levels=(1,),
                       layers_per_block=1)
    net = build_unet(cfg, seed=1)
    emb = net.time_embedding(torch.randn(3, 32))
    tbs = temb_projections(net, emb)
    blocks = [m for m in net.modules() if isinstance(m, ResnetBlock2D) and m.time_emb_proj is not None]
    assert len(tbs) == len(blocks) > 0
    for b in blocks:
        ref = b.time_emb_proj(F.silu(emb))
        assert tbs[id(b)].is_contiguous() and tbs[id(b)].shape == ref.shape
        torch.testing.assert_close(tbs[id(b)], ref, rtol=1e-6, atol=1e-6)
    x = torch.randn(3, 3, 16, 16)
    y = net(x, 321)
    blocks[0].time_emb_proj.weight.requires_grad_(True)  # -> per-block path
    assert temb_projections(net, emb) == {}
    y2 = net(x, 321)
    torch.testing.assert_close(y, y2, rtol=1e-5, atol=1e-5)


def test_score_gemm_chunks_equal_plain_bmm():
    """unet2d.score_gemm: query-row chunks (k repeated per chunk) give alpha q kᵀ for strided
    q / k views (the thirds of a fused projection), at the chunk counts the size rule picks."""
    from samplers_amd.networks.unet2d import _score_chunks, score_gemm

    assert _score_chunks(1, 256, 256) == 8 and _score_chunks(64, 256, 256) == 4
    assert _score_chunks(2, 4096, 4096) == 1
    g = torch.Generator().manual_seed(2)
    for b, n, d in ((1, 256, 64), (2, 64, 32), (40, 64, 16)):
        qkv = torch.randn(b, n, 3 * d, generator=g)
        q, k, _ = qkv.split(d, dim=-1)
        out = torch.empty(b, n, n)
        score_gemm(q, k, 0.25, out)
        torch.testing.assert_close(out, 0.25 * q @ k.transpose(1, 2), rtol=1e-5, atol=1e-5)


def _tiny_sd_dir(tmp_path, legacy_vae: bool):
    """A diffusers-layout SD directory with a tiny UNet2DConditionModel + AutoencoderKL, key
    names as diffusers writes them (``legacy_vae``: the VAE attention under the pre-0.14 names
    query / key / value / proj_attn with 1x1-conv-shaped weights, as older exports store it)."""
    import json

    from safetensors.torch import save_file

    from samplers_amd.networks.latent import LatentDiffusionNetwork
    from samplers_amd.networks.unet2d_condition import UNet2DConditionConfig
    from samplers_amd.networks.vae import VAEConfig

    ucfg = UNet2DConditionConfig(sample_size=8, block_out_channels=(32, 64), cross_attention_levels=(0,),
                                 layers_per_block=1, attention_heads=2, cross_attention_dim=24,
                                 norm_num_groups=8)
    vcfg = VAEConfig(block_out_channels=(16, 32), layers_per_block=1, norm_num_groups=8)
    src = LatentDiffusionNetwork.from_config(ucfg, vcfg, seed=5)
    for comp, mod in (("unet", src.unet), ("vae", src.vae)):
        (tmp_path / comp).mkdir()
        state = {}
        for k, v in mod.state_dict().items():
            if comp == "vae" and legacy_vae and ".attentions." in k:
                k = (k.replace(".to_q.", ".query.").replace(".to_k.", ".key.")
                     .replace(".to_v.", ".value.").replace(".to_out.0.", ".proj_attn."))
                if v.dim() == 2:
                    v = v[:, :, None, None]
            state[k] = v.contiguous()
        save_file(state, str(tmp_path / comp / "diffusion_pytorch_model.safetensors"))
    (tmp_path / "unet" / "config.json").write_text(json.dumps({
        "_class_name": "UNet2DConditionModel", "act_fn": "silu", "attention_head_dim": 2,
        "block_out_channels": [32, 64], "center_input_sample": False, "cross_attention_dim": 24,
        "down_block_types": ["CrossAttnDownBlock2D", "DownBlock2D"], "flip_sin_to_cos": True,
        "freq_shift": 0, "in_channels": 4, "layers_per_block": 1, "norm_eps": 1e-5,
        "norm_num_groups": 8, "out_channels": 4, "sample_size": 8,
        "up_block_types": ["UpBlock2D", "CrossAttnUpBlock2D"]}))
    (tmp_path / "vae" / "config.json").write_text(json.dumps({
        "_class_name": "AutoencoderKL", "act_fn": "silu", "block_out_channels": [16, 32],
        "in_channels": 3, "latent_channels": 4, "layers_per_block": 1, "norm_num_groups": 8,
        "out_channels": 3, "sample_size": 16}))
    (tmp_path / "scheduler").mkdir()
    (tmp_path / "scheduler" / "scheduler_config.json").write_text(json.dumps({
        "_class_name": "PNDMScheduler", "beta_end": 0.012, "beta_schedule": "scaled_linear",
        "beta_start": 0.00085, "num_train_timesteps": 1000, "set_alpha_to_one": False,
        "skip_prk_steps": True, "steps_offset": 1, "trained_betas": None}))
    return src, ucfg


@pytest.mark.parametrize("legacy_vae", [False, True])
def test_sd_from_pretrained_loads_a_local_diffusers_layout_checkpoint(tmp_path, legacy_vae):
    """f4 (stable_diffusion.py:89-105 loads the pipeline by hub name): ``unet/``, ``vae/`` and
    ``scheduler/`` of a local diffusers-layout directory round-trip to the same modules, ε,
    decode and encode, and the PNDM timestep list."""
    from samplers_amd.networks.latent import LatentDiffusionNetwork, StableDiffusionCondition

    src, ucfg = _tiny_sd_dir(tmp_path, legacy_vae)
    ctx = torch.randn(1, ucfg.context_tokens, 24, generator=torch.Generator().manual_seed(3))
    net = LatentDiffusionNetwork.from_pretrained(str(tmp_path), null_prompt_embeds=ctx)
    for a, b in ((src.unet, net.unet), (src.vae, net.vae)):
        sa, sb = a.state_dict(), b.state_dict()
        assert list(sa) == list(sb)
        for k in sa:
            assert torch.equal(sa[k], sb[k]), k
    assert torch.equal(net.alphas_cumprod, src.alphas_cumprod)
    assert torch.equal(net.null_prompt_embeds, ctx)
    src.null_prompt_embeds = ctx.clone()
    g = torch.Generator().manual_seed(4)
    z = torch.randn(2, 4, 8, 8, generator=g)
    x = torch.rand(2, 3, 16, 16, generator=g) * 2 - 1
    for m in (src, net):
        m.set_sampling_parameters(10, batch_size=1)
        m.set_condition(StableDiffusionCondition())
    with torch.no_grad():
        assert torch.equal(net(z, 501), src(z, 501))
        assert torch.equal(net.decode(z), src.decode(z))
        assert torch.equal(net.encode(x), src.encode(x))
    assert net.timesteps_host == src.timesteps_host


def test_sd_from_pretrained_never_fetches_and_rejects_unsupported(tmp_path):
    import json

    from samplers_amd.networks.latent import LatentDiffusionNetwork

    with pytest.raises(FileNotFoundError, match="never fetches"):
        LatentDiffusionNetwork.from_pretrained("runwayml/stable-diffusion-v1-5", cache_dir=str(tmp_path))
    _tiny_sd_dir(tmp_path, False)
    sch = tmp_path / "scheduler" / "scheduler_config.json"
    raw = json.loads(sch.read_text())
    sch.write_text(json.dumps(dict(raw, skip_prk_steps=False)))
    with pytest.raises(NotImplementedError, match="Runge-Kutta"):
        LatentDiffusionNetwork.from_pretrained(str(tmp_path))
    sch.write_text(json.dumps(dict(raw, prediction_type="v_prediction")))
    with pytest.raises(NotImplementedError, match="prediction_type"):
        LatentDiffusionNetwork.from_pretrained(str(tmp_path))


def test_sd_from_pretrained_without_null_embeds_refuses_empty_prompts(tmp_path):
    """real weights must not be conditioned on the synthetic null context — without
    ``null_prompt_embeds`` an empty prompt raises; prompt embeddings still work; a wrongly shaped
    null embedding is refused with a clear message (2-d (77, d) is accepted)."""
    from samplers_amd.networks.latent import LatentDiffusionNetwork, StableDiffusionCondition

    _, ucfg = _tiny_sd_dir(tmp_path, False)
    net = LatentDiffusionNetwork.from_pretrained(str(tmp_path))
    net.set_sampling_parameters(10, batch_size=1)
    with pytest.raises(ValueError, match="null_prompt_embeds"):
        net.set_condition(StableDiffusionCondition())
    pe = torch.randn(1, ucfg.context_tokens, 24)
    net.set_condition(StableDiffusionCondition(prompt=None, prompt_embeds=pe, guidance_scale=1.0))
    with pytest.raises(ValueError, match="CLIP embedding"):
        LatentDiffusionNetwork.from_pretrained(str(tmp_path), null_prompt_embeds=torch.randn(1, 5, 24))
    ok = LatentDiffusionNetwork.from_pretrained(str(tmp_path), null_prompt_embeds=pe[0])
    assert torch.equal(ok.null_prompt_embeds, pe)

"""Prior modules on the CPU: architecture sizes, diffusers-compatible parameter names, the
fused-norm layer's CPU semantics."""

import torch

from samplers_amd.networks.layers import GroupNormAct
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

"""Latent VAE: a structural equivalent of diffusers' ``AutoencoderKL`` (SD 1.5 config).

The reference reaches it through ``StableDiffusionNetwork._decode`` /
``_encode`` (``/root/reference/samplers/networks/diffusers/stable_diffusion.py:330-345``):
``decode(z) = vae.decode(z / scaling_factor)`` and ``encode(x) = posterior
mean * scaling_factor``.  Architecture (SD 1.5): 128/256/512/512 channels, 2
residual blocks per encoder level and 3 per decoder level, single-head
self-attention in both mid blocks, GroupNorm(32, eps=1e-6) + SiLU, 4 latent
channels, 8x spatial reduction; 83.65 M parameters with random weights (no
checkpoint offline).  Its 3x3 convolutions run on this project's fp32-MFMA tiles (Winograd,
stride-2, thin conv_in / conv_out), GroupNorm(+SiLU) and upsampling on HIP kernels, the
channel-changing 1x1 shortcuts on the split-bf16 GEMM; the mid
blocks' single-head attention and the 1x1 quant / post-quant convs are torch ops.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from .layers import Conv3x3, GroupNormAct, conv1x1_small
from .unet2d import Downsample2D, ResnetBlock2D, SpatialSelfAttention, Upsample2D, _as_nchw


@dataclass(frozen=True)
class VAEConfig:
    in_channels: int = 3
    out_channels: int = 3
    latent_channels: int = 4
    block_out_channels: tuple[int, ...] = (128, 256, 512, 512)
    layers_per_block: int = 2
    norm_num_groups: int = 32
    norm_eps: float = 1e-6
    scaling_factor: float = 0.18215


SD15_VAE = VAEConfig()


class _Block(nn.Module):
    def __init__(self) -> None:
        super().__init__()
        self.resnets = nn.ModuleList()


class _Mid(nn.Module):
    def __init__(self, ch: int, g: int, eps: float) -> None:
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch, None, g, eps), ResnetBlock2D(ch, ch, None, g, eps)])
        self.attentions = nn.ModuleList([SpatialSelfAttention(ch, g, eps, None)])

    def forward(self, x: Tensor) -> Tensor:
        return self.resnets[1](self.attentions[0](self.resnets[0](x)))


class Encoder(nn.Module):
    def __init__(self, c: VAEConfig) -> None:
        super().__init__()
        ch, g, eps = c.block_out_channels, c.norm_num_groups, c.norm_eps
        self.conv_in = Conv3x3(c.in_channels, ch[0])
        self.down_blocks = nn.ModuleList()
        cout = ch[0]
        for i, co in enumerate(ch):
            cin, cout = cout, co
            blk = _Block()
            for j in range(c.layers_per_block):
                blk.resnets.append(ResnetBlock2D(cin if j == 0 else cout, cout, None, g, eps))
            blk.downsamplers = nn.ModuleList([Downsample2D(cout)]) if i < len(ch) - 1 else None
            self.down_blocks.append(blk)
        self.mid_block = _Mid(ch[-1], g, eps)
        self.conv_norm_out = GroupNormAct(g, ch[-1], eps=eps, act=True)
        self.conv_out = Conv3x3(ch[-1], 2 * c.latent_channels)

    def forward(self, x: Tensor) -> Tensor:
        h = self.conv_in(x)
        for blk in self.down_blocks:
            for res in blk.resnets:
                h = res(h)
            if blk.downsamplers is not None:
                h = blk.downsamplers[0](h)
        h = self.mid_block(h)
        return self.conv_out(self.conv_norm_out(h))


class Decoder(nn.Module):
    def __init__(self, c: VAEConfig) -> None:
        super().__init__()
        ch, g, eps = c.block_out_channels, c.norm_num_groups, c.norm_eps
        rev = list(reversed(ch))
        self.conv_in = Conv3x3(c.latent_channels, rev[0])
        self.mid_block = _Mid(rev[0], g, eps)
        self.up_blocks = nn.ModuleList()
        prev = rev[0]
        for i, co in enumerate(rev):
            blk = _Block()
            for j in range(c.layers_per_block + 1):
                blk.resnets.append(ResnetBlock2D(prev if j == 0 else co, co, None, g, eps))
            blk.upsamplers = nn.ModuleList([Upsample2D(co)]) if i < len(rev) - 1 else None
            self.up_blocks.append(blk)
            prev = co
        self.conv_norm_out = GroupNormAct(g, ch[0], eps=eps, act=True)
        self.conv_out = Conv3x3(ch[0], c.out_channels)

    def forward(self, z: Tensor) -> Tensor:
        h = self.mid_block(self.conv_in(z))
        for blk in self.up_blocks:
            for res in blk.resnets:
                h = res(h)
            if blk.upsamplers is not None:
                h = blk.upsamplers[0](h)
        return self.conv_out(self.conv_norm_out(h))


class AutoencoderKL(nn.Module):
    """``encode`` -> posterior mean (unscaled), ``decode`` of unscaled latents."""

    def __init__(self, config: VAEConfig = SD15_VAE) -> None:
        super().__init__()
        self.config = config
        self.encoder = Encoder(config)
        self.decoder = Decoder(config)
        self.quant_conv = nn.Conv2d(2 * config.latent_channels, 2 * config.latent_channels, 1)
        self.post_quant_conv = nn.Conv2d(config.latent_channels, config.latent_channels, 1)

    @property
    def downscale(self) -> int:
        return 2 ** (len(self.config.block_out_channels) - 1)

    def encode_mean(self, x: Tensor) -> Tensor:
        moments = conv1x1_small(self.quant_conv, self.encoder(x))
        return _as_nchw(moments[:, : self.config.latent_channels])

    def decode(self, z: Tensor) -> Tensor:
        return _as_nchw(self.decoder(conv1x1_small(self.post_quant_conv, z)))


def build_vae(config: VAEConfig = SD15_VAE, *, seed: int = 0, device=None,
              dtype: torch.dtype = torch.float32) -> AutoencoderKL:
    state = torch.random.get_rng_state()
    torch.manual_seed(seed)
    try:
        vae = AutoencoderKL(config)
    finally:
        torch.random.set_rng_state(state)
    return vae.to(device=device, dtype=dtype).eval().requires_grad_(False)

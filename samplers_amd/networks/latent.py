"""Latent diffusion prior (the reference's ``StableDiffusionNetwork`` role).

Mirrors the parts of ``/root/reference/samplers/networks/diffusers/stable_diffusion.py``
that the latent samplers use: ``get_latent_shape`` (``:135-144``), ``_decode``
(``:330-336``: ``vae.decode(z / scaling_factor)``), ``_encode`` (``:338-345``:
posterior mean × ``scaling_factor``), the padded ``alphas_cumprod`` and an
ascending timestep buffer.

What differs, and why: the text encoder, classifier-free guidance and
IP-adapter paths (``set_condition``, ``forward`` CFG, ``:146-328``) need the
CLIP weights and tokenizer, which are not available offline; they are out of
the hot-path scope.  The ε-network is therefore an unconditional
latent UNet (``UNet2DModel`` over 4-channel latents).  The schedule is SD 1.5's
(scaled-linear betas 0.00085–0.012, ``steps_offset=1``) with PNDM's
``skip_prk_steps`` timestep list (the second-to-last timestep repeated); that
list is restated from diffusers' published algorithm and is not pinned by any
reference fixture (diffusers is absent) — "parity unpinned" for the schedule.
"""

from __future__ import annotations

import numpy as np
import torch
from torch import Tensor

from samplers_amd.dtypes import Device, DType, Shape

from .base import LatentEpsilonNetwork, NoCondition
from .ddpm import DDPMSchedule
from .unet2d import UNet2DConfig, UNet2DModel, build_unet
from .vae import SD15_VAE, AutoencoderKL, VAEConfig, build_vae

LATENT_UNET_64 = UNet2DConfig(sample_size=64, in_channels=4, out_channels=4,
                              block_out_channels=(128, 256, 512, 512), attention_levels=(1, 2),
                              layers_per_block=2, attention_head_dim=64)


def pndm_timesteps(num_inference_steps: int, num_train_timesteps: int = 1000,
                   steps_offset: int = 1) -> np.ndarray:
    """Descending PLMS timesteps of PNDMScheduler(skip_prk_steps=True)."""
    ratio = num_train_timesteps // num_inference_steps
    ts = (np.arange(0, num_inference_steps) * ratio).round().astype(np.int64) + steps_offset
    plms = np.concatenate([ts[:-1], ts[-2:-1], ts[-1:]])[::-1].copy()
    return plms


class LatentDiffusionNetwork(LatentEpsilonNetwork[NoCondition]):
    """ε-UNet over VAE latents."""

    def __init__(self, unet: UNet2DModel, vae: AutoencoderKL, *,
                 schedule: DDPMSchedule | None = None, pndm: bool = True) -> None:
        schedule = schedule or DDPMSchedule(beta_start=0.00085, beta_end=0.012,
                                            beta_schedule="scaled_linear", steps_offset=1)
        acp = schedule.alphas_cumprod
        super().__init__(alphas_cumprod=torch.cat([acp.new_tensor([1.0]), acp]))
        self.schedule, self.pndm = schedule, pndm
        self.unet = unet.eval().requires_grad_(False)
        self.vae = vae.eval().requires_grad_(False)
        self.scaling_factor = vae.config.scaling_factor
        self.latent_num_channels = vae.config.latent_channels
        self.latent_resolution_ratio = vae.downscale
        self.to(device=next(unet.parameters()).device)

    @classmethod
    def from_config(cls, unet_config: UNet2DConfig = LATENT_UNET_64,
                    vae_config: VAEConfig = SD15_VAE, *, seed: int = 0, device: Device = None,
                    torch_dtype: DType = None) -> "LatentDiffusionNetwork":
        dt = torch_dtype or torch.float32
        return cls(build_unet(unet_config, seed=seed, device=device, dtype=dt),
                   build_vae(vae_config, seed=seed + 1, device=device, dtype=dt))

    @classmethod
    def from_pretrained(cls, *args, **kwargs):
        raise NotImplementedError("no offline Stable Diffusion checkpoint; use from_config")

    def forward(self, latents: Tensor, t: Tensor | int) -> Tensor:
        if self._num_sampling_steps is None:
            raise RuntimeError("Call `set_sampling_parameters()` before sampling.")
        return self.unet(latents, t)

    def set_sampling_parameters(self, num_sampling_steps: int, batch_size: int = 1,
                                num_reconstructions: int = 1):
        self._batch_size = batch_size
        self._num_sampling_steps = num_sampling_steps
        self._num_reconstructions = num_reconstructions
        if self.pndm:
            ts = torch.from_numpy(pndm_timesteps(num_sampling_steps,
                                                 self.schedule.num_train_timesteps,
                                                 self.schedule.steps_offset))
        else:
            ts = self.schedule.set_timesteps(num_sampling_steps)
        self._set_timesteps_buffer(torch.flip(ts, dims=(0,)))

    def get_latent_shape(self, x_shape: Shape) -> Shape:
        c, h, w = x_shape
        f = self.latent_resolution_ratio
        if h % f or w % f:
            raise ValueError(f"Height and width must be divisible by {f} (got {h}x{w}).")
        return (self.latent_num_channels, h // f, w // f)

    def _decode(self, z: Tensor, *, differentiable: bool = False) -> Tensor:
        return self.vae.decode(z / self.scaling_factor)

    def _encode(self, x: Tensor, *, differentiable: bool = False) -> Tensor:
        return self.vae.encode_mean(x) * self.scaling_factor

    @property
    def is_condition_initialized(self) -> bool:
        return True

    def to(self, *args, **kwargs):
        super().to(*args, **kwargs)
        self._acp_host = None
        return self

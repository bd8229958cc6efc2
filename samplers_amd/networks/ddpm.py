"""Pixel-space DDPM prior (mirrors ``/root/reference/samplers/networks/diffusers/ddpm.py``).

The reference adapts a diffusers ``DDPMPipeline`` (UNet2DModel + DDPMScheduler).
Here the scheduler arithmetic is restated (linear betas, ``leading`` timestep
spacing, the diffusers defaults for ``google/ddpm-celebahq-256``) and the UNet
is :mod:`samplers_amd.networks.unet2d`.  The reference's index convention is
kept exactly: ``alphas_cumprod = cat([1.0], scheduler.alphas_cumprod)`` while
the UNet is called with the raw scheduler timestep, so
``predict_x0`` at timestep t uses diffusers' alpha_bar[t-1].
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Any

import numpy as np
import torch
from torch import Tensor

from samplers_amd.dtypes import Device, DType

from .base import EpsilonNetwork, NoCondition
from .unet2d import CELEBAHQ_256, UNet2DConfig, UNet2DModel, build_unet


@dataclass
class DDPMSchedule:
    """Noise schedule + ``set_timesteps`` of diffusers' ``DDPMScheduler`` (defaults)."""

    num_train_timesteps: int = 1000
    beta_start: float = 1e-4
    beta_end: float = 0.02
    beta_schedule: str = "linear"
    steps_offset: int = 0

    def __post_init__(self) -> None:
        if self.beta_schedule == "linear":
            betas = torch.linspace(self.beta_start, self.beta_end, self.num_train_timesteps,
                                   dtype=torch.float32)
        elif self.beta_schedule == "scaled_linear":
            betas = torch.linspace(self.beta_start**0.5, self.beta_end**0.5,
                                   self.num_train_timesteps, dtype=torch.float32) ** 2
        else:
            raise ValueError(f"unsupported beta_schedule {self.beta_schedule!r}")
        self.betas = betas
        self.alphas_cumprod = torch.cumprod(1.0 - betas, dim=0)
        self.timesteps = torch.arange(self.num_train_timesteps - 1, -1, -1, dtype=torch.long)

    def set_timesteps(self, num_inference_steps: int) -> Tensor:
        """Descending timesteps with ``leading`` spacing: ``arange(N) * (T // N)`` reversed."""
        if num_inference_steps > self.num_train_timesteps:
            raise ValueError("num_inference_steps cannot exceed num_train_timesteps")
        ratio = self.num_train_timesteps // num_inference_steps
        ts = (np.arange(0, num_inference_steps) * ratio).round()[::-1].copy().astype(np.int64)
        self.timesteps = torch.from_numpy(ts + self.steps_offset)
        return self.timesteps


class DDPMNetwork(EpsilonNetwork[NoCondition]):
    """ε-network over a pixel-space UNet and a DDPM schedule."""

    # its UNet runs on this project's kernels and torch's caching allocator only, so a DPS step
    # over it can be captured into a hipGraph (DPSSampler(graph=True); the automatic replay rule,
    # dps.graph_auto, is off: GRAPH_AUTO_MAX_BATCH = 0, replay measured slower at every batch)
    graph_capturable = True

    def __init__(self, unet: UNet2DModel, schedule: DDPMSchedule | None = None):
        schedule = schedule or DDPMSchedule()
        acp = schedule.alphas_cumprod
        super().__init__(alphas_cumprod=torch.cat([acp.new_tensor([1.0]), acp]))
        self.schedule = schedule
        self.unet = unet.eval().requires_grad_(False)
        self.to(device=next(unet.parameters()).device)

    @classmethod
    def from_config(cls, config: UNet2DConfig = CELEBAHQ_256, *, seed: int = 0,
                    device: Device = None, torch_dtype: DType = None,
                    schedule: DDPMSchedule | None = None) -> "DDPMNetwork":
        """Random-weight prior with the architecture of ``config`` (fixed seed)."""
        unet = build_unet(config, seed=seed, device=device, dtype=torch_dtype or torch.float32)
        return cls(unet, schedule)

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: str, cache_dir: str | None = None,
                        torch_dtype: DType = None, device: Device = None,
                        **pipeline_kwargs: Any) -> "DDPMNetwork":
        """Load a diffusers-layout checkpoint from a LOCAL directory.

        Expects ``unet/diffusion_pytorch_model.safetensors`` (+ optional
        ``unet/config.json`` and ``scheduler/scheduler_config.json``).  Nothing
        is downloaded: a hub name without a local copy raises ``FileNotFoundError``.
        """
        from .checkpoint import load_state, meta_module, read_json, resolve_root, weights_path

        root = resolve_root(pretrained_model_name_or_path, cache_dir, ("unet",),
                            pipeline_kwargs.get("variant"), "DDPMNetwork.from_config")
        config = CELEBAHQ_256
        raw = read_json(root / "unet" / "config.json")
        if raw:
            attn = tuple(i for i, t in enumerate(raw.get("down_block_types", [])) if "Attn" in t)
            config = UNet2DConfig(
                sample_size=raw.get("sample_size", 256),
                in_channels=raw.get("in_channels", 3),
                out_channels=raw.get("out_channels", 3),
                block_out_channels=tuple(raw.get("block_out_channels", config.block_out_channels)),
                attention_levels=attn or config.attention_levels,
                layers_per_block=raw.get("layers_per_block", 2),
                norm_num_groups=raw.get("norm_num_groups", 32),
                norm_eps=raw.get("norm_eps", 1e-6),
                freq_shift=raw.get("freq_shift", 1),
                flip_sin_to_cos=raw.get("flip_sin_to_cos", False),
                attention_head_dim=raw.get("attention_head_dim"),
            )
        schedule = DDPMSchedule()
        raw = read_json(root / "scheduler" / "scheduler_config.json")
        if raw:
            schedule = DDPMSchedule(
                num_train_timesteps=raw.get("num_train_timesteps", 1000),
                beta_start=raw.get("beta_start", 1e-4), beta_end=raw.get("beta_end", 0.02),
                beta_schedule=raw.get("beta_schedule", "linear"),
                steps_offset=raw.get("steps_offset", 0),
            )
        unet = meta_module(UNet2DModel, config)
        load_state(unet, weights_path(root, "unet", pipeline_kwargs.get("variant")),
                   dtype=torch_dtype or torch.float32)
        unet = unet.to(device=device)
        return cls(unet, schedule)

    def forward(self, sample: Tensor, t: Tensor | int) -> Tensor:
        if self._num_sampling_steps is None:
            raise RuntimeError("Call `set_sampling_parameters()` before sampling.")
        return self.unet(sample, t)

    def set_sampling_parameters(self, num_sampling_steps: int, batch_size: int = 1,
                                num_reconstructions: int = 1):
        self._batch_size = batch_size
        self._num_sampling_steps = num_sampling_steps
        self._num_reconstructions = num_reconstructions
        ts = self.schedule.set_timesteps(num_sampling_steps)
        # bridge kernels need ascending timesteps (s < t < ell), ddpm.py:55-58
        self._set_timesteps_buffer(torch.flip(ts, dims=(0,)))

    @property
    def is_condition_initialized(self) -> bool:
        return True

    @property
    def dtype(self) -> torch.dtype:
        """The prior's parameter dtype, as the reference's ``_pipeline.dtype`` (``ddpm.py:86-89``):
        ``from_config`` / ``from_pretrained(torch_dtype=torch.bfloat16)`` gives a bf16 network."""
        return next(self.unet.parameters()).dtype

    def to(self, *args, **kwargs):
        super().to(*args, **kwargs)
        self._acp_host = None
        return self

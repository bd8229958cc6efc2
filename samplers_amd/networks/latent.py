"""Latent diffusion prior (the reference's ``StableDiffusionNetwork`` role).

Mirrors ``/root/reference/samplers/networks/diffusers/stable_diffusion.py``:
``get_latent_shape`` (``:135-144``), ``set_condition`` (``:146-293``: input checks, the
batch-size check, per-reconstruction repetition of the embeddings, classifier-free
guidance), ``forward`` (``:295-328``: CFG batch doubling, ``u + s·(c − u)``, optional
guidance rescale), ``_decode`` (``:330-336``: ``vae.decode(z / scaling_factor)``),
``_encode`` (``:338-345``: posterior mean × ``scaling_factor``), the padded
``alphas_cumprod`` and an ascending timestep buffer.

The ε-network is the SD 1.5 ``UNet2DConditionModel`` structure
(``unet2d_condition.py``, 859.5 M parameters) over 4x64x64 latents, cross-attending to a
77 x 768 context.  What differs, and why:

* no text encoder (CLIP weights are not available offline; SURVEY.md §2 keeps it out of
  scope): conditions are given as ``prompt_embeds`` / ``negative_prompt_embeds``; the
  empty prompt ``""`` maps to a fixed synthetic null context (``null_context``), any other
  prompt string raises ``NotImplementedError``; IP-adapter inputs likewise;
* CFG with identical conditional and unconditional contexts (the reference's default
  ``StableDiffusionCondition()``: prompt ``""``, no negative prompt, guidance 7.5) is
  evaluated as a single pass: ``u + s·(c − u)`` with ``c = u`` is exactly ``u``, and the
  guidance rescale of identical tensors is the identity, so the result is the same and
  the doubled batch is skipped;
* the schedule is SD 1.5's (scaled-linear betas 0.00085–0.012, ``steps_offset=1``) with
  PNDM's ``skip_prk_steps`` timestep list, restated from diffusers' published algorithm
  and not pinned by any reference fixture (diffusers is absent) — "parity unpinned".

An unconditional ``UNet2DModel`` prior (``UNet2DConfig``) is still accepted (small test
priors); it ignores the context.
"""

from __future__ import annotations

import dataclasses
from typing import Any

import numpy as np
import torch
from torch import Tensor

from samplers_amd.dtypes import Device, DType, Shape

from .base import LatentEpsilonNetwork
from .ddpm import DDPMSchedule
from .unet2d import UNet2DConfig, UNet2DModel, build_unet
from .unet2d_condition import (SD15_UNET, UNet2DConditionConfig, UNet2DConditionModel,
                               build_unet_condition, null_context)
from .vae import SD15_VAE, AutoencoderKL, VAEConfig, build_vae

# the round-1 unconditional latent prior (kept for small CPU/GPU tests)
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


@dataclasses.dataclass(slots=True)
class StableDiffusionCondition:
    """Same fields as the reference's (``stable_diffusion.py:14-33``)."""

    prompt: str | list[str] | None = ""
    negative_prompt: str | list[str] | None = None
    guidance_scale: float = 7.5
    guidance_rescale: float = 0.0
    prompt_embeds: Tensor | None = None
    negative_prompt_embeds: Tensor | None = None
    clip_skip: int | None = None
    cross_attention_kwargs: dict[str, Any] | None = None
    ip_adapter_image: Any = None
    ip_adapter_image_embeds: list[Tensor] | None = None


@dataclasses.dataclass(slots=True)
class ConditioningState:
    """Per-run tensors (``stable_diffusion.py:36-47``).  ``prompt_embeds`` holds the
    unconditional rows first when CFG runs (``cat([negative, positive])``), and may have one
    row shared by the whole batch."""

    prompt_embeds: Tensor
    do_classifier_free_guidance: bool
    guidance_scale: float
    guidance_rescale: float


def rescale_noise_cfg(noise_cfg: Tensor, noise_pred_text: Tensor, guidance_rescale: float) -> Tensor:
    """Guidance rescale of arXiv:2305.08891 §3.4 (diffusers' ``rescale_noise_cfg``)."""
    dims = list(range(1, noise_pred_text.ndim))
    std_text = noise_pred_text.std(dim=dims, keepdim=True)
    std_cfg = noise_cfg.std(dim=dims, keepdim=True)
    rescaled = noise_cfg * (std_text / std_cfg)
    return guidance_rescale * rescaled + (1 - guidance_rescale) * noise_cfg


class LatentDiffusionNetwork(LatentEpsilonNetwork[StableDiffusionCondition]):
    """ε-UNet over VAE latents (SD 1.5 structure)."""

    def __init__(self, unet: UNet2DConditionModel | UNet2DModel, vae: AutoencoderKL, *,
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
        self.conditional = isinstance(unet, UNet2DConditionModel)
        dev = next(unet.parameters()).device
        if self.conditional:
            self.register_buffer("null_prompt_embeds", null_context(unet.config, device=dev))
        self._conditioning: ConditioningState | None = None
        self.to(device=dev)

    @classmethod
    def from_config(cls, unet_config: UNet2DConditionConfig | UNet2DConfig = SD15_UNET,
                    vae_config: VAEConfig = SD15_VAE, *, seed: int = 0, device: Device = None,
                    torch_dtype: DType = None) -> "LatentDiffusionNetwork":
        dt = torch_dtype or torch.float32
        if isinstance(unet_config, UNet2DConditionConfig):
            unet = build_unet_condition(unet_config, seed=seed, device=device, dtype=dt)
        else:
            unet = build_unet(unet_config, seed=seed, device=device, dtype=dt)
        return cls(unet, build_vae(vae_config, seed=seed + 1, device=device, dtype=dt))

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: str, cache_dir: str | None = None,
                        torch_dtype: DType = None, device: Device = None, *,
                        variant: str | None = None, null_prompt_embeds: Tensor | None = None,
                        **pipeline_kwargs: Any) -> "LatentDiffusionNetwork":
        """Load a diffusers-layout Stable Diffusion checkpoint from a LOCAL directory
        (``stable_diffusion.py:89-105`` loads the pipeline by hub name).

        Reads ``unet/`` and ``vae/`` (``diffusion_pytorch_model[.variant].safetensors`` +
        ``config.json``) and ``scheduler/scheduler_config.json`` (PNDM with
        ``skip_prk_steps``, DDIM or DDPM, ``leading`` spacing); nothing is downloaded, so a hub
        name without a local copy raises ``FileNotFoundError``.  The text encoder is not read
        (out of scope, module doc): conditions come as ``prompt_embeds``, and the empty prompt
        maps to ``null_prompt_embeds`` — the caller's CLIP embedding of ``""`` (77 x 768 or
        1 x 77 x 768); without it an empty prompt raises (the synthetic null context stands in
        for random weights only).  Weights are computed in fp32 unless ``torch_dtype``
        says otherwise (fp16 variants are upcast)."""
        from .checkpoint import load_state, meta_module, read_json, resolve_root, weights_path

        root = resolve_root(pretrained_model_name_or_path, cache_dir, ("unet", "vae"), variant,
                            "LatentDiffusionNetwork.from_config")
        dt = torch_dtype or torch.float32
        unet_config = unet_condition_config_from_json(read_json(root / "unet" / "config.json"))
        vae_config = vae_config_from_json(read_json(root / "vae" / "config.json"))
        schedule, pndm = schedule_from_json(read_json(root / "scheduler" / "scheduler_config.json"))
        unet = meta_module(UNet2DConditionModel, unet_config)
        load_state(unet, weights_path(root, "unet", variant), dtype=dt)
        vae = meta_module(AutoencoderKL, vae_config)
        load_state(vae, weights_path(root, "vae", variant), dtype=dt)
        net = cls(unet.to(device=device), vae.to(device=device), schedule=schedule, pndm=pndm)
        if null_prompt_embeds is None:
            # real weights with the synthetic null context would condition every empty prompt on
            # a random tensor: empty prompts raise until real embeddings are supplied (_embed)
            net._null_context_synthetic = True
        else:
            want = tuple(net.null_prompt_embeds.shape)
            got = tuple(null_prompt_embeds.shape)
            if got[-2:] != want[-2:] or null_prompt_embeds.numel() != want[1] * want[2]:
                raise ValueError(f"null_prompt_embeds: expected the CLIP embedding of '' as ({want[1]}, {want[2]}) "
                                 f"or (1, {want[1]}, {want[2]}), got {got}")
            net.null_prompt_embeds = null_prompt_embeds.reshape(want).to(
                device=net.null_prompt_embeds.device, dtype=dt)
        return net

    # -- conditioning --------------------------------------------------------------------

    def _embed(self, prompt, what: str) -> Tensor:
        """Embeddings of a prompt: only the empty prompt has one offline (the null context)."""
        prompts = [prompt] if isinstance(prompt, str) else list(prompt)
        if any(p != "" for p in prompts):
            raise NotImplementedError(
                f"no text encoder offline: pass {what}_embeds instead of a non-empty {what}")
        if getattr(self, "_null_context_synthetic", False):
            raise ValueError(
                f"this network was loaded from a checkpoint without null_prompt_embeds: the empty {what} "
                "needs the CLIP embedding of '' (pass null_prompt_embeds= to from_pretrained, or "
                f"{what}_embeds in the condition); the synthetic null context is for random weights only")
        return self.null_prompt_embeds.expand(len(prompts), -1, -1)

    def set_condition(self, condition: StableDiffusionCondition | None) -> None:
        """``stable_diffusion.py:146-293`` without the text encoder (see the module doc)."""
        if not self.are_sampling_parameters_initialized:
            raise RuntimeError("Call `set_sampling_parameters()` before conditioning.")
        condition = condition if condition is not None else StableDiffusionCondition()
        if condition.prompt is not None and condition.prompt_embeds is not None:
            raise ValueError("Cannot forward both `prompt` and `prompt_embeds`.")
        if condition.prompt is None and condition.prompt_embeds is None:
            raise ValueError("Provide either `prompt` or `prompt_embeds`.")
        if condition.negative_prompt is not None and condition.negative_prompt_embeds is not None:
            raise ValueError("Cannot forward both `negative_prompt` and `negative_prompt_embeds`.")
        if condition.ip_adapter_image is not None or condition.ip_adapter_image_embeds is not None:
            raise NotImplementedError("IP-adapter conditioning is out of scope (SURVEY.md §2)")

        if isinstance(condition.prompt, str):
            batch_size = 1
        elif isinstance(condition.prompt, list):
            batch_size = len(condition.prompt)
        else:
            batch_size = condition.prompt_embeds.shape[0]
        if batch_size != self._batch_size:
            raise ValueError(
                f"Batch size mismatch: received {batch_size} prompt(s) but the sampler was "
                f"initialised with batch_size={self._batch_size}. Supply exactly this number "
                "of prompts/embeddings, or call 'set_sampling_parameters' again.")
        if not self.conditional:
            self._conditioning = ConditioningState(self.alphas_cumprod.new_zeros(0), False, 1.0, 0.0)
            return

        dev, dt = self.device, self.alphas_cumprod.dtype
        if condition.prompt_embeds is not None:
            pos = condition.prompt_embeds.to(device=dev, dtype=dt)
        else:
            pos = self._embed(condition.prompt, "prompt")
        do_cfg = condition.guidance_scale > 1.0
        neg = None
        if do_cfg:
            if condition.negative_prompt_embeds is not None:
                neg = condition.negative_prompt_embeds.to(device=dev, dtype=dt)
            else:
                negp = condition.negative_prompt if condition.negative_prompt is not None else ""
                if isinstance(negp, str):
                    negp = [negp] * batch_size
                neg = self._embed(negp, "negative_prompt")
            if neg.shape != pos.shape:
                raise ValueError(f"negative_prompt_embeds {tuple(neg.shape)} and prompt_embeds "
                                 f"{tuple(pos.shape)} must have the same shape")
        # identical rows everywhere: keep one row and let the attention broadcast it
        shared = bool((pos == pos[:1]).all())
        if do_cfg and torch.equal(neg, pos):
            do_cfg, neg = False, None  # u + s (c - u) with c == u is u (module doc)
        if shared and neg is None:
            embeds = pos[:1].contiguous()
        else:
            r = self._num_reconstructions or 1
            pos = pos.repeat_interleave(r, dim=0)  # num_images_per_prompt (diffusers layout)
            embeds = pos if neg is None else torch.cat([neg.repeat_interleave(r, dim=0), pos])
        self._conditioning = ConditioningState(embeds.contiguous(), do_cfg,
                                               float(condition.guidance_scale),
                                               float(condition.guidance_rescale))

    @property
    def is_condition_initialized(self) -> bool:
        return self._conditioning is not None

    @property
    def dtype(self) -> torch.dtype:
        """The priors' parameter dtype, as the reference's ``_pipeline.dtype``
        (``stable_diffusion.py:353-356``): ``torch_dtype=torch.bfloat16`` gives a bf16 network."""
        return next(self.unet.parameters()).dtype

    def clear_condition(self):
        self._conditioning = None

    # -- ε and the VAE ---------------------------------------------------------------------

    def forward(self, latents: Tensor, t: Tensor | int) -> Tensor:
        if self._num_sampling_steps is None:
            raise RuntimeError("Call `set_sampling_parameters()` before sampling.")
        if not self.conditional:
            return self.unet(latents, t)
        if not self.is_condition_initialized:
            raise RuntimeError("Call `set_condition()` before sampling.")
        state = self._conditioning
        if not state.do_classifier_free_guidance:
            return self.unet(latents, t, state.prompt_embeds)
        noise = self.unet(torch.cat([latents, latents]), t, state.prompt_embeds)
        uncond, text = noise.chunk(2)
        out = uncond + state.guidance_scale * (text - uncond)
        if state.guidance_rescale > 0.0:
            out = rescale_noise_cfg(out, text, state.guidance_rescale)
        return out

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

    def to(self, *args, **kwargs):
        super().to(*args, **kwargs)
        self._acp_host = None
        return self


# ---------------------------------------------------------------------------------------------
# diffusers config.json -> this build's configs (from_pretrained)
# ---------------------------------------------------------------------------------------------

def _only(raw: dict, key: str, allowed, what: str) -> None:
    if key in raw and raw[key] not in allowed:
        raise NotImplementedError(f"{what}: {key}={raw[key]!r} is not supported (supported: {allowed})")


def unet_condition_config_from_json(raw: dict) -> UNet2DConditionConfig:
    """diffusers ``UNet2DConditionModel`` config -> ``UNet2DConditionConfig`` (SD 1.x layout:
    CrossAttnDownBlock2D levels, conv ``proj_in`` / ``proj_out``, one head count).  Missing keys
    take SD 1.5's values; other architectures raise ``NotImplementedError``."""
    d = SD15_UNET
    if not raw:
        return d
    what = "unet/config.json"
    _only(raw, "act_fn", ("silu",), what)
    _only(raw, "use_linear_projection", (False,), what)
    _only(raw, "center_input_sample", (False,), what)
    _only(raw, "mid_block_type", ("UNetMidBlock2DCrossAttn", None), what)
    _only(raw, "class_embed_type", (None,), what)
    _only(raw, "addition_embed_type", (None,), what)
    _only(raw, "upcast_attention", (False, None), what)
    _only(raw, "time_embedding_type", ("positional",), what)
    for key in ("transformer_layers_per_block", "layers_per_block", "cross_attention_dim"):
        if isinstance(raw.get(key), (list, tuple)):
            raise NotImplementedError(f"{what}: per-level {key} is not supported")
    heads = raw.get("num_attention_heads") or raw.get("attention_head_dim", d.attention_heads)
    if isinstance(heads, (list, tuple)):
        if len(set(heads)) != 1:
            raise NotImplementedError(f"{what}: per-level head counts {heads} are not supported")
        heads = heads[0]
    down = raw.get("down_block_types")
    levels = d.cross_attention_levels
    if down is not None:
        levels = tuple(i for i, t in enumerate(down) if t.startswith("CrossAttn"))
        up = raw.get("up_block_types")
        if up is not None and tuple(i for i, t in enumerate(reversed(up)) if t.startswith("CrossAttn")) != levels:
            raise NotImplementedError(f"{what}: up blocks do not mirror the down blocks")
    return UNet2DConditionConfig(
        sample_size=raw.get("sample_size", d.sample_size),
        in_channels=raw.get("in_channels", d.in_channels),
        out_channels=raw.get("out_channels", d.out_channels),
        block_out_channels=tuple(raw.get("block_out_channels", d.block_out_channels)),
        cross_attention_levels=levels,
        layers_per_block=raw.get("layers_per_block", d.layers_per_block),
        attention_heads=int(heads),
        cross_attention_dim=raw.get("cross_attention_dim", d.cross_attention_dim),
        norm_num_groups=raw.get("norm_num_groups", d.norm_num_groups),
        norm_eps=raw.get("norm_eps", d.norm_eps),
        flip_sin_to_cos=raw.get("flip_sin_to_cos", d.flip_sin_to_cos),
        freq_shift=raw.get("freq_shift", d.freq_shift),
    )


def vae_config_from_json(raw: dict) -> VAEConfig:
    """diffusers ``AutoencoderKL`` config -> ``VAEConfig`` (missing keys: SD 1.5's)."""
    d = SD15_VAE
    if not raw:
        return d
    _only(raw, "act_fn", ("silu",), "vae/config.json")
    _only(raw, "use_quant_conv", (True,), "vae/config.json")
    _only(raw, "use_post_quant_conv", (True,), "vae/config.json")
    return VAEConfig(
        in_channels=raw.get("in_channels", d.in_channels),
        out_channels=raw.get("out_channels", d.out_channels),
        latent_channels=raw.get("latent_channels", d.latent_channels),
        block_out_channels=tuple(raw.get("block_out_channels", d.block_out_channels)),
        layers_per_block=raw.get("layers_per_block", d.layers_per_block),
        norm_num_groups=raw.get("norm_num_groups", d.norm_num_groups),
        norm_eps=raw.get("norm_eps", d.norm_eps),
        scaling_factor=raw.get("scaling_factor") or d.scaling_factor,
    )


def schedule_from_json(raw: dict) -> tuple[DDPMSchedule, bool]:
    """``scheduler_config.json`` -> (schedule, pndm).  The reference's pipeline keeps its own
    scheduler (SD 1.5 ships ``PNDMScheduler(skip_prk_steps=True)``); its ``alphas_cumprod``
    and timestep list are what the samplers read (``stable_diffusion.py:72-75, 130-133``).
    Supported: PNDM with ``skip_prk_steps``, DDIM and DDPM, ``leading`` spacing, epsilon
    prediction."""
    if not raw:
        return DDPMSchedule(beta_start=0.00085, beta_end=0.012, beta_schedule="scaled_linear",
                            steps_offset=1), True
    what = "scheduler/scheduler_config.json"
    cls = raw.get("_class_name", "PNDMScheduler")
    if cls not in ("PNDMScheduler", "DDIMScheduler", "DDPMScheduler"):
        raise NotImplementedError(f"{what}: {cls} is not supported")
    _only(raw, "prediction_type", ("epsilon",), what)
    _only(raw, "timestep_spacing", ("leading",), what)
    if raw.get("trained_betas") is not None:
        raise NotImplementedError(f"{what}: trained_betas are not supported")
    pndm = cls == "PNDMScheduler"
    if pndm and not raw.get("skip_prk_steps", False):
        raise NotImplementedError(f"{what}: PNDM with Runge-Kutta warm-up steps is not supported")
    schedule = DDPMSchedule(num_train_timesteps=raw.get("num_train_timesteps", 1000),
                            beta_start=raw.get("beta_start", 0.00085),
                            beta_end=raw.get("beta_end", 0.012),
                            beta_schedule=raw.get("beta_schedule", "scaled_linear"),
                            steps_offset=raw.get("steps_offset", 0))
    return schedule, pndm

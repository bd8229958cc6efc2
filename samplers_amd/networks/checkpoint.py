"""Local diffusers-layout checkpoints (safetensors + JSON), never fetched.

The reference loads its priors through ``diffusers.*Pipeline.from_pretrained`` by hub name
(``/root/reference/samplers/networks/diffusers/ddpm.py:22-38``,
``stable_diffusion.py:89-105``).  This build has no network and no diffusers: a prior is read
from a directory in diffusers' layout — ``<component>/diffusion_pytorch_model[.variant].safetensors``,
``<component>/config.json``, ``scheduler/scheduler_config.json`` — and a name that is not such a
directory raises ``FileNotFoundError``.  Only safetensors are read (no pickled ``.bin``).

The modules of ``unet2d.py``, ``unet2d_condition.py`` and ``vae.py`` carry diffusers' state-dict
names, so the state dict maps one to one, except for the names and shapes of older exports that
diffusers itself converts on load: the legacy attention names (``query`` / ``key`` / ``value`` /
``proj_attn``) and attention projections stored as 1x1 convolutions ([C, C, 1, 1]).
"""

from __future__ import annotations

import json
from pathlib import Path

import torch
from torch import nn

_LEGACY_ATTN_KEYS = {".query.": ".to_q.", ".key.": ".to_k.", ".value.": ".to_v.",
                     ".proj_attn.": ".to_out.0."}


def resolve_root(name_or_path: str, cache_dir: str | None, components: tuple[str, ...],
                 variant: str | None = None, what: str = "from_config") -> Path:
    """The checkpoint directory: ``name_or_path`` itself, else ``cache_dir / name_or_path``;
    every component's weights must be there."""
    root = Path(name_or_path)
    if cache_dir is not None and not root.exists():
        root = Path(cache_dir) / name_or_path
    for comp in components:
        w = weights_path(root, comp, variant)
        if not w.exists():
            raise FileNotFoundError(
                f"no local checkpoint at {w}; this build never fetches weights "
                f"(use {what} for a random-weight prior)")
    return root


def weights_path(root: Path, component: str, variant: str | None = None) -> Path:
    suffix = f".{variant}" if variant else ""
    return root / component / f"diffusion_pytorch_model{suffix}.safetensors"


def read_json(path: Path) -> dict:
    return json.loads(path.read_text()) if path.exists() else {}


def load_state(module: nn.Module, path: Path, *, dtype: torch.dtype = torch.float32) -> None:
    """Load a safetensors state dict into ``module`` (strict: every key on both sides), after
    the legacy-name and 1x1-shape conversions of the module doc; tensors cast to ``dtype``."""
    from safetensors.torch import load_file

    want = module.state_dict()
    fixed = {}
    for k, v in load_file(str(path)).items():
        for old, new in _LEGACY_ATTN_KEYS.items():
            k = k.replace(old, new)
        if k in want and v.shape != want[k].shape and v.numel() == want[k].numel() and (
                v.dim() == 4 and v.shape[2:] == (1, 1) or want[k].dim() == 4 and want[k].shape[2:] == (1, 1)):
            v = v.reshape(want[k].shape)  # a 1x1 conv stored as a linear, or the reverse
        fixed[k] = v.to(dtype)
    missing = sorted(set(want) - set(fixed))
    unexpected = sorted(set(fixed) - set(want))
    if missing or unexpected:
        raise ValueError(f"{path}: state dict does not match the module "
                         f"(missing {missing[:5]}{'...' if len(missing) > 5 else ''}, "
                         f"unexpected {unexpected[:5]}{'...' if len(unexpected) > 5 else ''})")
    bad = [k for k in want if fixed[k].shape != want[k].shape]
    if bad:
        raise ValueError(f"{path}: shape mismatch for {bad[:5]}")
    module.load_state_dict(fixed, assign=True)
    left = [n for n, t in list(module.named_parameters()) + list(module.named_buffers()) if t.is_meta]
    if left:
        raise ValueError(f"{path}: tensors not in the checkpoint left uninitialised: {left[:5]}")


def meta_module(build, *args) -> nn.Module:
    """Build a module's structure without initialising its weights (they are loaded next)."""
    with torch.device("meta"):
        return build(*args)

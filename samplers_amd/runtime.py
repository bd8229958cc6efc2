"""Process-level runtime setup for the MI355X path.

MIOpen (the convolution library behind the PyTorch-ROCm prior) picks a solver
per convolution shape by timing candidates the first time it meets the shape,
and compiles the winning kernels; on a fresh gfx950 box that costs minutes and,
when the search is cut short, a slower solver.  ``configure_miopen`` points
MIOpen's user find-db and kernel cache at a writable in-tree directory and
seeds it with ``samplers_amd/miopen_db/*.ufdb.txt`` — solver choices measured
on MI355X by this project's own runs (a text table of solver names and
timings, not code).  Existing settings of MIOPEN_USER_DB_PATH /
MIOPEN_CUSTOM_CACHE_DIR are respected.

The priors' convolutions run on this project's tiles, so MIOpen only serves
shapes outside the tiles' rules; ``ensure_miopen`` runs the setup once, right
before the first such fallback (MIOpen reads the variables when torch creates
its handle, at the first MIOpen convolution), not at import.
"""

from __future__ import annotations

import contextlib
import os
from pathlib import Path

PACKAGE = Path(__file__).resolve().parent
SEED_DB = PACKAGE / "miopen_db"

# Batch-dependent kernel choices.  Split-K (§3 "Round 4"): a launch whose tiles
# leave CUs idle cuts K into parts and adds them in a fixed order; the parts are chosen per
# launch from its tile count.  hipBLASLt (the d = 512 attention's score / value GEMMs) picks its
# algorithm per problem size, batch count included.  So the same sample is summed in a different
# order at a different batch size (micro_batch, world size) and agrees to fp32 rounding only.
# ``batch_invariant(True)`` removes both: every launch unsplit and those GEMMs issued one batch
# entry at a time, so a sharded or micro-batched solve is bitwise the single-process one.
def _env_on(name: str, default: str) -> bool:
    return os.environ.get(name, default).lower() not in ("0", "off", "false", "")


_FLAGS = {"split_k": _env_on("SAMPLERS_AMD_SPLIT_K", "1"),
          "batch_invariant": _env_on("SAMPLERS_AMD_BATCH_INVARIANT", "0")}


def split_k_enabled() -> bool:
    return _FLAGS["split_k"] and not _FLAGS["batch_invariant"]


def batch_invariant_enabled() -> bool:
    return _FLAGS["batch_invariant"]


def _set(flag: str, enabled: bool) -> bool:
    prev = _FLAGS[flag]
    _FLAGS[flag] = bool(enabled)
    return prev


def set_split_k(enabled: bool) -> bool:
    """Enable / disable split-K for under-filled launches; returns the previous setting."""
    return _set("split_k", enabled)


def set_batch_invariant(enabled: bool) -> bool:
    """Batch-invariant summation order for every launch (module comment); returns the previous
    setting."""
    return _set("batch_invariant", enabled)


@contextlib.contextmanager
def split_k(enabled: bool):
    """``with split_k(False): ...`` — no split-K launches inside the block."""
    prev = set_split_k(enabled)
    try:
        yield
    finally:
        set_split_k(prev)


@contextlib.contextmanager
def batch_invariant(enabled: bool = True):
    """``with batch_invariant(): ...`` — results independent of the batch a sample is in."""
    prev = set_batch_invariant(enabled)
    try:
        yield
    finally:
        set_batch_invariant(prev)


def _writable_cache_dir() -> Path:
    for cand in (PACKAGE.parent / ".miopen_cache",
                 Path(os.environ.get("XDG_CACHE_HOME", Path.home() / ".cache")) / "samplers_amd_miopen"):
        try:
            cand.mkdir(parents=True, exist_ok=True)
            probe = cand / ".w"
            probe.write_text("")
            probe.unlink()
            return cand
        except OSError:
            continue
    raise OSError("no writable directory for the MIOpen cache")


def configure_miopen() -> Path | None:
    """Set MIOpen's user-db / kernel-cache directory (idempotent); returns it."""
    if os.environ.get("MIOPEN_USER_DB_PATH"):
        cache = Path(os.environ["MIOPEN_USER_DB_PATH"])
    else:
        try:
            cache = _writable_cache_dir()
        except OSError:
            return None
        os.environ["MIOPEN_USER_DB_PATH"] = str(cache)
    os.environ.setdefault("MIOPEN_CUSTOM_CACHE_DIR", str(cache))
    try:
        cache.mkdir(parents=True, exist_ok=True)
        for src in SEED_DB.glob("*.ufdb.txt"):
            _merge_find_db(src, cache / src.name)
    except OSError:
        pass
    return cache


_CONFIGURED = [False]


def ensure_miopen() -> None:
    """``configure_miopen`` once per process; called by the MIOpen fallbacks of
    ``networks/layers.py`` before they reach ``F.conv2d`` / ``nn.Conv2d``."""
    if not _CONFIGURED[0]:
        _CONFIGURED[0] = True
        configure_miopen()


def _merge_find_db(src: Path, dst: Path) -> None:
    """Add the seed's entries (one ``key=solver:time,...`` line per convolution) that
    ``dst`` lacks; entries MIOpen already measured on this machine are kept.  The merged
    file is written to a private temporary and renamed into place, so the ranks of a
    multi-GPU launch starting together never see (or write) a half-written database."""
    have_lines = dst.read_text().splitlines() if dst.exists() else []
    have = {line.split("=", 1)[0] for line in have_lines if "=" in line}
    extra = [line for line in src.read_text().splitlines()
             if "=" in line and line.split("=", 1)[0] not in have]
    if not extra and dst.exists():
        return
    tmp = dst.with_name(f"{dst.name}.{os.getpid()}.tmp")
    tmp.write_text("\n".join(have_lines + extra) + "\n")
    os.replace(tmp, dst)

"""Multi-GPU sampling: shard the observation batch, one process per GPU.

DPS samples are independent, so a node-wide run needs no
data-path collective: rank r solves a contiguous block of observations (and
their R reconstructions) with Philox noise keyed by the *global* flat sample
index (``sample_offset``), which makes the result bit-identical to the
single-GPU run whatever the world size.  The only collective is one RCCL
``all_gather`` of the x-hat shards at the end (over xGMI; ``backend="nccl"`` is
RCCL on ROCm), plus a 8-byte broadcast of the seed at the start.

PSLD and ReSample couple the batch through their norms (``psld.py:130,138``,
``resample_kernels.py:26,67``: one scalar over the whole flat batch); their samplers take
a ``group`` and sum those scalars over it (``all_reduce_sum_``, a few bytes per step), so
the sharded run equals the single-process one up to the summation order of the norms.
"""

from __future__ import annotations

import inspect
from typing import Callable

import torch
import torch.distributed as dist
from torch import Tensor

from samplers_amd.inverse_problem import InverseProblem


def shard_bounds(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced [start, stop) block of ``total`` items for ``rank``."""
    if world <= 0 or not (0 <= rank < world):
        raise ValueError("bad rank / world size")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def broadcast_seed(seed: int | None, device: torch.device, group=None) -> int:
    """Rank 0's seed (drawn from torch's CPU generator if None) on every rank."""
    if seed is None:
        seed = int(torch.randint(0, 2**62, (1,), dtype=torch.int64).item())
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        t = torch.tensor([seed], dtype=torch.int64, device=device)
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        seed = int(t.item())
    return seed


_MAX_RANK = 8  # trailing dims a gathered shard may have (shape exchange buffer)
# dtypes a gathered shard may have, by code (exchanged with the shape: an idle rank's
# placeholder must match the active ranks' dtype byte for byte, or RCCL's all-gather sizes
# disagree — a bf16 / fp16 network returns in its own dtype)
_DTYPES = (torch.float32, torch.float16, torch.bfloat16, torch.float64)


def _trailing_shape(local: Tensor | None, counts: list[int], rank: int, group=None,
                    device: torch.device | None = None) -> tuple[tuple[int, ...], torch.dtype]:
    """The per-item shape and dtype of the gathered tensor, taken from the first rank that
    holds items.  An idle rank (count 0) cannot know them: what a sampler returns depends on
    its options (PSLD / ReSample with ``decode_output=False`` return latents, not
    ``x_shape``; a reduced-precision network returns its own dtype), so the active ranks'
    shape and dtype code are exchanged first (an 80-byte all-gather)."""
    buf = torch.full((_MAX_RANK + 2,), -1, dtype=torch.int64, device=device)
    if local is not None and counts[rank] > 0:
        tail = tuple(local.shape[1:])
        if len(tail) > _MAX_RANK:
            raise ValueError(f"shards with more than {_MAX_RANK} trailing dims")
        if local.dtype not in _DTYPES:
            raise ValueError(f"cannot gather shards of dtype {local.dtype}")
        buf[0] = len(tail)
        buf[1] = _DTYPES.index(local.dtype)
        if tail:
            buf[2:2 + len(tail)] = torch.tensor(tail, dtype=torch.int64)
    out = torch.empty((len(counts), _MAX_RANK + 2), dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(out.view(-1), buf, group=group)
    first = next(r for r, c in enumerate(counts) if c > 0)
    nd = int(out[first, 0])
    return tuple(int(v) for v in out[first, 2:2 + nd].tolist()), _DTYPES[int(out[first, 1])]


def gather_shards(local: Tensor | None, counts: list[int], group=None, *,
                  device: torch.device | None = None) -> Tensor:
    """All-gather variable-size leading-axis shards into the full tensor on every rank.
    ``local`` may be None on a rank that holds no items (its placeholder takes the trailing
    shape and the dtype the active ranks report)."""
    world = len(counts)
    if world == 1:
        return local
    rank = dist.get_rank(group)
    device = local.device if local is not None else device
    if any(c == 0 for c in counts):
        tail, dtype = _trailing_shape(local, counts, rank, group, device)
        if local is None or counts[rank] == 0:
            local = torch.empty((0, *tail), device=device, dtype=dtype)
    width = max(counts)
    pad = torch.zeros((width, *local.shape[1:]), device=local.device, dtype=local.dtype)
    pad[: local.shape[0]] = local
    out = torch.empty((world * width, *local.shape[1:]), device=local.device, dtype=local.dtype)
    dist.all_gather_into_tensor(out, pad.contiguous(), group=group)
    return torch.cat([out[r * width: r * width + c] for r, c in enumerate(counts)])


def all_reduce_sum_(t: Tensor, group=None) -> Tensor:
    """In-place sum over the ranks of ``group`` (no-op in a single process): the batch-global
    norms of PSLD (``psld.py:130,138``) and ReSample (``resample_kernels.py:26,67``) — a few
    bytes per step, RCCL over xGMI with ``backend="nccl"``."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, group=group)
    return t


_ACTIVE_GROUPS: dict = {}  # rank tuple -> process group of the ranks holding observations
_ACTIVE_WORLD: list = [None]  # the default group _ACTIVE_GROUPS was built under


def _active_group(ranks: tuple[int, ...]):
    """One process group per rank set, not one per call.  The cache belongs to the default
    group it was built under: a destroyed and re-initialised world (a new WORLD object, whose
    id() CPython may reuse) starts a fresh cache instead of returning dead subgroups."""
    world = dist.group.WORLD
    if _ACTIVE_WORLD[0] is not world:
        _ACTIVE_GROUPS.clear()
        _ACTIVE_WORLD[0] = world
    if ranks not in _ACTIVE_GROUPS:
        _ACTIVE_GROUPS[ranks] = dist.new_group(list(ranks), use_local_synchronization=True)
    return _ACTIVE_GROUPS[ranks]


def _parameters(fn) -> dict:
    try:
        return dict(inspect.signature(fn).parameters)
    except (TypeError, ValueError):
        return {}


def sharded_call(sampler: Callable[..., Tensor], inverse_problem: InverseProblem, *,
                 num_reconstructions: int = 1, seed: int | None = None, group=None,
                 **kwargs) -> Tensor:
    """Run ``sampler`` on this rank's block of observations and all-gather x-hat.

    ``sampler`` is a posterior sampler accepting ``seed``/``sample_offset``.  One that also
    names a ``group`` parameter (``PSLDSampler``, ``ReSampleSampler``: batch-coupled norms)
    receives ``group`` (narrowed to the ranks that hold observations when there are more
    ranks than observations, so an idle rank is never waited for in the per-step norm
    reductions); one with ``keep_reconstruction_dim`` (``DPSSampler``, ``PGDMSampler``)
    squeezes an R = 1 axis exactly as its single-process call would.  Returns the same
    tensor the single-process call would, on every rank.
    """
    params = _parameters(sampler)
    coupled = "group" in params
    keep = bool(kwargs.pop("keep_reconstruction_dim", False))
    squeezes = "keep_reconstruction_dim" in params or any(
        v.kind is inspect.Parameter.VAR_KEYWORD for v in params.values())
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    obs = inverse_problem.observation
    batch_shape = tuple(inverse_problem.batch_shape)
    if len(batch_shape) > 1:
        raise ValueError("flatten multi-axis observation batches before sharding")
    total = batch_shape[0] if batch_shape else 1
    if not batch_shape:
        obs = obs.unsqueeze(0)
    start, stop = shard_bounds(total, rank, world)
    seed = broadcast_seed(seed, obs.device, group)
    local = InverseProblem(inverse_problem.operator, obs[start:stop], inverse_problem.noise)
    counts = [b - a for a, b in (shard_bounds(total, r, world) for r in range(world))]
    if stop > start:
        if coupled:
            kwargs["group"] = group
            active = [r for r, c in enumerate(counts) if c > 0]
            if len(active) < world:  # only the active ranks create (and use) the subgroup
                ranks = tuple(r if group is None else dist.get_global_rank(group, r) for r in active)
                kwargs["group"] = _active_group(ranks)
        if squeezes:
            kwargs["keep_reconstruction_dim"] = True
        out = sampler(local, num_reconstructions=num_reconstructions, seed=seed,
                      sample_offset=start * num_reconstructions, **kwargs)
    else:  # more ranks than observations: this rank only joins the gather (the shard shape
        out = None  # comes from the active ranks: latents when a sampler skips the decode)
    full = gather_shards(None if out is None else out.contiguous(), counts, group,
                         device=obs.device)
    if not batch_shape:
        full = full.squeeze(0)
    if squeezes and num_reconstructions == 1 and not keep:
        full = full.squeeze(len(batch_shape))
    return full

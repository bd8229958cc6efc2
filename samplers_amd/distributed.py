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


def gather_shards(local: Tensor, counts: list[int], group=None) -> Tensor:
    """All-gather variable-size leading-axis shards into the full tensor on every rank."""
    world = len(counts)
    if world == 1:
        return local
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


_ACTIVE_GROUPS: dict = {}  # (rank tuple, world) -> process group of the ranks holding observations


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
                # one process group per rank set (and default group: a re-initialised world
                # gets new ones), not one per call
                key = (ranks, id(dist.group.WORLD))
                if key not in _ACTIVE_GROUPS:
                    _ACTIVE_GROUPS[key] = dist.new_group(list(ranks), use_local_synchronization=True)
                kwargs["group"] = _ACTIVE_GROUPS[key]
        if squeezes:
            kwargs["keep_reconstruction_dim"] = True
        out = sampler(local, num_reconstructions=num_reconstructions, seed=seed,
                      sample_offset=start * num_reconstructions, **kwargs)
    else:  # more ranks than observations: this rank only joins the gather
        out = torch.empty((0, num_reconstructions, *inverse_problem.operator.x_shape),
                          device=obs.device, dtype=torch.float32)
    full = gather_shards(out.contiguous(), counts, group)
    if not batch_shape:
        full = full.squeeze(0)
    if squeezes and num_reconstructions == 1 and not keep:
        full = full.squeeze(len(batch_shape))
    return full

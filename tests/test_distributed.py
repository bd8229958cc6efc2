"""Multi-process plumbing on CPU (gloo, world_size 2): sharding, seed broadcast and the
final gather reproduce the single-process result exactly."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import philox
from samplers_amd.distributed import gather_shards, shard_bounds, sharded_call
from samplers_amd.inverse_problem import InverseProblem
from samplers_amd.noise import GaussianNoise
from samplers_amd.operators import IdentityOperator

SHAPE = (2, 3, 4)
N = 24


def fake_sampler(problem, *, num_reconstructions, seed, sample_offset, keep_reconstruction_dim,
                 **_):
    """Deterministic per-global-sample output (Philox keyed by the flat sample index) plus the
    observation, standing in for DPS (which needs a GPU)."""
    b = problem.observation.shape[0]
    rows = []
    for i in range(b * num_reconstructions):
        z = torch.from_numpy(philox.normals(seed, 0, sample_offset + i, N)).reshape(SHAPE)
        rows.append(z + problem.observation[i // num_reconstructions])
    return torch.stack(rows).reshape(b, num_reconstructions, *SHAPE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, batch, R, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        obs = torch.arange(batch * N, dtype=torch.float32).reshape(batch, *SHAPE)
        prob = InverseProblem(IdentityOperator(SHAPE), obs, GaussianNoise(0.1))
        torch.manual_seed(123)  # seed drawn on rank 0, broadcast
        if rank == 1:
            torch.manual_seed(999)  # a different local RNG must not matter
        out = sharded_call(fake_sampler, prob, num_reconstructions=R)
        if rank == 0:
            torch.save(out, result_path)
        # every rank holds the full result
        t = torch.tensor([float(out.sum())])
        dist.all_reduce(t)
        assert abs(t.item() - world * float(out.sum())) < 1e-3 * abs(t.item()) + 1e-3
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("batch,R", [(5, 1), (4, 3), (1, 2)])
def test_sharded_equals_single_process(tmp_path, batch, R):
    path = tmp_path / "out.pt"
    mp.spawn(_worker, args=(2, _free_port(), batch, R, str(path)), nprocs=2, join=True)
    sharded = torch.load(path, weights_only=True)
    torch.manual_seed(123)
    obs = torch.arange(batch * N, dtype=torch.float32).reshape(batch, *SHAPE)
    prob = InverseProblem(IdentityOperator(SHAPE), obs, GaussianNoise(0.1))
    single = sharded_call(fake_sampler, prob, num_reconstructions=R)
    assert torch.equal(sharded, single)
    assert single.shape == ((batch, *SHAPE) if R == 1 else (batch, R, *SHAPE))


def test_shard_bounds_cover_exactly():
    for total in (0, 1, 7, 64, 512):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def test_gather_single_rank_is_identity():
    t = torch.randn(3, 2)
    assert gather_shards(t, [3]) is t

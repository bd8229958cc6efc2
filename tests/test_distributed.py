"""Multi-process plumbing on CPU (gloo, world_size 2): sharding, seed broadcast and the
final gather reproduce the single-process result exactly."""

import os
import tempfile

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
    """A rendezvous for the workers: a FileStore path (file:// init), not a TCP port — a port
    picked free here can be taken by another socket before rank 0 binds it (a rare flaky
    failure of these tests); gloo's own pair connections use OS-assigned ports."""
    return "file://" + os.path.join(tempfile.mkdtemp(prefix="sp_rdv_"), "store")


def _worker(rank, world, port, batch, R, result_path):
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
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


# --- batch-coupled samplers: PSLD / ReSample global norms over ranks -------

def _norm_worker(rank, world, port, result_path):
    """Each rank holds a contiguous shard of a batch of 5 and computes the samplers' global
    quantities with the production code (the generic-operator terms, which are plain torch
    and so run on CPU): PSLD's ‖y − A x̂₀‖² (``generic_pixel_terms`` + ``all_reduce_sum_``),
    ReSample's MSE sum of squares and its gradient (``_GenericConsistency``)."""
    import stand_ins as si

    from samplers_amd.distributed import all_reduce_sum_
    from samplers_amd.samplers.psld import generic_pixel_terms
    from samplers_amd.samplers.resample import _GenericConsistency

    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        out = _norm_terms(si, generic_pixel_terms, _GenericConsistency, all_reduce_sum_,
                          rank, world)
        if rank == 0:
            torch.save(out, result_path)
    finally:
        dist.destroy_process_group()


def _norm_terms(si, generic_pixel_terms, consistency, reduce, rank, world):
    shape, batch, R = (3, 8, 8), 5, 2
    op = si.torch_operator(shape, torch.arange(0, 192, 3))
    gen = torch.Generator().manual_seed(4)
    y = torch.randn(batch, *op.y_shape, generator=gen)
    x0 = torch.randn(batch * R, *shape, generator=gen)
    hty = op.apply_transpose(y).reshape(batch, -1)
    start, stop = shard_bounds(batch, rank, world)
    ys, hs, xs = y[start:stop], hty[start:stop], x0[start * R:stop * R]
    x_eff, ss, _ = generic_pixel_terms(op, ys.reshape(stop - start, -1), hs, R, xs)
    ss = reduce(ss)
    total = batch * R * op.y_shape[0]
    cons = consistency(op, ys.reshape(stop - start, -1), R)
    g, ss2 = cons.mse_grad_ss(xs, total)
    full_g = torch.zeros(batch * R, *shape)
    full_g[start * R:stop * R] = g
    reduce(full_g)  # disjoint rows: the sum assembles the full gradient
    return {"psld_ss": ss, "rs_ss": ss2, "rs_grad": full_g, "x_eff_rows": (start * R, x_eff)}


def test_batch_global_norms_match_single_process(tmp_path):
    import stand_ins as si

    from samplers_amd.distributed import all_reduce_sum_
    from samplers_amd.samplers.psld import generic_pixel_terms
    from samplers_amd.samplers.resample import _GenericConsistency

    path = tmp_path / "norms.pt"
    mp.spawn(_norm_worker, args=(2, _free_port(), str(path)), nprocs=2, join=True)
    sharded = torch.load(path, weights_only=True)
    single = _norm_terms(si, generic_pixel_terms, _GenericConsistency, all_reduce_sum_, 0, 1)
    # sums of squares: the same terms in a different association order
    assert torch.allclose(sharded["psld_ss"], single["psld_ss"], rtol=1e-6)
    assert torch.allclose(sharded["rs_ss"], single["rs_ss"], rtol=1e-6)
    assert torch.equal(sharded["rs_grad"], single["rs_grad"])  # per-sample: bit-identical
    r0, xe = sharded["x_eff_rows"]
    assert torch.equal(xe, single["x_eff_rows"][1][r0:r0 + xe.shape[0]])


# --- sharded_call with a batch-coupled sampler (group-taking, never squeezes R) -----------

LATENT = (2, 2, 3)  # a latent shape unlike SHAPE (PSLD / ReSample with decode_output=False)


def coupled_sampler(problem, *, num_reconstructions, seed, sample_offset, group=None,
                    decode_output=True, out_dtype=None):
    """A PSLD-like sampler: every sample is scaled by a batch-global sum of squares,
    reduced over ``group`` three times (one per 'step'); the R axis is always kept.
    ``decode_output=False`` returns a latent-shaped slice, as PSLD / ReSample do."""
    from samplers_amd.distributed import all_reduce_sum_

    obs = problem.observation
    x = obs.repeat_interleave(num_reconstructions, 0)
    for _ in range(3):
        ss = all_reduce_sum_(x.square().sum().reshape(1), group)
        x = x / ss.sqrt()
    out = x.reshape(obs.shape[0], num_reconstructions, *SHAPE)
    if not decode_output:
        out = out.reshape(obs.shape[0], num_reconstructions, -1)[..., :12].reshape(
            obs.shape[0], num_reconstructions, *LATENT)
    return out if out_dtype is None else out.to(out_dtype)  # a bf16 / fp16 network's dtype


def _coupled_worker(rank, world, port, batch, R, decode, result_path, out_dtype=None):
    dist.init_process_group("gloo", init_method=port, rank=rank, world_size=world)
    try:
        obs = torch.arange(1, batch * N + 1, dtype=torch.float32).reshape(batch, *SHAPE)
        prob = InverseProblem(IdentityOperator(SHAPE), obs, GaussianNoise(0.1))
        out = sharded_call(coupled_sampler, prob, num_reconstructions=R, seed=3,
                           decode_output=decode, out_dtype=out_dtype)
        assert out.dtype == (out_dtype or torch.float32)  # the idle rank's too
        if rank == 0:
            torch.save(out, result_path)
        # a second call on the same world reuses the cached subgroup of active ranks
        again = sharded_call(coupled_sampler, prob, num_reconstructions=R, seed=3,
                             decode_output=decode, out_dtype=out_dtype)
        assert torch.equal(again, out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,batch,R,decode,out_dtype", [
    (2, 5, 1, True, None), (3, 2, 2, True, None), (4, 3, 1, False, None),
    (3, 2, 1, True, torch.bfloat16), (3, 1, 2, False, torch.float16)])
def test_sharded_coupled_sampler_equals_single_process(tmp_path, world, batch, R, decode,
                                                       out_dtype):
    """(3, 2, 2): one rank holds no observation and must not be waited for by the others'
    per-step reductions (they reduce over the subgroup of active ranks).  (4, 3, 1, False):
    an idle rank while the sampler returns latents — its placeholder shard takes the shape
    the active ranks report, not x_shape.  The reduced-precision cases: an idle rank's
    placeholder takes the active ranks' dtype (a float32 placeholder beside bf16 shards would
    make the all-gather's byte counts disagree)."""
    path = tmp_path / "out.pt"
    mp.spawn(_coupled_worker, args=(world, _free_port(), batch, R, decode, str(path), out_dtype),
             nprocs=world, join=True)
    sharded = torch.load(path, weights_only=True)
    obs = torch.arange(1, batch * N + 1, dtype=torch.float32).reshape(batch, *SHAPE)
    prob = InverseProblem(IdentityOperator(SHAPE), obs, GaussianNoise(0.1))
    single = sharded_call(coupled_sampler, prob, num_reconstructions=R, seed=3,
                          decode_output=decode, out_dtype=out_dtype)
    assert sharded.dtype == single.dtype
    assert single.shape == (batch, R, *(SHAPE if decode else LATENT))  # R kept
    assert sharded.shape == single.shape
    rtol = 1e-6 if out_dtype is None else 1e-2
    assert torch.allclose(sharded.float(), single.float(), rtol=rtol, atol=0)

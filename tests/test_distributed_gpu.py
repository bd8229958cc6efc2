"""The batch-coupled samplers sharded over two ranks on the HIP path.

PSLD's two norms (psld.py:130,138) and ReSample's consistency losses and MSE totals
(resample_kernels.py:26,67) are scalars over the whole flat batch; sharded over ranks they
are summed by ``all_reduce_sum_`` once per step.  Two processes share the box's one GPU
(gloo over device tensors: the collective is the same call RCCL serves on a multi-GPU
node) and run ``sharded_call`` on their halves of the batch; the gathered result must
equal the single-process run on the whole batch.  Tolerance: relative L2 1e-5 (the only
difference is the order in which the norms' partial sums are added), and the idle-rank
case (more ranks than observations) is exercised by the ReSample batch of 3 over 2.
"""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import stand_ins as si

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(kind: str, device):
    """kind: psld | resample | resample_latent (decode_output=False: latent shards)."""
    from samplers_amd.distributed import sharded_call
    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.noise import GaussianNoise, PoissonNoise
    from samplers_amd.operators import IdentityOperator, InpaintingOperator
    from samplers_amd.samplers.psld import PSLDSampler
    from samplers_amd.samplers.resample import ReSampleSampler

    shape = (3, 32, 32)
    net = si.make_samplers_amd_latent_net("conv", 0.1, device=device)
    if kind == "psld":
        b, R = 4, 2
        op = InpaintingOperator(shape, si.fixture_mask(shape, "center"))
        x = si.fixture_x_true(b, shape, 5)
        y = op.apply(x) + 0.05 * torch.randn(b, op._kept_indices.numel(),
                                             generator=torch.Generator().manual_seed(6))
        prob = InverseProblem(op.to(device), y.to(device), GaussianNoise(0.05).to(device))
        return sharded_call(PSLDSampler(net), prob, num_reconstructions=R, seed=11,
                            num_sampling_steps=8)
    b, R = 3, 1
    x = si.fixture_x_true(b, shape, 7)
    y = torch.poisson((x + 1) * 8, generator=torch.Generator().manual_seed(8)) / 8 - 1
    prob = InverseProblem(IdentityOperator(shape), y.to(device), PoissonNoise(1.0).to(device))
    # 12 steps, split 3 ways: time travel at 10 (pixel-space solve) and the final latent solve
    return sharded_call(ReSampleSampler(net), prob, num_reconstructions=R, seed=13,
                        num_sampling_steps=12, max_optimization_iters=24, inter_timesteps=3,
                        time_travel_interval=5, stage_splits=3,
                        decode_output=kind != "resample_latent")


def _worker(rank, world, port, kind, path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = _run(kind, torch.device("cuda:0"))
        torch.cuda.synchronize()
        if rank == 0:
            torch.save(out.cpu(), path)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind,world", [("psld", 2), ("resample", 2), ("resample", 4),
                                        ("resample_latent", 4)])
def test_batch_coupled_sampler_sharded_equals_single(cuda, tmp_path, kind, world):
    path = tmp_path / "out.pt"
    mp.spawn(_worker, args=(world, _free_port(), kind, str(path)), nprocs=world, join=True)
    sharded = torch.load(path, weights_only=True)
    single = _run(kind, cuda).cpu()
    assert sharded.shape == single.shape
    assert torch.isfinite(single).all()
    assert si.relative_error(sharded, single) < 1e-5

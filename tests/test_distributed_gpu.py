"""The samplers sharded over ranks on the HIP path.

DPS (configs[2]'s path, ``dps.py:91-130``): samples are independent, so ``sharded_call`` gives
each rank a contiguous block of observations, keys the Philox noise by the global sample
index and all-gathers x̂ once.  The sharded result must be **bitwise** the single-process
one at world sizes 2, 4 and 8, with an uneven split and with idle ranks (more
ranks than observations).  With the full ddpm-celebahq-256 UNet the bitwise claim holds in
batch-invariant mode (``runtime.batch_invariant()``: split-K off, the d = 512 attention's
hipBLASLt GEMMs one batch entry at a time); by default the per-rank batch picks different K
splits and GEMM algorithms and the result agrees to fp32 rounding (relative L2 1e-5).

PSLD's two norms (psld.py:130,138) and ReSample's consistency losses and MSE totals
(resample_kernels.py:26,67) are scalars over the whole flat batch; sharded over ranks they
are summed by ``all_reduce_sum_`` once per step.  Tolerance: relative L2 1e-5 (the only
difference is the order in which the norms' partial sums are added), and the idle-rank
case (more ranks than observations) is exercised by the ReSample batch of 3 over 2 and 4.

All ranks share the box's one GPU (gloo over device tensors: the collective is the same call
RCCL serves on a multi-GPU node); the rendezvous is a FileStore (no TCP port race).
"""

import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import stand_ins as si

pytestmark = pytest.mark.gpu

UNET_STEPS = 5  # DPS steps of the full-UNet cases (3 guided iterations + the final x̂)


def _rendezvous() -> str:
    return "file://" + os.path.join(tempfile.mkdtemp(prefix="sp_rdv_"), "store")


def _dps_problem(kind: str, b: int, device):
    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.noise import GaussianNoise
    from samplers_amd.operators import GaussianBlurOperator, RandomInpaintingOperator

    shape = (3, 256, 256) if kind.startswith("dps_unet") else (3, 32, 32)
    if kind.endswith("blur"):
        op = GaussianBlurOperator(shape, kernel_size=9, sigma=3.0)
    else:
        op = RandomInpaintingOperator(shape, 0.5, seed=1)
    op = op.to(device)
    x = si.fixture_x_true(b, shape, 5).to(device)
    gen = torch.Generator().manual_seed(6)
    y = op.apply(x)
    y = y + (0.05 * torch.randn(tuple(y.shape), generator=gen)).to(device)
    return InverseProblem(op, y, GaussianNoise(0.05).to(device)), shape


def _unet_net(device):
    from samplers_amd.networks.ddpm import DDPMNetwork

    return DDPMNetwork.from_config(seed=0, device=device)


def _run(kind: str, device):
    """kind: dps | dps_blur (stand-in prior, 3x32², B = 5, R = 2), dps_unet / dps_unet_invariant
    (full UNet, 3x256², B = 3), psld | resample | resample_latent (latent stand-in)."""
    from samplers_amd.distributed import sharded_call
    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.noise import GaussianNoise, PoissonNoise
    from samplers_amd.operators import IdentityOperator, InpaintingOperator
    from samplers_amd.runtime import batch_invariant
    from samplers_amd.samplers import DPSSampler
    from samplers_amd.samplers.psld import PSLDSampler
    from samplers_amd.samplers.resample import ReSampleSampler

    if kind in ("dps", "dps_blur"):
        prob, _ = _dps_problem(kind, 5, device)
        net = si.make_samplers_amd_net("conv", 3, 0.1, device=device)
        return sharded_call(DPSSampler(net), prob, num_reconstructions=2, seed=17,
                            num_sampling_steps=12)
    if kind.startswith("dps_unet"):
        prob, _ = _dps_problem(kind, 3, device)
        with batch_invariant(kind.endswith("invariant")):
            return sharded_call(DPSSampler(_unet_net(device)), prob, seed=19,
                                num_sampling_steps=UNET_STEPS)
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


def _worker(rank, world, init, kind, path):
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    try:
        out = _run(kind, torch.device("cuda:0"))
        torch.cuda.synchronize()
        # every rank holds the gathered tensor; each writes its own copy
        torch.save(out.cpu(), f"{path}.{rank}")
    finally:
        dist.destroy_process_group()


def _sharded(kind: str, world: int, tmp_path) -> list[torch.Tensor]:
    path = str(tmp_path / "out.pt")
    mp.spawn(_worker, args=(world, _rendezvous(), kind, path), nprocs=world, join=True)
    return [torch.load(f"{path}.{r}", weights_only=True) for r in range(world)]


@pytest.mark.parametrize("kind,world", [("dps", 2), ("dps", 4), ("dps", 8), ("dps_blur", 8)])
def test_dps_sharded_bitwise_equals_single(cuda, tmp_path, kind, world):
    """B = 5 observations x R = 2: world 2 splits 3 / 2, world 4 2 / 1 / 1 / 1, world 8 leaves
    three ranks idle (they only join the gather)."""
    outs = _sharded(kind, world, tmp_path)
    single = _run(kind, cuda).cpu()
    assert single.shape == (5, 2, 3, 32, 32) and torch.isfinite(single).all()
    for r, out in enumerate(outs):
        assert torch.equal(out, single), f"rank {r} of {world}: differs from the single process"


@pytest.mark.timeout(600)
@pytest.mark.parametrize("kind", ["dps_unet_invariant", "dps_unet"])
def test_dps_unet_sharded_equals_single(cuda, tmp_path, kind, parity_record):
    """The full prior, B = 3 over 2 ranks (2 / 1): bitwise in batch-invariant mode; by default
    (split-K parts and hipBLASLt algorithms follow the per-rank batch) to fp32 rounding."""
    outs = _sharded(kind, 2, tmp_path)
    single = _run(kind, cuda).cpu()
    assert single.shape == (3, 3, 256, 256) and torch.isfinite(single).all()
    err = si.relative_error(outs[0], single)
    parity_record("sharded_vs_single_rel_l2", err, 1e-5, sampler="DPS", world=2, kind=kind)
    assert torch.equal(outs[0], outs[1])
    if kind.endswith("invariant"):
        assert torch.equal(outs[0], single), f"batch-invariant: rel L2 {err:.3e}, expected bitwise"
    else:
        assert err < 1e-5, err


@pytest.mark.parametrize("kind,world", [("psld", 2), ("resample", 2), ("resample", 4),
                                        ("resample_latent", 4)])
def test_batch_coupled_sampler_sharded_equals_single(cuda, tmp_path, kind, world):
    sharded = _sharded(kind, world, tmp_path)[0]
    single = _run(kind, cuda).cpu()
    assert sharded.shape == single.shape
    assert torch.isfinite(single).all()
    assert si.relative_error(sharded, single) < 1e-5


@pytest.mark.timeout(600)
def test_dps_unet_micro_batch_bitwise_when_batch_invariant(cuda):
    """with the full prior, micro_batch changes every launch's batch; in
    batch-invariant mode the chunked solve is bitwise the whole-batch one (the guidance passes'
    per-sample partial sums and the Philox streams are batch-invariant by construction)."""
    from samplers_amd.runtime import batch_invariant
    from samplers_amd.samplers import DPSSampler

    prob, _ = _dps_problem("dps_unet", 3, cuda)
    net = _unet_net(cuda)
    with batch_invariant():
        a = DPSSampler(net)(prob, seed=23, num_sampling_steps=UNET_STEPS)
        b = DPSSampler(net)(prob, seed=23, num_sampling_steps=UNET_STEPS, micro_batch=1)
    assert torch.isfinite(a).all()
    assert torch.equal(a, b), si.relative_error(b.cpu(), a.cpu())

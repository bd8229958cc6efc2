"""Whole trajectories with the real priors in the loop.

The per-layer tests pin one call of each prior; these pin what the samplers compose from
them over several steps, so that error compounding of the device arithmetic (Winograd
F(2x2,3x3) tiles, the split-bf16 1x1 shortcut / linear GEMMs, single-pass GroupNorm, fused
attention, the guidance passes) along a trajectory is bounded:

* ``DPSSampler.__call__`` with the full ddpm-celebahq-256 UNet (113.7 M, default backends:
  ``SAMPLERS_AMD_SHORTCUT=x6``) at 3x256², B = 2, 6 guided iterations + the final
  prediction, for configs[1] (50 % random inpainting) and configs[2] (9x9 Gaussian blur),
  against ``oracle/dps_loop.py`` (``dps.py:91-126``) on the CPU with the same weights and
  the same injected noise;
* ``PSLDSampler.__call__`` with the SD 1.5 VAE and the 859.5 M ε-UNet at 3x256² (latents
  4x32x32), B = 2, centre inpainting, 3 guided iterations + the final decode, **with
  classifier-free guidance on** (distinct prompt embeddings, guidance 7.5: the UNet batch is
  doubled, ``stable_diffusion.py:300-320``), against ``oracle/latent_loops.py``
  (``psld.py:118-161``).

Tolerance: relative L2 <= 2e-4 on the returned x̂ (fp32 on both sides; one prior call agrees
to ~1e-5, see test_latent_full_gpu.py; the steps compound it roughly linearly).

Long horizon (round 4): ``DPSSampler.__call__`` with the full UNet for 50 guided iterations at
3x256², B = 1, inpainting, against the oracle loop on the CPU (about 80 s of CPU time); the
sample is compared after 1, 2, 5, 10, 25 and 50 iterations (``callback``) and the final x̂ at
the end, every error appended to ``gpurun_out/parity_record.jsonl`` (``parity_record``), so the
drift's growth with the step count is on record, not only the final bound.
"""

from __future__ import annotations

import copy

import numpy as np
import pytest
import torch

import stand_ins as si

pytestmark = pytest.mark.gpu

TOL = 2e-4


def _dps_problem(kind: str, shape, b: int, device):
    """(GPU inverse problem, CPU apply op, observation) for configs[1] / configs[2]."""
    from oracle import blur as oblur
    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.noise import GaussianNoise
    from samplers_amd.operators import GaussianBlurOperator, RandomInpaintingOperator

    x_true = si.fixture_x_true(b, shape, 11)
    gen = torch.Generator().manual_seed(12)
    if kind == "inpaint":
        op = RandomInpaintingOperator(shape, 0.5, seed=1)
        kept = op._kept_indices.cpu()

        def apply(v):
            return v.reshape(v.shape[0], -1)[:, kept]
    else:
        op = GaussianBlurOperator(shape, kernel_size=9, sigma=3.0)
        k1d = oblur.taps(9, 3.0)

        def apply(v):
            return oblur.blur(v, k1d).to(v.dtype)
    y = apply(x_true)
    y = y + 0.05 * torch.randn(y.shape, generator=gen)
    problem = InverseProblem(op.to(device), y.to(device), GaussianNoise(0.05).to(device))
    return problem, apply, y


@pytest.mark.parametrize("kind", ["inpaint", "blur"])
def test_dps_trajectory_celebahq_unet_matches_oracle(cuda, kind, parity_record):
    from oracle import dps_loop
    from samplers_amd.networks.ddpm import DDPMNetwork
    from samplers_amd.networks.unet2d import build_unet
    from samplers_amd.samplers import DPSSampler

    shape, b, steps = (3, 256, 256), 2, 8
    problem, apply, y = _dps_problem(kind, shape, b, cuda)
    gen = torch.Generator().manual_seed(13)
    init = torch.randn((b, *shape), generator=gen)
    xi = {i: torch.randn((b, *shape), generator=gen) for i in range(steps - 1, 1, -1)}

    net = DDPMNetwork.from_config(seed=0, device=cuda)
    fn = lambda k, i, s: (init if k == "init" else xi[i]).to(cuda)  # noqa: E731
    out = DPSSampler(net)(problem, num_sampling_steps=steps, gamma=1.0, eta=1.0,
                          noise_fn=fn).cpu()

    unet = build_unet(seed=0)
    acp = net.alphas_cumprod.cpu()
    ts = net.schedule.set_timesteps(steps).flip(0).tolist()
    ref = dps_loop.dps_reference(lambda v, t: unet(v, t), acp, ts, apply,
                                 dps_loop.gaussian_log_prob(0.05), y, init, lambda i: xi[i],
                                 gamma=1.0, eta=1.0)
    assert torch.isfinite(out).all()
    err = si.relative_error(out, ref)
    print(f"DPS {kind}: {steps - 2} guided steps + final x0, rel L2 vs oracle {err:.3e}")
    parity_record("x0_rel_l2", err, TOL, sampler="DPS", operator=kind, guided_steps=steps - 2,
                  batch=b, image=list(shape))
    assert err < TOL, f"DPS {kind}: {steps - 2} steps, rel L2 {err:.3e}"


def test_psld_trajectory_sd15_cfg_matches_oracle(cuda, parity_record):
    from oracle.latent_loops import psld_reference
    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.networks.latent import LatentDiffusionNetwork, StableDiffusionCondition
    from samplers_amd.noise import GaussianNoise
    from samplers_amd.operators import CenterInpaintingOperator
    from samplers_amd.samplers.psld import PSLDSampler

    b, shape, steps = 2, (3, 256, 256), 4  # PNDM list of 4: 3 guided iterations
    lshape = (4, 32, 32)
    gen = torch.Generator().manual_seed(21)
    pos = torch.randn(b, 77, 768, generator=gen)
    cond = StableDiffusionCondition(prompt=None, prompt_embeds=pos, guidance_scale=7.5)
    op = CenterInpaintingOperator(shape, 0.5)
    kept = op._kept_indices.cpu()
    n = int(np.prod(shape))

    def apply(v):
        return v.reshape(v.shape[0], -1)[:, kept]

    def adjoint(v):
        out = torch.zeros(v.shape[0], n, dtype=v.dtype)
        out = out.index_put((torch.arange(v.shape[0])[:, None], kept[None, :]), v)
        return out.reshape(v.shape[0], *shape)

    x_true = si.fixture_x_true(b, shape, 22)
    y = apply(x_true) + 0.05 * torch.randn(b, kept.numel(), generator=gen)
    z0 = torch.randn(b, *lshape, generator=gen)
    xi = {i: torch.randn(b, *lshape, generator=gen) for i in range(16)}

    cpu = LatentDiffusionNetwork.from_config(seed=0)
    gpu = copy.deepcopy(cpu).to(cuda)
    fn = lambda k, i, s: (z0 if k == "init" else xi[i]).to(cuda)  # noqa: E731
    problem = InverseProblem(op.to(cuda), y.to(cuda), GaussianNoise(0.05).to(cuda))
    out = PSLDSampler(gpu)(problem, num_sampling_steps=steps, condition=cond, noise_fn=fn).cpu()

    cpu.set_sampling_parameters(steps, batch_size=b)
    cpu.set_condition(cond)
    assert cpu._conditioning.do_classifier_free_guidance  # the doubled-batch path
    ref = psld_reference(lambda v, t: cpu(v, t), cpu.alphas_cumprod, cpu.timesteps_host, apply,
                         adjoint, lambda v: cpu.decode(v, differentiable=True),
                         lambda v: cpu.encode(v, differentiable=True), y, z0, lambda i: xi[i])
    assert torch.isfinite(out).all()
    err = si.relative_error(out, ref.reshape(out.shape))
    print(f"PSLD SD1.5 CFG: 3 guided steps + final decode, rel L2 vs oracle {err:.3e}")
    parity_record("x0_rel_l2", err, TOL, sampler="PSLD", cfg=True, guided_steps=3, batch=b,
                  image=list(shape))
    assert err < TOL, f"PSLD CFG: 3 steps, rel L2 {err:.3e}"


LONG_CHECKPOINTS = (1, 2, 5, 10, 25, 50)
LONG_TOL = 1e-3  # the sample after k guided iterations and the final x̂, relative L2


def _heartbeat(what: str, every: float = 20.0):
    """A line on the real stderr every `every` s while a long CPU oracle runs (pytest captures
    the test's own output; a silent minute reads as a hung GPU test on the pool)."""
    import sys
    import threading
    import time

    stop = threading.Event()
    t0 = time.perf_counter()

    def run():
        while not stop.wait(every):
            print(f"[{what}] still running at {time.perf_counter() - t0:.0f}s", file=sys.__stderr__,
                  flush=True)

    threading.Thread(target=run, daemon=True).start()
    return stop


@pytest.mark.timeout(900)
def test_dps_long_trajectory_celebahq_unet_matches_oracle(cuda, parity_record):
    """50 guided DPS iterations with the full prior (dps.py:90-122 runs N - 2 of them; the
    headline's N = 1000 is 998), the sample checked along the way and the final x̂ at the end."""
    from oracle import dps_loop
    from samplers_amd.networks.ddpm import DDPMNetwork
    from samplers_amd.networks.unet2d import build_unet
    from samplers_amd.samplers import DPSSampler

    shape, b, guided = (3, 256, 256), 1, LONG_CHECKPOINTS[-1]
    steps = guided + 2
    problem, apply, y = _dps_problem("inpaint", shape, b, cuda)
    gen = torch.Generator().manual_seed(31)
    init = torch.randn((b, *shape), generator=gen)
    xi = {i: torch.randn((b, *shape), generator=gen) for i in range(steps - 1, 1, -1)}

    net = DDPMNetwork.from_config(seed=0, device=cuda)
    seen: dict[int, torch.Tensor] = {}

    def keep(i, x):
        done = steps - 1 - i + 1  # guided iterations finished (i runs steps-1 .. 2)
        if done in LONG_CHECKPOINTS:
            seen[done] = x.detach().cpu().clone()

    fn = lambda k, i, s: (init if k == "init" else xi[i]).to(cuda)  # noqa: E731
    out = DPSSampler(net)(problem, num_sampling_steps=steps, gamma=1.0, eta=1.0, noise_fn=fn,
                          callback=keep).cpu()
    assert sorted(seen) == list(LONG_CHECKPOINTS)

    stop = _heartbeat("long DPS oracle")
    try:
        unet = build_unet(seed=0)
        acp = net.alphas_cumprod.cpu()
        ts = net.schedule.set_timesteps(steps).flip(0).tolist()
        lp = dps_loop.gaussian_log_prob(0.05)
        eps = lambda v, t: unet(v, t)  # noqa: E731
        sample, done, errs = init, 0, {}
        for c in LONG_CHECKPOINTS:
            i_cur = steps - 1 - done  # the next loop index of dps.py's loop
            sample = dps_loop.dps_reference(eps, acp, ts[:i_cur + 1], apply, lp, y, sample,
                                            lambda i: xi[i], gamma=1.0, eta=1.0,
                                            steps_limit=c - done, return_sample=True)
            done = c
            errs[c] = si.relative_error(seen[c], sample)
            parity_record("sample_rel_l2", errs[c], LONG_TOL, sampler="DPS", operator="inpaint",
                          guided_steps=c, of=guided, batch=b, image=list(shape))
        ref = dps_loop.dps_reference(eps, acp, ts[:2], apply, lp, y, sample, lambda i: xi[i],
                                     gamma=1.0, eta=1.0)
    finally:
        stop.set()
    err = si.relative_error(out, ref)
    parity_record("x0_rel_l2", err, LONG_TOL, sampler="DPS", operator="inpaint",
                  guided_steps=guided, batch=b, image=list(shape))
    print("DPS long trajectory: " + ", ".join(f"{k}: {v:.2e}" for k, v in errs.items())
          + f"; final x0 {err:.2e}")
    assert all(v < LONG_TOL for v in errs.values()), errs
    assert err < LONG_TOL, err


@pytest.mark.timeout(900)
def test_psld_long_trajectory_sd15_cfg_matches_oracle(cuda, parity_record):
    """20 guided PSLD iterations through the SD 1.5 VAE and ε-UNet with CFG on (psld.py's loop
    over the PNDM timesteps), batch 1 at 3x256²: the final x̂ against oracle/latent_loops.py on
    the CPU with the same weights and injected noise."""
    from oracle.latent_loops import psld_reference
    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.networks.latent import LatentDiffusionNetwork, StableDiffusionCondition
    from samplers_amd.noise import GaussianNoise
    from samplers_amd.operators import CenterInpaintingOperator
    from samplers_amd.samplers.psld import PSLDSampler

    b, shape, steps = 1, (3, 256, 256), 21  # PNDM list of 21: 20 guided iterations
    lshape = (4, 32, 32)
    gen = torch.Generator().manual_seed(23)
    cond = StableDiffusionCondition(prompt=None, prompt_embeds=torch.randn(b, 77, 768, generator=gen),
                                    guidance_scale=7.5)
    op = CenterInpaintingOperator(shape, 0.5)
    kept = op._kept_indices.cpu()
    n = int(np.prod(shape))

    def apply(v):
        return v.reshape(v.shape[0], -1)[:, kept]

    def adjoint(v):
        out = torch.zeros(v.shape[0], n, dtype=v.dtype)
        out = out.index_put((torch.arange(v.shape[0])[:, None], kept[None, :]), v)
        return out.reshape(v.shape[0], *shape)

    x_true = si.fixture_x_true(b, shape, 24)
    y = apply(x_true) + 0.05 * torch.randn(b, kept.numel(), generator=gen)
    z0 = torch.randn(b, *lshape, generator=gen)
    xi = {i: torch.randn(b, *lshape, generator=gen) for i in range(steps + 2)}

    cpu = LatentDiffusionNetwork.from_config(seed=0)
    gpu = copy.deepcopy(cpu).to(cuda)
    fn = lambda k, i, s: (z0 if k == "init" else xi[i]).to(cuda)  # noqa: E731
    problem = InverseProblem(op.to(cuda), y.to(cuda), GaussianNoise(0.05).to(cuda))
    out = PSLDSampler(gpu)(problem, num_sampling_steps=steps, condition=cond, noise_fn=fn).cpu()

    stop = _heartbeat("long PSLD oracle")
    try:
        cpu.set_sampling_parameters(steps, batch_size=b)
        cpu.set_condition(cond)
        ref = psld_reference(lambda v, t: cpu(v, t), cpu.alphas_cumprod, cpu.timesteps_host, apply,
                             adjoint, lambda v: cpu.decode(v, differentiable=True),
                             lambda v: cpu.encode(v, differentiable=True), y, z0, lambda i: xi[i])
    finally:
        stop.set()
    assert torch.isfinite(out).all()
    err = si.relative_error(out, ref.reshape(out.shape))
    print(f"PSLD SD1.5 CFG: {steps - 1} guided steps + final decode, rel L2 vs oracle {err:.3e}")
    parity_record("x0_rel_l2", err, LONG_TOL, sampler="PSLD", cfg=True, guided_steps=steps - 1, batch=b,
                  image=list(shape))
    assert err < LONG_TOL, f"PSLD CFG: {steps - 1} steps, rel L2 {err:.3e}"

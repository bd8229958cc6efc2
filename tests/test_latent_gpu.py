"""PGDM and PSLD on the GPU against the reference's golden vectors and the oracle loops.

Tolerance: relative L2 <= max(1e-5, 20 x the case's fp32-vs-fp64 sensitivity), the
sensitivity measured here with the fp64 oracle (tests/test_oracle_latent.py pins the
fp32 oracle to the reference bit-exactly).  PGDM amplifies perturbations strongly on
these stand-in priors (its outputs reach 1e7), hence the per-case bound.
"""

import types

import numpy as np
import pytest
import torch

import stand_ins as si
from golden_cases import dps_case_names, load_dps_case
from oracle import blur as oblur
from oracle.latent_loops import pgdm_reference, psld_reference
from samplers_amd.inverse_problem import InverseProblem
from samplers_amd.noise import GaussianNoise
from samplers_amd.operators import GaussianBlurOperator, IdentityOperator, InpaintingOperator
from samplers_amd.samplers.pgdm import PGDMSampler
from samplers_amd.samplers.psld import PSLDSampler
from test_oracle_latent import oracle_pgdm, oracle_psld

pytestmark = pytest.mark.gpu


def _problem(case, device):
    op = (IdentityOperator(case.shape) if case.kept is None
          else InpaintingOperator(case.shape, case.mask).to(device))
    return InverseProblem(op, case.y.to(device), GaussianNoise(0.05).to(device))


def _noise_fn(case, device):
    init, steps = case.noise()
    return lambda kind, i, s: (init if kind == "init" else steps[i]).to(device)


def _tol(case, oracle_fn):
    cond = si.relative_error(oracle_fn(case, torch.float64), case.out)
    return max(1e-5, 20 * cond)


@pytest.mark.parametrize("name", dps_case_names("pgdm"))
def test_pgdm_matches_reference_golden(cuda, name):
    case = load_dps_case(name)
    m = case.meta
    net = si.make_samplers_amd_net(m["prior"], case.shape[0], m["coef"], device=cuda)
    out = PGDMSampler(net)(_problem(case, cuda), num_sampling_steps=m["N"],
                           num_reconstructions=m["R"], guidance_weight=m["guidance_weight"],
                           eta=m["eta"], noise_fn=_noise_fn(case, cuda))
    assert tuple(out.shape) == tuple(m["out_shape"])
    assert si.relative_error(out.cpu(), case.out) < _tol(case, oracle_pgdm)


def test_pgdm_inpainting_matches_oracle(cuda):
    """The reference cannot run PGDM with a flattened observation (F5); the oracle loop
    with A^+ = A^T pins it."""
    shape, b, N = (3, 32, 32), 2, 8
    mask = si.fixture_mask(shape, "random")
    op = InpaintingOperator(shape, mask)
    kept = op._kept_indices
    x_true = si.fixture_x_true(b, shape, 0)
    y = op.apply(x_true) + 0.05 * torch.randn(b, kept.numel(), generator=torch.Generator().manual_seed(1))
    init, steps = si.replay_noise(5, (b, *shape), N)
    net = si.make_samplers_amd_net("conv", 3, 0.1, device=cuda)
    fn = lambda kind, i, s: (init if kind == "init" else steps[i]).to(cuda)  # noqa: E731
    out = PGDMSampler(net)(InverseProblem(op.to(cuda), y.to(cuda), GaussianNoise(0.05).to(cuda)),
                           num_sampling_steps=N, guidance_weight=0.05, noise_fn=fn)
    acp = torch.cat([torch.ones(1), si.ddpm_alphas_cumprod()]).clip(1e-6, 1)
    kc = kept.cpu()

    def apply(x):
        return x.reshape(x.shape[0], -1)[:, kc]

    def pinv(v):
        o = torch.zeros(v.shape[0], int(np.prod(shape)), dtype=v.dtype)
        o[:, kc] = v
        return o.reshape(v.shape[0], *shape)

    def run(dt):
        c = si.EpsCore("conv", 3, 0.1).to(dt)
        return pgdm_reference(lambda x, t: c(x, t), acp.to(dt),
                              si.leading_timesteps_ascending(N).tolist(), apply, pinv, y.to(dt),
                              init.to(dt), lambda i: steps[i].to(dt), guidance_weight=0.05, eta=1.0)

    ref = run(torch.float32)
    cond = si.relative_error(run(torch.float64), ref)  # PGDM amplifies rounding (outputs ~1e4)
    assert si.relative_error(out.cpu(), ref) < max(1e-4, 20 * cond)


def test_pgdm_rejects_operator_without_pinv(cuda):
    net = si.make_samplers_amd_net("linear", 3, 0.1, device=cuda)
    op = GaussianBlurOperator((3, 32, 32)).to(cuda)
    ip = InverseProblem(op, torch.zeros(1, 3, 32, 32, device=cuda), GaussianNoise(0.1).to(cuda))
    with pytest.raises(NotImplementedError):
        PGDMSampler(net)(ip, num_sampling_steps=4)


@pytest.mark.parametrize("name", dps_case_names("psld"))
def test_psld_matches_reference_golden(cuda, name):
    case = load_dps_case(name)
    m = case.meta
    net = si.make_samplers_amd_latent_net(m["prior"], m["coef"], device=cuda)
    out = PSLDSampler(net)(_problem(case, cuda), num_sampling_steps=m["N"],
                           num_reconstructions=m["R"], gamma=m["gamma"], omega=m["omega"],
                           eta=m["eta"], noise_fn=_noise_fn(case, cuda))
    assert tuple(out.shape) == tuple(m["out_shape"])
    assert si.relative_error(out.cpu(), case.out) < _tol(case, oracle_psld)


def test_psld_batched_inpainting_matches_oracle(cuda):
    """Batch > 1 with a flattened observation (fails in the reference, F5)."""
    shape, b, N = (3, 32, 32), 3, 8
    mask = si.fixture_mask(shape, "center")
    op = InpaintingOperator(shape, mask)
    kc = op._kept_indices
    x_true = si.fixture_x_true(b, shape, 2)
    y = op.apply(x_true) + 0.05 * torch.randn(b, kc.numel(), generator=torch.Generator().manual_seed(3))
    net = si.make_samplers_amd_latent_net("conv", 0.1, device=cuda)
    lat = net.get_latent_shape(shape)
    init, steps = si.replay_noise(9, (b, *lat), N)
    fn = lambda kind, i, s: (init if kind == "init" else steps[i]).to(cuda)  # noqa: E731
    out = PSLDSampler(net)(InverseProblem(op.to(cuda), y.to(cuda), GaussianNoise(0.05).to(cuda)),
                           num_sampling_steps=N, noise_fn=fn)
    core, vae = si.EpsCore("conv", 4, 0.1), si.LatentCore()
    acp = torch.cat([torch.ones(1), si.ddpm_alphas_cumprod()]).clip(1e-6, 1)
    n = int(np.prod(shape))

    def apply(x):
        return x.reshape(x.shape[0], -1)[:, kc]

    def adjoint(v):
        o = torch.zeros(v.shape[0], n, dtype=v.dtype)
        o[:, kc] = v
        return o.reshape(v.shape[0], *shape)

    ref = psld_reference(lambda x, t: core(x, t), acp, si.leading_timesteps_ascending(N).tolist(),
                         apply, adjoint, vae.decode, vae.encode, y, init, lambda i: steps[i])
    assert si.relative_error(out.cpu(), ref) < 1e-4


def test_psld_blur_matches_oracle(cuda):
    shape, b, N = (3, 32, 32), 2, 6
    k = oblur.taps(9, 3.0)
    x_true = si.fixture_x_true(b, shape, 4)
    y = oblur.blur(x_true, k).float() + 0.05 * torch.randn(b, *shape, generator=torch.Generator().manual_seed(4))
    net = si.make_samplers_amd_latent_net("conv", 0.1, device=cuda)
    lat = net.get_latent_shape(shape)
    init, steps = si.replay_noise(13, (b, *lat), N)
    fn = lambda kind, i, s: (init if kind == "init" else steps[i]).to(cuda)  # noqa: E731
    op = GaussianBlurOperator(shape, 9, 3.0).to(cuda)
    out = PSLDSampler(net)(InverseProblem(op, y.to(cuda), GaussianNoise(0.05).to(cuda)),
                           num_sampling_steps=N, noise_fn=fn)
    core, vae = si.EpsCore("conv", 4, 0.1), si.LatentCore()
    acp = torch.cat([torch.ones(1), si.ddpm_alphas_cumprod()]).clip(1e-6, 1)
    ref = psld_reference(lambda x, t: core(x, t), acp, si.leading_timesteps_ascending(N).tolist(),
                         lambda x: oblur.blur(x, k).float(), lambda v: oblur.blur_adjoint(v, k).float(),
                         vae.decode, vae.encode, y, init, lambda i: steps[i])
    assert si.relative_error(out.cpu(), ref) < 1e-4


def test_psld_requires_latent_network(cuda):
    net = si.make_samplers_amd_net("linear", 3)
    with pytest.raises(TypeError, match="latent diffusion model"):
        PSLDSampler(net)


@pytest.mark.parametrize("name", dps_case_names("rs"))
def test_resample_matches_reference_golden(cuda, name):
    from samplers_amd.noise import PoissonNoise
    from samplers_amd.samplers.resample import ReSampleSampler
    from test_oracle_latent import oracle_resample

    case = load_dps_case(name)
    m = case.meta
    op = (IdentityOperator(case.shape) if case.kept is None
          else InpaintingOperator(case.shape, case.mask).to(cuda))
    noise = PoissonNoise(1.0) if m["noise"] == "poisson" else GaussianNoise(1e-3)
    prob = InverseProblem(op, case.y.to(cuda), noise.to(cuda))
    gen = torch.Generator().manual_seed(m["seed"])
    drawn = []

    def fn(kind, key, shape):  # the reference's sequential draw order
        t = torch.randn(shape, generator=gen)
        drawn.append(list(shape))
        return t.to(cuda)

    net = si.make_samplers_amd_latent_net("conv", 0.1, device=cuda)
    out = ReSampleSampler(net)(prob, num_sampling_steps=m["N"], num_reconstructions=m["R"],
                               max_optimization_iters=m["max_iters"], eta=m["eta"],
                               inter_timesteps=m["inter_timesteps"],
                               time_travel_interval=m["time_travel_interval"],
                               stage_splits=m["stage_splits"], noise_fn=fn)
    assert drawn == m["draw_shapes"]
    assert tuple(out.shape) == tuple(m["out_shape"])
    assert si.relative_error(out.cpu(), case.out) < _tol(case, oracle_resample)


def test_adamw_step_matches_torch(cuda):
    from samplers_amd import _hip
    from samplers_amd.samplers.resample import adamw_coefficients

    torch.manual_seed(0)
    p0 = torch.randn(1003)
    ref = p0.clone().requires_grad_()
    opt = torch.optim.AdamW([ref], lr=5e-3)
    p = p0.clone().to(cuda)
    mm, vv = torch.zeros_like(p), torch.zeros_like(p)
    lib = _hip.load_library()
    for step in range(1, 6):
        g = torch.randn(1003)
        ref.grad = g.clone()
        opt.step()
        gd = g.to(cuda)  # held while the kernel runs
        _hip.check(lib.sp_adamw_step(p.data_ptr(), gd.data_ptr(), mm.data_ptr(),
                                     vv.data_ptr(), p.numel(), adamw_coefficients(step, 5e-3),
                                     torch.cuda.current_stream().cuda_stream), "adamw")
    torch.testing.assert_close(p.cpu(), ref.detach(), rtol=1e-6, atol=1e-6)


def test_resample_requires_latent_network(cuda):
    from samplers_amd.samplers.resample import ReSampleSampler

    with pytest.raises(TypeError, match="latent diffusion model"):
        ReSampleSampler(si.make_samplers_amd_net("linear", 3))


@pytest.mark.parametrize("kind", ["identity", "inpaint", "mask", "blur"])
def test_pixel_optimization_device_stop_matches_reference_loop(cuda, kind):
    """ReSample's pixel-space hard consistency (resample_kernels.py:32-54) with the stopping
    test on the device (sp_pixel_opt_step / sp_adamw_step_until + sp_opt_check) runs exactly
    the iterations of the reference loop (torch AdamW + MSELoss + .item() per iteration):
    the threshold is placed between two consecutive losses of the reference, at an
    iteration that is not a multiple of the host's flag-check interval."""
    from samplers_amd.operators import GaussianBlurOperator, get_mask_random
    from samplers_amd.samplers.resample import ReSampleSampler, _Consistency, _finish_log

    torch.manual_seed(0)
    shape, b = (3, 16, 24), 2
    if kind == "identity":
        op = IdentityOperator(shape)
    elif kind == "blur":
        op = GaussianBlurOperator(shape, 5, 1.5).to(cuda)
    else:
        op = InpaintingOperator(shape, get_mask_random(shape, 0.4, seed=2),
                                flatten=(kind == "inpaint")).to(cuda)
    x_true = torch.rand(b, *shape) * 2 - 1
    x0 = torch.randn(b, *shape)
    y = op.apply(x_true.to(cuda)).reshape(b, -1).cpu()
    total = y.numel()

    def reference(n_iter, thr=None):
        opt = x0.clone().requires_grad_()
        adam = torch.optim.AdamW([opt], lr=1e-2)
        losses = []
        for _ in range(n_iter):
            adam.zero_grad()
            loss = torch.nn.MSELoss()(y, op.apply(opt.to(cuda)).reshape(b, -1).cpu())
            loss.backward()
            adam.step()
            losses.append(loss.item())
            if thr is not None and loss.item() < thr:
                break
        return opt.detach(), losses

    _, losses = reference(40)
    stop_at = 22  # 0-based iteration whose loss first falls below the threshold
    assert losses[stop_at] < losses[stop_at - 1]
    thr = 0.5 * (losses[stop_at] + losses[stop_at - 1])
    assert all(v >= thr for v in losses[:stop_at])
    ref, ref_losses = reference(2000, thr)
    assert len(ref_losses) == stop_at + 1
    cons = _Consistency(op, y.to(cuda), 1)
    holder = types.SimpleNamespace()  # stands in for the sampler: receives the solve's record
    out = ReSampleSampler._pixel_optimization(holder, x0.to(cuda), cons, total, thr ** 0.5, 2000)
    err = float((out.cpu() - ref).norm() / ref.norm())
    _finish_log(holder)  # the sampler reads the queued loss logs once, at the end of its call
    (rec,) = holder.optimization_log  # the iterations the stopping rule ran, from the device
    assert rec["kind"] == "pixel" and rec["iterations"] == stop_at + 1 and rec["stopped_early"]
    assert abs(rec["final_loss"] - ref_losses[-1]) <= 1e-5 * abs(ref_losses[-1])
    one_more, _ = reference(stop_at + 2)
    assert err < 1e-5, err
    assert float((one_more - ref).norm() / ref.norm()) > 100 * max(err, 1e-7)


@pytest.mark.parametrize("steps,interval", [(30, 10), (24, 5), (101, 10)])
def test_resample_whole_call_projection_counts_match_the_sampler(cuda, steps, interval):
    """tools/bench_resample.py projects a whole ReSample call from per-iteration costs times the
    loop's counts (project_full_call walks resample.py's loop control without running it).  The
    counts must be the sampler's own: the pixel- and latent-space solves its optimization_log
    records, run here with stand-in priors (max_optimization_iters = 2: a few launches each)."""
    import importlib.util
    import pathlib

    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.noise import PoissonNoise
    from samplers_amd.operators import IdentityOperator
    from samplers_amd.samplers.resample import ReSampleSampler

    path = pathlib.Path(__file__).resolve().parents[1] / "tools" / "bench_resample.py"
    spec = importlib.util.spec_from_file_location("bench_resample_tool", path)
    tool = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(tool)
    shape = (3, 16, 16)
    net = si.make_samplers_amd_latent_net("linear", 0.1, device=cuda)
    x = si.fixture_x_true(1, shape, 3)
    y = torch.poisson((x + 1) * 8, generator=torch.Generator().manual_seed(4)) / 8 - 1
    prob = InverseProblem(IdentityOperator(shape), y.to(cuda), PoissonNoise(1.0).to(cuda))
    sampler = ReSampleSampler(net)
    sampler(prob, num_sampling_steps=steps, max_optimization_iters=2, time_travel_interval=interval,
            seed=5)
    log = sampler.optimization_log
    net.set_sampling_parameters(steps, batch_size=1)
    proj = tool.project_full_call(len(net.timesteps_host), 2, interval, 1.0, 1.0, 1.0, 1.0, 1)
    assert proj["pixel_solves"] == sum(r["kind"] == "pixel" for r in log)
    assert proj["latent_solves"] == sum(r["kind"] == "latent" for r in log)
    assert proj["main_loop_iterations"] == len(net.timesteps_host) - 2
    assert all(r["loop_trips"] >= r["iterations"] for r in log)

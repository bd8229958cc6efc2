"""DPSSampler on the GPU against the reference's golden vectors and the oracle.

Tolerance: 1e-5 relative L2 on the final x-hat.  The reference's own fp32-vs-fp64
sensitivity on these cases is <= 1e-6 (tests/test_oracle.py::test_golden_conditioning),
so 1e-5 leaves 10x headroom for the different summation order of the fused kernels
and the device's fma contraction.
"""

import math

import numpy as np
import pytest
import torch

import stand_ins as si
from golden_cases import dps_case_names, load_dps_case
from oracle import blur as oblur
from oracle import dps_loop
from samplers_amd.inverse_problem import InverseProblem
from samplers_amd.noise import GaussianNoise, PoissonNoise
from samplers_amd.operators import GaussianBlurOperator, IdentityOperator, InpaintingOperator
from samplers_amd.samplers import DPSSampler

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _problem(case, device):
    m = case.meta
    shape = case.shape
    if m["op"] == "identity":
        op = IdentityOperator(shape)
    else:
        op = InpaintingOperator(shape, case.mask).to(device)
    noise = GaussianNoise(0.05) if m["noise"] == "gauss" else PoissonNoise(1.0)
    return InverseProblem(op, case.y.to(device), noise.to(device))


def _noise_fn(case, device):
    init, steps = case.noise()

    def fn(kind, i, shape):
        t = init if kind == "init" else steps[i]
        assert tuple(t.shape) == tuple(shape)
        return t.to(device)

    return fn


@pytest.mark.parametrize("name", dps_case_names())
def test_dps_matches_reference_golden(cuda, name):
    case = load_dps_case(name)
    m = case.meta
    net = si.make_samplers_amd_net(m["prior"], case.shape[0], m["coef"], device=cuda)
    out = DPSSampler(net)(_problem(case, cuda), num_sampling_steps=m["N"], num_reconstructions=m["R"],
                          gamma=m["gamma"], eta=m["eta"], noise_fn=_noise_fn(case, cuda))
    assert tuple(out.shape) == tuple(m["out_shape"])
    err = si.relative_error(out.cpu(), case.out)
    assert err < TOL, err


def test_dps_micro_batch_equals_full_batch(cuda):
    case = load_dps_case("dps_rnd_poiss_conv_b4")
    m = case.meta
    net = si.make_samplers_amd_net(m["prior"], case.shape[0], m["coef"], device=cuda)
    kw = dict(num_sampling_steps=m["N"], gamma=m["gamma"], eta=m["eta"], rng="philox", seed=5)
    a = DPSSampler(net)(_problem(case, cuda), **kw)
    b = DPSSampler(net)(_problem(case, cuda), micro_batch=1, **kw)
    assert torch.equal(a, b)


def test_dps_philox_sharding_is_world_size_invariant(cuda):
    """Running samples [0,2) and [2,4) as two shards reproduces the 4-sample run."""
    case = load_dps_case("dps_id_gauss_conv_b4")
    m = case.meta
    net = si.make_samplers_amd_net(m["prior"], case.shape[0], m["coef"], device=cuda)
    kw = dict(num_sampling_steps=m["N"], gamma=m["gamma"], eta=m["eta"], rng="philox", seed=11)
    full = DPSSampler(net)(_problem(case, cuda), **kw)
    shards = []
    for b0 in (0, 2):
        p = _problem(case, cuda)
        p = InverseProblem(p.operator, p.observation[b0:b0 + 2], p.noise)
        shards.append(DPSSampler(net)(p, sample_offset=b0, **kw))
    assert torch.equal(full, torch.cat(shards))


def test_dps_torch_rng_mode_runs(cuda):
    case = load_dps_case("dps_id_gauss_lin_b1")
    m = case.meta
    net = si.make_samplers_amd_net(m["prior"], case.shape[0], m["coef"], device=cuda)
    torch.manual_seed(0)
    a = DPSSampler(net)(_problem(case, cuda), num_sampling_steps=m["N"], rng="torch", gamma=0.01)
    torch.manual_seed(0)
    b = DPSSampler(net)(_problem(case, cuda), num_sampling_steps=m["N"], rng="torch", gamma=0.01)
    assert torch.equal(a, b) and torch.isfinite(a).all()


@pytest.mark.parametrize("noise_kind", ["gauss", "poisson"])
def test_dps_blur_matches_oracle(cuda, noise_kind):
    """Blur has no reference implementation: the oracle loop (dps.py restated) with the
    oracle blur pins it."""
    shape, b, N = (3, 32, 32), 2, 8
    x_true = si.fixture_x_true(b, shape, 0)
    k = oblur.taps(9, 3.0)
    gen = torch.Generator().manual_seed(3)
    y = oblur.blur(x_true, k).float() + 0.05 * torch.randn(b, *shape, generator=gen)
    noise = GaussianNoise(0.05) if noise_kind == "gauss" else PoissonNoise(1.0)
    op = GaussianBlurOperator(shape, 9, 3.0).to(cuda)
    net = si.make_samplers_amd_net("conv", 3, 0.1, device=cuda)
    init, steps = si.replay_noise(21, (b, *shape), N)
    fn = lambda kind, i, s: (init if kind == "init" else steps[i]).to(cuda)  # noqa: E731
    out = DPSSampler(net)(InverseProblem(op, y.to(cuda), noise.to(cuda)), num_sampling_steps=N,
                          gamma=1e-2, eta=1.0, noise_fn=fn)
    core = si.EpsCore("conv", 3, 0.1)
    acp = torch.cat([torch.ones(1), si.ddpm_alphas_cumprod()]).clip(1e-6, 1)
    lp = dps_loop.gaussian_log_prob(0.05) if noise_kind == "gauss" else dps_loop.poisson_log_prob(1.0)
    ref = dps_loop.dps_reference(lambda x, t: core(x, t), acp,
                                 si.leading_timesteps_ascending(N).tolist(),
                                 lambda x: oblur.blur(x, k).float(), lp, y, init,
                                 lambda i: steps[i], gamma=1e-2, eta=1.0)
    assert si.relative_error(out.cpu(), ref) < 1e-4


@pytest.mark.parametrize("name", dps_case_names("dps_*_bounded"))
def test_dps_bounded_golden_elementwise(cuda, name):
    """The bounded-magnitude golden trajectories (|x-hat| of order 1): every element, not only
    the relative L2 that the large pixels of the diverging cases dominate."""
    case = load_dps_case(name)
    m = case.meta
    net = si.make_samplers_amd_net(m["prior"], case.shape[0], m["coef"], device=cuda)
    out = DPSSampler(net)(_problem(case, cuda), num_sampling_steps=m["N"], num_reconstructions=m["R"],
                          gamma=m["gamma"], eta=m["eta"], noise_fn=_noise_fn(case, cuda))
    ref = case.out.numpy()
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())

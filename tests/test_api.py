"""Plugin-API behaviour on the host (mirrors the reference's own tests:
tests/operators/test_inpainting.py, test_linear.py, tests/samplers/test_batch_view.py,
plus the error conventions of SURVEY.md §8b)."""

import math

import numpy as np
import pytest
import torch

from samplers_amd.inverse_problem import InverseProblem
from samplers_amd.noise import GaussianNoise, PoissonNoise
from samplers_amd.operators import (CenterInpaintingOperator, CenterOutpaintingOperator,
                                    GaussianBlurOperator, GeneralSVDOperator, IdentityOperator,
                                    InpaintingOperator, RandomInpaintingOperator,
                                    SidePaintingOperator, get_mask_inpaint_center,
                                    get_mask_side_painting)
from samplers_amd.samplers.utils.batch_view import BatchView
from samplers_amd.samplers.utils.bridge_kernels import bridge_coefficients


def _roundtrip(op, x):
    kept = op.apply_V_transpose(x)
    recon = op.apply_V(kept)
    bm = op.mask.unsqueeze(0).expand_as(x)
    assert torch.equal(recon[~bm], x[~bm])
    assert torch.all(recon[bm] == 0)
    m, n = op.shape
    assert m == int((~op.mask).sum()) and n == op.mask.numel()
    assert op.get_singular_values().numel() == m


@pytest.mark.parametrize("b,c,h,w", [(2, 3, 4, 4), (1, 1, 5, 7)])
def test_center_inpaint_roundtrip(b, c, h, w):
    _roundtrip(CenterInpaintingOperator((c, h, w), paint_fraction=0.5), torch.randn(b, c, h, w))


@pytest.mark.parametrize("b,c,h,w", [(2, 3, 4, 4), (1, 1, 6, 6)])
def test_center_outpaint_roundtrip(b, c, h, w):
    _roundtrip(CenterOutpaintingOperator((c, h, w), keep_fraction=0.5), torch.randn(b, c, h, w))


@pytest.mark.parametrize("left", [True, False])
def test_side_paint_roundtrip(left):
    _roundtrip(SidePaintingOperator((3, 4, 8), paint_fraction=0.5, left=left), torch.randn(2, 3, 4, 8))


def test_manual_mask_constructor_counts():
    mask = get_mask_inpaint_center((3, 4, 4), 0.25, 0.75)
    op = InpaintingOperator((3, 4, 4), mask)
    m, n = op.shape
    assert m + int(mask.sum()) == n
    assert op.y_shape == (m,)


def test_inpaint_packed_order_is_nonzero_order():
    mask = torch.rand(3, 9, 11) < 0.5
    op = InpaintingOperator((3, 9, 11), mask)
    x = torch.randn(2, 3, 9, 11)
    kept = torch.nonzero(~mask.flatten()).squeeze(1)
    assert torch.equal(op.apply(x), x.reshape(2, -1)[:, kept])


def test_mask_must_match_x_shape():
    with pytest.raises(ValueError):
        InpaintingOperator((3, 4, 4), torch.zeros(4, 4, dtype=torch.bool))


def test_uint8_mask_becomes_bool():
    op = InpaintingOperator((1, 2, 2), torch.tensor([[[0, 3], [1, 0]]], dtype=torch.uint8))
    assert op.mask.dtype == torch.bool and op.shape == (2, 4)


def test_flatten_false_is_constructible():
    mask = get_mask_side_painting((2, 3, 4), 0.5, True)
    op = InpaintingOperator((2, 3, 4), mask, flatten=False)
    x = torch.randn(5, 2, 3, 4)
    assert op.y_shape == (2, 3, 4)
    assert torch.equal(op.apply(x), x.masked_fill(mask, 0))


def test_fraction_validation():
    with pytest.raises(ValueError):
        CenterInpaintingOperator((1, 4, 4), paint_fraction=1.5)
    with pytest.raises(ValueError):
        get_mask_side_painting((1, 4, 4), 0.0)
    with pytest.raises(ValueError):
        get_mask_inpaint_center((1, 4, 4), 0.7, 0.2)


def test_random_mask_fraction():
    op = RandomInpaintingOperator((3, 64, 64), 0.5, seed=1)
    frac = op.mask.float().mean().item()
    assert 0.45 < frac < 0.55
    assert torch.equal(op.mask[0], op.mask[2])


@pytest.fixture(scope="module")
def svd_op():
    torch.manual_seed(0)
    H = torch.randn(12, 7)
    U, s, Vh = torch.linalg.svd(H, full_matrices=False)
    return GeneralSVDOperator(U, s, Vh)


def _dense(op):
    return (op._U * op._singular_values.unsqueeze(0)) @ op._V_transpose


def test_svd_apply(svd_op):
    x = torch.randn(5, svd_op.shape[1])
    torch.testing.assert_close(svd_op.apply(x), x @ _dense(svd_op).T)


def test_svd_transpose(svd_op):
    y = torch.randn(5, svd_op.shape[0])
    torch.testing.assert_close(svd_op.apply_transpose(y), y @ _dense(svd_op))


def test_svd_pinv(svd_op):
    y = torch.randn(5, svd_op.shape[0])
    torch.testing.assert_close(svd_op.apply_pseudo_inverse(y), y @ torch.linalg.pinv(_dense(svd_op)).T)


def test_identity_flatten_roundtrip():
    op = IdentityOperator((3, 4, 5), flatten=True)
    x = torch.randn(2, 3, 4, 5)
    assert op.y_shape == (60,)
    assert torch.equal(op.apply_transpose(op.apply(x)), x)
    assert IdentityOperator((3, 4, 5)).apply(x) is x


def test_blur_host_adjoint_and_normalisation():
    op = GaussianBlurOperator((2, 16, 18), 9, 3.0)
    assert abs(op.taps.sum().item() - 1) < 1e-6
    ones = torch.ones(1, 2, 16, 18)
    torch.testing.assert_close(op.apply(ones), ones)
    x, y = torch.randn(3, 2, 16, 18), torch.randn(3, 2, 16, 18)
    lhs = (op.apply(x) * y).sum()
    rhs = (x * op.apply_transpose(y)).sum()
    assert abs(lhs - rhs) < 1e-4 * abs(lhs)
    with pytest.raises(NotImplementedError):
        op.apply_pseudo_inverse(y)


def test_blur_rejects_tiny_images():
    with pytest.raises(ValueError):
        GaussianBlurOperator((1, 8, 8), 9, 3.0)


def test_batch_view_shapes():
    assert BatchView((2, 3), 4, (3, 64, 64)).shape == (2, 3, 4, 3, 64, 64)
    assert BatchView((), 2, (1, 8, 8)).shape == (2, 1, 8, 8)
    v = BatchView((2,), 3, (1, 4))
    assert v.flat_shape == (6, 1, 4) and v.per_sample_broadcast_shape == (6, 1, 1)
    obs = torch.arange(8.0).reshape(2, 1, 4)
    rep = v.repeat_observation(obs)
    assert rep.shape == (6, 1, 4) and torch.equal(rep[2], obs[0]) and torch.equal(rep[3], obs[1])
    flat_obs = torch.arange(6.0).reshape(2, 3)
    assert v.repeat_observation(flat_obs, sample_ndim=1).shape == (6, 3)


def test_noise_validation_and_log_prob():
    with pytest.raises(ValueError):
        GaussianNoise(0.0)
    with pytest.raises(ValueError):
        PoissonNoise(-1.0)
    with pytest.raises(ValueError):
        GaussianNoise(torch.ones(2))
    r = torch.randn(3, 10)
    g = GaussianNoise(0.5)
    torch.testing.assert_close(g.log_prob(r), -(r**2).sum(1) / (2 * 0.25))
    torch.testing.assert_close(g.score(r), -r / 0.25)
    p = PoissonNoise(2.0)
    torch.testing.assert_close(p.log_prob(r), -(r**2).sum(1) / 2.001)
    assert abs(g.grad_scale() - 4.0) < 1e-6
    assert abs(p.grad_scale() - 2 / 2.001) < 1e-6


def test_inverse_problem_from_clean_data():
    op = CenterInpaintingOperator((3, 8, 8), 0.5)
    x = torch.randn(2, 3, 8, 8)
    gen = torch.Generator().manual_seed(0)
    ip = InverseProblem.from_clean_data(x, operator=op, noise=GaussianNoise(0.1), rng=gen)
    assert tuple(ip.batch_shape) == (2,)
    assert ip.observation.shape == (2, op.shape[0])
    assert torch.allclose(ip.residual(x), ip.observation - op.apply(x))


def test_bridge_coefficients_ddpm_limit():
    """With s = 0 (alpha_bar_s = 1) and eta = 1 the bridge is the DDPM posterior."""
    betas = np.linspace(1e-4, 0.02, 1000, dtype=np.float32)
    acp = np.concatenate([[1.0], np.cumprod(1 - betas)]).astype(np.float32)
    c = bridge_coefficients(acp, ell=500, t=499, s=0, eta=1.0)
    a_l, a_t = np.float64(acp[500]), np.float64(acp[499])
    beta = 1 - a_l / a_t
    post_var = (1 - a_t) / (1 - a_l) * beta
    assert math.isclose(c.std, math.sqrt(post_var), rel_tol=1e-5)
    assert math.isclose(c.c_s, math.sqrt(a_t) * beta / (1 - a_l), rel_tol=1e-4)


def test_hip_path_refuses_host_tensors():
    from samplers_amd._hip import HipLibraryError
    from samplers_amd.samplers import DPSSampler
    import stand_ins as si

    net = si.make_samplers_amd_net("linear", 3)
    ip = InverseProblem(IdentityOperator((3, 8, 8)), torch.zeros(1, 3, 8, 8), GaussianNoise(0.1))
    with pytest.raises(HipLibraryError):
        DPSSampler(net)(ip, num_sampling_steps=4)
    assert not net.are_sampling_parameters_initialized  # state cleared on error


# --- the drop-in boundary for reference-style plugins (no GPU needed) ---------------------

def test_grad_scale_probe_for_reference_style_noise():
    import stand_ins as si

    from samplers_amd.noise import GaussianNoise, PoissonNoise, probe_grad_scale

    assert si.reference_style_gaussian(0.05).grad_scale() == GaussianNoise(0.05).grad_scale()
    assert probe_grad_scale(PoissonNoise(1.0)) == pytest.approx(PoissonNoise(1.0).grad_scale(),
                                                                rel=1e-6)
    assert si.laplace_noise(0.1).grad_scale() is None  # not c * r: generic path


@pytest.mark.parametrize("kind", ["huber", "clipped"])
def test_grad_scale_probe_rejects_densities_quadratic_only_near_zero(kind):
    """A Huber loss with delta = 10 or a Gaussian whose residual is clipped at 50 has score
    -c r for |r| up to ~10 (the old single-scale probe accepted them); the multi-scale
    probe sees the residuals at 1e2 x and sends them to the generic autograd path."""
    from samplers_amd.noise import NoiseModel, probe_grad_scale

    class Odd(NoiseModel):
        def __init__(self):
            super().__init__()
            self.register_buffer("sigma", torch.tensor(0.5))

        def log_prob(self, r):
            if kind == "huber":
                a = r.abs()
                v = torch.where(a < 10.0, 0.5 * r.square(), 10.0 * (a - 5.0))
            else:
                v = 0.5 * r.clamp(-50.0, 50.0).square()
            return -(v / self.sigma ** 2).sum(dim=tuple(range(1, r.ndim)))

        def sample(self, shape, **kw):
            return torch.zeros(shape)

    assert probe_grad_scale(Odd()) is None


def test_reference_style_noise_is_instantiable():
    """grad_scale is not abstract: a subclass of the reference ABC's shape instantiates."""
    import stand_ins as si

    noise = si.reference_style_gaussian(0.1)
    assert noise.log_prob(torch.ones(2, 3)).shape == (2,)


def test_timesteps_host_follows_a_directly_registered_buffer():
    import stand_ins as si

    net = si.make_reference_style_net("linear", 3)
    assert net.timesteps_host is None
    net.set_sampling_parameters(5)
    assert net.timesteps_host == [0, 200, 400, 600, 800]
    net.set_sampling_parameters(4)  # a new buffer: a new host copy
    assert net.timesteps_host == [0, 250, 500, 750]


def test_skip_grad_take_without_delivery_returns_none():
    from samplers_amd.networks.layers import SkipGrad

    box = SkipGrad()
    assert box.take() is None
    box.grad = torch.ones(2)
    assert torch.equal(box.take(), torch.ones(2)) and box.grad is None


def test_resnet_block_rejects_box_in_with_skip():
    from samplers_amd.networks.layers import SkipGrad
    from samplers_amd.networks.unet2d import ResnetBlock2D

    blk = ResnetBlock2D(64, 32, None, 32, 1e-6)
    with pytest.raises(ValueError, match="exclusive"):
        blk(torch.zeros(1, 32, 8, 8), skip=torch.zeros(1, 32, 8, 8), box_in=SkipGrad())


def test_torch_operator_stand_in_matches_native_inpainting_on_cpu():
    import stand_ins as si

    from samplers_amd.operators import InpaintingOperator

    shape = (3, 8, 8)
    mask = si.fixture_mask(shape, "random")
    native = InpaintingOperator(shape, mask)
    plain = si.torch_operator(shape, native._kept_indices)
    x = torch.randn(2, *shape)
    assert plain.y_shape == native.y_shape
    assert torch.equal(plain.apply(x), native.apply(x))
    assert torch.equal(plain.apply_transpose(plain.apply(x)), native.apply_transpose(native.apply(x)))


@pytest.mark.parametrize("name", sorted(p.stem for p in __import__("pathlib").Path(
    __file__).resolve().parent.joinpath("golden").glob("*.npz")))
def test_from_clean_data_reproduces_golden_observation(name):
    """A15: ``InverseProblem.from_clean_data`` (``inverse_problem.py:34-67``) with the golden
    generator's inputs (x_true seed 0, noise generator seed 7) gives the reference's y
    bit for bit (tests/golden/make_golden.py: build_problem)."""
    import stand_ins as si
    from golden_cases import load_dps_case

    case = load_dps_case(name)
    m = case.meta
    bs = m["batch_shape"]
    x_true = si.fixture_x_true(int(np.prod(bs)) if bs else 1, case.shape, 0)
    x_true = x_true.reshape(*bs, *case.shape)
    op = (IdentityOperator(case.shape) if case.kept is None
          else InpaintingOperator(case.shape, case.mask))
    noise = PoissonNoise(1.0) if m["noise"] == "poisson" else GaussianNoise(0.05)
    prob = InverseProblem.from_clean_data(x_true, operator=op, noise=noise,
                                          rng=torch.Generator().manual_seed(7))
    assert prob.observation.dtype == case.y.dtype
    assert torch.equal(prob.observation, case.y)


def test_fp32_view_of_networks():
    """fp32 networks pass through; bf16 / fp16 get the fp32 boundary (inputs cast in, outputs
    cast out, the rest delegated); non-float dtypes are refused at sampler entry."""
    from samplers_amd.networks.base import Fp32Boundary, fp32_view

    class Net:
        def __init__(self, dt):
            self.dtype, self.calls = dt, []

        def forward(self, x, t):
            self.calls.append(x.dtype)
            return x * 2

        def set_sampling_parameters(self, n):
            self.n = n

    f = Net(torch.float32)
    assert fp32_view(f) is f
    b = Net(torch.bfloat16)
    v = fp32_view(b)
    assert isinstance(v, Fp32Boundary) and v.dtype == torch.float32
    x = torch.ones(2, 3, requires_grad=True)
    out = v(x, 5)
    assert b.calls == [torch.bfloat16] and out.dtype == torch.float32
    (g,) = torch.autograd.grad(out.sum(), x)  # the VJP flows through both casts
    assert torch.equal(g, torch.full((2, 3), 2.0))
    v.set_sampling_parameters(7)
    assert b.n == 7
    with pytest.raises(TypeError, match="dtype"):
        fp32_view(Net(torch.int32))
    # float64: refused with a message saying why (fp32 samples in a float64 tensor would be a
    # silent precision loss against the reference's float64 loop)
    with pytest.raises(TypeError, match="float64"):
        fp32_view(Net(torch.float64))


def test_x6_size_rule(monkeypatch):
    """SAMPLERS_AMD_X6_MIN_TILES: the bf16x6 GEMMs serve a call only with at least that many
    256 x 128 output tiles; the default (0) keeps them everywhere their shape rules hold."""
    from samplers_amd.networks.layers import x6_enough_tiles

    monkeypatch.delenv("SAMPLERS_AMD_X6_MIN_TILES", raising=False)
    assert x6_enough_tiles(256, 128) and x6_enough_tiles(1 * 32 * 32, 512)
    monkeypatch.setenv("SAMPLERS_AMD_X6_MIN_TILES", "128")
    assert x6_enough_tiles(64 * 256 * 256, 128)         # headline 256² level: 16384 tiles
    assert x6_enough_tiles(64 * 16 * 16, 512)           # headline 16² level: 256 tiles
    assert not x6_enough_tiles(1 * 32 * 32, 512)        # batch 1, 32² level: 16 tiles
    assert x6_enough_tiles(1 * 256 * 256, 128)          # batch 1, 256² level: 256 tiles

"""The CPU oracle against the reference's golden vectors (no GPU needed)."""

import numpy as np
import pytest
import torch

import stand_ins as si
from golden_cases import dps_case_names, load_dps_case
from oracle import blur as oblur
from oracle import closed_form, dps_loop, inpaint, philox


def _oracle_dps(case, dtype=torch.float32):
    m = case.meta
    shape = case.shape
    core = si.EpsCore(m["prior"], shape[0], m["coef"]).to(dtype)
    acp = si.ddpm_alphas_cumprod()
    acp = torch.cat([acp.new_tensor([1.0]), acp]).clip(1e-6, 1).to(dtype)
    ts = si.leading_timesteps_ascending(m["N"]).tolist()
    if case.kept is None:
        apply_op = lambda x: x  # noqa: E731
    else:
        kept = torch.from_numpy(case.kept.astype(np.int64))
        apply_op = lambda x: x.reshape(*x.shape[:-3], -1)[..., kept]  # noqa: E731
    lp = dps_loop.gaussian_log_prob(0.05) if m["noise"] == "gauss" else dps_loop.poisson_log_prob(1.0)
    init, steps = case.noise()
    y = case.y.to(dtype)
    out = dps_loop.dps_reference(lambda x, t: core(x, t), acp, ts, apply_op, lp, y, init.to(dtype),
                                 lambda i: steps[i].to(dtype), gamma=m["gamma"], eta=m["eta"],
                                 leading_size=case.lead)
    return out.reshape(case.out.shape)


@pytest.mark.parametrize("name", dps_case_names())
def test_oracle_dps_matches_reference(name):
    case = load_dps_case(name)
    out = _oracle_dps(case)
    err = si.relative_error(out, case.out)
    assert err < 2e-6, err


@pytest.mark.parametrize("name", dps_case_names())
def test_golden_conditioning(name):
    """fp64 oracle vs the fp32 reference: how much fp32 rounding moves the result.

    The GPU parity tolerance is derived from this (tests/test_dps_gpu.py)."""
    case = load_dps_case(name)
    out64 = _oracle_dps(case, torch.float64)
    err = si.relative_error(out64, case.out)
    assert err < 1e-3, err


def test_philox_known_answers():
    for ctr, key, expected in philox.KAT:
        got = philox.philox4x32_10(np.array(ctr, dtype=np.uint32), key)
        assert [int(v) for v in got] == list(expected)


def test_philox_normals_moments():
    z = philox.normals(seed=99, step=3, sample=5, n=400_000)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    # different step / sample / seed -> different streams
    assert not np.allclose(z[:64], philox.normals(99, 4, 5, 64))
    assert not np.allclose(z[:64], philox.normals(99, 3, 6, 64))
    assert not np.allclose(z[:64], philox.normals(98, 3, 5, 64))


@pytest.mark.parametrize("name", [n for n in dps_case_names() if "rnd" in n or "ctr" in n])
def test_kept_indices_bit_exact(name):
    from samplers_amd.operators.inpainting import keep_bitmask

    case = load_dps_case(name)
    mask = case.mask.numpy()
    kept = inpaint.kept_indices(mask)
    assert np.array_equal(kept, case.kept.astype(np.int64))
    bits, rank = keep_bitmask(~mask.reshape(-1))
    assert np.array_equal(inpaint.rank_of(bits, rank, kept), np.arange(kept.size))


def test_blur_adjoint_identity():
    k = oblur.taps(9, 3.0)
    x = torch.randn(2, 3, 20, 23, dtype=torch.float64)
    y = torch.randn(2, 3, 20, 23, dtype=torch.float64)
    lhs = (oblur.blur(x, k) * y).sum()
    rhs = (x * oblur.blur_adjoint(y, k)).sum()
    assert abs(lhs - rhs) < 1e-10 * abs(lhs)


def test_closed_form_matches_autograd_loop():
    """One step of the closed form equals one step of the autograd restatement."""
    torch.manual_seed(0)
    b, shape = 3, (2, 6, 5)
    n = 60
    core = si.EpsCore("conv", 2, 0.1).double()
    acp = torch.cat([torch.ones(1), si.ddpm_alphas_cumprod()]).double()
    x = torch.randn(b, *shape, dtype=torch.float64)
    y = torch.randn(b, *shape, dtype=torch.float64)
    xi = torch.randn(b, *shape, dtype=torch.float64)
    ts = [0, 400, 800]
    lp = dps_loop.gaussian_log_prob(0.05)
    # loop with 1 guided iteration then final predict; recover x after the step
    after = {}

    def eps_fn(s, t):
        if t == ts[1] and not s.requires_grad:
            after["x"] = s.detach().clone()
        return core(s, t)

    dps_loop.dps_reference(eps_fn, acp, ts, lambda v: v, lp, y, x, lambda i: xi, gamma=0.3, eta=1.0)
    # closed form
    t, tp = 800, 400
    a, k = float(acp[t].sqrt()), float((1 - acp[t]).sqrt())
    gs = 1 / 0.05**2
    v, rsq = closed_form.residual_pass(x.reshape(b, n).numpy(),
                                       core(x, t).detach().reshape(b, n).numpy(),
                                       y.reshape(b, n).numpy(), 1, a, k, gs, *closed_form.identity_ops())
    xr = x.clone().requires_grad_()
    e = core(xr, t)
    (w,) = torch.autograd.grad(e, xr, grad_outputs=torch.from_numpy(v).reshape_as(e))
    from samplers_amd.samplers.utils.bridge_kernels import bridge_coefficients

    br = bridge_coefficients(acp.float().numpy(), t, tp, 0, 1.0)
    out = closed_form.update_pass(x.reshape(b, n).numpy(), core(x, t).detach().reshape(b, n).numpy(),
                                  v, w.reshape(b, n).numpy(), rsq, xi.reshape(b, n).numpy(), a, k,
                                  br.c_ell, br.c_s, br.std, 0.3)
    ref = after["x"].reshape(b, n).numpy()
    assert np.abs(out - ref).max() / np.abs(ref).max() < 1e-6


@pytest.mark.parametrize("name", dps_case_names("dps_*_bounded"))
def test_oracle_bounded_golden_elementwise(name):
    """The oracle on the bounded-magnitude cases, element by element."""
    case = load_dps_case(name)
    ref = case.out.numpy()
    np.testing.assert_allclose(_oracle_dps(case).numpy(), ref, rtol=1e-5,
                               atol=1e-6 * np.abs(ref).max())

"""PGDM / PSLD CPU restatements against the reference's golden vectors (no GPU)."""

import numpy as np
import pytest
import torch

import stand_ins as si
from golden_cases import dps_case_names, load_dps_case
from oracle.latent_loops import pgdm_reference, psld_reference


def _acp(dtype):
    acp = si.ddpm_alphas_cumprod()
    return torch.cat([acp.new_tensor([1.0]), acp]).clip(1e-6, 1).to(dtype)


def _ops(case, dtype):
    shape = case.shape
    if case.kept is None:
        return (lambda x: x), (lambda y: y.reshape(y.shape[0], *shape))
    kept = torch.from_numpy(case.kept.astype(np.int64))
    n = int(np.prod(shape))

    def apply(x):
        return x.reshape(x.shape[0], -1)[:, kept]

    def adjoint(y):
        out = torch.zeros(y.shape[0], n, dtype=y.dtype)
        out[:, kept] = y
        return out.reshape(y.shape[0], *shape)

    return apply, adjoint


def oracle_pgdm(case, dtype=torch.float32):
    m = case.meta
    core = si.EpsCore(m["prior"], case.shape[0], m["coef"]).to(dtype)
    apply, adjoint = _ops(case, dtype)
    init, steps = case.noise()
    rows = case.observation_rows().to(dtype).reshape(case.lead, *case.shape) \
        if case.kept is None else case.observation_rows().to(dtype)
    out = pgdm_reference(lambda x, t: core(x, t), _acp(dtype),
                         si.leading_timesteps_ascending(m["N"]).tolist(), apply, adjoint, rows,
                         init.to(dtype), lambda i: steps[i].to(dtype),
                         guidance_weight=m["guidance_weight"], eta=m["eta"])
    return out.reshape(case.out.shape)


def oracle_psld(case, dtype=torch.float32):
    m = case.meta
    core = si.EpsCore(m["prior"], 4, m["coef"]).to(dtype)
    vae = si.LatentCore().to(dtype)
    apply, adjoint = _ops(case, dtype)
    init, steps = case.noise()
    rows = case.observation_rows().to(dtype)
    if case.kept is None:
        rows = rows.reshape(case.lead, *case.shape)
    out = psld_reference(lambda x, t: core(x, t), _acp(dtype),
                         si.leading_timesteps_ascending(m["N"]).tolist(), apply, adjoint,
                         vae.decode, vae.encode, rows, init.to(dtype),
                         lambda i: steps[i].to(dtype), gamma=m["gamma"], omega=m["omega"],
                         eta=m["eta"])
    return out.reshape(case.out.shape)


@pytest.mark.parametrize("name", dps_case_names("pgdm"))
def test_oracle_pgdm_matches_reference(name):
    case = load_dps_case(name)
    assert si.relative_error(oracle_pgdm(case), case.out) < 2e-6
    assert si.relative_error(oracle_pgdm(case, torch.float64), case.out) < 1e-3


@pytest.mark.parametrize("name", dps_case_names("psld"))
def test_oracle_psld_matches_reference(name):
    case = load_dps_case(name)
    assert si.relative_error(oracle_psld(case), case.out) < 2e-6
    assert si.relative_error(oracle_psld(case, torch.float64), case.out) < 1e-3


def sequential_draws(seed: int):
    gen = torch.Generator().manual_seed(seed)
    return lambda shape: torch.randn(shape, generator=gen)


def oracle_resample(case, dtype=torch.float32):
    from oracle.resample_loop import resample_reference

    m = case.meta
    core = si.EpsCore("conv", 4, 0.1).to(dtype)
    vae = si.LatentCore().to(dtype)
    apply, _ = _ops(case, dtype)
    rows = case.observation_rows().to(dtype)
    if case.kept is None:
        rows = rows.reshape(case.lead, *case.shape)
    eps = 1e-3  # Poisson -> 1e-3; the Gaussian case uses sigma = 1e-3
    out = resample_reference(lambda x, t: core(x, t), _acp(dtype),
                             si.leading_timesteps_ascending(m["N"]).tolist(), apply, vae.decode,
                             vae.encode, rows, sequential_draws(m["seed"]),
                             latent_shape=tuple(m["latent_shape"]), leading=case.lead, eps=eps,
                             max_iters=m["max_iters"], eta=m["eta"],
                             inter_timesteps=m["inter_timesteps"],
                             time_travel_interval=m["time_travel_interval"],
                             stage_splits=m["stage_splits"])
    return out.reshape(case.out.shape)


@pytest.mark.parametrize("name", dps_case_names("rs"))
def test_oracle_resample_matches_reference(name):
    case = load_dps_case(name)
    assert si.relative_error(oracle_resample(case), case.out) < 2e-6

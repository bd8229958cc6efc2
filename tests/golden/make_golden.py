"""Generate golden vectors by running the REFERENCE samplers (survey container only).

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

Imports thomashirtz/samplers read-only from /root/reference, the way its own
tests do (``tests/samplers/test_resample.py:16-60``: the ``samplers.networks``
and ``samplers.samplers`` packages are stubbed in ``sys.modules`` because
diffusers is absent), drives ``DPSSampler`` / ``PGDMSampler`` / ``PSLDSampler``
with the deterministic stand-in priors of ``tests/stand_ins.py`` under
``torch.manual_seed`` and stores inputs and outputs.  The noise stream is not
stored: it is the reference's own draw order (``randn`` then one ``randn_like``
per step) from the seed, which ``stand_ins.replay_noise`` regenerates; this
script asserts that the replay reproduces the captured stream.

Nothing under /root/reference is copied; the .npz files hold only data.
"""

from __future__ import annotations

import importlib.util
import json
import sys
import types
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
sys.dont_write_bytecode = True
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(REF))

import stand_ins as si  # noqa: E402


def _load(rel: str, name: str):
    spec = importlib.util.spec_from_file_location(name, REF / rel)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_reference():
    from samplers.inverse_problem import InverseProblem  # noqa: F401  (plain import works)

    base = _load("samplers/networks/base.py", "samplers.networks.base")
    pkg = types.ModuleType("samplers.networks")
    pkg.__path__ = [str(REF / "samplers" / "networks")]
    pkg.EpsilonNetwork, pkg.LatentEpsilonNetwork, pkg.base = (base.EpsilonNetwork,
                                                              base.LatentEpsilonNetwork, base)
    sys.modules["samplers.networks"] = pkg
    sbase = _load("samplers/samplers/base.py", "samplers.samplers.base")
    spkg = types.ModuleType("samplers.samplers")
    spkg.__path__ = [str(REF / "samplers" / "samplers")]
    spkg.PosteriorSampler, spkg.base = sbase.PosteriorSampler, sbase
    sys.modules["samplers.samplers"] = spkg
    upkg = types.ModuleType("samplers.samplers.utils")
    upkg.__path__ = [str(REF / "samplers" / "samplers" / "utils")]
    sys.modules["samplers.samplers.utils"] = upkg
    for mod in ("batch_view", "bridge_kernels", "resample_kernels"):
        m = _load(f"samplers/samplers/utils/{mod}.py", f"samplers.samplers.utils.{mod}")
        setattr(upkg, mod, m)
    ref = types.SimpleNamespace(base=base)
    for mod in ("dps", "pgdm", "psld", "resample"):
        setattr(ref, mod, _load(f"samplers/samplers/{mod}.py", f"samplers.samplers.{mod}"))
    import samplers.inverse_problem as ip
    import samplers.noise as noise
    import samplers.operators as ops

    ref.ip, ref.noise, ref.ops = ip, noise, ops
    return ref


def ref_network(ref, kind: str, channels: int, coef: float):
    class RefStandIn(ref.base.EpsilonNetwork):
        def __init__(self):
            acp = si.ddpm_alphas_cumprod()
            super().__init__(alphas_cumprod=torch.cat([acp.new_tensor([1.0]), acp]))
            self.core = si.EpsCore(kind, channels, coef)

        def forward(self, x, t):
            return self.core(x, t)

        @classmethod
        def from_pretrained(cls, *a, **k):
            raise NotImplementedError

        def set_sampling_parameters(self, num_sampling_steps, batch_size=1, num_reconstructions=1):
            self._batch_size = batch_size
            self._num_sampling_steps = num_sampling_steps
            self.register_buffer("timesteps", si.leading_timesteps_ascending(num_sampling_steps))

        def is_condition_initialized(self):
            return True

    return RefStandIn()


def ref_latent_network(ref, kind: str, coef: float):
    class RefLatent(ref.base.LatentEpsilonNetwork):
        def __init__(self):
            acp = si.ddpm_alphas_cumprod()
            super().__init__(alphas_cumprod=torch.cat([acp.new_tensor([1.0]), acp]))
            self.core = si.EpsCore(kind, 4, coef)
            self.vae = si.LatentCore()

        def forward(self, x, t):
            return self.core(x, t)

        @classmethod
        def from_pretrained(cls, *a, **k):
            raise NotImplementedError

        def set_sampling_parameters(self, num_sampling_steps, batch_size=1, num_reconstructions=1):
            self._batch_size = batch_size
            self._num_sampling_steps = num_sampling_steps
            self.register_buffer("timesteps", si.leading_timesteps_ascending(num_sampling_steps))

        def get_latent_shape(self, x_shape):
            return self.vae.latent_shape(x_shape)

        def _decode(self, z, *, differentiable=False):
            return self.vae.decode(z)

        def _encode(self, x, *, differentiable=False):
            return self.vae.encode(x)

        def is_condition_initialized(self):
            return True

    return RefLatent()


class Capture:
    """Records every torch.randn / torch.randn_like the reference draws."""

    def __init__(self):
        self.draws = []

    def __enter__(self):
        self._randn, self._randn_like = torch.randn, torch.randn_like

        def randn(*a, **k):
            out = self._randn(*a, **k)
            self.draws.append(out.detach().clone())
            return out

        def randn_like(*a, **k):
            out = self._randn_like(*a, **k)
            self.draws.append(out.detach().clone())
            return out

        torch.randn, torch.randn_like = randn, randn_like
        return self

    def __exit__(self, *exc):
        torch.randn, torch.randn_like = self._randn, self._randn_like
        return False


DPS_CASES = [
    # name, op, noise, prior, coef, batch_shape, R, shape, N, gamma, eta
    ("dps_id_gauss_lin_b1", "identity", "gauss", "linear", 0.1, (1,), 1, (3, 32, 32), 25, 1e-2, 1.0),
    ("dps_id_gauss_conv_b4", "identity", "gauss", "conv", 0.1, (4,), 1, (3, 32, 32), 25, 1e-2, 1.0),
    ("dps_rnd_gauss_lin_b4", "random", "gauss", "linear", 0.3, (4,), 1, (3, 32, 32), 25, 1e-2, 0.0),
    ("dps_rnd_poiss_conv_b4", "random", "poisson", "conv", 0.1, (4,), 1, (3, 32, 32), 25, 1e-3, 1.0),
    ("dps_ctr_gauss_conv_b2_64", "center", "gauss", "conv", 0.1, (2,), 1, (3, 64, 64), 6, 1e-2, 1.0),
    ("dps_id_poiss_lin_b1_64", "identity", "poisson", "linear", 0.3, (1,), 1, (3, 64, 64), 6, 1e-3, 0.0),
    ("dps_rnd_gauss_conv_r3", "random", "gauss", "conv", 0.1, (), 3, (3, 32, 32), 10, 1e-2, 1.0),
    ("dps_rnd_gauss_conv_b3_odd", "random", "gauss", "conv", 0.1, (3,), 1, (1, 5, 7), 10, 1e-2, 1.0),
    # bounded-magnitude trajectories (|out| of order 1-10, the linear stand-in near the
    # data's own scale): small-valued pixels are pinned too, not only the diverging ones
    ("dps_rnd_gauss_lin_bounded", "random", "gauss", "linear", 0.9, (4,), 1, (3, 32, 32), 50, 1e-3, 1.0),
    ("dps_ctr_gauss_lin_bounded", "center", "gauss", "linear", 0.5, (2,), 1, (3, 32, 32), 50, 1e-2, 0.0),
    ("dps_id_poiss_lin_bounded", "identity", "poisson", "linear", 0.9, (2,), 1, (3, 16, 16), 30, 1e-3, 1.0),
    ("dps_rnd_gauss_conv_bounded", "random", "gauss", "conv", 0.9, (2,), 1, (3, 16, 16), 50, 1e-3, 1.0),
]


def build_problem(ref, op_kind, noise_kind, batch_shape, shape, seed_data=0):
    x_true = si.fixture_x_true(int(np.prod(batch_shape)) if batch_shape else 1, shape, seed_data)
    x_true = x_true.reshape(*batch_shape, *shape)
    mask = None
    if op_kind == "identity":
        op = ref.ops.IdentityOperator(x_shape=shape)
    else:
        mask = si.fixture_mask(shape, op_kind)
        op = ref.ops.InpaintingOperator(shape, mask)
    noise = ref.noise.GaussianNoise(sigma=0.05) if noise_kind == "gauss" else ref.noise.PoissonNoise(rate=1.0)
    gen = torch.Generator().manual_seed(7)
    prob = ref.ip.InverseProblem.from_clean_data(x_true, operator=op, noise=noise, rng=gen)
    return prob, mask


def make_dps(ref, case):
    name, op_kind, noise_kind, prior, coef, batch_shape, R, shape, N, gamma, eta = case
    prob, mask = build_problem(ref, op_kind, noise_kind, batch_shape, shape)
    net = ref_network(ref, prior, shape[0], coef)
    sampler = ref.dps.DPSSampler(net)
    seed = 1000 + len(name)
    torch.manual_seed(seed)
    with Capture() as cap:
        out = sampler(inverse_problem=prob, num_sampling_steps=N, num_reconstructions=R, gamma=gamma,
                      eta=eta)
    lead = (int(np.prod(batch_shape)) if batch_shape else 1) * R
    init, steps = si.replay_noise(seed, (lead, *shape), N)
    replay = [init] + [steps[i] for i in range(N - 1, 1, -1)]
    assert len(replay) == len(cap.draws), (len(replay), len(cap.draws))
    for a, b in zip(replay, cap.draws):
        assert torch.equal(a, b), "noise replay diverged from the reference draw order"
    meta = dict(kind="dps", op=op_kind, noise=noise_kind, prior=prior, coef=coef,
                batch_shape=list(batch_shape), R=R, shape=list(shape), N=N, gamma=gamma, eta=eta,
                seed=seed, out_shape=list(out.shape))
    arrays = dict(y=prob.observation.numpy(), out=out.detach().numpy())
    if mask is not None:
        arrays["mask"] = mask.numpy()
        arrays["kept"] = prob.operator._kept_indices.numpy().astype(np.int32)
    return name, meta, arrays


PGDM_CASES = [
    # name, op, prior, coef, batch_shape, R, shape, N, guidance_weight, eta
    # (the reference PGDM tiles y with the data rank, pgdm.py:102 / batch_view.py:128-137, so
    #  only non-flattened observations run there: inpainting PGDM is pinned by the oracle)
    ("pgdm_id_conv_b2", "identity", "conv", 0.1, (2,), 1, (3, 32, 32), 12, 0.05, 1.0),
    ("pgdm_id_lin_r2", "identity", "linear", 0.3, (), 2, (3, 32, 32), 12, 0.1, 0.0),
    ("pgdm_id_conv_b1_64", "identity", "conv", 0.1, (1,), 1, (3, 64, 64), 6, 0.05, 1.0),
]

PSLD_CASES = [
    # name, op, prior, coef, batch_shape, R, shape, N, gamma, omega, eta
    ("psld_id_conv_b2", "identity", "conv", 0.1, (2,), 1, (3, 32, 32), 10, 1.0, 0.1, 1.0),
    # flattened y only runs unbatched with R = 1 in the reference
    ("psld_rnd_conv_r1", "random", "conv", 0.1, (), 1, (3, 32, 32), 10, 1.0, 0.1, 1.0),
    ("psld_ctr_lin_b1", "center", "linear", 0.3, (), 1, (3, 32, 32), 8, 0.5, 0.2, 0.0),
]


def make_pgdm(ref, case):
    name, op_kind, prior, coef, batch_shape, R, shape, N, gw, eta = case
    prob, mask = build_problem(ref, op_kind, "gauss", batch_shape, shape)
    net = ref_network(ref, prior, shape[0], coef)
    seed = 2000 + len(name)
    torch.manual_seed(seed)
    with Capture() as cap:
        out = ref.pgdm.PGDMSampler(net)(inverse_problem=prob, num_sampling_steps=N,
                                        num_reconstructions=R, guidance_weight=gw, eta=eta)
    lead = (int(np.prod(batch_shape)) if batch_shape else 1) * R
    _check_replay(cap, seed, (lead, *shape), N)
    meta = dict(kind="pgdm", op=op_kind, noise="gauss", prior=prior, coef=coef,
                batch_shape=list(batch_shape), R=R, shape=list(shape), N=N, guidance_weight=gw,
                eta=eta, seed=seed, out_shape=list(out.shape))
    arrays = dict(y=prob.observation.numpy(), out=out.detach().numpy())
    if mask is not None:
        arrays["mask"] = mask.numpy()
        arrays["kept"] = prob.operator._kept_indices.numpy().astype(np.int32)
    return name, meta, arrays


def make_psld(ref, case):
    name, op_kind, prior, coef, batch_shape, R, shape, N, gamma, omega, eta = case
    prob, mask = build_problem(ref, op_kind, "gauss", batch_shape, shape)
    net = ref_latent_network(ref, prior, coef)
    seed = 3000 + len(name)
    torch.manual_seed(seed)
    with Capture() as cap:
        out = ref.psld.PSLDSampler(net)(inverse_problem=prob, num_sampling_steps=N,
                                        num_reconstructions=R, gamma=gamma, omega=omega, eta=eta)
    lead = (int(np.prod(batch_shape)) if batch_shape else 1) * R
    _check_replay(cap, seed, (lead, *net.get_latent_shape(shape)), N)
    meta = dict(kind="psld", op=op_kind, noise="gauss", prior=prior, coef=coef,
                batch_shape=list(batch_shape), R=R, shape=list(shape),
                latent_shape=list(net.get_latent_shape(shape)), N=N, gamma=gamma, omega=omega,
                eta=eta, seed=seed, out_shape=list(out.shape))
    arrays = dict(y=prob.observation.numpy(), out=out.detach().numpy())
    if mask is not None:
        arrays["mask"] = mask.numpy()
        arrays["kept"] = prob.operator._kept_indices.numpy().astype(np.int32)
    return name, meta, arrays


RESAMPLE_CASES = [
    # name, op, noise, batch_shape, R, shape, N, max_iters, inter, interval, splits, eta
    ("rs_id_poiss_b2", "identity", "poisson", (2,), 1, (3, 32, 32), 10, 4, 2, 2, 3, 1.0),
    ("rs_rnd_gauss_r1", "random", "gauss_small", (), 1, (3, 32, 32), 10, 3, 2, 2, 3, 0.5),
    ("rs_id_poiss_plateau", "identity", "poisson", (1,), 1, (3, 32, 32), 6, 205, 1, 2, 3, 1.0),
]


def make_resample(ref, case):
    name, op_kind, noise_kind, batch_shape, R, shape, N, iters, inter, interval, splits, eta = case
    nk = "gauss" if noise_kind.startswith("gauss") else "poisson"
    prob, mask = build_problem(ref, op_kind, nk, batch_shape, shape)
    if noise_kind == "gauss_small":  # eps = sigma = 1e-3: no early stop in a few iterations
        prob = ref.ip.InverseProblem(prob.operator, prob.observation,
                                     ref.noise.GaussianNoise(sigma=1e-3))
    net = ref_latent_network(ref, "conv", 0.1)
    seed = 4000 + len(name)
    torch.manual_seed(seed)
    with Capture() as cap:
        out = ref.resample.ReSampleSampler(net)(
            prob, num_sampling_steps=N, num_reconstructions=R, max_optimization_iters=iters,
            eta=eta, inter_timesteps=inter, time_travel_interval=interval, stage_splits=splits)
    shapes = [list(d.shape) for d in cap.draws]
    gen = torch.Generator().manual_seed(seed)
    for d in cap.draws:  # the stream is the seed's sequential randn draws
        assert torch.equal(torch.randn(d.shape, generator=gen), d)
    meta = dict(kind="resample", op=op_kind, noise=noise_kind, batch_shape=list(batch_shape), R=R,
                shape=list(shape), latent_shape=list(net.get_latent_shape(shape)), N=N,
                max_iters=iters, inter_timesteps=inter, time_travel_interval=interval,
                stage_splits=splits, eta=eta, seed=seed, draw_shapes=shapes,
                out_shape=list(out.shape), prior="conv", coef=0.1)
    arrays = dict(y=prob.observation.numpy(), out=out.detach().numpy())
    if mask is not None:
        arrays["mask"] = mask.numpy()
        arrays["kept"] = prob.operator._kept_indices.numpy().astype(np.int32)
    return name, meta, arrays


def _check_replay(cap, seed, flat_shape, N):
    init, steps = si.replay_noise(seed, flat_shape, N)
    replay = [init] + [steps[i] for i in range(N - 1, 1, -1)]
    assert len(replay) == len(cap.draws), (len(replay), len(cap.draws))
    for a, b in zip(replay, cap.draws):
        assert torch.equal(a, b), "noise replay diverged from the reference draw order"


def main():
    ref = load_reference()
    index = {}
    for maker, cases in ((make_pgdm, PGDM_CASES), (make_psld, PSLD_CASES),
                         (make_resample, RESAMPLE_CASES)):
        for case in cases:
            name, meta, arrays = maker(ref, case)
            np.savez_compressed(HERE / f"{name}.npz", meta=json.dumps(meta), **arrays)
            index[name] = meta
            print(name, meta["out_shape"], float(np.abs(arrays["out"]).max()))
    for case in DPS_CASES:
        name, meta, arrays = make_dps(ref, case)
        np.savez_compressed(HERE / f"{name}.npz", meta=json.dumps(meta), **arrays)
        index[name] = meta
        print(name, meta["out_shape"], float(np.abs(arrays["out"]).max()))
    (HERE / "index.json").write_text(json.dumps(index, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()

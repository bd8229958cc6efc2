"""BASELINE configs[3] / [4] on their real priors: the SD 1.5 VAE (decode / encode forward +
input VJP at 512²), the SD 1.5 ε-UNet (UNet2DConditionModel structure, 64x64 latents), the
ddpm-celebahq-256 UNet at full size, and one PSLD iteration / a short ReSample run at 3x512²
through all of them — the device path (HIP GroupNorm, Winograd / direct / thin / stride-2
MFMA convolutions, upsampling, fused guidance kernels) against the same modules with the
same weights in plain torch fp32 on the CPU (``oracle/latent_loops.py`` /
``oracle/resample_loop.py`` restating ``psld.py:118-153`` and ``resample.py`` +
``resample_kernels.py``).

Tolerance: relative L2 <= 1e-4 (fp32 on both sides; the two differ in convolution algorithm
— Winograd F(2x2,3x3) vs oneDNN direct — and in summation orders, ~1e-6 per layer, compounded
over ~60 layers).  Parity to diffusers itself is unpinned (diffusers and the weights are
absent).
"""

from __future__ import annotations

import copy

import numpy as np
import pytest
import torch

import stand_ins as si

pytestmark = pytest.mark.gpu

TOL = 1e-4


def _kernel_names(fn) -> set[str]:
    """Names of the device kernels ``fn`` launches (torch profiler)."""
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    return {e.name for e in prof.events() if e.device_type.name == "CUDA"}


def _fwd_vjp(module_fn, x: torch.Tensor, cot: torch.Tensor):
    xr = x.detach().clone().requires_grad_(True)
    with torch.enable_grad():
        out = module_fn(xr)
    (g,) = torch.autograd.grad(out, xr, grad_outputs=cot.to(out.device))
    return out.detach().cpu(), g.detach().cpu()


def _check(name, gpu, cpu, record=None):
    for tag, a, b in zip(("out", "vjp"), gpu, cpu):
        err = si.relative_error(a, b)
        if record is not None:
            record(f"{tag}_rel_l2", err, TOL, module=name)
        assert err < TOL, f"{name} {tag}: rel L2 {err:.3e}"


@pytest.fixture(scope="module")
def vae_pair():
    from samplers_amd.networks.vae import build_vae

    cpu = build_vae(seed=1)
    return cpu, copy.deepcopy(cpu).to("cuda:0")


def test_vae_decode_512_fwd_vjp_matches_cpu(cuda, vae_pair, parity_record):
    cpu, gpu = vae_pair
    gen = torch.Generator().manual_seed(0)
    z = torch.randn(1, 4, 64, 64, generator=gen)
    cot = torch.randn(1, 3, 512, 512, generator=gen)
    got = _fwd_vjp(gpu.decode, z.to(cuda), cot)
    names = _kernel_names(lambda: gpu.decode(z.to(cuda)))
    assert any("wino3x3" in n for n in names), "decoder 3x3 convs not on the Winograd tile"
    assert any("gn_fwd" in n for n in names), "decoder GroupNorm not on the HIP kernel"
    # the Upsample2D blocks: the upsample inside the Winograd tile's loads (round 5), or the
    # streaming upsample kernel where the fused tile does not serve the shape
    assert any("k_wino3x3_xi<false, 16, 1>" in n or "upsample2x" in n for n in names)
    assert any("conv3x3_thin" in n for n in names)  # conv_out 128 -> 3
    _check("decode", got, _fwd_vjp(cpu.decode, z, cot), parity_record)


def test_vae_encode_512_fwd_vjp_matches_cpu(cuda, vae_pair, parity_record):
    cpu, gpu = vae_pair
    gen = torch.Generator().manual_seed(1)
    x = torch.rand(1, 3, 512, 512, generator=gen) * 2 - 1
    cot = torch.randn(1, 4, 64, 64, generator=gen)
    got = _fwd_vjp(gpu.encode_mean, x.to(cuda), cot)
    names = _kernel_names(lambda: gpu.encode_mean(x.to(cuda)))
    assert any("conv3x3_s2" in n for n in names), "encoder downsampling not on the stride-2 tile"
    assert any("wino3x3" in n for n in names)
    _check("encode", got, _fwd_vjp(cpu.encode_mean, x, cot), parity_record)


def test_vae_decode_128_batch_matches_cpu(cuda, vae_pair, parity_record):
    cpu, gpu = vae_pair
    gen = torch.Generator().manual_seed(2)
    z = torch.randn(3, 4, 16, 16, generator=gen)
    cot = torch.randn(3, 3, 128, 128, generator=gen)
    _check("decode128", _fwd_vjp(gpu.decode, z.to(cuda), cot), _fwd_vjp(cpu.decode, z, cot), parity_record)


def test_sd15_unet_fwd_vjp_matches_cpu(cuda, parity_record):
    """The 859.5 M-parameter SD 1.5 ε-UNet at 4x64x64, cross-attending to a 77x768
    context (``stable_diffusion.py:306-313``): forward + input VJP."""
    from samplers_amd.networks.unet2d_condition import build_unet_condition, null_context

    cpu = build_unet_condition(seed=0)
    gpu = copy.deepcopy(cpu).to(cuda)
    gen = torch.Generator().manual_seed(3)
    z = torch.randn(2, 4, 64, 64, generator=gen)
    ctx = torch.cat([null_context(), torch.randn(1, 77, 768, generator=gen)])
    cot = torch.randn(2, 4, 64, 64, generator=gen)
    got = _fwd_vjp(lambda v: gpu(v, 601, ctx.to(cuda)), z.to(cuda), cot)
    names = _kernel_names(lambda: gpu(z.to(cuda), 601, ctx.to(cuda)))
    assert any("wino3x3" in n for n in names) and any("gn_fwd" in n for n in names)
    _check("sd15-unet", got, _fwd_vjp(lambda v: cpu(v, 601, ctx), z, cot), parity_record)
    del gpu
    torch.cuda.empty_cache()


def test_celebahq_unet_full_size_fwd_vjp_matches_cpu(cuda, parity_record):
    """The headline prior (ddpm-celebahq-256, 6 levels, 113.7 M) at 3x256², B=2."""
    from samplers_amd.networks.unet2d import build_unet

    cpu = build_unet(seed=0)
    gpu = copy.deepcopy(cpu).to(cuda)
    gen = torch.Generator().manual_seed(4)
    x = torch.randn(2, 3, 256, 256, generator=gen)
    cot = torch.randn(2, 3, 256, 256, generator=gen)
    got = _fwd_vjp(lambda v: gpu(v, 999), x.to(cuda), cot)
    names = _kernel_names(lambda: gpu(x.to(cuda), 999))
    for k in ("wino3x3", "gn_fwd", "conv3x3_s2", "conv3x3_thin", "upsample2x"):
        assert any(k in n for n in names), k
    _check("celebahq-unet", got, _fwd_vjp(lambda v: cpu(v, 999), x, cot), parity_record)
    del gpu
    torch.cuda.empty_cache()


# ---- PSLD / ReSample through the SD 1.5 VAE and ε-UNet at 3x512² ----------------------------

def _latent_nets(batch: int):
    from samplers_amd.networks.latent import LatentDiffusionNetwork, StableDiffusionCondition

    cpu = LatentDiffusionNetwork.from_config(seed=0)
    gpu = copy.deepcopy(cpu).to("cuda:0")
    for net in (cpu, gpu):
        net.set_sampling_parameters(100, batch_size=batch)
        net.set_condition(StableDiffusionCondition(prompt=[""] * batch))
    return cpu, gpu


def _center_gather(shape):
    from samplers_amd.operators import CenterInpaintingOperator

    op = CenterInpaintingOperator(shape, 0.5)
    kept = op._kept_indices.cpu()
    n = int(np.prod(shape))

    def apply(x):
        return x.reshape(x.shape[0], -1)[:, kept]

    def adjoint(v):
        out = torch.zeros(v.shape[0], n, dtype=v.dtype)
        out[:, kept] = v
        return out.reshape(v.shape[0], *shape)

    return op, apply, adjoint


def test_psld_step_512_sd15_matches_oracle(cuda, parity_record):
    """One PSLD iteration (``psld.py:118-153``: ε-UNet fwd, decode fwd, pixel pass, encode fwd,
    encode / decode / UNet VJPs, bridge update) at B=2, centre inpainting (configs[3])."""
    from oracle.latent_loops import psld_reference
    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.noise import GaussianNoise
    from samplers_amd.samplers.psld import FusedPSLDStep

    b, shape = 2, (3, 512, 512)
    cpu, gpu = _latent_nets(b)
    op, apply, adjoint = _center_gather(shape)
    gen = torch.Generator().manual_seed(5)
    x_true = torch.rand(b, *shape, generator=gen) * 2 - 1
    y = apply(x_true) + 0.05 * torch.randn(b, op._kept_indices.numel(), generator=gen)
    z0 = torch.randn(b, 4, 64, 64, generator=gen)
    xi = torch.randn(b, 4, 64, 64, generator=gen)
    ts = cpu.timesteps_host
    i = len(ts) - 1

    problem = InverseProblem(op.to(cuda), y.to(cuda), GaussianNoise(0.05).to(cuda))
    step = FusedPSLDStep(gpu, problem, y.to(cuda), 1, (4, 64, 64))
    z = z0.to(cuda).contiguous()
    step(z, i, ts[i], ts[i - 1], ts[0], xi=xi.to(cuda))

    ref = psld_reference(lambda v, t: cpu(v, t), cpu.alphas_cumprod, ts, apply, adjoint,
                         lambda v: cpu.decode(v, differentiable=True),
                         lambda v: cpu.encode(v, differentiable=True), y, z0,
                         lambda k: xi, steps_limit=1)
    err = si.relative_error(z.cpu(), ref)
    parity_record("latent_rel_l2", err, TOL, sampler="PSLD", guided_steps=1, batch=b, image=list(shape))
    assert err < TOL, err


def test_resample_512_sd15_matches_oracle(cuda, parity_record):
    """A short ReSample run (``resample.py:99-224``) at 3x512², B=1, Poisson: ε-DDIM steps, the
    DPS conditioning through the decoder VJP, a time-travel block with pixel-space hard
    consistency + encode + stochastic resampling, and the final latent-space optimisation
    (decoder fwd + VJP per AdamW iteration), against the oracle loop on the CPU."""
    from oracle.resample_loop import resample_reference
    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.noise import PoissonNoise
    from samplers_amd.operators import IdentityOperator
    from samplers_amd.samplers.resample import ReSampleSampler

    b, shape = 1, (3, 512, 512)
    cpu, gpu = _latent_nets(b)
    gen = torch.Generator().manual_seed(6)
    x_true = torch.rand(b, *shape, generator=gen) * 2 - 1
    y = x_true + PoissonNoise(1.0).sample(tuple(x_true.shape), generator=gen)
    kw = dict(max_optimization_iters=3, eta=1.0, inter_timesteps=5, time_travel_interval=2,
              stage_splits=3)
    gen_gpu = torch.Generator().manual_seed(60)
    out = ReSampleSampler(gpu)(
        InverseProblem(IdentityOperator(shape), y.to(cuda), PoissonNoise(1.0).to(cuda)),
        num_sampling_steps=4, noise_fn=lambda kind, key, s: torch.randn(s, generator=gen_gpu),
        **kw)
    cpu.set_sampling_parameters(4, batch_size=b)
    gen_cpu = torch.Generator().manual_seed(60)
    ref = resample_reference(lambda v, t: cpu(v, t), cpu.alphas_cumprod, cpu.timesteps_host,
                             lambda v: v, lambda v: cpu.decode(v, differentiable=True),
                             lambda v: cpu.encode(v), y,
                             lambda s: torch.randn(s, generator=gen_cpu), latent_shape=(4, 64, 64),
                             leading=b, eps=1e-3, max_iters=kw["max_optimization_iters"],
                             eta=kw["eta"], inter_timesteps=kw["inter_timesteps"],
                             time_travel_interval=kw["time_travel_interval"],
                             stage_splits=kw["stage_splits"])
    err = si.relative_error(out.cpu(), ref.reshape(out.shape))
    parity_record("x0_rel_l2", err, TOL, sampler="ReSample", noise="poisson", batch=b,
                  image=list(shape), max_optimization_iters=kw["max_optimization_iters"])
    assert err < TOL, err

"""PSLD benchmark (BASELINE.json configs[3], "config 4"): latent-space inpainting at 512².

    python tools/bench_psld.py [--batch 32 --steps 3 --warmup 2]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        tools/bench_psld.py --gpus N            (batch per rank; RCCL all-reduce of the norms)

Workload: PSLD (psld.py:118-153) with a centre-inpainting mask on 3x512x512 images,
GaussianNoise(0.05), SD 1.5 VAE architecture (83.65 M parameters) + SD 1.5
UNet2DConditionModel (859.5 M, null 77x768 context), random weights with fixed seeds, fp32, 100-step schedule (psld.py:50).  One
step = one PSLD iteration over the batch: latent UNet forward, VAE decode forward,
HIP pixel pass, VAE encode forward, encode/decode/UNet VJPs, HIP glue and update
(samplers_amd.samplers.psld.FusedPSLDStep).  Prints one JSON line; "vae_tflops" (per GPU) is
the algorithmic VAE work (7.13 TFLOP per sample-step) over the step
time, an upper bound on what the VAE convolutions achieve.

With N ranks each holds ``--batch`` samples of a global batch of N x batch (sample
offset rank x batch for the Philox noise) and the step's two batch-global norms
(psld.py:130,138) are summed over ranks by one 8-byte all-reduce; value = N x batch x K /
the max-over-ranks wall time of the K timed steps (weak scaling, as bench.py).
"""

from __future__ import annotations

import argparse
import json
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import samplers_amd  # noqa: E402,F401

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from bench import (MFMA_BF16_PEAK_TFLOPS, MFMA_F32_PEAK_TFLOPS, conv_summary, host_cpu, self_launch,  # noqa: E402
                   setup_dist)

VAE_FLOP_PER_SAMPLE = 7.13e12
# SD 1.5 UNet at 64x64 latents: 0.80 TFLOP forward + 0.92 input VJP (torch FlopCounterMode)
UNET_FLOP_PER_SAMPLE = 1.73e12


def heartbeat(path: Path, every: float = 30.0) -> None:
    def beat():
        while True:
            time.sleep(every)
            with open(path, "a") as f:
                f.write(f"{time.time():.0f}\n")

    threading.Thread(target=beat, daemon=True).start()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--batch", type=int, default=32, help="samples per rank")
    p.add_argument("--image", type=int, default=512)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--heartbeat", default="gpurun_out/psld_heartbeat.log")
    p.add_argument("--cfg", action="store_true",
                   help="classifier-free guidance on: distinct (seeded random) prompt embeddings, "
                        "guidance 7.5, so the UNet batch doubles (stable_diffusion.py:300-320)")
    p.add_argument("--dtype", choices=("fp32", "bf16"), default="fp32",
                   help="the priors' dtype: bf16 = the reference's own PSLD run (scripts/run_psld.py:14-20, "
                        "torch_dtype=torch.bfloat16) on the bf16 NHWC kernels; the sample, guidance and "
                        "DDIM update stay fp32 (networks.base.Fp32Boundary)")
    p.add_argument("--cpu-baseline", action="store_true",
                   help="also time one PSLD iteration of oracle/latent_loops.py on the host cores "
                        "(batch 1, same networks)")
    args = p.parse_args()
    Path(args.heartbeat).parent.mkdir(parents=True, exist_ok=True)
    heartbeat(Path(args.heartbeat))
    torch.backends.cudnn.benchmark = False
    # `--gpus N` without a launcher starts its N ranks itself (before anything touches the GPU)
    status = self_launch(args.gpus, sys.argv[1:], script=__file__)
    if status is not None:
        sys.exit(status)
    rank, world, dev = setup_dist(args.gpus)
    group = dist.group.WORLD if world > 1 else None

    from samplers_amd import _hip
    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.networks.latent import LatentDiffusionNetwork, StableDiffusionCondition
    from samplers_amd.noise import GaussianNoise
    from samplers_amd.operators import CenterInpaintingOperator
    from samplers_amd.samplers.dps import initial_sample
    from samplers_amd.samplers.psld import FusedPSLDStep

    _hip.load_library()
    shape = (3, args.image, args.image)
    op = CenterInpaintingOperator(shape, 0.5).to(dev)
    gen = torch.Generator().manual_seed(1000 + rank)
    x_true = (torch.rand((args.batch, *shape), generator=gen) * 2 - 1).to(dev)
    y = op.apply(x_true)
    y = y + (0.05 * torch.randn(tuple(y.shape), generator=gen)).to(dev)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    net = LatentDiffusionNetwork.from_config(seed=0, device=dev, torch_dtype=dtype)
    net.set_sampling_parameters(100, batch_size=args.batch)
    if args.cfg:  # distinct conditional / unconditional contexts: the doubled-batch path
        pe = torch.randn(args.batch, 77, 768, generator=torch.Generator().manual_seed(77))
        cond = StableDiffusionCondition(prompt=None, prompt_embeds=pe, guidance_scale=7.5)
    else:
        cond = StableDiffusionCondition(prompt=[""] * args.batch)  # reference default: CFG collapses
    net.set_condition(cond)
    problem = InverseProblem(op, y, GaussianNoise(0.05).to(dev))
    lat = tuple(net.get_latent_shape(shape))
    from samplers_amd.networks.base import fp32_view

    step = FusedPSLDStep(fp32_view(net), problem, y.reshape(args.batch, -1), 1, lat, group=group)
    seed, off = 20260101, rank * args.batch
    z = initial_sample((args.batch, *lat), dev, rng="philox", seed=seed, sample_offset=off,
                       noise_fn=None)
    ts = net.timesteps_host
    it = iter(range(len(ts) - 1, 1, -1))

    def one():
        i = next(it)
        step(z, i, ts[i], ts[i - 1], ts[0], seed=seed, sample_offset=off)

    t0 = time.perf_counter()
    for k in range(args.warmup):
        one()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[psld] warmup {k + 1} done at {time.perf_counter() - t0:.1f}s",
                  file=sys.stderr, flush=True)
    torch.cuda.reset_peak_memory_stats()
    from samplers_amd.samplers.dps import KernelTimer

    timer = KernelTimer()  # dispatch-packet events on the library's timed kernels (conv tiles)
    timer.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        one()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[psld] step {k + 1} at {time.perf_counter() - t0:.1f}s", file=sys.stderr,
                  flush=True)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if not torch.isfinite(z).all():
        raise SystemExit("non-finite latents")
    ms = dt / args.steps * 1e3
    bf = args.dtype == "bf16"
    conv = conv_summary(timer.summary(), ("conv3x3_bf16",)) if bf else conv_summary(timer.summary())
    timer.close()
    roofline = None
    peak = MFMA_BF16_PEAK_TFLOPS if bf else MFMA_F32_PEAK_TFLOPS
    if conv:
        roofline = {"kernel": "3x3 conv tiles (" + " + ".join(conv["kernels"]) + ")",
                    "bound": "mfma", "achieved": round(conv["tflops"], 2),
                    "peak": peak, "unit": "TFLOP/s",
                    "frac": round(conv["tflops"] / peak, 4), "traffic": None,
                    "algorithmic_flops_per_launch": conv["flops"] / conv["count"],
                    "flops_basis": ("bf16 implicit GEMM: 18*N*Cin*Cout*H*W per launch (forward or input VJP), "
                                    "dense bf16 MFMA peak" if bf else
                                    "executed MFMA FLOPs (Winograd: 8*N*Cin*Cout*H*W, direct: 18*...)"),
                    "avg_launch_ms": round(conv["ms"] / conv["count"], 4),
                    "share_of_step": round(conv["ms"] / args.steps / ms, 4)}
    cpu = None
    if args.cpu_baseline and rank == 0:
        cpu = cpu_baseline_psld(args.image, cond if args.cfg else None, dtype)
    if world > 1:
        dist.destroy_process_group()
    if rank != 0:
        return
    print(json.dumps({
        "metric": "posterior samples/sec (batch×steps/s), PSLD SD1.5 512² (BASELINE configs[3])",
        "value": round(args.batch * world * args.steps / dt, 4),
        "unit": "samples/sec (batch×steps/s)",
        "n_gpus": world, "scaling": "weak", "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 2),
        "higher_is_better": True, "dtype": "bf16" if bf else "f32",
        "data": "synthetic (seeded U(-1,1) images, centre mask, sigma=0.05); random-init SD1.5 "
                "VAE + SD1.5 UNet2DConditionModel architecture (859.5 M, null 77x768 context)",
        "config": {"workload": f"PSLD + CenterInpainting(0.5) + GaussianNoise(0.05), 3x{args.image}²",
                   "batch_per_gpu": args.batch, "global_batch": args.batch * world,
                   "parallelism": f"dp{world}", "schedule": "100-step PNDM (psld.py:50)"},
        "vae_tflops": round(VAE_FLOP_PER_SAMPLE * args.batch / (ms / 1e3) / 1e12, 2),
        "model_tflops": round((VAE_FLOP_PER_SAMPLE + UNET_FLOP_PER_SAMPLE) * args.batch
                              / (ms / 1e3) / 1e12, 2),
        "peak_gib": round(torch.cuda.max_memory_allocated() / 2**30, 1),
        "cfg": bool(args.cfg),
        "roofline": roofline,
        "cpu_baseline": cpu,
    }), flush=True)


def cpu_baseline_psld(image: int, cond, dtype=torch.float32) -> dict:
    """One PSLD iteration (oracle/latent_loops.py, psld.py:118-153 semantics) at batch 1 on
    the host cores with the same random-init SD 1.5 networks (CPU copies, in ``dtype`` behind the
    same fp32 boundary as the device run), at the CPU share the job is given (bench.host_cpu)."""
    import numpy as np

    from oracle.latent_loops import psld_reference
    from samplers_amd.networks.latent import LatentDiffusionNetwork, StableDiffusionCondition
    from samplers_amd.operators import CenterInpaintingOperator

    host = host_cpu()
    torch.set_num_threads(host["cpu_share"])
    shape = (3, image, image)
    net = LatentDiffusionNetwork.from_config(seed=0, torch_dtype=dtype)
    net.set_sampling_parameters(100, batch_size=1)
    if cond is not None:
        cond = StableDiffusionCondition(prompt=None, prompt_embeds=cond.prompt_embeds[:1],
                                        guidance_scale=cond.guidance_scale)
    net.set_condition(cond if cond is not None else StableDiffusionCondition(prompt=[""]))
    kept = CenterInpaintingOperator(shape, 0.5)._kept_indices
    n = int(np.prod(shape))

    def apply(v):
        return v.reshape(v.shape[0], -1)[:, kept]

    def adjoint(v):
        out = torch.zeros(v.shape[0], n, dtype=v.dtype)
        out = out.index_put((torch.arange(v.shape[0])[:, None], kept[None, :]), v)
        return out.reshape(v.shape[0], *shape)

    gen = torch.Generator().manual_seed(5)
    y = apply(torch.rand(1, *shape, generator=gen) * 2 - 1)
    z = torch.randn(1, *net.get_latent_shape(shape), generator=gen)
    ts = net.timesteps_host
    t0 = time.perf_counter()
    f32 = lambda t: t.to(torch.float32)  # noqa: E731
    psld_reference(lambda v, t: f32(net(v.to(dtype), t)), net.alphas_cumprod.float(), ts, apply, adjoint,
                   lambda v: f32(net.decode(v.to(dtype), differentiable=True)),
                   lambda v: f32(net.encode(v.to(dtype), differentiable=True)), y, z,
                   lambda i: torch.randn(z.shape, generator=gen), steps_limit=1)
    dt = time.perf_counter() - t0
    return {"value": round(1 / dt, 5), "unit": "samples/sec (batch×steps/s)",
            "cores": host["cpu_share"], "kind": "port", "cpu_model": host["model"],
            "sample": f"one PSLD iteration of oracle/latent_loops.py at batch 1, 3x{image}², "
                      f"same random-init SD 1.5 VAE + UNet{' with CFG' if cond is not None else ''}, "
                      f"{'bf16 networks behind the fp32 boundary' if dtype == torch.bfloat16 else 'fp32'}, "
                      f"torch-CPU {torch.__version__}: {dt:.1f} s"}


if __name__ == "__main__":
    main()

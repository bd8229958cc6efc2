"""ReSample benchmark (BASELINE.json configs[4], "config 5"): SD1.5 latent, 512², Poisson noise.

    python tools/bench_resample.py [--batch 32 --steps 3 --warmup 2]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        tools/bench_resample.py --gpus N        (batch per rank)

Config 5 is 256 samples sharded over 8 GPUs: 32 per GPU, which is what one process here
runs (the batch shards with no data-path collective; the batch-global losses are 8-byte
all-reduces).  Workload: ReSample (resample.py:131-228) with IdentityOperator on 3x512x512,
PoissonNoise(rate=1.0) (config 5 fixes no rate), the SD 1.5 VAE architecture
(83.65 M parameters) + SD1.5 UNet2DConditionModel (859.5 M), random weights with fixed seeds, fp32.

A full ReSample run (100 steps, default max_optimization_iters=2000) is 98 main-loop
iterations plus time-travel blocks, three pixel-space and four latent-space hard
consistency solves; at B = 32 it runs for tens of minutes, so this tool times its pieces
on the same tensors and reports each:

  step          one main-loop iteration over the batch: latent UNet (epsilon-form DDIM,
                HIP sp_ddim_eps_step) + DPS conditioning (VAE decode forward + VJP, HIP
                norm gradient).  "value" = batch x steps / s of these iterations, the
                metric's unit (posterior samples/sec)
  pixel_iter    one pixel-space AdamW iteration (sp_pixel_opt_step + sp_opt_check; the
                host reads the device stop flag every 16 iterations)
  latent_iter   one latent-space AdamW iteration (VAE decode forward + VJP, HIP MSE
                gradient and AdamW)

With N ranks each holds ``--batch`` samples (Philox sample offset rank x batch); the
consistency losses and MSE totals are batch-global through 8-byte RCCL all-reduces
(resample.py's norms), and every figure is the max over ranks of the wall
time; "value" = N x batch x K / that time (weak scaling, as bench.py).

Prints one JSON line (rank 0).
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import samplers_amd  # noqa: E402,F401

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from bench import MFMA_F32_PEAK_TFLOPS, conv_summary, host_cpu, self_launch, setup_dist  # noqa: E402

sys.path.insert(0, str(ROOT / "tools"))
from bench_psld import VAE_FLOP_PER_SAMPLE, heartbeat  # noqa: E402

DECODE_FLOP_PER_SAMPLE = 4.96e12  # decode forward + VJP at 512²


def timed(fn, reps: int, label: str, world: int = 1, rank: int = 0) -> float:
    """Mean wall time of ``reps`` calls, bracketed by barriers, max over ranks."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(reps):
        fn()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[resample] {label} {k + 1}/{reps} at {time.perf_counter() - t0:.1f}s",
                  file=sys.stderr, flush=True)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=torch.device("cuda", torch.cuda.current_device()),
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--batch", type=int, default=32, help="samples per rank")
    p.add_argument("--image", type=int, default=512)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--pixel-iters", type=int, default=200)
    p.add_argument("--latent-iters", type=int, default=3)
    p.add_argument("--heartbeat", default="gpurun_out/resample_heartbeat.log")
    p.add_argument("--full-call", type=int, default=0, metavar="N",
                   help="also time one whole ReSampleSampler.__call__ with N sampling steps "
                        "(time travel every 5 indices, the reference's stopping rules, "
                        "--max-iters AdamW iterations at most)")
    p.add_argument("--max-iters", type=int, default=2000,
                   help="max_optimization_iters of the whole call (resample.py:56 default 2000; "
                        "the plateau rule needs > 200)")
    p.add_argument("--time-travel-interval", type=int, default=10,
                   help="time_travel_interval of the whole call (resample.py:59 default 10)")
    p.add_argument("--full-batch", type=int, default=0,
                   help="samples per rank of the whole call (default: --batch)")
    p.add_argument("--cpu-baseline", action="store_true",
                   help="also time one main-loop iteration and one latent AdamW iteration of "
                        "oracle/resample_loop.py on the host cores (batch 1)")
    args = p.parse_args()
    Path(args.heartbeat).parent.mkdir(parents=True, exist_ok=True)
    heartbeat(Path(args.heartbeat))
    # `--gpus N` without a launcher starts its N ranks itself (before anything touches the GPU)
    status = self_launch(args.gpus, sys.argv[1:], script=__file__)
    if status is not None:
        sys.exit(status)
    rank, world, dev = setup_dist(args.gpus)
    group = dist.group.WORLD if world > 1 else None

    from samplers_amd import _hip
    from samplers_amd.networks.latent import LatentDiffusionNetwork, StableDiffusionCondition
    from samplers_amd.noise import PoissonNoise
    from samplers_amd.operators import IdentityOperator
    from samplers_amd.samplers.dps import initial_sample
    from samplers_amd.samplers.resample import ReSampleSampler, _Consistency

    _hip.load_library()
    shape = (3, args.image, args.image)
    b = args.batch
    op = IdentityOperator(shape)
    gen = torch.Generator().manual_seed(1000 + rank)
    x_true = torch.rand((b, *shape), generator=gen) * 2 - 1
    noise = PoissonNoise(1.0)
    y = noise.sample(tuple(x_true.shape), generator=gen) + x_true  # y = A x + Poisson noise
    y = y.to(dev)
    net = LatentDiffusionNetwork.from_config(seed=0, device=dev)
    net.set_sampling_parameters(100, batch_size=b)
    net.set_condition(StableDiffusionCondition(prompt=[""] * b))  # reference default prompt, CFG collapses
    lat = tuple(net.get_latent_shape(shape))
    sampler = ReSampleSampler(net)
    cons = _Consistency(op, y.reshape(b, -1), 1, group)
    total = b * world * cons.m  # MSE mean over the global batch
    seed, off = 20260101, rank * b
    z = initial_sample((b, *lat), dev, rng="philox", seed=seed, sample_offset=off, noise_fn=None)
    ts, acp = net.timesteps_host, net.alphas_cumprod_host
    it = iter(range(len(ts) - 1, 1, -1))

    def one():
        nonlocal z
        i = next(it)
        z_next, pseudo, sqrt_a = sampler._ddim_eps(z, ts[i], ts[i - 1], 1.0, None, seed, i, off)
        z = sampler._dps_conditioning(z_next, pseudo, sqrt_a, float(acp[ts[i]]), cons)

    t0 = time.perf_counter()
    for k in range(args.warmup):
        one()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[resample] warmup {k + 1} done at {time.perf_counter() - t0:.1f}s",
                  file=sys.stderr, flush=True)
    torch.cuda.reset_peak_memory_stats()
    step_s = timed(one, args.steps, "step", world, rank)
    if not torch.isfinite(z).all():
        raise SystemExit("non-finite latents")

    x_pix = net.decode(z, differentiable=False).reshape(b, *shape).contiguous()
    sampler._pixel_optimization(x_pix, cons, total, 1e-3, 16)  # warm
    pix_s = timed(lambda: sampler._pixel_optimization(x_pix, cons, total, 0.0, args.pixel_iters),
                  1, "pixel", world, rank) / args.pixel_iters
    sampler._latent_optimization(z, cons, total, 1e-3, 1)  # warm
    from samplers_amd.samplers.dps import KernelTimer

    timer = KernelTimer()  # the decoder fwd + VJP's conv tiles during the latent AdamW iterations
    timer.clear()
    lat_s = timed(lambda: sampler._latent_optimization(z, cons, total, 0.0, args.latent_iters),
                  1, "latent", world, rank) / args.latent_iters
    conv = conv_summary(timer.summary())
    timer.close()
    roofline = None
    if conv:
        roofline = {"kernel": "3x3 conv tiles (" + " + ".join(conv["kernels"]) + "), latent AdamW "
                              "iterations (VAE decode forward + VJP)",
                    "bound": "mfma", "achieved": round(conv["tflops"], 2),
                    "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(conv["tflops"] / MFMA_F32_PEAK_TFLOPS, 4), "traffic": None,
                    "algorithmic_flops_per_launch": conv["flops"] / conv["count"],
                    "flops_basis": "executed MFMA FLOPs (Winograd: 8*N*Cin*Cout*H*W, direct: 18*...)",
                    "avg_launch_ms": round(conv["ms"] / conv["count"], 4),
                    "share_of_iteration": round(conv["ms"] / (args.latent_iters * lat_s * 1e3), 4)}

    # one epsilon-form DDIM step alone (the time-travel re-noising steps: UNet forward only)
    ddim_s = timed(lambda: sampler._ddim_eps(z, ts[5], ts[4], 1.0, None, seed, 5, off), 2, "ddim",
                   world, rank)
    projection = project_full_call(len(ts), args.max_iters, args.time_travel_interval, step_s,
                                   ddim_s, pix_s, lat_s, b * world)

    full = None
    if args.full_call:
        # one whole ReSample solve: main loop, time travel (pixel-space hard consistency in
        # the later stages), stochastic resampling and the final latent-space solve, with
        # the reference's stopping rules (resample_kernels.py:32-93)
        from samplers_amd.inverse_problem import InverseProblem

        fb = args.full_batch or b
        prob = InverseProblem(op, y[:fb], noise)
        kw = dict(num_sampling_steps=args.full_call, max_optimization_iters=args.max_iters,
                  time_travel_interval=args.time_travel_interval, seed=seed, sample_offset=off,
                  group=group, condition=StableDiffusionCondition(prompt=[""] * fb))
        wall = timed(lambda: sampler(prob, **kw), 1, "full call", world, rank)
        log = getattr(sampler, "optimization_log", [])
        full = {"num_sampling_steps": args.full_call, "guided_iterations": args.full_call - 2,
                "batch_per_gpu": fb, "max_optimization_iters": args.max_iters,
                "time_travel_interval": args.time_travel_interval,
                "wall_s": round(wall, 2), "gpu_s_per_sample": round(wall / fb, 3),
                "samples_x_steps_per_s": round(fb * world * (args.full_call - 2) / wall, 4),
                # every hard-consistency solve: the AdamW iterations the reference's stopping
                # rules ran (loss below eps^2; latent: from iteration 200 a rising loss)
                "solves": log,
                "adamw_iterations": {k: sum(r["iterations"] for r in log if r["kind"] == k)
                                     for k in ("pixel", "latent")}}
    cpu = None
    if args.cpu_baseline and rank == 0:
        cpu = cpu_baseline_resample(args.image)
        # the same whole call on the host at batch 1, from its two measured iterations (a time-
        # travel DDIM step priced as a main-loop iteration, the pixel solves' AdamW as free:
        # both favour the CPU)
        c = projection
        cpu_wall = (c["main_loop_iterations"] + c["time_travel_ddim_steps"]) / cpu["value"] + \
            c["latent_solves"] * args.max_iters * cpu["latent_iter_s"]
        cpu["projected_full_call_s_batch1"] = round(cpu_wall, 1)
        cpu["samples_per_s_whole_call"] = round(1 / cpu_wall, 7)

    n = b * shape[0] * args.image * args.image
    peak_gib = round(torch.cuda.max_memory_allocated() / 2**30, 1)
    if world > 1:
        dist.destroy_process_group()
    if rank != 0:
        return
    print(json.dumps({
        "metric": "posterior samples/sec (batch×steps/s), ReSample SD1.5 512² Poisson "
                  "(BASELINE configs[4], 32 per GPU of 256 over 8)",
        "value": round(b * world / step_s, 4),
        "unit": "samples/sec (batch×steps/s)",
        "n_gpus": world, "scaling": "weak", "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(step_s * 1e3, 2), "higher_is_better": True, "dtype": "f32",
        "data": "synthetic (seeded U(-1,1) images, Poisson(rate=1) noise); random-init SD1.5 VAE "
                "+ SD1.5 UNet2DConditionModel architectures (null 77x768 context)",
        "config": {"workload": f"ReSample + Identity + PoissonNoise(1.0), 3x{args.image}²",
                   "batch_per_gpu": b, "global_batch": b * world,
                   "parallelism": f"dp{world}", "schedule": "100-step PNDM (resample.py:52)"},
        "decode_vjp_tflops": round(DECODE_FLOP_PER_SAMPLE * b / step_s / 1e12, 2),
        "pixel_iter_ms": round(pix_s * 1e3, 4),
        "pixel_iter_GBps": round(4 * 7 * n / pix_s / 1e9, 1),  # x,m,v,y read; x,m,v written
        "latent_iter_ms": round(lat_s * 1e3, 2),
        "latent_iter_tflops": round(DECODE_FLOP_PER_SAMPLE * b / lat_s / 1e12, 2),
        "peak_gib": peak_gib,
        "vae_flop_per_sample_step": VAE_FLOP_PER_SAMPLE,
        "roofline": roofline,
        "ddim_step_ms": round(ddim_s * 1e3, 2),
        "pixel_iters_timed": args.pixel_iters, "latent_iters_timed": args.latent_iters,
        "projected_full_call": projection,
        "full_call": full,
        "cpu_baseline": cpu,
    }), flush=True)


def project_full_call(n_ts: int, max_iters: int, interval: int, step_s: float, ddim_s: float,
                      pix_s: float, lat_s: float, batch: int, inter: int = 5, splits: int = 3) -> dict:
    """A whole ReSampleSampler.__call__ at these settings from the measured per-iteration costs:
    the sampler's own loop control (samplers/resample.py __call__, resample.py:131-228) walked
    without running it, counting main-loop iterations, time-travel DDIM steps and the pixel- /
    latent-space solves, each solve priced at ``max_iters`` AdamW iterations (every solve of the
    random-init prior ran all of them: profiles/round4/secondary/)."""
    total = n_ts - 1
    split = total // splits
    main = travel = pix = lat = 0
    for idx in range(n_ts - 1, 1, -1):
        main += 1
        if idx <= total - split and idx % interval == 0:
            travel += sum(1 for kk in range(idx, max(idx - inter, 1), -1) if kk > 1)
            if idx >= split:
                pix += 1
            else:
                lat += 1
    lat += 1  # the final latent-space solve
    parts = {"main_loop": main * step_s, "time_travel_ddim": travel * ddim_s,
             "pixel_solves": pix * max_iters * pix_s, "latent_solves": lat * max_iters * lat_s}
    wall = sum(parts.values())
    return {"main_loop_iterations": main, "time_travel_ddim_steps": travel, "pixel_solves": pix,
            "latent_solves": lat, "adamw_iterations_per_solve": max_iters,
            "seconds": {k: round(v, 1) for k, v in parts.items()}, "wall_s": round(wall, 1),
            "samples_per_s_whole_call": round(batch / wall, 5),
            "samples_x_guided_steps_per_s": round(batch * (n_ts - 2) / wall, 4),
            "basis": "measured per-iteration costs of this run x the loop's counts (no solve "
                     "stopped early: the stopping rules never fired on the random-init prior)"}


def cpu_baseline_resample(image: int) -> dict:
    """One ReSample main-loop iteration (ε-form DDIM step + DPS conditioning through the
    decoder VJP) and one latent-space AdamW iteration (decoder forward + VJP), restated by
    oracle/resample_loop.py, at batch 1 on the host cores with the same random-init SD 1.5
    networks (CPU copies)."""
    from oracle.resample_loop import ddim_step_eps
    from samplers_amd.networks.latent import LatentDiffusionNetwork, StableDiffusionCondition

    host = host_cpu()
    torch.set_num_threads(host["cpu_share"])
    shape = (3, image, image)
    net = LatentDiffusionNetwork.from_config(seed=0)
    net.set_sampling_parameters(100, batch_size=1)
    net.set_condition(StableDiffusionCondition(prompt=[""]))
    gen = torch.Generator().manual_seed(5)
    y = (torch.rand(1, *shape, generator=gen) * 2 - 1).reshape(1, -1)
    z = torch.randn(1, *net.get_latent_shape(shape), generator=gen)
    acp, ts = net.alphas_cumprod, net.timesteps_host
    i = len(ts) - 1
    t0 = time.perf_counter()
    zr = z.clone().requires_grad_()
    z_next, _x0, pseudo = ddim_step_eps(zr, lambda v, t: net(v, t), acp, ts[i], ts[i - 1], 1.0,
                                        lambda s: torch.randn(s, generator=gen))
    norm = torch.linalg.norm(y - net.decode(pseudo, differentiable=True).reshape(1, -1))
    (g,) = torch.autograd.grad(norm, zr)
    z = z_next.detach() - g * 0.5 * acp[ts[i]]
    step_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    zo = z.clone().requires_grad_()
    opt = torch.optim.AdamW([zo], lr=5e-3)
    opt.zero_grad()
    loss = torch.nn.MSELoss()(y, net.decode(zo, differentiable=True).reshape(1, -1))
    loss.backward()
    opt.step()
    lat_s = time.perf_counter() - t0
    return {"value": round(1 / step_s, 5), "unit": "samples/sec (batch×steps/s)",
            "cores": host["cpu_share"], "kind": "port", "cpu_model": host["model"],
            "latent_iter_s": round(lat_s, 2),
            "sample": f"one main-loop iteration ({step_s:.1f} s) and one latent AdamW iteration "
                      f"({lat_s:.1f} s) of oracle/resample_loop.py at batch 1, 3x{image}², same "
                      f"random-init SD 1.5 VAE + UNet, fp32, torch-CPU {torch.__version__}"}


if __name__ == "__main__":
    main()

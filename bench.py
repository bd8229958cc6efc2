"""Headline benchmark: posterior samples/sec of DPS on CelebA-HQ-256 (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Without a launcher, ``--gpus N`` (N > 1) starts its N ranks itself (a child
torch.distributed.run on 127.0.0.1) and exits with its status.

Workload (BASELINE.json configs[1], "config 2"): DPS + 50 % random inpainting
mask + GaussianNoise(sigma=0.05) on 3x256x256 images, prior = the
ddpm-celebahq-256 UNet architecture (113.7 M parameters, random weights with a
fixed seed — no checkpoint offline), fp32, 64 samples per GPU, DDPM schedule
with 1000 steps.  One bench step = one guided DPS iteration over the whole
per-GPU batch: UNet forward + HIP residual pass + UNet input-VJP + HIP update
pass (``samplers_amd.samplers.dps.FusedDPSStep``), timesteps walking down from
t = 999 as in the sampler.  Inputs are resident in HBM before timing starts.

value = (samples per GPU x GPUs x K steps) / max-over-ranks wall time of the K
timed steps (weak scaling: the per-GPU batch is fixed).  The sample batch is
sharded over ranks with no data-path collective (DPS samples are independent,
SURVEY.md F6); Philox noise is keyed by the global sample index.

Also reported:
  roofline      the dominant HIP kernel of the step.  Since the prior's 3x3
                convolutions run on this project's fp32-MFMA tile it is that
                kernel: algorithmic FLOPs (2*9*N*Cin*Cout*H*W per launch, fwd and
                input VJP) / its launch times from HIP events attached to the
                dispatch packets on the launch stream, against the 157.3 TFLOP/s
                dense fp32 MFMA peak
  guidance_roofline  the dominant guidance pass (pass 1 / pass 2): algorithmic
                bytes per launch / mean launch time, against the
                8 TB/s HBM peak; traffic = PMC-measured HBM bytes per launch
                (profiles/pmc_traffic.json, separate rocprofv3 --pmc passes)
  cpu_baseline  oracle/dps_loop.py (torch-CPU restatement of dps.py) with the
                same UNet, timed on this host's cores for a bounded sample
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
import samplers_amd  # noqa: E402,F401

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, MI355X_MICROARCH.md
MFMA_F32_PEAK_TFLOPS = 157.3  # dense fp32 MFMA (v_mfma_f32_32x32x2_f32), MI355X_MICROARCH.md
MFMA_BF16_PEAK_TFLOPS = 2516.6  # dense bf16 MFMA: 256 CUs x 4 SIMDs x 1024 FLOP/clk x 2.4 GHz (~2.5 PF)

# DPS workloads of BASELINE.json (configs[0..2]); inpaint is the headline metric's config
CONFIGS = {
    "inpaint": "DPS + InpaintingMask(50% random) + GaussianNoise(0.05) (BASELINE configs[1])",
    "blur": "DPS + GaussianBlur(9x9, sigma=3) + GaussianNoise(0.05) (BASELINE configs[2])",
    "identity": "DPS + IdentityOperator + GaussianNoise(0.05) (BASELINE configs[0] on the GPU)",
}
METRIC = "posterior samples/sec (batch×steps/s), DPS CelebA-HQ-256 @1/2/4/8 GPU"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=64, help="samples per GPU")
    p.add_argument("--image", type=int, default=256)
    p.add_argument("--config", choices=sorted(CONFIGS), default="inpaint",
                   help="DPS workload: inpaint = BASELINE configs[1] (headline), blur = configs[2] "
                        "(64 per GPU of the 512 sharded over 8), identity = configs[0] on the GPU")
    p.add_argument("--micro-batch", type=int, default=0)
    p.add_argument("--reuse-v", action="store_true",
                   help="pass 2 re-reads pass 1's v instead of re-deriving it from y (the default)")
    p.add_argument("--graph", action="store_true",
                   help="replay one hipGraph-captured step (samplers/graph.py); kernel times and "
                        "the roofline then come from the eager warmup steps")
    p.add_argument("--dtype", choices=("fp32", "bf16"), default="fp32",
                   help="the prior's dtype (fp32: the headline, the reference's run_dps.py:14; bf16: the "
                        "reference's bf16 precision on the bf16 NHWC kernels, behind the fp32 sampler loop)")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    return p.parse_args()


def log(msg: str) -> None:
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def launch_command(argv: list[str], gpus: int, port: int, script: str | None = None) -> list[str]:
    """The torch.distributed.run command that starts `gpus` ranks of `script` (this file by
    default) with the same arguments (one process per GPU, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
            str(Path(script or __file__).resolve()), *argv]


def self_launch(gpus: int, argv: list[str], script: str | None = None) -> int | None:
    """`python bench.py --gpus N` without a launcher (no WORLD_SIZE in the environment)
    starts its N ranks itself as a child torch.distributed.run and returns its exit status;
    None when this process is already a rank (or N = 1).  Runs before anything touches the
    GPU (device_count does not initialise HIP on this image), so nothing is exec'd from a
    process holding a GPU context."""
    if gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    backend = os.environ.get("SAMPLERS_AMD_DIST_BACKEND", "nccl")
    have = torch.cuda.device_count()
    if backend == "nccl" and have < gpus:
        raise SystemExit(f"--gpus {gpus}: only {have} GPU(s) visible (RCCL needs one per rank; "
                         "SAMPLERS_AMD_DIST_BACKEND=gloo rehearses more ranks than GPUs)")
    cmd = launch_command(argv, gpus, free_port(), script)
    log(f"starting {gpus} ranks: {' '.join(cmd[1:])}")
    import subprocess

    return subprocess.run(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")).returncode


def setup_dist(gpus: int):
    """One rank per GPU over RCCL (backend "nccl").  SAMPLERS_AMD_DIST_BACKEND=gloo is a
    rehearsal mode for a box with fewer GPUs than ranks: ranks share devices round-robin
    and the collectives go through host memory (not a measurement configuration)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != gpus:
        raise SystemExit(f"--gpus {gpus} but WORLD_SIZE={world}")
    backend = os.environ.get("SAMPLERS_AMD_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        extra = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **extra)
    return rank, world, torch.device("cuda", local)


def measure_gather(x: torch.Tensor, reps: int = 3) -> dict:
    """The design's only data-path collective: ``distributed.gather_shards`` of the x-hat
    shards (one ``all_gather_into_tensor``, RCCL over xGMI with backend "nccl"), as the sampler
    runs it once at the end of a solve (``dps.py:125-130`` is the result it assembles).  Timed
    like the steps (barrier + device sync on both sides, max over ranks): the first call (it
    includes the communicator's lazy setup) and the best of `reps` more.  Returns the
    collective's record for the JSON line: the backend and world size torch.distributed
    reports, bytes per rank, gathered bytes, and the times."""
    from samplers_amd.distributed import gather_shards

    world = dist.get_world_size() if dist.is_initialized() else 1
    rec = {"op": "all_gather_into_tensor (samplers_amd.distributed.gather_shards)",
           "backend": dist.get_backend() if dist.is_initialized() else None,
           "world_size": world, "bytes_per_rank": x.numel() * x.element_size(),
           "gathered_bytes": x.numel() * x.element_size() * world}
    if world == 1:
        return dict(rec, gather_ms=0.0, first_gather_ms=0.0, note="one rank: nothing to gather")
    if rec["backend"] == "gloo":
        rec["rehearsal"] = ("gloo through host memory, ranks sharing the visible GPUs: checks the "
                            "sharded path and its gather, not a measurement of RCCL over xGMI")
    sync = torch.cuda.synchronize if x.is_cuda else (lambda: None)
    counts = [x.shape[0]] * world
    times = []
    for _ in range(1 + reps):
        dist.barrier()
        sync()
        t0 = time.perf_counter()
        full = gather_shards(x, counts)
        sync()
        dist.barrier()
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                          device=x.device if x.is_cuda else None)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        times.append(float(dt.item()) * 1e3)
    if tuple(full.shape) != (x.shape[0] * world, *x.shape[1:]):
        raise SystemExit(f"gather returned {tuple(full.shape)}")
    rank = dist.get_rank()
    if not torch.equal(full[rank * x.shape[0]:(rank + 1) * x.shape[0]], x):
        raise SystemExit(f"rank {rank}: its slice of the gathered x differs from its shard")
    return dict(rec, gather_ms=round(min(times[1:]), 4), first_gather_ms=round(times[0], 4),
                gathered_shape=list(full.shape), own_slice_checked=True)


def build_workload(config: str, batch: int, image: int, rank: int, device, dtype=torch.float32):
    from samplers_amd.inverse_problem import InverseProblem
    from samplers_amd.networks.ddpm import DDPMNetwork
    from samplers_amd.noise import GaussianNoise
    from samplers_amd.operators import (GaussianBlurOperator, IdentityOperator,
                                        RandomInpaintingOperator)

    shape = (3, image, image)
    if config == "inpaint":
        op = RandomInpaintingOperator(shape, fraction=0.5, seed=1).to(device)
    elif config == "blur":
        op = GaussianBlurOperator(shape, kernel_size=9, sigma=3.0).to(device)
    else:
        op = IdentityOperator(shape)
    noise = GaussianNoise(0.05).to(device)
    gen = torch.Generator().manual_seed(1000 + rank)  # per-rank shard of the synthetic dataset
    x_true = torch.rand((batch, *shape), generator=gen) * 2 - 1
    y_clean = op.apply(x_true.to(device))  # HIP operator
    y = y_clean + (0.05 * torch.randn(tuple(y_clean.shape), generator=gen)).to(device)
    net = DDPMNetwork.from_config(seed=0, device=device, torch_dtype=dtype)
    net.set_sampling_parameters(1000, batch_size=batch)
    return InverseProblem(op, y, noise), net, shape


def guidance_bytes(n: int, m: int, index_bytes: int) -> dict[str, float]:
    """Algorithmic HBM bytes per sample (fp32): SURVEY.md §8d, 4(7n + 2m) + index."""
    return {
        "dps_residual": 4.0 * (3 * n + m),  # read x, eps, y; write v (blur: halo re-reads excluded)
        "dps_update": 4.0 * (4 * n + m),    # read x, eps, w, y; write x'
        "dps_update_reuse_v": 4.0 * 5 * n,  # read x, eps, w, v; write x'
        "index_per_launch": float(index_bytes),  # inpaint keep bits + ranks / blur taps, per launch
    }


def load_pmc() -> dict:
    """PMC-measured HBM bytes per launch (profiles/pmc_traffic.json), keyed kernel@config."""
    pmc = ROOT / "profiles" / "pmc_traffic.json"
    try:
        return json.loads(pmc.read_text()) if pmc.exists() else {}
    except (ValueError, OSError):
        return {}


def conv_summary(kern: dict, names=("wino3x3_fwd", "wino3x3_bwd_input", "conv3x3_fwd",
                                    "conv3x3_bwd_input")) -> dict | None:
    """The prior's 3x3 convolution tiles (Winograd F(2x2,3x3) and direct, fwd + input VJP;
    ``names=("conv3x3_bf16",)``: the bf16 implicit-GEMM tile): count, ms, executed MFMA FLOPs,
    and direct-convolution-equivalent FLOPs."""
    parts = {k: kern[k] for k in names if k in kern}
    if not parts:
        return None
    out = {k: sum(p[k] for p in parts.values()) for k in ("count", "ms", "flops")}
    out["effective_flops"] = sum(p["flops"] * (18 / 8 if k.startswith("wino") else 1)
                                 for k, p in parts.items())
    out["tflops"] = out["flops"] / out["ms"] / 1e9
    out["effective_tflops"] = out["effective_flops"] / out["ms"] / 1e9
    out["kernels"] = sorted(parts)
    return out


def host_cpu() -> dict:
    """The host's CPU model, the cores this process may run on, and the cgroup CPU quota
    (a container's share of the machine, which can be far below the visible core count)."""
    model = "unknown"
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    for path, parse_q in (("/sys/fs/cgroup/cpu.max", lambda s: s.split()),
                          ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            if parse_q is not None:
                q, p = parse_q(Path(path).read_text())
                if q != "max":
                    quota = float(q) / float(p)
            else:
                q = float(Path(path).read_text())
                p = float(Path("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read_text())
                if q > 0:
                    quota = q / p
            break
        except (OSError, ValueError):
            continue
    omp = os.environ.get("OMP_NUM_THREADS", "")
    share = int(omp) if omp.isdigit() and int(omp) > 0 else None
    if share is None and quota:
        share = max(1, int(quota + 0.5))
    return {"model": model, "affinity_cores": affinity, "cgroup_cpus": quota,
            "cpu_share": min(share or affinity, affinity)}


class _Heartbeat:
    """A line on stderr every `every` s while a long CPU leg runs (a silent run is taken to be
    hung by the GPU pool's watchdog)."""

    def __init__(self, what: str, every: float = 30.0):
        import threading

        self.what, self.every, self.stop = what, every, threading.Event()
        self.t0 = time.perf_counter()
        self.th = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        while not self.stop.wait(self.every):
            log(f"{self.what}: still running at {time.perf_counter() - self.t0:.0f}s")

    def __enter__(self):
        self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        return False


def cpu_baseline(image: int, seconds: float, config: str = "inpaint", dtype=torch.float32) -> dict:
    """oracle/dps_loop.py (dps.py:91-122 semantics) on the host cores with the same UNet and
    workload per sample (the config's operator: 50 % random mask, 9x9 / sigma 3 blur or identity).  The thread count is probed first at batch 1 (the CPU share this
    process is given — OMP_NUM_THREADS / the cgroup quota — and multiples of it up to every
    core the process may run on), then batch 1 and batch 8 are timed on the best count for
    about `seconds` / 2 each; the best per-sample rate is reported."""
    with _Heartbeat("cpu baseline"):
        return _cpu_baseline(image, seconds, config, dtype)


def _cpu_apply_op(config: str, shape: tuple):
    """(the config's forward operator A on the CPU, its description) for the oracle loop."""
    if config == "blur":
        from oracle import blur as oblur

        k1d = oblur.taps(9, 3.0)
        return (lambda v: oblur.blur(v, k1d).to(v.dtype)), "9x9 / sigma 3 Gaussian blur (reflect)"
    if config == "identity":
        return (lambda v: v), "identity operator"
    from samplers_amd.operators import get_mask_random

    mask = get_mask_random(shape, 0.5, seed=1)
    kept = torch.nonzero(~mask.flatten()).squeeze(1)
    return (lambda v: v.reshape(v.shape[0], -1)[:, kept]), "50% random mask"


def _cpu_baseline(image: int, seconds: float, config: str = "inpaint", dtype=torch.float32) -> dict:
    from oracle import dps_loop
    from samplers_amd.networks.unet2d import build_unet

    host = host_cpu()
    share, cores = host["cpu_share"], host["affinity_cores"]
    candidates = sorted({min(cores, share * k) for k in (1, 2, 4)})
    shape = (3, image, image)
    unet = build_unet(seed=0).to(dtype)  # bf16: the same UNet's CPU copy behind the fp32 loop
    eps = (lambda v, t: unet(v, t)) if dtype == torch.float32 else (lambda v, t: unet(v.to(dtype), t).float())
    apply_op, op_desc = _cpu_apply_op(config, shape)
    betas = torch.linspace(1e-4, 0.02, 1000, dtype=torch.float32)
    acp = torch.cat([torch.ones(1), torch.cumprod(1 - betas, 0)]).clip(1e-6, 1)
    ts = list(range(1000))
    lp = dps_loop.gaussian_log_prob(0.05)
    def point(batch: int, nthreads: int, budget: float) -> dict:
        torch.set_num_threads(nthreads)
        gen = torch.Generator().manual_seed(1000)
        x_true = torch.rand((batch, *shape), generator=gen) * 2 - 1
        y0 = apply_op(x_true)
        y = y0 + 0.05 * torch.randn(y0.shape, generator=gen)
        x = torch.randn((batch, *shape), generator=gen)
        noise = lambda i: torch.randn((batch, *shape), generator=gen)  # noqa: E731
        # one warm-up iteration, then as many as fit in the budget (at least 1)
        x = dps_loop.dps_reference(eps, acp, ts, apply_op, lp, y, x, noise,
                                   gamma=1.0, eta=1.0, steps_limit=1, return_sample=True)
        done, t0 = 0, time.perf_counter()
        while done < 1 or time.perf_counter() - t0 < budget:
            x = dps_loop.dps_reference(eps, acp, ts, apply_op, lp, y, x,
                                       noise, gamma=1.0, eta=1.0, steps_limit=1,
                                       return_sample=True)
            done += 1
        dt = time.perf_counter() - t0
        rec = {"batch": batch, "threads": nthreads, "iterations": done,
               "samples_per_s": round(batch * done / dt, 4)}
        log(f"cpu baseline: batch {batch}, {nthreads} threads: {rec['samples_per_s']} samples/s")
        return rec

    probe = [point(1, t, 0.0) for t in candidates]  # thread-count probe: one timed iteration
    nthreads = max(probe, key=lambda p: p["samples_per_s"])["threads"]
    sweep = [point(b, nthreads, seconds / 2) for b in ((1, 8) if image <= 256 else (1, 2))]
    best = max(sweep, key=lambda p: p["samples_per_s"])
    return {
        "value": best["samples_per_s"],
        "unit": "samples/sec (batch×steps/s)",
        "cores": best["threads"],
        "kind": "port",
        "cpu_model": host["model"],
        "host_cores": cores,
        "cpu_share": share,
        "cgroup_cpus": host["cgroup_cpus"],
        "thread_probe": probe,
        "sweep": sweep,
        "sample": f"batch {' and '.join(str(p['batch']) for p in sweep)} on the best of {candidates} threads (probed at batch 1): "
                  f"guided DPS iterations (t=999) of oracle/dps_loop.py at 3x{image}x{image}, "
                  f"{op_desc}, same random-init UNet, "
                  f"{'bf16 UNet behind the fp32 loop' if dtype == torch.bfloat16 else 'fp32'}, torch-CPU {torch.__version__}; "
                  f"best = batch {best['batch']} on {best['threads']} threads, "
                  f"{best['iterations']} iterations",
    }


def main():
    args = parse()
    if args.graph and args.warmup < 1:
        raise SystemExit("--graph needs --warmup >= 1 (kernel records come from the warmup)")
    status = self_launch(args.gpus, sys.argv[1:])
    if status is not None:
        sys.exit(status)
    rank, world, device = setup_dist(args.gpus)
    torch.backends.cudnn.benchmark = False  # MIOpen immediate mode: no exhaustive search
    from samplers_amd import _hip
    from samplers_amd.samplers.dps import FusedDPSStep, KernelTimer

    _hip.load_library()
    bf = args.dtype == "bf16"
    problem, net, shape = build_workload(args.config, args.batch, args.image, rank, device,
                                         torch.bfloat16 if bf else torch.float32)
    n = int(np.prod(shape))
    m = int(problem.operator.hip_descriptor().m)
    index_bytes = 12 * ((n + 63) // 64) if args.config == "inpaint" else 0
    timer = KernelTimer()
    from samplers_amd.networks.base import fp32_view

    step = FusedDPSStep(fp32_view(net), problem, problem.observation, 1, gamma=1.0, eta=1.0,
                        micro_batch=args.micro_batch or None, timer=timer, reuse_v=args.reuse_v)
    from samplers_amd.samplers.dps import initial_sample

    seed = 20260101
    x = initial_sample((args.batch, *shape), device, rng="philox", seed=seed,
                       sample_offset=rank * args.batch, noise_fn=None)
    ts = net.timesteps_host
    it = iter(range(len(ts) - 1, 1, -1))

    def one_step():
        i = next(it)
        step(x, i, ts[i], ts[i - 1], ts[0], seed=seed, sample_offset=rank * args.batch)

    t_w = time.perf_counter()
    for k in range(args.warmup):
        one_step()
        torch.cuda.synchronize()
        log(f"warmup step {k + 1}/{args.warmup} done at {time.perf_counter() - t_w:.1f}s")
    graph = None
    if args.graph:
        # kernel times of the (eager) warmup steps stand in for the replays' (events cannot
        # be captured); the timed region is K replays of the captured step
        kern_warm = timer.summary()
        timer.close()
        step.timer = None
        from samplers_amd.samplers.graph import GraphedStepLoop

        rest = [next(it) for _ in range(args.steps)]
        graph = GraphedStepLoop(step, x, [(i, ts[i], ts[i - 1], ts[0]) for i in rest], seed=seed,
                                sample_offset=rank * args.batch)
        graph.capture()
        log("captured one step into a hipGraph")
    else:
        timer.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # the timed steps run under the samplers' solve guard: it counts the single-pass GroupNorm
    # chunk partials the kernels had to recompute because a team member was not resident
    # (exact, so a cost and not an error; the counter is read after the clock stops)
    guard = _hip.solve_guard()
    guard.__enter__()
    t0 = time.perf_counter()
    if graph is not None:
        graph.replay()
    else:
        for _ in range(args.steps):
            one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    guard.__exit__(None, None, None)
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if not torch.isfinite(x).all():
        raise SystemExit("non-finite samples")

    # the x-hat gather that ends a sharded solve (after the clock: once per solve of 998 steps)
    collective = measure_gather(x)
    kern = kern_warm if graph is not None else timer.summary()
    kern_steps = args.warmup if graph is not None else args.steps  # steps the records cover
    nbytes = guidance_bytes(n, m, index_bytes)
    rl = {}
    for name in ("dps_residual", "dps_update"):
        d = kern[name]
        avg_ms = d["ms"] / d["count"]
        key = "dps_update_reuse_v" if (name == "dps_update" and step.needs_v) else name
        per_launch = nbytes[key] * d["samples"] / d["count"] + nbytes["index_per_launch"]
        rl[name] = {"avg_ms": avg_ms, "bytes": per_launch, "gbs": per_launch / avg_ms / 1e6}
    g_dom = max(rl, key=lambda k: rl[k]["avg_ms"])
    pmc = load_pmc()
    tag = "" if args.config == "inpaint" else f"_{args.config}"
    g_rec = pmc.get(f"{g_dom}@B{args.batch}_{args.image}{tag}")
    guidance_roofline = {
        "kernel": g_dom, "bound": "hbm", "achieved": round(rl[g_dom]["gbs"], 1),
        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(rl[g_dom]["gbs"] / HBM_PEAK_GBS, 4),
        "traffic": g_rec["hbm_bytes_per_launch"] if g_rec else None,
        "algorithmic_bytes_per_launch": rl[g_dom]["bytes"],
        "avg_launch_ms": round(rl[g_dom]["avg_ms"], 5),
    }
    if g_dom == "dps_update" and step.needs_v:
        # SURVEY §8d's minimal K2 bytes (read x, eps, w, y; write x'): pass 2 re-reads v
        # instead (one more coalesced stream, measured faster than the gather), which the
        # figure above counts; this one prices the launch at the minimum
        d = kern["dps_update"]
        min_bytes = nbytes["dps_update"] * d["samples"] / d["count"] + nbytes["index_per_launch"]
        guidance_roofline["minimal_bytes_per_launch"] = min_bytes
        guidance_roofline["frac_minimal"] = round(min_bytes / rl[g_dom]["avg_ms"] / 1e6
                                                  / HBM_PEAK_GBS, 4)
    conv = conv_summary(kern, ("conv3x3_bf16",)) if bf else conv_summary(kern)
    peak = MFMA_BF16_PEAK_TFLOPS if bf else MFMA_F32_PEAK_TFLOPS
    if conv and conv["ms"] > sum(rl[k]["avg_ms"] * kern[k]["count"] for k in rl):
        # the prior's MFMA convolution tile dominates the step
        c_rec = None if bf else pmc.get(f"conv3x3_tiles@B{args.batch}_{args.image}{tag}")
        roofline = {
            "kernel": "3x3 conv tiles (" + " + ".join(conv["kernels"]) + ")", "bound": "mfma",
            "achieved": round(conv["tflops"], 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(conv["tflops"] / peak, 4),
            "traffic": c_rec["hbm_bytes_per_launch"] if c_rec else None,
            "algorithmic_flops_per_launch": conv["flops"] / conv["count"],
            "flops_basis": ("bf16 implicit GEMM: 18*N*Cin*Cout*H*W (+ 2*N*Cs*Cout*H*W where a 1x1 shortcut is fused) per launch, dense bf16 MFMA peak" if bf else
                            "executed MFMA FLOPs (Winograd: 8*N*Cin*Cout*H*W, direct: 18*...)"),
            "effective_tflops": round(conv["effective_tflops"], 2),
            "avg_launch_ms": round(conv["ms"] / conv["count"], 4),
            "launches_per_step": conv["count"] / kern_steps,
            "share_of_step": round(conv["ms"] / kern_steps / (elapsed / args.steps * 1e3), 4),
        }
    else:
        roofline = guidance_roofline

    total = args.batch * world * args.steps
    value = total / elapsed
    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "samples/sec (batch×steps/s)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16" if bf else "f32",
        "arithmetic": ({
            "guidance, bridge update, sample": "fp32",
            "prior (UNet forward + input VJP)": "bf16 activations / weights on the bf16 NHWC kernels (conv, "
                                                "GroupNorm, attention), fp32 accumulation and statistics"}
            if bf else {
            "guidance, GroupNorm, 3x3 convs (Winograd / direct / stride-2), attention": "fp32 (fp32 MFMA, fp32 VALU)",
            "1x1 shortcuts, attention / transformer linears":
                "fp32 operands on bf16 MFMAs: exact three-term splits, six partial products, fp32 "
                "accumulation (relative L2 error 1.1e-7 vs fp64, hipBLASLt fp32 2.0e-7; "
                "SAMPLERS_AMD_SHORTCUT=torch / SAMPLERS_AMD_LINEAR=torch select hipBLASLt fp32)"}),
        "data": "synthetic (seeded U(-1,1) images, sigma=0.05 Gaussian noise; "
                "random-init ddpm-celebahq-256 UNet architecture)",
        "config": {"workload": f"{CONFIGS[args.config]}, 3x{args.image}x{args.image}, "
                               "ddpm-celebahq-256 prior, 1000-step DDPM schedule",
                   "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                   "parallelism": f"sample-batch shards x{world}, no collective inside a step; "
                                  "one all-gather of x-hat per solve (timed after the steps: "
                                  "'collective')",
                   "execution": "hipGraph replay of one captured step" if graph is not None
                   else "eager"},
        # gloo over ranks sharing GPUs (SAMPLERS_AMD_DIST_BACKEND=gloo): a rehearsal of the sharded
        # path and its gather, not a throughput measurement
        "rehearsal": bool(world > 1 and collective.get("backend") == "gloo"),
        "roofline": roofline,
        "guidance_roofline": guidance_roofline,
        "guidance_kernels": {k: {"avg_ms": round(v["avg_ms"], 5), "GB/s": round(v["gbs"], 1)}
                             for k, v in rl.items()},
        "groupnorm_recomputed_partials": guard.recomputed,
        "collective": collective,
        # a whole 1000-step solve (998 guided steps) of the same shards including its gather
        "solve_rate_incl_gather": round(args.batch * world * 998 / (
            998 * elapsed / args.steps + collective["gather_ms"] / 1e3), 3),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("timing the CPU baseline ...")
        result["cpu_baseline"] = cpu_baseline(args.image, args.cpu_seconds, args.config,
                                              torch.bfloat16 if bf else torch.float32)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

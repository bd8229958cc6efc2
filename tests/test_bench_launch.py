"""bench.py's launcher plumbing (CPU): `python bench.py --gpus N` without WORLD_SIZE starts
N ranks through torch.distributed.run with the same arguments; a rank (WORLD_SIZE set) or
N = 1 runs in-process."""

from __future__ import annotations

import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_launch_command_forwards_arguments():
    argv = ["--gpus", "4", "--steps", "3", "--warmup", "1", "--config", "blur"]
    cmd = bench.launch_command(argv, 4, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29511" in cmd
    i = cmd.index(str(ROOT / "bench.py"))
    assert cmd[i + 1:] == argv


def test_self_launch_is_noop_for_one_gpu_or_inside_a_rank(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.self_launch(1, ["--gpus", "1"]) is None
    monkeypatch.setenv("WORLD_SIZE", "2")
    assert bench.self_launch(2, ["--gpus", "2"]) is None


def test_self_launch_spawns_ranks(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("SAMPLERS_AMD_DIST_BACKEND", "gloo")  # no GPU count check
    seen = {}

    def fake_run(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return subprocess.CompletedProcess(cmd, 3)

    monkeypatch.setattr(subprocess, "run", fake_run)
    assert bench.self_launch(2, ["--gpus", "2", "--steps", "1"]) == 3
    assert "--nproc-per-node=2" in seen["cmd"] and seen["cmd"][-3:] == ["--gpus", "2", "--steps", "1"][-3:]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_self_launch_refuses_more_rccl_ranks_than_gpus(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setenv("SAMPLERS_AMD_DIST_BACKEND", "nccl")
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 1)
    with pytest.raises(SystemExit, match="only 1 GPU"):
        bench.self_launch(8, ["--gpus", "8"])


def test_bench_help_runs_without_gpu():
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--help"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0 and "--gpus" in out.stdout


def _gather_worker(rank, world, port, out_path):
    import os

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = torch.full((3, 2, 4, 4), float(rank))
        rec = bench.measure_gather(x, reps=2)
        if rank == 0:
            torch.save(rec, out_path)
    finally:
        dist.destroy_process_group()


def test_measure_gather_records_the_collective(tmp_path):
    """The bench line's 'collective' record at world size 2 (gloo on CPU): the backend and world
    size torch.distributed reports, the bytes, the gathered shape, and finite times."""
    import torch
    import torch.multiprocessing as mp

    port = bench.free_port()
    path = tmp_path / "rec.pt"
    mp.spawn(_gather_worker, args=(2, port, str(path)), nprocs=2, join=True)
    rec = torch.load(path, weights_only=True)
    assert rec["backend"] == "gloo" and rec["world_size"] == 2
    assert rec["bytes_per_rank"] == 3 * 2 * 4 * 4 * 4 and rec["gathered_bytes"] == 2 * rec["bytes_per_rank"]
    assert rec["gathered_shape"] == [6, 2, 4, 4]
    assert 0 < rec["gather_ms"] < 60_000 and 0 < rec["first_gather_ms"] < 60_000


def test_measure_gather_single_rank():
    import torch

    rec = bench.measure_gather(torch.zeros(2, 3))
    assert rec["world_size"] == 1 and rec["gather_ms"] == 0.0 and rec["backend"] is None

"""MIOpen find-db seeding (samplers_amd/runtime.py): merge, idempotence, no partial files."""

from pathlib import Path

from samplers_amd import runtime


def test_find_db_merge_keeps_local_entries(tmp_path: Path):
    src = tmp_path / "seed.ufdb.txt"
    src.write_text("a=solverA:1.0\nb=solverB:2.0\n")
    dst = tmp_path / "cache" / "seed.ufdb.txt"
    dst.parent.mkdir()
    dst.write_text("a=measured_here:0.5\n")
    runtime._merge_find_db(src, dst)
    lines = dst.read_text().splitlines()
    assert lines == ["a=measured_here:0.5", "b=solverB:2.0"]
    runtime._merge_find_db(src, dst)  # idempotent
    assert dst.read_text().splitlines() == lines
    assert not list(dst.parent.glob("*.tmp"))


def test_find_db_seed_copy(tmp_path: Path):
    src = next(runtime.SEED_DB.glob("*.ufdb.txt"))
    dst = tmp_path / src.name
    runtime._merge_find_db(src, dst)
    assert dst.read_text().splitlines() == [l for l in src.read_text().splitlines() if "=" in l]


def test_batch_invariant_mode_turns_split_k_off_and_restores():
    """runtime.batch_invariant / split_k: split-K is off inside either block, the
    previous settings come back after it, and the split-K workspace helpers then hand out no
    workspace (so no launch is split) without asking the library."""
    from samplers_amd import runtime
    from samplers_amd.networks import layers

    assert runtime.split_k_enabled() and not runtime.batch_invariant_enabled()
    with runtime.batch_invariant():
        assert runtime.batch_invariant_enabled() and not runtime.split_k_enabled()
        assert layers._wino_workspace(None, 1, 128, 128, 8, 8, "cpu") is None
        assert layers.x6_workspace(None, 1, 64, 128, 128, "cpu") == (None, 0)
        assert layers._s2_workspace(None, 1, 128, 128, 16, 16, 0, "cpu") == (None, 0)
    assert runtime.split_k_enabled() and not runtime.batch_invariant_enabled()
    with runtime.split_k(False):
        assert not runtime.split_k_enabled() and not runtime.batch_invariant_enabled()
    assert runtime.split_k_enabled()


def test_batch_invariant_bmm_equals_torch_bmm():
    import torch

    from samplers_amd import runtime
    from samplers_amd.networks.unet2d import bmm, score_gemm

    g = torch.Generator().manual_seed(0)
    a, b = torch.randn(5, 16, 8, generator=g), torch.randn(5, 8, 12, generator=g)
    with runtime.batch_invariant():
        out = bmm(a, b)
        s = score_gemm(a, b.transpose(1, 2), 0.5, torch.empty(5, 16, 12))
    torch.testing.assert_close(out, torch.bmm(a, b))
    torch.testing.assert_close(s, 0.5 * torch.bmm(a, b))

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

"""The C-ABI library loads and exports every entry point include/samplers_hip.h declares.

No compute call is made (this runs without a GPU)."""

import ctypes
import re
from pathlib import Path

import pytest

from samplers_amd import _hip

HEADER = Path(__file__).resolve().parents[1] / "include" / "samplers_hip.h"


def declared_functions() -> list[str]:
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*[A-Za-z_][\w\s\*]*?\b(sp_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_entry_points():
    names = declared_functions()
    assert "sp_dps_residual" in names and "sp_dps_update" in names
    assert len(names) >= 10


def test_library_exports_every_declared_symbol():
    if not _hip.LIB_PATH.exists():
        pytest.fail(f"{_hip.LIB_PATH} missing: run `make` / __graft_entry__.build()")
    lib = ctypes.CDLL(str(_hip.LIB_PATH))
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header_exactly():
    assert sorted(_hip.SIGNATURES) == declared_functions()


def test_struct_layouts_match_header():
    # sp_op: 4*int32 + 2*int64 + 3 pointers + 2*int32 = 16 + 16 + 24 + 8
    assert ctypes.sizeof(_hip.SpOp) == 64
    assert ctypes.sizeof(_hip.SpDpsCoefs) == 32
    assert ctypes.sizeof(_hip.SpStepRec) == 48


def test_library_loads_without_gpu():
    lib = _hip.load_library()
    assert lib.sp_version() >= 100
    assert lib.sp_vec_partials(2048) == 1  # one partial per 2 float4 groups x 256 threads
    assert lib.sp_vec_partials(4096) == 2
    assert lib.sp_vec_partials(0) == -1


def test_x6_gemm_pack_sizes_on_the_host():
    """The bf16x6 GEMM's shape rules and packed size are host-side C (no GPU needed): the pack
    holds three bf16 terms of the [M (padded to 128)][K] operand."""
    lib = _hip.load_library()
    assert lib.sp_gemm_x6_packed_size(256, 128) == 256 * 128 * 6 // 4
    assert lib.sp_gemm_x6_supported(128, 256, 256 * 256)
    assert not lib.sp_gemm_x6_supported(128, 250, 256 * 256)  # K % 16


def test_conv_backend_selection(monkeypatch):
    """``SAMPLERS_AMD_CONV`` picks the tile per shape: the fp32 Winograd tile where its rules
    hold, the direct tile under ``direct``, MIOpen under ``miopen``."""
    from samplers_amd.networks.layers import _conv_algo, conv_backend

    lib = _hip.load_library()
    monkeypatch.setenv("SAMPLERS_AMD_CONV", "direct")
    assert conv_backend() == "direct"
    assert _conv_algo(lib, 128, 128, 256, 256, "direct") == "direct"
    assert _conv_algo(lib, 128, 128, 256, 256, "auto") == "wino"
    assert _conv_algo(lib, 512, 512, 16, 16, "auto") == "wino"
    assert _conv_algo(lib, 128, 128, 256, 256, "miopen") is None

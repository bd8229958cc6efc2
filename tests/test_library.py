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
    assert lib.sp_vec_partials(4096) == 1
    assert lib.sp_vec_partials(0) == -1


def test_x6_shape_rules_and_pack_sizes_on_the_host():
    """The bf16x6 kernels' shape rules and packed sizes are host-side C (no GPU needed): the
    direct 3x3 conv takes cout % 128, cin % 16, h % 8, w % 32; its pack holds three bf16 terms
    of the [cout (padded to 128)][9 cin] operand."""
    lib = _hip.load_library()
    assert lib.sp_conv3x3_x6_supported(128, 128, 256, 256)
    assert lib.sp_conv3x3_x6_supported(512, 256, 64, 64)
    assert not lib.sp_conv3x3_x6_supported(64, 128, 32, 32)   # cout % 128
    assert not lib.sp_conv3x3_x6_supported(128, 8, 32, 32)    # cin % 16
    assert not lib.sp_conv3x3_x6_supported(128, 128, 16, 16)  # w % 32
    assert not lib.sp_conv3x3_x6_supported(128, 128, 4, 32)   # h % 8
    assert lib.sp_conv3x3_x6_packed_size(128, 64) == 128 * 9 * 64 * 6 // 4
    assert lib.sp_conv3x3_x6_packed_size(96, 64) == 128 * 9 * 64 * 6 // 4  # rows padded
    assert lib.sp_gemm_x6_packed_size(256, 128) == 256 * 128 * 6 // 4


def test_conv_backend_selection(monkeypatch):
    """``SAMPLERS_AMD_CONV`` picks the tile per shape: x6d where the direct bf16x6 conv's rules
    hold, the fp32 Winograd tile elsewhere (the UNet's 16² / 8² levels)."""
    from samplers_amd.networks.layers import _conv_algo, conv_backend

    lib = _hip.load_library()
    monkeypatch.setenv("SAMPLERS_AMD_CONV", "x6d")
    assert conv_backend() == "x6d"
    assert _conv_algo(lib, 128, 128, 256, 256, "x6d") == "x6d"
    assert _conv_algo(lib, 512, 512, 16, 16, "x6d") == "wino"
    assert _conv_algo(lib, 128, 128, 256, 256, "auto") == "wino"
    assert _conv_algo(lib, 128, 128, 256, 256, "miopen") is None

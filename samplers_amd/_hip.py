"""ctypes binding of ``libsamplers_hip.so`` (the C ABI in ``include/samplers_hip.h``).

This is the only door from Python to the HIP kernels.  It fails loudly: if the
library is missing or a call returns a non-zero status, an exception is raised;
there is no silent fallback to eager PyTorch on the GPU path.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libsamplers_hip.so"
# the bounds-checked debug build (`make debug`; SAMPLERS_HIP_LIB=DEBUG_LIB_PATH selects it)
DEBUG_LIB_PATH = Path(__file__).resolve().parent / "lib" / "debug" / "libsamplers_hip.so"

SP_OP_IDENTITY, SP_OP_INPAINT, SP_OP_BLUR, SP_OP_MASK = 0, 1, 2, 3

_ERRORS = {-1: "invalid argument", -2: "kernel launch failed", -3: "unsupported"}


class HipLibraryError(RuntimeError):
    """The HIP library is missing, failed to load, or a call returned an error."""


class SpOp(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int32),
        ("channels", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("n", ctypes.c_int64),
        ("m", ctypes.c_int64),
        ("keep_bits", ctypes.c_void_p),
        ("word_rank", ctypes.c_void_p),
        ("taps", ctypes.c_void_p),
        ("radius", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class SpDpsCoefs(ctypes.Structure):
    _fields_ = [
        ("a", ctypes.c_float),
        ("k", ctypes.c_float),
        ("grad_scale", ctypes.c_float),
        ("c_ell", ctypes.c_float),
        ("c_s", ctypes.c_float),
        ("std", ctypes.c_float),
        ("gamma", ctypes.c_float),
        ("norm_eps", ctypes.c_float),
    ]


class SpStepRec(ctypes.Structure):
    """One record of the device-resident step schedule (include/samplers_hip.h)."""
    _fields_ = [("c", SpDpsCoefs), ("step", ctypes.c_int64), ("t", ctypes.c_int64)]


class SpEpsCoefs(ctypes.Structure):
    _fields_ = [(f, ctypes.c_float) for f in ("sqrt_oma", "oma", "sqrt_a", "sqrt_a_prev", "sigma", "dir")]


class SpAdamWCoefs(ctypes.Structure):
    _fields_ = [(f, ctypes.c_float) for f in ("decay", "beta1", "beta2", "eps", "step_size", "bc2_sqrt")]


_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_F = ctypes.c_float
_OPP = ctypes.POINTER(SpOp)
_COP = ctypes.POINTER(SpDpsCoefs)

# name -> (restype, argtypes); mirrors include/samplers_hip.h one-to-one
SIGNATURES = {
    "sp_version": (ctypes.c_int, []),
    "sp_timing_enable": (ctypes.c_int, [ctypes.c_int]),
    "sp_timing_collect": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int32),
                                         ctypes.POINTER(ctypes.c_float), ctypes.c_int]),
    "sp_timing_collect_work": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int32),
                                              ctypes.POINTER(ctypes.c_float),
                                              ctypes.POINTER(ctypes.c_double), ctypes.c_int]),
    "sp_last_error": (ctypes.c_char_p, []),
    "sp_debug_build": (ctypes.c_int, []),
    "sp_debug_violations": (_I64, [ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]),
    "sp_debug_selftest": (ctypes.c_int, [_P]),
    "sp_rsq_partials": (_I64, [_OPP]),
    "sp_vec_partials": (_I64, [_I64]),
    "sp_dps_residual": (ctypes.c_int, [_OPP, _P, _P, _P, _I64, _I64, _COP, _P, _P, _P]),
    "sp_dps_update": (ctypes.c_int, [_OPP, _P, _P, _P, _P, _P, _P, _P, _U64, _I64, _I64,
                                     _I64, _I64, _COP, _P, _P]),
    "sp_predict_x0": (ctypes.c_int, [_P, _P, _I64, _F, _F, _P, _P]),
    "sp_randn": (ctypes.c_int, [_P, _I64, _I64, _U64, _I64, _I64, _P]),
    "sp_op_apply": (ctypes.c_int, [_OPP, _P, _P, _I64, _P]),
    "sp_op_adjoint": (ctypes.c_int, [_OPP, _P, _P, _I64, _P]),
    "sp_residual_grad": (ctypes.c_int, [_P, _P, _I64, _I64, _I64, _F, _P, _P, _P]),
    "sp_psld_pixel": (ctypes.c_int, [_OPP, _P, _P, _I64, _I64, _P, _P, _P, _P]),
    "sp_sum_partials": (ctypes.c_int, [_P, _I64, _P, _P]),
    "sp_scaled_combine": (ctypes.c_int, [_P, _F, _P, _F, _P, _I64, _P, _P]),
    "sp_psld_cotangent": (ctypes.c_int, [_OPP, _P, _P, _P, _P, _F, _I64, _P, _P]),
    "sp_ddim_eps_step": (ctypes.c_int, [_P, _P, _I64, _I64, ctypes.POINTER(SpEpsCoefs), _P, _U64,
                                        _I64, _I64, _P, _P, _P, _P]),
    "sp_stochastic_resample": (ctypes.c_int, [_P, _P, _I64, _I64, _F, _F, _P, _U64, _I64, _I64, _P,
                                              _P]),
    "sp_adamw_step": (ctypes.c_int, [_P, _P, _P, _P, _I64, ctypes.POINTER(SpAdamWCoefs), _P]),
    "sp_adamw_step_until": (ctypes.c_int, [_P, _P, _P, _P, _I64, ctypes.POINTER(SpAdamWCoefs), _P,
                                           _P]),
    "sp_pixel_opt_step": (ctypes.c_int, [_OPP, _P, _P, _P, _P, _I64, _I64, _F,
                                         ctypes.POINTER(SpAdamWCoefs), _P, _P, _P]),
    "sp_opt_check": (ctypes.c_int, [_P, _I64, _F, ctypes.c_double, _P, _P, _P]),
    "sp_opt_check_plateau": (ctypes.c_int, [_P, _I64, _F, ctypes.c_double, _I64, _I64, _P, _P, _P,
                                            _P]),
    "sp_conv3x3_supported": (ctypes.c_int, [ctypes.c_int32] * 4),
    "sp_conv3x3_packed_size": (_I64, [ctypes.c_int32, ctypes.c_int32]),
    "sp_conv3x3_pack": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_conv3x3_fwd": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_conv3x3_bwd_input": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_conv3x3_thin_supported": (ctypes.c_int, [ctypes.c_int32] * 4),
    "sp_conv3x3_thin_fwd": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_conv3x3_thin_bwd_input": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                                 ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_conv3x3_s2_supported": (ctypes.c_int, [ctypes.c_int32] * 5),
    "sp_upsample2x_supported": (ctypes.c_int, [ctypes.c_int32] * 2),
    "sp_upsample2x": (ctypes.c_int, [_P, _I64, ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_upsample2x_vjp": (ctypes.c_int, [_P, _I64, ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_attention_supported": (ctypes.c_int, [_I64, _I64, _I64, ctypes.c_int32]),
    "sp_attention_fwd": (ctypes.c_int, [_P, _P, _P, _I64, _I64, ctypes.c_int32, _F, _P, _P, _P]),
    "sp_attention_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I64, _I64, ctypes.c_int32, _F,
                                        _P, _P, _P, _P, _P]),
    "sp_attention_mh_supported": (ctypes.c_int, [_I64, ctypes.c_int32, _I64, _I64, ctypes.c_int32]),
    "sp_attention6_supported": (ctypes.c_int, [_I64, ctypes.c_int32, _I64, ctypes.c_int32]),
    "sp_attention6_fwd_mh": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, _I64, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int32, _F, _P, _P, _P]),
    "sp_attention6_workspace": (_I64, [_I64, ctypes.c_int32, _I64, ctypes.c_int32]),
    "sp_attention6_fwd_ws": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, _I64, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int32, _F, _P, _P, _P, _I64, _P]),
    "sp_attention_bf16x6": (ctypes.c_int, [ctypes.c_int32]),
    "sp_attention_bf16x6_enabled": (ctypes.c_int, []),
    "sp_attention_fwd_mh": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, _I64, _I64, ctypes.c_int32,
                                           ctypes.c_int32, ctypes.c_int32, _I64, ctypes.c_int32, _F, _P, _P,
                                           _P]),
    "sp_attention_bwd_mh": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I64, ctypes.c_int32, _I64, _I64,
                                           ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _I64,
                                           ctypes.c_int32, _F, _P, _P, _P, _P, _P]),
    "sp_conv3x3_s2_pack": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_conv3x3_s2_fwd": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_conv3x3_s2_bwd_input": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_conv3x3_s2_workspace": (_I64, [_I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32]),
    "sp_conv3x3_s2_fwd_ws": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int32, _P, _P, _I64, _P]),
    "sp_conv3x3_s2_bwd_input_ws": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                  ctypes.c_int32, ctypes.c_int32, _P, _P, _I64, _P]),
    "sp_wino3x3_supported": (ctypes.c_int, [ctypes.c_int32] * 4),
    "sp_gemm_x6_supported": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, _I64]),
    "sp_gemm_x6_packed_size": (_I64, [ctypes.c_int32, ctypes.c_int32]),
    "sp_gemm_x6_pack": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_gemm_x6": (ctypes.c_int, [_P, ctypes.c_int32, _P, ctypes.c_int32, _P, _P, _P, _I64, _I64,
                                  _P, ctypes.c_int32, _P, ctypes.c_int32, _P]),
    "sp_linear_x6_supported": (ctypes.c_int, [_I64, ctypes.c_int32, ctypes.c_int32]),
    "sp_linear_x6": (ctypes.c_int, [_P, _P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_gemm_x6_layout_supported": (ctypes.c_int, [_I64, _I64, ctypes.c_int32, ctypes.c_int32]),
    "sp_gemm_x6_layout": (ctypes.c_int, [_P, _P, _P, _P, _I64, _I64, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_gemm_x6_workspace": (_I64, [_I64, _I64, ctypes.c_int32, ctypes.c_int32]),
    "sp_gemm_x6_ws": (ctypes.c_int, [_P, ctypes.c_int32, _P, ctypes.c_int32, _P, _P, _P, _I64, _I64,
                                     _P, ctypes.c_int32, _P, ctypes.c_int32, _P, _I64, _P]),
    "sp_linear_x6_ws": (ctypes.c_int, [_P, _P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32, _P, _P, _I64,
                                       _P]),
    "sp_gemm_x6_layout_ws": (ctypes.c_int, [_P, _P, _P, _P, _I64, _I64, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int32, _P, _P, _I64, _P]),
    "sp_layernorm_supported": (ctypes.c_int, [_I64, ctypes.c_int32]),
    "sp_layernorm_fwd": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, _F, _P, _P, _P, _P]),
    "sp_layernorm_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I64, ctypes.c_int32, _P, _P]),
    "sp_geglu_fwd": (ctypes.c_int, [_P, _I64, ctypes.c_int32, _P, _P]),
    "sp_geglu_bwd": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, _P, _P]),
    "sp_softmax_rows_supported": (ctypes.c_int, [_I64, ctypes.c_int32]),
    "sp_softmax_rows": (ctypes.c_int, [_P, _I64, ctypes.c_int32, _P, _P]),
    "sp_softmax_bwd_rows": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, _F, _P]),
    "sp_conv1x1_small_supported": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, _I64]),
    "sp_conv1x1_small": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32, _I64,
                                        ctypes.c_int32, _P, _P]),
    "sp_wino3x3_packed_size": (_I64, [ctypes.c_int32, ctypes.c_int32]),
    "sp_wino3x3_pack": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_wino3x3_fwd": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_wino3x3_bwd_input": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_sched_timestep": (ctypes.c_int, [_P, _P, _P, _P]),
    "sp_sched_advance": (ctypes.c_int, [_P, _P]),
    "sp_dps_residual_sched": (ctypes.c_int, [_OPP, _P, _P, _P, _I64, _I64, _P, _P, _P, _P, _P]),
    "sp_dps_update_sched": (ctypes.c_int, [_OPP, _P, _P, _P, _P, _P, _P, _U64, _I64, _I64, _I64,
                                           _P, _P, _P, _P]),
    "sp_groupnorm_workspace": (_I64, [_I64, ctypes.c_int32, _I64, ctypes.c_int32]),
    "sp_groupnorm_silu_fwd": (ctypes.c_int, [_P, _P, _P, _P, _I64, ctypes.c_int32, _I64,
                                             ctypes.c_int32, _F, ctypes.c_int32, _P, _P, _P, _P,
                                             _P]),
    "sp_groupnorm_silu_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _P, _I64, ctypes.c_int32,
                                             _I64, ctypes.c_int32, ctypes.c_int32, _P, _P, _P]),
    "sp_groupnorm_silu_fwd2": (ctypes.c_int, [_P, _P, ctypes.c_int32, _P, _P, _P, _I64,
                                              ctypes.c_int32, _I64, ctypes.c_int32, _F,
                                              ctypes.c_int32, _P, _P, _P, _P, _P, _I64, _P]),
    "sp_groupnorm_silu_bwd2": (ctypes.c_int, [_P, _P, _P, ctypes.c_int32, _P, _P, _P, _P, _P,
                                              _I64, ctypes.c_int32, _I64, ctypes.c_int32,
                                              ctypes.c_int32, _P, _P, _P, _P, _P, _P, _P, _I64,
                                              _P]),
    "sp_groupnorm_single_pass": (ctypes.c_int, [ctypes.c_int32]),
    "sp_groupnorm_team_bytes": (_I64, [_I64, ctypes.c_int32, _I64, ctypes.c_int32]),
    "sp_groupnorm_team_timeouts": (_I64, []),
    "sp_groupnorm_set_spin_limit": (ctypes.c_int, [ctypes.c_int32]),
    "sp_wino3x3_fwd_res": (ctypes.c_int, [_P, _P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_wino3x3_workspace": (_I64, [_I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                    ctypes.c_int32]),
    "sp_wino3x3_fwd_ws": (ctypes.c_int, [_P, _P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, _P, _P, _I64, _P]),
    "sp_wino3x3_bwd_input_ws": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                               ctypes.c_int32, ctypes.c_int32, _P, _P, _I64, _P]),
    "sp_wino3x3_up_supported": (ctypes.c_int, [ctypes.c_int32] * 4),
    "sp_wino3x3_fwd_up": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_wino3x3_bwd_input_pool": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                                 ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_conv3x3_bf16_supported": (ctypes.c_int, [ctypes.c_int32] * 4),
    "sp_conv3x3_bf16_packed_size": (_I64, [ctypes.c_int32, ctypes.c_int32]),
    "sp_conv3x3_bf16": (ctypes.c_int, [_P, _P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, _P, _P]),
    "sp_conv3x3_bf16_workspace": (_I64, [_I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "sp_conv3x3_bf16_ws": (ctypes.c_int, [_P, _P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int32, _P, _P, _I64, _P]),
    "sp_conv3x3_bf16_up": (ctypes.c_int, [_P, _P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int32, _P, _P]),
    "sp_pool2x2_bf16": (ctypes.c_int, [_P, _I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P]),
    "sp_layernorm_bf16_supported": (ctypes.c_int, [_I64, ctypes.c_int32]),
    "sp_layernorm_bf16_fwd": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, ctypes.c_float, _P, _P, _P, _P]),
    "sp_layernorm_bf16_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I64, ctypes.c_int32, _P, _P]),
    "sp_groupnorm_bf16_fwd_ex": (ctypes.c_int, [_P, _P, ctypes.c_int32, ctypes.c_int32, _P, _P, _P, _I64, _I64,
                                                ctypes.c_int32, ctypes.c_float, ctypes.c_int32, _P, ctypes.c_int32,
                                                _P, _P, _I64, _P]),
    "sp_groupnorm_bf16_bwd_ex": (ctypes.c_int, [_P, _P, _P, ctypes.c_int32, ctypes.c_int32, _P, _P, _P, _P, _I64,
                                                _I64, ctypes.c_int32, ctypes.c_int32, _P, _P, ctypes.c_int32, _P, _P,
                                                _P, _P, _I64, _P]),
    "sp_conv3x3_bf16_blk_supported": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "sp_conv3x3_bf16_ex": (ctypes.c_int, [_P, ctypes.c_int32, _P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int32, ctypes.c_int32, _P, _P, _I64, _P]),
    "sp_conv3x3_bf16_sc_supported": (ctypes.c_int, [ctypes.c_int32] * 6),
    "sp_conv3x3_bf16_sc_packed_size": (_I64, [ctypes.c_int32, ctypes.c_int32]),
    "sp_conv3x3_bf16_sc_workspace": (_I64, [_I64] + [ctypes.c_int32] * 5),
    "sp_conv3x3_bf16_sc": (ctypes.c_int, [_P, ctypes.c_int32, _P, _P, _P, _P, ctypes.c_int32, ctypes.c_int32, _P, _I64,
                                          ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P, _I64,
                                          _P]),
    "sp_conv3x3_bf16_gnvjp_supported": (ctypes.c_int, [_I64] + [ctypes.c_int32] * 6),
    "sp_conv3x3_bf16_gnvjp_workspace": (_I64, [_I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "sp_conv3x3_bf16_gnvjp": (ctypes.c_int, [_P, ctypes.c_int32, _P, _I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P, _P, ctypes.c_int32, _P, _P, _P, _P,
                                             ctypes.c_int32, ctypes.c_int32, _P, _P, ctypes.c_int32, _P, _P, _P, _P, _I64, _P]),
    "sp_conv3x3_bf16_gn_supported": (ctypes.c_int, [_I64] + [ctypes.c_int32] * 5),
    "sp_conv3x3_bf16_gn_workspace": (_I64, [_I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "sp_conv3x3_bf16_gn": (ctypes.c_int, [_P, ctypes.c_int32, _P, _P, _P, _I64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _P, _P, _P, _P, ctypes.c_int32,
                                          ctypes.c_float, ctypes.c_int32, _P, ctypes.c_int32, _P, _P, _I64, _P]),
    "sp_geglu_bf16_fwd": (ctypes.c_int, [_P, _I64, ctypes.c_int32, _P, _P]),
    "sp_geglu_bf16_bwd": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, _P, _P]),
    "sp_groupnorm_bf16_supported": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "sp_groupnorm_bf16_workspace": (_I64, [_I64, ctypes.c_int32, _I64]),
    "sp_groupnorm_bf16_fwd": (ctypes.c_int, [_P, _P, ctypes.c_int32, ctypes.c_int32, _P, _P, _P, _I64, _I64,
                                             ctypes.c_int32, _F, ctypes.c_int32, _P, _P, _P, _I64, _P]),
    "sp_groupnorm_bf16_bwd": (ctypes.c_int, [_P, _P, _P, ctypes.c_int32, ctypes.c_int32, _P, _P, _P, _P, _I64,
                                             _I64, ctypes.c_int32, ctypes.c_int32, _P, _P, _P, _P, _P, _P, _I64,
                                             _P]),
    "sp_attention_bf16_supported": (ctypes.c_int, [_I64, ctypes.c_int32, _I64, _I64, ctypes.c_int32]),
    "sp_attention_bf16_bwd_supported": (ctypes.c_int, [_I64, ctypes.c_int32, _I64, _I64, ctypes.c_int32]),
    "sp_attention_bf16_bwd": (ctypes.c_int, [_P, _P, _P, _P, _P, _P, _I64, ctypes.c_int32, _I64, _I64,
                                             ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _F, _P, _P, _P, _P,
                                             _P]),
    "sp_attention_bf16_fwd": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, _I64, _I64, ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _F,
                                             _P, _P, _P]),
}

_lib = None


def load_library() -> ctypes.CDLL:
    """Load (once) and type the HIP library; raise HipLibraryError if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    path = Path(os.environ.get("SAMPLERS_HIP_LIB", LIB_PATH))
    if not path.exists():
        raise HipLibraryError(
            f"{path} not found: build it with `make` (or __graft_entry__.build()) before "
            "running the GPU path; there is no CPU fallback."
        )
    # torch first: the library must bind to the HIP runtime torch already loaded
    import torch  # noqa: F401

    lib = ctypes.CDLL(str(path))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if os.environ.get("SAMPLERS_AMD_GN_SINGLE_PASS", "1") == "0":  # two-pass GroupNorm kernels
        lib.sp_groupnorm_single_pass(0)
    _lib = lib
    return lib


def check(status: int, what: str) -> None:
    if status != 0:
        detail = load_library().sp_last_error().decode(errors="replace")
        raise HipLibraryError(f"{what} failed: {_ERRORS.get(status, status)} {detail}".strip())


def debug_violations(reset: bool = True) -> tuple[int, str | None]:
    """(violated SP_DCHECK invariants since the last reset, "file-id:line" of the first) from the
    bounds-checked debug library; (0, None) under the release library.  Waits for the device."""
    site = ctypes.c_int32(0)
    n = int(load_library().sp_debug_violations(int(reset), ctypes.byref(site)))
    if n < 0:
        check(n, "sp_debug_violations")
    return n, (f"{site.value >> 16}:{site.value & 0xFFFF}" if n else None)


class solve_guard:
    """Counts, once per sampler call, the single-pass GroupNorm chunk partials that had to be
    recomputed because a team member was not resident (``sp_groupnorm_team_timeouts``).  The
    kernels recompute them exactly, so this is a diagnostic (``self.recomputed``), not an
    error.  The counter read waits for the device, so it runs at the end of a solve, never
    inside the step loop."""

    def __enter__(self):
        self.lib = load_library()
        self.before = int(self.lib.sp_groupnorm_team_timeouts())
        self.recomputed = 0
        return self

    def __exit__(self, exc_type, exc, tb):
        if exc_type is None:
            self.recomputed = int(self.lib.sp_groupnorm_team_timeouts()) - self.before
        return False


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    if not t.is_cuda:
        raise HipLibraryError("HIP path needs device tensors")
    if t.dtype != torch.float32 and t.dtype not in (torch.int32, torch.int64, torch.uint8):
        raise HipLibraryError(f"HIP path computes in fp32, got {t.dtype}")
    if not t.is_contiguous():
        raise HipLibraryError("HIP path needs contiguous tensors")
    return t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(t: torch.Tensor) -> int:
    """The handle of torch's current stream on t's device (the raw accessor: no Stream object
    per call, which at batch 1 is a measurable part of a launch's host cost)."""
    if _raw_stream is not None:
        return _raw_stream(t.get_device())
    return torch.cuda.current_stream(t.device).cuda_stream


def require_cuda(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise HipLibraryError(
            f"{what}: samplers_amd runs its hot path on MI355X (HIP); got a {t.device} tensor. "
            "The CPU restatement lives in oracle/ and is test infrastructure only."
        )

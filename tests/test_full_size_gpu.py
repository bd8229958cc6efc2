"""Parity at BASELINE.json's full sizes (3 x 256 x 256, 64 samples per GPU) for the guided
step's HIP passes, through what the domain makes checkable at that size:

* inpainting gather / scatter: bit-exact against numpy fancy indexing (the packed order of
  torch.nonzero(~mask), inpainting.py:49-50) on all 64 x 196,608 elements;
* the two fused DPS passes (residual + update, injected noise): every element against the
  float64 closed form (oracle/closed_form.py) at 2e-5 x max|ref|, and every per-sample
  ||y - A x0||^2 at 2e-5 relative;
* the blur residual pass (config 3, streaming kernel) and the update pass against the
  float64 closed form on 8 of the samples (the reflect-padded 9x9 oracle is torch-CPU);
* Philox noise: the 64-sample draw equals two 32-sample draws with sample offsets, bit for
  bit (the multi-GPU sharding invariant), and has standard-normal moments."""

import math

import numpy as np
import pytest
import torch

from oracle import blur as oblur
from oracle import closed_form
from samplers_amd import _hip
from samplers_amd.operators import GaussianBlurOperator, RandomInpaintingOperator

pytestmark = pytest.mark.gpu

SHAPE, B = (3, 256, 256), 64
N = math.prod(SHAPE)


def _stream():
    return torch.cuda.current_stream().cuda_stream


def test_inpaint_operator_full_size_bit_exact(cuda):
    op = RandomInpaintingOperator(SHAPE, 0.5, seed=1).to(cuda)
    kept = op._kept_indices.cpu().numpy()
    x = torch.randn(B, N, generator=torch.Generator().manual_seed(3))
    y = op.apply(x.reshape(B, *SHAPE).to(cuda)).cpu().numpy()
    assert np.array_equal(y, x.numpy()[:, kept])
    back = op.apply_transpose(torch.from_numpy(y).to(cuda)).reshape(B, N).cpu().numpy()
    ref = np.zeros((B, N), np.float32)
    ref[:, kept] = y
    assert np.array_equal(back, ref)


def _record_max_err(record, v, v_ref, out, out_ref):
    """max |error| / max |reference| of pass 1's v and pass 2's x' (the tests' 2e-5 bound)."""
    record("pass1_v_max_err_over_max", float(np.abs(v - v_ref).max() / np.abs(v_ref).max()), 2e-5)
    record("pass2_x_max_err_over_max", float(np.abs(out - out_ref).max() / np.abs(out_ref).max()),
           2e-5)


def test_dps_passes_full_size(cuda, parity_record):
    op = RandomInpaintingOperator(SHAPE, 0.5, seed=1).to(cuda)
    desc = op.hip_descriptor()
    m = int(desc.m)
    lib = _hip.load_library()
    g = torch.Generator().manual_seed(7)
    x, eps, w, xi = (torch.randn(B, N, generator=g) for _ in range(4))
    y = torch.randn(B, m, generator=g)
    a, k, gs = 0.31, math.sqrt(1 - 0.31**2), 400.0
    c = _hip.SpDpsCoefs(a, k, gs, 0.97, 0.11, 0.05, 1.0, 1e-9)
    P = int(lib.sp_rsq_partials(desc))
    xd, ed, yd, wd, xid = (t.to(cuda) for t in (x, eps, y, w, xi))
    v = torch.empty_like(xd)
    part = torch.empty(B, P, device=cuda)
    _hip.check(lib.sp_dps_residual(desc, xd.data_ptr(), ed.data_ptr(), yd.data_ptr(), B, 1, c,
                                   v.data_ptr(), part.data_ptr(), _stream()), "residual")
    out = torch.empty_like(xd)
    _hip.check(lib.sp_dps_update(desc, xd.data_ptr(), ed.data_ptr(), yd.data_ptr(), v.data_ptr(),
                                 wd.data_ptr(), part.data_ptr(), xid.data_ptr(), 0, 0, 0, B, 1, c,
                                 out.data_ptr(), _stream()), "update")
    apply_np, adjoint_np = closed_form.inpaint_ops(op._kept_indices.cpu().numpy(), N)
    v_ref, rsq_ref = closed_form.residual_pass(x.numpy(), eps.numpy(), y.numpy(), 1, a, k, gs,
                                               apply_np, adjoint_np)
    np.testing.assert_allclose(v.cpu().numpy(), v_ref, rtol=0, atol=2e-5 * np.abs(v_ref).max())
    np.testing.assert_allclose(part.sum(1).cpu().numpy(), rsq_ref, rtol=2e-5)
    out_ref = closed_form.update_pass(x.numpy(), eps.numpy(), v_ref, w.numpy(), rsq_ref,
                                      xi.numpy(), a, k, 0.97, 0.11, 0.05, 1.0)
    _record_max_err(parity_record, v.cpu().numpy(), v_ref, out.cpu().numpy(), out_ref)
    np.testing.assert_allclose(out.cpu().numpy(), out_ref, rtol=0,
                               atol=2e-5 * np.abs(out_ref).max())


def test_blur_passes_full_size(cuda, parity_record):
    """configs[2]'s two passes at 3 x 256 x 256, 8 samples: the streaming residual pass and
    the update pass (bridge + injected noise + guidance through the re-read v)."""
    b = 8
    op = GaussianBlurOperator(SHAPE, 9, 3.0).to(cuda)
    desc = op.hip_descriptor()
    lib = _hip.load_library()
    g = torch.Generator().manual_seed(9)
    x, eps, y, w, xi = (torch.randn(b, N, generator=g) for _ in range(5))
    a, k, gs = 0.5, math.sqrt(0.75), 400.0
    c = _hip.SpDpsCoefs(a, k, gs, 0.9, 0.2, 0.1, 1.0, 1e-9)
    part = torch.empty(b, int(lib.sp_rsq_partials(desc)), device=cuda)
    v = torch.empty(b, N, device=cuda)
    xd, ed, yd, wd, xid = (t.to(cuda) for t in (x, eps, y, w, xi))  # held: read asynchronously
    _hip.check(lib.sp_dps_residual(desc, xd.data_ptr(), ed.data_ptr(), yd.data_ptr(), b, 1, c,
                                   v.data_ptr(), part.data_ptr(), _stream()), "residual")
    out = torch.empty_like(xd)
    _hip.check(lib.sp_dps_update(desc, xd.data_ptr(), ed.data_ptr(), yd.data_ptr(), v.data_ptr(),
                                 wd.data_ptr(), part.data_ptr(), xid.data_ptr(), 0, 0, 0, b, 1, c,
                                 out.data_ptr(), _stream()), "update")
    apply_np, adjoint_np = oblur.blur_ops(SHAPE, oblur.taps(9, 3.0))
    v_ref, rsq_ref = closed_form.residual_pass(x.numpy(), eps.numpy(), y.numpy(), 1, a, k, gs,
                                               apply_np, adjoint_np)
    np.testing.assert_allclose(v.cpu().numpy(), v_ref, rtol=0, atol=2e-5 * np.abs(v_ref).max())
    np.testing.assert_allclose(part.sum(1).cpu().numpy(), rsq_ref, rtol=2e-5)
    out_ref = closed_form.update_pass(x.numpy(), eps.numpy(), v_ref, w.numpy(), rsq_ref,
                                      xi.numpy(), a, k, 0.9, 0.2, 0.1, 1.0)
    _record_max_err(parity_record, v.cpu().numpy(), v_ref, out.cpu().numpy(), out_ref)
    np.testing.assert_allclose(out.cpu().numpy(), out_ref, rtol=0,
                               atol=2e-5 * np.abs(out_ref).max())


def test_philox_full_size_shard_invariant(cuda):
    lib = _hip.load_library()
    full = torch.empty(B, N, device=cuda)
    _hip.check(lib.sp_randn(full.data_ptr(), B, N, 20260101, 999, 0, _stream()), "randn")
    halves = torch.empty_like(full)
    for b0 in (0, B // 2):
        _hip.check(lib.sp_randn(halves[b0].data_ptr(), B // 2, N, 20260101, 999, b0, _stream()),
                   "randn")
    assert torch.equal(full, halves)
    assert abs(float(full.mean())) < 1e-3 and abs(float(full.std()) - 1.0) < 1e-3

"""HIP kernels of libsamplers_hip.so against the CPU oracle (GPU)."""

import math

import numpy as np
import pytest
import torch

from oracle import blur as oblur
from oracle import closed_form, philox
from samplers_amd import _hip
from samplers_amd.operators import (GaussianBlurOperator, IdentityOperator, InpaintingOperator,
                                    get_mask_random)

pytestmark = pytest.mark.gpu


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _op_factory(kind, shape, device):
    if kind == "identity":
        return IdentityOperator(shape)
    if kind in ("inpaint", "mask"):
        m = get_mask_random(shape, 0.5, seed=3)
        return InpaintingOperator(shape, m, flatten=(kind == "inpaint")).to(device)
    if kind == "blur":
        return GaussianBlurOperator(shape, 9, 3.0).to(device)
    raise ValueError(kind)


def _np_ops(kind, op, shape):
    n = math.prod(shape)
    if kind == "identity":
        return closed_form.identity_ops()
    if kind == "inpaint":
        return closed_form.inpaint_ops(op._kept_indices.cpu().numpy(), n)
    if kind == "mask":
        return closed_form.mask_ops(~op.mask.cpu().numpy())
    return oblur.blur_ops(shape, oblur.taps(9, 3.0))


def test_library_version(cuda):
    assert _hip.load_library().sp_version() >= 100


@pytest.mark.parametrize("n", [4096, 3 * 32 * 32, 35, 196608])
def test_philox_normals_match_oracle(cuda, n):
    lib = _hip.load_library()
    b, seed, step, off = 3, 0x1234_5678_9ABC, 17, 5
    out = torch.empty(b, n, device=cuda)
    _hip.check(lib.sp_randn(out.data_ptr(), b, n, seed, step, off, _stream()), "sp_randn")
    got = out.cpu().numpy()
    for i in range(b):
        ref = philox.normals(seed, step, off + i, n)
        np.testing.assert_allclose(got[i], ref, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("shape", [(3, 32, 32), (1, 5, 7), (3, 64, 48)])
def test_inpaint_gather_scatter_bit_exact(cuda, shape):
    m = get_mask_random(shape, 0.5, seed=11)
    op = InpaintingOperator(shape, m).to(cuda)
    x = torch.randn(4, *shape)
    y = op.apply(x.to(cuda)).cpu()
    kept = torch.nonzero(~m.flatten()).squeeze(1)
    assert torch.equal(y, x.reshape(4, -1)[:, kept])
    back = op.apply_transpose(y.to(cuda)).cpu()
    ref = torch.zeros(4, math.prod(shape))
    ref[:, kept] = y
    assert torch.equal(back, ref.reshape(4, *shape))


def test_mask_operator_bit_exact(cuda):
    shape = (3, 16, 20)
    m = get_mask_random(shape, 0.3, seed=2)
    op = InpaintingOperator(shape, m, flatten=False).to(cuda)
    x = torch.randn(2, *shape)
    assert torch.equal(op.apply(x.to(cuda)).cpu(), x.masked_fill(m, 0))


@pytest.mark.parametrize("shape,ks", [((3, 32, 32), 9), ((2, 40, 70), 9), ((1, 19, 130), 5),
                                      ((3, 256, 256), 9), ((1, 17, 17), 17)])
def test_blur_forward_adjoint(cuda, shape, ks):
    op = GaussianBlurOperator(shape, ks, 3.0).to(cuda)
    k = oblur.taps(ks, 3.0)
    x = torch.randn(2, *shape, dtype=torch.float64)
    y = op.apply(x.float().to(cuda)).cpu().double()
    np.testing.assert_allclose(y.numpy(), oblur.blur(x, k).numpy(), rtol=0, atol=2e-5)
    s = torch.randn(2, *shape, dtype=torch.float64)
    at = op.apply_transpose(s.float().to(cuda)).cpu().double()
    np.testing.assert_allclose(at.numpy(), oblur.blur_adjoint(s, k).numpy(), rtol=0, atol=2e-5)


@pytest.mark.parametrize("kind", ["identity", "inpaint", "mask", "blur"])
@pytest.mark.parametrize("shape,batch,ydiv", [((3, 32, 32), 4, 1), ((3, 40, 36), 6, 3),
                                              ((1, 19, 21), 2, 2)])
def test_fused_dps_passes_match_closed_form(cuda, kind, shape, batch, ydiv):
    torch.manual_seed(0)
    op = _op_factory(kind, shape, cuda)
    apply_np, adjoint_np = _np_ops(kind, op, shape)
    lib = _hip.load_library()
    desc = op.hip_descriptor()
    n = math.prod(shape)
    m = int(desc.m)
    x = torch.randn(batch, n)
    eps = torch.randn(batch, n)
    rows = batch // ydiv
    y = torch.randn(rows, m)
    w = torch.randn(batch, n)
    xi = torch.randn(batch, n)
    a, k, gs = 0.3, math.sqrt(1 - 0.09), 400.0
    coefs = _hip.SpDpsCoefs(a, k, gs, 0.9, 0.2, 0.1, 0.05, 1e-9)
    P = lib.sp_rsq_partials(desc)
    assert P > 0
    xd, ed, yd, wd, xid = (t.to(cuda).contiguous() for t in (x, eps, y, w, xi))
    v = torch.empty_like(xd)
    part = torch.empty(batch, P, device=cuda)
    _hip.check(lib.sp_dps_residual(desc, xd.data_ptr(), ed.data_ptr(), yd.data_ptr(), batch, ydiv,
                                   coefs, v.data_ptr(), part.data_ptr(), _stream()), "residual")
    v_ref, rsq_ref = closed_form.residual_pass(x.numpy(), eps.numpy(), y.numpy(), ydiv, a, k, gs,
                                               apply_np, adjoint_np)
    scale = np.abs(v_ref).max()
    np.testing.assert_allclose(v.cpu().numpy(), v_ref, rtol=0, atol=2e-5 * scale)
    np.testing.assert_allclose(part.sum(1).cpu().numpy(), rsq_ref, rtol=2e-5)
    out_ref = closed_form.update_pass(x.numpy(), eps.numpy(), v_ref, w.numpy(), rsq_ref, xi.numpy(),
                                      a, k, 0.9, 0.2, 0.1, 0.05)
    for v_in in ([v, None] if kind != "blur" else [v]):
        out = torch.empty_like(xd)
        _hip.check(lib.sp_dps_update(desc, xd.data_ptr(), ed.data_ptr(), yd.data_ptr(),
                                     None if v_in is None else v_in.data_ptr(), wd.data_ptr(),
                                     part.data_ptr(), xid.data_ptr(), 0, 0, 0, batch, ydiv, coefs,
                                     out.data_ptr(), _stream()), "update")
        np.testing.assert_allclose(out.cpu().numpy(), out_ref, rtol=0,
                                   atol=2e-5 * np.abs(out_ref).max())


def test_update_philox_noise_is_shard_invariant(cuda):
    """Philox noise depends on (seed, step, global sample) only: two half-batch calls with
    sample offsets reproduce one full-batch call bit-for-bit."""
    shape = (3, 16, 16)
    op = IdentityOperator(shape)
    lib = _hip.load_library()
    desc = op.hip_descriptor()
    b, n = 6, math.prod(shape)
    x, eps, y, w = (torch.randn(b, n, device=cuda) for _ in range(4))
    coefs = _hip.SpDpsCoefs(0.5, 0.8, 10.0, 0.9, 0.2, 0.3, 0.1, 1e-9)
    P = lib.sp_rsq_partials(desc)
    part = torch.rand(b, P, device=cuda)
    full = torch.empty_like(x)
    _hip.check(lib.sp_dps_update(desc, x.data_ptr(), eps.data_ptr(), y.data_ptr(), None,
                                 w.data_ptr(), part.data_ptr(), None, 77, 9, 0, b, 1, coefs,
                                 full.data_ptr(), _stream()), "update")
    halves = torch.empty_like(x)
    for b0 in (0, 3):
        _hip.check(lib.sp_dps_update(desc, x[b0].data_ptr(), eps[b0].data_ptr(), y[b0].data_ptr(),
                                     None, w[b0].data_ptr(), part[b0].data_ptr(), None, 77, 9, b0, 3,
                                     1, coefs, halves[b0].data_ptr(), _stream()), "update")
    assert torch.equal(full, halves)


def test_predict_x0(cuda):
    x, e = torch.randn(5, 1001, device=cuda), torch.randn(5, 1001, device=cuda)
    out = torch.empty_like(x)
    lib = _hip.load_library()
    _hip.check(lib.sp_predict_x0(x.data_ptr(), e.data_ptr(), x.numel(), 0.25, 0.9, out.data_ptr(),
                                 _stream()), "predict")
    torch.testing.assert_close(out, (x - 0.9 * e) / 0.25, rtol=1e-6, atol=1e-6)


def test_residual_grad(cuda):
    lib = _hip.load_library()
    b, m, ydiv = 4, 5000, 2
    y, z = torch.randn(b // ydiv, m, device=cuda), torch.randn(b, m, device=cuda)
    g = torch.empty_like(z)
    P = lib.sp_vec_partials(m)
    part = torch.empty(b, P, device=cuda)
    _hip.check(lib.sp_residual_grad(y.data_ptr(), z.data_ptr(), b, m, ydiv, 3.0, g.data_ptr(),
                                    part.data_ptr(), _stream()), "residual_grad")
    r = y.repeat_interleave(ydiv, 0) - z
    torch.testing.assert_close(g, 3.0 * r)
    torch.testing.assert_close(part.sum(1), (r * r).sum(1), rtol=1e-5, atol=1e-3)


def test_bad_arguments_return_einval(cuda):
    lib = _hip.load_library()
    desc = IdentityOperator((3, 4, 4)).hip_descriptor()
    coefs = _hip.SpDpsCoefs()
    assert lib.sp_dps_residual(desc, None, None, None, 1, 1, coefs, None, None, _stream()) == -1
    bad = _hip.SpOp()
    bad.kind = 42
    assert lib.sp_rsq_partials(bad) == -1
    with pytest.raises(_hip.HipLibraryError):
        _hip.check(-1, "x")


def test_dispatch_packet_timing(cuda):
    from samplers_amd.samplers.dps import KernelTimer

    lib = _hip.load_library()
    op = IdentityOperator((3, 64, 64))
    desc = op.hip_descriptor()
    b, n = 8, 3 * 64 * 64
    x, eps, y, w = (torch.randn(b, n, device=cuda) for _ in range(4))
    v = torch.empty_like(x)
    P = lib.sp_rsq_partials(desc)
    part = torch.empty(b, P, device=cuda)
    c = _hip.SpDpsCoefs(0.5, 0.8, 10.0, 0.9, 0.2, 0.3, 0.1, 1e-9)
    timer = KernelTimer()
    try:
        for _ in range(3):
            with timer.span("dps_residual", b):
                _hip.check(lib.sp_dps_residual(desc, x.data_ptr(), eps.data_ptr(), y.data_ptr(), b, 1,
                                               c, v.data_ptr(), part.data_ptr(), _stream()), "k1")
            with timer.span("dps_update", b):
                _hip.check(lib.sp_dps_update(desc, x.data_ptr(), eps.data_ptr(), y.data_ptr(),
                                             v.data_ptr(), w.data_ptr(), part.data_ptr(), None, 1, 2,
                                             0, b, 1, c, x.data_ptr(), _stream()), "k2")
        s = timer.summary()
    finally:
        timer.close()
    assert s["dps_residual"]["count"] == 3 and s["dps_update"]["count"] == 3
    assert 0 < s["dps_residual"]["ms"] < 100 and 0 < s["dps_update"]["ms"] < 100
    assert s["dps_update"]["samples"] == 3 * b


@pytest.mark.parametrize("shape,ks,batch,ydiv,asym", [
    ((3, 32, 256), 9, 2, 1, False), ((2, 64, 256), 9, 3, 3, False), ((1, 96, 256), 5, 2, 1, False),
    ((3, 32, 256), 3, 1, 1, False), ((1, 64, 256), 7, 2, 2, False), ((3, 256, 256), 9, 2, 1, False),
    ((2, 96, 256), 9, 2, 1, True), ((1, 64, 256), 5, 1, 1, True)])
def test_blur_streaming_residual_pass(cuda, shape, ks, batch, ydiv, asym):
    """The streaming blur pass (256-column planes, one wave per row segment, odd segments
    swept bottom-up) against the closed form with the fold-corrected reflect adjoint: every
    radius it serves, one and several segments per plane, shared observations, and
    asymmetric taps (which a mirrored sweep must reverse in its vertical passes)."""
    torch.manual_seed(1)
    op = GaussianBlurOperator(shape, ks, 3.0).to(cuda)
    k1d = oblur.taps(ks, 3.0)
    if asym:
        k1d = np.random.default_rng(ks).uniform(0.05, 1.0, ks).astype(np.float32)
        k1d /= k1d.sum()
        op.taps.copy_(torch.from_numpy(k1d))
    apply_np, adjoint_np = oblur.blur_ops(shape, k1d)
    lib = _hip.load_library()
    desc = op.hip_descriptor()
    n = math.prod(shape)
    P = lib.sp_rsq_partials(desc)
    assert P == shape[0] * (shape[1] // 32)  # streaming layout: one partial per segment
    x, eps = torch.randn(batch, n), torch.randn(batch, n)
    y = torch.randn(batch // ydiv, n)
    a, k, gs = 0.3, math.sqrt(1 - 0.09), 400.0
    coefs = _hip.SpDpsCoefs(a, k, gs, 0.9, 0.2, 0.1, 0.05, 1e-9)
    xd, ed, yd = (t.to(cuda).contiguous() for t in (x, eps, y))
    v = torch.full_like(xd, float("nan"))
    part = torch.full((batch, P), float("nan"), device=cuda)
    _hip.check(lib.sp_dps_residual(desc, xd.data_ptr(), ed.data_ptr(), yd.data_ptr(), batch, ydiv,
                                   coefs, v.data_ptr(), part.data_ptr(), _stream()), "residual")
    v_ref, rsq_ref = closed_form.residual_pass(x.numpy(), eps.numpy(), y.numpy(), ydiv, a, k, gs,
                                               apply_np, adjoint_np)
    np.testing.assert_allclose(v.cpu().numpy(), v_ref, rtol=0, atol=2e-5 * np.abs(v_ref).max())
    np.testing.assert_allclose(part.sum(1).cpu().numpy(), rsq_ref, rtol=2e-5)

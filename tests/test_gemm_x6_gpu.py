"""The bf16x6 1x1-conv GEMM (csrc/sp_gemm_x6.hip) against fp64: Y = W cat(x1, x2) (+ bias)
(+ residual), and the two-output transposed form of the UNet shortcut's input VJP.

Tolerance: relative L2 <= 1.5x the error of torch's fp32 GEMM on the same data, and < 1e-6
(three exact bf16 terms per operand, six partial products, fp32 accumulation)."""

import pytest
import torch

from samplers_amd import _hip

pytestmark = pytest.mark.gpu

CASES = [  # n, c1, c2, o1, o2, h, w
    (2, 64, 64, 128, 0, 16, 16),
    (1, 128, 0, 128, 0, 32, 32),
    (2, 128, 0, 64, 64, 16, 32),
    (3, 96, 32, 256, 0, 16, 16),
    (2, 128, 0, 96, 32, 32, 16),
]


def _rel(a, b):
    return float((a.double().cpu() - b).norm() / b.norm())


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("extras", [False, True])
def test_gemm_x6_matches_fp64(cuda, case, extras):
    n, c1, c2, o1, o2, h, w = case
    lib = _hip.load_library()
    k, m, hw = c1 + c2, o1 + o2, h * w
    assert lib.sp_gemm_x6_supported(m, k, hw)
    g = torch.Generator().manual_seed(sum(case))
    x1 = torch.randn(n, c1, h, w, generator=g)
    x2 = torch.randn(n, c2, h, w, generator=g) if c2 else None
    W = torch.randn(m, k, generator=g) * k ** -0.5
    bias = torch.randn(m, generator=g) if extras else None
    res = torch.randn(n, o1, h, w, generator=g) if extras and not o2 else None
    x = x1 if x2 is None else torch.cat([x1, x2], 1)
    ref = torch.einsum("ok,nkp->nop", W.double(), x.reshape(n, k, hw).double())
    if bias is not None:
        ref = ref + bias.double()[None, :, None]
    if res is not None:
        ref = ref + res.reshape(n, o1, hw).double()
    t32 = torch.einsum("ok,nkp->nop", W.to(cuda), x.reshape(n, k, hw).to(cuda))
    if bias is not None:
        t32 = t32 + bias.to(cuda)[None, :, None]
    if res is not None:
        t32 = t32 + res.reshape(n, o1, hw).to(cuda)

    st = torch.cuda.current_stream().cuda_stream
    wg = W.to(cuda)
    wp = torch.empty(int(lib.sp_gemm_x6_packed_size(m, k)), device=cuda)
    _hip.check(lib.sp_gemm_x6_pack(wg.data_ptr(), m, k, 0, wp.data_ptr(), st), "pack")
    x1g = x1.to(cuda)
    x2g = None if x2 is None else x2.to(cuda)
    bg = None if bias is None else bias.to(cuda)  # held by name for the call
    rg = None if res is None else res.to(cuda)
    y1 = torch.full((n, o1, h, w), float("nan"), device=cuda)
    y2 = torch.full((n, o2, h, w), float("nan"), device=cuda) if o2 else None
    _hip.check(lib.sp_gemm_x6(x1g.data_ptr(), c1, None if x2g is None else x2g.data_ptr(), c2,
                              wp.data_ptr(), None if bg is None else bg.data_ptr(),
                              None if rg is None else rg.data_ptr(), n, hw, y1.data_ptr(),
                              o1, None if y2 is None else y2.data_ptr(), o2, st), "sp_gemm_x6")
    torch.cuda.synchronize()
    y = y1.reshape(n, o1, hw) if y2 is None else torch.cat([y1, y2], 1).reshape(n, m, hw)
    assert torch.isfinite(y).all()
    e6, e32 = _rel(y, ref), _rel(t32, ref)
    assert e6 <= 1.5 * e32 + 1e-9 and e6 < 1e-6, (e6, e32)


def test_gemm_x6_transposed_pack_is_the_vjp(cuda):
    """trans = 1 packs W stored [K][M]: the shortcut's input VJP W^T dy into two outputs."""
    lib = _hip.load_library()
    n, co, c1, c2, h, w = 2, 128, 64, 64, 16, 16
    g = torch.Generator().manual_seed(3)
    W = torch.randn(co, c1 + c2, generator=g) * 0.1
    dy = torch.randn(n, co, h, w, generator=g)
    ref = torch.einsum("ok,nop->nkp", W.double(), dy.reshape(n, co, h * w).double())
    st = torch.cuda.current_stream().cuda_stream
    wg = W.to(cuda)
    wp = torch.empty(int(lib.sp_gemm_x6_packed_size(c1 + c2, co)), device=cuda)
    _hip.check(lib.sp_gemm_x6_pack(wg.data_ptr(), c1 + c2, co, 1, wp.data_ptr(), st), "pack")
    d1 = torch.empty(n, c1, h, w, device=cuda)
    d2 = torch.empty(n, c2, h, w, device=cuda)
    dyg = dy.to(cuda)
    _hip.check(lib.sp_gemm_x6(dyg.data_ptr(), co, None, 0, wp.data_ptr(), None, None, n, h * w,
                              d1.data_ptr(), c1, d2.data_ptr(), c2, st), "sp_gemm_x6")
    torch.cuda.synchronize()
    got = torch.cat([d1, d2], 1).reshape(n, c1 + c2, h * w)
    assert _rel(got, ref) < 1e-6


def test_gemm_x6_rejects_bad_shapes(cuda):
    lib = _hip.load_library()
    assert not lib.sp_gemm_x6_supported(96, 64, 256)     # M % 128
    assert not lib.sp_gemm_x6_supported(128, 24, 256)    # K % 16
    assert not lib.sp_gemm_x6_supported(128, 64, 200)    # HW % 256
    x = torch.empty(1, device=cuda)
    # residual with a split output is refused
    assert lib.sp_gemm_x6(x.data_ptr(), 64, None, 0, x.data_ptr(), None, x.data_ptr(), 1, 256,
                          x.data_ptr(), 64, x.data_ptr(), 64, 0) != 0


# --- token-major mode: nn.Linear on [tokens][features] (sp_linear_x6) ----------------------

LINEAR_CASES = [  # tokens, k, m
    (512, 320, 320),
    (256, 768, 320),
    (1024, 64, 96),
    (768, 512, 1280),
]


@pytest.mark.parametrize("case", LINEAR_CASES)
@pytest.mark.parametrize("extras", [False, True])
def test_linear_x6_matches_fp64(cuda, case, extras):
    t, k, m = case
    lib = _hip.load_library()
    assert lib.sp_linear_x6_supported(t, k, m)
    g = torch.Generator().manual_seed(t + k + m)
    x = torch.randn(t, k, generator=g)
    W = torch.randn(m, k, generator=g) * k ** -0.5
    bias = torch.randn(m, generator=g) if extras else None
    res = torch.randn(t, m, generator=g) if extras else None
    ref = x.double() @ W.double().t()
    if bias is not None:
        ref = ref + bias.double()
    if res is not None:
        ref = ref + res.double()
    t32 = torch.nn.functional.linear(x.to(cuda), W.to(cuda), None if bias is None else bias.to(cuda))
    if res is not None:
        t32 = t32 + res.to(cuda)
    st = torch.cuda.current_stream().cuda_stream
    wg = W.to(cuda)
    wp = torch.empty(int(lib.sp_gemm_x6_packed_size(m, k)), device=cuda)
    _hip.check(lib.sp_gemm_x6_pack(wg.data_ptr(), m, k, 0, wp.data_ptr(), st), "pack")
    xg = x.to(cuda)
    bg = None if bias is None else bias.to(cuda)  # held by name for the call
    rg = None if res is None else res.to(cuda)
    y = torch.full((t, m), float("nan"), device=cuda)
    _hip.check(lib.sp_linear_x6(xg.data_ptr(), wp.data_ptr(), None if bg is None else bg.data_ptr(),
                                None if rg is None else rg.data_ptr(), t, k, m, y.data_ptr(), st),
               "sp_linear_x6")
    torch.cuda.synchronize()
    assert torch.isfinite(y).all()
    e6, e32 = _rel(y, ref), _rel(t32, ref)
    assert e6 <= 1.5 * e32 + 1e-9 and e6 < 1e-6, (e6, e32)


def test_linear_x6_input_vjp(cuda):
    """dx = dy W through a W^T pack (trans = 1): the Linear's input VJP."""
    lib = _hip.load_library()
    t, k, m = 512, 320, 640
    g = torch.Generator().manual_seed(11)
    W = torch.randn(m, k, generator=g) * 0.05
    dy = torch.randn(t, m, generator=g)
    ref = dy.double() @ W.double()
    st = torch.cuda.current_stream().cuda_stream
    wg = W.to(cuda)
    wt = torch.empty(int(lib.sp_gemm_x6_packed_size(k, m)), device=cuda)
    _hip.check(lib.sp_gemm_x6_pack(wg.data_ptr(), k, m, 1, wt.data_ptr(), st), "pack")
    dx = torch.empty(t, k, device=cuda)
    dyg = dy.to(cuda)
    _hip.check(lib.sp_linear_x6(dyg.data_ptr(), wt.data_ptr(), None, None, t, m, k, dx.data_ptr(), st),
               "sp_linear_x6")
    torch.cuda.synchronize()
    assert _rel(dx, ref) < 1e-6


# --- split-K (the _ws entry points): under-filled launches cut K into parts ---------------

SPLIT_CASES = [  # kind, n, hw, k, m, o2, in_tm, out_tm, extras
    ("gemm", 2, 256, 128, 128, 0, 0, 0, True),
    ("gemm", 1, 256, 512, 256, 0, 0, 0, True),
    ("gemm", 2, 512, 128, 128, 64, 0, 0, True),     # two outputs (the shortcut VJP form)
    ("linear", 1, 256, 512, 320, 0, 1, 1, True),
    ("linear", 1, 512, 768, 1280, 0, 1, 1, False),
    ("layout", 1, 256, 512, 512, 0, 1, 0, True),    # the 16² attention's proj_out at batch 1
    ("layout", 2, 256, 320, 640, 0, 0, 1, True),
    ("layout", 1, 256, 256, 96, 0, 1, 1, False),
]


@pytest.mark.parametrize("case", SPLIT_CASES)
def test_x6_split_k_workspace(cuda, case):
    """A launch whose tiles fill less than half the CUs splits K (sp_gemm_x6_workspace > 0):
    against fp64 within the unsplit bound, bitwise repeatable, and equal to the unsplit launch
    to fp32 rounding; a NULL workspace runs unsplit."""
    kind, n, hw, k, m, o2, in_tm, out_tm, extras = case
    lib = _hip.load_library()
    nb = int(lib.sp_gemm_x6_workspace(n, hw, k, m))
    assert nb > 0
    o1 = m - o2
    g = torch.Generator().manual_seed(n + hw + k + m)
    x = torch.randn(n, k, hw, generator=g)                      # [n][k][hw]
    W = torch.randn(m, k, generator=g) * k ** -0.5
    bias = torch.randn(m, generator=g) if extras else None
    res = torch.randn(n, o1, hw, generator=g) if extras and not o2 else None
    ref = torch.einsum("ok,nkp->nop", W.double(), x.double())  # [n][m][hw]
    t32 = torch.einsum("ok,nkp->nop", W.to(cuda), x.to(cuda))
    if bias is not None:
        ref, t32 = ref + bias.double()[None, :, None], t32 + bias.to(cuda)[None, :, None]
    if res is not None:
        ref, t32 = ref + res.double(), t32 + res.to(cuda)
    tm = lambda a: a.transpose(1, 2).reshape(n * hw, a.shape[1]).contiguous()  # noqa: E731
    st = torch.cuda.current_stream().cuda_stream
    wp = torch.empty(int(lib.sp_gemm_x6_packed_size(m, k)), device=cuda)
    wg = W.to(cuda)
    _hip.check(lib.sp_gemm_x6_pack(wg.data_ptr(), m, k, 0, wp.data_ptr(), st), "pack")
    xg = (tm(x) if in_tm else x).to(cuda)
    bg = None if bias is None else bias.to(cuda)
    rg = None if res is None else (tm(res) if out_tm else res).to(cuda)
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    ws = torch.empty(nb // 4, device=cuda)

    def run(ws_ptr, ws_bytes):
        if kind == "gemm":
            y1 = torch.full((n, o1, hw), float("nan"), device=cuda)
            y2 = torch.full((n, o2, hw), float("nan"), device=cuda) if o2 else None
            _hip.check(lib.sp_gemm_x6_ws(xg.data_ptr(), k, None, 0, wp.data_ptr(), p(bg), p(rg), n, hw,
                                         y1.data_ptr(), o1, p(y2), o2, ws_ptr, ws_bytes, st), "sp_gemm_x6_ws")
            return y1 if y2 is None else torch.cat([y1, y2], 1)
        y = torch.full((n * hw, m) if out_tm else (n, m, hw), float("nan"), device=cuda)
        if kind == "linear":
            _hip.check(lib.sp_linear_x6_ws(xg.data_ptr(), wp.data_ptr(), p(bg), p(rg), n * hw, k, m,
                                           y.data_ptr(), ws_ptr, ws_bytes, st), "sp_linear_x6_ws")
        else:
            _hip.check(lib.sp_gemm_x6_layout_ws(xg.data_ptr(), wp.data_ptr(), p(bg), p(rg), n, hw, k, m,
                                                in_tm, out_tm, y.data_ptr(), ws_ptr, ws_bytes, st),
                       "sp_gemm_x6_layout_ws")
        return y.reshape(n, hw, m).transpose(1, 2) if out_tm else y

    ys = [run(ws.data_ptr(), nb) for _ in range(3)]
    y0 = run(None, 0)                       # unsplit
    torch.cuda.synchronize()
    assert torch.isfinite(ys[0]).all()
    assert all(torch.equal(ys[0], y) for y in ys[1:])
    e6, e32 = _rel(ys[0], ref), _rel(t32, ref)
    assert e6 <= 1.5 * e32 + 1e-9 and e6 < 1e-6, (e6, e32)
    assert _rel(ys[0], y0.double().cpu()) < 3e-7

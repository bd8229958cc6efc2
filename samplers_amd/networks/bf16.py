"""The priors' layers at bf16 — the reference's reduced-precision runs on this project's kernels.

The reference's adapters take any ``torch_dtype`` (``/root/reference/samplers/networks/diffusers/
stable_diffusion.py:90-101``, ``ddpm.py:23-34``) and its PSLD driver runs SD 1.5 in bf16
(``scripts/run_psld.py:14-20``).  With a bf16 network the layers of ``unet2d.py``,
``unet2d_condition.py`` and ``vae.py`` dispatch here on the device:

* activations are channels-last bf16 (``torch.channels_last``: the memory is [n][h][w][c]);
  the transformer blocks' token rows ([b][h w][c]) are then views, no transposes;
* 3x3 convolutions (stride 1; the stride-2 downsamplers at full resolution read at every other
  position) and their input VJPs on ``sp_conv3x3_bf16`` (implicit GEMM on the bf16 MFMAs, fp32
  accumulation, bias and residual in the epilogue);
* GroupNorm(+time-embedding bias)(+SiLU) and its input VJP on ``sp_groupnorm_bf16_fwd/bwd``
  (fp32 statistics);
* the SD UNet's self- and cross-attention on ``sp_attention_bf16_fwd`` / ``_bwd`` (flash-style,
  scores never in HBM, either direction; head dim 160 — the 16² / 8² levels — takes the VJP on
  the exact-fp32 fused kernels with the operands widened);
* the transformers' GEGLU gate and LayerNorm, forward and VJP, on ``sp_geglu_bf16_*`` /
  ``sp_layernorm_bf16_*`` (the LayerNorm VJP adds the residual branch's gradient handed over by the
  residual linear: no autograd accumulation adds in x + f(norm(x)));
* 1x1 convolutions and linears are bf16 GEMMs (hipBLASLt through ``F.linear``); the d = 512
  single-head attention (score matrix kept) is torch bf16 ops.

Semantics follow PyTorch's bf16 modules (fp32 accumulation / statistics, one rounding to bf16
per layer output), which is what the reference computes in bf16.  Every entry here raises
``HipLibraryError`` when the library is missing: there is no silent CPU fallback.
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from .. import _hip

BF16 = torch.bfloat16
CL = torch.channels_last


def is_bf16_device(x: Tensor) -> bool:
    return x.is_cuda and x.dtype == BF16


def nhwc(t: Tensor) -> Tensor:
    """``t`` (n, c, h, w) with [n][h][w][c] memory."""
    return t if t.is_contiguous(memory_format=CL) else t.contiguous(memory_format=CL)


def _p(t: Tensor | None, *, cl: bool = True) -> int | None:
    """Device pointer of a bf16 tensor laid out as the kernels read it (channels-last for 4-d)."""
    if t is None:
        return None
    if not t.is_cuda or t.dtype != BF16:
        raise _hip.HipLibraryError(f"bf16 path needs bf16 device tensors, got {t.dtype} on {t.device}")
    ok = t.is_contiguous(memory_format=CL) if (cl and t.dim() == 4) else t.is_contiguous()
    if not ok:
        raise _hip.HipLibraryError("bf16 path needs channels-last / contiguous tensors")
    return t.data_ptr()


def _f32(t: Tensor | None) -> Tensor | None:
    return None if t is None else t.detach().to(torch.float32).contiguous()


def _cached(module: nn.Module, name: str, key, build):
    cache = module.__dict__.setdefault("_bf16_cache", {})
    hit = cache.get(name)
    if hit is None or hit[0] != key:
        with torch.no_grad():
            hit = (key, build())
        cache[name] = hit
    return hit[1]


def _wkey(*ts: Tensor | None):
    return tuple((None if t is None else (t.data_ptr(), t._version, t.device, t.dtype)) for t in ts)


# ---------------------------------------------------------------------------------------------
# 3x3 convolution
# ---------------------------------------------------------------------------------------------

def _ceil(a: int, b: int) -> int:
    return -(-a // b) * b


def conv_pack(module: nn.Module, vjp: bool) -> Tensor:
    """``module``'s 3x3 weights as sp_conv3x3_bf16 reads them: [co block of 64][ci block of 16]
    [tap][64 co][16 ci] bf16, zero-padded; ``vjp``: the pack of W'[ci][co][2-ky][2-kx]."""
    w = module.weight

    def build():
        wt = w.detach()
        if vjp:
            wt = wt.transpose(0, 1).flip(2, 3)
        co, ci = wt.shape[:2]
        cop, cip = _ceil(co, 64), _ceil(ci, 16)
        wp = torch.zeros(cop, cip, 3, 3, device=w.device, dtype=torch.float32)
        wp[:co, :ci] = wt.float()
        wp = wp.reshape(cop // 64, 64, cip // 16, 16, 9).permute(0, 2, 4, 1, 3).contiguous()
        return wp.to(BF16)

    return _cached(module, f"pack{int(vjp)}", _wkey(w), build)


def _bias_f32(module: nn.Module, bias: Tensor | None) -> Tensor | None:
    if bias is None:
        return None
    return _cached(module, f"bias{id(bias)}", _wkey(bias), lambda: bias.detach().float().contiguous())


def _pad_channels(x: Tensor, c: int) -> Tensor:
    """x (n, c0, h, w) zero-padded to c channels (differentiable; channels-last result)."""
    if x.shape[1] == c:
        return nhwc(x)
    n, c0, h, w = x.shape
    out = torch.empty(n, c, h, w, device=x.device, dtype=x.dtype, memory_format=CL).zero_()
    out[:, :c0] = x  # autograd: the gradient of x is the first c0 channels
    return out


def _conv_launch(x: Tensor, pack: Tensor, bias: Tensor | None, res: Tensor | None, cout: int,
                 shape: tuple | None = None) -> Tensor:
    """conv3x3 on the bf16 tile; ``shape`` given: x is a flat buffer in the channel-blocked layout
    [n][cin / 16][h][w][16] of that (n, cin, h, w) (``blocked_ok``), else a channels-last tensor."""
    from ..runtime import split_k_enabled
    from .layers import _query

    lib = _hip.load_library()
    n, cin, h, w = x.shape if shape is None else shape
    y = torch.empty(n, cout, h, w, device=x.device, dtype=BF16, memory_format=CL)
    # split-K where the tiles leave CUs idle (torch's caching allocator on the launch stream)
    nb = _query("sp_conv3x3_bf16_workspace", n, cin, cout, h, w) if split_k_enabled() else 0
    ws = torch.empty(max(nb // 4, 1), device=x.device, dtype=torch.float32)
    _hip.check(lib.sp_conv3x3_bf16_ex(_p(x, cl=shape is None), 0 if shape is None else 1, _p(pack, cl=False),
                                      None if bias is None else bias.data_ptr(), _p(res), n, cin, cout, h, w, _p(y),
                                      ws.data_ptr() if nb else None, nb, _hip.stream_of(x)), "sp_conv3x3_bf16_ex")
    return y


def shortcut_pack(block: nn.Module) -> Tensor:
    """conv_shortcut's [cout][cs] weights as sp_conv3x3_bf16_sc reads them: [co block of 64][cs / 16]
    [64 co][16 ci] bf16, rows past cout zero."""
    w = block.conv_shortcut.weight

    def build():
        co, cs = w.shape[0], w.shape[1]
        cop = _ceil(co, 64)
        wp = torch.zeros(cop, cs, device=w.device, dtype=torch.float32)
        wp[:co] = w.detach().reshape(co, cs).float()
        return wp.reshape(cop // 64, 64, cs // 16, 16).permute(0, 2, 1, 3).contiguous().to(BF16)

    return _cached(block.conv_shortcut, "scpack", _wkey(w), build)


def _sc_bias(block: nn.Module) -> Tensor | None:
    """conv2's bias + conv_shortcut's (fp32): the bias of the fused conv2 + shortcut launch."""
    b2, bs = block.conv2.bias, block.conv_shortcut.bias
    if b2 is None and bs is None:
        return None
    return _cached(block.conv_shortcut, "scbias", _wkey(b2, bs),
                   lambda: ((b2.detach().float() if b2 is not None else 0) + (bs.detach().float() if bs is not None else 0)).contiguous())


def sc_ok(cout: int, c1: int, c2: int, h: int, w: int) -> bool:
    """Whether conv2 + the 1x1 shortcut run as one sp_conv3x3_bf16_sc launch
    (``SAMPLERS_AMD_BF16_SC=0``: shortcut GEMMs + residual epilogue, for A/B)."""
    import os

    from .layers import _query

    return (os.environ.get("SAMPLERS_AMD_BF16_SC", "1") != "0"
            and bool(_query("sp_conv3x3_bf16_sc_supported", cout, cout, c1, c2, h, w)))


def _conv_sc_launch(z: Tensor, pack: Tensor, bias: Tensor | None, x1: Tensor, x2: Tensor | None, wsp: Tensor, cout: int,
                    shape: tuple | None = None) -> Tensor:
    """conv3x3(z) + conv1x1(cat(x1, x2)) + bias on sp_conv3x3_bf16_sc (``shape``: z flat channel-blocked)."""
    from ..runtime import split_k_enabled
    from .layers import _query

    lib = _hip.load_library()
    n, cin, h, w = z.shape if shape is None else shape
    c1, c2 = x1.shape[1], (0 if x2 is None else x2.shape[1])
    y = torch.empty(n, cout, h, w, device=x1.device, dtype=BF16, memory_format=CL)
    nb = _query("sp_conv3x3_bf16_sc_workspace", n, cin, c1 + c2, cout, h, w) if split_k_enabled() else 0
    ws = torch.empty(max(nb // 4, 1), device=x1.device, dtype=torch.float32)
    _hip.check(lib.sp_conv3x3_bf16_sc(_p(z, cl=shape is None), 0 if shape is None else 1, _p(pack, cl=False),
                                      None if bias is None else bias.data_ptr(), _p(x1), _p(x2), c1, c2,
                                      _p(wsp, cl=False), n, cin, cout, h, w, _p(y), ws.data_ptr() if nb else None, nb,
                                      _hip.stream_of(x1)), "sp_conv3x3_bf16_sc")
    return y


def blocked_ok(cin: int, cout: int, h: int, w: int) -> bool:
    """Whether a conv's input can be handed over channel-blocked ([n][cin/16][h][w][16]: each 16-channel
    stage of the tile then reads whole cache lines instead of 32 bytes of every pixel's row);
    ``SAMPLERS_AMD_BF16_BLOCKED=0`` keeps NHWC (A/B)."""
    import os

    return (cin % 16 == 0 and os.environ.get("SAMPLERS_AMD_BF16_BLOCKED", "1") != "0"
            and bool(_hip.load_library().sp_conv3x3_bf16_blk_supported(cin, cout, h, w)))


class _ConvBf16Fn(torch.autograd.Function):
    """conv3x3(x) + bias (+ res) on sp_conv3x3_bf16; the input VJP on the same kernel with the
    flipped / transposed pack (weights frozen); the residual's gradient is dy itself."""

    @staticmethod
    def forward(ctx, x, res, module, bias):
        ctx.module, ctx.cin, ctx.has_res = module, x.shape[1], res is not None
        return _conv_launch(x, conv_pack(module, False), bias, res, module.weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        module = ctx.module
        cout = module.weight.shape[0]
        dx = None
        if ctx.needs_input_grad[0]:
            d = _pad_channels(dy.to(BF16), _ceil(cout, 16))
            dx = _conv_launch(d, conv_pack(module, True), None, None, ctx.cin)
        dres = dy if (ctx.has_res and ctx.needs_input_grad[1]) else None
        return dx, dres, None, None


def conv_supported(module: nn.Module, x: Tensor) -> bool:
    if not (is_bf16_device(x) and x.dim() == 4) or module.weight.requires_grad:
        return False
    if tuple(module.weight.shape[2:]) != (3, 3):
        return False
    n, cin, h, w = x.shape
    return bool(_hip.load_library().sp_conv3x3_bf16_supported(_ceil(cin, 16), module.weight.shape[0], h, w))


def conv3x3(module: nn.Module, x: Tensor, res: Tensor | None = None, bias: Tensor | None = None) -> Tensor:
    """``module(x)`` (3x3, stride 1, padding 1) + ``res`` on the bf16 tile; ``bias`` overrides the
    module's.  Inputs with fewer than 16-multiple channels (conv_in: 3 / 4) are zero-padded."""
    cin = x.shape[1]
    xp = _pad_channels(x, _ceil(cin, 16))
    b = module.bias if bias is None else bias
    r = None if res is None else nhwc(res.to(BF16))
    return _ConvBf16Fn.apply(xp, r, module, _bias_f32(module, b))


class _UpConvBf16Fn(torch.autograd.Function):
    """conv3x3(upsample_nearest2x(x)) (diffusers Upsample2D) on sp_conv3x3_bf16_up: the patch
    reads the half-resolution pixel, the upsampled tensor is never written; VJP: the
    full-resolution input VJP, then the 2 x 2 block sums (sp_pool2x2_bf16)."""

    @staticmethod
    def forward(ctx, x, module, bias):
        lib = _hip.load_library()
        n, cin, h, w = x.shape
        cout = module.weight.shape[0]
        ctx.module, ctx.xs = module, x.shape
        y = torch.empty(n, cout, 2 * h, 2 * w, device=x.device, dtype=BF16, memory_format=CL)
        _hip.check(lib.sp_conv3x3_bf16_up(_p(x), _p(conv_pack(module, False), cl=False),
                                          None if bias is None else bias.data_ptr(), None, n, cin, cout, 2 * h,
                                          2 * w, _p(y), _hip.stream_of(x)), "sp_conv3x3_bf16_up")
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _hip.load_library()
        module = ctx.module
        n, cin, h, w = ctx.xs
        cout = module.weight.shape[0]
        d = _pad_channels(dy.to(BF16), _ceil(cout, 16))
        full = _conv_launch(d, conv_pack(module, True), None, None, cin)
        dx = torch.empty(n, cin, h, w, device=dy.device, dtype=BF16, memory_format=CL)
        _hip.check(lib.sp_pool2x2_bf16(_p(full), n, cin, 2 * h, 2 * w, _p(dx), _hip.stream_of(dy)),
                   "sp_pool2x2_bf16")
        return dx, None, None


def upsample_conv_supported(module: nn.Module, x: Tensor) -> bool:
    return (is_bf16_device(x) and x.dim() == 4 and x.shape[1] % 16 == 0 and not module.weight.requires_grad
            and bool(_hip.load_library().sp_conv3x3_bf16_supported(x.shape[1], module.weight.shape[0],
                                                                   2 * x.shape[2], 2 * x.shape[3])))


def upsample_conv3x3(module: nn.Module, x: Tensor) -> Tensor:
    return _UpConvBf16Fn.apply(nhwc(x), module, _bias_f32(module, module.bias))


class _StridedBf16Fn(torch.autograd.Function):
    """A 3x3 / stride-2 convolution as the stride-1 one at full resolution read at every other
    position (``phase`` 0: padding 1; 1: diffusers' padding (0, 1, 0, 1)); VJP: dy scattered to
    those positions, then the stride-1 input VJP."""

    @staticmethod
    def forward(ctx, x, module, bias, phase):
        ctx.module, ctx.phase, ctx.xs = module, phase, x.shape
        y = _conv_launch(x, conv_pack(module, False), bias, None, module.weight.shape[0])
        return nhwc(y[:, :, phase::2, phase::2])

    @staticmethod
    def backward(ctx, dy):
        module = ctx.module
        n, cin, h, w = ctx.xs
        cout = module.weight.shape[0]
        full = torch.empty(n, _ceil(cout, 16), h, w, device=dy.device, dtype=BF16, memory_format=CL).zero_()
        full[:, :cout, ctx.phase::2, ctx.phase::2] = dy
        return _conv_launch(full, conv_pack(module, True), None, None, cin), None, None, None


def conv3x3_stride2(module: nn.Module, x: Tensor, padding: int) -> Tensor:
    xp = _pad_channels(x, _ceil(x.shape[1], 16))
    return _StridedBf16Fn.apply(xp, module, _bias_f32(module, module.bias), 0 if padding else 1)


def strided_supported(module: nn.Module, x: Tensor) -> bool:
    return conv_supported(module, x) and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0


def pointwise(x: Tensor, weight: Tensor, bias: Tensor | None) -> Tensor:
    """A 1x1 convolution of channels-last x as one bf16 GEMM over its pixel rows (hipBLASLt)."""
    n, c, h, w = x.shape
    co = weight.shape[0]
    rows = nhwc(x).permute(0, 2, 3, 1).reshape(n * h * w, c)
    y = F.linear(rows, weight.reshape(co, c), bias)
    return y.reshape(n, h, w, co).permute(0, 3, 1, 2)


# ---------------------------------------------------------------------------------------------
# GroupNorm (+ per-(n, c) bias) (+ SiLU)
# ---------------------------------------------------------------------------------------------

def _gn_params(norm: nn.GroupNorm) -> tuple[Tensor | None, Tensor | None]:
    return (_cached(norm, "gamma", _wkey(norm.weight), lambda: _f32(norm.weight)) if norm.weight is not None else None,
            _cached(norm, "beta", _wkey(norm.bias), lambda: _f32(norm.bias)) if norm.bias is not None else None)


def _gn_ws(lib, n: int, c: int, hw: int, device) -> tuple[Tensor, int]:
    nb = int(lib.sp_groupnorm_bf16_workspace(n, c, hw))
    return torch.empty(nb, device=device, dtype=torch.uint8), nb


def _gn_fwd_raw(norm: nn.GroupNorm, x1: Tensor, x2: Tensor | None, cb: Tensor | None,
                blocked: bool = False) -> tuple[Tensor, Tensor]:
    """(z, stats) of ``sp_groupnorm_bf16_fwd_ex`` over cat(x1, x2) (+ cb) read in place; ``blocked``:
    z as a flat buffer in the channel-blocked layout a conv tile reads (``_conv_launch(shape=)``)."""
    lib = _hip.load_library()
    n, c1, h, w = x1.shape
    c2 = 0 if x2 is None else x2.shape[1]
    c, hw, g = c1 + c2, h * w, norm.num_groups
    gamma, beta = _gn_params(norm)
    if blocked:
        z = torch.empty(n * c * hw, device=x1.device, dtype=BF16)
    else:
        z = torch.empty(n, c, h, w, device=x1.device, dtype=BF16, memory_format=CL)
    stats = torch.empty(2, n * g, device=x1.device, dtype=torch.float32)
    ws, nb = _gn_ws(lib, n, c, hw, x1.device)
    _hip.check(lib.sp_groupnorm_bf16_fwd_ex(_p(x1), _p(x2), c1, c2, None if cb is None else cb.data_ptr(),
                                            None if gamma is None else gamma.data_ptr(),
                                            None if beta is None else beta.data_ptr(), n, hw, g, float(norm.eps),
                                            int(norm.act), _p(z, cl=not blocked), int(blocked), stats.data_ptr(),
                                            ws.data_ptr(), nb, _hip.stream_of(x1)), "sp_groupnorm_bf16_fwd_ex")
    return z, stats


def _gn_bwd_raw(norm: nn.GroupNorm, dz: Tensor, x1: Tensor, x2: Tensor | None, cb: Tensor | None, stats: Tensor,
                add1: Tensor | None = None, add2: Tensor | None = None, out1: Tensor | None = None,
                out2: Tensor | None = None, blocked: bool = False,
                add1b: Tensor | None = None, add_cat: bool = False) -> tuple[Tensor, Tensor | None]:
    """Input VJP of ``_gn_fwd_raw`` into the parts' layouts, + the addends (channels-last, shaped
    like the parts) added in the kernel; ``out1`` / ``out2`` may be the addends (in place);
    ``add1b``: a second addend of dx1 (a skip tensor's up-block gradient, layers.SkipGrad);
    ``add_cat``: ``add1`` is one channels-last addend over cat(x1, x2)'s channels (``add2`` None);
    ``blocked`` (one part): dx1 as a flat channel-blocked buffer for the next conv VJP."""
    lib = _hip.load_library()
    n, c1, h, w = x1.shape
    c2 = 0 if x2 is None else x2.shape[1]
    gamma, beta = _gn_params(norm)
    dz = nhwc(dz.to(BF16))
    if blocked:
        dx1 = torch.empty(n * c1 * h * w, device=x1.device, dtype=BF16)
    else:
        dx1 = torch.empty_like(x1, memory_format=CL) if out1 is None else out1
    dx2 = None if x2 is None else (torch.empty_like(x2, memory_format=CL) if out2 is None else out2)
    ws, nb = _gn_ws(lib, n, c1 + c2, h * w, x1.device)
    _hip.check(lib.sp_groupnorm_bf16_bwd_ex(_p(dz), _p(x1), _p(x2), c1, c2, None if cb is None else cb.data_ptr(),
                                            None if gamma is None else gamma.data_ptr(),
                                            None if beta is None else beta.data_ptr(), stats.data_ptr(), n, h * w,
                                            norm.num_groups, int(norm.act), _p(dx1, cl=not blocked), _p(dx2),
                                            2 if add_cat else int(blocked), _p(add1), _p(add2), _p(add1b),
                                            ws.data_ptr(), nb,
                                            _hip.stream_of(dz)), "sp_groupnorm_bf16_bwd_ex")
    return dx1, dx2


def gnvjp_ok(n: int, cin: int, cout: int, h: int, w: int, c1: int, groups: int) -> bool:
    """Whether a conv input VJP (cin cotangent channels -> cout) and the GroupNorm VJP it feeds run as
    ``sp_conv3x3_bf16_gnvjp`` (the GroupNorm sums from the conv's epilogue).  Off by default
    (``SAMPLERS_AMD_BF16_GNVJP=1`` turns it on): measured 10 % slower per DPS bf16 step — the
    epilogue's SiLU-derivative terms (an exp and a reciprocal per output element, per lane 128 of
    them) cost the conv tile more than the sums pass's HBM reads (profiles/round6/bf16/gn_sums_epilogue_ab/)."""
    import os

    from .layers import _query

    return (os.environ.get("SAMPLERS_AMD_BF16_GNVJP", "0") == "1"
            and bool(_query("sp_conv3x3_bf16_gnvjp_supported", n, cin, cout, h, w, c1, groups)))


def _conv_gn_vjp(dy: Tensor, pack: Tensor, cin: int, norm: nn.GroupNorm, x1: Tensor, x2: Tensor | None,
                 cb: Tensor | None, stats: Tensor, dy_blocked: bool = False, add1: Tensor | None = None,
                 add2: Tensor | None = None, out1: Tensor | None = None, out2: Tensor | None = None,
                 add1b: Tensor | None = None, blocked: bool = False) -> tuple[Tensor, Tensor | None]:
    """GN^T(conv^T dy) (+ addends) on ``sp_conv3x3_bf16_gnvjp``: ``dy`` channels-last (or flat
    channel-blocked with ``dy_blocked``) with ``cin`` channels; the GroupNorm over cat(x1, x2) with
    ``stats``; outputs as ``_gn_bwd_raw``."""
    from .layers import _query

    lib = _hip.load_library()
    n, c1, h, w = x1.shape
    c2 = 0 if x2 is None else x2.shape[1]
    cout = c1 + c2
    gamma, beta = _gn_params(norm)
    dz = torch.empty(n, cout, h, w, device=x1.device, dtype=BF16, memory_format=CL)
    if blocked:
        dx1 = torch.empty(n * c1 * h * w, device=x1.device, dtype=BF16)
    else:
        dx1 = torch.empty_like(x1, memory_format=CL) if out1 is None else out1
    dx2 = None if x2 is None else (torch.empty_like(x2, memory_format=CL) if out2 is None else out2)
    nb = _query("sp_conv3x3_bf16_gnvjp_workspace", n, cout, h, w)
    ws = torch.empty(nb, device=x1.device, dtype=torch.uint8)
    _hip.check(lib.sp_conv3x3_bf16_gnvjp(_p(dy, cl=not dy_blocked), int(dy_blocked), _p(pack, cl=False), n, cin, cout,
                                         h, w, _p(dz), _p(x1), _p(x2), c1, None if cb is None else cb.data_ptr(),
                                         None if gamma is None else gamma.data_ptr(),
                                         None if beta is None else beta.data_ptr(), stats.data_ptr(), norm.num_groups,
                                         int(norm.act), _p(dx1, cl=not blocked), _p(dx2), int(blocked), _p(add1),
                                         _p(add2), _p(add1b), ws.data_ptr(), nb, _hip.stream_of(x1)),
               "sp_conv3x3_bf16_gnvjp")
    return dx1, dx2


def gnfwd_ok(n: int, cin: int, cout: int, h: int, w: int, groups: int) -> bool:
    """Whether a conv and the GroupNorm over its output run as ``sp_conv3x3_bf16_gn`` (the moments
    from the conv's epilogue).  Off by default (``SAMPLERS_AMD_BF16_GNFWD=1`` turns it on): measured
    1.7 % slower per DPS bf16 step — the epilogue's reduction (shuffles, two more barriers) costs the
    conv tile more than the statistics pass's read (profiles/round6/bf16/gn_sums_epilogue_ab/)."""
    import os

    from .layers import _query

    return (os.environ.get("SAMPLERS_AMD_BF16_GNFWD", "0") == "1"
            and bool(_query("sp_conv3x3_bf16_gn_supported", n, cin, cout, h, w, groups)))


def _conv_gn(x: Tensor, pack: Tensor, bias: Tensor | None, cout: int, norm: nn.GroupNorm, cb: Tensor | None,
             shape: tuple | None = None, blocked: bool = False) -> tuple[Tensor, Tensor, Tensor]:
    """(y, z, stats): y = conv3x3(x) + bias, z = act(GN(y + cb)) on ``sp_conv3x3_bf16_gn`` (``shape``:
    x flat channel-blocked as ``_conv_launch``; ``blocked``: z flat channel-blocked as ``_gn_fwd_raw``)."""
    from .layers import _query

    lib = _hip.load_library()
    n, cin, h, w = x.shape if shape is None else shape
    g = norm.num_groups
    gamma, beta = _gn_params(norm)
    y = torch.empty(n, cout, h, w, device=x.device, dtype=BF16, memory_format=CL)
    if blocked:
        z = torch.empty(n * cout * h * w, device=x.device, dtype=BF16)
    else:
        z = torch.empty(n, cout, h, w, device=x.device, dtype=BF16, memory_format=CL)
    stats = torch.empty(2, n * g, device=x.device, dtype=torch.float32)
    nb = _query("sp_conv3x3_bf16_gn_workspace", n, cout, h, w)
    ws = torch.empty(nb, device=x.device, dtype=torch.uint8)
    _hip.check(lib.sp_conv3x3_bf16_gn(_p(x, cl=shape is None), 0 if shape is None else 1, _p(pack, cl=False),
                                      None if bias is None else bias.data_ptr(), None, n, cin, cout, h, w, _p(y),
                                      None if cb is None else cb.data_ptr(),
                                      None if gamma is None else gamma.data_ptr(),
                                      None if beta is None else beta.data_ptr(), g, float(norm.eps), int(norm.act),
                                      _p(z, cl=not blocked), int(blocked), stats.data_ptr(), ws.data_ptr(), nb,
                                      _hip.stream_of(x)), "sp_conv3x3_bf16_gn")
    return y, z, stats


class _GroupNormBf16Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x1, x2, norm, cb):
        z, stats = _gn_fwd_raw(norm, x1, x2, cb)
        ctx.save_for_backward(x1, x2, cb, stats)
        ctx.norm = norm
        return z

    @staticmethod
    def backward(ctx, dz):
        x1, x2, cb, stats = ctx.saved_tensors
        dx1, dx2 = _gn_bwd_raw(ctx.norm, dz, x1, x2, cb, stats)
        return dx1, dx2, None, None


def group_norm_supported(norm: nn.GroupNorm, x: Tensor, c2: int = 0) -> bool:
    if not (is_bf16_device(x) and x.dim() == 4) or any(p.requires_grad for p in norm.parameters()):
        return False
    return bool(_hip.load_library().sp_groupnorm_bf16_supported(x.shape[1], c2, norm.num_groups))


def group_norm(norm: nn.GroupNorm, x1: Tensor, x2: Tensor | None = None, chan_bias: Tensor | None = None) -> Tensor:
    """``act(GroupNorm(cat(x1, x2) + chan_bias[:, :, None, None]))`` (``norm.act``: SiLU), the two
    parts read in place."""
    cb = None if chan_bias is None else chan_bias.detach().to(torch.float32).reshape(x1.shape[0], -1).contiguous()
    return _GroupNormBf16Fn.apply(nhwc(x1), None if x2 is None else nhwc(x2), norm, cb)


# ---------------------------------------------------------------------------------------------
# LayerNorm and the residual linears around it (x + f(norm(x)) of the transformer blocks)
# ---------------------------------------------------------------------------------------------

class _LayerNormBf16Fn(torch.autograd.Function):
    """``module(x)`` on ``sp_layernorm_bf16_fwd``; the VJP adds the residual branch's gradient of
    ``x`` when the linear that consumed the residual handed it over (``box``, layers.SkipGrad)."""

    @staticmethod
    def forward(ctx, x, module, box):
        lib = _hip.load_library()
        c = x.shape[-1]
        x2 = x.reshape(-1, c).contiguous()
        rows = x2.shape[0]
        w = _cached(module, "ln_w", _wkey(module.weight), lambda: _f32(module.weight))
        b = _cached(module, "ln_b", _wkey(module.bias), lambda: _f32(module.bias))
        y = torch.empty_like(x2)
        stats = torch.empty(2, rows, device=x.device, dtype=torch.float32)
        _hip.check(lib.sp_layernorm_bf16_fwd(_p(x2), w.data_ptr(), b.data_ptr(), rows, c, float(module.eps), _p(y),
                                             stats[0].data_ptr(), stats[1].data_ptr(), _hip.stream_of(x2)),
                   "sp_layernorm_bf16_fwd")
        ctx.save_for_backward(x2, w, stats)
        ctx.box, ctx.shape = box, x.shape
        return y.reshape(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w, stats = ctx.saved_tensors
        lib = _hip.load_library()
        rows, c = x2.shape
        d2 = dy.to(BF16).reshape(rows, c).contiguous()
        add = ctx.box.take() if ctx.box is not None else None
        if add is not None:
            add = add.to(BF16).reshape(rows, c).contiguous()
        dx = torch.empty_like(x2)
        _hip.check(lib.sp_layernorm_bf16_bwd(_p(d2), _p(x2), w.data_ptr(), stats[0].data_ptr(), stats[1].data_ptr(),
                                             _p(add), rows, c, _p(dx), _hip.stream_of(d2)), "sp_layernorm_bf16_bwd")
        return dx.reshape(ctx.shape), None, None


def layer_norm_supported(module: nn.Module, x: Tensor) -> bool:
    """bf16 device rows, frozen affine LayerNorm over the last dim (``SAMPLERS_AMD_BF16_LN=0``:
    torch, for A/B)."""
    import os

    c = x.shape[-1]
    return (is_bf16_device(x) and os.environ.get("SAMPLERS_AMD_BF16_LN", "1") != "0" and module.weight is not None and module.bias is not None
            and not module.weight.requires_grad and tuple(module.normalized_shape) == (c,)
            and bool(_hip.load_library().sp_layernorm_bf16_supported(x.numel() // max(c, 1), c)))


def layer_norm(x: Tensor, module: nn.Module, box=None) -> Tensor:
    return _LayerNormBf16Fn.apply(x, module, box)


class _LinearResBf16Fn(torch.autograd.Function):
    """``F.linear(x, w2d, bias) + res`` (hipBLASLt bf16 GEMM, the residual added to its output);
    input VJP dx = dy W, and the residual's gradient dy handed to ``box`` (the LayerNorm VJP that
    adds it) instead of autograd's accumulation add."""

    @staticmethod
    def forward(ctx, x, w2d, bias, res, box):
        y = F.linear(x, w2d, bias)
        y += res
        ctx.w2d, ctx.box = w2d, box
        return y

    @staticmethod
    def backward(ctx, dy):
        dx = torch.matmul(dy, ctx.w2d)
        dres = dy
        if ctx.box is not None and ctx.box.enabled:
            ctx.box.grad, dres = dy, None
        return dx, None, None, dres, None


def linear_res(x: Tensor, w2d: Tensor, bias: Tensor | None, res: Tensor, box=None) -> Tensor:
    return _LinearResBf16Fn.apply(x, w2d.detach(), None if bias is None else bias.detach(), res, box)


# ---------------------------------------------------------------------------------------------
# GEGLU (the SD 1.5 transformers' feed-forward gate)
# ---------------------------------------------------------------------------------------------

class _GegluBf16Fn(torch.autograd.Function):
    """``a * gelu(gate)`` with ``a, gate = h.chunk(2, -1)`` on ``sp_geglu_bf16_fwd``; the VJP writes
    the projection's whole cotangent [T][2F] (``sp_geglu_bf16_bwd``: no chunk-gradient concat)."""

    @staticmethod
    def forward(ctx, h):
        lib = _hip.load_library()
        f = h.shape[-1] // 2
        h2 = h.reshape(-1, 2 * f).contiguous()
        y = torch.empty(h2.shape[0], f, device=h.device, dtype=BF16)
        _hip.check(lib.sp_geglu_bf16_fwd(_p(h2), h2.shape[0], f, _p(y), _hip.stream_of(h2)), "sp_geglu_bf16_fwd")
        ctx.save_for_backward(h2)
        ctx.shape = h.shape
        return y.reshape(*h.shape[:-1], f)

    @staticmethod
    def backward(ctx, dy):
        (h2,) = ctx.saved_tensors
        lib = _hip.load_library()
        rows, f2 = h2.shape
        d2 = dy.to(BF16).reshape(rows, f2 // 2).contiguous()
        dh = torch.empty_like(h2)
        _hip.check(lib.sp_geglu_bf16_bwd(_p(h2), _p(d2), rows, f2 // 2, _p(dh), _hip.stream_of(d2)),
                   "sp_geglu_bf16_bwd")
        return dh.reshape(ctx.shape)


def geglu_supported(h: Tensor) -> bool:
    """bf16 device rows of whole 16-feature blocks (``SAMPLERS_AMD_BF16_GEGLU=0``: torch, for A/B)."""
    import os

    return is_bf16_device(h) and h.shape[-1] % 16 == 0 and os.environ.get("SAMPLERS_AMD_BF16_GEGLU", "1") != "0"


def geglu(h: Tensor) -> Tensor:
    return _GegluBf16Fn.apply(h)


# ---------------------------------------------------------------------------------------------
# ResnetBlock2D as one autograd function
# ---------------------------------------------------------------------------------------------

def _rows(t: Tensor) -> Tensor:
    """A channels-last (n, c, h, w) tensor as its [n h w][c] pixel rows (a view)."""
    return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])


def _shortcut_w(block: nn.Module, c1: int) -> tuple[Tensor, Tensor]:
    """conv_shortcut's [cout][cin] weight split at c1 (x's channels | the skip's), contiguous."""
    w = block.conv_shortcut.weight
    return _cached(block.conv_shortcut, f"split{c1}", _wkey(w),
                   lambda: tuple(t.contiguous() for t in w.detach().reshape(w.shape[0], -1).split(
                       [c1, w.shape[1] - c1], dim=1)))


class _ResnetBlockBf16Fn(torch.autograd.Function):
    """A whole ResnetBlock2D at bf16 (the structure of unet2d._ResnetBlockFn):

    fwd  z1 = silu(GN1(cat(x1, x2)))   both parts read in place
         h1 = conv1(z1)
         z2 = silu(GN2(h1 + tb))
         out = conv2(z2) + shortcut(x)   an identity shortcut added in conv2's epilogue; a 1x1
                                         shortcut over cat(x1, x2) summed into conv2's own
                                         contraction (sp_conv3x3_bf16_sc: its stages read the
                                         parts in place), else two GEMMs over the parts' rows
    bwd  dx = GN1^T(conv1^T(GN2^T(conv2^T dout))) + shortcut^T dout, the shortcut's gradient
         added by GN1's VJP kernel into the parts' gradients (no autograd accumulation add).
    Skip tensors (layers.SkipGrad, as unet2d._ResnetBlockFn): ``box_out`` receives dx2 (the
    up-block's gradient of its skip part) instead of autograd; ``box_in`` (x1 is a skip tensor)
    delivers that gradient, added by GN1's VJP kernel (its add1b) — no accumulation add.
    Saves x1, x2, h1 and the GroupNorm statistics (weights are frozen: no z1 / z2)."""

    @staticmethod
    def forward(ctx, block, tb, x1, x2, box_in=None, box_out=None):
        cout = block.conv2.weight.shape[0]
        n, c1, hh, ww = x1.shape
        cin = c1 + (0 if x2 is None else x2.shape[1])
        # the GroupNorm outputs feed only the convs: handed over channel-blocked where the tile takes it
        b1, b2 = blocked_ok(cin, cout, hh, ww), blocked_ok(cout, cout, hh, ww)
        z1, st1 = _gn_fwd_raw(block.norm1, x1, x2, None, blocked=b1)
        cmid = block.conv1.weight.shape[0]
        if gnfwd_ok(n, cin, cmid, hh, ww, block.norm2.num_groups):  # GN2's moments from conv1's epilogue
            h1, z2, st2 = _conv_gn(z1, conv_pack(block.conv1, False), _bias_f32(block.conv1, block.conv1.bias), cmid,
                                   block.norm2, tb, shape=(n, cin, hh, ww) if b1 else None, blocked=b2)
            del z1
        else:
            h1 = _conv_launch(z1, conv_pack(block.conv1, False), _bias_f32(block.conv1, block.conv1.bias), None,
                              cmid, shape=(n, cin, hh, ww) if b1 else None)
            del z1
            z2, st2 = _gn_fwd_raw(block.norm2, h1, None, tb, blocked=b2)
        c2 = 0 if x2 is None else x2.shape[1]
        if block.conv_shortcut is not None and sc_ok(cout, x1.shape[1], c2, hh, ww):
            # conv2 + the 1x1 shortcut as one contraction: no shortcut tensor, no residual read
            out = _conv_sc_launch(z2, conv_pack(block.conv2, False), _sc_bias(block), x1, x2, shortcut_pack(block),
                                  cout, shape=(n, cout, hh, ww) if b2 else None)
            ctx.block = block
            ctx.box_in, ctx.box_out = box_in, box_out
            ctx.save_for_backward(x1, x2, h1, tb, st1, st2)
            return out
        if block.conv_shortcut is None:
            short = x1
        else:
            c1 = x1.shape[1]
            w1, w2 = _shortcut_w(block, c1)
            n, _, h, w = x1.shape
            b = block.conv_shortcut.bias
            r = (torch.addmm(b, _rows(x1), w1.t()) if b is not None else _rows(x1) @ w1.t())
            if x2 is not None:
                r.addmm_(_rows(x2), w2.t())
            short = r.reshape(n, h, w, cout).permute(0, 3, 1, 2)
        out = _conv_launch(z2, conv_pack(block.conv2, False), _bias_f32(block.conv2, block.conv2.bias), short, cout,
                           shape=(n, cout, hh, ww) if b2 else None)
        ctx.block = block
        ctx.box_in, ctx.box_out = box_in, box_out
        ctx.save_for_backward(x1, x2, h1, tb, st1, st2)
        return out

    @staticmethod
    def backward(ctx, dout):
        import os

        x1, x2, h1, tb, st1, st2 = ctx.saved_tensors
        blk = ctx.block
        dout = nhwc(dout.to(BF16))
        cout = blk.conv2.weight.shape[0]
        cmid = blk.conv1.weight.shape[0]
        cin = blk.conv1.weight.shape[1]
        n, _, hh, ww = h1.shape
        c1 = x1.shape[1]
        # dh1 feeds only conv1's VJP: channel-blocked where the tile takes it
        bl = cmid % 16 == 0 and blocked_ok(cmid, cin, hh, ww)
        dpad = _pad_channels(dout, _ceil(cout, 16))
        if gnvjp_ok(n, dpad.shape[1], cmid, hh, ww, cmid, blk.norm2.num_groups):  # GN2 sums from conv2^T's epilogue
            dh1, _ = _conv_gn_vjp(dpad, conv_pack(blk.conv2, True), dpad.shape[1], blk.norm2, h1, None, tb, st2,
                                  blocked=bl)
        else:
            dz2 = _conv_launch(dpad, conv_pack(blk.conv2, True), None, None, cmid)
            dh1, _ = _gn_bwd_raw(blk.norm2, dz2, h1, None, tb, st2, blocked=bl)
            del dz2
        del dpad
        extra = ctx.box_in.take() if ctx.box_in is not None else None
        if extra is not None:
            extra = nhwc(extra.to(BF16))
        fused_gn1 = cmid % 16 == 0 and gnvjp_ok(n, cmid, cin, hh, ww, c1, blk.norm1.num_groups)
        if blk.conv_shortcut is None:  # identity shortcut: dx1 = GN1^T dz1 + dout (+ skip grad)
            adds = dict(add1=dout, add1b=extra)
        elif fused_gn1 or os.environ.get("SAMPLERS_AMD_BF16_SCVJP", "1") == "0":
            # s = shortcut^T dout per part (pixel rows), then += GN1^T dz1 in place
            w1, w2 = _shortcut_w(blk, c1)
            d = _rows(dout)
            s1 = (d @ w1).reshape(n, hh, ww, c1).permute(0, 3, 1, 2)
            s2 = None if x2 is None else (d @ w2).reshape(n, hh, ww, x2.shape[1]).permute(0, 3, 1, 2)
            adds = dict(add1=s1, add2=s2, out1=s1, out2=s2, add1b=extra)
        else:  # shortcut^T dout over cat(x1, x2)'s channels as one GEMM (dout read once), added by GN1's VJP
            wfull = _cached(blk.conv_shortcut, "w2d", _wkey(blk.conv_shortcut.weight),
                            lambda: blk.conv_shortcut.weight.detach().reshape(cout, cin).contiguous())
            sc = (_rows(dout) @ wfull).reshape(n, hh, ww, cin).permute(0, 3, 1, 2)
            adds = dict(add1=sc, add1b=extra, add_cat=True)
        if fused_gn1:  # GN1 sums: conv1^T's epilogue
            dx1, dx2 = _conv_gn_vjp(dh1, conv_pack(blk.conv1, True), cmid, blk.norm1, x1, x2, None, st1,
                                    dy_blocked=bl, **adds)
        else:
            if bl:
                dz1 = _conv_launch(dh1, conv_pack(blk.conv1, True), None, None, cin, shape=(n, cmid, hh, ww))
            else:
                dz1 = _conv_launch(_pad_channels(dh1, _ceil(cmid, 16)), conv_pack(blk.conv1, True), None, None, cin)
            dx1, dx2 = _gn_bwd_raw(blk.norm1, dz1, x1, x2, None, st1, **adds)
        del dh1
        if ctx.box_out is not None:  # x2 (a skip): its down-path consumer adds this gradient
            ctx.box_out.grad, dx2 = dx2, None
        return None, None, dx1, dx2, None, None


def resnet_block_supported(block: nn.Module, x: Tensor, skip: Tensor | None) -> bool:
    """Whether ``resnet_block`` serves the block: bf16 device tensors, frozen weights, both 3x3
    convolutions and both norms on the bf16 kernels, channel counts in whole 16-blocks
    (``SAMPLERS_AMD_BF16_RESNET=0``: module by module, for A/B measurements)."""
    import os

    if os.environ.get("SAMPLERS_AMD_BF16_RESNET", "1") == "0":
        return False
    if not is_bf16_device(x) or x.dim() != 4 or (skip is not None and not is_bf16_device(skip)):
        return False
    c2 = 0 if skip is None else skip.shape[1]
    cin, cout = x.shape[1] + c2, block.conv2.weight.shape[0]
    if cin % 16 or cout % 16 or block.conv1.weight.shape[1] != cin or block.conv1.weight.shape[0] != cout:
        return False
    if block.conv_shortcut is None and skip is not None:  # an identity shortcut of cat(x, skip)
        return False
    if any(p.requires_grad for p in block.parameters()):
        return False
    lib = _hip.load_library()
    n, _, h, w = x.shape
    return bool(lib.sp_groupnorm_bf16_supported(x.shape[1], c2, block.norm1.num_groups)
                and lib.sp_groupnorm_bf16_supported(cout, 0, block.norm2.num_groups)
                and lib.sp_conv3x3_bf16_supported(cin, cout, h, w) and lib.sp_conv3x3_bf16_supported(cout, cout, h, w))


def resnet_block(block: nn.Module, x: Tensor, skip: Tensor | None, tb: Tensor | None, box_in=None,
                 box_out=None) -> Tensor:
    """``block(x, temb, skip)`` at bf16 as ``_ResnetBlockBf16Fn`` (``tb``: the block's
    time-embedding projection, [n, cout], or None; ``box_in`` / ``box_out``: enabled SkipGrad
    mailboxes of x / skip, or None)."""
    cb = None if tb is None else tb.detach().to(torch.float32).reshape(x.shape[0], -1).contiguous()
    return _ResnetBlockBf16Fn.apply(block, cb, nhwc(x), None if skip is None else nhwc(skip), box_in,
                                    None if skip is None else box_out)


# ---------------------------------------------------------------------------------------------
# multi-head attention (SD 1.5 UNet: head dims 40 / 80 / 160, 4096 .. 64 tokens, 77 context rows)
# ---------------------------------------------------------------------------------------------

def attention_supported(b: int, heads: int, n: int, m: int, d: int) -> bool:
    return bool(_hip.load_library().sp_attention_bf16_supported(b, heads, n, m, d))


def _attn_fwd(q: Tensor, k: Tensor, v: Tensor, b: int, heads: int, n: int, m: int, d: int, rsq: int, rskv: int,
              kv_shared: bool, offs=(0, 0, 0)) -> tuple[Tensor, Tensor]:
    lib = _hip.load_library()
    c = heads * d
    out = torch.empty(b, n, c, device=q.device, dtype=BF16)
    lse = torch.empty(b * heads, n, device=q.device, dtype=torch.float32)
    _hip.check(lib.sp_attention_bf16_fwd(_p(q, cl=False) + offs[0], _p(k, cl=False) + offs[1],
                                         _p(v, cl=False) + offs[2], b, heads, n, m, d, rsq, rskv, int(kv_shared), c,
                                         1.0 / math.sqrt(d), _p(out, cl=False), lse.data_ptr(), _hip.stream_of(q)),
               "sp_attention_bf16_fwd")
    return out, lse


class _SelfAttnBf16Fn(torch.autograd.Function):
    """Self-attention on the fused projection's bf16 output qkv ([b][n][3 heads d], q, k, v its
    thirds read in place).  VJP: the exact-fp32 fused kernels (sp_attention_bwd_mh) on q, k, v,
    the output and its cotangent widened to fp32, the cotangent of qkv rounded back to bf16."""

    @staticmethod
    def forward(ctx, qkv, heads):
        b, n, c3 = qkv.shape
        c = c3 // 3
        d = c // heads
        qkv = qkv.contiguous()
        out, lse = _attn_fwd(qkv, qkv, qkv, b, heads, n, n, d, c3, c3, False, offs=(0, 2 * c, 4 * c))
        ctx.save_for_backward(qkv, out, lse)
        ctx.heads = heads
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        lib = _hip.load_library()
        b, n, c3 = qkv.shape
        c = c3 // 3
        heads = ctx.heads
        d = c // heads
        if lib.sp_attention_bf16_bwd_supported(b, heads, n, n, d):  # the bf16 VJP kernels
            do = dout.to(BF16).contiguous()
            dqkv = torch.empty_like(qkv)
            delta = torch.empty(b * heads, n, device=qkv.device, dtype=torch.float32)
            base, dbase = _p(qkv, cl=False), _p(dqkv, cl=False)
            _hip.check(lib.sp_attention_bf16_bwd(base, base + 2 * c, base + 4 * c, _p(out, cl=False),
                                                 _p(do, cl=False), lse.data_ptr(), b, heads, n, n, d, c3, c3, 0, c,
                                                 c3, c3, 1.0 / math.sqrt(d), delta.data_ptr(), dbase, dbase + 2 * c,
                                                 dbase + 4 * c, _hip.stream_of(do)), "sp_attention_bf16_bwd")
            return dqkv, None
        q32, o32, do32 = qkv.float(), out.float(), dout.float().contiguous()
        dqkv = torch.empty_like(q32)
        delta = torch.empty(b * heads, n, device=qkv.device, dtype=torch.float32)
        base, dbase = q32.data_ptr(), dqkv.data_ptr()
        _hip.check(lib.sp_attention_bwd_mh(base, base + 4 * c, base + 8 * c, _hip.ptr(o32), _hip.ptr(do32),
                                           _hip.ptr(lse), b, heads, n, n, d, c3, c3, b, c, 1.0 / math.sqrt(d),
                                           _hip.ptr(delta), dbase, dbase + 4 * c, dbase + 8 * c,
                                           _hip.stream_of(do32)), "sp_attention_bwd_mh")
        return dqkv.to(BF16), None


class _CrossAttnBf16Fn(torch.autograd.Function):
    """Cross-attention of bf16 token rows q ([b][n][heads d]) to a context's k, v ([bc][m][heads
    d], bc = 1 or b); VJP dq only (the context is a constant of the prior's call), on the fp32
    kernels as above."""

    @staticmethod
    def forward(ctx, q, k, v, heads):
        b, n, c = q.shape
        bc, m, _ = k.shape
        d = c // heads
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        out, lse = _attn_fwd(q, k, v, b, heads, n, m, d, c, c, bc == 1)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.heads = heads
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        lib = _hip.load_library()
        b, n, c = q.shape
        bc, m, _ = k.shape
        heads = ctx.heads
        if lib.sp_attention_bf16_bwd_supported(b, heads, n, m, c // heads):  # the bf16 VJP kernels
            do = dout.to(BF16).contiguous()
            dq = torch.empty_like(q)
            delta = torch.empty(b * heads, n, device=q.device, dtype=torch.float32)
            _hip.check(lib.sp_attention_bf16_bwd(_p(q, cl=False), _p(k, cl=False), _p(v, cl=False),
                                                 _p(out, cl=False), _p(do, cl=False), lse.data_ptr(), b, heads, n,
                                                 m, c // heads, c, c, int(bc == 1), c, c, c,
                                                 1.0 / math.sqrt(c // heads), delta.data_ptr(), _p(dq, cl=False),
                                                 None, None, _hip.stream_of(do)), "sp_attention_bf16_bwd")
            return dq, None, None, None
        q32, k32, v32, o32 = q.float(), k.float(), v.float(), out.float()
        do32 = dout.float().contiguous()
        dq = torch.empty_like(q32)
        delta = torch.empty(b * heads, n, device=q.device, dtype=torch.float32)
        _hip.check(lib.sp_attention_bwd_mh(_hip.ptr(q32), _hip.ptr(k32), _hip.ptr(v32), _hip.ptr(o32),
                                           _hip.ptr(do32), _hip.ptr(lse), b, heads, n, m, c // heads, c, c, bc, c,
                                           1.0 / math.sqrt(c // heads), _hip.ptr(delta), _hip.ptr(dq), None, None,
                                           _hip.stream_of(do32)), "sp_attention_bwd_mh")
        return dq.to(BF16), None, None, None


def self_attention(qkv: Tensor, heads: int) -> Tensor:
    return _SelfAttnBf16Fn.apply(qkv, heads)


def cross_attention(q: Tensor, k: Tensor, v: Tensor, heads: int) -> Tensor:
    return _CrossAttnBf16Fn.apply(q, k, v, heads)


def vjp_supported(b: int, heads: int, n: int, m: int, d: int) -> bool:
    """A fused VJP serves this shape: the bf16 kernels (head dims 40 / 64 / 80), else the exact-fp32
    ones on the operands widened to fp32 (head dim 160)."""
    lib = _hip.load_library()
    return bool(lib.sp_attention_bf16_bwd_supported(b, heads, n, m, d) or lib.sp_attention_mh_supported(b, heads, n, m, d))

"""Fused GroupNorm (+ time-embedding bias) (+ SiLU) and 3x3 convolutions for the priors.

``GroupNormAct`` is a drop-in ``nn.GroupNorm`` (same parameters, same state-dict
keys) whose forward optionally adds a per-(sample, channel) bias to its input and
applies SiLU to its output — the ``norm -> silu`` pairs and the ``h + temb`` add of
diffusers' ``ResnetBlock2D`` that the reference's priors run
(``/root/reference/samplers/networks/diffusers/ddpm.py:40-43``,
``stable_diffusion.py:330-345``).  On device tensors it runs the HIP kernels of
``csrc/sp_groupnorm.hip`` (``sp_groupnorm_silu_fwd2/bwd2``) through a
``torch.autograd.Function`` whose backward is the fused input VJP; on CPU tensors
(the oracle's CPU baseline and the CPU tests) it is plain torch.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from .. import _hip
from ..runtime import batch_invariant_enabled, split_k_enabled


def group_norm_act_torch(x: Tensor, groups: int, weight: Tensor | None, bias: Tensor | None,
                         eps: float, act: bool, chan_bias: Tensor | None = None) -> Tensor:
    """Plain-torch semantics of the fused op (CPU path and test reference)."""
    if chan_bias is not None:
        x = x + chan_bias[:, :, None, None]
    y = F.group_norm(x, groups, weight, bias, eps)
    return F.silu(y) if act else y


# Per-shape answers of the library's pure shape queries (tile support, workspace sizes), cached:
# at batch 1 a step makes ~600 launches and each query is a ctypes round trip on the host path.
_shape_cache: dict = {}


def _query(fn_name: str, *args: int) -> int:
    key = (fn_name, args)
    v = _shape_cache.get(key)
    if v is None:
        v = _shape_cache[key] = int(getattr(_hip.load_library(), fn_name)(*args))
    return v


def _hw(t: Tensor) -> int:
    """Pixels per channel plane of an [n][c][...] tensor (1 for [n][c])."""
    hw = 1
    for d in t.shape[2:]:
        hw *= d
    return hw


# The single-pass GroupNorm kernels' team words (sp_groupnorm_team_bytes): one zeroed region per
# (device, stream), owned here and handed to every call on that stream (the kernels leave it
# zero, so no call needs a memset).  The library allocates nothing.  Grown by
# replacement: the old region goes back to torch's caching allocator on the same stream, so any
# reuse of it is ordered after the launches that still name it.  Never used while a stream is
# being captured into a graph (those calls take the two-pass kernels; a region allocated inside
# a capture would belong to the graph's pool).  SAMPLERS_AMD_GN_TEAM=0: no region (the library
# then zeroes words in the call's workspace, one memset per call).
_team_regions: dict = {}


def _team_enabled() -> bool:
    import os

    return os.environ.get("SAMPLERS_AMD_GN_TEAM", "1").lower() not in ("0", "off", "false")


def gn_team_region(x: Tensor, n: int, c: int, hw: int, groups: int) -> tuple[Tensor | None, int]:
    """(region, bytes) for a GroupNorm call on x's device and the current stream, or (None, 0)."""
    if not _team_enabled() or torch.cuda.is_current_stream_capturing():
        return None, 0
    need = _query("sp_groupnorm_team_bytes", n, c, hw, groups)
    if need <= 0:
        return None, 0
    key = (x.device.index, _hip.stream_of(x))
    t = _team_regions.get(key)
    if t is None or t.numel() < need:
        size = max(need * 2, 4 << 20)
        t = _team_regions[key] = torch.zeros(size, device=x.device, dtype=torch.uint8)
    return t, t.numel()


def release_team_regions() -> None:
    """Drop the cached team regions (e.g. before destroying a stream they were used on)."""
    _team_regions.clear()


def gn_forward(norm: "GroupNormAct", x1: Tensor, x2: Tensor | None = None,
               chan_bias: Tensor | None = None) -> tuple[Tensor, Tensor]:
    """HIP GroupNorm(+bias)(+SiLU) forward over x1, or over cat(x1, x2) along channels read in
    place; returns (z, stats = [mean; rstd] per (sample, group))."""
    lib = _hip.load_library()
    n, c1 = x1.shape[0], x1.shape[1]
    c = c1 + (x2.shape[1] if x2 is not None else 0)
    hw = _hw(x1) if x1.numel() else 1
    g = norm.num_groups
    z = torch.empty((n, c) + tuple(x1.shape[2:]), device=x1.device, dtype=torch.float32)
    stats = torch.empty(2, n * g, device=x1.device, dtype=torch.float32)
    work = torch.empty(max(_query("sp_groupnorm_workspace", n, c, hw, g), 1), device=x1.device,
                       dtype=torch.float32)
    team, tb = gn_team_region(x1, n, c, hw, g)
    sp = _hip.ptr(stats)
    _hip.check(lib.sp_groupnorm_silu_fwd2(
        _hip.ptr(x1), _hip.ptr(x2), c1, _hip.ptr(chan_bias), _hip.ptr(norm.weight),
        _hip.ptr(norm.bias), n, c, hw, g, float(norm.eps), int(norm.act),
        _hip.ptr(z), sp, sp + 4 * n * g, _hip.ptr(work), _hip.ptr(team), tb, _hip.stream_of(x1)),
        "sp_groupnorm_silu_fwd2")
    return z, stats


def gn_backward(norm: "GroupNormAct", dz: Tensor, x1: Tensor, x2: Tensor | None,
                chan_bias: Tensor | None, stats: Tensor, add1: Tensor | None = None,
                add2: Tensor | None = None, out1: Tensor | None = None,
                out2: Tensor | None = None, add1b: Tensor | None = None) -> tuple[Tensor, Tensor | None]:
    """Input VJP of ``gn_forward`` into the parts' shapes, plus the optional addends
    (out1 / out2 may be the addends themselves: accumulate in place); ``add1b`` is a second
    addend of a one-part input, added after ``add1``."""
    lib = _hip.load_library()
    n, c1 = x1.shape[0], x1.shape[1]
    c = dz.shape[1]
    hw = _hw(x1) if x1.numel() else 1
    g = norm.num_groups
    dx1 = torch.empty_like(x1) if out1 is None else out1
    dx2 = None if x2 is None else (torch.empty_like(x2) if out2 is None else out2)
    work = torch.empty(max(_query("sp_groupnorm_workspace", n, c, hw, g), 1), device=x1.device,
                       dtype=torch.float32)
    team, tb = gn_team_region(x1, n, c, hw, g)
    sp = _hip.ptr(stats)
    _hip.check(lib.sp_groupnorm_silu_bwd2(
        _hip.ptr(dz.contiguous()), _hip.ptr(x1), _hip.ptr(x2), c1, _hip.ptr(chan_bias),
        _hip.ptr(norm.weight), _hip.ptr(norm.bias), sp, sp + 4 * n * g, n, c,
        hw, g, int(norm.act), _hip.ptr(dx1), _hip.ptr(dx2), _hip.ptr(add1),
        _hip.ptr(add2), _hip.ptr(add1b), _hip.ptr(work), _hip.ptr(team), tb, _hip.stream_of(x1)),
        "sp_groupnorm_silu_bwd2")
    return dx1, dx2


class _GroupNormActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, chan_bias, groups: int, eps: float, act: bool, box=None):
        lib = _hip.load_library()
        n, c = x.shape[0], x.shape[1]
        hw = _hw(x) if x.numel() else 1
        x = x.contiguous()
        z = torch.empty_like(x)
        stats = torch.empty(2, n * groups, device=x.device, dtype=torch.float32)
        work = torch.empty(max(_query("sp_groupnorm_workspace", n, c, hw, groups), 1),
                           device=x.device, dtype=torch.float32)
        cb = None if chan_bias is None else chan_bias.contiguous()
        team, tb = gn_team_region(x, n, c, hw, groups)
        _hip.check(lib.sp_groupnorm_silu_fwd2(
            _hip.ptr(x), None, c, _hip.ptr(cb), _hip.ptr(weight), _hip.ptr(bias), n, c, hw, groups,
            float(eps), int(act), _hip.ptr(z), _hip.ptr(stats[0]), _hip.ptr(stats[1]),
            _hip.ptr(work), _hip.ptr(team), tb, _hip.stream_of(x)), "sp_groupnorm_silu_fwd2")
        ctx.save_for_backward(x, weight, bias, cb, stats)
        ctx.cfg = (groups, float(eps), bool(act))
        ctx.box = box
        return z

    @staticmethod
    def backward(ctx, dz):
        x, weight, bias, cb, stats = ctx.saved_tensors
        groups, eps, act = ctx.cfg
        lib = _hip.load_library()
        n, c = x.shape[0], x.shape[1]
        hw = _hw(x) if x.numel() else 1
        dz = dz.contiguous()
        dx = torch.empty_like(x)
        work = torch.empty(max(_query("sp_groupnorm_workspace", n, c, hw, groups), 1),
                           device=x.device, dtype=torch.float32)
        add = ctx.box.take() if ctx.box is not None else None
        add = None if add is None else add.contiguous()  # the residual branch's gradient of x
        team, tb = gn_team_region(x, n, c, hw, groups)
        _hip.check(lib.sp_groupnorm_silu_bwd2(
            _hip.ptr(dz), _hip.ptr(x), None, c, _hip.ptr(cb), _hip.ptr(weight), _hip.ptr(bias),
            _hip.ptr(stats[0]), _hip.ptr(stats[1]), n, c, hw, groups, int(act), _hip.ptr(dx), None,
            _hip.ptr(add), None, None, _hip.ptr(work), _hip.ptr(team), tb, _hip.stream_of(x)),
            "sp_groupnorm_silu_bwd2")
        d_w = d_b = d_cb = None
        need_w, need_b, need_cb = ctx.needs_input_grad[1], ctx.needs_input_grad[2], ctx.needs_input_grad[3]
        if need_cb:
            d_cb = dx.sum(dim=tuple(range(2, dx.ndim)))
        if need_w or need_b:
            # parameter gradients (not on the sampler's path, which differentiates
            # w.r.t. the sample only): recomputed with torch from the saved stats
            mean, rstd = stats[0].view(n, groups, 1), stats[1].view(n, groups, 1)
            xb = x if cb is None else x + cb[:, :, None, None]
            xh = ((xb.reshape(n, groups, -1) - mean) * rstd).reshape_as(x)
            shape = (1, c) + (1,) * (x.ndim - 2)
            y = xh * (weight.view(shape) if weight is not None else 1) + (
                bias.view(shape) if bias is not None else 0)
            dy = dz
            if act:
                s = torch.sigmoid(y)
                dy = dz * s * (1 + y * (1 - s))
            red = (0,) + tuple(range(2, x.ndim))
            if need_w:
                d_w = (dy * xh).sum(dim=red)
            if need_b:
                d_b = dy.sum(dim=red)
        return dx, d_w, d_b, d_cb, None, None, None, None


class GroupNormAct(nn.GroupNorm):
    """``nn.GroupNorm`` with an optional fused input bias and SiLU (``act=True``)."""

    def __init__(self, num_groups: int, num_channels: int, eps: float = 1e-5, affine: bool = True,
                 act: bool = False) -> None:
        super().__init__(num_groups, num_channels, eps=eps, affine=affine)
        self.act = act

    def forward(self, x: Tensor, chan_bias: Tensor | None = None, box: SkipGrad | None = None) -> Tensor:
        """``box``: a residual consumer of ``x`` hands its gradient over to be summed inside the
        VJP kernel (``SkipGrad``)."""
        if not x.is_cuda:
            if box is not None:
                box.enabled = False
            return group_norm_act_torch(x, self.num_groups, self.weight, self.bias, self.eps,
                                        self.act, chan_bias)
        if x.dtype != torch.float32:
            # reduced-precision priors (the reference's bf16 / fp16 runs): bf16 on the NHWC
            # kernels (networks/bf16.py), fp16 on torch's GroupNorm
            if box is not None:
                box.enabled = False
            from . import bf16
            if bf16.group_norm_supported(self, x):
                return bf16.group_norm(self, x, None, chan_bias)
            return group_norm_act_torch(x, self.num_groups, self.weight, self.bias, self.eps, self.act,
                                        chan_bias)
        return _GroupNormActFn.apply(x, self.weight, self.bias, chan_bias, self.num_groups,
                                     self.eps, self.act, box)

    def extra_repr(self) -> str:
        return super().extra_repr() + f", act={'silu' if self.act else 'none'}"


# ---------------------------------------------------------------------------------------
# 3x3 convolution on fp32 MFMA
# ---------------------------------------------------------------------------------------

def miopen_fallback(x: Tensor) -> None:
    """Before a device convolution goes to MIOpen: point its find-db / kernel cache at the
    seeded in-tree directory (``runtime.ensure_miopen``, once per process)."""
    if x.is_cuda:
        from samplers_amd.runtime import ensure_miopen

        ensure_miopen()


def conv_backend() -> str:
    """``SAMPLERS_AMD_CONV``: ``auto`` (default: Winograd F(2x2,3x3) tile where its shape
    rules hold, else the direct tile, else MIOpen), ``direct`` (direct tile or MIOpen),
    ``miopen`` (always torch/MIOpen).  (Two split-bf16 3x3 backends, a Winograd and a direct
    one, were measured 1.2-1.6x and 1.1-1.3x slower than the fp32 Winograd tile on every
    UNet shape and were removed from the library; DESIGN.md §3 keeps the measurements.)"""
    import os

    return os.environ.get("SAMPLERS_AMD_CONV", "auto").lower()


def _conv_algo(lib, cin: int, cout: int, h: int, w: int, backend: str) -> str | None:
    if backend == "miopen":
        return None
    if backend == "auto" and _query("sp_wino3x3_supported", cin, cout, h, w):
        return "wino"
    if _query("sp_conv3x3_supported", cin, cout, h, w):
        return "direct"
    if _query("sp_conv3x3_thin_supported", cin, cout, h, w):
        return "thin"  # few channels on one side (conv_in / conv_out): VALU direct conv
    return None


def conv3x3_forward(module: "Conv3x3", x: Tensor, res: Tensor | None = None,
                    bias: Tensor | None = None) -> Tensor:
    """conv(x) + bias (+ res) on the module's tile (the residual rides in the Winograd
    epilogue), MIOpen + an add where no tile serves the shape.  ``bias`` overrides the
    module's (the fused ResnetBlock folds the shortcut's bias into it)."""
    lib = _hip.load_library()
    n, cin, h, w = x.shape
    cout = module.out_channels
    bias = module.bias if bias is None else bias.contiguous()
    algo = _conv_algo(lib, cin, cout, h, w, conv_backend())
    if algo is None:
        miopen_fallback(x)
        y = F.conv2d(x, module.weight, bias, padding=1)
        return y if res is None else y.add_(res)
    x = x.contiguous()
    y = torch.empty(n, cout, h, w, device=x.device, dtype=torch.float32)
    if algo == "thin":
        _hip.check(lib.sp_conv3x3_thin_fwd(_hip.ptr(x), _hip.ptr(module.weight.detach().contiguous()),
                                           _hip.ptr(bias), n, cin, cout, h, w, _hip.ptr(y),
                                           _hip.stream_of(x)), "sp_conv3x3_thin_fwd")
        return y if res is None else y.add_(res)
    pk = tile_pack(module, algo, False)
    if algo == "wino":
        # split-K where the tiles leave CUs idle (small batches, low-resolution levels)
        ws = _wino_workspace(lib, n, cin, cout, h, w, x.device)  # held until queued
        _hip.check(lib.sp_wino3x3_fwd_ws(_hip.ptr(x), _hip.ptr(pk), _hip.ptr(bias),
                                         None if res is None else _hip.ptr(res.contiguous()), n,
                                         cin, cout, h, w, _hip.ptr(y), _hip.ptr(ws),
                                         0 if ws is None else ws.numel() * 4, _hip.stream_of(x)),
                   "sp_wino3x3_fwd_ws")
        return y
    _hip.check(lib.sp_conv3x3_fwd(_hip.ptr(x), _hip.ptr(pk), _hip.ptr(bias), n, cin, cout, h, w,
                                  _hip.ptr(y), _hip.stream_of(x)), "sp_direct_conv3x3_fwd")
    return y if res is None else y.add_(res)


def _wino_workspace(lib, n: int, cin: int, cout: int, h: int, w: int, device) -> Tensor | None:
    """A workspace for the Winograd tile's split-K parts, or None when the shape fills the
    chip unsplit (sp_wino3x3_workspace).  From torch's caching allocator on the launch
    stream, so a graph capture records it and a later reuse is ordered after the launch."""
    nb = _query("sp_wino3x3_workspace", n, cin, cout, h, w) if split_k_enabled() else 0
    if nb <= 0:
        return None
    return torch.empty(nb // 4, device=device, dtype=torch.float32)


def x6_workspace(lib, n: int, hw: int, k: int, m: int, device) -> tuple[Tensor | None, int]:
    """The bf16x6 GEMM's split-K workspace for an under-filled launch (sp_gemm_x6_workspace;
    n images of hw pixels, or n = 1 and hw = tokens), and its size in bytes; (None, 0) when the
    launch fills the chip unsplit.  Torch's caching allocator on the launch stream, as
    _wino_workspace; the caller holds it until the launch is queued."""
    nb = _query("sp_gemm_x6_workspace", n, hw, k, m) if split_k_enabled() else 0
    if nb <= 0:
        return None, 0
    return torch.empty(nb // 4, device=device, dtype=torch.float32), nb


def conv3x3_input_vjp(module: "Conv3x3", dy: Tensor, x_shape) -> Tensor:
    """d conv(x) / dx applied to dy (weights frozen)."""
    lib = _hip.load_library()
    n, cin, h, w = x_shape
    cout = module.out_channels
    algo = _conv_algo(lib, cout, cin, h, w, conv_backend())
    dy = dy.contiguous()
    if algo is None:
        miopen_fallback(dy)
        return torch.nn.grad.conv2d_input(tuple(x_shape), module.weight, dy, padding=1)
    dx = torch.empty(tuple(x_shape), device=dy.device, dtype=torch.float32)
    if algo == "thin":
        _hip.check(lib.sp_conv3x3_thin_bwd_input(_hip.ptr(dy), _hip.ptr(module.weight.detach().contiguous()),
                                                 n, cin, cout, h, w, _hip.ptr(dx),
                                                 _hip.stream_of(dy)), "sp_conv3x3_thin_bwd_input")
        return dx
    if algo == "wino":
        ws = _wino_workspace(lib, n, cout, cin, h, w, dy.device)  # the VJP's K is cout
        _hip.check(lib.sp_wino3x3_bwd_input_ws(_hip.ptr(dy), _hip.ptr(tile_pack(module, algo, True)),
                                               n, cin, cout, h, w, _hip.ptr(dx), _hip.ptr(ws),
                                               0 if ws is None else ws.numel() * 4,
                                               _hip.stream_of(dy)), "sp_wino3x3_bwd_input_ws")
        return dx
    _hip.check(lib.sp_conv3x3_bwd_input(_hip.ptr(dy), _hip.ptr(tile_pack(module, algo, True)), n, cin,
                                        cout, h, w, _hip.ptr(dx), _hip.stream_of(dy)),
               "sp_direct_conv3x3_bwd_input")
    return dx


class _Conv3x3Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, module):
        ctx.module = module
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x if weight.requires_grad else None, weight)
        ctx.x_shape = x.shape
        return conv3x3_forward(module, x)

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = conv3x3_input_vjp(ctx.module, dy, ctx.x_shape)
        if ctx.needs_input_grad[1]:
            dw = torch.nn.grad.conv2d_weight(x, weight.shape, dy.contiguous(), padding=1)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.sum(dim=(0, 2, 3))
        return dx, dw, db, None


def tile_pack(module: nn.Conv2d, algo: str, input_vjp: bool) -> Tensor:
    """``module``'s 3x3 weights transformed / packed for a stride-1 tile (``algo`` "wino" or
    "direct", forward or input VJP), cached on the module and rebuilt when the weight changes."""
    w = module.weight
    key = (w.data_ptr(), w._version, w.device)
    cache = module.__dict__.setdefault("_tile_packs", {})
    if cache.get("key") != key:
        cache.clear()
        cache["key"] = key
    if (algo, input_vjp) not in cache:
        lib = _hip.load_library()
        cout, cin = w.shape[0], w.shape[1]
        wc = w.detach().contiguous()
        size_fn, fn = ((lib.sp_wino3x3_packed_size, lib.sp_wino3x3_pack) if algo == "wino"
                       else (lib.sp_conv3x3_packed_size, lib.sp_conv3x3_pack))
        out = torch.empty(int(size_fn(cin, cout)), device=w.device)
        _hip.check(fn(_hip.ptr(wc), cout, cin, int(input_vjp), _hip.ptr(out), _hip.stream_of(wc)),
                   f"sp_{algo}3x3_pack")
        cache[(algo, input_vjp)] = out
    return cache[(algo, input_vjp)]


class Conv3x3(nn.Conv2d):
    """``nn.Conv2d(cin, cout, 3, padding=1)`` whose device forward / input VJP run this
    project's kernels: the fp32-MFMA tiles — Winograd F(2x2,3x3) (``csrc/sp_wino.hip``;
    cin % 8, cout % 64, W % 32 and H % 8, or 16x16, or 8x8) or the direct implicit GEMM
    (``csrc/sp_conv.hip``; cin % 4, cout % 128, H % 8, W % 32) — or, with few channels on
    one side (conv_in / conv_out), the thin VALU kernel (``csrc/sp_conv_thin.hip``);
    MIOpen elsewhere.  Transformed / packed weights are cached
    per algorithm and rebuilt when the parameter changes."""

    def __init__(self, cin: int, cout: int) -> None:
        super().__init__(cin, cout, 3, padding=1)

    def _pack(self, algo: str, input_vjp: bool) -> Tensor:
        return tile_pack(self, algo, input_vjp)

    def forward(self, x: Tensor) -> Tensor:
        if x.is_cuda and x.dtype == torch.bfloat16:
            from . import bf16
            if bf16.conv_supported(self, x):
                return bf16.conv3x3(self, x)
        if x.is_cuda and x.dtype == torch.float32 and x.dim() == 4:
            lib = _hip.load_library()
            n, cin, h, w = x.shape
            if _conv_algo(lib, cin, self.out_channels, h, w, conv_backend()) is not None:
                return _Conv3x3Fn.apply(x, self.weight, self.bias, self)
        miopen_fallback(x)
        return super().forward(x)


# ---------------------------------------------------------------------------------------
# 2x nearest upsampling of Upsample2D
# ---------------------------------------------------------------------------------------

def _upsample2x_call(fn_name: str, src: Tensor, out_shape) -> Tensor:
    lib = _hip.load_library()
    n, c, h, w = (src.shape if fn_name == "sp_upsample2x" else out_shape)
    src = src.contiguous()
    out = torch.empty(tuple(out_shape), device=src.device, dtype=torch.float32)
    _hip.check(getattr(lib, fn_name)(_hip.ptr(src), n * c, h, w, _hip.ptr(out),
                                     _hip.stream_of(src)), fn_name)
    return out


class _Upsample2xFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        n, c, h, w = x.shape
        ctx.x_shape = x.shape
        return _upsample2x_call("sp_upsample2x", x, (n, c, 2 * h, 2 * w))

    @staticmethod
    def backward(ctx, dy):
        return _upsample2x_call("sp_upsample2x_vjp", dy, ctx.x_shape)


def _upconv_enabled() -> bool:
    import os

    return os.environ.get("SAMPLERS_AMD_UPCONV", "1").lower() not in ("0", "off", "false")


def upsample_conv_supported(module: "Conv3x3", x: Tensor) -> bool:
    """``module(upsample_nearest2x(x))`` (diffusers Upsample2D) runs fused on the Winograd tile
    (``sp_wino3x3_fwd_up`` / ``sp_wino3x3_bwd_input_pool``): the upsampled tensor is never
    written.  Frozen weights only, and only where the unfused launches would not split K (an
    under-filled launch keeps the split unfused pair, which is faster there); the results are
    then bitwise the unfused pair's.  ``SAMPLERS_AMD_UPCONV=0`` turns it off."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.numel() > 0):
        return False
    if not _upconv_enabled() or conv_backend() != "auto" or module.weight.requires_grad:
        return False
    n, cin, h, w = x.shape
    cout = module.out_channels
    if not _query("sp_wino3x3_up_supported", cin, cout, 2 * h, 2 * w):
        return False
    return not split_k_enabled() or (_query("sp_wino3x3_workspace", n, cin, cout, 2 * h, 2 * w) <= 0 and
                                     _query("sp_wino3x3_workspace", n, cout, cin, 2 * h, 2 * w) <= 0)


class _UpsampleConv3x3Fn(torch.autograd.Function):
    """conv(upsample_nearest2x(x)) with the upsample inside the Winograd tile's input loads, and
    its VJP's 2x2 block sums inside the input-VJP tile's epilogue (``csrc/sp_wino.hip``, UP)."""

    @staticmethod
    def forward(ctx, x, weight, bias, module):
        lib = _hip.load_library()
        n, cin, h, w = x.shape
        cout = module.out_channels
        ctx.module, ctx.x_shape = module, x.shape
        x = x.contiguous()
        y = torch.empty(n, cout, 2 * h, 2 * w, device=x.device, dtype=torch.float32)
        _hip.check(lib.sp_wino3x3_fwd_up(_hip.ptr(x), _hip.ptr(tile_pack(module, "wino", False)),
                                         _hip.ptr(bias), n, cin, cout, 2 * h, 2 * w, _hip.ptr(y),
                                         _hip.stream_of(x)), "sp_wino3x3_fwd_up")
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _hip.load_library()
        n, cin, h, w = ctx.x_shape
        cout = ctx.module.out_channels
        dy = dy.contiguous()
        dx = torch.empty(tuple(ctx.x_shape), device=dy.device, dtype=torch.float32)
        _hip.check(lib.sp_wino3x3_bwd_input_pool(_hip.ptr(dy), _hip.ptr(tile_pack(ctx.module, "wino", True)),
                                                 n, cin, cout, 2 * h, 2 * w, _hip.ptr(dx),
                                                 _hip.stream_of(dy)), "sp_wino3x3_bwd_input_pool")
        return dx, None, None, None


def upsample_conv(module: "Conv3x3", x: Tensor) -> Tensor:
    """``module(upsample_nearest2x(x))``: fused where ``upsample_conv_supported``, else the pair."""
    if x.is_cuda and x.dtype == torch.bfloat16:
        from . import bf16
        if bf16.upsample_conv_supported(module, x):
            return bf16.upsample_conv3x3(module, x)
    if upsample_conv_supported(module, x):
        return _UpsampleConv3x3Fn.apply(x, module.weight, module.bias, module)
    return module(upsample_nearest2x(x))


def upsample_nearest2x(x: Tensor) -> Tensor:
    """``F.interpolate(x, scale_factor=2.0, mode="nearest")``: the streaming kernels of
    ``csrc/sp_upsample.hip`` (forward and the 2x2-block-sum VJP) on fp32 CUDA tensors whose
    width is a multiple of 4, torch elsewhere."""
    if (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and x.numel() > 0 and
            _hip.load_library().sp_upsample2x_supported(x.shape[2], x.shape[3])):
        return _Upsample2xFn.apply(x)
    return F.interpolate(x, scale_factor=2.0, mode="nearest")


# ---------------------------------------------------------------------------------------
# 3x3 / stride 2 convolution of Downsample2D (zero row / column bottom / right) on fp32 MFMA
# ---------------------------------------------------------------------------------------

def _s2_packed(module: nn.Conv2d, input_vjp: bool) -> Tensor:
    w = module.weight
    key = (w.data_ptr(), w._version, w.device)
    cache = module.__dict__.setdefault("_s2_packs", {})
    if cache.get("key") != key:
        cache.clear()
        cache["key"] = key
    if input_vjp not in cache:
        lib = _hip.load_library()
        cout, cin = w.shape[0], w.shape[1]
        wc = w.detach().contiguous()
        out = torch.empty(cin * cout * 9, device=w.device)
        _hip.check(lib.sp_conv3x3_s2_pack(_hip.ptr(wc), cout, cin, int(input_vjp), _hip.ptr(out),
                                          _hip.stream_of(wc)), "sp_conv3x3_s2_pack")
        cache[input_vjp] = out
    return cache[input_vjp]


def downsample_s2_supported(module: nn.Conv2d, x: Tensor) -> bool:
    """The stride-2 tile serves this call (forward and input VJP shape rules)."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4) or conv_backend() == "miopen":
        return False
    lib = _hip.load_library()
    _, cin, h, w = x.shape
    cout = module.out_channels
    return bool(lib.sp_conv3x3_s2_supported(cin, cout, h, w, 0) and
                lib.sp_conv3x3_s2_supported(cin, cout, h, w, 1))


class SkipGrad:
    """Hand-off of a UNet skip tensor's gradient from its up-block consumer (which runs
    first in the backward pass) to its down-path consumer, which adds it inside its own
    input-VJP kernel (GroupNorm's second addend, or the stride-2 conv's accumulate mode)
    instead of autograd's separate accumulation add.  ``enabled`` is cleared in the forward
    pass when the down-path consumer cannot take it (the autograd add then happens)."""

    __slots__ = ("grad", "enabled")

    def __init__(self) -> None:
        self.grad: Tensor | None = None
        self.enabled = True

    def take(self) -> Tensor | None:
        """The delivered gradient, or ``None`` when the up-block consumer did not deliver one
        (it fell back to the autograd path, which then accumulates its gradient itself)."""
        g, self.grad = self.grad, None
        return g


def _s2_workspace(lib, n: int, cin: int, cout: int, h: int, w: int, vjp: int, device) -> tuple[Tensor | None, int]:
    """The stride-2 tile's split-K workspace for an under-filled launch (sp_conv3x3_s2_workspace)
    and its bytes, or (None, 0); allocated as _wino_workspace."""
    nb = _query("sp_conv3x3_s2_workspace", n, cin, cout, h, w, vjp) if split_k_enabled() else 0
    if nb <= 0:
        return None, 0
    return torch.empty(nb // 4, device=device, dtype=torch.float32), nb


class _ConvS2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, module, box=None):
        lib = _hip.load_library()
        x = x.contiguous()
        n, cin, h, w = x.shape
        cout = module.out_channels
        y = torch.empty(n, cout, h // 2, w // 2, device=x.device, dtype=torch.float32)
        ws, nb = _s2_workspace(lib, n, cin, cout, h, w, 0, x.device)
        _hip.check(lib.sp_conv3x3_s2_fwd_ws(_hip.ptr(x), _hip.ptr(_s2_packed(module, False)),
                                            _hip.ptr(bias.contiguous()) if bias is not None else None,
                                            n, cin, cout, h, w, _hip.ptr(y), _hip.ptr(ws), nb, _hip.stream_of(x)),
                   "sp_conv3x3_s2_fwd")
        ctx.module = module
        ctx.box = box
        ctx.x_shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        """Input VJP only: the tile serves frozen weights (``downsample_conv``)."""
        dx = None
        if ctx.needs_input_grad[0]:
            lib = _hip.load_library()
            n, cin, h, w = ctx.x_shape
            # with a skip gradient pending, accumulate into its buffer (dx = skip grad + VJP)
            dx = ctx.box.take() if ctx.box is not None else None
            acc = dx is not None
            if dx is None:
                dx = torch.empty(tuple(ctx.x_shape), device=dy.device, dtype=torch.float32)
            ws, nb = _s2_workspace(lib, n, cin, ctx.module.out_channels, h, w, 1, dy.device)
            _hip.check(lib.sp_conv3x3_s2_bwd_input_ws(_hip.ptr(dy.contiguous()),
                                                      _hip.ptr(_s2_packed(ctx.module, True)),
                                                      n, cin, ctx.module.out_channels, h, w, int(acc),
                                                      _hip.ptr(dx), _hip.ptr(ws), nb, _hip.stream_of(dy)),
                       "sp_conv3x3_s2_bwd_input")
        return dx, None, None, None, None


# A 3x3 / stride-2 convolution is the stride-1 / padding-1 convolution read at every other
# position: with padding 1 on all sides (diffusers' downsample_padding=1) at the even rows and
# columns, with one zero row / column bottom / right (downsample_padding=0) at the odd ones.
# Where no stride-2 tile serves a shape (channels or widths outside its rules), the stride-1
# MFMA tiles compute it at full resolution (4x the MACs, on tiles ~50x faster than MIOpen's
# naive kernel that these shapes otherwise reach); the input VJP is the stride-1 VJP of dy
# scattered to those positions (zeros elsewhere).

def strided_full_supported(module: nn.Conv2d, x: Tensor) -> bool:
    """The stride-1 tiles serve ``module`` (3x3, frozen weights) at ``x``'s full resolution,
    forward and input VJP."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4) or module.weight.requires_grad:
        return False
    backend = conv_backend()
    if backend == "miopen":
        return False
    lib = _hip.load_library()
    _, cin, h, w = x.shape
    cout = module.out_channels
    fwd = _conv_algo(lib, cin, cout, h, w, backend)
    vjp = _conv_algo(lib, cout, cin, h, w, backend)
    ok = ("wino", "direct")
    return h % 2 == 0 and w % 2 == 0 and fwd in ok and vjp in ok


class _ConvS2FullFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, module, phase):
        y = conv3x3_forward(module, x.contiguous())
        ctx.module, ctx.phase, ctx.x_shape = module, phase, x.shape
        return y[:, :, phase::2, phase::2].contiguous()

    @staticmethod
    def backward(ctx, dy):
        dx = None
        if ctx.needs_input_grad[0]:
            n, _, h, w = ctx.x_shape
            dyf = dy.new_zeros((n, ctx.module.out_channels, h, w))
            dyf[:, :, ctx.phase::2, ctx.phase::2] = dy
            dx = conv3x3_input_vjp(ctx.module, dyf, ctx.x_shape)
        return dx, None, None, None, None


def conv3x3_stride2(module: nn.Conv2d, x: Tensor, padding: int) -> Tensor:
    """``module(x)`` for a 3x3 / stride-2 ``nn.Conv2d`` with ``padding=1`` (``padding=1``), or
    ``module(F.pad(x, (0, 1, 0, 1)))`` with ``padding=0``, through the stride-1 tiles at full
    resolution where they serve the shape, else torch / MIOpen."""
    if x.is_cuda and x.dtype == torch.bfloat16:
        from . import bf16
        if bf16.strided_supported(module, x):
            return bf16.conv3x3_stride2(module, x, padding)
    if strided_full_supported(module, x):
        return _ConvS2FullFn.apply(x, module.weight, module.bias, module, 0 if padding else 1)
    miopen_fallback(x)
    return module(x) if padding else module(F.pad(x, (0, 1, 0, 1)))


def downsample_conv(module: nn.Conv2d, x: Tensor, box: SkipGrad | None = None) -> Tensor:
    """``module(F.pad(x, (0, 1, 0, 1)))`` for a 3x3 / stride-2 / padding-0 ``nn.Conv2d``
    (diffusers' Downsample2D with downsample_padding=0): the stride-2 MFMA tile
    (``csrc/sp_conv_s2.hip``) where its shape rules hold, else the stride-1 tiles at full
    resolution (``conv3x3_stride2``), else MIOpen on the padded input."""
    if x.is_cuda and x.dtype == torch.bfloat16:
        if box is not None:
            box.enabled = False
        return conv3x3_stride2(module, x, padding=0)
    if downsample_s2_supported(module, x) and not module.weight.requires_grad:
        return _ConvS2Fn.apply(x, module.weight, module.bias, module,
                               box if box is not None and box.enabled else None)
    if box is not None:
        box.enabled = False
    return conv3x3_stride2(module, x, padding=0)


# ---------------------------------------------------------------------------------------
# nn.Linear on token-major activations: fp32 arithmetic on the bf16 MFMAs (csrc/sp_gemm_x6.hip)
# ---------------------------------------------------------------------------------------

def x6_enough_tiles(rows: int, cols: int) -> bool:
    """Whether a bf16x6 GEMM call of ``rows`` pixels / tokens x ``cols`` output features should
    run on the x6 tile: at least ``SAMPLERS_AMD_X6_MIN_TILES`` of its 256 x 128 output tiles
    (default 0: always — measured, round 4: sending the calls below 128 tiles to hipBLASLt's
    fp32 GEMM made the batch-1 DPS step 14.6 -> 28.1 ms, hipBLASLt's choices for these small
    shapes being worse still; profiles/round4/b1/x6_min_tiles_ab.txt)."""
    import os

    need = int(os.environ.get("SAMPLERS_AMD_X6_MIN_TILES", "0"))
    return need <= 0 or -(-rows // 256) * -(-cols // 128) >= need


def linear_backend() -> str:
    """``SAMPLERS_AMD_LINEAR``: ``x6`` (default: ``sp_linear_x6`` where its shape rules hold —
    exact three-term bf16 splits of the fp32 operands, six partial products, fp32
    accumulation) or ``torch`` (hipBLASLt fp32)."""
    import os

    return os.environ.get("SAMPLERS_AMD_LINEAR", "x6").lower()


def _linear_pack(module: nn.Module, w2d: Tensor, trans: bool) -> Tensor:
    """``w2d`` ([out, in]) packed for sp_linear_x6 (trans: as Wᵀ for the input VJP), cached on
    ``module`` and rebuilt when the weight changes."""
    key = (w2d.data_ptr(), module.weight._version, w2d.device)
    cache = module.__dict__.setdefault("_x6_linear_packs", {})
    if cache.get("key") != key:
        cache.clear()
        cache["key"] = key
    if trans not in cache:
        lib = _hip.load_library()
        m, k = w2d.shape
        wc = w2d.detach().contiguous()
        rows, cols = (k, m) if trans else (m, k)
        out = torch.empty(int(lib.sp_gemm_x6_packed_size(rows, cols)), device=w2d.device)
        _hip.check(lib.sp_gemm_x6_pack(_hip.ptr(wc), rows, cols, int(trans), _hip.ptr(out), _hip.stream_of(wc)),
                   "sp_gemm_x6_pack")
        cache[trans] = out
    return cache[trans]


class _LinearX6Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, module, w2d, res=None, box=None):
        lib = _hip.load_library()
        m, k = w2d.shape
        x2 = x.reshape(-1, k).contiguous()
        t = x2.shape[0]
        y = torch.empty(t, m, device=x.device, dtype=torch.float32)
        r2 = None if res is None else res.reshape(t, m).contiguous()
        ws, nb = x6_workspace(lib, 1, t, k, m, x.device)
        _hip.check(lib.sp_linear_x6_ws(_hip.ptr(x2), _hip.ptr(_linear_pack(module, w2d, False)),
                                       _hip.ptr(None if bias is None else bias.detach().contiguous()),
                                       _hip.ptr(r2), t, k, m, _hip.ptr(y), _hip.ptr(ws), nb, _hip.stream_of(x2)),
                   "sp_linear_x6")
        ctx.module, ctx.w2d, ctx.shape = module, w2d, x.shape
        ctx.box = box if res is not None else None
        return y.reshape(*x.shape[:-1], m)

    @staticmethod
    def backward(ctx, dy):
        """Input VJP only (the priors' weights are frozen): dx = dy W; the residual's gradient
        is dy itself — handed to ``box`` (the LayerNorm VJP that adds it) when one was given."""
        lib = _hip.load_library()
        m, k = ctx.w2d.shape
        d2 = dy.reshape(-1, m).contiguous()
        t = d2.shape[0]
        dx = torch.empty(t, k, device=dy.device, dtype=torch.float32)
        ws, nb = x6_workspace(lib, 1, t, m, k, dy.device)
        _hip.check(lib.sp_linear_x6_ws(_hip.ptr(d2), _hip.ptr(_linear_pack(ctx.module, ctx.w2d, True)), None, None,
                                       t, m, k, _hip.ptr(dx), _hip.ptr(ws), nb, _hip.stream_of(d2)), "sp_linear_x6")
        dres = None
        if ctx.needs_input_grad[5]:
            if ctx.box is not None and ctx.box.enabled:
                ctx.box.grad = d2
            else:
                dres = dy
        return dx.reshape(ctx.shape), None, None, None, None, dres, None


def linear(x: Tensor, module: nn.Module, w2d: Tensor | None = None, bias: Tensor | None = None,
           res: Tensor | None = None, box: "SkipGrad | None" = None) -> Tensor:
    """``F.linear(x, w2d, bias) (+ res)`` (``w2d`` defaults to ``module.weight``, ``bias`` to
    ``module.bias``) on ``sp_linear_x6`` when x is a CUDA fp32 token-major batch whose token
    count and widths fit its rules and the weights are frozen; hipBLASLt otherwise.  ``res``
    (shaped like the output) is added in the GEMM's epilogue; its gradient goes to ``box``
    when the residual's other consumer (a ``LayerNorm`` given the same box) adds it in its VJP."""
    w2d = module.weight if w2d is None else w2d
    bias = getattr(module, "bias", None) if bias is None else bias
    if batch_invariant_enabled() and x.dim() == 3 and x.shape[0] > 1:
        # one batch entry per call: the backend (x6 tile or hipBLASLt) and hipBLASLt's algorithm
        # are chosen from the token count, which would otherwise include the batch
        if box is not None:
            box.enabled = False
        y = torch.cat([linear(x[i:i + 1], module, w2d, bias) for i in range(x.shape[0])])
        return y if res is None else y + res
    m, k = w2d.shape
    t = x.numel() // k if x.dim() else 0
    if (x.is_cuda and x.dtype == torch.float32 and not w2d.requires_grad
            and (bias is None or not bias.requires_grad) and linear_backend() == "x6"
            and (res is None or (res.dtype == torch.float32 and res.numel() == t * m))):
        if _query("sp_linear_x6_supported", t, k, m) and x6_enough_tiles(t, m):
            return _LinearX6Fn.apply(x, w2d, bias, module, w2d, res, box)
    if (res is not None and x.is_cuda and x.dtype == torch.bfloat16 and res.dtype == torch.bfloat16
            and not w2d.requires_grad and (bias is None or not bias.requires_grad) and res.shape[-1] == m):
        from . import bf16
        return bf16.linear_res(x, w2d, bias, res, box)
    if box is not None:
        box.enabled = False
    y = F.linear(x, w2d, bias)
    return y if res is None else y + res


class _ProjLayoutFn(torch.autograd.Function):
    """1x1 projection between the NCHW planes and token-major rows (``sp_gemm_x6_layout``)."""

    @staticmethod
    def forward(ctx, x, weight, bias, module, w2d, n, hw, in_tm, out_tm, res=None, box=None):
        lib = _hip.load_library()
        m, k = w2d.shape
        xc = x.contiguous()
        y = torch.empty((n * hw, m) if out_tm else (n, m, hw), device=x.device, dtype=torch.float32)
        rc = None if res is None else res.contiguous()
        ws, nb = x6_workspace(lib, n, hw, k, m, x.device)
        _hip.check(lib.sp_gemm_x6_layout_ws(_hip.ptr(xc), _hip.ptr(_linear_pack(module, w2d, False)),
                                            _hip.ptr(None if bias is None else bias.detach().contiguous()),
                                            _hip.ptr(rc), n, hw, k, m, int(in_tm), int(out_tm), _hip.ptr(y),
                                            _hip.ptr(ws), nb, _hip.stream_of(xc)), "sp_gemm_x6_layout")
        ctx.module, ctx.w2d, ctx.geo, ctx.shape = module, w2d, (n, hw, in_tm, out_tm), x.shape
        ctx.res_shape = None if res is None else res.shape
        ctx.box = box if res is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        lib = _hip.load_library()
        m, k = ctx.w2d.shape
        n, hw, in_tm, out_tm = ctx.geo
        dc = dy.contiguous()
        dx = torch.empty((n * hw, k) if in_tm else (n, k, hw), device=dy.device, dtype=torch.float32)
        ws, nb = x6_workspace(lib, n, hw, m, k, dy.device)
        _hip.check(lib.sp_gemm_x6_layout_ws(_hip.ptr(dc), _hip.ptr(_linear_pack(ctx.module, ctx.w2d, True)),
                                            None, None, n, hw, m, k, int(out_tm), int(in_tm), _hip.ptr(dx),
                                            _hip.ptr(ws), nb, _hip.stream_of(dc)), "sp_gemm_x6_layout")
        dres = None
        if ctx.res_shape is not None and ctx.needs_input_grad[9]:
            if ctx.box is not None and ctx.box.enabled:
                ctx.box.grad = dc.reshape(ctx.res_shape)  # summed by the norm's VJP kernel
            else:
                dres = dy.reshape(ctx.res_shape)
        return dx.reshape(ctx.shape), None, None, None, None, None, None, None, None, dres, None


def _layout_ok(x: Tensor, w2d: Tensor, n: int, hw: int) -> bool:
    m, k = w2d.shape
    return (x.is_cuda and x.dtype == torch.float32 and not w2d.requires_grad and linear_backend() == "x6"
            and bool(_hip.load_library().sp_gemm_x6_layout_supported(n, hw, k, m))
            and x6_enough_tiles(n * hw, m))


def proj_nchw_to_tokens(x: Tensor, module, w2d: Tensor | None = None, bias: Tensor | None = None) -> Tensor:
    """A 1x1 projection (``module``: a 1x1 ``nn.Conv2d``, an ``nn.Linear`` or a weight holder;
    ``w2d`` [c_out][c] defaults to its weight) of NCHW ``x``, returned as token rows
    ``(b, h w, c_out)``: the transpose happens in the GEMM's stores (HIP, CUDA fp32, frozen
    weights), else reshape + transpose + linear in torch."""
    b, c, h, w = x.shape
    if batch_invariant_enabled() and b > 1 and x.is_cuda:
        # one sample per call: the backend (x6 tile or hipBLASLt) follows the per-call row count
        # (sp_gemm_x6_layout_supported's size guard, hipBLASLt's algorithm), never the batch
        return torch.cat([proj_nchw_to_tokens(x[i:i + 1], module, w2d, bias) for i in range(b)])
    w2d = module.weight.reshape(module.weight.shape[0], c) if w2d is None else w2d
    bias = getattr(module, "bias", None) if bias is None else bias
    co = w2d.shape[0]
    if _layout_ok(x, w2d, b, h * w):
        y = _ProjLayoutFn.apply(x, w2d, bias, module, w2d, b, h * w, False, True, None)
        return y.reshape(b, h * w, co)
    return linear(x.reshape(b, c, h * w).transpose(1, 2), module, w2d, bias)


def proj_tokens_to_nchw(tokens: Tensor, module, res: Tensor, w2d: Tensor | None = None,
                        bias: Tensor | None = None, box: SkipGrad | None = None) -> Tensor:
    """The reverse projection: token rows ``(b, h w, c)`` to NCHW, plus the residual ``res``
    (b, c_out, h, w) in the epilogue (HIP), else torch.  ``box``: the residual's gradient goes
    to the norm that reads ``res`` (``GroupNormAct(..., box=box)``)."""
    b, co, h, w = res.shape
    c = tokens.shape[-1]
    if batch_invariant_enabled() and b > 1 and tokens.is_cuda:  # one sample per call, as above
        if box is not None:
            box.enabled = False
        return torch.cat([proj_tokens_to_nchw(tokens[i:i + 1], module, res[i:i + 1], w2d, bias)
                          for i in range(b)])
    w2d = module.weight.reshape(co, c) if w2d is None else w2d
    bias = getattr(module, "bias", None) if bias is None else bias
    if _layout_ok(tokens, w2d, b, h * w) and res.dtype == torch.float32:
        y = _ProjLayoutFn.apply(tokens, w2d, bias, module, w2d, b, h * w, True, False, res, box)
        return y.reshape(b, co, h, w)
    if box is not None:
        box.enabled = False
    out = linear(tokens, module, w2d, bias)
    return out.transpose(1, 2).reshape(b, co, h, w) + res


class _Conv1x1SmallFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        lib = _hip.load_library()
        n, c, h, w = x.shape
        co = weight.shape[0]
        xc = x.contiguous()
        y = torch.empty(n, co, h, w, device=x.device, dtype=torch.float32)
        _hip.check(lib.sp_conv1x1_small(_hip.ptr(xc), _hip.ptr(weight), _hip.ptr(bias), n, c, co, h * w, 0,
                                        _hip.ptr(y), _hip.stream_of(xc)), "sp_conv1x1_small")
        ctx.save_for_backward(weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        (weight,) = ctx.saved_tensors
        lib = _hip.load_library()
        n, co, h, w = dy.shape
        c = weight.shape[1]
        dc = dy.contiguous()
        dx = torch.empty(n, c, h, w, device=dy.device, dtype=torch.float32)
        _hip.check(lib.sp_conv1x1_small(_hip.ptr(dc), _hip.ptr(weight), None, n, co, c, h * w, 1,
                                        _hip.ptr(dx), _hip.stream_of(dc)), "sp_conv1x1_small")
        return dx, None, None


def conv1x1_small(conv: nn.Conv2d, x: Tensor) -> Tensor:
    """``conv(x)`` for the VAE's 4- / 8-channel 1x1 quant convs on a HIP kernel (CUDA fp32,
    frozen weights), else torch."""
    co, c = conv.weight.shape[:2]
    if x.is_cuda and x.dtype == torch.bfloat16 and not conv.weight.requires_grad:
        from . import bf16
        return bf16.pointwise(x, conv.weight, conv.bias)
    if (x.is_cuda and x.dtype == torch.float32 and not conv.weight.requires_grad
            and (conv.bias is None or not conv.bias.requires_grad)
            and _hip.load_library().sp_conv1x1_small_supported(c, co, x.shape[2] * x.shape[3])):
        w2d = conv.weight.detach().reshape(co, c).contiguous()
        b = None if conv.bias is None else conv.bias.detach().contiguous()
        return _Conv1x1SmallFn.apply(x, w2d, b)
    miopen_fallback(x)
    return conv(x)


class Linear(nn.Linear):
    """``nn.Linear`` (same parameters and state-dict keys) whose device forward / input VJP run
    ``sp_linear_x6`` where it applies (``linear``)."""

    def forward(self, x: Tensor, res: Tensor | None = None, box: "SkipGrad | None" = None) -> Tensor:
        return linear(x, self, res=res, box=box)


# ---- transformer-block glue: LayerNorm, GEGLU (csrc/sp_transformer.hip) -------------------
def _hip_rows_ok(x: Tensor, *params: Tensor | None) -> bool:
    return (x.is_cuda and x.dtype == torch.float32
            and all(p is None or not p.requires_grad for p in params))


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, box):
        lib = _hip.load_library()
        c = x.shape[-1]
        x2 = x.reshape(-1, c).contiguous()
        rows = x2.shape[0]
        y = torch.empty_like(x2)
        stats = torch.empty(2, rows, device=x.device, dtype=torch.float32)
        _hip.check(lib.sp_layernorm_fwd(_hip.ptr(x2), _hip.ptr(weight), _hip.ptr(bias), rows, c, float(eps),
                                        _hip.ptr(y), _hip.ptr(stats[0]), _hip.ptr(stats[1]),
                                        _hip.stream_of(x2)), "sp_layernorm_fwd")
        ctx.save_for_backward(x2, weight, stats)
        ctx.box, ctx.shape = box, x.shape
        return y.reshape(x.shape)

    @staticmethod
    def backward(ctx, dy):
        """Input VJP (frozen weights), plus the residual branch's gradient of the same tensor
        when its consumer handed it over (``box``)."""
        x2, weight, stats = ctx.saved_tensors
        lib = _hip.load_library()
        rows, c = x2.shape
        d2 = dy.reshape(rows, c).contiguous()
        add = ctx.box.take() if ctx.box is not None else None
        dx = torch.empty_like(x2)
        _hip.check(lib.sp_layernorm_bwd(_hip.ptr(d2), _hip.ptr(x2), _hip.ptr(weight), _hip.ptr(stats[0]),
                                        _hip.ptr(stats[1]), _hip.ptr(add), rows, c, _hip.ptr(dx),
                                        _hip.stream_of(d2)), "sp_layernorm_bwd")
        return dx.reshape(ctx.shape), None, None, None, None


def layer_norm(x: Tensor, module: nn.LayerNorm, box: SkipGrad | None = None) -> Tensor:
    """``module(x)`` (torch.nn.LayerNorm over the last dim, elementwise affine) on the HIP row
    kernel for CUDA fp32 activations with frozen parameters, else torch.  ``box``: the residual
    gradient of ``x`` that a ``linear(..., res=x, box=box)`` consumer hands over, added inside
    the VJP kernel."""
    c = x.shape[-1]
    if (_hip_rows_ok(x, module.weight, module.bias) and module.weight is not None
            and tuple(module.normalized_shape) == (c,)):
        lib = _hip.load_library()
        if lib.sp_layernorm_supported(x.numel() // c, c):
            return _LayerNormFn.apply(x, module.weight.detach().contiguous(),
                                      module.bias.detach().contiguous(), module.eps, box)
    if x.is_cuda and x.dtype == torch.bfloat16:
        from . import bf16
        if bf16.layer_norm_supported(module, x):
            return bf16.layer_norm(x, module, box)
    if box is not None:
        box.enabled = False
    return F.layer_norm(x, module.normalized_shape, module.weight, module.bias, module.eps)


class LayerNorm(nn.LayerNorm):
    """``nn.LayerNorm`` (same parameters and state-dict keys) on ``sp_layernorm_fwd/bwd``."""

    def forward(self, x: Tensor, box: SkipGrad | None = None) -> Tensor:
        return layer_norm(x, self, box)


class _GegluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h):
        lib = _hip.load_library()
        f = h.shape[-1] // 2
        h2 = h.reshape(-1, 2 * f).contiguous()
        rows = h2.shape[0]
        y = torch.empty(rows, f, device=h.device, dtype=torch.float32)
        _hip.check(lib.sp_geglu_fwd(_hip.ptr(h2), rows, f, _hip.ptr(y), _hip.stream_of(h2)), "sp_geglu_fwd")
        ctx.save_for_backward(h2)
        ctx.shape = h.shape
        return y.reshape(*h.shape[:-1], f)

    @staticmethod
    def backward(ctx, dy):
        (h2,) = ctx.saved_tensors
        lib = _hip.load_library()
        rows, f2 = h2.shape
        d2 = dy.reshape(rows, f2 // 2).contiguous()
        dh = torch.empty_like(h2)
        _hip.check(lib.sp_geglu_bwd(_hip.ptr(h2), _hip.ptr(d2), rows, f2 // 2, _hip.ptr(dh), _hip.stream_of(d2)),
                   "sp_geglu_bwd")
        return dh.reshape(ctx.shape)


def geglu(h: Tensor) -> Tensor:
    """``a * gelu(gate)`` with ``a, gate = h.chunk(2, -1)`` (diffusers GEGLU after its
    projection): one HIP pass each way on CUDA fp32 and bf16, torch otherwise."""
    f = h.shape[-1] // 2
    if (h.is_cuda and h.dtype == torch.float32 and h.shape[-1] % 8 == 0
            and (h.numel() // 2) < 2**31):
        return _GegluFn.apply(h)
    if h.is_cuda and h.dtype == torch.bfloat16:
        from . import bf16
        if bf16.geglu_supported(h):
            return bf16.geglu(h)
    a, gate = h.chunk(2, dim=-1)
    return a * F.gelu(gate)

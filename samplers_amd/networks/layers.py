"""Fused GroupNorm (+ time-embedding bias) (+ SiLU) for the priors.

``GroupNormAct`` is a drop-in ``nn.GroupNorm`` (same parameters, same state-dict
keys) whose forward optionally adds a per-(sample, channel) bias to its input and
applies SiLU to its output — the ``norm -> silu`` pairs and the ``h + temb`` add of
diffusers' ``ResnetBlock2D`` that the reference's priors run
(``/root/reference/samplers/networks/diffusers/ddpm.py:40-43``,
``stable_diffusion.py:330-345``).  On device tensors it runs the HIP kernels of
``csrc/sp_groupnorm.hip`` (``sp_groupnorm_silu_fwd/bwd``) through a
``torch.autograd.Function`` whose backward is the fused input VJP; on CPU tensors
(the oracle's CPU baseline and the CPU tests) it is plain torch.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from .. import _hip


def group_norm_act_torch(x: Tensor, groups: int, weight: Tensor | None, bias: Tensor | None,
                         eps: float, act: bool, chan_bias: Tensor | None = None) -> Tensor:
    """Plain-torch semantics of the fused op (CPU path and test reference)."""
    if chan_bias is not None:
        x = x + chan_bias[:, :, None, None]
    y = F.group_norm(x, groups, weight, bias, eps)
    return F.silu(y) if act else y


class _GroupNormActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, chan_bias, groups: int, eps: float, act: bool):
        lib = _hip.load_library()
        n, c = x.shape[0], x.shape[1]
        hw = x[0, 0].numel() if x.numel() else 1
        x = x.contiguous()
        z = torch.empty_like(x)
        stats = torch.empty(2, n * groups, device=x.device, dtype=torch.float32)
        work = torch.empty(max(int(lib.sp_groupnorm_workspace(n, c, hw, groups)), 1),
                           device=x.device, dtype=torch.float32)
        cb = None if chan_bias is None else chan_bias.contiguous()
        _hip.check(lib.sp_groupnorm_silu_fwd(
            _hip.ptr(x), _hip.ptr(cb), _hip.ptr(weight), _hip.ptr(bias), n, c, hw, groups,
            float(eps), int(act), _hip.ptr(z), _hip.ptr(stats[0]), _hip.ptr(stats[1]),
            _hip.ptr(work), _hip.stream_of(x)), "sp_groupnorm_silu_fwd")
        ctx.save_for_backward(x, weight, bias, cb, stats)
        ctx.cfg = (groups, float(eps), bool(act))
        return z

    @staticmethod
    def backward(ctx, dz):
        x, weight, bias, cb, stats = ctx.saved_tensors
        groups, eps, act = ctx.cfg
        lib = _hip.load_library()
        n, c = x.shape[0], x.shape[1]
        hw = x[0, 0].numel() if x.numel() else 1
        dz = dz.contiguous()
        dx = torch.empty_like(x)
        work = torch.empty(max(int(lib.sp_groupnorm_workspace(n, c, hw, groups)), 1),
                           device=x.device, dtype=torch.float32)
        _hip.check(lib.sp_groupnorm_silu_bwd(
            _hip.ptr(dz), _hip.ptr(x), _hip.ptr(cb), _hip.ptr(weight), _hip.ptr(bias),
            _hip.ptr(stats[0]), _hip.ptr(stats[1]), n, c, hw, groups, int(act), _hip.ptr(dx),
            _hip.ptr(work), _hip.stream_of(x)), "sp_groupnorm_silu_bwd")
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
        return dx, d_w, d_b, d_cb, None, None, None


class GroupNormAct(nn.GroupNorm):
    """``nn.GroupNorm`` with an optional fused input bias and SiLU (``act=True``)."""

    def __init__(self, num_groups: int, num_channels: int, eps: float = 1e-5, affine: bool = True,
                 act: bool = False) -> None:
        super().__init__(num_groups, num_channels, eps=eps, affine=affine)
        self.act = act

    def forward(self, x: Tensor, chan_bias: Tensor | None = None) -> Tensor:
        if not x.is_cuda:
            return group_norm_act_torch(x, self.num_groups, self.weight, self.bias, self.eps,
                                        self.act, chan_bias)
        if x.dtype != torch.float32:
            raise _hip.HipLibraryError(f"GroupNormAct computes in fp32, got {x.dtype}")
        return _GroupNormActFn.apply(x, self.weight, self.bias, chan_bias, self.num_groups,
                                     self.eps, self.act)

    def extra_repr(self) -> str:
        return super().extra_repr() + f", act={'silu' if self.act else 'none'}"

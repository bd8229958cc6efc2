"""Pixel-space DDPM prior: a structural equivalent of diffusers' ``UNet2DModel``.

The reference never builds this network itself; ``DDPMNetwork.forward`` is
``self.unet(sample=sample, timestep=t).sample`` over a diffusers
``UNet2DModel`` loaded by name (``/root/reference/samplers/networks/diffusers/
ddpm.py:40-43``).  Neither diffusers nor the checkpoint is available here, so
this module rebuilds the architecture of ``google/ddpm-celebahq-256`` (six
levels of 128/128/256/256/512/512 channels, two residual blocks per level,
single-head self-attention at 16x16, GroupNorm(32, eps=1e-6) + SiLU,
sinusoidal time embedding with ``freq_shift=1``) with random weights.  It is
the prior of the hot path.  PyTorch-ROCm drives it (module graph, autograd of the input
VJP), but its layers run this project's HIP kernels (``samplers_amd/csrc``): 3x3 convs on
the fp32-MFMA Winograd / stride-2 / thin tiles, GroupNorm(+SiLU) single-pass kernels, the
1x1 shortcuts and attention projections on the split-bf16 GEMM, nearest upsampling; the
16x16 attention's scores / softmax stay batched hipBLASLt GEMMs (about 1 % of the step).

Parameters can be loaded from a local safetensors file whose keys follow the
diffusers naming (``load_state_dict`` accepts them unchanged), so a real
checkpoint drops in without network access.
"""

from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from .. import _hip
from ..runtime import batch_invariant_enabled
from .layers import (Conv3x3, GroupNormAct, Linear, SkipGrad, conv3x3_forward, conv3x3_input_vjp,
                     downsample_conv, gn_backward, gn_forward, miopen_fallback, proj_nchw_to_tokens,
                     proj_tokens_to_nchw, upsample_conv, upsample_nearest2x, x6_enough_tiles, x6_workspace,
                     _query)


@dataclass(frozen=True)
class UNet2DConfig:
    sample_size: int = 256
    in_channels: int = 3
    out_channels: int = 3
    block_out_channels: tuple[int, ...] = (128, 128, 256, 256, 512, 512)
    # index of the levels carrying self-attention (AttnDownBlock2D / AttnUpBlock2D)
    attention_levels: tuple[int, ...] = (4,)
    layers_per_block: int = 2
    norm_num_groups: int = 32
    norm_eps: float = 1e-6
    freq_shift: int = 1
    flip_sin_to_cos: bool = False
    attention_head_dim: int | None = None  # None -> one head spanning all channels


CELEBAHQ_256 = UNet2DConfig()


def timestep_embedding(t: Tensor, dim: int, *, flip_sin_to_cos: bool, freq_shift: float) -> Tensor:
    """Sinusoidal embedding of integer timesteps (``Timesteps`` in diffusers)."""
    half = dim // 2
    exponent = -math.log(10000.0) * torch.arange(half, dtype=torch.float32, device=t.device)
    exponent = exponent / (half - freq_shift)
    emb = t.float()[:, None] * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


def temb_projection_groups(model: nn.Module, emb: Tensor) -> list[tuple[list[int], Tensor]]:
    """Every ResnetBlock2D's ``time_emb_proj(silu(emb))`` of ``model`` at once: one SiLU and one
    batched GEMM per projection width (the blocks' weights stacked, cached on the model) instead
    of a SiLU, a copy and a GEMM per block — 3 launches instead of ~70 per UNet forward, which
    is most of the step's launches at batch 1.  Returns [(block ids, [blocks][B][C])] per width;
    empty when a projection is trainable (the per-block path keeps the gradients)."""
    blocks = [m for m in model.modules() if isinstance(m, ResnetBlock2D) and m.time_emb_proj is not None]
    if not blocks or any(p.requires_grad for b in blocks for p in b.time_emb_proj.parameters()):
        return []
    key = (emb.device, emb.dtype, tuple((b.time_emb_proj.weight.data_ptr(), b.time_emb_proj.weight._version,
                                         b.time_emb_proj.bias.data_ptr(), b.time_emb_proj.bias._version)
                                        for b in blocks))
    cache = model.__dict__.setdefault("_temb_stacks", {})
    if cache.get("key") != key:
        groups: dict[int, list] = {}
        for b in blocks:
            groups.setdefault(b.time_emb_proj.out_features, []).append(b)
        cache.clear()
        cache["key"] = key
        cache["groups"] = [
            ([id(b) for b in members],
             torch.stack([b.time_emb_proj.weight.detach().t() for b in members]).to(emb.device, emb.dtype),
             torch.stack([b.time_emb_proj.bias.detach()[None] for b in members]).to(emb.device, emb.dtype))
            for members in groups.values()]
    s = F.silu(emb)
    return [(ids, torch.baddbmm(bias, s.expand(len(ids), *s.shape), wt))  # [blocks][B][C]
            for ids, wt, bias in cache["groups"]]


def temb_projections(model: nn.Module, emb: Tensor) -> dict[int, Tensor]:
    """Every ResnetBlock2D's ``time_emb_proj(silu(emb))`` of ``model`` at once (see
    ``temb_projection_groups``): {id(block): [B, C] contiguous}; empty when a projection is
    trainable (the per-block path keeps the gradients)."""
    out = {}
    for ids, y in temb_projection_groups(model, emb):
        out.update(zip(ids, y.unbind(0)))
    return out


def timestep_rows(model: nn.Module, timestep: Tensor | int, sample: Tensor) -> tuple[Tensor, dict] | None:
    """(emb, {block: time_emb_proj(silu(emb))}) of a UNet (``UNet2DModel``,
    ``UNet2DConditionModel``: a ``time_embedding`` MLP, ResnetBlock2D projections) for a host
    timestep from a table over t = 0 .. T-1 built once per device / dtype / weight version (frozen time-embedding
    weights only): a step then launches no sinusoid, MLP or projection kernels and copies
    no timestep to the device (at batch 1 each is a host-bound launch; the H2D copy of a
    pageable tensor also waits on the stream).  At batch 1 the rows are views of the table;
    at larger batches the table row is broadcast to the batch (one copy per projection
    width), so the values are the same at every batch size (a projection recomputed at M = B
    rows would round differently from the table's M = T: DESIGN.md §6).  None (the per-step
    path) for device or per-sample timesteps, or trainable weights."""
    if torch.is_tensor(timestep):
        if timestep.is_cuda or timestep.numel() != 1 or timestep.is_floating_point():
            return None
        t = int(timestep.reshape(-1)[0])
    elif isinstance(timestep, int):
        t = timestep
    else:
        return None
    slots = model.__dict__.get("_t_slots")
    if slots is None:  # the module tree is fixed after construction; its Parameter objects are not
        blocks = [m for m in model.modules() if isinstance(m, ResnetBlock2D) and m.time_emb_proj is not None]
        mods = [model.time_embedding.linear_1, model.time_embedding.linear_2] + [b.time_emb_proj for b in blocks]
        slots = model.__dict__["_t_slots"] = [(m, name) for m in mods for name in ("weight", "bias")
                                              if m._parameters.get(name) is not None]
    # read the live parameters (load_state_dict(..., assign=True) replaces the objects): the table
    # key below then follows a replaced tensor as it follows an in-place update
    params = [m._parameters[name] for m, name in slots]
    if t < 0 or not sample.is_cuda or any(p.requires_grad for p in params):
        return None
    key = (sample.device, sample.dtype, tuple((p.data_ptr(), p._version) for p in params))
    tab = model.__dict__.get("_t_rows")
    if tab is None or tab[0] != key or t >= tab[1].shape[0]:
        cfg = model.config
        with torch.no_grad():
            ts = torch.arange(max(1000, t + 1), device=sample.device)
            t_emb = timestep_embedding(ts, cfg.block_out_channels[0], flip_sin_to_cos=cfg.flip_sin_to_cos,
                                       freq_shift=cfg.freq_shift).to(sample.dtype)
            emb_all = model.time_embedding(t_emb)
            tab = (key, emb_all, temb_projection_groups(model, emb_all))
        model.__dict__["_t_rows"] = tab
    _, emb_all, groups = tab
    b = sample.shape[0]
    out = {}
    for ids, y in groups:  # y: [blocks][T][C]
        rows = y[:, t:t + 1]
        if b > 1:
            rows = rows.expand(len(ids), b, y.shape[2]).contiguous()
        out.update(zip(ids, rows.unbind(0)))
    return emb_all[t:t + 1].expand(b, -1), out


class TimestepEmbedding(nn.Module):
    def __init__(self, in_dim: int, out_dim: int) -> None:
        super().__init__()
        self.linear_1 = nn.Linear(in_dim, out_dim)
        self.linear_2 = nn.Linear(out_dim, out_dim)

    def forward(self, x: Tensor) -> Tensor:
        return self.linear_2(F.silu(self.linear_1(x)))


def _shortcut_backend() -> str:
    """``SAMPLERS_AMD_SHORTCUT``: ``x6`` (default: the 1x1 GEMM on bf16 MFMAs over exact
    three-term splits of the fp32 operands, ``csrc/sp_gemm_x6.hip``, where its shape rules
    hold) or ``torch`` (hipBLASLt fp32 GEMMs)."""
    import os

    return os.environ.get("SAMPLERS_AMD_SHORTCUT", "x6").lower()


def _pointwise_pack(conv: nn.Conv2d, trans: bool) -> Tensor:
    """conv's 1x1 weights [cout, cin] (trans: as [cin, cout] for the input VJP) packed for
    sp_gemm_x6, cached on the module and rebuilt when the weight changes."""
    w = conv.weight
    key = (w.data_ptr(), w._version, w.device)
    cache = conv.__dict__.setdefault("_x6_packs", {})
    if cache.get("key") != key:
        cache.clear()
        cache["key"] = key
    if trans not in cache:
        lib = _hip.load_library()
        cout, cin = w.shape[0], w.shape[1]
        m, k = (cin, cout) if trans else (cout, cin)
        wc = w.detach().reshape(cout, cin).contiguous()
        out = torch.empty(int(lib.sp_gemm_x6_packed_size(m, k)), device=w.device)
        _hip.check(lib.sp_gemm_x6_pack(_hip.ptr(wc), m, k, int(trans), _hip.ptr(out), _hip.stream_of(wc)),
                   "sp_gemm_x6_pack")
        cache[trans] = out
    return cache[trans]


def _x6_ok(m: int, c1: int, c2: int, o1: int, o2: int, hw: int, n: int) -> bool:
    return (_shortcut_backend() == "x6" and bool(_query("sp_gemm_x6_supported", m, c1 + c2, hw))
            and c1 % 8 == 0 and c2 % 8 == 0 and o1 % 32 == 0 and o2 % 32 == 0
            and x6_enough_tiles(n * hw, o1 + o2))


def _shortcut_forward(conv: nn.Conv2d, x1: Tensor, x2: Tensor | None) -> Tensor:
    """1x1 conv_shortcut over cat(x1, x2) without its bias (the caller folds it into conv2's):
    one pass of the bf16x6 1x1 GEMM over both parts read in place (``csrc/sp_gemm_x6.hip``),
    or W[:, :c1] x1 + W[:, c1:] x2 as broadcast-batched fp32 GEMMs, the second part
    accumulated in place (no concatenated input; 25-35 % faster than MIOpen's 1x1 path on
    these shapes, tools/bench_shortcut.py)."""
    n, c1 = x1.shape[:2]
    c2 = 0 if x2 is None else x2.shape[1]
    cout = conv.out_channels
    hw = x1[0, 0].numel()
    if _x6_ok(cout, c1, c2, cout, 0, hw, n):
        lib = _hip.load_library()
        x1 = x1.contiguous()
        x2 = None if x2 is None else x2.contiguous()
        y = torch.empty((n, cout) + tuple(x1.shape[2:]), device=x1.device, dtype=torch.float32)
        ws, nb = x6_workspace(lib, n, hw, c1 + c2, cout, x1.device)
        _hip.check(lib.sp_gemm_x6_ws(_hip.ptr(x1), c1, _hip.ptr(x2), c2, _hip.ptr(_pointwise_pack(conv, False)),
                                     None, None, n, hw, _hip.ptr(y), cout, None, 0, _hip.ptr(ws), nb,
                                     _hip.stream_of(x1)), "sp_gemm_x6")
        return y
    if batch_invariant_enabled() and n > 1:  # hipBLASLt's algorithm follows the batch count
        return torch.cat([_shortcut_forward(conv, x1[i:i + 1], None if x2 is None else x2[i:i + 1])
                          for i in range(n)])
    w = conv.weight[:, :, 0, 0]
    y = torch.matmul(w[:, :c1], x1.reshape(n, c1, -1))
    if x2 is not None:
        w2 = w[:, c1:]
        y.baddbmm_(w2.expand(n, *w2.shape), x2.reshape(n, x2.shape[1], -1))
    return y.reshape((n, w.shape[0]) + tuple(x1.shape[2:]))


def _shortcut_input_vjp(conv: nn.Conv2d, dy: Tensor, c1: int, c2: int) -> tuple[Tensor, Tensor | None]:
    """(W[:, :c1]^T dy, W[:, c1:]^T dy): one pass of the bf16x6 1x1 GEMM writing both parts,
    or two fp32 batched GEMMs."""
    n, cout = dy.shape[:2]
    hw = dy[0, 0].numel()
    if _x6_ok(c1 + c2, cout, 0, c1, c2, hw, n):
        lib = _hip.load_library()
        dy = dy.contiguous()
        d1 = torch.empty((n, c1) + tuple(dy.shape[2:]), device=dy.device, dtype=torch.float32)
        d2 = torch.empty((n, c2) + tuple(dy.shape[2:]), device=dy.device, dtype=torch.float32) if c2 else None
        ws, nb = x6_workspace(lib, n, hw, cout, c1 + c2, dy.device)
        _hip.check(lib.sp_gemm_x6_ws(_hip.ptr(dy), cout, None, 0, _hip.ptr(_pointwise_pack(conv, True)), None, None,
                                     n, hw, _hip.ptr(d1), c1, _hip.ptr(d2), c2, _hip.ptr(ws), nb,
                                     _hip.stream_of(dy)), "sp_gemm_x6")
        return d1, d2
    if batch_invariant_enabled() and n > 1:
        parts = [_shortcut_input_vjp(conv, dy[i:i + 1], c1, c2) for i in range(n)]
        return (torch.cat([p[0] for p in parts]),
                None if not c2 else torch.cat([p[1] for p in parts]))
    dyv = dy.reshape(n, cout, -1)
    w = conv.weight[:, :, 0, 0]
    d1 = torch.matmul(w[:, :c1].t(), dyv).reshape((n, c1) + tuple(dy.shape[2:]))
    d2 = None if not c2 else torch.matmul(w[:, c1:].t(), dyv).reshape((n, c2) + tuple(dy.shape[2:]))
    return d1, d2


def _folded_bias(block: "ResnetBlock2D") -> Tensor | None:
    """conv2.bias + conv_shortcut.bias (the shortcut's bias rides in conv2's epilogue), cached
    on the block while both are unchanged (frozen weights: one add per weight update instead
    of one launch per forward — ~20 per UNet forward, host-bound at batch 1)."""
    b2, bs = block.conv2.bias, block.conv_shortcut.bias
    if bs is None or b2 is None:
        return bs if b2 is None else b2
    key = (b2.data_ptr(), b2._version, bs.data_ptr(), bs._version)
    hit = block.__dict__.get("_folded_bias")
    if hit is None or hit[0] != key:
        with torch.no_grad():
            hit = (key, b2 + bs)
        block.__dict__["_folded_bias"] = hit
    return hit[1]


class _ResnetBlockFn(torch.autograd.Function):
    """A whole ResnetBlock2D on the HIP kernels with its input VJP written by hand:

    fwd  z1 = silu(GN1(cat(x1, x2)))   both parts read in place (no torch.cat)
         h1 = conv1(z1)
         z2 = silu(GN2(h1 + tb))
         out = conv2(z2) + shortcut(x)   the residual added in the Winograd epilogue
    bwd  dx = GN1^T(conv1^T(GN2^T(conv2^T dout))) + shortcut^T dout, the residual branch's
         gradient added by GN1's backward kernel into the parts' gradients (no autograd
         accumulation add, no contiguous copies of cat slices).
    Saves x1, x2, h1 and the GroupNorm statistics (the conv inputs z1, z2 are only needed
    for weight gradients, which the samplers never take: weights are frozen)."""

    @staticmethod
    def forward(ctx, block, tb, x1, x2, box_in=None, box_out=None):
        z1, st1 = gn_forward(block.norm1, x1, x2)
        h1 = conv3x3_forward(block.conv1, z1)
        del z1
        z2, st2 = gn_forward(block.norm2, h1, None, tb)
        bias = block.conv2.bias
        if block.conv_shortcut is None:
            short = x1
        else:
            short = _shortcut_forward(block.conv_shortcut, x1, x2)
            bias = _folded_bias(block)
        out = conv3x3_forward(block.conv2, z2, res=short, bias=bias)
        ctx.block = block
        ctx.box_in, ctx.box_out = box_in, box_out
        ctx.save_for_backward(x1, x2, h1, tb, st1, st2)
        return out

    @staticmethod
    def backward(ctx, dout):
        x1, x2, h1, tb, st1, st2 = ctx.saved_tensors
        blk = ctx.block
        dout = dout.contiguous()
        dz2 = conv3x3_input_vjp(blk.conv2, dout, h1.shape)
        dh1, _ = gn_backward(blk.norm2, dz2, h1, None, tb, st2)
        del dz2
        zshape = (x1.shape[0], blk.conv1.in_channels) + tuple(x1.shape[2:])
        dz1 = conv3x3_input_vjp(blk.conv1, dh1, zshape)
        del dh1
        # x1 is a skip tensor whose up-block consumer left its gradient: added in the kernel
        extra = ctx.box_in.take() if ctx.box_in is not None else None
        if blk.conv_shortcut is None:  # identity shortcut: dx1 = GN1^T dz1 + dout (+ skip grad)
            dx1, dx2 = gn_backward(blk.norm1, dz1, x1, x2, None, st1, add1=dout, add1b=extra)
        else:  # dx = shortcut^T dout, then += GN1^T dz1 in place
            s1, s2 = _shortcut_input_vjp(blk.conv_shortcut, dout, x1.shape[1],
                                         0 if x2 is None else x2.shape[1])
            dx1, dx2 = gn_backward(blk.norm1, dz1, x1, x2, None, st1, add1=s1, add2=s2,
                                   out1=s1, out2=s2, add1b=extra)
        if ctx.box_out is not None:  # x2 (a skip): its down-path consumer adds this gradient
            ctx.box_out.grad, dx2 = dx2, None
        return None, None, dx1, dx2, None, None


class ResnetBlock2D(nn.Module):
    """GN-SiLU-conv x2 with an optional time-embedding bias (``temb=None``: VAE blocks).

    ``forward(x, temb, skip)`` takes the up path's skip tensor separately: on the device
    with frozen fp32 weights the whole block runs as ``_ResnetBlockFn`` over cat(x, skip)
    read in place; otherwise (CPU, training) it is the module-by-module graph on
    ``torch.cat([x, skip], 1)``."""

    def __init__(self, cin: int, cout: int, temb: int | None, groups: int, eps: float) -> None:
        super().__init__()
        self.norm1 = GroupNormAct(groups, cin, eps=eps, act=True)
        self.conv1 = Conv3x3(cin, cout)
        self.time_emb_proj = nn.Linear(temb, cout) if temb else None
        self.norm2 = GroupNormAct(groups, cout, eps=eps, act=True)
        self.conv2 = Conv3x3(cout, cout)
        self.conv_shortcut = nn.Conv2d(cin, cout, 1) if cin != cout else None

    def _frozen(self) -> bool:
        params = self.__dict__.get("_param_list")
        if params is None:
            params = self.__dict__["_param_list"] = list(self.parameters())
        return not any(p.requires_grad for p in params)

    def _forward_bf16(self, x: Tensor, skip: Tensor | None, tb: Tensor | None, box_in: SkipGrad | None,
                      box_out: SkipGrad | None) -> Tensor:
        """The block at bf16 on the NHWC kernels (networks/bf16.py): GN1 over cat(x, skip) read in
        place, conv1, GN2 with the time-embedding bias, conv2 with the shortcut added in its
        epilogue — as one autograd function (``bf16.resnet_block``) where the kernels serve the
        shapes, module by module otherwise.  Skip gradients: handed over through the SkipGrad
        mailboxes where both consumers are fused blocks (added in GN1's VJP kernel), else
        summed by autograd (the box disabled in the forward pass)."""
        from . import bf16

        if bf16.resnet_block_supported(self, x, skip):
            box_in = box_in if box_in is not None and box_in.enabled else None
            box_out = box_out if box_out is not None and box_out.enabled and skip is not None else None
            return bf16.resnet_block(self, x, skip, tb, box_in, box_out)
        for box in (box_in, box_out):
            if box is not None:
                box.enabled = False
        c2 = 0 if skip is None else skip.shape[1]
        if bf16.group_norm_supported(self.norm1, x, c2):
            z1 = bf16.group_norm(self.norm1, x, skip)
        else:
            z1 = self.norm1(x if skip is None else torch.cat([x, skip], dim=1))
        h = self.conv1(z1)
        z2 = self.norm2(h, tb)
        xin = x if skip is None else torch.cat([bf16.nhwc(x), bf16.nhwc(skip)], dim=1)
        short = xin if self.conv_shortcut is None else bf16.pointwise(xin, self.conv_shortcut.weight,
                                                                         self.conv_shortcut.bias)
        if bf16.conv_supported(self.conv2, z2):
            return bf16.conv3x3(self.conv2, z2, res=short)
        return self.conv2(z2) + short

    def _fusable(self, x: Tensor) -> bool:
        params = self.__dict__.get("_param_list")
        if params is None:  # fixed after construction; walking the submodules per call is host time
            params = self.__dict__["_param_list"] = list(self.parameters())
        return (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
                and not any(p.requires_grad for p in params)
                and (x.shape[2] * x.shape[3]) % 4 == 0)

    def forward(self, x: Tensor, temb: Tensor | None = None, skip: Tensor | None = None,
                box_in: SkipGrad | None = None, box_out: SkipGrad | None = None,
                tb: Tensor | None = None) -> Tensor:
        """``box_in``: ``x`` is a UNet skip tensor (the mailbox of its up-block gradient);
        ``box_out``: the mailbox of ``skip`` (see ``SkipGrad``); ``tb``: this block's
        ``time_emb_proj(silu(temb))`` already computed (``temb_projections``)."""
        if box_in is not None and skip is not None:
            raise ValueError("box_in (x is a skip tensor) and skip (an up-block input) are exclusive")
        if tb is None and self.time_emb_proj is not None:
            tb = self.time_emb_proj(F.silu(temb))
        if x.is_cuda and x.dtype == torch.bfloat16 and self._frozen():
            return self._forward_bf16(x, skip, tb, box_in, box_out)
        if (self._fusable(x) and (skip is None or skip.dtype == x.dtype)
                and (box_in is None or box_in.enabled)):
            x1 = x.contiguous()
            x2 = None if skip is None else skip.contiguous()
            if x1 is not x or (x2 is not None and x2 is not skip):
                # copies: gradients flow through autograd as usual; both sides of the
                # hand-off see the boxes disabled
                for box in (box_in, box_out):
                    if box is not None:
                        box.enabled = False
                box_in = box_out = None
            box_in = box_in if box_in is not None and box_in.enabled else None
            box_out = box_out if box_out is not None and box_out.enabled and x2 is not None else None
            return _ResnetBlockFn.apply(self, None if tb is None else tb.contiguous(), x1, x2,
                                        box_in, box_out)
        if box_in is not None:
            box_in.enabled = False
        if skip is not None:
            x = torch.cat([x, skip], dim=1)
        h = self.conv1(self.norm1(x))  # silu(norm1(x)), fused
        # silu(norm2(h + temb_proj)): the time-embedding add rides in the fused norm
        h = self.conv2(self.norm2(h, tb))
        if self.conv_shortcut is not None:
            miopen_fallback(x)
            x = self.conv_shortcut(x)
        return x + h


def attention_backend() -> str:
    """``SAMPLERS_AMD_ATTN``: ``gemm`` (default: scores materialised, batched fp32 GEMMs +
    the HIP row softmax and its VJP) or ``sdpa`` (``F.scaled_dot_product_attention``)."""
    import os

    return os.environ.get("SAMPLERS_AMD_ATTN", "gemm").lower()


def _score_chunks(b: int, n: int, m: int) -> int:
    """Query-row chunks of a score GEMM (n x m scores, one per batch entry).  hipBLASLt serves
    the 16² level's 256 x 256 x 512 product with one 256 x 256 macro tile per batch entry (one
    CU at b = 1: 119 µs); cut into row chunks (k repeated per chunk) it spreads over more
    workgroups: 23 µs at b = 1 (8 chunks), 74 vs 120 µs at b = 64 (4 chunks).  The VAE's
    4096-token scores already fill the chip (chunking measured slower at b >= 2).
    tools/bench_score_gemm.py, profiles/round4/score_gemm.jsonl."""
    if n * m > 1024 * 1024 or n % 8:
        return 1
    return 4 if b >= 32 else 8


def bmm(a: Tensor, bm: Tensor, out: Tensor | None = None) -> Tensor:
    """``torch.bmm``; in batch-invariant mode (``runtime.batch_invariant``) one GEMM per batch
    entry, so hipBLASLt's algorithm (and summation order) does not follow the batch count."""
    if not batch_invariant_enabled() or a.shape[0] == 1:
        return torch.bmm(a, bm) if out is None else torch.bmm(a, bm, out=out)
    if out is None:
        out = torch.empty(a.shape[0], a.shape[1], bm.shape[2], device=a.device, dtype=a.dtype)
    for i in range(a.shape[0]):
        torch.bmm(a[i:i + 1], bm[i:i + 1], out=out[i:i + 1])
    return out


def score_gemm(a: Tensor, bm: Tensor, alpha: float, out: Tensor) -> Tensor:
    """out[i] = alpha · a[i] bm[i]ᵀ for a (b, n, d), bm (b, m, d) (strided views allowed),
    out (b, n, m) contiguous; query rows chunked where that fills the chip (``_score_chunks``)."""
    b, n, d = a.shape
    m = bm.shape[1]
    if batch_invariant_enabled() and b > 1:  # one batch entry per GEMM (``bmm``)
        for i in range(b):
            score_gemm(a[i:i + 1], bm[i:i + 1], alpha, out[i:i + 1])
        return out
    ch = _score_chunks(b, n, m)
    if ch == 1:
        return torch.baddbmm(out, a, bm.transpose(1, 2), beta=0.0, alpha=alpha, out=out)
    r = n // ch
    ac = a.reshape(b * ch, r, d)  # a view: the chunks of a batch entry are consecutive rows
    bc = bm.unsqueeze(1).expand(b, ch, m, d).reshape(b * ch, m, d)
    oc = out.view(b * ch, r, m)
    torch.baddbmm(oc, ac, bc.transpose(1, 2), beta=0.0, alpha=alpha, out=oc)
    return out


class _ScoreAttentionQKV(torch.autograd.Function):
    """``_ScoreAttention`` on the fused projection's output ``qkv`` ([b][n][3c], q, k, v its
    thirds read in place); the VJP writes dq, dk, dv straight into one [b][n][3c] cotangent
    (GEMM outputs with row stride 3c), so no concatenation follows."""

    @staticmethod
    def forward(ctx, qkv: Tensor) -> Tensor:
        lib = _hip.load_library()
        b, n, c3 = qkv.shape
        c = c3 // 3
        q, k, v = qkv.split(c, dim=-1)
        scale = 1.0 / math.sqrt(c)
        p = score_gemm(q, k, scale, torch.empty(b, n, n, device=qkv.device, dtype=qkv.dtype))
        _hip.check(lib.sp_softmax_rows(_hip.ptr(p), b * n, n, None, _hip.stream_of(p)), "sp_softmax_rows")
        ctx.save_for_backward(qkv, p)
        ctx.scale = scale
        return bmm(p, v)

    @staticmethod
    def backward(ctx, dout: Tensor):
        qkv, p = ctx.saved_tensors
        lib = _hip.load_library()
        b, n, c3 = qkv.shape
        c = c3 // 3
        q, k, v = qkv.split(c, dim=-1)
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = dqkv.split(c, dim=-1)
        bmm(p.transpose(1, 2), dout, out=dv)
        ds = score_gemm(dout, v, 1.0, torch.empty(b, n, n, device=qkv.device, dtype=qkv.dtype))
        _hip.check(lib.sp_softmax_bwd_rows(_hip.ptr(p), _hip.ptr(ds), b * n, n, ctx.scale, _hip.stream_of(ds)),
                   "sp_softmax_bwd_rows")
        bmm(ds, k, out=dq)
        bmm(ds.transpose(1, 2), q, out=dk)
        return dqkv


class _ScoreAttention(torch.autograd.Function):
    """softmax(q kᵀ · scale) v over (batch, n, d) with the scores materialised: the score /
    value GEMMs on hipBLASLt (batched fp32; q, k, v may be strided views, e.g. the thirds of a
    fused projection), the row softmax and its VJP on HIP (``sp_softmax_rows`` /
    ``sp_softmax_bwd_rows``, one pass over the scores each).  Saves q, k, v and P."""

    @staticmethod
    def forward(ctx, q: Tensor, k: Tensor, v: Tensor) -> Tensor:
        lib = _hip.load_library()
        bh, n, d = q.shape
        m = k.shape[1]
        scale = 1.0 / math.sqrt(d)
        p = score_gemm(q, k, scale, torch.empty(bh, n, m, device=q.device, dtype=q.dtype))
        _hip.check(lib.sp_softmax_rows(_hip.ptr(p), bh * n, m, None, _hip.stream_of(p)), "sp_softmax_rows")
        ctx.save_for_backward(q, k, v, p)
        ctx.scale = scale
        return bmm(p, v)

    @staticmethod
    def backward(ctx, dout: Tensor):
        q, k, v, p = ctx.saved_tensors
        lib = _hip.load_library()
        bh, n, m = p.shape
        need_q, need_k, need_v = ctx.needs_input_grad[:3]
        dv = bmm(p.transpose(1, 2), dout) if need_v else None
        dq = dk = None
        if need_q or need_k:
            ds = score_gemm(dout, v, 1.0, torch.empty(bh, n, m, device=dout.device, dtype=dout.dtype))
            _hip.check(lib.sp_softmax_bwd_rows(_hip.ptr(p), _hip.ptr(ds), bh * n, m, ctx.scale,
                                               _hip.stream_of(ds)), "sp_softmax_bwd_rows")
            dq = bmm(ds, k) if need_q else None
            dk = bmm(ds.transpose(1, 2), q) if need_k else None
        return dq, dk, dv


def _score_attention_ok(q: Tensor, k: Tensor) -> bool:
    return (q.is_cuda and q.dtype == torch.float32 and attention_backend() == "gemm"
            and bool(_hip.load_library().sp_softmax_rows_supported(q.shape[0] * q.shape[1], k.shape[1])))


def attention(q: Tensor, k: Tensor, v: Tensor) -> Tensor:
    """softmax(q k^T / sqrt(d)) v over (batch, heads, tokens, d).

    The priors' attention has one head of d = 512 (the VAE mid blocks at 64x64 = 4096
    tokens, the DDPM UNet at 16x16) or 8 heads of 64 (the latent UNet).  At d = 512 the
    fused flash kernels of PyTorch-ROCm run fp32 at 54 TFLOP/s forward and 25 backward
    (their Q/K/V tiles do not fit on chip); materialising the scores (B x N x N fp32:
    2 GiB for 32 VAE samples, small beside 288 GB) turns both directions into large
    batched GEMMs on hipBLASLt (about 0.9 of the fp32 MFMA peak at these sizes) plus one
    HIP softmax pass each way (``_ScoreAttention``)."""
    b, nh, n, d = q.shape
    qf, kf, vf = (t.reshape(b * nh, n, d) for t in (q, k, v))
    if _score_attention_ok(qf, kf):
        return _ScoreAttention.apply(qf, kf, vf).reshape(b, nh, n, d)
    if attention_backend() == "sdpa" or not q.is_cuda:
        return F.scaled_dot_product_attention(q, k, v)
    s = torch.baddbmm(torch.empty(b * nh, n, n, device=q.device, dtype=q.dtype), qf,
                      kf.transpose(1, 2), beta=0.0, alpha=1.0 / math.sqrt(d))
    return torch.bmm(torch.softmax(s, dim=-1), vf).reshape(b, nh, n, d)


class _QKVHolder:
    """[W_q; W_k; W_v] and [b_q; b_k; b_v] of one attention block, outside the module tree
    (``layers.linear`` caches the packed weight on this object)."""

    def __init__(self, weight: Tensor, bias: Tensor | None) -> None:
        self.weight, self.bias = weight, bias


class SpatialSelfAttention(nn.Module):
    """GroupNorm -> single/multi-head attention over H*W tokens -> residual."""

    def __init__(self, channels: int, groups: int, eps: float, head_dim: int | None) -> None:
        super().__init__()
        self.heads = 1 if head_dim is None else channels // head_dim
        self.group_norm = GroupNormAct(groups, channels, eps=eps)
        self.to_q = Linear(channels, channels)
        self.to_k = Linear(channels, channels)
        self.to_v = Linear(channels, channels)
        self.to_out = nn.ModuleList([Linear(channels, channels)])

    def _qkv(self) -> _QKVHolder:
        mods = (self.to_q, self.to_k, self.to_v)
        key = tuple((m.weight.data_ptr(), m.weight._version, m.weight.device) for m in mods)
        cache = self.__dict__.setdefault("_qkv_cache", {})
        if cache.get("key") != key:
            w = torch.cat([m.weight.detach() for m in mods], 0)
            b = None if mods[0].bias is None else torch.cat([m.bias.detach() for m in mods], 0)
            cache.clear()
            cache.update(key=key, holder=_QKVHolder(w, b))
        return cache["holder"]

    def forward(self, x: Tensor) -> Tensor:
        b, c, h, w = x.shape
        fast = (self.heads == 1 and x.is_cuda and x.dtype == torch.float32 and not self.to_q.weight.requires_grad
                and attention_backend() == "gemm"
                and bool(_hip.load_library().sp_softmax_rows_supported(b * h * w, h * w)))
        box = SkipGrad() if fast and torch.is_grad_enabled() else None  # x's residual gradient
        z = self.group_norm(x, box=box)
        if fast:
            # one projection for q, k, v from the NCHW planes straight into token rows; the
            # attention reads its thirds in place; to_out writes NCHW with the residual added
            # (its gradient summed in the norm's VJP kernel)
            hold = self._qkv()
            qkv = proj_nchw_to_tokens(z, hold, hold.weight, hold.bias).reshape(b, h * w, 3 * c)
            o = _ScoreAttentionQKV.apply(qkv)
            return proj_tokens_to_nchw(o, self.to_out[0], x, self.to_out[0].weight, self.to_out[0].bias, box)
        if box is not None:
            box.enabled = False
        tokens = z.reshape(b, c, h * w).transpose(1, 2)
        q, k, v = self.to_q(tokens), self.to_k(tokens), self.to_v(tokens)
        nh = self.heads
        q, k, v = (t.reshape(b, h * w, nh, c // nh).transpose(1, 2) for t in (q, k, v))
        o = attention(q, k, v)
        o = self.to_out[0](o.transpose(1, 2).reshape(b, h * w, c))
        return x + o.transpose(1, 2).reshape(b, c, h, w)


class Downsample2D(nn.Module):
    """Stride-2 3x3 conv with diffusers' ``downsample_padding=0`` (pad right/bottom by 1)."""

    def __init__(self, channels: int) -> None:
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, stride=2, padding=0)

    def forward(self, x: Tensor, box: SkipGrad | None = None) -> Tensor:
        return downsample_conv(self.conv, x, box)


class Upsample2D(nn.Module):
    def __init__(self, channels: int) -> None:
        super().__init__()
        self.conv = Conv3x3(channels, channels)

    def forward(self, x: Tensor) -> Tensor:
        return upsample_conv(self.conv, x)


class _Level(nn.Module):
    def __init__(self) -> None:
        super().__init__()
        self.resnets = nn.ModuleList()
        self.attentions = nn.ModuleList()


class UNet2DModel(nn.Module):
    """Epsilon-prediction UNet; ``forward(sample, timestep) -> eps`` (same shape as sample)."""

    def __init__(self, config: UNet2DConfig = CELEBAHQ_256) -> None:
        super().__init__()
        self.config = config
        ch = config.block_out_channels
        g, eps = config.norm_num_groups, config.norm_eps
        temb = ch[0] * 4
        self.time_embedding = TimestepEmbedding(ch[0], temb)
        self.conv_in = Conv3x3(config.in_channels, ch[0])

        self.down_blocks = nn.ModuleList()
        cout = ch[0]
        for i, c in enumerate(ch):
            cin, cout = cout, c
            lvl = _Level()
            for j in range(config.layers_per_block):
                lvl.resnets.append(ResnetBlock2D(cin if j == 0 else cout, cout, temb, g, eps))
                if i in config.attention_levels:
                    lvl.attentions.append(SpatialSelfAttention(cout, g, eps, config.attention_head_dim))
            lvl.downsamplers = nn.ModuleList([Downsample2D(cout)]) if i < len(ch) - 1 else None
            self.down_blocks.append(lvl)

        mid = ch[-1]
        self.mid_block = _Level()
        self.mid_block.resnets.append(ResnetBlock2D(mid, mid, temb, g, eps))
        self.mid_block.attentions.append(SpatialSelfAttention(mid, g, eps, config.attention_head_dim))
        self.mid_block.resnets.append(ResnetBlock2D(mid, mid, temb, g, eps))

        self.up_blocks = nn.ModuleList()
        rev = list(reversed(ch))
        nlev = len(ch)
        prev = rev[0]
        for i, c in enumerate(rev):
            skip_in = rev[min(i + 1, nlev - 1)]
            lvl = _Level()
            for j in range(config.layers_per_block + 1):
                res_skip = skip_in if j == config.layers_per_block else c
                res_in = prev if j == 0 else c
                lvl.resnets.append(ResnetBlock2D(res_in + res_skip, c, temb, g, eps))
                if (nlev - 1 - i) in config.attention_levels:
                    lvl.attentions.append(SpatialSelfAttention(c, g, eps, config.attention_head_dim))
            lvl.upsamplers = nn.ModuleList([Upsample2D(c)]) if i < nlev - 1 else None
            self.up_blocks.append(lvl)
            prev = c

        self.conv_norm_out = GroupNormAct(g, ch[0], eps=eps, act=True)
        self.conv_out = Conv3x3(ch[0], config.out_channels)

    def _timestep_rows(self, timestep: Tensor | int, sample: Tensor) -> tuple[Tensor, dict] | None:
        return timestep_rows(self, timestep, sample)

    def forward(self, sample: Tensor, timestep: Tensor | int) -> Tensor:
        cfg = self.config
        b = sample.shape[0]
        table = self._timestep_rows(timestep, sample)
        if table is not None:
            emb, tbs = table
        else:
            if not torch.is_tensor(timestep):
                timestep = torch.tensor([timestep], dtype=torch.long, device=sample.device)
            timestep = timestep.reshape(-1).to(sample.device).expand(b)
            t_emb = timestep_embedding(
                timestep, cfg.block_out_channels[0],
                flip_sin_to_cos=cfg.flip_sin_to_cos, freq_shift=cfg.freq_shift,
            ).to(sample.dtype)
            emb = self.time_embedding(t_emb)
            tbs = temb_projections(self, emb)

        # every skip tensor has two consumers (the next down-path layer and an up-block
        # resnet); with grad on the device their gradients meet inside the down-path
        # consumer's VJP kernel (SkipGrad) instead of an autograd accumulation add
        # (SAMPLERS_AMD_SKIPGRAD=0: autograd sums them, for A/B measurements and tests)
        import os

        mail = torch.is_grad_enabled() and sample.is_cuda and os.environ.get("SAMPLERS_AMD_SKIPGRAD", "1") != "0"
        new_box = (lambda: SkipGrad()) if mail else (lambda: None)  # noqa: E731
        h = self.conv_in(sample)
        skips, boxes = [h], [new_box()]
        for lvl in self.down_blocks:
            for j, res in enumerate(lvl.resnets):
                h = res(h, emb, box_in=boxes[-1] if skips[-1] is h else None, tb=tbs.get(id(res)))
                if len(lvl.attentions):
                    h = lvl.attentions[j](h)
                skips.append(h)
                boxes.append(new_box())
            if lvl.downsamplers is not None:
                h = lvl.downsamplers[0](h, box=boxes[-1])
                skips.append(h)
                boxes.append(new_box())

        m0, m1 = self.mid_block.resnets
        h = m0(h, emb, box_in=boxes[-1], tb=tbs.get(id(m0)))
        h = self.mid_block.attentions[0](h)
        h = m1(h, emb, tb=tbs.get(id(m1)))

        for lvl in self.up_blocks:
            for j, res in enumerate(lvl.resnets):
                h = res(h, emb, skip=skips.pop(), box_out=boxes.pop(), tb=tbs.get(id(res)))
                if len(lvl.attentions):
                    h = lvl.attentions[j](h)
            if lvl.upsamplers is not None:
                h = lvl.upsamplers[0](h)

        return _as_nchw(self.conv_out(self.conv_norm_out(h)))


def _as_nchw(y: Tensor) -> Tensor:
    """The network's output in the NCHW layout the samplers read (the bf16 layers return
    channels-last tensors; fp32 outputs are already NCHW)."""
    return y if y.is_contiguous() else y.contiguous()


def build_unet(config: UNet2DConfig = CELEBAHQ_256, *, seed: int = 0, device=None,
               dtype: torch.dtype = torch.float32) -> UNet2DModel:
    """Random-init prior with a fixed seed (weights are deterministic across boxes)."""
    gen_state = torch.random.get_rng_state()
    torch.manual_seed(seed)
    try:
        net = UNet2DModel(config)
    finally:
        torch.random.set_rng_state(gen_state)
    return net.to(device=device, dtype=dtype).eval().requires_grad_(False)


def count_parameters(module: nn.Module) -> int:
    return sum(p.numel() for p in module.parameters())

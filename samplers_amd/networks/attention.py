"""Multi-head attention for the latent prior with an O(N·d) memory footprint under autograd.

Self-attention over the latent tokens runs on the fused fp32-MFMA kernels of
``csrc/sp_attention.hip`` (the score matrix never reaches HBM; ``_FusedAttention``); the
chunked GEMM path below serves the other calls (cross-attention to the 77-token context,
other head dims) and ``SAMPLERS_AMD_LATENT_ATTN=gemm``.

The SD 1.5 ε-UNet (``unet2d_condition.py``) runs self-attention over 64x64 = 4096 latent
tokens with 8 heads per sample.  At the config-4 batch (32 latents) one layer's score
matrix is 32·8·4096²·4 B = 17 GiB; autograd would keep the softmax of every such layer
for the input VJP (five of them at 64x64 plus the 32x32 ones, ~90 GiB), beside the VAE
activations PSLD holds at 512² in the same graph.  ``attention`` therefore saves only
q, k, v, the output and the row log-sum-exp, and recomputes the probabilities chunk by
chunk in the backward pass (the FlashAttention recurrence, with the chunk sized so its
score block stays around ``SAMPLERS_AMD_ATTN_CHUNK_MIB`` MiB of HBM).  Every GEMM is a
batched fp32 GEMM on hipBLASLt (``torch.baddbmm`` / ``torch.bmm``); no precision is
dropped.

Backward (per chunk of batch·heads rows), with P = exp(S − lse), S = scale·q kᵀ:
    dv = Pᵀ do        dP = do vᵀ        dS = P ∘ (dP − rowsum(do ∘ o))
    dq = scale·dS k   dk = scale·dSᵀ q
"""

from __future__ import annotations

import math
import os

import torch
from torch import Tensor


def _chunk_rows(bh: int, n: int, m: int) -> int:
    budget = int(os.environ.get("SAMPLERS_AMD_ATTN_CHUNK_MIB", "2048")) * 2**20
    return max(1, min(bh, budget // max(1, n * m * 4)))


def _scores(q: Tensor, k: Tensor, scale: float) -> Tensor:
    s = torch.empty(q.shape[0], q.shape[1], k.shape[1], device=q.device, dtype=q.dtype)
    return torch.baddbmm(s, q, k.transpose(1, 2), beta=0.0, alpha=scale)


class _RecomputeAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q: Tensor, k: Tensor, v: Tensor) -> Tensor:
        bh, n, d = q.shape
        m = k.shape[1]
        scale = 1.0 / math.sqrt(d)
        out = torch.empty(bh, n, v.shape[2], device=q.device, dtype=q.dtype)
        lse = torch.empty(bh, n, device=q.device, dtype=q.dtype)
        step = _chunk_rows(bh, n, m)
        for a in range(0, bh, step):
            b = min(bh, a + step)
            s = _scores(q[a:b], k[a:b], scale)
            torch.logsumexp(s, dim=-1, out=lse[a:b])
            s.sub_(lse[a:b, :, None]).exp_()
            torch.bmm(s, v[a:b], out=out[a:b])
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.scale = scale
        return out

    @staticmethod
    def backward(ctx, dout: Tensor):
        q, k, v, out, lse = ctx.saved_tensors
        return _gemm_backward(q, k, v, out, lse, dout.contiguous(), ctx.scale,
                              ctx.needs_input_grad[:3])


def _gemm_backward(q: Tensor, k: Tensor, v: Tensor, out: Tensor, lse: Tensor, dout: Tensor,
                   scale: float, needs) -> tuple:
    """The recompute-attention VJP on batched GEMMs, score blocks chunk by chunk."""
    bh, n, _ = q.shape
    m = k.shape[1]
    need_q, need_k, need_v = needs
    dq = torch.empty_like(q) if need_q else None
    dk = torch.empty_like(k) if need_k else None
    dv = torch.empty_like(v) if need_v else None
    delta = (dout * out).sum(dim=-1)  # rowsum(do ∘ o) = rowsum(P ∘ dP)
    step = _chunk_rows(bh, n, m)
    for a in range(0, bh, step):
        b = min(bh, a + step)
        p = _scores(q[a:b], k[a:b], scale)
        p.sub_(lse[a:b, :, None]).exp_()
        if need_v:
            torch.bmm(p.transpose(1, 2), dout[a:b], out=dv[a:b])
        if not (need_q or need_k):
            continue
        dp = torch.bmm(dout[a:b], v[a:b].transpose(1, 2))
        dp.sub_(delta[a:b, :, None]).mul_(p)  # dS
        del p
        if need_q:
            torch.bmm(dp, k[a:b], out=dq[a:b]).mul_(scale)
        if need_k:
            torch.bmm(dp.transpose(1, 2), q[a:b], out=dk[a:b]).mul_(scale)
    return dq, dk, dv


# Under ~512 tokens the fused VJP kernels' grid is too small for them (one workgroup per 64
# keys at d 160, one wave per SIMD) and the GEMM VJP wins: 256 tokens, d 160, 256 heads: 0.70
# vs 0.45 ms per layer; 1024 tokens, d 80: 3.45 vs 3.85 (tools/bench_attention.py, MI355X).
FUSED_BWD_MIN_TOKENS = 512


# Above this many bytes of pre-split K / V images (~1.9x the fp32 K + V of the call: 2.5 GB for
# SD's 4096-token attn1 at batch 128) the split-bf16 forward splits per workgroup instead
# (sp_attention6_fwd_ws with no workspace: same results, one split per 128-query workgroup).
SPLIT_WS_MAX_BYTES = int(os.environ.get("SAMPLERS_AMD_ATTN6_WS_MIB", "1024")) * 2**20


def split_bf16_forward(q: Tensor, k: Tensor, v: Tensor, batch: int, heads: int, n: int, d: int, rs: int,
                       ro: int, scale: float, out: Tensor, lse: Tensor, offsets=(0, 0, 0)) -> bool:
    """Self-attention forward on the split-bf16 kernel (``csrc/sp_attention6.hip``: fp32 operands
    as exact three-term bf16 splits on the bf16 MFMAs, error at or below the exact-fp32
    kernel's) with a workspace for K and V split once per head; False when the library's
    setting (``sp_attention_bf16x6``) or the shape leaves the call to the fp32 kernel."""
    from .. import _hip

    lib = _hip.load_library()
    if not (lib.sp_attention_bf16x6_enabled() and lib.sp_attention6_supported(batch, heads, n, d)):
        return False
    nb = int(lib.sp_attention6_workspace(batch, heads, n, d))
    if nb > SPLIT_WS_MAX_BYTES:  # the per-workgroup split form needs no workspace
        nb = 0
    ws = torch.empty(max(nb, 1), device=q.device, dtype=torch.uint8)
    _hip.check(lib.sp_attention6_fwd_ws(q.data_ptr() + offsets[0], k.data_ptr() + offsets[1],
                                        v.data_ptr() + offsets[2], batch, heads, n, d, rs, ro, scale,
                                        _hip.ptr(out), _hip.ptr(lse), _hip.ptr(ws) if nb else None, nb,
                                        _hip.stream_of(q)),
               "sp_attention6_fwd_ws")
    return True


class _FusedAttention(torch.autograd.Function):
    """Self-attention on the fused fp32-MFMA kernels (``csrc/sp_attention.hip``): no score
    matrix in HBM, forward or VJP; saves q, k, v, the output and the row log-sum-exp."""

    @staticmethod
    def forward(ctx, q: Tensor, k: Tensor, v: Tensor) -> Tensor:
        from .. import _hip

        lib = _hip.load_library()
        bh, n, d = q.shape
        scale = 1.0 / math.sqrt(d)
        out = torch.empty_like(q)
        lse = torch.empty(bh, n, device=q.device, dtype=q.dtype)
        if not split_bf16_forward(q, k, v, bh, 1, n, d, d, d, scale, out, lse):
            _hip.check(lib.sp_attention_fwd(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), bh, n, d, scale,
                                            _hip.ptr(out), _hip.ptr(lse), _hip.stream_of(q)),
                       "sp_attention_fwd")
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.scale = scale
        return out

    @staticmethod
    def backward(ctx, dout: Tensor):
        from .. import _hip

        q, k, v, out, lse = ctx.saved_tensors
        lib = _hip.load_library()
        bh, n, d = q.shape
        dout = dout.contiguous()
        need_q, need_k, need_v = ctx.needs_input_grad[:3]
        if n < FUSED_BWD_MIN_TOKENS:  # few tokens: the GEMM VJP is faster (tools/bench_attention.py)
            return _gemm_backward(q, k, v, out, lse, dout, ctx.scale, (need_q, need_k, need_v))
        dq = torch.empty_like(q) if need_q else None
        dk = torch.empty_like(k) if (need_k or need_v) else None
        dv = torch.empty_like(v) if (need_k or need_v) else None
        delta = torch.empty(bh, n, device=q.device, dtype=q.dtype)
        _hip.check(lib.sp_attention_bwd(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(out),
                                        _hip.ptr(dout), _hip.ptr(lse), bh, n, d, ctx.scale,
                                        _hip.ptr(delta), _hip.ptr(dq), _hip.ptr(dk), _hip.ptr(dv),
                                        _hip.stream_of(q)), "sp_attention_bwd")
        return dq, (dk if need_k else None), (dv if need_v else None)


class _FusedQKVAttention(torch.autograd.Function):
    """Multi-head self-attention straight on the fused projection's output ``qkv``
    ([b][n][3 heads d]: the q, k, v thirds) into ``out`` ([b][n][heads d]), on the fused
    kernels' strided entry points: no head split / merge copies either way; the VJP writes
    dq, dk, dv into one [b][n][3 heads d] buffer, the fused projection's cotangent."""

    @staticmethod
    def forward(ctx, qkv: Tensor, heads: int) -> Tensor:
        from .. import _hip

        lib = _hip.load_library()
        b, n, c3 = qkv.shape
        c = c3 // 3
        d = c // heads
        scale = 1.0 / math.sqrt(d)
        qkv = qkv.contiguous()
        out = torch.empty(b, n, c, device=qkv.device, dtype=torch.float32)
        lse = torch.empty(b * heads, n, device=qkv.device, dtype=torch.float32)
        base = qkv.data_ptr()
        if not split_bf16_forward(qkv, qkv, qkv, b, heads, n, d, c3, c, scale, out, lse,
                                  offsets=(0, 4 * c, 8 * c)):
            _hip.check(lib.sp_attention_fwd_mh(base, base + 4 * c, base + 8 * c, b, heads, n, n, d, c3, c3, b,
                                               c, scale, _hip.ptr(out), _hip.ptr(lse), _hip.stream_of(qkv)),
                       "sp_attention_fwd_mh")
        ctx.save_for_backward(qkv, out, lse)
        ctx.heads, ctx.scale = heads, scale
        return out

    @staticmethod
    def backward(ctx, dout: Tensor):
        from .. import _hip

        qkv, out, lse = ctx.saved_tensors
        lib = _hip.load_library()
        b, n, c3 = qkv.shape
        c = c3 // 3
        heads = ctx.heads
        d = c // heads
        dout = dout.contiguous()
        dqkv = torch.empty_like(qkv)
        delta = torch.empty(b * heads, n, device=qkv.device, dtype=torch.float32)
        base, dbase = qkv.data_ptr(), dqkv.data_ptr()
        _hip.check(lib.sp_attention_bwd_mh(base, base + 4 * c, base + 8 * c, _hip.ptr(out), _hip.ptr(dout),
                                           _hip.ptr(lse), b, heads, n, n, d, c3, c3, b, c, ctx.scale,
                                           _hip.ptr(delta), dbase, dbase + 4 * c, dbase + 8 * c,
                                           _hip.stream_of(dout)),
                   "sp_attention_bwd_mh")
        return dqkv, None


class _FusedCrossAttention(torch.autograd.Function):
    """Multi-head cross-attention of token rows q ([b][n][heads d]) to a context's keys and
    values ([bc][m][heads d], bc = 1: one context for the whole batch, or bc = b) on the fused
    kernels (keys past m masked; scores never in HBM), output in the token layout; the VJP
    is dq only (the context is a constant of the prior's call)."""

    @staticmethod
    def forward(ctx, q: Tensor, k: Tensor, v: Tensor, heads: int) -> Tensor:
        from .. import _hip

        lib = _hip.load_library()
        b, n, c = q.shape
        bc, m, _ = k.shape
        d = c // heads
        scale = 1.0 / math.sqrt(d)
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        out = torch.empty(b, n, c, device=q.device, dtype=torch.float32)
        lse = torch.empty(b * heads, n, device=q.device, dtype=torch.float32)
        _hip.check(lib.sp_attention_fwd_mh(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), b, heads, n, m, d, c, c, bc, c,
                                           scale, _hip.ptr(out), _hip.ptr(lse), _hip.stream_of(q)),
                   "sp_attention_fwd_mh")
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.heads, ctx.scale = heads, scale
        return out

    @staticmethod
    def backward(ctx, dout: Tensor):
        from .. import _hip

        q, k, v, out, lse = ctx.saved_tensors
        lib = _hip.load_library()
        b, n, c = q.shape
        bc, m, _ = k.shape
        heads = ctx.heads
        dout = dout.contiguous()
        dq = torch.empty_like(q)
        delta = torch.empty(b * heads, n, device=q.device, dtype=torch.float32)
        _hip.check(lib.sp_attention_bwd_mh(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(out), _hip.ptr(dout),
                                           _hip.ptr(lse), b, heads, n, m, c // heads, c, c, bc, c, ctx.scale,
                                           _hip.ptr(delta), _hip.ptr(dq), None, None, _hip.stream_of(dout)),
                   "sp_attention_bwd_mh")
        return dq, None, None, None


def fused_cross_supported(q: Tensor, k: Tensor, heads: int) -> bool:
    """``_FusedCrossAttention`` serves this call: fp32 device tensors, a context that needs no
    gradient, one context row or one per sample, the kernels' head dims and query counts."""
    if not (q.is_cuda and q.dtype == torch.float32 and k.dtype == torch.float32 and q.dim() == 3
            and k.dim() == 3 and not k.requires_grad):
        return False
    if os.environ.get("SAMPLERS_AMD_LATENT_ATTN", "fused").lower() == "gemm":
        return False
    from .. import _hip

    b, n, c = q.shape
    bc, m, ck = k.shape
    return (ck == c and c % heads == 0 and bc in (1, b)
            and bool(_hip.load_library().sp_attention_mh_supported(b, heads, n, m, c // heads)))


def fused_cross_attention(q: Tensor, k: Tensor, v: Tensor, heads: int) -> Tensor:
    return _FusedCrossAttention.apply(q, k, v, heads)


def fused_qkv_supported(x: Tensor, heads: int) -> bool:
    """``_FusedQKVAttention`` serves self-attention over ``x`` ((b, n, c) fp32 on the device)
    with this head count: the fused kernels' head dims and token counts, and at least
    ``FUSED_BWD_MIN_TOKENS`` tokens (below that the GEMM VJP wins, see above)."""
    if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 3):
        return False
    if os.environ.get("SAMPLERS_AMD_LATENT_ATTN", "fused").lower() == "gemm":
        return False
    from .. import _hip

    b, n, c = x.shape
    return (c % heads == 0 and n >= FUSED_BWD_MIN_TOKENS
            and bool(_hip.load_library().sp_attention_supported(b * heads, n, n, c // heads)))


def fused_qkv_attention(qkv: Tensor, heads: int) -> Tensor:
    return _FusedQKVAttention.apply(qkv, heads)


def fused_supported(q: Tensor, k: Tensor) -> bool:
    """The fused kernels serve this call (fp32 device self-attention at their head dims and
    token counts; ``SAMPLERS_AMD_LATENT_ATTN=gemm`` forces the GEMM path)."""
    if not (q.is_cuda and q.dtype == torch.float32 and k.dtype == torch.float32 and q.dim() == 3):
        return False
    if os.environ.get("SAMPLERS_AMD_LATENT_ATTN", "fused").lower() == "gemm":
        return False
    from .. import _hip

    bh, n, d = q.shape
    return k.shape == q.shape and bool(_hip.load_library().sp_attention_supported(bh, n, k.shape[1], d))


def attention(q: Tensor, k: Tensor, v: Tensor) -> Tensor:
    """softmax(q kᵀ/√d) v over (batch·heads, tokens, d) fp32 tensors.  On the device:
    self-attention at the fused kernels' shapes runs on them (``_FusedAttention``); other
    calls (cross-attention to the 77-token context) recompute the score blocks in the VJP
    instead of keeping them (see the module doc)."""
    if not q.is_cuda:
        return torch.softmax(_scores(q, k, 1.0 / math.sqrt(q.shape[-1])), dim=-1) @ v
    q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
    if v.shape == q.shape and fused_supported(q, k):
        return _FusedAttention.apply(q, k, v)
    return _RecomputeAttention.apply(q, k, v)

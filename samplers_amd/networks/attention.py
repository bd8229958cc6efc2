"""Multi-head attention for the latent prior with an O(N·d) memory footprint under autograd.

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
        scale = ctx.scale
        dout = dout.contiguous()
        bh, n, _ = q.shape
        m = k.shape[1]
        need_q, need_k, need_v = ctx.needs_input_grad[:3]
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


def attention(q: Tensor, k: Tensor, v: Tensor) -> Tensor:
    """softmax(q kᵀ/√d) v over (batch·heads, tokens, d) fp32 tensors; on the device the
    score blocks are recomputed in the VJP instead of being kept (see the module doc)."""
    if not q.is_cuda:
        return torch.softmax(_scores(q, k, 1.0 / math.sqrt(q.shape[-1])), dim=-1) @ v
    return _RecomputeAttention.apply(q.contiguous(), k.contiguous(), v.contiguous())

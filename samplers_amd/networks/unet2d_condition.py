"""Latent ε-prior of Stable Diffusion 1.5: a structural equivalent of diffusers'
``UNet2DConditionModel`` (the network ``StableDiffusionNetwork.forward`` calls with
``encoder_hidden_states``, ``/root/reference/samplers/networks/diffusers/stable_diffusion.py:300-313``).

Architecture (SD 1.5 ``unet/config.json``): 4 → 4 latent channels, levels of
320/640/1280/1280 channels, 2 residual blocks per down level and 3 per up level,
``CrossAttnDownBlock2D`` ×3 + ``DownBlock2D`` / ``UpBlock2D`` + ``CrossAttnUpBlock2D`` ×3,
``UNetMidBlock2DCrossAttn``; 8 attention heads (head dim 40/80/160); one
``Transformer2DModel`` per residual block at the cross-attention levels (GroupNorm(32,
eps=1e-6) → 1x1 ``proj_in`` → LayerNorm / self-attention / LayerNorm / cross-attention to
the 77 x 768 text context / LayerNorm / GEGLU feed-forward (4x) → 1x1 ``proj_out`` →
residual); GroupNorm(32, eps=1e-5) + SiLU in the residual blocks; sinusoidal time
embedding with ``flip_sin_to_cos=True, freq_shift=0`` into a 1280-wide MLP; stride-2
downsampling with ``padding=1``.  859.5 M parameters, random-initialised with a fixed
seed (no checkpoint offline); the parameter names follow diffusers' state-dict keys, so a
local SD 1.5 ``unet`` safetensors file loads unchanged (``load_state_dict``).

On the device the residual blocks run this project's kernels exactly as in the pixel
UNet (``unet2d.ResnetBlock2D``: HIP GroupNorm+SiLU, Winograd / direct fp32-MFMA 3x3
convolutions, residual in the conv epilogue, skip gradients added inside the VJP
kernels); in the transformer blocks every ``nn.Linear`` (to_q/k/v/out, GEGLU, FF out,
proj_in/out) runs on the split-bf16 GEMM (``layers.Linear``: fp32 operands as exact
three-term bf16 splits on the bf16 MFMAs), self-attention on the fused fp32-MFMA kernels
(``attention.py``, scores never in HBM); cross-attention's scores / softmax over the 77
context tokens and the LayerNorms are torch ops.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import Tensor, nn

from .attention import (attention, fused_cross_attention, fused_cross_supported, fused_qkv_attention,
                        fused_qkv_supported)
from .layers import (Conv3x3, GroupNormAct, LayerNorm, Linear, SkipGrad, conv3x3_stride2, geglu,
                     linear, proj_nchw_to_tokens, proj_tokens_to_nchw)
from .unet2d import (ResnetBlock2D, TimestepEmbedding, Upsample2D, _as_nchw, temb_projections,
                     timestep_embedding, timestep_rows)


@dataclass(frozen=True)
class UNet2DConditionConfig:
    sample_size: int = 64
    in_channels: int = 4
    out_channels: int = 4
    block_out_channels: tuple[int, ...] = (320, 640, 1280, 1280)
    # levels built as CrossAttnDownBlock2D (and, mirrored, CrossAttnUpBlock2D)
    cross_attention_levels: tuple[int, ...] = (0, 1, 2)
    layers_per_block: int = 2
    attention_heads: int = 8
    cross_attention_dim: int = 768
    norm_num_groups: int = 32
    norm_eps: float = 1e-5
    transformer_norm_eps: float = 1e-6
    flip_sin_to_cos: bool = True
    freq_shift: int = 0
    context_tokens: int = 77  # CLIP ViT-L/14 sequence length (the synthetic null context)


SD15_UNET = UNet2DConditionConfig()


class _Holder:
    """A weight outside the module tree (the concatenated q/k/v projection): ``linear`` caches
    its packed form on this object."""

    def __init__(self, weight: Tensor) -> None:
        self.weight = weight


class Attention(nn.Module):
    """diffusers ``Attention`` without biases on q/k/v (``to_out.0`` has one): self-attention
    when ``context`` is None, else cross-attention to it."""

    def __init__(self, dim: int, heads: int, context_dim: int | None = None) -> None:
        super().__init__()
        kv_dim = context_dim or dim
        self.heads = heads
        self.to_q = Linear(dim, dim, bias=False)
        self.to_k = Linear(kv_dim, dim, bias=False)
        self.to_v = Linear(kv_dim, dim, bias=False)
        self.to_out = nn.ModuleList([Linear(dim, dim)])

    def _qkv_weight(self) -> Tensor:
        """[W_q; W_k; W_v] ([3 dim][dim]), rebuilt when a weight changes (state-dict load)."""
        ws = (self.to_q.weight, self.to_k.weight, self.to_v.weight)
        key = tuple((w.data_ptr(), w._version, w.device) for w in ws)
        cache = self.__dict__.setdefault("_qkv", {})
        if cache.get("key") != key:
            holder = _Holder(torch.cat([w.detach() for w in ws], 0))
            cache.clear()
            cache.update(key=key, holder=holder)
        return cache["holder"]

    def _split(self, t: Tensor) -> Tensor:
        b, n, c = t.shape
        h = self.heads
        return t.reshape(b, n, h, c // h).transpose(1, 2).reshape(b * h, n, c // h)

    def _forward_bf16(self, x: Tensor, context: Tensor | None) -> Tensor | None:
        """bf16 attention on the fused kernels (networks/bf16.py), or None where they do not
        serve the shape."""
        from . import bf16

        b, n, c = x.shape
        d = c // self.heads
        if context is None:
            if not (bf16.attention_supported(b, self.heads, n, n, d) and bf16.vjp_supported(b, self.heads, n, n, d)):
                return None
            qkv = torch.nn.functional.linear(x, self._qkv_weight().weight)
            return bf16.self_attention(qkv, self.heads)
        bc, m = context.shape[0], context.shape[1]
        if bc not in (1, b) or context.requires_grad or not (
                bf16.attention_supported(b, self.heads, n, m, d) and bf16.vjp_supported(b, self.heads, n, m, d)):
            return None
        q, k, v = self.to_q(x), self.to_k(context), self.to_v(context)
        return bf16.cross_attention(q, k, v, self.heads)

    def forward(self, x: Tensor, context: Tensor | None = None, res: Tensor | None = None,
                box: SkipGrad | None = None) -> Tensor:
        """``res`` is added in ``to_out``'s epilogue (the block's residual); ``box`` carries
        its gradient to the LayerNorm VJP that adds it (``layers.linear``)."""
        b, n, c = x.shape
        if x.is_cuda and x.dtype == torch.bfloat16 and not self.to_q.weight.requires_grad:
            o = self._forward_bf16(x, context)
            if o is not None:
                return self.to_out[0](o, res, box)
        if context is None and not self.to_q.weight.requires_grad and fused_qkv_supported(x, self.heads):
            # one projection for q, k, v; attention reads its thirds in place
            h = self._qkv_weight()
            qkv = linear(x, h, h.weight, None)
            if qkv.dim() == 3 and qkv.is_cuda:
                o = fused_qkv_attention(qkv, self.heads)
                return self.to_out[0](o, res, box)
        if context is not None and x.is_cuda and not self.to_q.weight.requires_grad:
            # cross-attention straight on the projections' token rows (one context row may
            # serve the whole batch); keys past the context's length masked in the kernel
            q, k, v = self.to_q(x), self.to_k(context), self.to_v(context)
            if fused_cross_supported(q, k, self.heads) and not v.requires_grad:
                return self.to_out[0](fused_cross_attention(q, k, v, self.heads), res, box)
            q = self._split(q)
            k, v = self._split(k), self._split(v)
            if k.shape[0] == self.heads and b > 1:
                k, v = (t.unsqueeze(0).expand(b, *t.shape).reshape(b * self.heads, *t.shape[1:])
                        for t in (k, v))
            o = attention(q, k, v).reshape(b, self.heads, n, -1).transpose(1, 2).reshape(b, n, c)
            return self.to_out[0](o, res, box)
        q = self._split(self.to_q(x))
        src = x if context is None else context
        k, v = self._split(self.to_k(src)), self._split(self.to_v(src))
        if src.shape[0] == 1 and b > 1:  # one context row shared by the whole batch:
            # project it once, then broadcast the (heads, tokens, d) keys / values
            k, v = (t.unsqueeze(0).expand(b, *t.shape).reshape(b * self.heads, *t.shape[1:])
                    for t in (k, v))
        o = attention(q, k, v)
        o = o.reshape(b, self.heads, n, -1).transpose(1, 2).reshape(b, n, c)
        return self.to_out[0](o, res, box)


class GEGLU(nn.Module):
    def __init__(self, dim: int, inner: int) -> None:
        super().__init__()
        self.proj = Linear(dim, 2 * inner)

    def forward(self, x: Tensor) -> Tensor:
        return geglu(self.proj(x))  # a * gelu(gate), a, gate = proj(x).chunk(2, -1)


class FeedForward(nn.Module):
    def __init__(self, dim: int, mult: int = 4) -> None:
        super().__init__()
        # diffusers' ModuleList layout: [GEGLU, Dropout, Linear]
        self.net = nn.ModuleList([GEGLU(dim, dim * mult), nn.Dropout(0.0), Linear(dim * mult, dim)])

    def forward(self, x: Tensor, res: Tensor | None = None, box: SkipGrad | None = None) -> Tensor:
        return self.net[2](self.net[0](x), res, box)


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim: int, heads: int, context_dim: int) -> None:
        super().__init__()
        self.norm1 = LayerNorm(dim)
        self.attn1 = Attention(dim, heads)
        self.norm2 = LayerNorm(dim)
        self.attn2 = Attention(dim, heads, context_dim)
        self.norm3 = LayerNorm(dim)
        self.ff = FeedForward(dim)

    def forward(self, x: Tensor, context: Tensor) -> Tensor:
        # x + f(norm(x)) three times: the residual is added in f's last linear, and its
        # gradient rides into the norm's VJP kernel (one box per residual)
        grad = torch.is_grad_enabled() and x.is_cuda
        box = (lambda: SkipGrad()) if grad else (lambda: None)  # noqa: E731
        b1 = box()
        x = self.attn1(self.norm1(x, b1), res=x, box=b1)
        b2 = box()
        x = self.attn2(self.norm2(x, b2), context, res=x, box=b2)
        b3 = box()
        return self.ff(self.norm3(x, b3), res=x, box=b3)


class Transformer2DModel(nn.Module):
    """GroupNorm → 1x1 proj_in → tokens → BasicTransformerBlock → 1x1 proj_out → residual."""

    def __init__(self, channels: int, heads: int, context_dim: int, groups: int, eps: float) -> None:
        super().__init__()
        self.norm = GroupNormAct(groups, channels, eps=eps)
        self.proj_in = nn.Conv2d(channels, channels, 1)
        self.transformer_blocks = nn.ModuleList([BasicTransformerBlock(channels, heads, context_dim)])
        self.proj_out = nn.Conv2d(channels, channels, 1)

    def forward(self, x: Tensor, context: Tensor) -> Tensor:
        # NCHW -> token rows and back inside the two 1x1 projections' loads / stores; the
        # residual x added in proj_out's epilogue
        box = SkipGrad() if torch.is_grad_enabled() and x.is_cuda else None  # x's residual gradient
        tokens = proj_nchw_to_tokens(self.norm(x, box=box), self.proj_in)
        for blk in self.transformer_blocks:
            tokens = blk(tokens, context)
        return proj_tokens_to_nchw(tokens, self.proj_out, x, box=box)


class Downsample2D(nn.Module):
    """Stride-2 3x3 conv with ``padding=1`` (diffusers' ``downsample_padding=1``)."""

    def __init__(self, channels: int) -> None:
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, stride=2, padding=1)

    def forward(self, x: Tensor, box: SkipGrad | None = None) -> Tensor:
        if box is not None:  # no accumulate mode on this path: autograd adds the skip gradient
            box.enabled = False
        return conv3x3_stride2(self.conv, x, padding=1)


class _Level(nn.Module):
    def __init__(self) -> None:
        super().__init__()
        self.resnets = nn.ModuleList()
        self.attentions = nn.ModuleList()


class UNet2DConditionModel(nn.Module):
    """``forward(sample, timestep, encoder_hidden_states) -> eps`` over latents."""

    def __init__(self, config: UNet2DConditionConfig = SD15_UNET) -> None:
        super().__init__()
        self.config = c = config
        ch, g, eps = c.block_out_channels, c.norm_num_groups, c.norm_eps
        temb = ch[0] * 4

        def xf(cc: int) -> Transformer2DModel:
            return Transformer2DModel(cc, c.attention_heads, c.cross_attention_dim, g,
                                      c.transformer_norm_eps)

        self.conv_in = Conv3x3(c.in_channels, ch[0])
        self.time_embedding = TimestepEmbedding(ch[0], temb)

        self.down_blocks = nn.ModuleList()
        cout = ch[0]
        for i, co in enumerate(ch):
            cin, cout = cout, co
            lvl = _Level()
            for j in range(c.layers_per_block):
                lvl.resnets.append(ResnetBlock2D(cin if j == 0 else cout, cout, temb, g, eps))
                if i in c.cross_attention_levels:
                    lvl.attentions.append(xf(cout))
            lvl.downsamplers = nn.ModuleList([Downsample2D(cout)]) if i < len(ch) - 1 else None
            self.down_blocks.append(lvl)

        mid = ch[-1]
        self.mid_block = _Level()
        self.mid_block.resnets.append(ResnetBlock2D(mid, mid, temb, g, eps))
        self.mid_block.attentions.append(xf(mid))
        self.mid_block.resnets.append(ResnetBlock2D(mid, mid, temb, g, eps))

        self.up_blocks = nn.ModuleList()
        rev = list(reversed(ch))
        nlev = len(ch)
        prev = rev[0]
        for i, co in enumerate(rev):
            skip_in = rev[min(i + 1, nlev - 1)]
            lvl = _Level()
            for j in range(c.layers_per_block + 1):
                res_skip = skip_in if j == c.layers_per_block else co
                res_in = prev if j == 0 else co
                lvl.resnets.append(ResnetBlock2D(res_in + res_skip, co, temb, g, eps))
                if (nlev - 1 - i) in c.cross_attention_levels:
                    lvl.attentions.append(xf(co))
            lvl.upsamplers = nn.ModuleList([Upsample2D(co)]) if i < nlev - 1 else None
            self.up_blocks.append(lvl)
            prev = co

        self.conv_norm_out = GroupNormAct(g, ch[0], eps=eps, act=True)
        self.conv_out = Conv3x3(ch[0], c.out_channels)

    def forward(self, sample: Tensor, timestep: Tensor | int, encoder_hidden_states: Tensor) -> Tensor:
        cfg = self.config
        b = sample.shape[0]
        table = timestep_rows(self, timestep, sample)  # host timestep: rows of a table over t
        if table is not None:
            emb, tbs = table
        else:
            if not torch.is_tensor(timestep):
                timestep = torch.tensor([timestep], dtype=torch.long, device=sample.device)
            timestep = timestep.reshape(-1).to(sample.device).expand(b)
            t_emb = timestep_embedding(timestep, cfg.block_out_channels[0],
                                       flip_sin_to_cos=cfg.flip_sin_to_cos,
                                       freq_shift=cfg.freq_shift).to(sample.dtype)
            emb = self.time_embedding(t_emb)
            tbs = temb_projections(self, emb)  # every block's time-embedding projection at once
        ctx = encoder_hidden_states.to(sample.dtype)

        # skip tensors' two gradients meet inside the down-path consumer's VJP kernel
        # (unet2d.UNet2DModel.forward, SkipGrad)
        mail = torch.is_grad_enabled() and sample.is_cuda
        new_box = (lambda: SkipGrad()) if mail else (lambda: None)  # noqa: E731
        h = self.conv_in(sample)
        skips, boxes = [h], [new_box()]
        for lvl in self.down_blocks:
            for j, res in enumerate(lvl.resnets):
                h = res(h, emb, box_in=boxes[-1] if skips[-1] is h else None, tb=tbs.get(id(res)))
                if len(lvl.attentions):
                    h = lvl.attentions[j](h, ctx)
                skips.append(h)
                boxes.append(new_box())
            if lvl.downsamplers is not None:
                h = lvl.downsamplers[0](h, box=boxes[-1])
                skips.append(h)
                boxes.append(new_box())

        m0, m1 = self.mid_block.resnets
        h = m0(h, emb, box_in=boxes[-1], tb=tbs.get(id(m0)))
        h = self.mid_block.attentions[0](h, ctx)
        h = m1(h, emb, tb=tbs.get(id(m1)))

        for lvl in self.up_blocks:
            for j, res in enumerate(lvl.resnets):
                h = res(h, emb, skip=skips.pop(), box_out=boxes.pop(), tb=tbs.get(id(res)))
                if len(lvl.attentions):
                    h = lvl.attentions[j](h, ctx)
            if lvl.upsamplers is not None:
                h = lvl.upsamplers[0](h)

        return _as_nchw(self.conv_out(self.conv_norm_out(h)))


def null_context(config: UNet2DConditionConfig = SD15_UNET, *, seed: int = 7,
                 device=None, dtype: torch.dtype = torch.float32) -> Tensor:
    """A fixed synthetic stand-in for the CLIP embedding of the empty prompt, (1, 77, 768)
    (the text encoder is out of scope): unit-variance rows, seeded."""
    gen = torch.Generator().manual_seed(seed)
    ctx = torch.randn(1, config.context_tokens, config.cross_attention_dim, generator=gen)
    return ctx.to(device=device, dtype=dtype)


def build_unet_condition(config: UNet2DConditionConfig = SD15_UNET, *, seed: int = 0, device=None,
                         dtype: torch.dtype = torch.float32) -> UNet2DConditionModel:
    state = torch.random.get_rng_state()
    torch.manual_seed(seed)
    try:
        net = UNet2DConditionModel(config)
    finally:
        torch.random.set_rng_state(state)
    return net.to(device=device, dtype=dtype).eval().requires_grad_(False)

"""Building blocks of the SD1.5 UNet / VAE, parameter-name compatible with diffusers checkpoints.

Module and parameter names follow the diffusers SD1.5 state dict (``down_blocks.0.resnets.0.norm1``,
``…attentions.0.transformer_blocks.0.attn1.to_q`` …) so ``weights.py`` loads the published
safetensors files with no renaming table.  The compute is laid out for MI355X instead of mirroring
diffusers' module graph:

* activations stay channels-last (NHWC memory) end to end: implicit-GEMM 3×3 conv kernels, and the
  transformer's token rows ``[N, H*W, C]`` are a free view of the same memory (no permute copies
  around every Transformer2D);
* GroupNorm + SiLU is one kernel (``functional.group_norm(..., silu=True)``);
* q/k/v of self-attention come from ONE fused projection GEMM (weights concatenated once by
  :meth:`Attention.fuse_qkv`); k/v of cross-attention from one GEMM over the 77 text tokens;
* the 1×1 ``proj_in``/``proj_out`` convolutions run as token-row GEMMs;
* GEGLU's ``h * gelu(g)`` is one elementwise kernel over the projection output.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import functional as SF


class GroupNorm(nn.GroupNorm):
    """``nn.GroupNorm`` whose forward optionally fuses the following SiLU and a per-(n, c) addend
    applied to its input (native kernel)."""

    def forward(self, x: torch.Tensor, silu: bool = False,  # type: ignore[override]
                add: Optional[torch.Tensor] = None) -> torch.Tensor:
        return SF.group_norm(x, self.weight, self.bias, self.num_groups, self.eps, silu, add)


def timestep_embedding(t: torch.Tensor, dim: int, flip_sin_to_cos: bool = True,
                       shift: float = 0.0, max_period: float = 10000.0) -> torch.Tensor:
    """Sinusoidal timestep features (diffusers ``get_timestep_embedding``)."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(half, dtype=torch.float32, device=t.device)
    freqs = torch.exp(exponent / (half - shift))
    args = t.float()[:, None] * freqs[None]
    emb = torch.cat([torch.sin(args), torch.cos(args)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


class TimestepEmbedding(nn.Module):
    def __init__(self, in_dim: int, dim: int):
        super().__init__()
        self.linear_1 = nn.Linear(in_dim, dim)
        self.linear_2 = nn.Linear(dim, dim)

    def forward(self, x):
        return self.linear_2(F.silu(self.linear_1(x)))


class TembAddends:
    """All ResNet time-embedding addends of one UNet forward, from ONE GEMM (see UNet.prepare)."""

    def __init__(self, all_: torch.Tensor):
        self.all = all_


class ResnetBlock2D(nn.Module):
    """GroupNorm+SiLU → conv1 → (+ time embedding) GroupNorm+SiLU → conv2 → + shortcut.

    Epilogues are folded instead of run as separate passes: conv1's bias and the time-embedding
    projection form one per-(n, c) addend that the second GroupNorm applies to its input; conv2's
    (and the 1×1 shortcut's) bias ride in the fused residual add.  Same maths as diffusers'
    ``ResnetBlock2D`` (output_scale_factor 1)."""

    def __init__(self, cin: int, cout: int, temb: Optional[int], groups: int, eps: float):
        super().__init__()
        self.norm1 = GroupNorm(groups, cin, eps=eps)
        self.conv1 = nn.Conv2d(cin, cout, 3, padding=1)
        self.time_emb_proj = nn.Linear(temb, cout) if temb else None
        self.norm2 = GroupNorm(groups, cout, eps=eps)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1)
        self.conv_shortcut = nn.Conv2d(cin, cout, 1) if cin != cout else None
        self._temb_off = None          # (start, end) in TembAddends.all, set by UNet.prepare
        self._out_bias: Optional[torch.Tensor] = None

    @torch.no_grad()
    def fuse_biases(self) -> None:
        b = self.conv2.bias
        if self.conv_shortcut is not None:
            b = b + self.conv_shortcut.bias
        self._out_bias = b.detach().clone()

    def _addend(self, temb, n: int) -> torch.Tensor:
        if isinstance(temb, TembAddends):
            s, e = self._temb_off
            return temb.all[:, s:e]
        if temb is not None and self.time_emb_proj is not None:
            return self.time_emb_proj(temb) + self.conv1.bias
        return self.conv1.bias.expand(n, -1)

    def forward(self, x, temb=None):
        """``temb``: ``silu(temb)`` [N, 1280], a :class:`TembAddends`, or None (VAE)."""
        h = SF.conv3x3(self.norm1(x, silu=True), self.conv1)
        h = self.norm2(h, silu=True, add=self._addend(temb, x.shape[0]))
        if self.conv_shortcut is not None:
            sc = SF.conv1x1(x, self.conv_shortcut.weight)
        else:
            sc = x
        bias = self._out_bias
        if bias is None or bias.device != h.device or bias.dtype != h.dtype:
            bias = self.conv2.bias if self.conv_shortcut is None \
                else self.conv2.bias + self.conv_shortcut.bias
        return SF.conv3x3(h, self.conv2, bias, residual=sc)   # conv2 + biases + shortcut, one pass


class Attention(nn.Module):
    """Multi-head attention with diffusers' parameter names (``to_q/to_k/to_v/to_out.0``)."""

    def __init__(self, dim: int, heads: int, context_dim: Optional[int] = None, bias_qkv=False):
        super().__init__()
        self.heads = heads
        self.is_cross = context_dim is not None
        kv_dim = context_dim or dim
        self.to_q = nn.Linear(dim, dim, bias=bias_qkv)
        self.to_k = nn.Linear(kv_dim, dim, bias=bias_qkv)
        self.to_v = nn.Linear(kv_dim, dim, bias=bias_qkv)
        self.to_out = nn.ModuleList([nn.Linear(dim, dim), nn.Dropout(0.0)])
        self._w_qkv: Optional[torch.Tensor] = None   # fused [3C, C] (self) / [2C, Ck] (cross kv)
        self._b_qkv: Optional[torch.Tensor] = None

    @torch.no_grad()
    def fuse_qkv(self) -> None:
        """Concatenate the projection weights once (after loading / moving / casting)."""
        if self.is_cross:
            self._w_qkv = torch.cat([self.to_k.weight, self.to_v.weight], 0).contiguous()
            parts = [self.to_k.bias, self.to_v.bias]
        else:
            self._w_qkv = torch.cat([self.to_q.weight, self.to_k.weight, self.to_v.weight],
                                    0).contiguous()
            parts = [self.to_q.bias, self.to_k.bias, self.to_v.bias]
        self._b_qkv = torch.cat(parts, 0).contiguous() if parts[0] is not None else None

    def unfuse(self) -> None:
        self._w_qkv = self._b_qkv = None

    def forward(self, x: torch.Tensor, context: Optional[torch.Tensor] = None) -> torch.Tensor:
        c = x.shape[-1]
        if self._w_qkv is not None and self._w_qkv.device == x.device \
                and self._w_qkv.dtype == x.dtype:
            if self.is_cross:
                q = SF.linear(x, self.to_q.weight, self.to_q.bias)
                kv = SF.linear(context, self._w_qkv, self._b_qkv)
                k, v = kv[..., :c], kv[..., c:]
            else:
                qkv = SF.linear(x, self._w_qkv, self._b_qkv)
                q, k, v = qkv[..., :c], qkv[..., c:2 * c], qkv[..., 2 * c:]
        else:
            ctx = context if self.is_cross else x
            q, k, v = self.to_q(x), self.to_k(ctx), self.to_v(ctx)
        o = SF.attention(q, k, v, self.heads)
        out = self.to_out[0]
        return SF.linear(o, out.weight, out.bias)


class GEGLU(nn.Module):
    def __init__(self, dim: int, inner: int):
        super().__init__()
        self.proj = nn.Linear(dim, inner * 2)

    def forward(self, x):
        return SF.geglu(SF.linear(x, self.proj.weight, self.proj.bias))


class FeedForward(nn.Module):
    def __init__(self, dim: int, mult: int = 4):
        super().__init__()
        inner = dim * mult
        self.net = nn.ModuleList([GEGLU(dim, inner), nn.Dropout(0.0), nn.Linear(inner, dim)])

    def forward(self, x, residual: Optional[torch.Tensor] = None):
        out = self.net[2]
        if residual is not None:       # residual + FF(x): the add rides in the GEMM epilogue
            return SF.linear_add(self.net[0](x), out.weight, out.bias, residual)
        return SF.linear(self.net[0](x), out.weight, out.bias)


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim: int, heads: int, context_dim: int):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim)
        self.attn1 = Attention(dim, heads)
        self.norm2 = nn.LayerNorm(dim)
        self.attn2 = Attention(dim, heads, context_dim)
        self.norm3 = nn.LayerNorm(dim)
        self.ff = FeedForward(dim)

    def forward(self, x, context):
        n1, n2, n3 = self.norm1, self.norm2, self.norm3
        h = SF.add_layernorm(x, None, n1.weight, n1.bias, n1.eps)
        x, h = SF.add_layernorm(x, self.attn1(h), n2.weight, n2.bias, n2.eps)
        x, h = SF.add_layernorm(x, self.attn2(h, context), n3.weight, n3.bias, n3.eps)
        return self.ff(h, residual=x)


class Transformer2DModel(nn.Module):
    """SD1.5 spatial transformer: GroupNorm → 1×1 proj_in → 1 block → 1×1 proj_out (+ residual)."""

    def __init__(self, channels: int, heads: int, context_dim: int, groups: int, eps: float):
        super().__init__()
        self.norm = GroupNorm(groups, channels, eps=eps)
        self.proj_in = nn.Conv2d(channels, channels, 1)
        self.transformer_blocks = nn.ModuleList([BasicTransformerBlock(channels, heads, context_dim)])
        self.proj_out = nn.Conv2d(channels, channels, 1)

    @staticmethod
    def _as_linear(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
        return SF.linear(x, conv.weight.view(conv.out_channels, conv.in_channels), conv.bias)

    def forward(self, x, context):
        n, c, h, w = x.shape
        residual = x
        y = self.norm(x)
        # channels-last: [N, C, H, W] with NHWC memory IS [N, H*W, C] token rows
        tokens = y.permute(0, 2, 3, 1).reshape(n, h * w, c)
        tokens = self._as_linear(self.proj_in, tokens)
        for blk in self.transformer_blocks:
            tokens = blk(tokens, context)
        po = self.proj_out                # proj_out + the block's residual in one GEMM epilogue
        res_tokens = residual.permute(0, 2, 3, 1).reshape(n, h * w, c)
        tokens = SF.linear_add(tokens, po.weight.view(po.out_channels, po.in_channels), po.bias,
                               res_tokens)
        return tokens.reshape(n, h, w, c).permute(0, 3, 1, 2)


class Downsample2D(nn.Module):
    def __init__(self, channels: int):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, stride=2, padding=1)

    def forward(self, x):
        return SF.conv3x3(x, self.conv, self.conv.bias, stride=2)


class Upsample2D(nn.Module):
    def __init__(self, channels: int):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, padding=1)

    def forward(self, x, size=None):
        """Nearest 2x, or to ``size`` — the next skip's spatial size, which differs from 2x when a
        latent side is not a multiple of 8 (e.g. 520 px → latent 65 → 33 → 17 → 9 → back up to 17),
        as diffusers' ``forward_upsample_size`` does."""
        if size is None or tuple(size) == (2 * x.shape[-2], 2 * x.shape[-1]):
            return SF.conv3x3(x, self.conv, self.conv.bias, up=True)   # upsample folded in
        x = F.interpolate(x, size=tuple(size), mode="nearest")
        if x.device.type == "cuda":
            x = x.contiguous(memory_format=torch.channels_last)
        return SF.conv3x3(x, self.conv, self.conv.bias)


class VAEAttention(nn.Module):
    """Single-head spatial self-attention of the VAE mid block (GroupNorm, biased q/k/v, residual)."""

    def __init__(self, channels: int, groups: int, eps: float):
        super().__init__()
        self.group_norm = GroupNorm(groups, channels, eps=eps)
        self.to_q = nn.Linear(channels, channels)
        self.to_k = nn.Linear(channels, channels)
        self.to_v = nn.Linear(channels, channels)
        self.to_out = nn.ModuleList([nn.Linear(channels, channels), nn.Dropout(0.0)])

    def forward(self, x):
        n, c, h, w = x.shape
        t = self.group_norm(x).permute(0, 2, 3, 1).reshape(n, h * w, c)
        o = SF.attention(self.to_q(t), self.to_k(t), self.to_v(t), 1)
        o = self.to_out[0](o).reshape(n, h, w, c).permute(0, 3, 1, 2)
        return o + x

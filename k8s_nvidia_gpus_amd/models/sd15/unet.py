"""SD1.5 denoising UNet (diffusers ``UNet2DConditionModel`` topology and parameter names).

The reference runs this network inside ``diffusers`` (reference sd15-api/configmap.yaml:41-47,
105-112: 30 steps × UNet on a CFG batch of 2 at 64×64 latents).  Same maths here, laid out for
MI355X (see ``nn.py``): channels-last activations, fused GroupNorm+SiLU, fused q/k/v projections,
native attention, and a forward with no host synchronisation and no data-dependent control flow,
so :class:`~k8s_nvidia_gpus_amd.models.sd15.pipeline.UNetRunner` can capture it in a HIP graph.

At SD1.5 size the model has 859 520 964 parameters (checked by the tests against the published
count of ``runwayml/stable-diffusion-v1-5/unet``).
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn as nn
import torch.nn.functional as F

from .config import UNetConfig
from .nn import (Downsample2D, GroupNorm, ResnetBlock2D, TembAddends, TimestepEmbedding,
                 Transformer2DModel, Upsample2D, timestep_embedding)


class DownBlock(nn.Module):
    """``CrossAttnDownBlock2D`` (with ``attentions``) or ``DownBlock2D`` (without)."""

    def __init__(self, cin, cout, cfg: UNetConfig, attention: bool, downsample: bool):
        super().__init__()
        g, eps = cfg.norm_num_groups, cfg.norm_eps
        self.resnets = nn.ModuleList([
            ResnetBlock2D(cin if i == 0 else cout, cout, cfg.time_embed_dim, g, eps)
            for i in range(cfg.layers_per_block)])
        if attention:
            self.attentions = nn.ModuleList([
                Transformer2DModel(cout, cfg.num_heads, cfg.cross_attention_dim, g,
                                   cfg.transformer_norm_eps)
                for _ in range(cfg.layers_per_block)])
        else:
            self.attentions = None
        self.downsamplers = nn.ModuleList([Downsample2D(cout)]) if downsample else None

    def forward(self, x, temb_act, context, skips: List[torch.Tensor]):
        for i, r in enumerate(self.resnets):
            x = r(x, temb_act)
            if self.attentions is not None:
                x = self.attentions[i](x, context)
            skips.append(x)
        if self.downsamplers is not None:
            x = self.downsamplers[0](x)
            skips.append(x)
        return x


class UpBlock(nn.Module):
    """``CrossAttnUpBlock2D`` / ``UpBlock2D``: ``layers_per_block + 1`` ResNets over concat skips."""

    def __init__(self, prev_out, cout, cin, cfg: UNetConfig, attention: bool, upsample: bool):
        super().__init__()
        g, eps = cfg.norm_num_groups, cfg.norm_eps
        n = cfg.layers_per_block + 1
        res = []
        for i in range(n):
            skip_ch = cin if i == n - 1 else cout
            res_in = prev_out if i == 0 else cout
            res.append(ResnetBlock2D(res_in + skip_ch, cout, cfg.time_embed_dim, g, eps))
        self.resnets = nn.ModuleList(res)
        if attention:
            self.attentions = nn.ModuleList([
                Transformer2DModel(cout, cfg.num_heads, cfg.cross_attention_dim, g,
                                   cfg.transformer_norm_eps) for _ in range(n)])
        else:
            self.attentions = None
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if upsample else None

    def forward(self, x, temb_act, context, skips: List[torch.Tensor]):
        for i, r in enumerate(self.resnets):
            s = skips.pop()
            x = torch.cat([x, s], dim=1)
            x = r(x, temb_act)
            if self.attentions is not None:
                x = self.attentions[i](x, context)
        if self.upsamplers is not None:
            x = self.upsamplers[0](x, skips[-1].shape[-2:] if skips else None)
        return x


class MidBlock(nn.Module):
    """``UNetMidBlock2DCrossAttn``: ResNet → Transformer2D → ResNet."""

    def __init__(self, ch, cfg: UNetConfig):
        super().__init__()
        g, eps = cfg.norm_num_groups, cfg.norm_eps
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch, cfg.time_embed_dim, g, eps)
                                      for _ in range(2)])
        self.attentions = nn.ModuleList([
            Transformer2DModel(ch, cfg.num_heads, cfg.cross_attention_dim, g,
                               cfg.transformer_norm_eps)])

    def forward(self, x, temb_act, context):
        x = self.resnets[0](x, temb_act)
        x = self.attentions[0](x, context)
        return self.resnets[1](x, temb_act)


class UNet2DConditionModel(nn.Module):
    def __init__(self, cfg: UNetConfig = UNetConfig()):
        super().__init__()
        self.cfg = cfg
        ch = cfg.block_out_channels
        self.conv_in = nn.Conv2d(cfg.in_channels, ch[0], 3, padding=1)
        self.time_embedding = TimestepEmbedding(ch[0], cfg.time_embed_dim)
        nb = len(ch)
        self.down_blocks = nn.ModuleList()
        cur = ch[0]
        for i in range(nb):
            self.down_blocks.append(DownBlock(cur, ch[i], cfg, cfg.down_attention[i],
                                              downsample=i < nb - 1))
            cur = ch[i]
        self.mid_block = MidBlock(ch[-1], cfg)
        rch = list(reversed(ch))
        up_attn = list(reversed(cfg.down_attention))
        self.up_blocks = nn.ModuleList()
        prev = rch[0]
        for i in range(nb):
            cout, cin = rch[i], rch[min(i + 1, nb - 1)]
            self.up_blocks.append(UpBlock(prev, cout, cin, cfg, up_attn[i], upsample=i < nb - 1))
            prev = cout
        self.conv_norm_out = GroupNorm(cfg.norm_num_groups, ch[0], eps=cfg.norm_eps)
        self.conv_out = nn.Conv2d(ch[0], cfg.out_channels, 3, padding=1)

    def attention_modules(self):
        from .nn import Attention

        return [m for m in self.modules() if isinstance(m, Attention)]

    def resnets(self) -> List[ResnetBlock2D]:
        return [m for m in self.modules() if isinstance(m, ResnetBlock2D)]

    @torch.no_grad()
    def prepare(self) -> "UNet2DConditionModel":
        """Inference layout (call after .to()): channels-last parameters, fused q/k/v weights,
        folded ResNet biases, and the 22 ResNet time-embedding projections stacked into one
        [ΣC, 1280] GEMM whose bias already holds each conv1 bias."""
        if next(self.parameters()).device.type == "cuda":
            self.to(memory_format=torch.channels_last)
        for a in self.attention_modules():
            a.fuse_qkv()
        ws, bs, off = [], [], 0
        for r in self.resnets():
            r.fuse_biases()
            c = r.conv1.out_channels
            r._temb_off = (off, off + c)
            off += c
            ws.append(r.time_emb_proj.weight)
            bs.append(r.time_emb_proj.bias + r.conv1.bias)
        self._temb_w = torch.cat(ws, 0).contiguous()
        self._temb_b = torch.cat(bs, 0).contiguous()
        return self

    def forward(self, sample: torch.Tensor, timestep: torch.Tensor,
                encoder_hidden_states: torch.Tensor) -> torch.Tensor:
        """``sample`` [N, 4, h, w], ``timestep`` [N] (or scalar), context [N, 77, 768] → ε."""
        if timestep.dim() == 0:
            timestep = timestep.expand(sample.shape[0])
        t = timestep_embedding(timestep, self.cfg.block_out_channels[0],
                               self.cfg.flip_sin_to_cos, self.cfg.freq_shift).to(sample.dtype)
        temb_act = F.silu(self.time_embedding(t))
        tw = getattr(self, "_temb_w", None)
        if tw is not None and tw.dtype == temb_act.dtype and tw.device == temb_act.device:
            temb_act = TembAddends(F.linear(temb_act, tw, self._temb_b))
        x = sample
        if x.device.type == "cuda":
            x = x.contiguous(memory_format=torch.channels_last)
        x = self.conv_in(x)
        skips: List[torch.Tensor] = [x]
        ctx = encoder_hidden_states
        for blk in self.down_blocks:
            x = blk(x, temb_act, ctx, skips)
        x = self.mid_block(x, temb_act, ctx)
        for blk in self.up_blocks:
            x = blk(x, temb_act, ctx, skips)
        x = self.conv_norm_out(x, silu=True)
        return self.conv_out(x)

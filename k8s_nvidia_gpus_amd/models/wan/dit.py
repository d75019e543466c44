"""Wan2.1 text-to-video diffusion transformer (flow matching), MI355X layout.

Parameter names follow the published ``wan2.1_t2v_*.safetensors`` state dict
(``patch_embedding``, ``text_embedding.{0,2}``, ``time_embedding.{0,2}``, ``time_projection.1``,
``blocks.N.{self_attn,cross_attn}.{q,k,v,o,norm_q,norm_k}``, ``blocks.N.norm3``,
``blocks.N.ffn.{0,2}``, ``blocks.N.modulation``, ``head.head``, ``head.modulation``) so
``weights.py`` loads the file the reference's ComfyUI graph names
(reference generate_wan_t2v.py:347) without a renaming table.  The execution plan is MI355X-first
rather than a transcription of the upstream module graph:

* one fused q|k|v GEMM per self-attention (weights concatenated once, :meth:`WanDiT.fuse`), q/k
  RMSNorm + 3-D RoPE in place on that output (``functional.rmsnorm_rope``), attention reading q/k/v
  as strided column views — no head split/permute copies;
* every projection runs on the hand-written gfx950 GEMM (``ops/csrc/gemm_bf16_epi.hip``) with its
  epilogue fused: bias everywhere, tanh-GELU on the FFN input, and the gated residual update
  ``x += gate · (y + b)`` of the o-projections and the FFN output straight from the fp32
  accumulators into the fp32 ``[B, L, C]`` residual stream; the LayerNorm (+ AdaLN modulation)
  that follows each update is one row kernel (``functional.add_ln``);
* cross-attention K/V of the text context are computed ONCE per prompt for all layers
  (:meth:`WanDiT.text_kv`) and reused by every sampling step — the 512-token context never changes
  during denoising;
* classifier-free guidance runs cond and uncond as one batch of 2 (one set of GEMM launches).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import functional as WF
from .config import WanDiTConfig


def sinusoidal(dim: int, t: torch.Tensor) -> torch.Tensor:
    """Wan's timestep features: ``[cos(t·ω), sin(t·ω)]``, ω_i = 10000^(−i/half), in float64."""
    half = dim // 2
    pos = t.to(torch.float64)
    omega = torch.pow(10000.0, -torch.arange(half, dtype=torch.float64, device=t.device) / half)
    s = pos[:, None] * omega[None]
    return torch.cat([torch.cos(s), torch.sin(s)], dim=1).float()


class RMSWeight(nn.Module):
    """Holds the ``weight`` of a Wan RMSNorm (applied by ``functional.rmsnorm_rope``)."""

    def __init__(self, dim: int):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim))


class LNAffine(nn.Module):
    def __init__(self, dim: int):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim))
        self.bias = nn.Parameter(torch.zeros(dim))


class Attn(nn.Module):
    def __init__(self, dim: int):
        super().__init__()
        self.q = nn.Linear(dim, dim)
        self.k = nn.Linear(dim, dim)
        self.v = nn.Linear(dim, dim)
        self.o = nn.Linear(dim, dim)
        self.norm_q = RMSWeight(dim)
        self.norm_k = RMSWeight(dim)


class Block(nn.Module):
    def __init__(self, cfg: WanDiTConfig):
        super().__init__()
        d = cfg.dim
        self.self_attn = Attn(d)
        self.cross_attn = Attn(d)
        self.norm3 = LNAffine(d)
        self.ffn = nn.Sequential(nn.Linear(d, cfg.ffn_dim), nn.GELU(approximate="tanh"),
                                 nn.Linear(cfg.ffn_dim, d))
        self.modulation = nn.Parameter(torch.randn(1, 6, d) / d ** 0.5)
        self._wqkv: Optional[torch.Tensor] = None
        self._bqkv: Optional[torch.Tensor] = None

    def fuse(self) -> None:
        sa = self.self_attn
        self._wqkv = torch.cat([sa.q.weight, sa.k.weight, sa.v.weight], 0).detach()
        self._bqkv = torch.cat([sa.q.bias, sa.k.bias, sa.v.bias], 0).detach()

    def qkv(self, h: torch.Tensor) -> torch.Tensor:
        w = self.self_attn.q.weight
        if self._wqkv is None or self._wqkv.dtype != w.dtype or self._wqkv.device != w.device:
            self.fuse()
        return WF.linear(h, self._wqkv, self._bqkv)


class Head(nn.Module):
    def __init__(self, cfg: WanDiTConfig):
        super().__init__()
        self.head = nn.Linear(cfg.dim, cfg.out_dim * math.prod(cfg.patch))
        self.modulation = nn.Parameter(torch.randn(1, 2, cfg.dim) / cfg.dim ** 0.5)


class WanDiT(nn.Module):
    def __init__(self, cfg: WanDiTConfig):
        super().__init__()
        self.cfg = cfg
        d = cfg.dim
        self.patch_embedding = nn.Conv3d(cfg.in_dim, d, kernel_size=cfg.patch, stride=cfg.patch)
        self.text_embedding = nn.Sequential(nn.Linear(cfg.text_dim, d), nn.GELU(approximate="tanh"),
                                            nn.Linear(d, d))
        self.time_embedding = nn.Sequential(nn.Linear(cfg.freq_dim, d), nn.SiLU(), nn.Linear(d, d))
        self.time_projection = nn.Sequential(nn.SiLU(), nn.Linear(d, 6 * d))
        self.blocks = nn.ModuleList([Block(cfg) for _ in range(cfg.layers)])
        self.head = Head(cfg)
        self._rope_cache = {}
        self._f32 = None        # (key, tensors) of :meth:`_fp32_params`

    # ------------------------------------------------------------------ helpers
    def fuse(self) -> "WanDiT":
        for b in self.blocks:
            b.fuse()
        return self

    def _fp32_params(self):
        """fp32 copies of the small per-block parameters the step reads, stacked once: AdaLN
        modulations with the ``1 +`` of both scale slots folded in ([blocks, 6, d]), norm3
        weight / bias, the head modulation — one add per step instead of ~150 tiny kernels."""
        ps = [b.modulation for b in self.blocks] + [self.head.modulation]
        key = tuple((p.data_ptr(), p._version, str(p.device)) for p in ps)
        if self._f32 is None or self._f32[0] != key:
            with torch.no_grad():
                mod = torch.stack([b.modulation.float()[0] for b in self.blocks])   # [n, 6, d]
                mod[:, 1] += 1.0
                mod[:, 4] += 1.0
                n3w = torch.stack([b.norm3.weight.float() for b in self.blocks])[:, None]
                n3b = torch.stack([b.norm3.bias.float() for b in self.blocks])[:, None]
                head = self.head.modulation.float()[0].clone()                    # [2, d]
                head[1] += 1.0
            self._f32 = (key, (mod, n3w, n3b, head))
        return self._f32[1]

    def grid(self, latent_shape: Sequence[int]) -> Tuple[int, int, int]:
        _, _, f, h, w = latent_shape
        pt, ph, pw = self.cfg.patch
        return f // pt, h // ph, w // pw

    def rope(self, grid, device) -> Tuple[torch.Tensor, torch.Tensor]:
        key = (tuple(grid), str(device))
        if key not in self._rope_cache:
            self._rope_cache[key] = WF.rope_table(grid, self.cfg.head_dim, self.cfg.rope_theta,
                                                  device)
        return self._rope_cache[key]

    def patchify(self, x: torch.Tensor) -> torch.Tensor:
        """[B, C, F, H, W] latent → [B, L, C·pt·ph·pw] rows in the conv weight's (c, t, h, w)
        order, so the patch embedding is one GEMM."""
        b, c, f, h, w = x.shape
        pt, ph, pw = self.cfg.patch
        x = x.reshape(b, c, f // pt, pt, h // ph, ph, w // pw, pw)
        x = x.permute(0, 2, 4, 6, 1, 3, 5, 7)
        return x.reshape(b, (f // pt) * (h // ph) * (w // pw), c * pt * ph * pw)

    def unpatchify(self, y: torch.Tensor, grid) -> torch.Tensor:
        """[B, L, pt·ph·pw·C] head rows (channel fastest) → [B, C, F, H, W]."""
        b = y.shape[0]
        f, h, w = grid
        pt, ph, pw = self.cfg.patch
        c = self.cfg.out_dim
        y = y.reshape(b, f, h, w, pt, ph, pw, c)
        y = y.permute(0, 7, 1, 4, 2, 5, 3, 6)
        return y.reshape(b, c, f * pt, h * ph, w * pw)

    # ------------------------------------------------------------------ text
    def embed_text(self, context: torch.Tensor) -> torch.Tensor:
        """[B, ≤text_len, text_dim] encoder states → [B, text_len, dim] (zero rows pad the tail
        before the embedding MLP, as the published model was trained)."""
        context = context[:, : self.cfg.text_len]
        b, l, c = context.shape
        if l < self.cfg.text_len:
            context = torch.cat([context, context.new_zeros(b, self.cfg.text_len - l, c)], 1)
        t0, t2 = self.text_embedding[0], self.text_embedding[2]
        h = WF.linear_gelu(context.to(t0.weight.dtype), t0.weight, t0.bias)
        return WF.linear(h, t2.weight, t2.bias)

    def text_kv(self, ctx: torch.Tensor) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        """Per-layer cross-attention (K, V) of the embedded context, K already RMS-normalised."""
        out = []
        for blk in self.blocks:
            ca = blk.cross_attn
            k = WF.linear(ctx, ca.k.weight, ca.k.bias)
            WF.rmsnorm_rope(k, ca.norm_k.weight, None, None, self.cfg.heads, self.cfg.eps)
            out.append((k, WF.linear(ctx, ca.v.weight, ca.v.bias)))
        return out

    # ------------------------------------------------------------------ forward
    def time_mod(self, t: torch.Tensor):
        t0, t2, tp = self.time_embedding[0], self.time_embedding[2], self.time_projection[1]
        s = sinusoidal(self.cfg.freq_dim, t).to(t0.weight.dtype)
        e = WF.linear(F.silu(WF.linear(s, t0.weight, t0.bias)), t2.weight, t2.bias)
        e0 = WF.linear(F.silu(e), tp.weight, tp.bias).float().view(-1, 6, self.cfg.dim)
        return e.float(), e0

    def forward(self, x: torch.Tensor, t: torch.Tensor, text_kv, out_dtype=torch.float32,
                sp=None):
        """x: [B, C, F, H, W] latent; t: [B] timesteps (flow sigma × 1000); text_kv: from
        :meth:`text_kv` (batch B).  Returns the velocity prediction [B, C, F, H, W].  With ``sp``
        (:class:`parallel.SequenceParallel`) this rank runs 1/P of the tokens through the blocks
        and self-attention exchanges heads↔tokens with its peers."""
        cfg = self.cfg
        grid = self.grid(x.shape)
        cos, sin = self.rope(grid, x.device)
        wdt = self.patch_embedding.weight.dtype
        pw = self.patch_embedding.weight.reshape(cfg.dim, -1)
        res = WF.linear(self.patchify(x.to(wdt)), pw, self.patch_embedding.bias).float()  # fp32 stream
        if sp is not None and sp.world > 1:
            sp.check(res.shape[1], cfg.heads)
            res, cos, sin = sp.shard(res), sp.shard(cos, 0), sp.shard(sin, 0)

            def attend(q, k, v, heads):
                return sp.attention(q, k, v, heads, WF.attention)
        else:
            attend = WF.attention
        b, l, d = res.shape
        e, e0 = self.time_mod(t)
        mod1, n3w, n3b, head1 = self._fp32_params()
        mods = mod1[:, None] + e0[None]               # [blocks, B, 6, d]; slots 1, 4 hold 1 + scale

        m = mods[0]
        h = WF.add_ln(res, None, None, m[:, 1], m[:, 0], cfg.eps, wdt)
        for i, blk in enumerate(self.blocks):
            m = mods[i]
            # self-attention; x += gate1 · o_proj(attn) fused into the o-projection
            qkv = blk.qkv(h)
            q, k, v = qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:]
            WF.rmsnorm_rope_qk(qkv, blk.self_attn.norm_q.weight, blk.self_attn.norm_k.weight,
                               cos, sin, cfg.heads, cfg.eps)
            so = blk.self_attn.o
            WF.linear_residual_(res, attend(q, k, v, cfg.heads), so.weight, so.bias, m[:, 2])
            h = WF.add_ln(res, None, None, n3w[i], n3b[i], cfg.eps, wdt)
            # cross-attention over the cached text K/V; x += o_proj(attn)
            ca = blk.cross_attn
            qc = WF.linear(h, ca.q.weight, ca.q.bias)
            WF.rmsnorm_rope(qc, ca.norm_q.weight, None, None, cfg.heads, cfg.eps)
            kc, vc = text_kv[i]
            WF.linear_residual_(res, WF.attention(qc, kc, vc, cfg.heads), ca.o.weight, ca.o.bias, None)
            h = WF.add_ln(res, None, None, m[:, 4], m[:, 3], cfg.eps, wdt)
            # feed-forward; x += gate2 · ffn(h)
            f = WF.linear_gelu(h, blk.ffn[0].weight, blk.ffn[0].bias)
            WF.linear_residual_(res, f, blk.ffn[2].weight, blk.ffn[2].bias, m[:, 5])
            if i + 1 < len(self.blocks):
                nm = mods[i + 1]
                h = WF.add_ln(res, None, None, nm[:, 1], nm[:, 0], cfg.eps, wdt)
            else:
                hm = head1 + e[:, None, :]                             # [B, 2, d]
                h = WF.add_ln(res, None, None, hm[:, 1], hm[:, 0], cfg.eps, wdt)
        y = WF.linear(h, self.head.head.weight, self.head.head.bias)
        if sp is not None and sp.world > 1:
            y = sp.gather(y)
        return self.unpatchify(y.to(out_dtype), grid)


def reference_forward(model: WanDiT, x: torch.Tensor, t: torch.Tensor,
                      context: torch.Tensor) -> torch.Tensor:
    """Plain fp32 PyTorch forward written against the upstream module semantics (per-head
    reshapes, complex-number RoPE, separate q/k/v, un-fused residual/LayerNorm, text K/V
    recomputed per layer): the numerics tests compare :meth:`WanDiT.forward` against it."""
    cfg = model.cfg
    P = {k: v.float() for k, v in model.state_dict().items()}
    b = x.shape[0]
    grid = model.grid(x.shape)
    f, hh, ww = grid
    d, nh = cfg.dim, cfg.heads
    hd = d // nh
    xe = F.conv3d(x.float(), P["patch_embedding.weight"], P["patch_embedding.bias"], stride=cfg.patch)
    xe = xe.flatten(2).transpose(1, 2)
    ctx = torch.cat([context.float(), context.new_zeros(b, cfg.text_len - context.shape[1],
                                                        context.shape[2]).float()], 1)
    ctx = F.linear(F.gelu(F.linear(ctx, P["text_embedding.0.weight"], P["text_embedding.0.bias"]),
                          approximate="tanh"), P["text_embedding.2.weight"], P["text_embedding.2.bias"])
    e = F.linear(F.silu(F.linear(sinusoidal(cfg.freq_dim, t), P["time_embedding.0.weight"],
                                 P["time_embedding.0.bias"])), P["time_embedding.2.weight"],
                 P["time_embedding.2.bias"])
    e0 = F.linear(F.silu(e), P["time_projection.1.weight"], P["time_projection.1.bias"]).view(b, 6, d)

    # complex RoPE exactly as the upstream formulation: freqs per section, polar form
    def params(max_len, dim):
        fr = torch.outer(torch.arange(max_len, dtype=torch.float64),
                         1.0 / torch.pow(cfg.rope_theta, torch.arange(0, dim, 2, dtype=torch.float64) / dim))
        return torch.polar(torch.ones_like(fr), fr)

    fr = torch.cat([params(1024, hd - 4 * (hd // 6)), params(1024, 2 * (hd // 6)),
                    params(1024, 2 * (hd // 6))], dim=1)
    c = hd // 2
    parts = fr.split([c - 2 * (c // 3), c // 3, c // 3], dim=1)
    fi = torch.cat([parts[0][:f].view(f, 1, 1, -1).expand(f, hh, ww, -1),
                    parts[1][:hh].view(1, hh, 1, -1).expand(f, hh, ww, -1),
                    parts[2][:ww].view(1, 1, ww, -1).expand(f, hh, ww, -1)], dim=-1).reshape(-1, 1, c)

    def rope(xx):
        xc = torch.view_as_complex(xx.to(torch.float64).reshape(b, -1, nh, c, 2))
        return torch.view_as_real(xc * fi[None]).flatten(3).float()

    def rms(xx, w):
        return xx * torch.rsqrt(xx.pow(2).mean(-1, keepdim=True) + cfg.eps) * w

    def ln(xx):
        return F.layer_norm(xx, (d,), eps=cfg.eps)

    def sdpa(q, k, v):
        q, k, v = (z.reshape(b, z.shape[1], nh, hd).transpose(1, 2) for z in (q, k, v))
        return F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(b, -1, d)

    xs = xe
    for i in range(cfg.layers):
        p = f"blocks.{i}."
        m = (P[p + "modulation"] + e0).chunk(6, dim=1)
        y = ln(xs) * (1 + m[1]) + m[0]
        q = rms(F.linear(y, P[p + "self_attn.q.weight"], P[p + "self_attn.q.bias"]), P[p + "self_attn.norm_q.weight"])
        k = rms(F.linear(y, P[p + "self_attn.k.weight"], P[p + "self_attn.k.bias"]), P[p + "self_attn.norm_k.weight"])
        v = F.linear(y, P[p + "self_attn.v.weight"], P[p + "self_attn.v.bias"])
        o = sdpa(rope(q).reshape(b, -1, d), rope(k).reshape(b, -1, d), v)
        xs = xs + F.linear(o, P[p + "self_attn.o.weight"], P[p + "self_attn.o.bias"]) * m[2]
        y = F.layer_norm(xs, (d,), P[p + "norm3.weight"], P[p + "norm3.bias"], cfg.eps)
        q = rms(F.linear(y, P[p + "cross_attn.q.weight"], P[p + "cross_attn.q.bias"]), P[p + "cross_attn.norm_q.weight"])
        k = rms(F.linear(ctx, P[p + "cross_attn.k.weight"], P[p + "cross_attn.k.bias"]), P[p + "cross_attn.norm_k.weight"])
        v = F.linear(ctx, P[p + "cross_attn.v.weight"], P[p + "cross_attn.v.bias"])
        xs = xs + F.linear(sdpa(q, k, v), P[p + "cross_attn.o.weight"], P[p + "cross_attn.o.bias"])
        y = ln(xs) * (1 + m[4]) + m[3]
        y = F.linear(F.gelu(F.linear(y, P[p + "ffn.0.weight"], P[p + "ffn.0.bias"]), approximate="tanh"),
                     P[p + "ffn.2.weight"], P[p + "ffn.2.bias"])
        xs = xs + y * m[5]
    hm = (P["head.modulation"] + e[:, None]).chunk(2, dim=1)
    y = F.linear(ln(xs) * (1 + hm[1]) + hm[0], P["head.head.weight"], P["head.head.bias"])
    pt, ph, pw = cfg.patch
    co = cfg.out_dim
    y = y.view(b, f, hh, ww, pt, ph, pw, co)
    y = torch.einsum("bfhwpqrc->bcfphqwr", y)
    return y.reshape(b, co, f * pt, hh * ph, ww * pw)

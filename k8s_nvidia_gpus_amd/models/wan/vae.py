"""Wan2.1 causal 3-D VAE decoder (latent [B, 16, T, H/8, W/8] → video [B, 3, 1+4(T−1), H, W]).

Reference workload: ``VAELoader(wan_2.1_vae.safetensors)`` + ``VAEDecode`` in the reference's
ComfyUI graph (generate_wan_t2v.py:349).  Parameter names/shapes are the published file's
(``decoder.conv1``, ``decoder.middle.{0,1,2}``, ``decoder.upsamples.N.{residual,shortcut,resample,
time_conv}``, ``decoder.head``, ``conv2``); encoder tensors are ignored (text-to-video decodes only).

MI355X layout instead of the upstream chunk-by-chunk decode:

* The upstream decoder walks the latent one frame at a time with a per-conv cache of the last two
  input frames; that is exactly a causal convolution over the whole sequence, except that the
  temporal upsampler's ``time_conv`` starts with ZERO history at latent frame 1 and frame 0 passes
  through un-doubled.  This module decodes the WHOLE sequence at once with that semantic made
  explicit (288 GB of HBM holds a 13-frame 512×320 decode many times over), so every convolution is
  one large launch instead of T small ones.
* Activations are per-frame channels-last images ``[B·T, C, H, W]``; a causal 3×3×3 convolution is
  ONE 2-D convolution whose input channels are the three temporal taps stacked
  (``[x_{t−2} | x_{t−1} | x_t]``, zero frames before t = 0) against the weight reshaped to
  ``[Cout, 3·Cin, 3, 3]`` — MIOpen's NHWC implicit GEMM with a 3× deeper K instead of a 3-D conv.
* ``reference_decode`` keeps the upstream chunked algorithm (per-frame loop, feature caches,
  ``nn.functional.conv3d``) for the equivalence tests.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .config import WanVAEConfig


class RMSNorm(nn.Module):
    """``normalize(x, dim=channels) · √C · γ`` (the upstream ``RMS_norm``, bias-free)."""

    def __init__(self, dim: int, images: bool):
        super().__init__()
        self.gamma = nn.Parameter(torch.ones(dim, 1, 1) if images else torch.ones(dim, 1, 1, 1))
        self.scale = dim ** 0.5

    def forward(self, x: torch.Tensor) -> torch.Tensor:       # x: [N, C, H, W]
        g = self.gamma.reshape(1, -1, 1, 1)
        return (F.normalize(x.float(), dim=1) * (self.scale * g.float())).to(x.dtype)


class CausalConv(nn.Module):
    """Causal Conv3d parameters (``weight [Cout, Cin, kt, kh, kw]``) executed as a tap-stacked
    2-D convolution over per-frame images."""

    def __init__(self, cin: int, cout: int, k=3, pad=1):
        super().__init__()
        kt, kh, kw = (k, k, k) if isinstance(k, int) else k
        self.weight = nn.Parameter(torch.randn(cout, cin, kt, kh, kw) * (cin * kt * kh * kw) ** -0.5)
        self.bias = nn.Parameter(torch.zeros(cout))
        self.pad = (pad, pad, pad) if isinstance(pad, int) else pad
        self._w2 = None

    def weight2d(self) -> torch.Tensor:
        if self._w2 is None or self._w2.dtype != self.weight.dtype or self._w2.device != self.weight.device:
            co, ci, kt, kh, kw = self.weight.shape
            self._w2 = self.weight.detach().permute(0, 2, 1, 3, 4).reshape(co, kt * ci, kh, kw).contiguous(
                memory_format=torch.channels_last)
        return self._w2

    def conv_stacked(self, xs: torch.Tensor) -> torch.Tensor:
        """The convolution on an input whose temporal taps are already stacked on channels."""
        return F.conv2d(xs, self.weight2d(), self.bias, padding=self.pad[1:])

    def forward(self, x: torch.Tensor, b: int) -> torch.Tensor:
        """x: [B·T, Cin, H, W] (frames of each sample consecutive) → [B·T, Cout, H, W]."""
        kt = self.weight.shape[2]
        if kt > 1:
            n, c, h, w = x.shape
            t = n // b
            xt = x.reshape(b, t, c, h, w)
            xp = torch.cat([xt.new_zeros(b, kt - 1, c, h, w), xt], 1)
            x = torch.cat([xp[:, i:i + t] for i in range(kt)], 2).reshape(n, kt * c, h, w)
            x = x.contiguous(memory_format=torch.channels_last)
        return F.conv2d(x, self.weight2d(), self.bias, padding=self.pad[1:])


def norm_silu_conv(norm: RMSNorm, conv: "CausalConv", x: torch.Tensor, b: int) -> torch.Tensor:
    """``conv(silu(norm(x)))`` — on the GPU one fused normalise/activate/tap-stack kernel
    (ops/csrc/wan_ops.hip) feeding one 2-D convolution."""
    if x.is_cuda and conv.weight.shape[2] == 3:
        from k8s_nvidia_gpus_amd.ops import wan_kernels as WK

        if WK.vae_rms_silu_supported(x):
            return conv.conv_stacked(WK.vae_rms_silu_stack(x, norm.gamma, x.shape[0] // b, 3))
    return conv(F.silu(norm(x)), b)


class ResidualBlock(nn.Module):
    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.residual = nn.ModuleList([RMSNorm(cin, False), nn.SiLU(), CausalConv(cin, cout),
                                       RMSNorm(cout, False), nn.SiLU(), nn.Dropout(0.0),
                                       CausalConv(cout, cout)])
        self.shortcut = CausalConv(cin, cout, 1, 0) if cin != cout else None

    def forward(self, x, b):
        r = self.residual
        h = norm_silu_conv(r[0], r[2], x, b)
        h = norm_silu_conv(r[3], r[6], h, b)
        return h + (self.shortcut(x, b) if self.shortcut is not None else x)


class AttentionBlock(nn.Module):
    def __init__(self, dim: int):
        super().__init__()
        self.norm = RMSNorm(dim, True)
        self.to_qkv = nn.Conv2d(dim, dim * 3, 1)
        self.proj = nn.Conv2d(dim, dim, 1)

    def forward(self, x, b):
        n, c, h, w = x.shape
        qkv = self.to_qkv(self.norm(x)).flatten(2).transpose(1, 2)          # [n, hw, 3c]
        q, k, v = qkv.unsqueeze(1).chunk(3, dim=-1)
        o = F.scaled_dot_product_attention(q, k, v).squeeze(1)             # [n, hw, c]
        o = o.transpose(1, 2).reshape(n, c, h, w).contiguous(memory_format=torch.channels_last)
        return x + self.proj(o)


class Resample(nn.Module):
    """2× nearest spatial upsample + 3×3 conv halving channels; ``temporal`` adds the causal
    (3,1,1) ``time_conv`` that doubles every frame after the first."""

    def __init__(self, dim: int, temporal: bool):
        super().__init__()
        self.resample = nn.ModuleList([nn.Identity(), nn.Conv2d(dim, dim // 2, 3, padding=1)])
        self.time_conv = CausalConv(dim, dim * 2, (3, 1, 1), (1, 0, 0)) if temporal else None

    def forward(self, x, b):
        n, c, h, w = x.shape
        t = n // b
        if self.time_conv is not None and t > 1:
            xt = x.reshape(b, t, c, h, w)
            rest = xt[:, 1:].reshape(b * (t - 1), c, h, w)
            y = self.time_conv(rest, b).reshape(b, t - 1, 2, c, h, w)      # (pair, c) channels
            y = y.reshape(b, 2 * (t - 1), c, h, w)                           # frame 2i, 2i+1
            x = torch.cat([xt[:, :1], y], 1).reshape(-1, c, h, w)
            x = x.contiguous(memory_format=torch.channels_last)
        x = F.interpolate(x.float(), scale_factor=2.0, mode="nearest-exact").to(x.dtype)
        return self.resample[1](x.contiguous(memory_format=torch.channels_last))


class Decoder(nn.Module):
    def __init__(self, cfg: WanVAEConfig):
        super().__init__()
        dims = [cfg.dim * u for u in [cfg.dim_mult[-1]] + list(cfg.dim_mult[::-1])]
        self.conv1 = CausalConv(cfg.z_dim, dims[0])
        self.middle = nn.ModuleList([ResidualBlock(dims[0], dims[0]), AttentionBlock(dims[0]),
                                     ResidualBlock(dims[0], dims[0])])
        ups: List[nn.Module] = []
        tu = cfg.temporal_upsample
        out_dim = dims[0]
        for i, (in_dim, out_dim) in enumerate(zip(dims[:-1], dims[1:])):
            if i in (1, 2, 3):
                in_dim = in_dim // 2
            for _ in range(cfg.num_res_blocks + 1):
                ups.append(ResidualBlock(in_dim, out_dim))
                in_dim = out_dim
            if i != len(cfg.dim_mult) - 1:
                ups.append(Resample(out_dim, tu[i]))
        self.upsamples = nn.ModuleList(ups)
        self.head = nn.ModuleList([RMSNorm(out_dim, False), nn.SiLU(), CausalConv(out_dim, 3)])

    def forward(self, x, b):
        x = self.conv1(x, b)
        for m in self.middle:
            x = m(x, b)
        for m in self.upsamples:
            x = m(x, b)
        return norm_silu_conv(self.head[0], self.head[2], x, b)


class WanVAE(nn.Module):
    def __init__(self, cfg: WanVAEConfig):
        super().__init__()
        self.cfg = cfg
        self.decoder = Decoder(cfg)
        self.conv2 = CausalConv(cfg.z_dim, cfg.z_dim, 1, 0)

    def frames(self, t_latent: int) -> int:
        return 1 + self.cfg.temporal_factor * (t_latent - 1)

    @torch.no_grad()
    def decode(self, z: torch.Tensor) -> torch.Tensor:
        """Normalised latent [B, z, T, h, w] → video in [−1, 1], [B, 3, 1+4(T−1), 8h, 8w]."""
        b, c, t, h, w = z.shape
        mean = torch.tensor(self.cfg.latent_mean, device=z.device).view(1, c, 1, 1, 1)
        std = torch.tensor(self.cfg.latent_std, device=z.device).view(1, c, 1, 1, 1)
        dt = self.conv2.weight.dtype
        z = (z.float() * std + mean).to(dt)
        x = z.permute(0, 2, 1, 3, 4).reshape(b * t, c, h, w).contiguous(memory_format=torch.channels_last)
        # MIOpen "find" per convolution shape (exhaustive solver search, cached in-process and in
        # its find-db): the immediate-mode heuristic picks 256x32 igemm tiles for the 288->96
        # full-resolution convs; the searched solvers halve the decode (87 -> 43 ms, 13 frames
        # 512x320; tools/wan_vae_prof.py)
        prev = torch.backends.cudnn.benchmark
        torch.backends.cudnn.benchmark = True
        try:
            x = self.decoder(self.conv2(x, b), b)
        finally:
            torch.backends.cudnn.benchmark = prev
        n, co, hh, ww = x.shape
        return x.reshape(b, n // b, co, hh, ww).permute(0, 2, 1, 3, 4).clamp_(-1, 1)


def convert_vae_keys(sd):
    return {k: v for k, v in sd.items() if k.startswith(("decoder.", "conv2."))}


# ---------------------------------------------------------------- upstream-algorithm reference
def reference_decode(vae: WanVAE, z: torch.Tensor) -> torch.Tensor:
    """The upstream decode algorithm in fp32: one latent frame per call, causal Conv3d with a
    two-frame feature cache per convolution, the temporal upsampler's ``'Rep'`` first-chunk marker
    (zero history for time_conv at latent frame 1).  Used only by the tests."""
    P = {k: v.float() for k, v in vae.state_dict().items()}
    cfg = vae.cfg
    b, c, t, h, w = z.shape
    mean = torch.tensor(cfg.latent_mean).view(1, c, 1, 1, 1)
    std = torch.tensor(cfg.latent_std).view(1, c, 1, 1, 1)
    z = z.float() * std + mean

    def cconv(x, name, pad, cache):
        wt, bs = P[name + ".weight"], P[name + ".bias"]
        p_t = 2 * pad[0]
        if cache is not None and p_t > 0:
            x = torch.cat([cache, x], 2)
            p_t -= cache.shape[2]
        x = F.pad(x, (pad[2], pad[2], pad[1], pad[1], p_t, 0))
        return F.conv3d(x, wt, bs)

    def rms(x, name, images=False):
        g = P[name + ".gamma"]
        return F.normalize(x, dim=1) * (x.shape[1] ** 0.5) * g

    state = {"caches": [], "idx": 0}

    def cached_conv(x, name, pad):
        i = state["idx"]
        state["idx"] += 1
        if i >= len(state["caches"]):
            state["caches"].append(None)
        prev = state["caches"][i]
        cx = x[:, :, -2:].clone()
        if cx.shape[2] < 2 and prev is not None:
            cx = torch.cat([prev[:, :, -1:], cx], 2)
        out = cconv(x, name, pad, prev)
        state["caches"][i] = cx
        return out

    def resblock(x, name, cin, cout):
        hdn = F.silu(rms(x, name + ".residual.0"))
        hdn = cached_conv(hdn, name + ".residual.2", (1, 1, 1))
        hdn = F.silu(rms(hdn, name + ".residual.3"))
        hdn = cached_conv(hdn, name + ".residual.6", (1, 1, 1))
        sc = cconv(x, name + ".shortcut", (0, 0, 0), None) if cin != cout else x
        return hdn + sc

    def attn(x, name):
        bb, cc, tt, hh, ww = x.shape
        y = x.permute(0, 2, 1, 3, 4).reshape(bb * tt, cc, hh, ww)
        idn = y
        y = F.normalize(y, dim=1) * (cc ** 0.5) * P[name + ".norm.gamma"]
        qkv = F.conv2d(y, P[name + ".to_qkv.weight"], P[name + ".to_qkv.bias"])
        qkv = qkv.reshape(bb * tt, 1, cc * 3, -1).permute(0, 1, 3, 2).chunk(3, dim=-1)
        y = F.scaled_dot_product_attention(*qkv).squeeze(1).permute(0, 2, 1).reshape(bb * tt, cc, hh, ww)
        y = F.conv2d(y, P[name + ".proj.weight"], P[name + ".proj.bias"]) + idn
        return y.reshape(bb, tt, cc, hh, ww).permute(0, 2, 1, 3, 4)

    def resample(x, name, temporal, slot):
        bb, cc, tt, hh, ww = x.shape
        if temporal:
            prev = state["tcache"].get(slot)
            if prev is None:
                state["tcache"][slot] = "Rep"
            else:
                cx = x[:, :, -2:].clone()
                if cx.shape[2] < 2 and not isinstance(prev, str):
                    cx = torch.cat([prev[:, :, -1:], cx], 2)
                if cx.shape[2] < 2 and isinstance(prev, str):
                    cx = torch.cat([torch.zeros_like(cx), cx], 2)
                x = cconv(x, name + ".time_conv", (1, 0, 0), None if isinstance(prev, str) else prev)
                state["tcache"][slot] = cx
                x = x.reshape(bb, 2, cc, tt, hh, ww)
                x = torch.stack((x[:, 0], x[:, 1]), 3).reshape(bb, cc, tt * 2, hh, ww)
        tt = x.shape[2]
        y = x.permute(0, 2, 1, 3, 4).reshape(bb * tt, cc, hh, ww)
        y = F.interpolate(y, scale_factor=2.0, mode="nearest-exact")
        y = F.conv2d(y, P[name + ".resample.1.weight"], P[name + ".resample.1.bias"], padding=1)
        return y.reshape(bb, tt, cc // 2, hh * 2, ww * 2).permute(0, 2, 1, 3, 4)

    state["tcache"] = {}
    x_all = cconv(z, "conv2", (0, 0, 0), None)
    outs = []
    dec = vae.decoder
    for i in range(t):
        state["idx"] = 0
        x = cached_conv(x_all[:, :, i:i + 1], "decoder.conv1", (1, 1, 1))
        x = resblock(x, "decoder.middle.0", 1, 1)
        x = attn(x, "decoder.middle.1")
        x = resblock(x, "decoder.middle.2", 1, 1)
        for j, m in enumerate(dec.upsamples):
            name = f"decoder.upsamples.{j}"
            if isinstance(m, ResidualBlock):
                cin = m.residual[2].weight.shape[1]
                cout = m.residual[2].weight.shape[0]
                x = resblock(x, name, cin, cout)
            else:
                x = resample(x, name, m.time_conv is not None, j)
        x = F.silu(rms(x, "decoder.head.0"))
        x = cached_conv(x, "decoder.head.2", (1, 1, 1))
        outs.append(x)
    return torch.cat(outs, 2).clamp(-1, 1)

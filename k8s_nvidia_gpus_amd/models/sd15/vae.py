"""SD1.5 VAE decoder (diffusers ``AutoencoderKL`` decoder half + ``post_quant_conv``).

The reference decodes with ``enable_vae_slicing`` (one image at a time, reference
sd15-api/configmap.yaml:43) to fit a 6 GB card; a 288 GB MI355X decodes the whole batch at once.
Text-to-image only needs the decoder: the checkpoint's ``encoder.*`` / ``quant_conv.*`` tensors are
skipped by the loader.  The mid-block attention is single-head over 512 channels (head dim 512,
outside the native attention kernel's head dims: it runs through PyTorch SDPA).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .config import VAEConfig
from .nn import GroupNorm, ResnetBlock2D, Upsample2D, VAEAttention


class VAEMidBlock(nn.Module):
    def __init__(self, ch: int, cfg: VAEConfig):
        super().__init__()
        g, eps = cfg.norm_num_groups, cfg.norm_eps
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch, None, g, eps) for _ in range(2)])
        self.attentions = nn.ModuleList([VAEAttention(ch, g, eps)])

    def forward(self, x):
        x = self.resnets[0](x)
        x = self.attentions[0](x)
        return self.resnets[1](x)


class UpDecoderBlock(nn.Module):
    def __init__(self, cin: int, cout: int, cfg: VAEConfig, upsample: bool):
        super().__init__()
        g, eps = cfg.norm_num_groups, cfg.norm_eps
        n = cfg.layers_per_block + 1
        self.resnets = nn.ModuleList([ResnetBlock2D(cin if i == 0 else cout, cout, None, g, eps)
                                      for i in range(n)])
        self.upsamplers = nn.ModuleList([Upsample2D(cout)]) if upsample else None

    def forward(self, x):
        for r in self.resnets:
            x = r(x)
        if self.upsamplers is not None:
            x = self.upsamplers[0](x)
        return x


class Decoder(nn.Module):
    def __init__(self, cfg: VAEConfig):
        super().__init__()
        ch = list(reversed(cfg.block_out_channels))
        self.conv_in = nn.Conv2d(cfg.latent_channels, ch[0], 3, padding=1)
        self.mid_block = VAEMidBlock(ch[0], cfg)
        self.up_blocks = nn.ModuleList()
        prev = ch[0]
        for i, c in enumerate(ch):
            self.up_blocks.append(UpDecoderBlock(prev, c, cfg, upsample=i < len(ch) - 1))
            prev = c
        self.conv_norm_out = GroupNorm(cfg.norm_num_groups, ch[-1], eps=cfg.norm_eps)
        self.conv_out = nn.Conv2d(ch[-1], cfg.out_channels, 3, padding=1)

    def forward(self, z):
        x = self.conv_in(z)
        x = self.mid_block(x)
        for b in self.up_blocks:
            x = b(x)
        return self.conv_out(self.conv_norm_out(x, silu=True))


class AutoencoderKLDecoder(nn.Module):
    def __init__(self, cfg: VAEConfig = VAEConfig()):
        super().__init__()
        self.cfg = cfg
        self.post_quant_conv = nn.Conv2d(cfg.latent_channels, cfg.latent_channels, 1)
        self.decoder = Decoder(cfg)

    @torch.no_grad()
    def prepare(self) -> "AutoencoderKLDecoder":
        if next(self.parameters()).device.type == "cuda":
            self.to(memory_format=torch.channels_last)
        for m in self.modules():
            if isinstance(m, ResnetBlock2D):
                m.fuse_biases()
        return self

    def decode(self, latents: torch.Tensor) -> torch.Tensor:
        """Scaled latents (as the UNet produces them) → images in [-1, 1], NCHW."""
        z = latents / self.cfg.scaling_factor
        if z.device.type == "cuda":
            z = z.contiguous(memory_format=torch.channels_last)
        return self.decoder(self.post_quant_conv(z))

    forward = decode

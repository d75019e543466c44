"""Wan2.1 text-to-video configurations (DiT, umT5 text encoder, causal 3-D VAE).

The reference drives Wan2.1 through an external ComfyUI server with three model files
(reference cluster-config/apps/llm/scripts/generate_wan_t2v.py:347-349):
``wan2.1_t2v_1.3B_bf16.safetensors`` (the DiT), ``umt5_xxl_fp16.safetensors`` (the text encoder)
and ``wan_2.1_vae.safetensors``; its job defaults are 512×320, 16 frames, 25 steps, CFG 6,
``uni_pc`` / ``simple`` (generate_wan_t2v.py:305-312).  These dataclasses hold the published
architecture hyper-parameters of those files; ``tiny()`` variants keep every structural feature
(GQA-free multi-head attention, 3-D RoPE split, per-layer relative bias, temporal upsampling) at a
size the CPU tests can run.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Tuple


@dataclass(frozen=True)
class WanDiTConfig:
    dim: int = 1536
    ffn_dim: int = 8960
    freq_dim: int = 256
    heads: int = 12
    layers: int = 30
    in_dim: int = 16
    out_dim: int = 16
    text_dim: int = 4096
    text_len: int = 512
    patch: Tuple[int, int, int] = (1, 2, 2)
    eps: float = 1e-6
    rope_theta: float = 10000.0
    rope_max_len: int = 1024

    @property
    def head_dim(self) -> int:
        return self.dim // self.heads

    @staticmethod
    def wan21_t2v_1_3b() -> "WanDiTConfig":
        return WanDiTConfig()

    @staticmethod
    def wan21_t2v_14b() -> "WanDiTConfig":
        return WanDiTConfig(dim=5120, ffn_dim=13824, heads=40, layers=40)

    @staticmethod
    def tiny() -> "WanDiTConfig":
        # head dim 128 and the 512-token context as in every published Wan2.1 checkpoint (the
        # loader infers heads = dim / 128 and the context length is not stored in the file)
        return WanDiTConfig(dim=256, ffn_dim=512, freq_dim=32, heads=2, layers=2, text_dim=64)


@dataclass(frozen=True)
class UMT5Config:
    vocab: int = 256384
    dim: int = 4096
    ffn_dim: int = 10240
    heads: int = 64
    head_dim: int = 64
    layers: int = 24
    buckets: int = 32
    max_distance: int = 128
    eps: float = 1e-6
    shared_pos: bool = False        # umT5: every layer owns its relative-position bias

    @staticmethod
    def umt5_xxl() -> "UMT5Config":
        return UMT5Config()

    @staticmethod
    def tiny(vocab: int = 512) -> "UMT5Config":
        return UMT5Config(vocab=vocab, dim=64, ffn_dim=128, heads=4, head_dim=16, layers=2,
                          buckets=8)


# Per-channel latent statistics of the Wan2.1 VAE (normalised latent = (z - mean) / std).
WAN21_LATENT_MEAN = (-0.7571, -0.7089, -0.9113, 0.1075, -0.1745, 0.9653, -0.1517, 1.5508,
                     0.4134, -0.0715, 0.5517, -0.3632, -0.1922, -0.9497, 0.2503, -0.2921)
WAN21_LATENT_STD = (2.8184, 1.4541, 2.3275, 2.6558, 1.2196, 1.7708, 2.6052, 2.0743,
                    3.2687, 2.1526, 2.8652, 1.5579, 1.6382, 1.1253, 2.8251, 1.9160)


@dataclass(frozen=True)
class WanVAEConfig:
    z_dim: int = 16
    dim: int = 96
    dim_mult: Tuple[int, ...] = (1, 2, 4, 4)
    num_res_blocks: int = 2
    temporal_downsample: Tuple[bool, ...] = (False, True, True)
    latent_mean: Tuple[float, ...] = WAN21_LATENT_MEAN
    latent_std: Tuple[float, ...] = WAN21_LATENT_STD

    @property
    def temporal_upsample(self) -> Tuple[bool, ...]:
        return tuple(reversed(self.temporal_downsample))

    @property
    def spatial_factor(self) -> int:
        return 2 ** (len(self.dim_mult) - 1)

    @property
    def temporal_factor(self) -> int:
        return 2 ** sum(self.temporal_downsample)

    @staticmethod
    def wan21() -> "WanVAEConfig":
        return WanVAEConfig()

    @staticmethod
    def tiny() -> "WanVAEConfig":
        return WanVAEConfig(dim=8)


def latent_frames(frames: int, temporal_factor: int = 4) -> int:
    """Latent length of a ``frames``-frame video: the first frame alone, then one latent frame per
    ``temporal_factor`` frames (ComfyUI's EmptyHunyuanLatentVideo: ``(length - 1) // 4 + 1``)."""
    return (max(1, frames) - 1) // temporal_factor + 1


@dataclass
class WanJobDefaults:
    """The reference client's defaults (generate_wan_t2v.py:305-312)."""
    width: int = 512
    height: int = 320
    frames: int = 16
    steps: int = 25
    cfg: float = 6.0
    sampler: str = "uni_pc"
    scheduler: str = "simple"
    shift: float = 8.0
    extra: List[str] = field(default_factory=list)

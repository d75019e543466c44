"""Architecture configs of the Stable Diffusion 1.5 model family (UNet, VAE decoder, CLIP text encoder).

The reference serves SD1.5 through ``diffusers.StableDiffusionPipeline.from_pretrained(MODEL_ID)``
inside a pulled CUDA image (reference cluster-config/apps/sd15-api/configmap.yaml:41-47,
deployment.yaml:21).  Here the model family is implemented in-tree (``unet.py``, ``vae.py``,
``clip.py``) so it runs on MI355X with this repository's HIP kernels and HIP-graph capture, and loads
the same checkpoint files (diffusers directory layout, safetensors; ``weights.py``).

``SD15`` holds the published SD1.5 hyper-parameters (runwayml/stable-diffusion-v1-5 ``config.json``
files); ``tiny()`` returns a structurally identical miniature used by the CPU tests.
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Tuple


@dataclass(frozen=True)
class UNetConfig:
    in_channels: int = 4
    out_channels: int = 4
    block_out_channels: Tuple[int, ...] = (320, 640, 1280, 1280)
    # True = CrossAttn{Down,Up}Block2D (ResNets + Transformer2D), False = plain {Down,Up}Block2D
    down_attention: Tuple[bool, ...] = (True, True, True, False)
    layers_per_block: int = 2
    num_heads: int = 8                 # diffusers' SD1.5 "attention_head_dim": 8 is the HEAD COUNT
    cross_attention_dim: int = 768
    norm_num_groups: int = 32
    norm_eps: float = 1e-5
    transformer_norm_eps: float = 1e-6  # Transformer2DModel.norm (GroupNorm) eps
    flip_sin_to_cos: bool = True
    freq_shift: float = 0.0

    @property
    def time_embed_dim(self) -> int:
        return self.block_out_channels[0] * 4


@dataclass(frozen=True)
class VAEConfig:
    latent_channels: int = 4
    out_channels: int = 3
    block_out_channels: Tuple[int, ...] = (128, 256, 512, 512)
    layers_per_block: int = 2
    norm_num_groups: int = 32
    norm_eps: float = 1e-6
    scaling_factor: float = 0.18215


@dataclass(frozen=True)
class CLIPTextConfig:
    vocab_size: int = 49408
    hidden_size: int = 768
    intermediate_size: int = 3072
    num_layers: int = 12
    num_heads: int = 12
    max_position_embeddings: int = 77
    layer_norm_eps: float = 1e-5
    bos_token_id: int = 49406
    eos_token_id: int = 49407


@dataclass(frozen=True)
class SchedulerConfig:
    num_train_timesteps: int = 1000
    beta_start: float = 0.00085
    beta_end: float = 0.012
    beta_schedule: str = "scaled_linear"
    steps_offset: int = 1
    set_alpha_to_one: bool = False


@dataclass(frozen=True)
class SD15Config:
    unet: UNetConfig = field(default_factory=UNetConfig)
    vae: VAEConfig = field(default_factory=VAEConfig)
    text: CLIPTextConfig = field(default_factory=CLIPTextConfig)
    scheduler: SchedulerConfig = field(default_factory=SchedulerConfig)
    vae_scale: int = 8                 # pixel / latent side ratio (2 ** (len(vae blocks) - 1))


SD15 = SD15Config()


def tiny() -> SD15Config:
    """Same topology as SD1.5 (every block type, skip wiring, attention kinds), tiny widths."""
    return SD15Config(
        unet=UNetConfig(block_out_channels=(32, 64, 64, 64), num_heads=2, cross_attention_dim=32,
                        norm_num_groups=8),
        vae=VAEConfig(block_out_channels=(16, 32, 32, 32), norm_num_groups=4),
        text=replace(CLIPTextConfig(), vocab_size=1000, hidden_size=32, intermediate_size=64,
                     num_layers=2, num_heads=2, bos_token_id=998, eos_token_id=999),
    )

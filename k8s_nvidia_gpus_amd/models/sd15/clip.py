"""CLIP ViT-L/14 text encoder (SD1.5's ``text_encoder``), parameter names of transformers'
``CLIPTextModel`` (``text_model.encoder.layers.{i}.self_attn.q_proj`` …).

Runs once per request on 77 tokens (negligible next to 30 UNet passes), so it is plain PyTorch:
causal self-attention through SDPA, quick-GELU MLP, final LayerNorm; the last hidden state is the
UNet's cross-attention context (reference: diffusers ``StableDiffusionPipeline._encode_prompt``).
The CPU tests check it bit-for-bit against ``transformers.CLIPTextModel`` with the same weights.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .config import CLIPTextConfig


class CLIPAttention(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        d = cfg.hidden_size
        self.heads = cfg.num_heads
        self.q_proj = nn.Linear(d, d)
        self.k_proj = nn.Linear(d, d)
        self.v_proj = nn.Linear(d, d)
        self.out_proj = nn.Linear(d, d)

    def forward(self, x):
        n, l, d = x.shape
        h = self.heads

        def split(t):
            return t.reshape(n, l, h, d // h).transpose(1, 2)

        o = F.scaled_dot_product_attention(split(self.q_proj(x)), split(self.k_proj(x)),
                                           split(self.v_proj(x)), is_causal=True)
        return self.out_proj(o.transpose(1, 2).reshape(n, l, d))


class CLIPMLP(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.fc1 = nn.Linear(cfg.hidden_size, cfg.intermediate_size)
        self.fc2 = nn.Linear(cfg.intermediate_size, cfg.hidden_size)

    def forward(self, x):
        x = self.fc1(x)
        return self.fc2(x * torch.sigmoid(1.702 * x))   # quick_gelu


class CLIPEncoderLayer(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.self_attn = CLIPAttention(cfg)
        self.layer_norm1 = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)
        self.mlp = CLIPMLP(cfg)
        self.layer_norm2 = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)

    def forward(self, x):
        x = x + self.self_attn(self.layer_norm1(x))
        return x + self.mlp(self.layer_norm2(x))


class _Embeddings(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.token_embedding = nn.Embedding(cfg.vocab_size, cfg.hidden_size)
        self.position_embedding = nn.Embedding(cfg.max_position_embeddings, cfg.hidden_size)
        self.register_buffer("position_ids", torch.arange(cfg.max_position_embeddings)[None],
                             persistent=False)

    def forward(self, ids):
        return self.token_embedding(ids) + self.position_embedding(self.position_ids[:, :ids.shape[1]])


class _Encoder(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.layers = nn.ModuleList([CLIPEncoderLayer(cfg) for _ in range(cfg.num_layers)])

    def forward(self, x):
        for layer in self.layers:
            x = layer(x)
        return x


class _TextTransformer(nn.Module):
    def __init__(self, cfg: CLIPTextConfig):
        super().__init__()
        self.embeddings = _Embeddings(cfg)
        self.encoder = _Encoder(cfg)
        self.final_layer_norm = nn.LayerNorm(cfg.hidden_size, eps=cfg.layer_norm_eps)

    def forward(self, ids):
        return self.final_layer_norm(self.encoder(self.embeddings(ids)))


class CLIPTextModel(nn.Module):
    def __init__(self, cfg: CLIPTextConfig = CLIPTextConfig()):
        super().__init__()
        self.cfg = cfg
        self.text_model = _TextTransformer(cfg)

    def forward(self, input_ids: torch.Tensor) -> torch.Tensor:
        """``input_ids`` [N, 77] → last hidden state [N, 77, hidden]."""
        return self.text_model(input_ids)

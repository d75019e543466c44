"""umT5 text encoder (Wan2.1's ``umt5_xxl``) and its SentencePiece tokenizer.

Reference workload: ``CLIPLoader(clip_name=umt5_xxl_fp16.safetensors, type=wan)`` +
``CLIPTextEncode`` in the reference's ComfyUI graph (generate_wan_t2v.py:14-139, 348).  Parameter
names are the Hugging Face T5 encoder's (``encoder.block.N.layer.0.SelfAttention.{q,k,v,o}``,
``…relative_attention_bias``, ``…layer.1.DenseReluDense.{wi_0,wi_1,wo}``,
``encoder.final_layer_norm``, ``shared``) — the layout of that file.

umT5 differs from T5 in one structural point: EVERY layer owns its relative-position bias table
(``UMT5Config.shared_pos = False``).  Encoding is a one-off per prompt (tens of tokens through a
5.7 B-parameter stack — bandwidth-bound on the 11 GB of weights), so it runs as plain bf16 GEMMs
with PyTorch's SDPA carrying the additive position bias; prompts are encoded at their true length
(no padding, no mask) and the DiT pads the states with zero rows to its 512-token context.
"""
from __future__ import annotations

import html
import math
import os
import re
from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .config import UMT5Config


def relative_bucket(rel: torch.Tensor, buckets: int, max_distance: int) -> torch.Tensor:
    """T5's bidirectional log-bucketing of ``key_pos − query_pos``."""
    half = buckets // 2
    out = (rel > 0).long() * half
    n = rel.abs()
    exact = half // 2
    large = exact + (torch.log(n.float().clamp(min=1) / exact) / math.log(max_distance / exact)
                     * (half - exact)).long()
    large = large.clamp(max=half - 1)
    return out + torch.where(n < exact, n, large)


class T5Norm(nn.Module):
    def __init__(self, dim: int, eps: float):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(dim))
        self.eps = eps

    def forward(self, x):
        xf = x.float()
        xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)
        return (xf * self.weight.float()).to(self.weight.dtype)


class SelfAttention(nn.Module):
    def __init__(self, cfg: UMT5Config, has_bias: bool):
        super().__init__()
        inner = cfg.heads * cfg.head_dim
        self.q = nn.Linear(cfg.dim, inner, bias=False)
        self.k = nn.Linear(cfg.dim, inner, bias=False)
        self.v = nn.Linear(cfg.dim, inner, bias=False)
        self.o = nn.Linear(inner, cfg.dim, bias=False)
        if has_bias:
            self.relative_attention_bias = nn.Embedding(cfg.buckets, cfg.heads)


class AttnLayer(nn.Module):
    def __init__(self, cfg: UMT5Config, has_bias: bool):
        super().__init__()
        self.SelfAttention = SelfAttention(cfg, has_bias)
        self.layer_norm = T5Norm(cfg.dim, cfg.eps)


class DenseGatedGelu(nn.Module):
    def __init__(self, cfg: UMT5Config):
        super().__init__()
        self.wi_0 = nn.Linear(cfg.dim, cfg.ffn_dim, bias=False)
        self.wi_1 = nn.Linear(cfg.dim, cfg.ffn_dim, bias=False)
        self.wo = nn.Linear(cfg.ffn_dim, cfg.dim, bias=False)


class FFLayer(nn.Module):
    def __init__(self, cfg: UMT5Config):
        super().__init__()
        self.DenseReluDense = DenseGatedGelu(cfg)
        self.layer_norm = T5Norm(cfg.dim, cfg.eps)


class T5Block(nn.Module):
    def __init__(self, cfg: UMT5Config, has_bias: bool):
        super().__init__()
        self.layer = nn.ModuleList([AttnLayer(cfg, has_bias), FFLayer(cfg)])


class Encoder(nn.Module):
    def __init__(self, cfg: UMT5Config):
        super().__init__()
        self.block = nn.ModuleList([T5Block(cfg, cfg.shared_pos is False or i == 0)
                                    for i in range(cfg.layers)])
        self.final_layer_norm = T5Norm(cfg.dim, cfg.eps)


class UMT5Encoder(nn.Module):
    def __init__(self, cfg: UMT5Config):
        super().__init__()
        self.cfg = cfg
        self.shared = nn.Embedding(cfg.vocab, cfg.dim)
        self.encoder = Encoder(cfg)

    def position_bias(self, table: nn.Embedding, n: int) -> torch.Tensor:
        pos = torch.arange(n, device=table.weight.device)
        b = relative_bucket(pos[None, :] - pos[:, None], self.cfg.buckets, self.cfg.max_distance)
        return table(b).permute(2, 0, 1)[None].float()          # [1, H, n, n]

    @torch.no_grad()
    def forward(self, ids: torch.Tensor) -> torch.Tensor:
        """ids [B, n] (all real tokens, no padding) → last hidden states [B, n, dim]."""
        cfg = self.cfg
        x = self.shared(ids)
        b, n, _ = x.shape
        bias = None
        for blk in self.encoder.block:
            att, ff = blk.layer
            sa = att.SelfAttention
            if hasattr(sa, "relative_attention_bias"):
                bias = self.position_bias(sa.relative_attention_bias, n)
            h = att.layer_norm(x)
            q, k, v = (lin(h).view(b, n, cfg.heads, cfg.head_dim).transpose(1, 2)
                       for lin in (sa.q, sa.k, sa.v))
            o = F.scaled_dot_product_attention(q.float(), k.float(), v.float(), attn_mask=bias,
                                               scale=1.0)
            x = x + sa.o(o.transpose(1, 2).reshape(b, n, -1).to(x.dtype))
            h = ff.layer_norm(x)
            d = ff.DenseReluDense
            g = F.gelu(d.wi_0(h).float(), approximate="tanh") * d.wi_1(h).float()
            x = x + d.wo(g.to(x.dtype))
        return self.encoder.final_layer_norm(x)


def convert_t5_keys(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Accept the HF layout with or without ``shared``/``encoder.embed_tokens`` duplication and
    drop decoder / lm-head tensors (encoder-only use)."""
    out = {}
    for k, v in sd.items():
        if k.startswith(("decoder.", "lm_head.")):
            continue
        if k == "encoder.embed_tokens.weight":
            out.setdefault("shared.weight", v)
            continue
        out[k] = v
    return out


# ---------------------------------------------------------------- tokenizer
_WS = re.compile(r"\s+")


def clean_prompt(text: str) -> str:
    """Wan's prompt cleaning ('whitespace' mode): HTML-unescape, collapse whitespace."""
    return _WS.sub(" ", html.unescape(html.unescape(text))).strip()


class UMT5Tokenizer:
    """SentencePiece (``spiece.model``) or ``tokenizer.json`` tokenizer with T5 conventions:
    ``</s>`` (id 1) appended, pad id 0, at most ``max_len`` ids."""

    EOS = 1
    PAD = 0

    def __init__(self, path: str, max_len: int = 512):
        self.max_len = max_len
        self._sp = self._hf = None
        if path.endswith(".json"):
            from tokenizers import Tokenizer

            self._hf = Tokenizer.from_file(path)
        else:
            import sentencepiece as spm

            self._sp = spm.SentencePieceProcessor(model_file=path)

    @classmethod
    def from_proto(cls, blob: bytes, max_len: int = 512) -> "UMT5Tokenizer":
        """SentencePiece model embedded in the text-encoder file (a ``spiece_model`` uint8
        tensor, as some single-file umT5 exports carry it)."""
        import sentencepiece as spm

        tok = cls.__new__(cls)
        tok.max_len = max_len
        tok._hf = None
        tok._sp = spm.SentencePieceProcessor(model_proto=blob)
        return tok

    @staticmethod
    def find(model_dir: str) -> Optional[str]:
        for name in ("tokenizer.json", "spiece.model", "umt5/tokenizer.json", "umt5/spiece.model",
                     "text_encoders/umt5-xxl/tokenizer.json", "text_encoders/umt5-xxl/spiece.model"):
            p = os.path.join(model_dir, name)
            if os.path.exists(p):
                return p
        return None

    def encode(self, text: str) -> List[int]:
        text = clean_prompt(text)
        if self._sp is not None:
            ids = list(self._sp.encode(text))
        else:
            ids = list(self._hf.encode(text, add_special_tokens=False).ids)
        ids = ids[: self.max_len - 1]
        return ids + [self.EOS]

"""Qwen2-family decoder configuration (the architecture of the reference's served model).

The reference serves Qwen2.5-7B-Instruct (abliterated) as a Q4_K_M GGUF with ``--ctx-size 4096``
and all layers on the GPU (reference cluster-config/apps/llm/deployment.yaml:31-34,64-72,76-84).
``QWEN25_7B`` is that architecture; ``from_gguf`` reads the same hyper-parameters from a file's
``qwen2.*`` metadata the way llama.cpp does, so any Qwen2-architecture GGUF loads.
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Any, Dict


@dataclass(frozen=True)
class LLMConfig:
    vocab: int = 152064
    dim: int = 3584
    layers: int = 28
    heads: int = 28
    kv_heads: int = 4
    ffn: int = 18944
    ctx: int = 32768            # trained context (qwen2.context_length)
    rope_theta: float = 1.0e6
    eps: float = 1e-6
    qkv_bias: bool = True
    tied_embeddings: bool = False
    name: str = "qwen2.5-7b"

    @property
    def head_dim(self) -> int:
        return self.dim // self.heads

    @property
    def group(self) -> int:
        return self.heads // self.kv_heads

    @property
    def kv_dim(self) -> int:
        return self.kv_heads * self.head_dim

    def params(self) -> int:
        d, f, kv = self.dim, self.ffn, self.kv_dim
        per_layer = d * d + 2 * d * kv + d * d + 3 * d * f + 2 * d + (d + 2 * kv if self.qkv_bias else 0)
        emb = self.vocab * d * (1 if self.tied_embeddings else 2)
        return self.layers * per_layer + emb + d


QWEN25_7B = LLMConfig()


def tiny(**kw) -> LLMConfig:
    """Miniature Qwen2-shaped model for CPU/GPU tests (all dims multiples of 256 where the
    K-quant formats need it)."""
    base = LLMConfig(vocab=512, dim=256, layers=2, heads=2, kv_heads=1, ffn=512, ctx=512,
                     rope_theta=1.0e4, name="tiny-qwen2")
    return replace(base, **kw)


def from_gguf(meta: Dict[str, Any]) -> LLMConfig:
    arch = meta.get("general.architecture", "qwen2")
    if arch != "qwen2":
        # e.g. llama: GGML_ROPE_TYPE_NORM (adjacent-pair rotation over permuted Q/K) and no QKV
        # bias — loading it through the Qwen2 (NeoX-rope, biased) kernels would run silently wrong
        raise ValueError(f"unsupported architecture {arch!r}: this engine implements the Qwen2 "
                         f"decoder (NeoX RoPE, QKV bias) of the reference's Qwen2.5 model only")

    def g(key, default=None):
        v = meta.get(f"{arch}.{key}", default)
        if v is None:
            raise ValueError(f"GGUF metadata lacks {arch}.{key}")
        return v

    heads = int(g("attention.head_count"))
    vocab = meta.get(f"{arch}.vocab_size")
    if vocab is None:
        toks = meta.get("tokenizer.ggml.tokens")
        vocab = len(toks) if toks is not None else None
    if vocab is None:
        raise ValueError("GGUF metadata lacks a vocabulary size")
    return LLMConfig(
        vocab=int(vocab), dim=int(g("embedding_length")), layers=int(g("block_count")),
        heads=heads, kv_heads=int(g("attention.head_count_kv", heads)),
        ffn=int(g("feed_forward_length")), ctx=int(g("context_length", 4096)),
        rope_theta=float(g("rope.freq_base", 10000.0)),
        eps=float(g("attention.layer_norm_rms_epsilon", 1e-6)),
        qkv_bias=True, name=str(meta.get("general.name", arch)))


def to_gguf_metadata(cfg: LLMConfig) -> Dict[str, Any]:
    a = "qwen2"
    return {
        "general.architecture": a, "general.name": cfg.name,
        f"{a}.block_count": cfg.layers, f"{a}.context_length": cfg.ctx,
        f"{a}.embedding_length": cfg.dim, f"{a}.feed_forward_length": cfg.ffn,
        f"{a}.attention.head_count": cfg.heads, f"{a}.attention.head_count_kv": cfg.kv_heads,
        f"{a}.rope.freq_base": float(cfg.rope_theta),
        f"{a}.attention.layer_norm_rms_epsilon": float(cfg.eps),
    }


def use_more_bits(i: int, n: int) -> bool:
    """Layers that a Q4_K_M file stores at Q6_K for attn_v / ffn_down (first and last eighth, and
    every third layer in between) — the mixed-precision recipe of the Q4_K_M file type."""
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2

"""Synthetic Qwen2 GGUF files (random weights, exact layout) for tests and offline runs.

There is no network here for the reference's checkpoint (reference
cluster-config/apps/llm/deployment.yaml:31-34 downloads it from Hugging Face at pod start), so the
engine's load path is exercised on files this module writes: llama.cpp's qwen2 tensor names, the
Q4_K_M type mix (``config.use_more_bits``), F32 norms/biases, and a byte-level BPE vocabulary in the
``tokenizer.ggml.*`` metadata.  Weights are Gaussian, quantised with ``quants.py``.
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import numpy as np

from . import gguf, quants
from .config import LLMConfig, to_gguf_metadata, use_more_bits
from .tokenizer import synthetic_vocab


def write_synthetic_gguf(path: str, cfg: LLMConfig, seed: int = 0,
                         tied: bool = False, f16_output: bool = False,
                         extra_metadata: Optional[Dict[str, Any]] = None) -> str:
    """``extra_metadata`` overrides / adds GGUF keys (e.g. another ``tokenizer.chat_template``)."""
    rng = np.random.default_rng(seed)
    md = to_gguf_metadata(cfg)
    md.update(synthetic_vocab(cfg.vocab))
    md.update(extra_metadata or {})
    md["general.file_type"] = 15          # LLAMA_FTYPE_MOSTLY_Q4_K_M
    tensors = []
    Q4, Q6 = gguf.Q4_K, gguf.Q6_K

    def mat(name, n, k, t, scale=None):
        w = rng.standard_normal((n, k)).astype(np.float32) * (scale or 1.0 / np.sqrt(k))
        if t == gguf.F16:
            tensors.append((name, (k, n), t, w.astype(np.float16)))
        else:
            tensors.append((name, (k, n), t, quants.quantize(w, t)))

    def vec(name, n, base=1.0, spread=0.1):
        v = (base + spread * rng.standard_normal(n)).astype(np.float32)
        tensors.append((name, (n,), gguf.F32, v))

    d, kv, f = cfg.dim, cfg.kv_dim, cfg.ffn
    mat("token_embd.weight", cfg.vocab, d, Q4, scale=1.0)
    for i in range(cfg.layers):
        p = f"blk.{i}."
        more = use_more_bits(i, cfg.layers)
        vec(p + "attn_norm.weight", d)
        mat(p + "attn_q.weight", d, d, Q4)
        mat(p + "attn_k.weight", kv, d, Q4)
        mat(p + "attn_v.weight", kv, d, Q6 if more else Q4)
        if cfg.qkv_bias:
            vec(p + "attn_q.bias", d, 0.0)
            vec(p + "attn_k.bias", kv, 0.0)
            vec(p + "attn_v.bias", kv, 0.0)
        mat(p + "attn_output.weight", d, d, Q4)
        vec(p + "ffn_norm.weight", d)
        mat(p + "ffn_gate.weight", f, d, Q4)
        mat(p + "ffn_up.weight", f, d, Q4)
        mat(p + "ffn_down.weight", d, f, Q6 if more else Q4)
    vec("output_norm.weight", d)
    if not tied:
        mat("output.weight", cfg.vocab, d, gguf.F16 if f16_output else Q6)
    gguf.write_gguf(path, md, tensors)
    return path


def load(path: str, device="cuda", max_ctx: int = 4096, slots: int = 4,
         dense: Optional[bool] = None):
    """GGUF file → (Engine, Tokenizer)."""
    from .engine import Engine
    from .tokenizer import Tokenizer
    from .weights import ModelWeights

    with gguf.GGUFFile(path) as g:
        tok = Tokenizer.from_gguf(g.metadata)      # refuses unknown pre-tokenisers / bad templates
        w = ModelWeights.from_gguf(g, device=device)
    return Engine(w, max_ctx=max_ctx, slots=slots, dense=dense), tok

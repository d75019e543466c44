"""Model weights of the Qwen2 engine: quantised matrices kept in their K-quant form on the GPU.

Decoding streams every weight once per token, so the engine keeps the file's 4/6-bit blocks in HBM
(~4.4 GB for Qwen2.5-7B Q4_K_M) and reads them with the GEMV kernels; with 288 GB per MI355X it
can also keep an fp16 copy for compute-bound prompt processing (``dense=True``, +15 GB).

* ``QWeight`` — one [N, K] matrix repacked on the GPU into aligned planes (Q4_K: nibbles + the
  6-bit scales/mins decoded to bytes + d/dmin; Q6_K: ql / qh / lane-ordered scales / d) — the
  file's information, 148 instead of 144 bytes per Q4_K block.  On the CPU (tests, no GPU)
  it holds the raw GGUF rows and dequantises with the numpy codecs.
* ``ModelWeights.from_gguf`` — tensor names of llama.cpp's qwen2 GGUF layout
  (``token_embd``, ``blk.N.attn_q`` …, ``output``); matrices of other types (F16/F32/Q8_0) are
  re-encoded to Q6_K at load.
* ``ModelWeights.random`` — random K-quant blocks of the exact architecture built directly on the
  device (no network for the real checkpoint: the benchmark streams the same bytes per token).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from . import gguf, quants
from .config import LLMConfig, from_gguf, use_more_bits

_QTYPE = {gguf.Q4_K: 0, gguf.Q6_K: 1}


class QWeight:
    """A quantised [N, K] matrix (``qtype`` 0 = Q4_K, 1 = Q6_K)."""

    def __init__(self, qtype: int, n: int, k: int, q: torch.Tensor, qh=None, sc=None, d=None,
                 raw: Optional[np.ndarray] = None):
        self.qtype, self.n, self.k = qtype, n, k
        self.q, self.qh, self.sc, self.d = q, qh, sc, d
        self.raw = raw          # CPU only: GGUF rows for the numpy decoder
        self.mfma = None        # on the GPU: MFMA-packed planes (mq, mqh, msc, md), see mfma_pack

    def mfma_pack(self) -> bool:
        """Add the MFMA-packed copy of the planes (the int8 matrix-core GEMV reads it); False
        when the matrix does not qualify (CPU, N % 16)."""
        if self.q.device.type != "cuda" or self.n % 16:
            return False
        if self.mfma is None:
            from k8s_nvidia_gpus_amd.ops import llm_kernels as LK

            self.mfma = LK.mfma_pack(self)
        return True

    def mfma_ptrs(self):
        return tuple(None if t is None else t.data_ptr() for t in self.mfma)

    @property
    def ggml_type(self) -> int:
        return gguf.Q4_K if self.qtype == 0 else gguf.Q6_K

    @property
    def device(self) -> torch.device:
        return self.q.device

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.q, self.qh, self.sc, self.d)
                   if t is not None)

    def ptrs(self):
        return tuple(None if t is None else t.data_ptr() for t in (self.q, self.qh, self.sc, self.d))

    @classmethod
    def from_raw(cls, raw: np.ndarray, ggml_type: int, device) -> "QWeight":
        """``raw``: uint8 [N, nb*block_bytes] GGUF rows."""
        per, size = gguf.BLOCK[ggml_type]
        n = raw.shape[0]
        k = raw.shape[1] // size * per
        dev = torch.device(device)
        if dev.type != "cuda":
            own = np.array(raw, dtype=np.uint8, copy=True)   # detach from the file mapping
            return cls(_QTYPE[ggml_type], n, k, torch.from_numpy(own), raw=own)
        t = torch.from_numpy(np.array(raw, dtype=np.uint8, copy=True)).to(dev)
        return cls.from_device_raw(t, ggml_type)

    @classmethod
    def from_device_raw(cls, t: torch.Tensor, ggml_type: int) -> "QWeight":
        per, size = gguf.BLOCK[ggml_type]
        n = t.shape[0]
        k = t.shape[1] // size * per
        from k8s_nvidia_gpus_amd.ops import llm_kernels as LK

        nb = k // 256
        if ggml_type == gguf.Q4_K:
            qs = torch.empty((n, nb * 128), dtype=torch.uint8, device=t.device)
            scm = torch.empty((n, nb * 16), dtype=torch.int8, device=t.device)
            dm = torch.empty((n, nb), dtype=torch.int32, device=t.device)
            LK.q4k_repack(t.contiguous(), qs, scm, dm)
            return cls(0, n, k, qs, sc=scm, d=dm)
        ql = torch.empty((n, nb * 128), dtype=torch.uint8, device=t.device)
        qh = torch.empty((n, nb * 64), dtype=torch.uint8, device=t.device)
        sc = torch.empty((n, nb * 16), dtype=torch.int8, device=t.device)
        d = torch.empty((n, nb), dtype=torch.int16, device=t.device)
        LK.q6k_repack(t.contiguous(), ql, qh, sc, d)
        return cls(1, n, k, ql, qh, sc, d)

    def dequant(self, dtype=torch.float32, rows: Optional[torch.Tensor] = None) -> torch.Tensor:
        if self.q.device.type == "cuda":
            from k8s_nvidia_gpus_amd.ops import llm_kernels as LK

            n = self.n if rows is None else rows.numel()
            out = torch.empty((n, self.k), dtype=dtype if dtype in (torch.float16, torch.float32)
                              else torch.float32, device=self.q.device)
            LK.dequant(self, out, None if rows is None else rows.to(torch.int32).contiguous())
            return out.to(dtype)
        raw = self.raw if rows is None else self.raw[rows.cpu().numpy()]
        return torch.from_numpy(quants.dequantize(raw, self.ggml_type)).to(dtype)

    @staticmethod
    def cat(parts: List["QWeight"]) -> "QWeight":
        """Row-concatenate matrices of one type (fused q/k/v projection)."""
        t = parts[0].qtype
        if any(p.qtype != t or p.k != parts[0].k for p in parts):
            raise ValueError("cat: matrices must share type and K")
        n = sum(p.n for p in parts)

        def c(attr):
            xs = [getattr(p, attr) for p in parts]
            return None if xs[0] is None else torch.cat(xs, 0).contiguous()

        raw = None if parts[0].raw is None else np.concatenate([p.raw for p in parts], 0)
        return QWeight(t, n, parts[0].k, c("q"), c("qh"), c("sc"), c("d"), raw=raw)


@dataclass
class LayerWeights:
    attn_norm: torch.Tensor
    wq: QWeight
    wk: QWeight
    wv: QWeight
    bq: Optional[torch.Tensor]
    bk: Optional[torch.Tensor]
    bv: Optional[torch.Tensor]
    wo: QWeight
    ffn_norm: torch.Tensor
    wg: QWeight
    wu: QWeight
    wd: QWeight
    # built by ModelWeights.finalize
    wqkv: List[QWeight] = field(default_factory=list)   # 1 (same type) or 2 ([q;k], v) matrices
    bqkv: Optional[torch.Tensor] = None


@dataclass
class ModelWeights:
    cfg: LLMConfig
    tok_embd: QWeight
    out_norm: torch.Tensor
    output: QWeight
    layers: List[LayerWeights]
    meta: Dict = field(default_factory=dict)

    def finalize(self) -> "ModelWeights":
        for L in self.layers:
            if L.wq.qtype == L.wk.qtype == L.wv.qtype:
                L.wqkv = [QWeight.cat([L.wq, L.wk, L.wv])]
            else:
                L.wqkv = [QWeight.cat([L.wq, L.wk]), L.wv]
            if L.bq is not None:
                L.bqkv = torch.cat([L.bq, L.bk, L.bv]).contiguous()
            else:
                L.bqkv = torch.zeros(self.cfg.dim + 2 * self.cfg.kv_dim, device=L.attn_norm.device)
            # the fused copies replace the separate q/k/v matrices (no double residency)
            L.wq = L.wk = L.wv = None  # type: ignore[assignment]
        return self

    def nbytes(self) -> int:
        n = self.tok_embd.nbytes() + self.output.nbytes()
        for L in self.layers:
            for w in L.wqkv + [L.wo, L.wg, L.wu, L.wd]:
                n += w.nbytes()
        return n

    # ------------------------------------------------------------------ GGUF
    @classmethod
    def from_gguf(cls, g: gguf.GGUFFile, device="cuda") -> "ModelWeights":
        cfg = from_gguf(g.metadata)
        dev = torch.device(device)

        def vec(name):
            return torch.from_numpy(np.array(g.tensor(name), np.float32)).to(dev)

        def opt_vec(name):
            return vec(name) if name in g.tensors else None

        def mat(name):
            ti = g.tensors[name]
            if ti.ggml_type in _QTYPE:
                raw = g.raw(name)
            else:   # F16 / F32 / Q8_0 …: re-encode at 6 bits
                w = quants.dequantize(g.tensor(name) if ti.ggml_type in (gguf.F32, gguf.F16, gguf.BF16)
                                      else g.raw(name), ti.ggml_type)
                raw = quants.quant_q6_k(w.reshape(ti.rows, -1))
                return QWeight.from_raw(raw, gguf.Q6_K, dev)
            return QWeight.from_raw(raw, ti.ggml_type, dev)

        layers = []
        for i in range(cfg.layers):
            p = f"blk.{i}."
            layers.append(LayerWeights(
                attn_norm=vec(p + "attn_norm.weight"), wq=mat(p + "attn_q.weight"),
                wk=mat(p + "attn_k.weight"), wv=mat(p + "attn_v.weight"),
                bq=opt_vec(p + "attn_q.bias"), bk=opt_vec(p + "attn_k.bias"),
                bv=opt_vec(p + "attn_v.bias"), wo=mat(p + "attn_output.weight"),
                ffn_norm=vec(p + "ffn_norm.weight"), wg=mat(p + "ffn_gate.weight"),
                wu=mat(p + "ffn_up.weight"), wd=mat(p + "ffn_down.weight")))
        emb = mat("token_embd.weight")
        out = mat("output.weight") if "output.weight" in g.tensors else emb
        return cls(cfg, emb, vec("output_norm.weight"), out, layers,
                   meta=dict(g.metadata)).finalize()

    # ------------------------------------------------------------------ synthetic
    @classmethod
    def random(cls, cfg: LLMConfig, device="cuda", seed: int = 0) -> "ModelWeights":
        """Random K-quant blocks of the exact architecture and Q4_K_M type mix, generated on the
        device (a 7B model in seconds).  Block scales are chosen so activations stay O(1)."""
        dev = torch.device(device)
        gen = torch.Generator(device=dev).manual_seed(seed)

        def mat(n, k, t):
            nb = k // 256
            per, size = gguf.BLOCK[t]
            raw = torch.randint(0, 256, (n, nb, size), dtype=torch.uint8, device=dev,
                                generator=gen)
            if t == gguf.Q4_K:
                # w = d*sc*q - dmin*m with sc, m, q uniform: zero mean when dmin = 7.5 d
                d = 1.0 / (31.5 * 4.6 * 1.15 * (k ** 0.5))
                hdr = torch.tensor([d, 7.5 * d], dtype=torch.float16).view(torch.uint8).to(dev)
                raw[:, :, 0:4] = hdr
            else:
                d = 1.0 / (74.0 * 18.5 * (k ** 0.5))
                raw[:, :, 208:210] = torch.tensor([d], dtype=torch.float16).view(torch.uint8).to(dev)
            raw = raw.view(n, nb * size)
            if dev.type == "cuda":
                return QWeight.from_device_raw(raw, t)
            return QWeight.from_raw(raw.numpy(), t, dev)

        def norm(n):
            return (1.0 + 0.1 * torch.randn(n, generator=gen, device=dev)).float()

        def bias(n):
            return (0.1 * torch.randn(n, generator=gen, device=dev)).float()

        Q4, Q6 = gguf.Q4_K, gguf.Q6_K
        d, kv, f = cfg.dim, cfg.kv_dim, cfg.ffn
        layers = []
        for i in range(cfg.layers):
            more = use_more_bits(i, cfg.layers)
            layers.append(LayerWeights(
                attn_norm=norm(d), wq=mat(d, d, Q4), wk=mat(kv, d, Q4),
                wv=mat(kv, d, Q6 if more else Q4),
                bq=bias(d) if cfg.qkv_bias else None, bk=bias(kv) if cfg.qkv_bias else None,
                bv=bias(kv) if cfg.qkv_bias else None, wo=mat(d, d, Q4), ffn_norm=norm(d),
                wg=mat(f, d, Q4), wu=mat(f, d, Q4), wd=mat(d, f, Q6 if more else Q4)))
        return cls(cfg, mat(cfg.vocab, d, Q4), norm(d), mat(cfg.vocab, d, Q6), layers,
                   meta={"synthetic": True}).finalize()

"""Qwen2 inference engine for one MI355X: K-quant GEMV decode on hand-written HIP kernels, replayed
from HIP graphs; prompt processing on an fp16 copy of the weights; a slot-based KV cache.

The reference runs ``llama-server -m <Q4_K_M gguf> --ctx-size 4096 --n-gpu-layers 35`` (reference
cluster-config/apps/llm/deployment.yaml:61-84); this is the in-tree MI355X engine behind the same
kind of server (``server.py``).  Design points:

* **Decode (the hot loop)** is HBM-bound: per token every weight byte is read once.  Per layer:
  fused q|k|v GEMV (RMSNorm + Q8 quantisation in its prologue, +bias) → split-context attention
  (RoPE and the KV-cache write fused in) + combine + Q8 → o_proj GEMV (+= residual) → gate|up
  pair GEMV (RMSNorm prologue, SwiGLU epilogue) → ffn_down GEMV (Q8 prologue, += residual); then
  the final norm and the lm_head: 6 launches per layer.
  ``T <= 4`` concurrent sequences share one weight pass (continuous batching).  Every step of a
  given ``T`` is captured once into a ``torch.cuda.CUDAGraph`` (a HIP graph on ROCm) and replayed,
  so the ~290 launches of a 28-layer step cost no host time.
* **Prefill** is compute-bound: with ``dense=True`` the engine keeps an fp16 copy of every matrix
  (HBM is plentiful: +15 GB for 7B) and runs the prompt through library GEMMs (hipBLASLt) and
  SDPA, writing the KV cache.  Without it, prompts run through the decode kernels 4 tokens at a
  time (causality comes from each token's own length).
* **KV cache**: fp16 ``[layers, slots, kv_heads, max_ctx, 128]`` — one contiguous slab per
  sequence slot; the server maps requests to slots.

On a CPU (tests) the same API runs the fp32 reference maths (dequantised weights, PyTorch ops);
the GPU path is compared against it.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

from .config import LLMConfig
from k8s_nvidia_gpus_amd.ops.llm_kernels import gate_up_interleave, gate_up_split

NORM_PROLOGUE_T = 2     # steps of up to this many tokens normalise in the GEMV prologues
from .weights import ModelWeights, QWeight


def rope_tables(max_ctx: int, head_dim: int, theta: float, device) -> tuple:
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    ang = torch.arange(max_ctx, dtype=torch.float64)[:, None] * inv[None, :]
    return ang.cos().float().to(device), ang.sin().float().to(device)


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """NeoX rotation (pairs i, i + d/2) — llama.cpp's rope type for qwen2.  x [..., P, d]."""
    h = x.shape[-1] // 2
    x0, x1 = x[..., :h], x[..., h:]
    return torch.cat([x0 * cos - x1 * sin, x0 * sin + x1 * cos], -1)


@dataclass
class StepBuffers:
    """Static tensors of one decode step size ``T`` (graph-captured)."""
    T: int
    tok: torch.Tensor
    pos: torch.Tensor
    slot: torch.Tensor
    h: torch.Tensor
    x8: torch.Tensor
    dx: torch.Tensor
    sx: torch.Tensor
    x8f: torch.Tensor       # second Q8 set: the ffn_down input written by the gate|up GEMV while
    dxf: torch.Tensor       # its own input (x8/dx/sx) is still being read
    sxf: torch.Tensor
    qkv: torch.Tensor
    qrot: torch.Tensor
    po: torch.Tensor
    pml: torch.Tensor
    t: torch.Tensor
    logits: torch.Tensor
    graphs: Dict[tuple, torch.cuda.CUDAGraph] = None   # keyed by (attention span, fused rope)
    ids: torch.Tensor = None         # int32 [T]: greedy next tokens (decode_greedy)
    meta: torch.Tensor = None        # int32 [3, T] on the GPU: tok / pos / slot are its rows
    host: torch.Tensor = None        # pinned staging copy of meta
    host_evt: torch.cuda.Event = None
    ids_host: List[torch.Tensor] = None   # two pinned [T] landing buffers of decode_greedy_async
    ids_flip: int = 0


class GreedyStep:
    """An enqueued greedy decode step (``Engine.decode_greedy_async``): ``result()`` waits for its
    token ids.  ``chainable`` is set when the next step may take its tokens straight from this
    one's device buffer (same batch size, one engine call)."""

    def __init__(self, value: Optional[List[int]] = None, host: Optional[torch.Tensor] = None,
                 event: Optional[torch.cuda.Event] = None, buffers: Optional["StepBuffers"] = None):
        self._value, self._host, self._event, self.buffers = value, host, event, buffers
        self.chainable = buffers is not None

    def result(self) -> List[int]:
        if self._value is None:
            self._event.synchronize()
            self._value = self._host.tolist()
        return self._value


class Engine:
    def __init__(self, weights: ModelWeights, max_ctx: int = 4096, slots: int = 4,
                 dense: Optional[bool] = None, use_graphs: bool = True):
        self.w = weights
        self.cfg: LLMConfig = weights.cfg
        self.device = weights.out_norm.device
        self.gpu = self.device.type == "cuda"
        chunk = 256
        self.max_ctx = (max_ctx + chunk - 1) // chunk * chunk
        self.slots = slots
        self.use_graphs = use_graphs and self.gpu
        c = self.cfg
        if c.head_dim != 128 and self.gpu:
            raise ValueError(f"head_dim {c.head_dim}: the decode kernels are built for 128")
        self.kv_dtype = torch.float16 if self.gpu else torch.float32
        shape = (c.layers, slots, c.kv_heads, self.max_ctx, c.head_dim)
        self.k_cache = torch.zeros(shape, dtype=self.kv_dtype, device=self.device)
        self.v_cache = torch.zeros(shape, dtype=self.kv_dtype, device=self.device)
        self.cos, self.sin = rope_tables(self.max_ctx, c.head_dim, c.rope_theta, self.device)
        self.dense = self.gpu if dense is None else dense
        self._dense_w: Optional[Dict[str, torch.Tensor]] = None
        self._bufs: Dict[int, StepBuffers] = {}
        # attn_norm / ffn_norm inside the q|k|v and gate|up GEMV prologues (each workgroup
        # normalises the L2-resident fp32 row itself) for steps of up to NORM_PROLOGUE_T tokens;
        # larger steps normalise + quantise once per input (rmsnorm_q8).  T=1 1.81 -> 1.74 ms
        # (profiles/r03/aa); from T = 3 the shared launch is faster (session AX).  rmsnorm_q8 sums
        # the squares in the 4-wave prologue's order, so both paths give the same bits and decode
        # stays batch-invariant (models with dim >= 8192 run 8-wave GEMVs there: one path for every
        # T).  Attribute, not a knob: the batch-invariance test runs both paths.
        self.norm_prologue = True
        self.norm_prologue_t = NORM_PROLOGUE_T
        # dense prefill on the fused glue kernels (llm_prefill.hip), SDPA's GQA path on the cache
        # slabs and q stored token-major (no transpose copy before o_proj); the PyTorch formulation
        # (prefill_native = False) is the oracle of test_native_prefill_equals_torch_prefill
        self.prefill_native = True
        self.prefill_gqa = True
        self.prefill_qtok = True
        # prompt attention on the hand-written causal GQA kernel over the cache slabs
        # (ops/csrc/llm_prefill_attn.hip); False = PyTorch SDPA (the oracle of its tests)
        self.prefill_attn_native = True
        # rejected variants (in-launch attention combine, fused residual norm, combine in the o_proj
        # prologue, MFMA attention, Infinity-Cache prefetch, ...): docs/experiments/llm_decode_rejected.md
        if self.gpu:
            from k8s_nvidia_gpus_amd.ops import llm_kernels as LK

            self.LK = LK
            self.max_T = LK.max_tokens()
            if LK.gemv_impl() == LK.GEMV_MFMA:
                # GEMVs on the int8 matrix cores: every matrix gets its MFMA-packed copy (the VALU
                # kernel keeps the two-type q|k + v launch up to 4 tokens, and any matrix with
                # N % 16 — steps then stay at the VALU kernel's 4 tokens)
                mats = [self.w.output] + [w for L in self.w.layers
                                          for w in [L.wo, L.wg, L.wu, L.wd] + list(L.wqkv)]
                if not all([w.mfma_pack() for w in mats]):
                    self.max_T = min(self.max_T, 4)
            # split-K combine scratch of the long-row GEMVs (ffn_down; o_proj of dim >= 8192)
            self.kscratch = LK.SplitKScratch(max(c.dim, c.ffn), self.device)
            if self.cfg.dim >= 8192:
                # such models normalise in the 8-wave GEMV prologues at every T (one reduction
                # order, so decode stays batch-invariant), and the prologue form takes at most 4
                # tokens: larger batches run as steps of 4
                self.max_T = min(self.max_T, 4)
        else:
            self.max_T = 4
        self.stats = {"decode_steps": 0, "decode_tokens": 0, "prefill_tokens": 0,
                      "graph_captures": 0}

    # ------------------------------------------------------------------ dense weights (prefill / CPU)
    @property
    def gu_blk(self) -> int:
        """Row-block size of the dense gate|up weight's interleave (0: [gate; up] halves)."""
        return 128 if self.cfg.ffn % 128 == 0 else 0

    def _gate_up(self, mm, xn: torch.Tensor, w: torch.Tensor, t: torch.Tensor) -> None:
        """t = silu(xn·gateᵀ) · (xn·upᵀ) (fp16, GPU prefill): one GEMM with the SwiGLU in its
        epilogue where the shape runs on the 256×256 kernel, else the GEMM and swiglu_f16."""
        if self.gu_blk:
            from k8s_nvidia_gpus_amd.ops import gemm_epi as GE

            if GE.supported(xn, w) and GE.linear_swiglu(xn, w, t) is not None:
                return
        self.LK.swiglu_f16(mm(xn, w), t, self.gu_blk)

    def _res_norm(self, mm_res, x: torch.Tensor, a: torch.Tensor, w: torch.Tensor,
                  norm_w: Optional[torch.Tensor], xn: torch.Tensor) -> torch.Tensor:
        """x += a·wᵀ, then (norm_w given) xn = fp16 RMSNorm(x) · norm_w (GPU prefill): one GEMM
        whose split-K finalize also normalises where the shape runs on the split-K 256×256 form
        (same bits as the two passes), else the residual GEMM and rmsnorm_f16."""
        if norm_w is not None:
            from k8s_nvidia_gpus_amd.ops import gemm_epi as GE

            if GE.supported(a, w) and GE.linear_residual_norm_(x, a, w, norm_w, self.cfg.eps, xn):
                return x
        x = mm_res(x, a, w)
        if norm_w is not None:
            self.LK.rmsnorm_f16(x, norm_w, self.cfg.eps, xn)
        return x

    def dense_weights(self) -> Dict[str, torch.Tensor]:
        if self._dense_w is None:
            dt = torch.float16 if self.gpu else torch.float32
            d: Dict[str, torch.Tensor] = {}
            for i, L in enumerate(self.w.layers):
                d[f"{i}.qkv"] = torch.cat([w.dequant(dt) for w in L.wqkv], 0)
                d[f"{i}.bqkv"] = L.bqkv.to(dt)
                d[f"{i}.o"] = L.wo.dequant(dt)
                if self.gu_blk:      # 128-row gate|up blocks: the fused-SwiGLU GEMM's layout
                    d[f"{i}.gu"] = gate_up_interleave(L.wg.dequant(dt), L.wu.dequant(dt),
                                                      self.gu_blk)
                else:
                    d[f"{i}.gu"] = torch.cat([L.wg.dequant(dt), L.wu.dequant(dt)], 0)
                d[f"{i}.down"] = L.wd.dequant(dt)
            d["out"] = self.w.output.dequant(dt)
            self._dense_w = d
        return self._dense_w

    def embed(self, tokens: torch.Tensor) -> torch.Tensor:
        return self.w.tok_embd.dequant(torch.float32, rows=tokens.to(self.device))

    # ------------------------------------------------------------------ dense forward
    def _forward_dense(self, tokens: torch.Tensor, slot: int, start: int) -> torch.Tensor:
        """Prompt tokens [P] of one sequence at positions start..start+P-1 → last-position logits
        (fp32 [vocab]).  Writes the KV cache."""
        if (self.gpu and self.prefill_native and self.cfg.head_dim == 128
                and self.cfg.dim <= 8192 and self.cfg.dim % 8 == 0 and self.cfg.ffn % 8 == 0):
            return self._forward_dense_native(tokens, slot, start)
        c = self.cfg
        W = self.dense_weights()
        dt = torch.float16 if self.gpu else torch.float32
        P = tokens.numel()
        end = start + P
        x = self.embed(tokens)                                  # fp32 [P, dim]
        cos, sin = self.cos[start:end], self.sin[start:end]
        mask = None
        if P > 1:
            qi = torch.arange(start, end, device=self.device)[:, None]
            kj = torch.arange(end, device=self.device)[None, :]
            mask = kj <= qi
        mm, mm_res = self._dense_ops()
        for i, L in enumerate(self.w.layers):
            xn = (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + c.eps) * L.attn_norm).to(dt)
            qkv = mm(xn, W[f"{i}.qkv"]).float() + L.bqkv
            q = qkv[:, :c.dim].view(P, c.heads, c.head_dim).transpose(0, 1)
            k = qkv[:, c.dim:c.dim + c.kv_dim].view(P, c.kv_heads, c.head_dim).transpose(0, 1)
            v = qkv[:, c.dim + c.kv_dim:].view(P, c.kv_heads, c.head_dim).transpose(0, 1)
            q = apply_rope(q, cos, sin)
            k = apply_rope(k, cos, sin)
            self.k_cache[i, slot, :, start:end] = k.to(self.kv_dtype)
            self.v_cache[i, slot, :, start:end] = v.to(self.kv_dtype)
            kk = self.k_cache[i, slot, :, :end].to(dt).repeat_interleave(c.group, 0)
            vv = self.v_cache[i, slot, :, :end].to(dt).repeat_interleave(c.group, 0)
            o = F.scaled_dot_product_attention(q.to(dt)[None], kk[None], vv[None],
                                               attn_mask=None if mask is None else mask[None, None])
            o = o[0].transpose(0, 1).reshape(P, c.dim)
            x = mm_res(x, o, W[f"{i}.o"])
            xn = (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + c.eps) * L.ffn_norm).to(dt)
            gu = mm(xn, W[f"{i}.gu"]).float()
            g, u = (gate_up_split(gu, self.gu_blk) if self.gu_blk
                    else (gu[:, :c.ffn], gu[:, c.ffn:]))
            t = F.silu(g) * u
            x = mm_res(x, t.to(dt), W[f"{i}.down"])
        xl = x[-1:]
        xn = (xl * torch.rsqrt(xl.pow(2).mean(-1, keepdim=True) + c.eps) * self.w.out_norm).to(dt)
        return mm(xn, W["out"]).float()[0]

    def _forward_dense_native(self, tokens: torch.Tensor, slot: int, start: int) -> torch.Tensor:
        """The GPU prefill: hand-written fp16 GEMMs (bias in the q|k|v epilogue, residual adds
        in the o_proj / ffn_down epilogues) and three glue kernels per layer use
        (ops/csrc/llm_prefill.hip: RMSNorm -> fp16, RoPE + KV-cache write, SwiGLU) instead of
        ~35 PyTorch elementwise launches (profiles/r03/ac)."""
        c, LK = self.cfg, self.LK
        W = self.dense_weights()
        dt = torch.float16
        P = tokens.numel()
        end = start + P
        x = self.embed(tokens)                                  # fp32 [P, dim]
        mask = None
        if P > 1:
            qi = torch.arange(start, end, device=self.device)[:, None]
            kj = torch.arange(end, device=self.device)[None, :]
            mask = kj <= qi
        mm, mm_res = self._dense_ops()
        # a chunk after cached positions (chunked prefill, prompt-cache continuation): causal
        # aligned bottom-right, which SDPA runs in its flash kernel; an explicit [P, end] mask
        # takes the materialising path, 4-5x slower per layer at 2-32k positions
        # (tools/debug/prefill_attn_probe.py, profiles/r05/prefill_attn_probe.log)
        lowright = None
        if P > 1 and start > 0 and self.prefill_gqa:
            from torch.nn.attention.bias import causal_lower_right

            lowright = causal_lower_right(P, end)
        xn = torch.empty(P, c.dim, dtype=dt, device=self.device)
        if self.prefill_qtok:          # [H][P][128] view of token-major storage: SDPA's output
            qh = torch.empty(P, c.heads, c.head_dim, dtype=dt,      # comes back token-major and
                             device=self.device).transpose(0, 1)    # the o reshape is a view
        else:
            qh = torch.empty(c.heads, P, c.head_dim, dtype=dt, device=self.device)
        t = torch.empty(P, c.ffn, dtype=dt, device=self.device)
        native_attn = self.prefill_attn_native and self.prefill_qtok
        if native_attn:
            o = torch.empty(P, c.dim, dtype=dt, device=self.device)
            oh = o.view(P, c.heads, c.head_dim).transpose(0, 1)
        scale = 1.0 / math.sqrt(c.head_dim)
        layers = self.w.layers
        normed = False                 # xn already holds this layer's attn_norm output
        for i, L in enumerate(layers):
            if not normed:
                LK.rmsnorm_f16(x, L.attn_norm, c.eps, xn)
            normed = False
            qkv = mm(xn, W[f"{i}.qkv"], W[f"{i}.bqkv"])
            LK.rope_kv_f16(qkv, self.cos, self.sin, start, c.heads, c.kv_heads, self.max_ctx, qh,
                           self.k_cache[i, slot], self.v_cache[i, slot])
            if native_attn:            # hand-written causal GQA kernel, K/V read in place
                LK.prefill_attn(qh, self.k_cache[i, slot], self.v_cache[i, slot], oh, start, scale)
                x = self._res_norm(mm_res, x, o, W[f"{i}.o"], L.ffn_norm, xn)
                self._gate_up(mm, xn, W[f"{i}.gu"], t)
                if i + 1 < len(layers):     # ffn_down's finalize also writes the next attn_norm
                    x = self._res_norm(mm_res, x, t, W[f"{i}.down"], layers[i + 1].attn_norm, xn)
                    normed = True
                else:
                    x = mm_res(x, t, W[f"{i}.down"])
                continue
            if self.prefill_gqa:       # K/V read in place by SDPA's GQA path; causal flag from 0
                o = F.scaled_dot_product_attention(
                    qh[None], self.k_cache[i, slot, :, :end][None],
                    self.v_cache[i, slot, :, :end][None],
                    attn_mask=None if (mask is None or start == 0) else lowright,
                    is_causal=mask is not None and start == 0, enable_gqa=True)
            else:
                kk = self.k_cache[i, slot, :, :end].repeat_interleave(c.group, 0)
                vv = self.v_cache[i, slot, :, :end].repeat_interleave(c.group, 0)
                o = F.scaled_dot_product_attention(
                    qh[None], kk[None], vv[None],
                    attn_mask=None if mask is None else mask[None, None])
            o = o[0].transpose(0, 1).reshape(P, c.dim)
            x = mm_res(x, o, W[f"{i}.o"])
            LK.rmsnorm_f16(x, L.ffn_norm, c.eps, xn)
            self._gate_up(mm, xn, W[f"{i}.gu"], t)
            x = mm_res(x, t, W[f"{i}.down"])
        LK.rmsnorm_f16(x[-1:], self.w.out_norm, c.eps, xn[:1])
        return mm(xn[:1], W["out"]).float()[0]

    def _forward_dense_native_multi(self, segs) -> torch.Tensor:
        """Prompt chunks of several sequences in one pass (llama-server fills one batch with the
        prompt tokens of every slot that needs them, reference cluster-config/apps/llm/
        deployment.yaml:76-84): the GEMMs and glue kernels run over all rows at once, RoPE + the
        KV write and attention per sequence.  ``segs``: [(tokens, slot, start)]; returns the
        last-token logits of each chunk, fp32 [len(segs), vocab]."""
        c, LK = self.cfg, self.LK
        W = self.dense_weights()
        dt = torch.float16
        lens = [int(t.numel()) for t, _, _ in segs]
        offs = [0]
        for n in lens:
            offs.append(offs[-1] + n)
        P = offs[-1]
        x = self.embed(torch.cat([t for t, _, _ in segs]))   # fp32 [P, dim]
        mm, mm_res = self._dense_ops()
        from torch.nn.attention.bias import causal_lower_right

        lowright = [causal_lower_right(n, st + n) if n > 1 and st > 0 else None
                    for n, (_, _, st) in zip(lens, segs)]
        xn = torch.empty(P, c.dim, dtype=dt, device=self.device)
        qh = torch.empty(P, c.heads, c.head_dim, dtype=dt, device=self.device).transpose(0, 1)
        o = torch.empty(P, c.dim, dtype=dt, device=self.device)
        t = torch.empty(P, c.ffn, dtype=dt, device=self.device)
        layers = self.w.layers
        normed = False                 # xn already holds this layer's attn_norm output
        for i, L in enumerate(layers):
            if not normed:
                LK.rmsnorm_f16(x, L.attn_norm, c.eps, xn)
            normed = False
            qkv = mm(xn, W[f"{i}.qkv"], W[f"{i}.bqkv"])
            for s, (_, slot, st) in enumerate(segs):
                a, b = offs[s], offs[s + 1]
                LK.rope_kv_f16(qkv[a:b], self.cos, self.sin, st, c.heads, c.kv_heads,
                               self.max_ctx, qh[:, a:b], self.k_cache[i, slot], self.v_cache[i, slot])
            for s, (_, slot, st) in enumerate(segs):
                a, b = offs[s], offs[s + 1]
                n, end = b - a, st + b - a
                if self.prefill_attn_native:
                    LK.prefill_attn(qh[:, a:b], self.k_cache[i, slot], self.v_cache[i, slot],
                                    o[a:b].view(n, c.heads, c.head_dim).transpose(0, 1), st,
                                    1.0 / math.sqrt(c.head_dim))
                    continue
                os_ = F.scaled_dot_product_attention(
                    qh[None, :, a:b], self.k_cache[i, slot, :, :end][None],
                    self.v_cache[i, slot, :, :end][None], attn_mask=lowright[s],
                    is_causal=n > 1 and st == 0, enable_gqa=True)
                o[a:b] = os_[0].transpose(0, 1).reshape(n, c.dim)
            x = self._res_norm(mm_res, x, o, W[f"{i}.o"], L.ffn_norm, xn)
            self._gate_up(mm, xn, W[f"{i}.gu"], t)
            if i + 1 < len(layers):
                x = self._res_norm(mm_res, x, t, W[f"{i}.down"], layers[i + 1].attn_norm, xn)
                normed = True
            else:
                x = mm_res(x, t, W[f"{i}.down"])
        last = torch.tensor([b - 1 for b in offs[1:]], device=self.device)
        xl = x.index_select(0, last)
        LK.rmsnorm_f16(xl, self.w.out_norm, c.eps, xn[:len(segs)])
        return mm(xn[:len(segs)], W["out"]).float()

    def _dense_ops(self):
        """Prompt-processing GEMMs: on the GPU the hand-written fp16 MFMA GEMMs
        (``ops/gemm_epi.py``: tile / split-K planned per shape, the residual add of o_proj and
        ffn_down fused into the epilogue straight into the fp32 stream); PyTorch on the CPU."""
        if self.gpu:
            from k8s_nvidia_gpus_amd.ops import gemm_epi as GE

            def mm(a, w, b=None):
                if GE.supported(a, w):
                    return GE.linear(a, w, b)
                y = a @ w.t()
                return y if b is None else y + b

            def mm_res(x, a, w):
                if GE.supported(a, w) and x.is_contiguous():
                    return GE.linear_residual_(x, a, w)
                return x + (a @ w.t()).float()
            return mm, mm_res
        return ((lambda a, w, b=None: a @ w.t() if b is None else a @ w.t() + b),
                (lambda x, a, w: x + (a @ w.t()).float()))

    # ------------------------------------------------------------------ native decode
    def _buffers(self, T: int) -> StepBuffers:
        b = self._bufs.get(T)
        if b is None:
            c, dev = self.cfg, self.device
            kmax = max(c.dim, c.ffn)
            nsplit = self.max_ctx // self.LK.attn_chunk()
            f32 = dict(dtype=torch.float32, device=dev)
            meta = torch.zeros(3, T, dtype=torch.int32, device=dev)
            b = StepBuffers(
                T=T, tok=meta[0], pos=meta[1], slot=meta[2], meta=meta,
                host=torch.zeros(3, T, dtype=torch.int32).pin_memory(),
                # decode_greedy_async's landing buffers, pinned here (at graph capture) rather than
                # at a request's first step
                ids_host=[torch.zeros(T, dtype=torch.int32).pin_memory() for _ in range(2)],
                ids=torch.zeros(T, dtype=torch.int32, device=dev),
                h=torch.zeros(T, c.dim, **f32),
                x8=torch.zeros(T, kmax, dtype=torch.int8, device=dev),
                dx=torch.zeros(T, kmax // 32, **f32), sx=torch.zeros(T, kmax // 16, **f32),
                x8f=torch.zeros(T, c.ffn, dtype=torch.int8, device=dev),
                dxf=torch.zeros(T, c.ffn // 32, **f32), sxf=torch.zeros(T, c.ffn // 16, **f32),
                qkv=torch.zeros(T, c.dim + 2 * c.kv_dim, **f32), qrot=torch.zeros(T, c.dim, **f32),
                po=torch.zeros(T, c.heads, nsplit, c.head_dim, **f32),
                pml=torch.zeros(T, c.heads, nsplit, 2, **f32), t=torch.zeros(T, c.ffn, **f32),
                logits=torch.zeros(T, c.vocab, **f32))
            self._bufs[T] = b
        return b

    def _q8(self, b: StepBuffers, k: int):
        """Views of the Q8 activation buffers for inner dimension ``k`` (contiguous [T, k])."""
        T = b.T
        return (b.x8.view(-1)[:T * k].view(T, k), b.dx.view(-1)[:T * k // 32].view(T, k // 32),
                b.sx.view(-1)[:T * k // 16].view(T, k // 16))

    def _span(self, max_pos: int) -> int:
        """Attention span bucket for a step whose furthest position is ``max_pos``: the next power
        of two (>= 256), so a graph covers many steps and never launches chunks far past the
        context in use."""
        span = 256
        while span <= max_pos:
            span *= 2
        return min(span, self.max_ctx)

    def _step_kernels(self, b: StepBuffers, span: int, fused: bool) -> None:
        """One decode step, per layer: q|k|v (one two-matrix launch when q|k and v have different
        quantisation types) → attention (+ its combine, which writes the Q8 o_proj input) → o_proj
        (+= residual) → gate|up (SwiGLU, Q8 out) → ffn_down (+= residual).  ``fused``: every token
        in its own slot, so RoPE + the KV write run inside the attention kernel (no rope_kv launch).
        Steps of up to NORM_PROLOGUE_T tokens normalise in the GEMV prologues, larger ones once per
        input with rmsnorm_q8."""
        LK, c = self.LK, self.cfg
        LK.dequant(self.w.tok_embd, b.h, rows=b.tok)          # embedding rows → residual
        qd = self._q8(b, c.dim)
        qf = (b.x8f, b.dxf, b.sxf)
        scale = 1.0 / math.sqrt(c.head_dim)
        pro = self.norm_prologue and (c.dim >= 8192 or b.T <= self.norm_prologue_t)

        def act(xf, norm_w):
            """GEMV input: (Q8 views, {}) quantised here, or ((None,) * 3, prologue kwargs)."""
            if pro:
                return (None, None, None), dict(xf=xf, norm_w=norm_w, eps=c.eps)
            LK.rmsnorm_q8(xf, norm_w, c.eps, *qd)
            return qd, {}

        for i, L in enumerate(self.w.layers):
            self._qkv(b, L, *act(b.h, L.attn_norm))
            if fused:
                LK.attn_decode(None, b.pos, b.slot, self.k_cache[i], self.v_cache[i], c.heads,
                               c.kv_heads, c.head_dim, self.max_ctx, scale, b.po, b.pml, *qd,
                               span=span, qkv=b.qkv, cos_t=self.cos, sin_t=self.sin)
            else:
                LK.rope_kv(b.qkv, b.pos, b.slot, self.cos, self.sin, c.heads, c.kv_heads,
                           c.head_dim, self.max_ctx, b.qrot, self.k_cache[i], self.v_cache[i])
                LK.attn_decode(b.qrot, b.pos, b.slot, self.k_cache[i], self.v_cache[i], c.heads,
                               c.kv_heads, c.head_dim, self.max_ctx, scale, b.po, b.pml, *qd,
                               span=span)
            LK.qgemv(L.wo, *qd, b.h, LK.RESID, kscratch=self.kscratch)
            xin = act(b.h, L.ffn_norm)
            if c.ffn % 32 == 0:      # the pair GEMV quantises silu(g)·u (the ffn_down input) itself
                LK.qgemv(L.wg, *xin[0], b.t, LK.PAIR, w1=L.wu, **xin[1], q8_out=qf)
                LK.qgemv(L.wd, *qf, b.h, LK.RESID, kscratch=self.kscratch)
            else:
                LK.qgemv(L.wg, *xin[0], b.t, LK.PAIR, w1=L.wu, **xin[1])
                LK.rmsnorm_q8(b.t, None, c.eps, *self._q8(b, c.ffn))
                LK.qgemv(L.wd, *self._q8(b, c.ffn), b.h, LK.RESID, kscratch=self.kscratch)
        LK.rmsnorm_q8(b.h, self.w.out_norm, c.eps, *qd)
        LK.qgemv(self.w.output, *qd, b.logits, LK.STORE)

    def _qkv(self, b: StepBuffers, L, q8, pro) -> None:
        """q|k|v projections from the Q8 input (or, with ``pro``, from fp32 rows normalised in the
        GEMV prologue): one launch, also when q|k and v are stored in different quantisation
        types (two-matrix GEMV)."""
        LK = self.LK
        if len(L.wqkv) == 2:
            w0, w1 = L.wqkv
            if LK.qgemv2(w0, w1, *q8, b.qkv[:, :w0.n], b.qkv[:, w0.n:], bias0=L.bqkv[:w0.n],
                         bias1=L.bqkv[w0.n:], **pro):
                return
        off = 0
        for w in L.wqkv:
            LK.qgemv(w, *q8, b.qkv[:, off:], LK.STORE, bias=L.bqkv[off:], ldo=b.qkv.stride(0),
                     **pro)
            off += w.n

    def _decode_native(self, tokens: Optional[Sequence[int]], positions: Sequence[int],
                       slots: Sequence[int], greedy: bool = False) -> torch.Tensor:
        """``tokens`` None: the tokens are the previous greedy step's ids of this batch size,
        still on the GPU (a chained step, ``decode_greedy_async``)."""
        T = len(positions)
        b = self._buffers(T)
        # one H2D copy per step from a pinned staging row (three synchronous pageable copies cost
        # ~3 x 10 us of idle GPU per token); the event guards the row against being rewritten
        # before the previous step's copy has read it
        if b.host_evt is not None:
            b.host_evt.synchronize()
        if tokens is None:
            b.host[1:].copy_(torch.tensor([list(positions), list(slots)], dtype=torch.int32))
            b.meta[1:].copy_(b.host[1:], non_blocking=True)
            b.meta[0].copy_(b.ids)                      # device to device, in stream order
        else:
            b.host.copy_(torch.tensor([list(tokens), list(positions), list(slots)],
                                      dtype=torch.int32))
            b.meta.copy_(b.host, non_blocking=True)
        if b.host_evt is None:
            b.host_evt = torch.cuda.Event()
        b.host_evt.record()
        span = self._span(max(positions))
        fused = len(set(slots)) == len(slots)

        def step():
            self._step_kernels(b, span, fused)
            if greedy:                 # the argmax inside the graph: one small copy per step
                self.LK.argmax_rows(b.logits, b.ids)

        if self.use_graphs:
            if b.graphs is None:
                b.graphs = {}
            g = b.graphs.get((span, fused, greedy))
            if g is None:
                s = torch.cuda.Stream(self.device)
                s.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(s):
                    step()                                  # warm-up outside capture
                torch.cuda.current_stream(self.device).wait_stream(s)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    step()
                b.graphs[(span, fused, greedy)] = g
                self.stats["graph_captures"] += 1
            g.replay()
        else:
            step()
        return b.ids if greedy else b.logits

    # ------------------------------------------------------------------ public API
    def decode(self, tokens: Sequence[int], positions: Sequence[int],
               slots: Sequence[int]) -> torch.Tensor:
        """One step for T sequences: token ``tokens[i]`` at ``positions[i]`` of slot ``slots[i]``.
        Returns fp32 logits [T, vocab] (a view of a reused buffer on the GPU: copy to keep)."""
        T = len(tokens)
        if T == 0:
            raise ValueError("decode: no tokens")
        for p in positions:
            if p >= self.max_ctx:
                raise ValueError(f"position {p} beyond the context ({self.max_ctx})")
        self.stats["decode_steps"] += 1
        self.stats["decode_tokens"] += T
        if self.gpu:
            if T <= self.max_T:
                return self._decode_native(tokens, positions, slots)
            # more sequences than one step takes: chunks of max_T reuse one step buffer, so each
            # chunk's logits are copied out before the next chunk overwrites them
            return torch.cat([self._decode_native(tokens[i:i + self.max_T],
                                                  positions[i:i + self.max_T],
                                                  slots[i:i + self.max_T]).clone()
                              for i in range(0, T, self.max_T)], 0)
        rows = [self._forward_dense(torch.tensor([t]), s, p)
                for t, p, s in zip(tokens, positions, slots)]
        return torch.stack(rows, 0)

    def decode_greedy(self, tokens: Sequence[int], positions: Sequence[int],
                      slots: Sequence[int]) -> List[int]:
        """:meth:`decode` + argmax of each row (the first index of the maximum, as torch.argmax),
        on the GPU inside the step's HIP graph: the host receives T token ids, not T x vocab
        logits, and no separate argmax launch follows the step."""
        T = len(tokens)
        if T == 0:
            raise ValueError("decode: no tokens")
        if not self.gpu:
            return torch.argmax(self.decode(tokens, positions, slots), -1).tolist()
        for p in positions:
            if p >= self.max_ctx:
                raise ValueError(f"position {p} beyond the context ({self.max_ctx})")
        self.stats["decode_steps"] += 1
        self.stats["decode_tokens"] += T
        out: List[int] = []
        for i in range(0, T, self.max_T):
            out += self._decode_native(tokens[i:i + self.max_T], positions[i:i + self.max_T],
                                       slots[i:i + self.max_T], greedy=True).tolist()
        return out

    def decode_greedy_async(self, tokens: Optional[Sequence[int]], positions: Sequence[int],
                            slots: Sequence[int],
                            chain: Optional[GreedyStep] = None) -> GreedyStep:
        """:meth:`decode_greedy` without waiting: the step is enqueued and its ids are copied to a
        pinned host buffer behind it, so the caller can do its host work for the previous step
        while this one runs.  ``tokens`` None with ``chain`` (a chainable step of the same batch
        size whose sequences are these, in this order): the tokens are ``chain``'s ids, read on
        the GPU — the next step is enqueued before ``chain``'s result reaches the host."""
        T = len(positions)
        if T == 0:
            raise ValueError("decode: no tokens")
        if tokens is None and (chain is None or not chain.chainable or chain.buffers.T != T):
            raise ValueError("decode_greedy_async: a chained step needs a chainable step of the "
                             "same size")
        if not self.gpu or T > self.max_T:
            toks = list(tokens) if tokens is not None else chain.result()
            return GreedyStep(value=self.decode_greedy(toks, positions, slots))
        for p in positions:
            if p >= self.max_ctx:
                raise ValueError(f"position {p} beyond the context ({self.max_ctx})")
        self.stats["decode_steps"] += 1
        self.stats["decode_tokens"] += T
        ids = self._decode_native(tokens, positions, slots, greedy=True)
        b = self._buffers(T)
        if b.ids_host is None:
            b.ids_host = [torch.zeros(T, dtype=torch.int32).pin_memory() for _ in range(2)]
        # two landing buffers: the previous step's may still be read by the caller
        host = b.ids_host[b.ids_flip]
        b.ids_flip ^= 1
        host.copy_(ids, non_blocking=True)
        evt = torch.cuda.Event()
        evt.record()
        return GreedyStep(host=host, event=evt, buffers=b)

    def prefill(self, tokens: Sequence[int], slot: int, start: int = 0) -> torch.Tensor:
        """Process prompt tokens of one sequence; returns the logits of its last token [vocab]."""
        P = len(tokens)
        if P == 0:
            raise ValueError("prefill: empty prompt")
        if start + P > self.max_ctx:
            raise ValueError(f"prompt of {P} tokens at {start} exceeds the context ({self.max_ctx})")
        self.stats["prefill_tokens"] += P
        if self.dense or not self.gpu:
            return self._forward_dense(torch.tensor(list(tokens), device=self.device), slot, start)
        logits = None
        for i in range(0, P, self.max_T):
            chunk = list(tokens[i:i + self.max_T])
            n = len(chunk)
            logits = self._decode_native(chunk, list(range(start + i, start + i + n)), [slot] * n)
            logits = logits[n - 1]
        return logits.clone()

    def prefill_many(self, items: Sequence[Tuple[Sequence[int], int, int]]) -> List[torch.Tensor]:
        """Prompt chunks of several sequences ``[(tokens, slot, start)]`` (distinct slots) in one
        pass on the GPU prompt path; each chunk's last-token logits [vocab].  Elsewhere (CPU, the
        decode-kernel prompt path) the chunks run one after the other."""
        items = [(list(t), int(s), int(st)) for t, s, st in items]
        slots = [s for _, s, _ in items]
        native = (self.gpu and self.dense and self.prefill_native and self.prefill_gqa
                  and self.prefill_qtok and self.cfg.head_dim == 128 and self.cfg.dim <= 8192
                  and self.cfg.dim % 8 == 0 and self.cfg.ffn % 8 == 0)
        if len(items) == 1 or not native or len(set(slots)) != len(slots):
            return [self.prefill(t, s, st) for t, s, st in items]
        for t, _, st in items:
            if not t:
                raise ValueError("prefill: empty prompt")
            if st + len(t) > self.max_ctx:
                raise ValueError(f"prompt of {len(t)} tokens at {st} exceeds the context "
                                 f"({self.max_ctx})")
        self.stats["prefill_tokens"] += sum(len(t) for t, _, _ in items)
        logits = self._forward_dense_native_multi(
            [(torch.tensor(t, device=self.device), s, st) for t, s, st in items])
        return [logits[i] for i in range(len(items))]

    def warmup(self, lengths: Sequence[int] = (1, 64, 512, 2048), slot: int = 0) -> None:
        """Run the prompt path once per length, from position 0 and as a continuation chunk, so
        the first request of each kind does not pay first-use costs (kernel images SDPA loads on
        first use of a shape class, allocator growth: ~250 ms on the first 512-token prompt,
        profiles/r05/serve).  Writes the KV of slot ``slot`` (and the first position of slots
        0..7), which the server then treats as empty."""
        for n in lengths:
            if 2 * n + 1 >= self.max_ctx:
                continue
            self.prefill([1] * n, slot, start=0)
            self.prefill([1] * n, slot, start=n)
        # prompt batches of 2..8 slots: their last-token rows meet the output matrix as M = 2..8
        # (a first use there cost ~50 ms of a batch's time to first token, session r05ai)
        for k in range(2, min(8, self.slots) + 1):
            self.prefill_many([([1], s, 0) for s in range(k)])
        if self.gpu:
            torch.cuda.synchronize(self.device)

    def capture(self, sizes: Sequence[int] = (1, 2, 3, 4)) -> None:
        """Capture every decode graph (batch sizes x attention-span buckets, sampled and greedy
        steps, one sequence per slot as the server runs them) up front — the server does this
        before it reports ready.  Writes only position ``span-1`` of the slots it uses."""
        if not self.gpu:
            return
        spans = []
        s = 256
        while True:
            spans.append(min(s, self.max_ctx))
            if s >= self.max_ctx:
                break
            s *= 2
        for T in sizes:
            if T <= self.max_T:
                slots = list(range(T)) if T <= self.slots else [0] * T
                for span in spans:
                    for greedy in (False, True):
                        self._decode_native([0] * T, [span - 1] * T, slots, greedy=greedy)
        torch.cuda.synchronize(self.device)


def sample(logits: torch.Tensor, temperature: float = 0.0, top_k: int = 0, top_p: float = 1.0,
           generator: Optional[torch.Generator] = None) -> int:
    """Greedy at temperature 0; otherwise top-k / top-p then temperature (``sampling.py`` has the
    full llama-server parameter set)."""
    from .sampling import SamplingParams, sample_token

    return sample_token(logits, SamplingParams(temperature, top_k, top_p), (), generator)


def generate(engine: Engine, prompt: Sequence[int], max_new: int, slot: int = 0,
             eos: Sequence[int] = (), temperature: float = 0.0, seed: Optional[int] = None) -> dict:
    """Single-sequence generation (benchmarks, tests).  Returns tokens and timings."""
    gen = None
    if temperature > 0:
        gen = torch.Generator(device=engine.device if engine.gpu else "cpu")
        gen.manual_seed(seed if seed is not None else 0)
    t0 = time.perf_counter()
    logits = engine.prefill(prompt, slot)
    tok = sample(logits, temperature, generator=gen)
    t1 = time.perf_counter()
    out = [tok]
    pos = len(prompt)
    while len(out) < max_new and tok not in eos and pos < engine.max_ctx - 1:
        logits = engine.decode([tok], [pos], [slot])[0]
        tok = sample(logits, temperature, generator=gen)
        out.append(tok)
        pos += 1
    t2 = time.perf_counter()
    n_dec = max(1, len(out) - 1)
    return {"tokens": out, "prefill_s": t1 - t0, "decode_s": t2 - t1,
            "decode_tok_s": n_dec / max(t2 - t1, 1e-9), "prompt_tokens": len(prompt)}

"""Hot-op dispatch of the Wan2.1 DiT: hand-written gfx950 kernels on the GPU, PyTorch reference
math elsewhere (same contract as ``models/sd15/functional.py``: no silent fallback — with a GPU
tensor and the native backend a missing kernel library raises).

The DiT block (reference workload: the ``wan2.1_t2v_1.3B`` model the reference's ComfyUI graph
loads, generate_wan_t2v.py:347) is, per token row of width C::

    h = LN(x) * (1 + scale1) + shift1          → q|k|v GEMM → RMSNorm(q), RMSNorm(k), 3-D RoPE
    x = x + gate1 * o_proj(attn(q, k, v))
    h = LN_affine(x)                           → q GEMM → RMSNorm(q) → attn(q, K_text, V_text)
    x = x + o_proj(...)
    h = LN(x) * (1 + scale2) + shift2          → FFN (GELU-tanh)
    x = x + gate2 * ffn(h)

so every residual update is immediately followed by a LayerNorm of the new residual.  The two fused
ops below cover all of it:

* ``add_ln(x, y, gate, mul, add, eps)`` — ``x += y · gate`` (fp32 residual stream, in place) then
  ``out = LN(x) · mul + add`` in bf16 for the next GEMM; ``mul``/``add`` are per-sample modulation
  rows (``1 + scale``, ``shift``) or, with batch stride 0, an affine LayerNorm's weight/bias;
* ``rmsnorm_rope(t, w, cos, sin, heads, eps)`` — in place on a strided column slice of the fused
  q|k|v projection: RMSNorm over the full width (Wan normalises q and k before the head split),
  then the rotary embedding of each head's adjacent pairs with a per-token angle table (the 3-D
  frame/height/width split is folded into the table).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

_BACKEND = os.environ.get("AMDK8S_WAN_BACKEND", "auto")   # auto | native | torch


def set_backend(name: str) -> None:
    global _BACKEND
    if name not in ("auto", "native", "torch"):
        raise ValueError(name)
    _BACKEND = name


def _native(t: torch.Tensor) -> bool:
    if _BACKEND == "torch":
        return False
    if _BACKEND == "native":
        if t.device.type != "cuda":
            raise RuntimeError("native Wan kernels need tensors on the GPU")
        return True
    return t.device.type == "cuda"


def _wk():
    from k8s_nvidia_gpus_amd.ops import wan_kernels

    return wan_kernels


# ---------------------------------------------------------------- residual add + LayerNorm
def add_ln_ref(x: torch.Tensor, y: Optional[torch.Tensor], gate: Optional[torch.Tensor],
               mul: torch.Tensor, add: torch.Tensor, eps: float,
               out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """Reference of :func:`add_ln`: updates ``x`` (fp32 [B, L, C]) in place, returns the LN output
    in ``out_dtype`` (default: bf16, or ``y``'s dtype).  ``gate``/``mul``/``add`` are [B, C] or
    [1, C] fp32."""
    if y is not None:
        upd = y.float() if gate is None else y.float() * gate.float()[:, None, :]
        x.add_(upd)
    n = F.layer_norm(x.float(), (x.shape[-1],), eps=eps)
    out = n * mul.float()[:, None, :] + add.float()[:, None, :]
    if out_dtype is None:
        out_dtype = torch.bfloat16 if y is None else y.dtype
    return out.to(out_dtype)


def add_ln(x: torch.Tensor, y: Optional[torch.Tensor], gate: Optional[torch.Tensor],
           mul: torch.Tensor, add: torch.Tensor, eps: float,
           out_dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    if _native(x) and _wk().add_ln_supported(x.shape[-1]):
        return _wk().add_ln(x, y, gate, mul, add, eps, out_dtype)
    return add_ln_ref(x, y, gate, mul, add, eps, out_dtype)


# ---------------------------------------------------------------- RMSNorm (+ RoPE), in place
def rope_table(grid, head_dim: int, theta: float = 10000.0, device=None):
    """cos/sin ``[F·H·W, head_dim/2]`` fp32 for Wan's 3-D rotary split: of the ``head_dim/2``
    complex pairs, the first ``d/2 − 2·(d//6)`` rotate with the frame index, the next ``d//6`` with
    the row, the last ``d//6`` with the column (each section its own 1/θ^(2i/D) spectrum)."""
    f, h, w = grid
    d = head_dim
    dims = (d - 4 * (d // 6), 2 * (d // 6), 2 * (d // 6))

    def inv(dd):
        return 1.0 / (theta ** (torch.arange(0, dd, 2, dtype=torch.float64) / dd))

    ff, hh, ww = torch.meshgrid(torch.arange(f, dtype=torch.float64),
                                torch.arange(h, dtype=torch.float64),
                                torch.arange(w, dtype=torch.float64), indexing="ij")
    ang = torch.cat([ff.reshape(-1, 1) * inv(dims[0])[None], hh.reshape(-1, 1) * inv(dims[1])[None],
                     ww.reshape(-1, 1) * inv(dims[2])[None]], dim=1)
    return ang.cos().float().to(device), ang.sin().float().to(device)


def rmsnorm_rope_ref(t: torch.Tensor, w: torch.Tensor, cos: Optional[torch.Tensor],
                     sin: Optional[torch.Tensor], heads: int, eps: float) -> torch.Tensor:
    b, l, c = t.shape
    xf = t.float()
    xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    if cos is not None:
        d = c // heads
        xp = xf.reshape(b, l, heads, d // 2, 2)
        c_ = cos[None, :, None, :]
        s_ = sin[None, :, None, :]
        x0, x1 = xp[..., 0], xp[..., 1]
        xf = torch.stack([x0 * c_ - x1 * s_, x0 * s_ + x1 * c_], dim=-1).reshape(b, l, c)
    t.copy_(xf.to(t.dtype))
    return t


def rmsnorm_rope(t: torch.Tensor, w: torch.Tensor, cos: Optional[torch.Tensor],
                 sin: Optional[torch.Tensor], heads: int, eps: float) -> torch.Tensor:
    """In place on ``t`` ([B, L, C], any row stride, unit inner stride)."""
    if _native(t) and _wk().rmsnorm_rope_supported(t, heads):
        return _wk().rmsnorm_rope(t, w, cos, sin, heads, eps)
    return rmsnorm_rope_ref(t, w, cos, sin, heads, eps)


def rmsnorm_rope_qk(qkv: torch.Tensor, wq: torch.Tensor, wk: torch.Tensor, cos, sin, heads: int,
                    eps: float) -> None:
    """q and k slices of the fused ``[B, L, 3C]`` projection, in place (one launch natively)."""
    c = qkv.shape[-1] // 3
    q = qkv[..., :c]
    if _native(qkv) and _wk().rmsnorm_rope_supported(q, heads):
        _wk().rmsnorm_rope(q, wq, cos, sin, heads, eps, w2=wk)
        return
    rmsnorm_rope_ref(q, wq, cos, sin, heads, eps)
    rmsnorm_rope_ref(qkv[..., c:2 * c], wk, cos, sin, heads, eps)


# ---------------------------------------------------------------- attention
def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int) -> torch.Tensor:
    """Unmasked multi-head attention on ``[B, L, H·d]`` rows (strided column views allowed): the
    SD family's gfx950 flash-attention kernel serves Wan's head dim 128."""
    from k8s_nvidia_gpus_amd.models.sd15 import functional as SF

    return SF.attention(q, k, v, heads)


def gelu_tanh(x: torch.Tensor) -> torch.Tensor:
    return F.gelu(x, approximate="tanh")


# ---------------------------------------------------------------- projections (hand-written GEMM)
def _ge():
    from k8s_nvidia_gpus_amd.ops import gemm_epi

    return gemm_epi


_GEMM = os.environ.get("AMDK8S_WAN_GEMM", "native")   # native | torch (A/B against hipBLASLt)


def _gemm_native(x: torch.Tensor, w: torch.Tensor) -> bool:
    return _GEMM != "torch" and _native(x) and _ge().supported(x, w)


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor]) -> torch.Tensor:
    """``x·wᵀ + b``: the gfx950 256×128-tile GEMM (``csrc/gemm_bf16_epi.hip``) on the GPU."""
    if _gemm_native(x, w):
        return _ge().linear(x, w, b)
    return F.linear(x, w, b)


def linear_gelu(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``gelu_tanh(x·wᵀ + b)``, bias and tanh-GELU in the GEMM's epilogue: the [B·L, ffn]
    pre-activation is never written to and re-read from HBM (Wan2.1-1.3B: 2 × 2560 × 8960 bf16 per
    block, 30 blocks per step)."""
    if _gemm_native(x, w):
        return _ge().linear_gelu(x, w, b)
    return F.gelu(F.linear(x, w, b), approximate="tanh")


def linear_residual_(res: torch.Tensor, x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor],
                     gate: Optional[torch.Tensor]) -> torch.Tensor:
    """``res += gate · (x·wᵀ + b)`` on the fp32 residual stream, in place (``gate`` [B, C] per
    sample or None): the projection's output goes straight into the residual from the GEMM's
    fp32 accumulators instead of a bf16 round trip through HBM."""
    if _gemm_native(x, w) and res.is_contiguous():
        return _ge().linear_residual_(res, x, w, b, gate)
    y = F.linear(x, w, b).float()
    if gate is not None:
        y = y * gate.float()[:, None, :]
    return res.add_(y)

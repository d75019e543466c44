"""Hot-op dispatch of the SD1.5 model family: hand-written gfx950 HIP kernels on the GPU, PyTorch
reference math elsewhere.

Each op has one native implementation (``k8s_nvidia_gpus_amd/ops/csrc/sd_*.hip`` through
``ops/sd_kernels.py``) and one plain-PyTorch reference used on CPU and by the numerics tests.
There is no silent fallback on a GPU: with ``backend() == "native"`` (the default for CUDA/HIP
tensors) a missing kernel library raises ``KernelLibraryError``.

Ops (all activations are channels-last, i.e. NHWC memory = ``[N, H*W, C]`` token rows):

* ``group_norm(x, w, b, groups, eps, silu)`` — GroupNorm with the SiLU that follows it in every
  ResNet block fused into the same pass (SD1.5 UNet: 61 GroupNorms per forward).
* ``attention(q, k, v, heads)`` — softmax(q·kᵀ/√d)·v over ``[N, L, heads*d]`` rows, head dims 40 /
  80 / 160 (UNet) and 64 (CLIP-free paths); q/k/v may be strided column views of one fused
  projection output.
* ``geglu(x)`` — ``h * gelu(g)`` for ``x = [h | g]`` (the transformer feed-forward's gate).
* ``linear(x, w, b)`` — the transformer projections (fused q|k|v, cross k|v, out, GEGLU in / out,
  the 1×1 proj_in / proj_out convolutions as token GEMMs) on the hand-written gfx950 GEMMs
  (``ops/csrc/gemm_bf16_epi.hip``: tile picked by problem size; fp16 operands, bias in the
  epilogue).
* ``conv3x3(x, conv, bias, stride, up, residual)`` — the 3×3 convolutions (ResNet conv1 / conv2,
  down- and up-samplers) as implicit GEMMs on the same kernel family: padding taps read a zero row,
  the nearest-2× upsample is folded into the input addressing, and conv2's bias + the block's
  residual (or 1×1-shortcut output) ride in the epilogue — no MIOpen, no separate add pass.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.nn.functional as F

_BACKEND = os.environ.get("AMDK8S_SD_BACKEND", "auto")   # auto | native | torch


def set_backend(name: str) -> None:
    global _BACKEND
    if name not in ("auto", "native", "torch"):
        raise ValueError(name)
    _BACKEND = name


def backend() -> str:
    return _BACKEND


def _native(t: torch.Tensor) -> bool:
    if _BACKEND == "torch":
        return False
    if _BACKEND == "native":
        if t.device.type != "cuda":
            raise RuntimeError("native SD kernels need tensors on the GPU")
        return True
    return t.device.type == "cuda"


def _sd():
    from k8s_nvidia_gpus_amd.ops import sd_kernels

    return sd_kernels


# ---------------------------------------------------------------- projections
_GEMM = os.environ.get("AMDK8S_SD_GEMM", "native")   # native | torch (A/B against hipBLASLt)


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    if _GEMM != "torch" and _native(x):
        from k8s_nvidia_gpus_amd.ops import gemm_epi

        if gemm_epi.supported(x, w):
            return gemm_epi.linear(x, w, b)
    return F.linear(x, w, b)


def linear_add(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor],
               r: torch.Tensor) -> torch.Tensor:
    """``x·wᵀ + b + r`` with the residual add in the GEMM epilogue (``r`` [..., N], x's dtype)."""
    if _GEMM != "torch" and _native(x) and r.dtype == x.dtype and r.stride(-1) == 1:
        from k8s_nvidia_gpus_amd.ops import gemm_epi

        if gemm_epi.supported(x, w):
            rr = r.reshape(-1, r.shape[-1])
            if rr.data_ptr() % 16 == 0 and rr.stride(0) % 8 == 0:
                return gemm_epi.linear_add(x, w, b, rr).view(r.shape)
    return F.linear(x, w, b) + r


_CONV = os.environ.get("AMDK8S_SD_CONV", "native")   # native | torch (A/B against MIOpen)


def _conv_weight(conv: torch.nn.Conv2d, dtype: torch.dtype) -> torch.Tensor:
    """The kernel's [Cout, 9·Cin] weight, packed once per (weight version, dtype)."""
    from k8s_nvidia_gpus_amd.ops import gemm_epi

    w = conv.weight
    key = (w.data_ptr(), w._version, dtype)
    cached = getattr(conv, "_amdk8s_wk", None)
    if cached is None or cached[0] != key:
        cached = (key, gemm_epi.conv_weight(w.detach().to(dtype)))
        conv._amdk8s_wk = cached
    return cached[1]


def conv3x3(x: torch.Tensor, conv: torch.nn.Conv2d, bias: Optional[torch.Tensor] = None,
            stride: int = 1, up: bool = False, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``conv2d(up2(x) if up else x, conv.weight, bias, stride, padding=1) (+ residual)``."""
    if _CONV != "torch" and _native(x):
        from k8s_nvidia_gpus_amd.ops import gemm_epi as GE

        if GE.conv3x3_supported(x, conv.out_channels) and stride in (1, 2) and not (up and stride != 1) \
                and (residual is None or (residual.dtype == x.dtype and residual.is_contiguous(
                    memory_format=torch.channels_last))):
            mode = GE.CONV_UP2 if up else (GE.CONV_S2 if stride == 2 else GE.CONV_S1)
            return GE.conv3x3(x, _conv_weight(conv, x.dtype), bias, mode, residual)
    if up:
        x = F.interpolate(x, scale_factor=2.0, mode="nearest")
        if x.device.type == "cuda":
            x = x.contiguous(memory_format=torch.channels_last)
    y = F.conv2d(x, conv.weight, bias, stride=stride, padding=1)
    return y if residual is None else add3(residual, y, None)


def conv1x1(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """1×1 convolution of a channels-last NCHW tensor as a token-row GEMM (no copies)."""
    n, c, h, wd = x.shape
    if _native(x) and x.is_contiguous(memory_format=torch.channels_last):
        rows = x.permute(0, 2, 3, 1).reshape(-1, c)
        out = linear(rows, w.view(w.shape[0], c), bias)
        return out.view(n, h, wd, -1).permute(0, 3, 1, 2)
    return F.conv2d(x, w, bias)


# ---------------------------------------------------------------- GroupNorm (+SiLU)
def group_norm_ref(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, groups: int,
                   eps: float, silu: bool = False, add: Optional[torch.Tensor] = None) -> torch.Tensor:
    xf = x.float()
    if add is not None:
        xf = xf + (add.float()[:, :, None, None] if x.dim() == 4 else add.float()[:, None, :])
    y = F.group_norm(xf, groups, weight.float(), bias.float(), eps).to(x.dtype)
    return F.silu(y) if silu else y


def group_norm(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, groups: int,
               eps: float, silu: bool = False, add: Optional[torch.Tensor] = None) -> torch.Tensor:
    """GroupNorm of ``x (+ add[n, c])`` over a 4-D NCHW-shaped tensor (channels-last memory on the
    GPU path); ``add`` is the ResNet block's time-embedding + conv-bias addend."""
    if _native(x) and _sd().group_norm_supported(x.shape[1] if x.dim() == 4 else x.shape[-1],
                                                 groups):
        return _sd().group_norm_nhwc(x, weight, bias, groups, eps, silu, add)
    return group_norm_ref(x, weight, bias, groups, eps, silu, add)


def add3(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``a + b + bias[c]`` (NCHW-shaped): residual add with the convolution bias folded in."""
    if _native(a) and a.shape == b.shape and a.shape[1] % 8 == 0:
        return _sd().add3(a, b, bias)
    out = a + b
    return out + bias[:, None, None] if bias is not None else out


# ---------------------------------------------------------------- (residual add +) LayerNorm
def add_layernorm(x: torch.Tensor, delta: Optional[torch.Tensor], weight: torch.Tensor,
                  bias: torch.Tensor, eps: float):
    """``LN(x)`` or, with ``delta``, ``(x + delta, LN(x + delta))`` — the transformer block's
    residual add fused in front of the next LayerNorm."""
    if _native(x) and _sd().layernorm_supported(x.shape[-1]):
        return _sd().add_layernorm(x, delta, weight, bias, eps)
    xs = x if delta is None else x + delta
    y = F.layer_norm(xs, (x.shape[-1],), weight, bias, eps)
    return y if delta is None else (xs, y)


# ---------------------------------------------------------------- attention
def attention_ref(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int,
                  scale: Optional[float] = None) -> torch.Tensor:
    n, lq, c = q.shape
    lk = k.shape[1]
    d = c // heads
    qh = q.reshape(n, lq, heads, d).transpose(1, 2)
    kh = k.reshape(n, lk, heads, d).transpose(1, 2)
    vh = v.reshape(n, lk, heads, d).transpose(1, 2)
    o = F.scaled_dot_product_attention(qh, kh, vh, scale=scale)
    return o.transpose(1, 2).reshape(n, lq, c)


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int,
              scale: Optional[float] = None) -> torch.Tensor:
    """``[N, Lq, H*d]`` × ``[N, Lk, H*d]`` → ``[N, Lq, H*d]`` (no mask, SD's attention)."""
    d = q.shape[-1] // heads
    if scale is None:
        scale = 1.0 / math.sqrt(d)
    if _native(q) and _sd().attention_supported(q, k, v, heads):
        return _sd().attention(q, k, v, heads, scale)
    return attention_ref(q, k, v, heads, scale)


# ---------------------------------------------------------------- GEGLU
def geglu_ref(x: torch.Tensor) -> torch.Tensor:
    h, g = x.chunk(2, dim=-1)
    return h * F.gelu(g)


def geglu(x: torch.Tensor) -> torch.Tensor:
    if _native(x):
        return _sd().geglu(x)
    return geglu_ref(x)

"""ctypes bindings of the SD1.5 hot-op kernels (``csrc/sd_norm.hip``, ``csrc/sd_attention.hip``).

Same conventions as ``kernels.py``: raw device pointers, torch's current stream (so the kernels are
captured by ``torch.cuda.graph``), no fallback when the library is missing on a GPU machine.
Shapes a kernel does not cover are reported by the ``*_supported`` predicates; the model's dispatch
(``models/sd15/functional.py``) routes only those to PyTorch.
"""
from __future__ import annotations

import ctypes
import threading

import torch

from .kernels import library

_DTYPE = {torch.float16: 0, torch.bfloat16: 1}
_declared = False
_lock = threading.Lock()


def _lib():
    global _declared
    lib = library()
    if not _declared:
        with _lock:
            vp, ci, cl, cf = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float
            lib.amdk8s_groupnorm_supported.argtypes = [ci, ci]
            lib.amdk8s_groupnorm_supported.restype = ci
            lib.amdk8s_groupnorm_set_fused.argtypes = [ci]
            lib.amdk8s_groupnorm_set_fused.restype = None
            lib.amdk8s_groupnorm_workspace.argtypes = [ci, ci, ci, ci]
            lib.amdk8s_groupnorm_workspace.restype = cl
            lib.amdk8s_groupnorm_nhwc.argtypes = [vp, vp, cl, vp, vp, vp, vp, ci, ci, ci, ci, cf,
                                                  ci, ci, vp]
            lib.amdk8s_groupnorm_nhwc.restype = ci
            lib.amdk8s_geglu.argtypes = [vp, vp, cl, ci, ci, vp]
            lib.amdk8s_geglu.restype = ci
            lib.amdk8s_add3.argtypes = [vp, vp, vp, vp, cl, ci, ci, vp]
            lib.amdk8s_add3.restype = ci
            lib.amdk8s_add_layernorm.argtypes = [vp, vp, vp, vp, vp, vp, cl, ci, cf, ci, vp]
            lib.amdk8s_add_layernorm.restype = ci
            if hasattr(lib, "amdk8s_attention_fwd"):
                lib.amdk8s_attention_supported.argtypes = [ci, ci, ci]
                lib.amdk8s_attention_supported.restype = ci
                lib.amdk8s_attention_fwd.argtypes = [vp, vp, vp, vp, ci, ci, ci, ci, ci, ci, ci, ci,
                                                     ci, ci, ci, ci, cf, ci, vp]
                lib.amdk8s_attention_fwd.restype = ci
            _declared = True
    return lib


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc})")


def group_norm_supported(c: int, groups: int) -> bool:
    return bool(_lib().amdk8s_groupnorm_supported(c, groups))


def set_group_norm_fused(v: int) -> None:
    """1: the single-launch GroupNorm where it pays (small images), 2: for every supported shape
    (tests), 0: always the two-launch form, -1: AMDK8S_GN_FUSED (default on)."""
    _lib().amdk8s_groupnorm_set_fused(int(v))


def group_norm_nhwc(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, groups: int,
                    eps: float, silu: bool = False, add: torch.Tensor = None) -> torch.Tensor:
    """GroupNorm(+SiLU) of ``x + add[n, c]`` (``x`` [N, C, H, W] channels-last or [N, L, C] rows;
    ``add`` an optional [N, C] per-image channel addend, any row stride)."""
    if x.dtype not in _DTYPE:
        raise TypeError(f"group_norm_nhwc: {x.dtype} (fp16/bf16 only)")
    lib = _lib()
    if x.dim() == 4:
        n, c, h, w = x.shape
        hw = h * w
        x = x.contiguous(memory_format=torch.channels_last)
        y = torch.empty_like(x, memory_format=torch.channels_last)
    elif x.dim() == 3:
        n, hw, c = x.shape
        x = x.contiguous()
        y = torch.empty_like(x)
    else:
        raise ValueError("group_norm_nhwc: 3-D or 4-D input")
    if not lib.amdk8s_groupnorm_supported(c, groups):
        raise ValueError(f"group_norm_nhwc: C={c}, groups={groups} not supported")
    w = weight.to(x.dtype).contiguous()
    b = bias.to(x.dtype).contiguous()
    ws = torch.empty(lib.amdk8s_groupnorm_workspace(n, hw, c, groups), dtype=torch.float32,
                     device=x.device)
    add_ptr, add_stride = None, 0
    if add is not None:
        if add.shape != (n, c) or add.stride(1) != 1:
            raise ValueError(f"group_norm_nhwc: addend must be [N, C] with unit column stride")
        add = add.to(x.dtype)
        if add.data_ptr() % 16 or add.stride(0) % 8:   # the kernels read 8-channel vectors
            add = add.contiguous()
        add_ptr, add_stride = add.data_ptr(), add.stride(0)
    rc = lib.amdk8s_groupnorm_nhwc(x.data_ptr(), add_ptr, add_stride, y.data_ptr(), w.data_ptr(),
                                   b.data_ptr(),
                                   ws.data_ptr(), n, hw, c, groups,
                                   float(eps), int(silu), _DTYPE[x.dtype], _stream(x))
    _check(rc, "amdk8s_groupnorm_nhwc")
    return y


def geglu(x: torch.Tensor) -> torch.Tensor:
    """``h * gelu(g)`` for ``x = [h | g]`` along the last dim."""
    if x.dtype not in _DTYPE:
        raise TypeError(f"geglu: {x.dtype} (fp16/bf16 only)")
    x = x.contiguous()
    d2 = x.shape[-1]
    d = d2 // 2
    m = x.numel() // d2
    out = torch.empty(x.shape[:-1] + (d,), dtype=x.dtype, device=x.device)
    _check(_lib().amdk8s_geglu(x.data_ptr(), out.data_ptr(), m, d, _DTYPE[x.dtype], _stream(x)),
           "amdk8s_geglu")
    return out


def add3(a: torch.Tensor, b: torch.Tensor, bias: torch.Tensor = None) -> torch.Tensor:
    """``a + b + bias[c]`` over channels-last [N, C, H, W] (or [..., C]) tensors of one dtype."""
    if a.dtype not in _DTYPE or b.dtype != a.dtype:
        raise TypeError("add3: fp16/bf16 operands of one dtype")
    fmt = torch.channels_last if a.dim() == 4 else torch.contiguous_format
    a = a.contiguous(memory_format=fmt)
    b = b.contiguous(memory_format=fmt)
    c = a.shape[1] if a.dim() == 4 else a.shape[-1]
    out = torch.empty_like(a, memory_format=fmt)
    bias_ptr = None
    if bias is not None:
        bias = bias.to(a.dtype).contiguous()
        bias_ptr = bias.data_ptr()
    _check(_lib().amdk8s_add3(a.data_ptr(), b.data_ptr(), bias_ptr, out.data_ptr(),
                              a.numel() // c, c, _DTYPE[a.dtype], _stream(a)), "amdk8s_add3")
    return out


def add_layernorm(x: torch.Tensor, delta, weight: torch.Tensor, bias: torch.Tensor,
                  eps: float):
    """LayerNorm over the last dim of ``x (+ delta)``.  Returns ``y`` (no delta) or ``(x + delta, y)``."""
    if x.dtype not in _DTYPE:
        raise TypeError(f"add_layernorm: {x.dtype} (fp16/bf16 only)")
    x = x.contiguous()
    c = x.shape[-1]
    y = torch.empty_like(x)
    xs = None
    dptr = sptr = None
    if delta is not None:
        delta = delta.contiguous()
        if delta.shape != x.shape or delta.dtype != x.dtype:
            raise ValueError("add_layernorm: delta must match x")
        xs = torch.empty_like(x)
        dptr, sptr = delta.data_ptr(), xs.data_ptr()
    w = weight.to(x.dtype).contiguous()
    b = bias.to(x.dtype).contiguous()
    _check(_lib().amdk8s_add_layernorm(x.data_ptr(), dptr, sptr, y.data_ptr(), w.data_ptr(),
                                       b.data_ptr(), x.numel() // c, c, float(eps),
                                       _DTYPE[x.dtype], _stream(x)), "amdk8s_add_layernorm")
    return y if delta is None else (xs, y)


def layernorm_supported(c: int) -> bool:
    return c % 8 == 0 and c // 8 <= 256


def attention_set_qt(qt: int) -> None:
    """Force the query tiles per wave of the attention kernel (0 = heuristic; 1 / 2 / 4) — for
    tuning sweeps (tools/attn_probe.py)."""
    lib = _lib()
    lib.amdk8s_attention_set_qt.argtypes = [ctypes.c_int]
    lib.amdk8s_attention_set_qt.restype = None
    lib.amdk8s_attention_set_qt(int(qt))


def attention_set_variant(v: int) -> None:
    """-1 = auto (default: head dims 40 / 64 / 80 / 128 / 160 → the 32x32x16 kernel of
    ``csrc/attn_d128.hip``, any other → the transposed-score kernel), 0 = transposed-score kernel
    (P stays in registers), 1 = P staged through LDS, 2 = the 32x32x16 kernel."""
    lib = _lib()
    lib.amdk8s_attention_set_variant.argtypes = [ctypes.c_int]
    lib.amdk8s_attention_set_variant.restype = None
    lib.amdk8s_attention_set_variant(int(v))


def attention_d128_set_nw(nw: int) -> None:
    """Waves per workgroup of the 32x32x16 kernel (0 = heuristic, 4 or 8) — for tuning sweeps."""
    lib = _lib()
    lib.amdk8s_attention_d128_set_nw.argtypes = [ctypes.c_int]
    lib.amdk8s_attention_d128_set_nw.restype = None
    lib.amdk8s_attention_d128_set_nw(int(nw))


def attention_supported(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int) -> bool:
    lib = _lib()
    if not hasattr(lib, "amdk8s_attention_fwd") or q.dtype not in _DTYPE:
        return False
    if q.stride(-1) != 1 or k.stride(-1) != 1 or v.stride(-1) != 1:
        return False
    d = q.shape[-1] // heads
    return bool(lib.amdk8s_attention_supported(d, q.shape[1], k.shape[1]))


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int,
              scale: float) -> torch.Tensor:
    """softmax(q kᵀ · scale) v per head; q/k/v ``[N, L, H*d]`` with unit inner stride."""
    n, lq, c = q.shape
    lk = k.shape[1]
    d = c // heads
    o = torch.empty((n, lq, c), dtype=q.dtype, device=q.device)
    rc = _lib().amdk8s_attention_fwd(
        q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), n, heads, lq, lk, d,
        q.stride(0), q.stride(1), k.stride(0), k.stride(1), v.stride(0), v.stride(1), o.stride(1),
        float(scale), _DTYPE[q.dtype], _stream(q))
    _check(rc, "amdk8s_attention_fwd")
    return o


def attention_causal(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, heads: int,
                     scale: float) -> torch.Tensor:
    """Causal self-attention (query i sees keys 0 .. i) per head on the 32x32x16 flash kernel
    (``csrc/attn_d128.hip``, head dims 40 / 64 / 80 / 128 / 160); q/k/v ``[N, L, H*d]`` with unit
    inner stride (any row / batch stride), fp16 or bf16.  The CLIP text encoder's attention."""
    n, L, c = q.shape
    d = c // heads
    lib = _lib()
    if not getattr(lib, "_causal_declared", False):
        ci, vp = ctypes.c_int, ctypes.c_void_p
        lib.amdk8s_attention_causal_fwd.argtypes = [vp, vp, vp, vp] + [ci] * 11 + \
            [ctypes.c_float, ci, vp]
        lib.amdk8s_attention_causal_fwd.restype = ci
        lib._causal_declared = True
    if q.dtype not in _DTYPE or k.shape != q.shape or v.shape != q.shape or c % heads:
        raise ValueError(f"attention_causal: q/k/v {tuple(q.shape)} {q.dtype}")
    if q.stride(-1) != 1 or k.stride(-1) != 1 or v.stride(-1) != 1:
        raise ValueError("attention_causal: unit inner stride required")
    o = torch.empty((n, L, c), dtype=q.dtype, device=q.device)
    rc = lib.amdk8s_attention_causal_fwd(
        q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), n, heads, L, d,
        q.stride(0), q.stride(1), k.stride(0), k.stride(1), v.stride(0), v.stride(1), o.stride(1),
        float(scale), _DTYPE[q.dtype], _stream(q))
    _check(rc, "amdk8s_attention_causal_fwd")
    return o

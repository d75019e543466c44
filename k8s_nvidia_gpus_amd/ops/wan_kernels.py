"""ctypes bindings of the Wan2.1 DiT row kernels (``csrc/wan_ops.hip``).

Same conventions as ``sd_kernels.py``: raw device pointers, torch's current stream, no fallback
when the library is missing on a GPU machine; ``*_supported`` predicates report what the kernels
cover and ``models/wan/functional.py`` routes only the rest to PyTorch.
"""
from __future__ import annotations

import ctypes
import threading
from typing import Optional, Tuple

import torch

from .kernels import library

_declared = False
_lock = threading.Lock()


def _lib():
    global _declared
    lib = library()
    if not _declared:
        with _lock:
            vp, ci, cl, cf = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float
            lib.amdk8s_wan_row_supported.argtypes = [ci]
            lib.amdk8s_wan_row_supported.restype = ci
            lib.amdk8s_wan_rms_supported.argtypes = [ci, ci]
            lib.amdk8s_wan_rms_supported.restype = ci
            lib.amdk8s_wan_add_ln.argtypes = [vp, vp, cl, vp, cl, vp, cl, vp, cl, vp, cl, ci, ci,
                                              cf, vp]
            lib.amdk8s_wan_add_ln.restype = ci
            lib.amdk8s_wan_rmsnorm_rope.argtypes = [vp, cl, vp, vp, vp, cl, ci, ci, ci, ci, cf, vp]
            lib.amdk8s_wan_rmsnorm_rope.restype = ci
            lib.amdk8s_wan_vae_supported.argtypes = [ci]
            lib.amdk8s_wan_vae_supported.restype = ci
            lib.amdk8s_wan_vae_rms_silu_stack.argtypes = [vp, vp, vp, cl, ci, ci, ci, ci, vp]
            lib.amdk8s_wan_vae_rms_silu_stack.restype = ci
            _declared = True
    return lib


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc})")


def add_ln_supported(c: int) -> bool:
    return bool(_lib().amdk8s_wan_row_supported(c))


def _row_vec(t: torch.Tensor, c: int) -> Tuple[torch.Tensor, int]:
    """fp32 [B, C] / [1, C] (any batch stride, unit inner stride, 16-byte aligned rows)."""
    if t.dtype != torch.float32 or t.stride(-1) != 1 or t.shape[-1] != c:
        t = t.float().contiguous()
    sb = t.stride(0) if t.shape[0] > 1 else 0
    if t.data_ptr() % 16 or sb % 4:
        t = t.contiguous()
        sb = c if t.shape[0] > 1 else 0
    return t, sb


def add_ln(x: torch.Tensor, y: Optional[torch.Tensor], gate: Optional[torch.Tensor],
           mul: torch.Tensor, add: torch.Tensor, eps: float,
           out_dtype: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """``x += y·gate`` (in place, fp32 [B, L, C] contiguous) then ``LN(x)·mul + add`` → bf16."""
    if x.dtype != torch.float32 or not x.is_contiguous():
        raise TypeError("add_ln: x must be a contiguous fp32 residual stream")
    if out_dtype != torch.bfloat16:
        raise TypeError("add_ln: bf16 output only")
    b, l, c = x.shape
    if y is not None:
        if y.dtype != torch.bfloat16 or y.stride(-1) != 1 or y.shape != x.shape:
            y = y.to(torch.bfloat16).contiguous()
        if (b > 1 and y.stride(0) != l * y.stride(1)) or y.stride(1) % 8 or y.data_ptr() % 16:
            y = y.contiguous()
    g_ptr, sg = None, 0
    if y is not None and gate is not None:
        gate, sg = _row_vec(gate, c)          # the local name keeps a converted copy alive
        g_ptr = gate.data_ptr()
    mul, sm = _row_vec(mul, c)
    add, sa = _row_vec(add, c)
    out = torch.empty((b, l, c), dtype=torch.bfloat16, device=x.device)
    rc = _lib().amdk8s_wan_add_ln(x.data_ptr(), y.data_ptr() if y is not None else None,
                                  y.stride(1) if y is not None else 0, g_ptr, sg, mul.data_ptr(), sm,
                                  add.data_ptr(), sa, out.data_ptr(), b * l, l, c, float(eps),
                                  _stream(x))
    _check(rc, "amdk8s_wan_add_ln")
    return out


def rmsnorm_rope_supported(t: torch.Tensor, heads: int) -> bool:
    c = t.shape[-1]
    if t.dtype != torch.bfloat16 or t.stride(-1) != 1 or c % heads:
        return False
    b, l, _ = t.shape
    if b > 1 and t.stride(0) != l * t.stride(1):
        return False
    if t.stride(1) % 8 or t.data_ptr() % 16:
        return False
    return bool(_lib().amdk8s_wan_rms_supported(c, c // heads))


def _weight32(*ws: torch.Tensor) -> torch.Tensor:
    """fp32 copy of the norm weight(s), cached on the first weight tensor itself (lives and dies
    with the model; keyed by the partner weight's identity and both versions)."""
    key = tuple((id(w), w._version) for w in ws)
    cached = getattr(ws[0], "_amdk8s_w32", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    t = torch.cat([w.detach().float().reshape(-1) for w in ws]).contiguous()
    ws[0]._amdk8s_w32 = (key, t)
    return t


def rmsnorm_rope(t: torch.Tensor, w: torch.Tensor, cos: Optional[torch.Tensor],
                 sin: Optional[torch.Tensor], heads: int, eps: float,
                 w2: Optional[torch.Tensor] = None) -> torch.Tensor:
    """In place: RMSNorm (weight ``w``) + optional RoPE on ``t`` [B, L, C] (strided rows); with
    ``w2`` the same is applied to the next C columns (the k slice after q) in the same launch."""
    b, l, c = t.shape
    nsec = 2 if w2 is not None else 1
    w32 = _weight32(w, w2) if w2 is not None else _weight32(w)
    if cos is not None:
        cos = cos.float().contiguous()
        sin = sin.float().contiguous()
        if cos.shape != (l, c // heads // 2):
            raise ValueError(f"rope table {tuple(cos.shape)} != ({l}, {c // heads // 2})")
    rc = _lib().amdk8s_wan_rmsnorm_rope(t.data_ptr(), t.stride(1), w32.data_ptr(),
                                        cos.data_ptr() if cos is not None else None,
                                        sin.data_ptr() if sin is not None else None, b * l, l, c,
                                        c // heads, nsec, float(eps), _stream(t))
    _check(rc, "amdk8s_wan_rmsnorm_rope")
    return t


def vae_rms_silu_supported(x: torch.Tensor) -> bool:
    return (x.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last)
            and bool(_lib().amdk8s_wan_vae_supported(x.shape[1])))


def vae_rms_silu_stack(x: torch.Tensor, gamma: torch.Tensor, frames: int, kt: int = 3) -> torch.Tensor:
    """``silu(RMS_norm(x))`` of channels-last frames ``x`` [B·T, C, H, W]; with ``kt = 3`` the
    result is written as the temporal-tap-stacked [B·T, 3C, H, W] input of a causal 3×3×3 conv."""
    n, c, h, w = x.shape
    g32 = _weight32(gamma.reshape(-1))
    out = torch.empty((n, kt * c, h, w), dtype=x.dtype, device=x.device,
                      memory_format=torch.channels_last)
    rc = _lib().amdk8s_wan_vae_rms_silu_stack(x.data_ptr(), g32.data_ptr(), out.data_ptr(), n * h * w,
                                              h * w, frames, c, kt, _stream(x))
    _check(rc, "amdk8s_wan_vae_rms_silu_stack")
    return out

"""ctypes bindings of the fused-epilogue GEMMs (``csrc/gemm_bf16_epi.hip``, and the w4a 256×256
kernel's epilogue variants in ``csrc/gemm_bf16_gfx950_w4a.hip``).

``linear(x, w, b)`` / ``linear_gelu(x, w, b)`` are ``F.linear`` (+ tanh-GELU) on hand-written
gfx950 kernels (bf16 or fp16 operands): the wave-grid family (256×128 … 64×64 tiles, picked by
problem size) or, for wide projections, the 256×256 w4a kernel; ``linear_residual_(res, x, w, b, gate)`` folds the
DiT's gated residual update ``res += gate · (x·wᵀ + b)`` into the GEMM's epilogue, so the
projection output never round-trips through HBM in bf16.  Same conventions as the other binding
modules: raw device pointers, torch's current stream, ``supported(...)`` predicates for what the
kernel covers (N % 8, K % 64), and no silent fallback once a caller has chosen the kernel.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch

from .kernels import library

EPI_STORE, EPI_GELU, EPI_RESID, EPI_ADD = 0, 1, 2, 3
CONV_S1, CONV_S2, CONV_UP2 = 1, 2, 3
_declared = False
_lock = threading.Lock()


def _lib():
    global _declared
    lib = library()
    if not _declared:
        with _lock:
            vp, ci = ctypes.c_void_p, ctypes.c_int
            lib.amdk8s_gemm_epi_supported.argtypes = [ci, ci, ci]
            lib.amdk8s_gemm_epi_supported.restype = ci
            lib.amdk8s_gemm_epi.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, vp, ci, ci, ci, ci, ci,
                                            ci, ci, ci, ci, ci, vp, vp]
            lib.amdk8s_conv3x3_epi.argtypes = [ci, ci, vp, vp, vp, vp, vp, ci, ci, ci, ci, ci, ci,
                                               ci, vp, vp]
            lib.amdk8s_gemm_epi_splits.argtypes = [ci, ci, ci]
            lib.amdk8s_gemm_epi_splits.restype = ci
            lib.amdk8s_conv3x3_epi.restype = ci
            lib.amdk8s_gemm_epi.restype = ci
            lib.amdk8s_gemm_w4a_epi.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, ci, ci, ci, ci, ci, ci,
                                                ci, ci, ci, vp]
            lib.amdk8s_gemm_w4a_epi.restype = ci
            lib.amdk8s_gemm_w4a_hybrid_plan.argtypes = [ci, ci, ci, ci, ctypes.POINTER(ci),
                                                         ctypes.POINTER(ci)]
            lib.amdk8s_gemm_w4a_hybrid_plan.restype = None
            lib.amdk8s_gemm_w4a_hybrid.argtypes = [ci, ci, vp, vp, vp, vp, ci, ci, ci, ci, ci, ci,
                                                   ci, ci, vp, ctypes.c_long, vp]
            lib.amdk8s_gemm_w4a_hybrid.restype = ci
            lib.amdk8s_gemm_w4a_splitk_set_ks.argtypes = [ci]
            lib.amdk8s_gemm_w4a_splitk_set_ks.restype = None
            lib.amdk8s_gemm_w4a_splitk_plan.argtypes = [ci, ci, ci, ci, ctypes.POINTER(ci)]
            lib.amdk8s_gemm_w4a_splitk_plan.restype = None
            lib.amdk8s_gemm_w4a_splitk.argtypes = [ci, ci, vp, vp, vp, vp, vp, ci, ci, ci, ci, ci,
                                                   ci, ci, ci, vp, ctypes.c_long, vp,
                                                   ctypes.c_float, vp, ci, vp]
            lib.amdk8s_gemm_w4a_splitk.restype = ci
            lib.amdk8s_gemm_epi_set_tile.argtypes = [ci]
            lib.amdk8s_gemm_epi_set_tile.restype = None
            lib.amdk8s_gemm_epi_set_splits.argtypes = [ci]
            lib.amdk8s_gemm_epi_set_splits.restype = None
            lib.amdk8s_gemm_epi_plan.argtypes = [ci, ci, ci, ctypes.POINTER(ci), ctypes.POINTER(ci)]
            lib.amdk8s_gemm_epi_plan.restype = None
            _declared = True
    return lib


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


TILES = ((256, 128), (128, 128), (128, 64), (64, 64))


_PINS = {"tile": -1, "splits": -1}


def set_tile(tile: int) -> None:
    """Pin the wave-grid kernel family's block tile (index into TILES); -1 = the planner.  A pin
    also keeps shapes off the split-K w4a form, so the pinned kernel is the one that runs."""
    _PINS["tile"] = int(tile)
    _lib().amdk8s_gemm_epi_set_tile(int(tile))


def set_splits(s: int) -> None:
    """Pin the split-K factor (1 = never split); -1 = the planner."""
    _PINS["splits"] = int(s)
    _lib().amdk8s_gemm_epi_set_splits(int(s))


def plan(m: int, n: int, k: int) -> tuple:
    """(block tile, split-K factor) the kernels use for an m × n × k problem."""
    t, sp = ctypes.c_int(), ctypes.c_int()
    _lib().amdk8s_gemm_epi_plan(m, n, k, ctypes.byref(t), ctypes.byref(sp))
    return TILES[t.value], sp.value


def _rows(x: torch.Tensor) -> torch.Tensor:
    """[.., K] → a 2-D [M, K] view with unit inner stride and 16-B aligned rows (copy if needed)."""
    x2 = x.reshape(-1, x.shape[-1])
    if x2.stride(-1) != 1 or x2.stride(0) % 8 or x2.data_ptr() % 16:
        x2 = x2.contiguous()
    return x2


_DT = {torch.bfloat16: 1, torch.float16: 0}


def supported(x: torch.Tensor, w: torch.Tensor) -> bool:
    if x.device.type != "cuda" or x.dtype not in _DT or w.dtype != x.dtype:
        return False
    n, k = w.shape
    if x.shape[-1] != k or w.stride(-1) != 1 or w.stride(0) % 8 or w.data_ptr() % 16:
        return False
    m = x.numel() // k
    return m > 0 and bool(_lib().amdk8s_gemm_epi_supported(m, n, k))


def _bias(b: Optional[torch.Tensor], n: int, dtype: torch.dtype) -> Optional[torch.Tensor]:
    if b is None:
        return None
    if b.dtype != dtype or not b.is_contiguous() or b.numel() != n or b.data_ptr() % 16:
        b = b.to(dtype).contiguous().clone()
    return b


def _ptr(t: Optional[torch.Tensor]):
    return t.data_ptr() if t is not None else None


def splits(m: int, n: int, k: int) -> int:
    """Split-K factor the kernels use for an m × n × k problem (1 = none)."""
    return plan(m, n, k)[1]


def _workspace(epi: int, m: int, n: int, k: int, dev) -> Optional[torch.Tensor]:
    sp = splits(m, n, k)
    if sp <= 1:
        return None
    return torch.empty(sp * m * n, dtype=torch.float32, device=dev)


def _run(epi, x2, w, b, out, res, gate, rows_per_gate, gate_stride, ldo, ldx, r=None, ldr=0):
    m, k = x2.shape
    n = w.shape[0]
    ws = _workspace(epi, m, n, k, x2.device)
    rc = _lib().amdk8s_gemm_epi(
        epi, _DT[x2.dtype], x2.data_ptr(), w.data_ptr(), _ptr(b), _ptr(out), _ptr(res), _ptr(gate),
        _ptr(r), m, n, k, x2.stride(0), w.stride(0), ldo, ldx, ldr, rows_per_gate, gate_stride,
        _ptr(ws), _stream(x2))
    if rc != 0:
        raise RuntimeError(f"amdk8s_gemm_epi failed (rc={rc}, M={m} N={n} K={k}, epi={epi})")


# Wide projections (N % 256 == 0, enough 256×256 tiles to fill the chip) run on the validator's
# 256x256 kernel (w4a: generated-assembly K-loop) with its bias / GELU / gated-residual store
# epilogue; everything else on the wave-grid kernel family above.  AMDK8S_GEMM_WIDE=epi forces the
# latter (A/B runs).
_WIDE = os.environ.get("AMDK8S_GEMM_WIDE", "w4a")


def use_w4a(m: int, n: int, k: int, dtype: torch.dtype) -> bool:
    """256×256 tiles whenever they fill at least 3/4 of the chip: the LLM prefill's q|k|v and o_proj
    at 3584 tokens (252 / 196 tiles) ran 136 / 137 us on the wave-grid family against hipBLASLt's
    90 / 75 (profiles/r05/prefill_gemm_3584.log)."""
    return (_WIDE == "w4a" and dtype in _DT and n % 256 == 0 and k % 64 == 0
            and ((m + 255) // 256) * (n // 256) >= 192)


def _w4a(epi: int, x2: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor],
         out: Optional[torch.Tensor], res: Optional[torch.Tensor] = None,
         gate: Optional[torch.Tensor] = None, rows_per_gate: int = 0, gate_stride: int = 0) -> None:
    """epi: 0 store, 1 + bias, 2 gelu(+ bias), 3 residual (``res`` fp32, optional gate)."""
    m, k = x2.shape
    n = w.shape[0]
    rc = _lib().amdk8s_gemm_w4a_epi(
        epi, _DT[x2.dtype], x2.data_ptr(), w.data_ptr(), out.data_ptr() if out is not None else None,
        b.data_ptr() if b is not None else None, res.data_ptr() if res is not None else None,
        gate.data_ptr() if gate is not None else None, m, n, k, x2.stride(0), w.stride(0),
        out.stride(0) if out is not None else 0, n, rows_per_gate, gate_stride, _stream(x2))
    if rc != 0:
        raise RuntimeError(f"amdk8s_gemm_w4a_epi failed (rc={rc}, M={m} N={n} K={k}, epi={epi})")


# A 256×256 grid that fills the chip 1 < waves < 2 times runs its partial last wave split over K on
# the otherwise idle CUs (amdk8s_gemm_w4a_hybrid); AMDK8S_GEMM_HYBRID=0 turns it off (A/B runs).
_HYBRID = os.environ.get("AMDK8S_GEMM_HYBRID", "1") != "0"
_CUS = {}


def _cus(dev) -> int:
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _CUS:
        _CUS[i] = torch.cuda.get_device_properties(i).multi_processor_count
    return _CUS[i]


def hybrid_plan(m: int, n: int, k: int, cus: int = 256) -> tuple:
    """(whole-wave columns na, K slices of the rest): ks == 1 means the plain w4a launch."""
    na, ks = ctypes.c_int(), ctypes.c_int()
    _lib().amdk8s_gemm_w4a_hybrid_plan(m, n, k, cus, ctypes.byref(na), ctypes.byref(ks))
    return na.value, ks.value


def _w4a_hybrid(epi: int, x2, w, b, out) -> bool:
    """The hybrid for store / bias / SwiGLU epilogues; False when its plan is the plain launch.
    fp16 only: its K slices meet as 16-bit partial tiles (the K-loop's C image in LDS is 16-bit),
    and 8 roundings at bf16's 8 mantissa bits would cost visible accuracy."""
    if not _HYBRID or epi not in (0, 1, EPI_W4A_SWIGLU) or x2.dtype != torch.float16:
        return False
    m, k = x2.shape
    n = w.shape[0]
    na, ks = hybrid_plan(m, n, k, _cus(x2.device))
    if ks <= 1:
        return False
    ws = torch.empty(ks * m * (n - na), dtype=x2.dtype, device=x2.device)
    rc = _lib().amdk8s_gemm_w4a_hybrid(
        epi, _DT[x2.dtype], x2.data_ptr(), w.data_ptr(), out.data_ptr(),
        b.data_ptr() if b is not None else None, m, n, k, x2.stride(0), w.stride(0),
        out.stride(0), na, ks, ws.data_ptr(), ws.numel(), _stream(x2))
    if rc != 0:
        raise RuntimeError(f"amdk8s_gemm_w4a_hybrid failed (rc={rc}, M={m} N={n} K={k})")
    return True


def _aligned16(*ts) -> bool:
    return all(t is None or t.data_ptr() % 16 == 0 for t in ts)


# A 256×256 grid far below the chip (LLM prefill chunks: q|k|v, o_proj, ffn_down at 512 tokens)
# runs with every tile split over K (amdk8s_gemm_w4a_splitk; fp16 only, like the hybrid)
# instead of on the wave-grid family; AMDK8S_GEMM_W4A_SPLITK=0 turns it off (A/B runs).
_W4A_SPLITK = os.environ.get("AMDK8S_GEMM_W4A_SPLITK", "1") != "0"


def set_w4a_splitk(ks: int) -> None:
    """Pin the split-K w4a form's slice count (A/B sweeps; 0 = the planner)."""
    _lib().amdk8s_gemm_w4a_splitk_set_ks(int(ks))


def splitk_plan(m: int, n: int, k: int, cus: int = 256) -> int:
    """K slices per 256×256 tile of the split-K w4a form (1: not used for this shape)."""
    ks = ctypes.c_int()
    _lib().amdk8s_gemm_w4a_splitk_plan(m, n, k, cus, ctypes.byref(ks))
    return ks.value


def _w4a_splitk(epi: int, x2, w, b, out=None, res=None, norm=None) -> bool:
    """The split-K w4a form with epilogue ``epi`` (0 store, 1 + bias, 3 += res fp32, 4 SwiGLU);
    False when it does not apply (dtype, layout, or the planner keeps the shape elsewhere).
    ``norm`` (epi 3): (weight fp32 [N], eps, y fp16 [M, N]) — y = RMSNorm of the updated rows."""
    if (not _W4A_SPLITK or _WIDE != "w4a" or x2.dtype != torch.float16 or w.dtype != x2.dtype
            or _PINS["tile"] >= 0 or _PINS["splits"] >= 0):
        return False
    m, k = x2.shape
    n = w.shape[0]
    if (w.stride(-1) != 1 or w.stride(0) % 8 or x2.stride(0) % 8
            or not _aligned16(x2, w, b, out, res)):
        return False
    if out is not None and (out.stride(-1) != 1 or out.stride(0) % 8):
        return False
    nw, eps, y = norm if norm is not None else (None, 0.0, None)
    if norm is not None and (n > 8192 or nw.dtype != torch.float32 or not nw.is_contiguous()
                             or y.dtype != torch.float16 or y.stride(-1) != 1 or y.stride(0) % 8
                             or not _aligned16(nw, y)):
        return False
    ks = splitk_plan(m, n, k, _cus(x2.device))
    if ks <= 1:
        return False
    ws = torch.empty(ks * m * n, dtype=x2.dtype, device=x2.device)
    rc = _lib().amdk8s_gemm_w4a_splitk(
        epi, _DT[x2.dtype], x2.data_ptr(), w.data_ptr(), _ptr(out), _ptr(b), _ptr(res), m, n, k,
        x2.stride(0), w.stride(0), out.stride(0) if out is not None else 0, n, ks, ws.data_ptr(),
        ws.numel(), _ptr(nw), float(eps), _ptr(y), y.stride(0) if y is not None else 0,
        _stream(x2))
    if rc != 0:
        raise RuntimeError(f"amdk8s_gemm_w4a_splitk failed (rc={rc}, M={m} N={n} K={k}, epi={epi})")
    return True


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None,
           gelu: bool = False) -> torch.Tensor:
    """``x·wᵀ + b`` (tanh-GELU with ``gelu``) in x's dtype: ``x`` [..., K], ``w`` [N, K]."""
    x2 = _rows(x)
    n = w.shape[0]
    out = torch.empty((x2.shape[0], n), dtype=x.dtype, device=x.device)
    bb = _bias(b, n, x.dtype)
    if use_w4a(x2.shape[0], n, x2.shape[1], x.dtype) and _aligned16(x2, w, bb):
        if gelu and bb is None:
            bb = torch.zeros(n, dtype=x.dtype, device=x.device)
        epi = 2 if gelu else (0 if bb is None else 1)
        if not _w4a_hybrid(epi, x2, w, bb, out):
            _w4a(epi, x2, w, bb, out)
    elif gelu or not _w4a_splitk(0 if bb is None else 1, x2, w, bb, out):
        _run(EPI_GELU if gelu else EPI_STORE, x2, w, bb, out, None, None, 0, 0, n, 0)
    return out.view(*x.shape[:-1], n)


EPI_W4A_SWIGLU = 4


def linear_swiglu(x: torch.Tensor, w: torch.Tensor,
                  out: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """``silu(gate) · up`` of ``x·wᵀ`` in one GEMM: ``w`` [2F, K] holds gate|up rows interleaved
    in 128-row blocks (``llm_kernels.gate_up_interleave``), so every 256×256 tile carries matching
    gate and up columns and its epilogue writes its 256 × 128 share of the [M, F] result from
    LDS — the [M, 2F] product is never stored.  The arithmetic is the separate swiglu_f16 pass's on the
    16-bit products, so the bits match that path.  None when the shape is not on the 256×256
    kernel (the caller runs the GEMM and swiglu_f16 instead)."""
    x2 = _rows(x)
    m, k = x2.shape
    n = w.shape[0]
    if (x.dtype not in _DT or w.dtype != x.dtype or n % 256 or k % 64 or not _aligned16(x2, w)
            or w.stride(-1) != 1 or w.stride(0) % 8):
        return None
    if out is None:
        out = torch.empty((m, n // 2), dtype=x.dtype, device=x.device)
    elif out.shape != (m, n // 2) or out.stride(-1) != 1 or out.stride(0) % 8 or not _aligned16(out):
        raise ValueError(f"linear_swiglu: out {tuple(out.shape)} is not a [{m}, {n // 2}] row-major tensor")
    if use_w4a(m, n, k, x.dtype):
        if not _w4a_hybrid(EPI_W4A_SWIGLU, x2, w, None, out):
            _w4a(EPI_W4A_SWIGLU, x2, w, None, out)
        return out
    return out if _w4a_splitk(EPI_W4A_SWIGLU, x2, w, None, out) else None


def linear_gelu(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor] = None) -> torch.Tensor:
    return linear(x, w, b, gelu=True)


def linear_residual_(res: torch.Tensor, x: torch.Tensor, w: torch.Tensor,
                     b: Optional[torch.Tensor] = None, gate: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``res += gate · (x·wᵀ + b)`` in place.  ``res`` fp32 [B, L, N] contiguous, ``x`` [B, L, K],
    ``gate`` fp32 [B, N] (per sample, e.g. an AdaLN gate; any batch stride) or None."""
    if res.dtype != torch.float32 or not res.is_contiguous():
        raise TypeError("linear_residual_: res must be a contiguous fp32 tensor")
    n = w.shape[0]
    if res.shape[-1] != n or res.numel() != x.numel() // x.shape[-1] * n:
        raise ValueError(f"residual {tuple(res.shape)} does not match x {tuple(x.shape)} · w {tuple(w.shape)}")
    x2 = _rows(x)
    rows_per_gate, gstride = 0, 0
    if gate is not None:
        gate = gate.reshape(-1, n)
        if gate.dtype != torch.float32 or gate.stride(-1) != 1:
            gate = gate.float().contiguous()
        if gate.data_ptr() % 16 or (gate.shape[0] > 1 and gate.stride(0) % 4):
            gate = gate.contiguous()
        if x2.shape[0] % gate.shape[0]:
            raise ValueError("rows are not a whole number of gate rows")
        rows_per_gate = x2.shape[0] // gate.shape[0]
        gstride = gate.stride(0) if gate.shape[0] > 1 else 0
    bb = _bias(b, n, x.dtype)
    if use_w4a(x2.shape[0], n, x2.shape[1], x.dtype) and _aligned16(x2, w, bb, res, gate):
        _w4a(3, x2, w, bb, None, res, gate, rows_per_gate, gstride)
    elif gate is not None or not _w4a_splitk(3, x2, w, bb, None, res):
        _run(EPI_RESID, x2, w, bb, None, res, gate, rows_per_gate, gstride, 0, n)
    return res


def linear_residual_norm_(res: torch.Tensor, x: torch.Tensor, w: torch.Tensor,
                          norm_w: torch.Tensor, eps: float, y: torch.Tensor) -> bool:
    """``res += x·wᵀ`` and ``y = fp16(RMSNorm(res) · norm_w)`` in one GEMM + one finalize pass,
    when the shape runs on the split-K 256×256 form (the LLM prefill chunk's o_proj and
    ffn_down).  The bits are those of ``linear_residual_`` followed by the rmsnorm_f16 kernel.
    Returns False without doing anything when it does not apply (the caller runs the two)."""
    if res.dtype != torch.float32 or not res.is_contiguous() or res.shape[-1] != w.shape[0]:
        return False
    x2 = _rows(x)
    if res.numel() != x2.shape[0] * w.shape[0] or y.shape != res.shape:
        return False
    if use_w4a(x2.shape[0], w.shape[0], x2.shape[1], x.dtype):
        return False
    return _w4a_splitk(3, x2, w, None, None, res, (norm_w, eps, y))


def linear_add(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], r: torch.Tensor,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x·wᵀ + b + r`` in x's dtype (``r`` [..., N] same dtype, unit inner stride); ``out`` may be
    ``r`` itself (in-place residual add)."""
    x2 = _rows(x)
    n = w.shape[0]
    r2 = r.reshape(-1, n)
    if r2.stride(-1) != 1 or r2.dtype != x.dtype or r2.shape[0] != x2.shape[0]:
        raise ValueError("linear_add: r must be [rows, N] in x's dtype with unit inner stride")
    if out is None:
        out = torch.empty((x2.shape[0], n), dtype=x.dtype, device=x.device)
    o2 = out.reshape(-1, n)
    _run(EPI_ADD, x2, w, _bias(b, n, x.dtype), o2, None, None, 0, 0, o2.stride(0), 0, r2, r2.stride(0))
    return out.view(*x.shape[:-1], n)


def conv_weight(w: torch.Tensor) -> torch.Tensor:
    """OIHW 3×3 conv weight → the kernel's [Cout, 3·3·Cin] (tap-major) layout."""
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous()


def conv3x3_supported(x: torch.Tensor, cout: int) -> bool:
    return (x.device.type == "cuda" and x.dtype == torch.float16 and x.dim() == 4
            and x.shape[1] % 64 == 0 and cout % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last))


def conv3x3(x: torch.Tensor, wk: torch.Tensor, b: Optional[torch.Tensor] = None,
            mode: int = CONV_S1, r: Optional[torch.Tensor] = None) -> torch.Tensor:
    """3×3 convolution (padding 1) of a channels-last fp16 NCHW tensor on the implicit-GEMM
    kernel: ``mode`` CONV_S1 (stride 1), CONV_S2 (stride 2), CONV_UP2 (nearest 2× upsample, then
    stride 1).  ``wk`` = :func:`conv_weight`; ``r`` (same shape as the output, channels-last) is
    added in the epilogue.  Returns a channels-last [N, Cout, Hout, Wout] tensor."""
    n, cin, h, w = x.shape
    cout = wk.shape[0]
    if not conv3x3_supported(x, cout) or wk.shape[1] != 9 * cin or wk.dtype != x.dtype:
        raise ValueError(f"conv3x3: unsupported input {tuple(x.shape)} {x.dtype} / weight {tuple(wk.shape)}")
    ho, wo = {CONV_S1: (h, w), CONV_S2: ((h + 1) // 2, (w + 1) // 2), CONV_UP2: (2 * h, 2 * w)}[mode]
    out = torch.empty((n, cout, ho, wo), dtype=x.dtype, device=x.device,
                      memory_format=torch.channels_last)
    if r is not None:
        if r.shape != out.shape or r.dtype != x.dtype or not r.is_contiguous(memory_format=torch.channels_last):
            raise ValueError("conv3x3: r must match the output (channels-last, same dtype)")
    bb = _bias(b, cout, x.dtype)
    epi = EPI_ADD if r is not None else EPI_STORE
    ws = _workspace(epi, n * ho * wo, cout, 9 * cin, x.device)
    rc = _lib().amdk8s_conv3x3_epi(epi, mode, x.data_ptr(), wk.data_ptr(), _ptr(bb), out.data_ptr(),
                                   _ptr(r), n, h, w, cin, cout, cout, cout, _ptr(ws), _stream(x))
    if rc != 0:
        raise RuntimeError(f"amdk8s_conv3x3_epi failed (rc={rc}, x={tuple(x.shape)}, Cout={cout}, mode={mode})")
    return out

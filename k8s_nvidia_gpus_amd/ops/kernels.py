"""Python bindings for the hand-written gfx950 HIP kernels (``_lib/libamdk8s_kernels.so``).

The library exposes a tiny C ABI (see ``csrc/*.hip``); we call it through ``ctypes`` with raw
device pointers and the current torch stream, so the kernels run on torch tensors, inside torch
streams and inside HIP-graph capture, without linking libtorch into the extension.

``import torch`` happens before the library is loaded: torch has already mapped
``libamdhip64.so.7`` and the extension's dependency on that soname binds to the same runtime.

There is deliberately **no** silent fallback: on a machine with a GPU, a missing or unloadable
library raises :class:`KernelLibraryError` (the validator must prove the native path ran).
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path
from typing import Optional

import torch

from . import build as _build

__all__ = [
    "KernelLibraryError",
    "library",
    "library_path",
    "gemm_bf16_nt",
    "gemm_bf16",
    "gemm_f16_nt",
    "gemm_shape_supported",
    "vector_add",
    "vector_add_bandwidth",
    "fill_uniform_bf16",
    "gemm_sample_check",
    "hbm_stream",
    "fp32_fma",
    "fp64_mfma",
]

GEMM_TILE_M = 256
GEMM_TILE_N = 256
GEMM_TILE_K = 64


class KernelLibraryError(RuntimeError):
    pass


_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None


def library_path() -> str:
    return str(_build.KERNEL_LIB)


def _declare(lib: ctypes.CDLL) -> None:
    vp, ci, cl, cf, cu64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_ulonglong
    lib.amdk8s_gemm_bf16_nt.argtypes = [vp, vp, vp, ci, ci, ci, ci, ci, ci, vp]
    lib.amdk8s_gemm_bf16_nt.restype = ci
    lib.amdk8s_gemm_bf16_nt_w4.argtypes = [vp, vp, vp, ci, ci, ci, ci, ci, ci, vp]
    lib.amdk8s_gemm_bf16_nt_w4.restype = ci
    lib.amdk8s_gemm_bf16_nt_w4a.argtypes = [vp, vp, vp, ci, ci, ci, ci, ci, ci, vp]
    lib.amdk8s_gemm_bf16_nt_w4a.restype = ci
    lib.amdk8s_gemm_f16_nt_w4a.argtypes = [vp, vp, vp, ci, ci, ci, ci, ci, ci, vp]
    lib.amdk8s_gemm_f16_nt_w4a.restype = ci
    lib.amdk8s_gemm_fp8_nt.argtypes = [vp, vp, vp, ci, ci, ci, ci, ci, ci, vp]
    lib.amdk8s_gemm_fp8_nt.restype = ci
    lib.amdk8s_gemm_fp8_nt_f8a.argtypes = [vp, vp, vp, ci, ci, ci, ci, ci, ci, vp]
    lib.amdk8s_gemm_fp8_nt_f8a.restype = ci
    lib.amdk8s_gemm_bf16_nt_sample_check.argtypes = [vp, vp, vp, vp, ci, ci, ci, ci, vp]
    lib.amdk8s_gemm_bf16_nt_sample_check.restype = ci
    lib.amdk8s_vector_add_f32.argtypes = [vp, vp, vp, ci, vp]
    lib.amdk8s_vector_add_f32.restype = ci
    lib.amdk8s_vector_add_f32_bw.argtypes = [vp, vp, vp, cl, ci, vp]
    lib.amdk8s_vector_add_f32_bw.restype = ci
    lib.amdk8s_vector_add_blocks.argtypes = [ci]
    lib.amdk8s_vector_add_blocks.restype = ci
    lib.amdk8s_fill_uniform_bf16.argtypes = [vp, cl, cu64, cf, cf, vp]
    lib.amdk8s_fill_uniform_bf16.restype = ci
    lib.amdk8s_fill_uniform_fp8.argtypes = [vp, cl, cu64, cf, cf, vp]
    lib.amdk8s_fill_uniform_fp8.restype = ci
    lib.amdk8s_hbm_stream.argtypes = [ci, vp, vp, cl, ci, ci, vp, vp]
    lib.amdk8s_hbm_stream.restype = ci
    lib.amdk8s_hbm_stream_variant.argtypes = [ci, vp, vp, cl, ci, ci, ci, ci, ci, ci, vp, vp]
    lib.amdk8s_hbm_stream_variant.restype = ci
    lib.amdk8s_fp32_fma.argtypes = [ci, ci, vp, vp]
    lib.amdk8s_fp32_fma.restype = ci
    lib.amdk8s_fp32_fma_flop.argtypes = [ci, ci]
    lib.amdk8s_fp32_fma_flop.restype = ctypes.c_double
    lib.amdk8s_fp64_mfma.argtypes = [ci, ci, vp, vp]
    lib.amdk8s_fp64_mfma.restype = ci
    lib.amdk8s_fp64_mfma_flop.argtypes = [ci, ci]
    lib.amdk8s_fp64_mfma_flop.restype = ctypes.c_double


def library(build_if_missing: bool = True) -> ctypes.CDLL:
    """Load (building first if needed and possible) the kernel library, once per process."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        alt = os.environ.get("AMDK8S_KERNEL_LIB")     # A/B: a variant build of the same sources
        path = Path(alt) if alt else _build.KERNEL_LIB
        stale = not alt and ((not path.exists()) or any(
            s.stat().st_mtime > path.stat().st_mtime for s in _build.kernel_sources()))
        if stale and build_if_missing and _build.toolchain_available() \
                and os.environ.get("AMDK8S_NO_BUILD") != "1":
            _build.build_kernel_library()
        if not path.exists():
            raise KernelLibraryError(
                f"{path} is missing; build it with `python -m k8s_nvidia_gpus_amd.ops.build kernels`")
        try:
            lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - depends on the host
            raise KernelLibraryError(f"cannot load {path}: {e}") from e
        _declare(lib)
        _lib = lib
        return lib


def _stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise KernelLibraryError(f"{what} failed with hipError {rc}")


def _require_gpu(t: torch.Tensor, name: str) -> None:
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be a GPU tensor (got {t.device})")


def gemm_shape_supported(m: int, n: int, k: int) -> bool:
    return m > 0 and n > 0 and k > 0 and m % GEMM_TILE_M == 0 and n % GEMM_TILE_N == 0 \
        and k % GEMM_TILE_K == 0


GEMM_VARIANTS = ("auto", "w8", "w4", "w4a")
DEFAULT_GEMM_VARIANT = os.environ.get("AMDK8S_GEMM_VARIANT", "auto")
# w4a — the one-wave-per-SIMD w4 kernel with its K-loop as generated assembly — is bit-identical to
# w4 and 3-4 % faster on every measured shape, 98-100 % of hipBLASLt (docs/gemm_tuning.md,
# profiles/r01_session4/).  It addresses a 256-row panel with 32-bit buffer offsets; beyond that
# (K ≳ 4M) w4's INTERLEAVED schedule takes over.  w8 and w4 stay selectable for A/B runs.
W4A_MAX_PANEL_BYTES = 1 << 31


def pick_gemm_variant(m: int, n: int, k: int, lda: Optional[int] = None,
                      ldb: Optional[int] = None) -> str:
    ld = max(lda or k, ldb or k)
    return "w4a" if 256 * ld * 2 < W4A_MAX_PANEL_BYTES else "w4"


def gemm_bf16_nt(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None,
                 variant: Optional[str] = None) -> torch.Tensor:
    """``out = a @ b.T`` with the hand-written 256×256×64 MFMA kernel.

    ``variant``: ``"w8"`` — 512 threads, 8 waves of 128×64 (gemm_bf16_gfx950.hip);
    ``"w4"`` — 256 threads, one wave per SIMD owning 128×128 (gemm_bf16_gfx950_w4.hip);
    ``"w4a"`` — w4 with its K-loop as generated assembly (gemm_bf16_gfx950_w4a.hip, bit-identical);
    ``"auto"`` (default) — :func:`pick_gemm_variant` by operand footprint.

    ``a``: [M, K] bf16, ``b``: [N, K] bf16 (nn.Linear weight layout), both row-major with unit
    inner stride.  M and N must be multiples of 256 and K a multiple of 64 — use :func:`gemm_bf16`
    for arbitrary shapes (it pads).
    """
    _require_gpu(a, "a")
    _require_gpu(b, "b")
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise TypeError("gemm_bf16_nt expects bf16 operands")
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[1]:
        raise ValueError(f"shape mismatch: a {tuple(a.shape)} b {tuple(b.shape)}")
    if a.stride(1) != 1 or b.stride(1) != 1:
        raise ValueError("operands must have unit inner stride")
    m, k = a.shape
    n = b.shape[0]
    if not gemm_shape_supported(m, n, k):
        raise ValueError(f"gemm_bf16_nt needs M,N % 256 == 0 and K % 64 == 0 (got {m}x{n}x{k})")
    if out is None:
        out = torch.empty((m, n), dtype=torch.bfloat16, device=a.device)
    elif out.shape != (m, n) or out.dtype != torch.bfloat16 or out.stride(1) != 1:
        raise ValueError("bad out tensor")
    lib = library()
    variant = variant or DEFAULT_GEMM_VARIANT
    if variant not in GEMM_VARIANTS:
        raise ValueError(f"unknown GEMM variant {variant!r} (have {GEMM_VARIANTS})")
    if variant == "auto":
        variant = pick_gemm_variant(m, n, k, a.stride(0), b.stride(0))
    fn = {"w8": lib.amdk8s_gemm_bf16_nt, "w4": lib.amdk8s_gemm_bf16_nt_w4,
          "w4a": lib.amdk8s_gemm_bf16_nt_w4a}[variant]
    rc = fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k,
            a.stride(0), b.stride(0), out.stride(0), _stream_handle(a.device))
    _check(rc, f"amdk8s_gemm_bf16_nt[{variant}]")
    return out


def gemm_f16_nt(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``out = a @ b.T`` in fp16 (fp32 accumulation, fp16 result) with the w4a kernel's generated
    K-loop on ``v_mfma_f32_16x16x32_f16`` — the same cycles per MFMA as bf16 on gfx950.
    Same shape contract as :func:`gemm_bf16_nt`."""
    _require_gpu(a, "a")
    _require_gpu(b, "b")
    if a.dtype != torch.float16 or b.dtype != torch.float16:
        raise TypeError("gemm_f16_nt expects fp16 operands")
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[1]:
        raise ValueError(f"shape mismatch: a {tuple(a.shape)} b {tuple(b.shape)}")
    if a.stride(1) != 1 or b.stride(1) != 1:
        raise ValueError("operands must have unit inner stride")
    m, k = a.shape
    n = b.shape[0]
    if not gemm_shape_supported(m, n, k):
        raise ValueError(f"gemm_f16_nt needs M,N % 256 == 0 and K % 64 == 0 (got {m}x{n}x{k})")
    if out is None:
        out = torch.empty((m, n), dtype=torch.float16, device=a.device)
    elif out.shape != (m, n) or out.dtype != torch.float16 or out.stride(1) != 1:
        raise ValueError("bad out tensor")
    rc = library().amdk8s_gemm_f16_nt_w4a(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k,
                                          a.stride(0), b.stride(0), out.stride(0),
                                          _stream_handle(a.device))
    _check(rc, "amdk8s_gemm_f16_nt_w4a")
    return out


FP8_DTYPE = torch.float8_e4m3fn  # OCP e4m3: gfx950's fp8 (not MI300's e4m3fnuz)


def gemm_fp8_shape_supported(m: int, n: int, k: int) -> bool:
    return m > 0 and n > 0 and k > 0 and m % 256 == 0 and n % 256 == 0 and k % 256 == 0


FP8_VARIANTS = ("f8a", "hipcc")
DEFAULT_FP8_VARIANT = os.environ.get("AMDK8S_FP8_VARIANT", "f8a")


def gemm_fp8_nt(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None,
                variant: Optional[str] = None) -> torch.Tensor:
    """``out = a @ b.T`` in fp8 (OCP e4m3) with fp32 accumulation and a bf16 result.

    The hand-written gfx950 kernels run ``v_mfma_scale_f32_16x16x128_f8f6f4`` with unit block
    scales — 2× the bf16 MFMA rate — on the bf16 w4 kernel's data path: ``"f8a"`` (default) with
    its K-loop as generated assembly (gemm_fp8_gfx950_f8a.hip), ``"hipcc"`` the compiler-scheduled
    original (gemm_fp8_gfx950.hip); both give the same bits.
    ``a``: [M, K], ``b``: [N, K], both ``torch.float8_e4m3fn``, row-major with unit inner stride and
    leading dimensions that are multiples of 16; M, N multiples of 256 and K a multiple of 256.
    """
    _require_gpu(a, "a")
    _require_gpu(b, "b")
    if a.dtype != FP8_DTYPE or b.dtype != FP8_DTYPE:
        raise TypeError("gemm_fp8_nt expects torch.float8_e4m3fn operands")
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[1]:
        raise ValueError(f"shape mismatch: a {tuple(a.shape)} b {tuple(b.shape)}")
    if a.stride(1) != 1 or b.stride(1) != 1:
        raise ValueError("operands must have unit inner stride")
    m, k = a.shape
    n = b.shape[0]
    if not gemm_fp8_shape_supported(m, n, k):
        raise ValueError(f"gemm_fp8_nt needs M,N % 256 == 0 and K % 256 == 0 (got {m}x{n}x{k})")
    if out is None:
        out = torch.empty((m, n), dtype=torch.bfloat16, device=a.device)
    elif out.shape != (m, n) or out.dtype != torch.bfloat16 or out.stride(1) != 1:
        raise ValueError("bad out tensor")
    variant = variant or DEFAULT_FP8_VARIANT
    if variant not in FP8_VARIANTS:
        raise ValueError(f"unknown fp8 GEMM variant {variant!r} (have {FP8_VARIANTS})")
    lib = library()
    fn = lib.amdk8s_gemm_fp8_nt_f8a if variant == "f8a" else lib.amdk8s_gemm_fp8_nt
    rc = fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), m, n, k, a.stride(0), b.stride(0),
            out.stride(0), _stream_handle(a.device))
    _check(rc, f"amdk8s_gemm_fp8_nt[{variant}]")
    return out


def uniform_fp8(shape, seed: int, device: torch.device, lo: float = -1.0,
                hi: float = 1.0) -> torch.Tensor:
    """Uniform [lo, hi) operands rounded to OCP e4m3 on the device (v_cvt_pk_fp8_f32)."""
    t = torch.empty(shape, dtype=FP8_DTYPE, device=device)
    if t.numel() % 4:
        raise ValueError("uniform_fp8 fills whole 4-byte words: numel must be a multiple of 4")
    rc = library().amdk8s_fill_uniform_fp8(t.data_ptr(), t.numel(), seed & (2 ** 64 - 1), lo, hi,
                                           _stream_handle(t.device))
    _check(rc, "amdk8s_fill_uniform_fp8")
    return t


def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def gemm_bf16(a: torch.Tensor, b: torch.Tensor, *, b_layout: str = "nk") -> torch.Tensor:
    """General ``a @ bᵀ`` (``b_layout='nk'``) or ``a @ b`` (``'kn'``) for any shape, via padding.

    The MFMA kernel only runs whole 256×256×64 tiles, so ragged shapes are zero-padded (zeros in
    K contribute nothing) and the result is sliced back.
    """
    if b_layout == "kn":
        b = b.t()
    elif b_layout != "nk":
        raise ValueError("b_layout must be 'nk' or 'kn'")
    m, k = a.shape
    n = b.shape[0]
    mp, np_, kp = _round_up(m, GEMM_TILE_M), _round_up(n, GEMM_TILE_N), _round_up(k, GEMM_TILE_K)
    if (mp, np_, kp) == (m, n, k) and a.stride(1) == 1 and b.stride(1) == 1 \
            and a.stride(0) % 8 == 0 and b.stride(0) % 8 == 0:
        return gemm_bf16_nt(a, b)
    ap = torch.zeros((mp, kp), dtype=torch.bfloat16, device=a.device)
    ap[:m, :k] = a
    bp = torch.zeros((np_, kp), dtype=torch.bfloat16, device=b.device)
    bp[:n, :k] = b
    return gemm_bf16_nt(ap, bp)[:m, :n]


def gemm_sample_check(a: torch.Tensor, b: torch.Tensor, coords: torch.Tensor) -> torch.Tensor:
    """fp32 on-device reference of ``(a @ b.T)[m, n]`` at ``coords`` ([S, 2] int32)."""
    coords = coords.to(device=a.device, dtype=torch.int32).contiguous()
    out = torch.empty(coords.shape[0], dtype=torch.float32, device=a.device)
    rc = library().amdk8s_gemm_bf16_nt_sample_check(
        a.data_ptr(), b.data_ptr(), coords.data_ptr(), out.data_ptr(), coords.shape[0], a.shape[1],
        a.stride(0), b.stride(0), _stream_handle(a.device))
    _check(rc, "amdk8s_gemm_bf16_nt_sample_check")
    return out


def vector_add(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 ``a + b`` with the reference-shaped kernel (256 threads, ⌈n/256⌉ blocks)."""
    _require_gpu(a, "a")
    if a.dtype != torch.float32 or b.dtype != torch.float32 or a.shape != b.shape:
        raise ValueError("vector_add expects two fp32 tensors of the same shape")
    a = a.contiguous()
    b = b.contiguous()
    if out is None:
        out = torch.empty_like(a)
    rc = library().amdk8s_vector_add_f32(a.data_ptr(), b.data_ptr(), out.data_ptr(), a.numel(),
                                         _stream_handle(a.device))
    _check(rc, "amdk8s_vector_add_f32")
    return out


def vector_add_blocks(n: int) -> int:
    return (n + 255) // 256


def vector_add_bandwidth(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """Streaming (16 B/lane, grid-stride) fp32 add for bandwidth measurement."""
    n = a.numel()
    cus = torch.cuda.get_device_properties(a.device).multi_processor_count
    rc = library().amdk8s_vector_add_f32_bw(a.data_ptr(), b.data_ptr(), out.data_ptr(), n, cus,
                                            _stream_handle(a.device))
    _check(rc, "amdk8s_vector_add_f32_bw")
    return out


def fill_uniform_bf16(t: torch.Tensor, seed: int, lo: float = -1.0, hi: float = 1.0) -> torch.Tensor:
    """Fill a bf16 GPU tensor with counter-hash uniform values in [lo, hi) (on the device)."""
    _require_gpu(t, "t")
    if t.dtype != torch.bfloat16 or not t.is_contiguous():
        raise ValueError("fill_uniform_bf16 expects a contiguous bf16 tensor")
    rc = library().amdk8s_fill_uniform_bf16(t.data_ptr(), t.numel(), seed & (2 ** 64 - 1), lo, hi,
                                            _stream_handle(t.device))
    _check(rc, "amdk8s_fill_uniform_bf16")
    return t


# ------------------------------------------------------------------------------------------------
# Load generators (csrc/loadgen.hip): the HBM / fp32 / fp64 targets of native/bin/amd-proftester.
# ------------------------------------------------------------------------------------------------
HBM_MODES = {"read": 0, "write": 1, "copy": 2}
_SINKS: dict = {}


def _sink(device: torch.device) -> torch.Tensor:
    key = (device.type, device.index)
    if key not in _SINKS:
        _SINKS[key] = torch.zeros(16, dtype=torch.int32, device=device)
    return _SINKS[key]


def hbm_stream(mode: str, src: Optional[torch.Tensor], dst: Optional[torch.Tensor],
               nbytes: Optional[int] = None, blocks_per_cu: int = 0,
               variant: Optional[tuple] = None) -> int:
    """Stream ``nbytes`` through HBM: ``mode`` = read (``src``), write (``dst``) or copy
    (``src`` → ``dst``).  Returns the bytes moved (2× for copy).  ``variant`` = (nt_load, nt_store,
    unroll) overrides the built-in policy for sweeps (tools/hbm_sweep.py)."""
    if mode not in HBM_MODES:
        raise ValueError(f"mode must be one of {tuple(HBM_MODES)}")
    ref = src if src is not None else dst
    if ref is None:
        raise ValueError("need a buffer")
    _require_gpu(ref, "buffer")
    m = HBM_MODES[mode]
    if m != 1 and (src is None or not src.is_contiguous()):
        raise ValueError("read/copy need a contiguous src")
    if m != 0 and (dst is None or not dst.is_contiguous()):
        raise ValueError("write/copy need a contiguous dst")
    avail = min(t.numel() * t.element_size() for t in (src, dst) if t is not None)
    nbytes = avail if nbytes is None else nbytes
    if nbytes > avail or nbytes % 16:
        raise ValueError(f"nbytes {nbytes} must be a multiple of 16 and fit the buffers ({avail})")
    cus = torch.cuda.get_device_properties(ref.device).multi_processor_count
    lib = library()
    sp = src.data_ptr() if src is not None else None
    dp = dst.data_ptr() if dst is not None else None
    sink = _sink(ref.device).data_ptr()
    if variant is None:
        rc = lib.amdk8s_hbm_stream(m, sp, dp, nbytes, cus, blocks_per_cu, sink, _stream_handle(ref.device))
    else:
        ntl, nts, unroll, chunked = (tuple(variant) + (0,))[:4]
        rc = lib.amdk8s_hbm_stream_variant(m, sp, dp, nbytes, cus, blocks_per_cu or 8, int(ntl), int(nts),
                                           int(unroll), int(chunked), sink, _stream_handle(ref.device))
    _check(rc, f"amdk8s_hbm_stream[{mode}]")
    return 2 * nbytes if m == 2 else nbytes


def fp32_fma(device: torch.device, iters: int = 20000, blocks_per_cu: int = 8) -> float:
    """One launch of the v_pk_fma_f32 load; returns the FLOP it executes."""
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    lib = library()
    blocks = cus * blocks_per_cu
    _check(lib.amdk8s_fp32_fma(blocks, iters, _sink(device).data_ptr(), _stream_handle(device)),
           "amdk8s_fp32_fma")
    return lib.amdk8s_fp32_fma_flop(blocks, iters)


def fp64_mfma(device: torch.device, iters: int = 3000, blocks_per_cu: int = 8) -> float:
    """One launch of the v_mfma_f64_16x16x4_f64 load; returns the FLOP it executes."""
    cus = torch.cuda.get_device_properties(device).multi_processor_count
    lib = library()
    blocks = cus * blocks_per_cu
    _check(lib.amdk8s_fp64_mfma(blocks, iters, _sink(device).data_ptr(), _stream_handle(device)),
           "amdk8s_fp64_mfma")
    return lib.amdk8s_fp64_mfma_flop(blocks, iters)

"""ctypes bindings of the LLM decode kernels (``csrc/llm_decode.hip``).

Same conventions as ``kernels.py`` / ``sd_kernels.py``: raw device pointers, torch's current stream
(so a decode step captures into one HIP graph), and no fallback — a missing library on a GPU host
raises ``KernelLibraryError`` from ``kernels.library()``.
"""
from __future__ import annotations

import ctypes
import threading

import torch

from .kernels import library

Q4K, Q6K = 0, 1
STORE, RESID, PAIR = 0, 1, 2

_declared = False
_lock = threading.Lock()


def _lib():
    global _declared
    lib = library()
    if not _declared:
        with _lock:
            vp, ci, cl, cf = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float
            lib.amdk8s_llm_max_tokens.restype = ci
            lib.amdk8s_llm_attn_chunk.restype = ci
            lib.amdk8s_llm_qgemv_mfma.argtypes = [ci, ci] + [vp] * 8 + [vp, vp, vp, vp, ci, vp, cf,
                                                                       vp, vp, ci, ci, ci, ci, ci,
                                                                       ci, vp, vp, vp,
                                                                       ci, vp, cl, vp, ci, vp]
            lib.amdk8s_llm_qgemv_mfma.restype = ci
            lib.amdk8s_llm_qgemv2_mfma.argtypes = [ci] + [vp] * 4 + [ci, vp, vp] + [ci] + [vp] * 4 \
                + [ci, vp, vp, ci, vp, vp, vp, vp, ci, vp, cf, ci, ci, vp]
            lib.amdk8s_llm_qgemv2_mfma.restype = ci
            lib.amdk8s_llm_mfma_pack.argtypes = [ci, vp, vp, vp, vp, ci, ci, vp, vp, vp, vp, vp]
            lib.amdk8s_llm_mfma_pack.restype = ci
            lib.amdk8s_llm_qgemv.argtypes = [ci, ci] + [vp] * 8 + [vp, vp, vp] \
                + [vp, ci, vp, cf] + [vp, vp] + [ci, ci, ci, ci, ci, ci] + [vp, vp, vp] + [vp]
            lib.amdk8s_llm_qgemv.restype = ci
            lib.amdk8s_llm_qgemv2.argtypes = [ci] + [vp] * 4 + [ci, vp, vp] + [ci] + [vp] * 4 \
                + [ci, vp, vp] + [ci, vp, vp, vp, vp, ci, vp, cf, ci, ci, ci, ci, vp]
            lib.amdk8s_llm_qgemv2.restype = ci
            lib.amdk8s_llm_argmax_rows.argtypes = [vp, ci, cl, ci, vp, vp]
            lib.amdk8s_llm_argmax_rows.restype = ci
            lib.amdk8s_llm_rmsnorm_q8.argtypes = [vp, vp, cf, ci, ci, vp, vp, vp, vp]
            lib.amdk8s_llm_rmsnorm_q8.restype = ci
            lib.amdk8s_llm_rope_kv.argtypes = [vp, ci, vp, vp, vp, vp, ci, ci, ci, ci, vp, vp, vp,
                                               ci, vp]
            lib.amdk8s_llm_rope_kv.restype = ci
            lib.amdk8s_llm_attn_decode.argtypes = [vp, vp, ci, vp, vp, vp, vp, vp, vp, ci, ci, ci,
                                                   ci, ci, cf, vp, vp, vp, vp, vp, vp, ci, vp]
            lib.amdk8s_llm_attn_decode.restype = ci
            lib.amdk8s_llm_dequant.argtypes = [ci, vp, vp, vp, vp, vp, ci, ci, vp, ci, vp]
            lib.amdk8s_llm_dequant.restype = ci
            lib.amdk8s_llm_q6k_repack.argtypes = [vp, cl, vp, vp, vp, vp, vp]
            lib.amdk8s_llm_q6k_repack.restype = ci
            lib.amdk8s_llm_q4k_repack.argtypes = [vp, cl, vp, vp, vp, vp]
            lib.amdk8s_llm_q4k_repack.restype = ci
            lib.amdk8s_llm_q6k_repack.restype = ci
            lib.amdk8s_llm_rmsnorm_f16.argtypes = [vp, ci, vp, cf, ci, ci, vp, ci, vp]
            lib.amdk8s_llm_rmsnorm_f16.restype = ci
            lib.amdk8s_llm_rope_kv_f16.argtypes = [vp, ci, vp, vp, ci, ci, ci, ci, ci, ci, cl, cl,
                                                   vp, vp, vp, vp]
            lib.amdk8s_llm_rope_kv_f16.restype = ci
            lib.amdk8s_llm_swiglu_f16.argtypes = [vp, ci, ci, ci, vp, vp]
            lib.amdk8s_llm_swiglu_f16.restype = ci
            _declared = True
    return lib


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t):
    return None if t is None else t.data_ptr()


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc})")


def max_tokens() -> int:
    """Tokens per decode step: 8 on the MFMA GEMV (two token quads per wave), 4 on the VALU one."""
    n = int(_lib().amdk8s_llm_max_tokens())
    return n if _GEMV[0] == GEMV_MFMA else min(n, 4)


def attn_chunk() -> int:
    return int(_lib().amdk8s_llm_attn_chunk())


GEMV_VALU, GEMV_MFMA = 0, 1
_GEMV = [GEMV_MFMA]


def gemv_impl(impl: int = None) -> int:
    """Process-wide quantised-GEMV implementation (GEMV_VALU / GEMV_MFMA); returns the previous one.
    Called with no argument it only queries.  The MFMA kernel needs the weights' MFMA-packed copy
    (:meth:`QWeight.mfma_pack`); without it a matrix stays on the VALU kernel at every T, so each
    matrix keeps one arithmetic (batch-invariant decode)."""
    prev = _GEMV[0]
    if impl is not None:
        _GEMV[0] = int(impl)
    return prev


def mfma_pack(w) -> tuple:
    """MFMA-packed copy (mq, mqh, msc, md) of a QWeight's planes (N % 16 == 0; mqh None for Q4_K)."""
    nb = w.k // 256
    dev = w.q.device
    mq = torch.empty(w.n * nb * 128, dtype=torch.uint8, device=dev)
    mqh = torch.empty(w.n * nb * 64, dtype=torch.uint8, device=dev) if w.qtype == 1 else None
    msc = torch.empty(w.n * nb * 16, dtype=torch.uint8, device=dev)
    md = torch.empty(w.n * nb, dtype=torch.int32, device=dev)
    _check(_lib().amdk8s_llm_mfma_pack(w.qtype, *w.ptrs(), w.n, nb, mq.data_ptr(), _p(mqh),
                                       msc.data_ptr(), md.data_ptr(), _stream(w.q)),
           "amdk8s_llm_mfma_pack")
    return mq, mqh, msc, md


class SplitKScratch:
    """Scratch of the MFMA GEMV's split-K combine (per engine): partial slabs and one arrival
    counter per row tile.  Zeroed once here; every launch leaves the counters zero again."""

    def __init__(self, max_n: int, device, max_split: int = 8):
        tiles = max(1, max_n // 16)
        self.part = torch.zeros(tiles * max_split * 2 * 64 * 4, dtype=torch.float32, device=device)
        self.cnt = torch.zeros(tiles, dtype=torch.int32, device=device)

    def args(self) -> tuple:
        return (self.part.data_ptr(), self.part.numel(), self.cnt.data_ptr(), self.cnt.numel())


def qgemv(w0, x8, dx, sx, out, mode: int = STORE, w1=None, bias=None, ldo: int = None,
          rows_per_wg: int = 0, waves: int = 0, xf=None, norm_w=None, eps: float = 1e-6,
          q8_out=None, kscratch: "SplitKScratch" = None, ksplit: int = -1) -> str:
    """``w0``/``w1``: :class:`~k8s_nvidia_gpus_amd.models.llm.weights.QWeight` on the GPU.
    Input: Q8 activations (``x8``/``dx``/``sx``, [T, K]) or fp32 rows ``xf`` [T, K] (pass
    ``x8=dx=sx=None``) that the kernel quantises itself, after an RMSNorm when ``norm_w`` is given.
    ``out`` fp32 [T, ldo] (a view with row stride ``ldo``).  ``waves`` per workgroup and
    ``rows_per_wg``: 0 = the kernel's default decomposition.  ``q8_out`` = (x8, dx, sx) [T, N]
    (pair mode only): write silu(g)·u quantised to Q8 — the ffn_down input — instead of ``out``.
    ``kscratch``: the engine's :class:`SplitKScratch`; with it, long-row matrices fed Q8
    (ffn_down) split their super-blocks over workgroups (``ksplit``: -1 = the matrix's default,
    1 = none, n = n slices; the MFMA kernel only).
    Returns the kernel that ran: "mfma" (:func:`gemv_impl` MFMA and packed weights) or "valu"."""
    t = (xf if xf is not None else x8).shape[0]
    ldo = out.stride(0) if ldo is None else ldo
    q8 = tuple(_p(t) for t in q8_out) if q8_out else (None,) * 3
    if (_GEMV[0] == GEMV_MFMA and w0.mfma is not None
            and (w1 is None or w1.mfma is not None)):
        b = w1.mfma_ptrs() if w1 is not None else (None,) * 4
        rc = _lib().amdk8s_llm_qgemv_mfma(
            w0.qtype, mode, *w0.mfma_ptrs(), *b, _p(x8), _p(dx), _p(sx), _p(xf),
            xf.stride(0) if xf is not None else 0, _p(norm_w), float(eps), _p(bias),
            out.data_ptr(), ldo, w0.n, w0.k, t, waves, rows_per_wg, *q8, int(ksplit),
            *(kscratch.args() if kscratch is not None else (None, 0, None, 0)),
            _stream(xf if xf is not None else x8))
        if rc != 4:
            _check(rc, "amdk8s_llm_qgemv_mfma")
            return "mfma"
    a = w0.ptrs()
    b = w1.ptrs() if w1 is not None else (None, None, None, None)
    ref = xf if xf is not None else x8
    rc = _lib().amdk8s_llm_qgemv(w0.qtype, mode, *a, *b, _p(x8), _p(dx), _p(sx), _p(xf),
                                 xf.stride(0) if xf is not None else 0, _p(norm_w), float(eps),
                                 _p(bias), out.data_ptr(), ldo, w0.n, w0.k, t,
                                 waves, rows_per_wg, *q8, _stream(ref))
    if rc == 4:
        raise RuntimeError(f"qgemv: {t} tokens need the MFMA GEMV (gemv_impl MFMA and the "
                           f"weights' mfma_pack); the VALU kernel takes at most 4")
    _check(rc, "amdk8s_llm_qgemv")
    return "valu"


def qgemv2(w0, w1, x8, dx, sx, out0, out1, bias0=None, bias1=None, rows_per_wg: int = 0,
           waves: int = 0, xf=None, norm_w=None, eps: float = 1e-6) -> bool:
    """Two store-mode GEMVs over the same Q8 input [T, K] in ONE launch (``out_i = W_i.x +
    bias_i``; ``out0``/``out1`` views with the same row stride) — q|k and v when their
    quantisation types differ.  Input as for :func:`qgemv`: Q8 (``x8``/``dx``/``sx``) or fp32
    rows ``xf`` (+ RMSNorm ``norm_w``) quantised in the prologue.  Returns False when the shape
    is not covered (K > 4096): the caller launches them with :func:`qgemv`."""
    if out0.stride(0) != out1.stride(0) or w0.k != w1.k:
        raise ValueError("qgemv2: both outputs need one row stride and both matrices one K")
    ref = xf if xf is not None else x8
    if _GEMV[0] == GEMV_MFMA and w0.mfma is not None and w1.mfma is not None:
        rc = _lib().amdk8s_llm_qgemv2_mfma(
            w0.qtype, *w0.mfma_ptrs(), w0.n, _p(bias0), out0.data_ptr(),
            w1.qtype, *w1.mfma_ptrs(), w1.n, _p(bias1), out1.data_ptr(), out0.stride(0),
            _p(x8), _p(dx), _p(sx), _p(xf), xf.stride(0) if xf is not None else 0, _p(norm_w),
            float(eps), w0.k, ref.shape[0], _stream(ref))
        if rc != 4:
            _check(rc, "amdk8s_llm_qgemv2_mfma")
            return True
        return False            # packed matrices stay on the MFMA kernel: separate launches
    rc = _lib().amdk8s_llm_qgemv2(w0.qtype, *w0.ptrs(), w0.n, _p(bias0), out0.data_ptr(),
                                  w1.qtype, *w1.ptrs(), w1.n, _p(bias1), out1.data_ptr(),
                                  out0.stride(0), _p(x8), _p(dx), _p(sx), _p(xf),
                                  xf.stride(0) if xf is not None else 0, _p(norm_w), float(eps),
                                  w0.k, ref.shape[0], waves, rows_per_wg, _stream(ref))
    if rc == 4:
        return False
    _check(rc, "amdk8s_llm_qgemv2")
    return True


def argmax_rows(x, out) -> None:
    """out (int32 [T]) = the first index of each row's maximum of x (fp32 [T, V], 16-B aligned)."""
    t, v = x.shape
    _check(_lib().amdk8s_llm_argmax_rows(x.data_ptr(), v, x.stride(0), t, out.data_ptr(),
                                         _stream(x)), "amdk8s_llm_argmax_rows")


def rmsnorm_q8(x, w, eps: float, x8, dx, sx) -> None:
    t, k = x.shape
    _check(_lib().amdk8s_llm_rmsnorm_q8(x.data_ptr(), _p(w), float(eps), k, t, x8.data_ptr(),
                                        dx.data_ptr(), sx.data_ptr(), _stream(x)),
           "amdk8s_llm_rmsnorm_q8")


def rope_kv(qkv, pos, slot, cos_t, sin_t, heads: int, kv_heads: int, head_dim: int,
            max_ctx: int, q_out, kc, vc) -> None:
    _check(_lib().amdk8s_llm_rope_kv(qkv.data_ptr(), qkv.stride(0), pos.data_ptr(),
                                     slot.data_ptr(), cos_t.data_ptr(), sin_t.data_ptr(), heads,
                                     kv_heads, head_dim, max_ctx, q_out.data_ptr(), kc.data_ptr(),
                                     vc.data_ptr(), qkv.shape[0], _stream(qkv)),
           "amdk8s_llm_rope_kv")


def attn_decode(q, pos, slot, kc, vc, heads: int, kv_heads: int, head_dim: int, max_ctx: int,
                scale: float, po, pml, x8, dx, sx, out=None, span: int = 0, qkv=None,
                cos_t=None, sin_t=None) -> None:
    """Split-context decode attention + combine + Q8 quantisation of the output.

    ``span``: context positions this call covers (multiple of ``attn_chunk()``, above every
    position; 0 = ``max_ctx``).  With ``qkv`` (the raw q|k|v projection) and the RoPE tables, the
    kernel also rotates q/k and writes the new K/V itself (``q`` unused, pass None) — only when
    every token of the step is in a distinct slot.  ``po`` / ``pml``: per-chunk partials
    (workspace); the combine launch merges them and writes the Q8 o_proj input x8 / dx / sx."""
    ref = qkv if qkv is not None else q
    _check(_lib().amdk8s_llm_attn_decode(_p(q), _p(qkv), qkv.stride(0) if qkv is not None else 0,
                                         _p(cos_t), _p(sin_t), pos.data_ptr(), slot.data_ptr(),
                                         kc.data_ptr(), vc.data_ptr(), heads, kv_heads, head_dim,
                                         max_ctx, span, float(scale), po.data_ptr(), pml.data_ptr(),
                                         _p(out), _p(x8), _p(dx), _p(sx),
                                         ref.shape[0], _stream(ref)),
           "amdk8s_llm_attn_decode")


def dequant(w, out, rows=None) -> None:
    """Rows of ``w`` (all, or the int32 indices ``rows``) → ``out`` (fp16 or fp32, [n, K])."""
    n = w.n if rows is None else rows.numel()
    if out.dtype not in (torch.float16, torch.float32) or tuple(out.shape) != (n, w.k):
        raise ValueError("dequant: out must be fp16/fp32 [rows, K]")
    _check(_lib().amdk8s_llm_dequant(w.qtype, *w.ptrs(), _p(rows), n, w.k, out.data_ptr(),
                                     int(out.dtype == torch.float32), _stream(out)),
           "amdk8s_llm_dequant")


def q6k_repack(raw, ql, qh, sc, d) -> None:
    _check(_lib().amdk8s_llm_q6k_repack(raw.data_ptr(), raw.numel() // 210, ql.data_ptr(),
                                        qh.data_ptr(), sc.data_ptr(), d.data_ptr(), _stream(raw)),
           "amdk8s_llm_q6k_repack")


def q4k_repack(raw, qs, scm, dm) -> None:
    _check(_lib().amdk8s_llm_q4k_repack(raw.data_ptr(), raw.numel() // 144, qs.data_ptr(),
                                        scm.data_ptr(), dm.data_ptr(), _stream(raw)),
           "amdk8s_llm_q4k_repack")


# ---------------------------------------------------------------------- prompt prefill (llm_prefill.hip)
def rmsnorm_f16(x, w, eps: float, y) -> None:
    """y (fp16 [P, K]) = RMSNorm(x fp32 [P, K]) * w — one launch (row stride of x / y free)."""
    p, k = x.shape
    _check(_lib().amdk8s_llm_rmsnorm_f16(x.data_ptr(), x.stride(0), w.data_ptr(), float(eps), p, k,
                                         y.data_ptr(), y.stride(0), _stream(x)),
           "amdk8s_llm_rmsnorm_f16")


def rope_kv_f16(qkv, cos_t, sin_t, start: int, heads: int, kv_heads: int, max_ctx: int, q_out,
                kc, vc) -> None:
    """q|k|v fp16 [P, (H + 2 Hkv) * 128] (bias included) -> rotated q fp16 [H, P, 128] (any head /
    position strides, unit inner stride) and the rotated k / v written into one slot's fp16 cache
    slabs ``kc`` / ``vc`` [Hkv, max_ctx, 128] at positions start .. start + P - 1."""
    p = qkv.shape[0]
    if tuple(q_out.shape) != (heads, p, 128) or q_out.stride(2) != 1:
        raise ValueError(f"rope_kv_f16: q_out {tuple(q_out.shape)} / {q_out.stride()} is not "
                         f"[{heads}, {p}, 128] with a unit inner stride")
    _check(_lib().amdk8s_llm_rope_kv_f16(qkv.data_ptr(), qkv.stride(0), cos_t.data_ptr(),
                                         sin_t.data_ptr(), start, p, heads, kv_heads, 128, max_ctx,
                                         q_out.stride(0), q_out.stride(1),
                                         q_out.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                                         _stream(qkv)), "amdk8s_llm_rope_kv_f16")


def swiglu_f16(gu, t, blk: int = 0) -> None:
    """t (fp16 [P, F]) = silu(gate) * up for gu fp16 [P, 2F] (both contiguous): gate = gu[:, :F],
    up = gu[:, F:] (blk 0), or gate|up interleaved in blocks of ``blk`` columns
    (``gate_up_interleave``)."""
    p, f = t.shape
    _check(_lib().amdk8s_llm_swiglu_f16(gu.data_ptr(), p, f, int(blk), t.data_ptr(), _stream(gu)),
           "amdk8s_llm_swiglu_f16")


def gate_up_interleave(wg, wu, blk: int = 128):
    """[2F, K] rows of gate and up interleaved in blocks of ``blk`` rows (gate rows blk·j..,
    then the same up rows): the layout whose 256-row GEMM tiles hold matching gate and up
    columns, so the SwiGLU runs in the GEMM epilogue (gemm_epi.linear_swiglu)."""
    f, k = wg.shape
    if f % blk:
        raise ValueError(f"gate rows {f} are not a multiple of {blk}")
    return torch.stack([wg.view(f // blk, blk, k), wu.view(f // blk, blk, k)], 1).reshape(2 * f, k)


def gate_up_split(gu, blk: int = 128):
    """Inverse view of ``gate_up_interleave`` on a product [.., 2F]: (gate, up) [.., F] each."""
    f2 = gu.shape[-1]
    v = gu.reshape(*gu.shape[:-1], f2 // (2 * blk), 2, blk)
    return v[..., 0, :].reshape(*gu.shape[:-1], f2 // 2), v[..., 1, :].reshape(*gu.shape[:-1], f2 // 2)


# ---------------------------------------------------------------------- prompt attention (llm_prefill_attn.hip)
_ATTN_WORK: dict = {}


def _declare_prefill_attn(lib) -> None:
    if getattr(lib, "_prefill_attn_declared", False):
        return
    vp, ci, cl, cf = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float
    lib.amdk8s_llm_prefill_attn.argtypes = [vp, cl, cl, vp, vp, cl, vp, cl, cl, ci, ci, ci, ci, cf,
                                            vp, cl, ci, ci, ci, ci, vp]
    lib.amdk8s_llm_prefill_attn.restype = ci
    lib.amdk8s_llm_prefill_attn_workspace.argtypes = [ci, ci, ci, ci, ci, ci, ci]
    lib.amdk8s_llm_prefill_attn_workspace.restype = cl
    lib.amdk8s_llm_prefill_attn_plan.argtypes = [ci, ci, ci, ci, ci, ci, ci, ctypes.POINTER(ci)]
    lib.amdk8s_llm_prefill_attn_plan.restype = ci
    lib._prefill_attn_declared = True


def prefill_attn_plan(P: int, start: int, heads: int, kv_heads: int, nsplit: int = 0,
                      nw: int = 0, ks: int = 0) -> dict:
    """The launch plan the kernel picks: waves per workgroup, key splits, key tiles per split,
    key slots per workgroup (``ks``: the waves split each step's keys, merged in LDS)."""
    lib = _lib()
    _declare_prefill_attn(lib)
    out = (ctypes.c_int * 4)()
    _check(lib.amdk8s_llm_prefill_attn_plan(P, start, heads, kv_heads, nsplit, nw, ks, out),
           "amdk8s_llm_prefill_attn_plan")
    return {"waves": out[0], "nsplit": out[1], "tiles_per_split": out[2], "key_slots": out[3]}


def prefill_attn(q, kc, vc, out, start: int, scale: float, nsplit: int = 0, nw: int = 0,
                 ks: int = 0) -> None:
    """Causal GQA attention of a prompt chunk against one slot's KV-cache slabs, in place.

    ``q`` / ``out``: [H, P, 128] views (unit inner stride, any head / token strides — the engine's
    token-major storage); ``kc`` / ``vc``: the slot's [Hkv, max_ctx, 128] slabs, positions
    0 .. start+P-1 written.  Query p sits at position start + p and sees keys 0 .. start + p.
    ``nsplit`` / ``nw`` / ``ks``: 0 = the kernel's plan (:func:`prefill_attn_plan`)."""
    H, P, D = q.shape
    hkv = kc.shape[0]
    if D != 128 or tuple(out.shape) != (H, P, D) or q.stride(2) != 1 or out.stride(2) != 1:
        raise ValueError(f"prefill_attn: q {tuple(q.shape)} / out {tuple(out.shape)} must be "
                         f"[H, P, 128] with a unit inner stride")
    if kc.shape != vc.shape or kc.shape[2] != 128 or kc.stride(1) != 128 or kc.stride(2) != 1 \
            or vc.stride() != kc.stride() or kc.shape[1] < start + P or H % hkv:
        raise ValueError("prefill_attn: kc / vc must be [Hkv, >= start+P, 128] slabs with rows of 128")
    if q.dtype != kc.dtype or out.dtype != q.dtype or q.dtype not in (torch.float16, torch.bfloat16):
        raise ValueError("prefill_attn: q, kc, vc, out must share fp16 or bf16")
    lib = _lib()
    _declare_prefill_attn(lib)
    need = int(lib.amdk8s_llm_prefill_attn_workspace(P, start, H, hkv, nsplit, nw, ks))
    if need < 0:
        raise ValueError("prefill_attn: bad shape")
    work = _ATTN_WORK.get(q.device)
    if need and (work is None or work.numel() * 4 < need):
        work = torch.empty((need + 3) // 4 + (1 << 20), dtype=torch.float32, device=q.device)
        _ATTN_WORK[q.device] = work
    _check(lib.amdk8s_llm_prefill_attn(
        q.data_ptr(), q.stride(1), q.stride(0), kc.data_ptr(), vc.data_ptr(), kc.stride(0),
        out.data_ptr(), out.stride(1), out.stride(0), P, int(start), H, hkv, float(scale),
        _p(work) if need else None, work.numel() * 4 if need else 0, int(nsplit), int(nw), int(ks),
        int(q.dtype == torch.bfloat16), _stream(q)), "amdk8s_llm_prefill_attn")

"""ggml block quantisation formats used by Q4_K_M GGUF files — numpy reference codecs.

The reference's model file is a ``Q4_K_M`` GGUF (reference cluster-config/apps/llm/deployment.yaml:31-34):
most matrices are ``Q4_K``; ``output.weight`` and part of ``attn_v``/``ffn_down`` are ``Q6_K``;
norms and biases are F32.  These vectorised numpy codecs are the fp32 ground truth the HIP kernels
(``ops/csrc/llm_decode.hip``) are tested against, and the quantisers write synthetic weights.

Block layouts (256 weights per super-block):

* ``Q4_K`` (144 B): ``d`` f16, ``dmin`` f16, ``scales[12]`` (eight 6-bit scales and eight 6-bit
  mins, packed), ``qs[128]``.  Weight ``64c + l`` (l < 32) is the low nibble of ``qs[32c + l]``,
  weight ``64c + 32 + l`` its high nibble; sub-block ``j`` (32 weights) has value
  ``d*sc_j*q - dmin*m_j``.
* ``Q6_K`` (210 B): ``ql[128]``, ``qh[64]``, ``scales[16]`` (int8, one per 16 weights), ``d`` f16.
  In half ``n`` (128 weights), weight ``128n + 32k + l`` takes its low 4 bits from ``ql[64n + l]``
  (k = 0, 2) or ``ql[64n + 32 + l]`` (k = 1, 3) — low nibble for k < 2, high for k ≥ 2 — and its
  high 2 bits from ``qh[32n + l] >> 2k``; value ``d * scales[8n + l//16 + 2k] * (q - 32)``.
* ``Q8_0`` (34 B / 32 weights): ``d`` f16, 32 int8.

These follow the published GGUF/ggml format definitions; no llama.cpp build or real checkpoint is
available offline, so parity with llama.cpp's own encoder is unpinned (the decoders are what the
engine needs, and the tests round-trip them against independent scalar decoders).
"""
from __future__ import annotations

import numpy as np

from . import gguf

QK_K = 256


def _f16(a: np.ndarray) -> np.ndarray:
    return a.view("<f2").astype(np.float32)


# ----------------------------------------------------------------------------- Q4_K
def _q4k_scale_min(scales: np.ndarray):
    """[nb, 12] packed bytes → (sc [nb, 8], m [nb, 8]) as uint8."""
    s = scales.astype(np.uint8)
    sc = np.empty(s.shape[:-1] + (8,), np.uint8)
    m = np.empty_like(sc)
    sc[..., :4] = s[..., 0:4] & 63
    m[..., :4] = s[..., 4:8] & 63
    sc[..., 4:] = (s[..., 8:12] & 0xF) | ((s[..., 0:4] >> 6) << 4)
    m[..., 4:] = (s[..., 8:12] >> 4) | ((s[..., 4:8] >> 6) << 4)
    return sc, m


def dequant_q4_k(raw: np.ndarray) -> np.ndarray:
    """uint8 [..., nb*144] → float32 [..., nb*256]."""
    lead = raw.shape[:-1]
    b = np.ascontiguousarray(raw).reshape(-1, 144)
    d = _f16(b[:, 0:2].copy())[:, 0]
    dmin = _f16(b[:, 2:4].copy())[:, 0]
    sc, m = _q4k_scale_min(b[:, 4:16])
    qs = b[:, 16:].reshape(-1, 4, 32)
    q = np.stack([qs & 0xF, qs >> 4], axis=2).reshape(-1, 8, 32).astype(np.float32)
    w = d[:, None, None] * sc[:, :, None] * q - dmin[:, None, None] * m[:, :, None]
    return w.reshape(lead + (-1,)).astype(np.float32)


def quant_q4_k(w: np.ndarray) -> np.ndarray:
    """float [..., K] (K % 256 == 0) → uint8 [..., K/256*144].  Min/max per 32-weight sub-block,
    6-bit scales and mins relative to per-super-block f16 ``d``/``dmin``."""
    lead = w.shape[:-1]
    x = np.asarray(w, np.float32).reshape(-1, 8, 32)
    mn = np.minimum(x.min(-1), 0.0)
    mx = x.max(-1)
    scale = (mx - mn) / 15.0
    mins = -mn
    d = (scale.max(-1) / 63.0).astype(np.float16)
    dmin = (mins.max(-1) / 63.0).astype(np.float16)
    df = d.astype(np.float32)
    dmf = dmin.astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        sc = np.where(df[:, None] > 0, np.rint(scale / df[:, None]), 0).clip(0, 63).astype(np.uint8)
        m = np.where(dmf[:, None] > 0, np.rint(mins / dmf[:, None]), 0).clip(0, 63).astype(np.uint8)
        step = df[:, None] * sc
        q = np.where(step[..., None] > 0,
                     np.rint((x + (dmf[:, None] * m)[..., None]) / step[..., None]), 0)
    q = q.clip(0, 15).astype(np.uint8)                      # [nb, 8, 32]
    nb = x.shape[0]
    out = np.zeros((nb, 144), np.uint8)
    out[:, 0:2] = d.reshape(-1, 1).view(np.uint8)
    out[:, 2:4] = dmin.reshape(-1, 1).view(np.uint8)
    s = np.zeros((nb, 12), np.uint8)
    s[:, 0:4] = (sc[:, 0:4] & 63) | ((sc[:, 4:8] >> 4) << 6)
    s[:, 4:8] = (m[:, 0:4] & 63) | ((m[:, 4:8] >> 4) << 6)
    s[:, 8:12] = (sc[:, 4:8] & 0xF) | ((m[:, 4:8] & 0xF) << 4)
    out[:, 4:16] = s
    qq = q.reshape(nb, 4, 2, 32)
    out[:, 16:] = (qq[:, :, 0, :] | (qq[:, :, 1, :] << 4)).reshape(nb, 128)
    return out.reshape(lead + (-1,))


# ----------------------------------------------------------------------------- Q6_K
def dequant_q6_k(raw: np.ndarray) -> np.ndarray:
    lead = raw.shape[:-1]
    b = np.ascontiguousarray(raw).reshape(-1, 210)
    ql = b[:, 0:128].reshape(-1, 2, 2, 32)          # [nb, half, (l | l+32), 32]
    qh = b[:, 128:192].reshape(-1, 2, 32)
    sc = b[:, 192:208].view(np.int8).astype(np.float32).reshape(-1, 2, 8)
    d = _f16(b[:, 208:210].copy())[:, 0]
    q = np.empty((b.shape[0], 2, 4, 32), np.int32)
    for k in range(4):
        lo = ql[:, :, k & 1, :]
        lo = (lo & 0xF) if k < 2 else (lo >> 4)
        q[:, :, k, :] = (lo | (((qh >> (2 * k)) & 3) << 4)).astype(np.int32) - 32
    # scale index 8n + l//16 + 2k  →  per (n, k, l): sc[n, 2k + l//16]
    s = np.empty((b.shape[0], 2, 4, 32), np.float32)
    for k in range(4):
        s[:, :, k, :16] = sc[:, :, 2 * k, None]
        s[:, :, k, 16:] = sc[:, :, 2 * k + 1, None]
    w = d[:, None, None, None] * s * q
    return w.reshape(lead + (-1,)).astype(np.float32)


def quant_q6_k(w: np.ndarray) -> np.ndarray:
    lead = w.shape[:-1]
    x = np.asarray(w, np.float32).reshape(-1, 16, 16)   # [nb, group, 16]
    amax = np.abs(x).max(-1)
    gscale = amax / 31.0
    d = (gscale.max(-1) / 127.0).astype(np.float16)
    df = d.astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        sc = np.where(df[:, None] > 0, np.rint(gscale / df[:, None]), 0).clip(-128, 127)
        step = df[:, None] * sc
        q = np.where(step[..., None] != 0, np.rint(x / step[..., None]), 0)
    q = (q.clip(-32, 31) + 32).astype(np.uint8).reshape(-1, 2, 4, 32)   # [nb, n, k, l]
    nb = x.shape[0]
    out = np.zeros((nb, 210), np.uint8)
    ql = np.zeros((nb, 2, 2, 32), np.uint8)
    ql[:, :, 0, :] = (q[:, :, 0, :] & 0xF) | ((q[:, :, 2, :] & 0xF) << 4)
    ql[:, :, 1, :] = (q[:, :, 1, :] & 0xF) | ((q[:, :, 3, :] & 0xF) << 4)
    qh = ((q[:, :, 0, :] >> 4) | ((q[:, :, 1, :] >> 4) << 2) | ((q[:, :, 2, :] >> 4) << 4)
          | ((q[:, :, 3, :] >> 4) << 6)).astype(np.uint8)
    out[:, 0:128] = ql.reshape(nb, 128)
    out[:, 128:192] = qh.reshape(nb, 64)
    # groups in x are 16 consecutive weights: group g = 128n/16 + ... → (n, k, l//16) ordering
    scg = sc.reshape(nb, 2, 4, 2)                      # weight index 128n + 32k + 16h + i
    sc_out = np.zeros((nb, 2, 8), np.int8)
    for k in range(4):
        sc_out[:, :, 2 * k] = scg[:, :, k, 0]
        sc_out[:, :, 2 * k + 1] = scg[:, :, k, 1]
    out[:, 192:208] = sc_out.reshape(nb, 16).view(np.uint8)
    out[:, 208:210] = d.reshape(-1, 1).view(np.uint8)
    return out.reshape(lead + (-1,))


# ----------------------------------------------------------------------------- Q8_0
def dequant_q8_0(raw: np.ndarray) -> np.ndarray:
    lead = raw.shape[:-1]
    b = np.ascontiguousarray(raw).reshape(-1, 34)
    d = _f16(b[:, 0:2].copy())[:, 0]
    q = b[:, 2:].view(np.int8).astype(np.float32)
    return (d[:, None] * q).reshape(lead + (-1,))


def quant_q8_0(w: np.ndarray) -> np.ndarray:
    lead = w.shape[:-1]
    x = np.asarray(w, np.float32).reshape(-1, 32)
    d = (np.abs(x).max(-1) / 127.0).astype(np.float16)
    df = d.astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        q = np.where(df[:, None] > 0, np.rint(x / df[:, None]), 0).clip(-127, 127).astype(np.int8)
    out = np.zeros((x.shape[0], 34), np.uint8)
    out[:, 0:2] = d.reshape(-1, 1).view(np.uint8)
    out[:, 2:] = q.view(np.uint8)
    return out.reshape(lead + (-1,))


DEQUANT = {gguf.Q4_K: dequant_q4_k, gguf.Q6_K: dequant_q6_k, gguf.Q8_0: dequant_q8_0}
QUANT = {gguf.Q4_K: quant_q4_k, gguf.Q6_K: quant_q6_k, gguf.Q8_0: quant_q8_0}


def dequantize(raw: np.ndarray, ggml_type: int) -> np.ndarray:
    if ggml_type == gguf.F32:
        return np.asarray(raw, np.float32)
    if ggml_type in (gguf.F16, gguf.BF16):
        return np.asarray(raw).astype(np.float32)
    if ggml_type not in DEQUANT:
        raise gguf.GGUFError(f"no decoder for ggml type {ggml_type}")
    return DEQUANT[ggml_type](raw)


def quantize(w: np.ndarray, ggml_type: int) -> np.ndarray:
    if ggml_type == gguf.F32:
        return np.asarray(w, np.float32)
    if ggml_type == gguf.F16:
        return np.asarray(w, np.float16)
    return QUANT[ggml_type](w)

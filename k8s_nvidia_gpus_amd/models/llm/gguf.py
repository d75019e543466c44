"""GGUF v3 container: reader (memory-mapped, nothing executed from the file) and writer.

The reference's LLM workload serves ``qwen2.5-7b-instruct-abliterated-v2.Q4_K_M.gguf`` with
llama.cpp (reference cluster-config/apps/llm/deployment.yaml:31-34,61,76-84).  This module reads the
same file format so the in-tree engine (``engine.py``) loads the same model file the reference's
init container downloads.  The writer exists for the offline build: there is no network for the
real checkpoint, so tests and the benchmark write synthetic GGUF files of the exact Qwen2.5-7B
architecture (``synthetic.py``).

Layout (little-endian): magic ``GGUF``, version u32, n_tensors u64, n_kv u64, the key/value
metadata, the tensor infos (name, n_dims u32, ne[n_dims] u64 with ne[0] the contiguous dimension,
ggml type u32, data offset u64), padding to ``general.alignment`` (default 32), then the tensor data.
"""
from __future__ import annotations

import mmap
import os
import struct
from dataclasses import dataclass
from typing import Any, BinaryIO, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

MAGIC = b"GGUF"
VERSION = 3
DEFAULT_ALIGNMENT = 32

# metadata value types
UINT8, INT8, UINT16, INT16, UINT32, INT32, FLOAT32, BOOL, STRING, ARRAY, UINT64, INT64, FLOAT64 = \
    range(13)
_SCALAR = {UINT8: "<B", INT8: "<b", UINT16: "<H", INT16: "<h", UINT32: "<I", INT32: "<i",
           FLOAT32: "<f", BOOL: "<?", UINT64: "<Q", INT64: "<q", FLOAT64: "<d"}
_NP = {UINT8: np.uint8, INT8: np.int8, UINT16: np.uint16, INT16: np.int16, UINT32: np.uint32,
       INT32: np.int32, FLOAT32: np.float32, BOOL: np.bool_, UINT64: np.uint64, INT64: np.int64,
       FLOAT64: np.float64}

# ggml tensor types this stack handles, with (weights per block, bytes per block)
F32, F16, Q4_0, Q4_1, Q8_0, Q4_K, Q5_K, Q6_K, BF16 = 0, 1, 2, 3, 8, 12, 13, 14, 30
TYPE_NAMES = {F32: "F32", F16: "F16", Q4_0: "Q4_0", Q4_1: "Q4_1", Q8_0: "Q8_0", Q4_K: "Q4_K",
              Q5_K: "Q5_K", Q6_K: "Q6_K", BF16: "BF16"}
BLOCK = {F32: (1, 4), F16: (1, 2), BF16: (1, 2), Q4_0: (32, 18), Q4_1: (32, 20), Q8_0: (32, 34),
         Q4_K: (256, 144), Q5_K: (256, 176), Q6_K: (256, 210)}


class GGUFError(ValueError):
    pass


def nbytes(ggml_type: int, n_elements: int) -> int:
    if ggml_type not in BLOCK:
        raise GGUFError(f"unsupported ggml type {ggml_type}")
    per, size = BLOCK[ggml_type]
    if n_elements % per:
        raise GGUFError(f"{n_elements} elements is not a whole number of {per}-blocks")
    return n_elements // per * size


@dataclass
class TensorInfo:
    name: str
    shape: Tuple[int, ...]      # ggml order: shape[0] is the contiguous (row) dimension
    ggml_type: int
    offset: int                 # from the start of the data section

    @property
    def n_elements(self) -> int:
        n = 1
        for d in self.shape:
            n *= d
        return n

    @property
    def nbytes(self) -> int:
        return nbytes(self.ggml_type, self.n_elements)

    @property
    def type_name(self) -> str:
        return TYPE_NAMES.get(self.ggml_type, str(self.ggml_type))

    @property
    def rows(self) -> int:
        return self.n_elements // self.shape[0]


class _Reader:
    def __init__(self, buf, pos: int = 0):
        self.buf = buf
        self.pos = pos

    def unpack(self, fmt: str):
        v = struct.unpack_from(fmt, self.buf, self.pos)
        self.pos += struct.calcsize(fmt)
        return v[0]

    def string(self) -> str:
        n = self.unpack("<Q")
        if n > len(self.buf) - self.pos:
            raise GGUFError("string runs past the end of the file")
        s = bytes(self.buf[self.pos:self.pos + n]).decode("utf-8", errors="replace")
        self.pos += n
        return s

    def value(self, vtype: int):
        if vtype in _SCALAR:
            return self.unpack(_SCALAR[vtype])
        if vtype == STRING:
            return self.string()
        if vtype == ARRAY:
            etype = self.unpack("<I")
            n = self.unpack("<Q")
            if etype in _NP:
                dt = np.dtype(_NP[etype]).newbyteorder("<")
                if n * dt.itemsize > len(self.buf) - self.pos:
                    raise GGUFError("array runs past the end of the file")
                arr = np.frombuffer(self.buf, dtype=dt, count=n, offset=self.pos).copy()
                self.pos += n * dt.itemsize
                return arr
            return [self.value(etype) for _ in range(n)]
        raise GGUFError(f"unknown metadata value type {vtype}")


class GGUFFile:
    """A GGUF file mapped read-only.  ``tensor(name)`` returns a zero-copy uint8 view of the raw
    blocks (or a typed view for F32/F16)."""

    def __init__(self, path: str):
        self.path = path
        self._f = open(path, "rb")
        size = os.fstat(self._f.fileno()).st_size
        if size < 24:
            raise GGUFError(f"{path}: too small for a GGUF header")
        self._mm = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ)
        r = _Reader(self._mm)
        if bytes(self._mm[:4]) != MAGIC:
            raise GGUFError(f"{path}: not a GGUF file")
        r.pos = 4
        self.version = r.unpack("<I")
        if self.version not in (2, 3):
            raise GGUFError(f"{path}: GGUF version {self.version} not supported")
        n_tensors = r.unpack("<Q")
        n_kv = r.unpack("<Q")
        self.metadata: Dict[str, Any] = {}
        for _ in range(n_kv):
            key = r.string()
            self.metadata[key] = r.value(r.unpack("<I"))
        self.tensors: Dict[str, TensorInfo] = {}
        for _ in range(n_tensors):
            name = r.string()
            nd = r.unpack("<I")
            shape = tuple(r.unpack("<Q") for _ in range(nd))
            t = r.unpack("<I")
            off = r.unpack("<Q")
            self.tensors[name] = TensorInfo(name, shape, t, off)
        align = int(self.metadata.get("general.alignment", DEFAULT_ALIGNMENT))
        self.data_offset = (r.pos + align - 1) // align * align
        for ti in self.tensors.values():
            end = self.data_offset + ti.offset + ti.nbytes
            if end > size:
                raise GGUFError(f"{path}: tensor {ti.name} runs past the end of the file")

    def close(self) -> None:
        try:
            self._mm.close()
        except BufferError:
            pass        # a caller still holds a zero-copy view; the mapping closes with it
        finally:
            self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def get(self, key: str, default=None):
        return self.metadata.get(key, default)

    def raw(self, name: str) -> np.ndarray:
        """Raw bytes of a tensor as uint8 ``[rows, row_bytes]`` (zero-copy view of the mapping)."""
        ti = self.tensors[name]
        start = self.data_offset + ti.offset
        a = np.frombuffer(self._mm, dtype=np.uint8, count=ti.nbytes, offset=start)
        return a.reshape(ti.rows, -1)

    def tensor(self, name: str) -> np.ndarray:
        """F32/F16/BF16 tensors as typed arrays in PyTorch order (reversed ggml shape); quantized
        tensors as raw block bytes ``[rows, row_bytes]``."""
        ti = self.tensors[name]
        shape = tuple(reversed(ti.shape))
        start = self.data_offset + ti.offset
        if ti.ggml_type == F32:
            return np.frombuffer(self._mm, dtype="<f4", count=ti.n_elements, offset=start).reshape(shape)
        if ti.ggml_type == F16:
            return np.frombuffer(self._mm, dtype="<f2", count=ti.n_elements, offset=start).reshape(shape)
        if ti.ggml_type == BF16:
            u = np.frombuffer(self._mm, dtype="<u2", count=ti.n_elements, offset=start)
            return (u.astype(np.uint32) << 16).view(np.float32).reshape(shape)
        return self.raw(name)


def _w_string(f: BinaryIO, s: str) -> None:
    b = s.encode("utf-8")
    f.write(struct.pack("<Q", len(b)))
    f.write(b)


def _infer_type(v) -> int:
    if isinstance(v, bool):
        return BOOL
    if isinstance(v, int):
        return INT64 if v < 0 or v >= 2 ** 32 else UINT32
    if isinstance(v, float):
        return FLOAT32
    if isinstance(v, str):
        return STRING
    if isinstance(v, (list, tuple, np.ndarray)):
        return ARRAY
    raise GGUFError(f"cannot store {type(v)} in GGUF metadata")


def _w_value(f: BinaryIO, v, vtype: Optional[int] = None) -> None:
    vtype = _infer_type(v) if vtype is None else vtype
    f.write(struct.pack("<I", vtype))
    _w_payload(f, v, vtype)


def _w_payload(f: BinaryIO, v, vtype: int) -> None:
    if vtype in _SCALAR:
        f.write(struct.pack(_SCALAR[vtype], v))
    elif vtype == STRING:
        _w_string(f, v)
    elif vtype == ARRAY:
        if isinstance(v, np.ndarray):
            inv = {np.dtype(t): k for k, t in _NP.items()}
            et = inv[v.dtype]
            f.write(struct.pack("<IQ", et, v.size))
            f.write(np.ascontiguousarray(v).astype(v.dtype.newbyteorder("<")).tobytes())
            return
        v = list(v)
        et = _infer_type(v[0]) if v else UINT32
        if et == UINT32 and any(isinstance(x, int) and x < 0 for x in v):
            et = INT32
        f.write(struct.pack("<IQ", et, len(v)))
        for x in v:
            _w_payload(f, x, et)
    else:
        raise GGUFError(f"bad value type {vtype}")


def write_gguf(path: str, metadata: Dict[str, Any],
               tensors: Sequence[Tuple[str, Tuple[int, ...], int, Any]],
               alignment: int = DEFAULT_ALIGNMENT) -> None:
    """Write a GGUF v3 file.  ``tensors``: (name, ggml shape, ggml type, data) where data is a
    numpy array (or any object with ``tobytes``) of exactly ``nbytes(type, prod(shape))`` bytes, or
    a callable ``data(f)`` that streams those bytes into the file (used for multi-GB tensors)."""
    md = dict(metadata)
    md.setdefault("general.alignment", alignment)
    infos = []
    off = 0
    for name, shape, t, data in tensors:
        n = 1
        for d in shape:
            n *= d
        nb = nbytes(t, n)
        infos.append((name, shape, t, off, nb, data))
        off += (nb + alignment - 1) // alignment * alignment
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<IQQ", VERSION, len(infos), len(md)))
        for k, v in md.items():
            _w_string(f, k)
            if k == "general.alignment":
                _w_value(f, int(v), UINT32)
            else:
                _w_value(f, v)
        for name, shape, t, o, _, _ in infos:
            _w_string(f, name)
            f.write(struct.pack("<I", len(shape)))
            for d in shape:
                f.write(struct.pack("<Q", d))
            f.write(struct.pack("<IQ", t, o))
        pad = (-f.tell()) % alignment
        f.write(b"\0" * pad)
        base = f.tell()
        for name, shape, t, o, nb, data in infos:
            f.seek(base + o)
            if callable(data):
                start = f.tell()
                data(f)
                wrote = f.tell() - start
            else:
                b = data.tobytes() if hasattr(data, "tobytes") else bytes(data)
                f.write(b)
                wrote = len(b)
            if wrote != nb:
                raise GGUFError(f"{name}: wrote {wrote} bytes, expected {nb}")
        end = base + off
        f.truncate(end)
    os.replace(tmp, path)


def summary(g: GGUFFile) -> Dict[str, Any]:
    """Type histogram and sizes (what `llama-gguf` / the reference's model card report)."""
    hist: Dict[str, int] = {}
    total = 0
    for ti in g.tensors.values():
        hist[ti.type_name] = hist.get(ti.type_name, 0) + 1
        total += ti.nbytes
    return {"tensors": len(g.tensors), "types": hist, "bytes": total,
            "architecture": g.get("general.architecture"), "version": g.version}


"""ctypes loader for the range-coder oracle (oracle/range_coder_oracle.c).  Test
infrastructure only: the checker for the gfx950 range-coder kernels, never the
thing measured or shipped.  Builds oracle/liboracle_range.so with gcc if needed."""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "oracle", "range_coder_oracle.c")
SO = os.path.join(REPO, "oracle", "liboracle_range.so")

_lib = None
_lock = threading.Lock()


class OracleIov(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_size_t)]


def build() -> str:
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(SRC):
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-o", SO, SRC])
    return SO


def lib() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            h = ctypes.CDLL(build())
            h.oracle_range_compress.restype = ctypes.c_size_t
            h.oracle_range_compress.argtypes = [ctypes.POINTER(OracleIov), ctypes.c_size_t, ctypes.c_size_t,
                                                ctypes.c_void_p, ctypes.c_size_t]
            h.oracle_range_decompress.restype = ctypes.c_size_t
            h.oracle_range_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                                  ctypes.c_size_t]
            for name in ("oracle_range_compress_ragged", "oracle_range_decompress_ragged"):
                fn = getattr(h, name)
                fn.restype = None
                fn.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64] + [ctypes.c_void_p] * 4
            _lib = h
    return _lib


def compress(slices, in_limit: int | None = None, out_limit: int | None = None) -> bytes:
    """compressor.rs:38 semantics: `slices` coded in order, output at most out_limit bytes."""
    arrs = [np.frombuffer(bytes(s), dtype=np.uint8) for s in slices]
    total = sum(a.size for a in arrs)
    keep = [a if a.size else np.zeros(1, np.uint8) for a in arrs]
    iov = (OracleIov * max(1, len(arrs)))()
    for i, (a, k) in enumerate(zip(arrs, keep)):
        iov[i].data = k.ctypes.data
        iov[i].len = a.size
    lim = (2 * total + 64) if out_limit is None else out_limit
    out = np.zeros(max(lim, 1), np.uint8)
    n = lib().oracle_range_compress(iov, len(arrs), total if in_limit is None else in_limit, out.ctypes.data, lim)
    return out[:n].tobytes()


def decompress(data: bytes, out_limit: int = 4096) -> bytes:
    src = np.frombuffer(bytes(data) or b"\x00", dtype=np.uint8).copy()
    out = np.zeros(max(out_limit, 1), np.uint8)
    n = lib().oracle_range_decompress(src.ctypes.data, len(data), out.ctypes.data, out_limit)
    return out[:n].tobytes()


def _ragged(name, data, in_off, in_len, out_off, out_lim):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    in_off = np.ascontiguousarray(in_off, dtype=np.uint64)
    in_len = np.ascontiguousarray(in_len, dtype=np.uint32)
    out_off = np.ascontiguousarray(out_off, dtype=np.uint64)
    out_lim = np.ascontiguousarray(out_lim, dtype=np.uint32)
    n = in_off.size
    out = np.zeros(max(1, int(out_off[-1]) + int(out_lim[-1])) if n else 1, np.uint8)
    sizes = np.zeros(n, np.uint32)
    getattr(lib(), name)(data.ctypes.data, in_off.ctypes.data, in_len.ctypes.data, n, out.ctypes.data,
                         out_off.ctypes.data, out_lim.ctypes.data, sizes.ctypes.data)
    return out, sizes


def compress_ragged(data, in_off, in_len, out_off, out_lim):
    """Packet p -> out[out_off[p] : +sizes[p]] (limit out_lim[p])."""
    return _ragged("oracle_range_compress_ragged", data, in_off, in_len, out_off, out_lim)


def decompress_ragged(data, in_off, in_len, out_off, out_lim):
    return _ragged("oracle_range_decompress_ragged", data, in_off, in_len, out_off, out_lim)

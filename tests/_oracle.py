"""ctypes loader for the CPU oracle (oracle/crc32_oracle.c).  Test infrastructure only.

Builds oracle/liboracle_crc32.so with gcc if it is not there yet.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "oracle", "crc32_oracle.c")
SO = os.path.join(REPO, "oracle", "liboracle_crc32.so")

_lib = None
_lock = threading.Lock()


class OracleIov(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_size_t)]


def build() -> str:
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(SRC):
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-pthread", "-o", SO, SRC])
    return SO


def lib() -> ctypes.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            h = ctypes.CDLL(build())
            h.oracle_crc32.restype = ctypes.c_uint32
            h.oracle_crc32.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
            h.oracle_crc32_iov.restype = ctypes.c_uint32
            h.oracle_crc32_iov.argtypes = [ctypes.POINTER(OracleIov), ctypes.c_size_t]
            h.oracle_crc_update.restype = ctypes.c_uint32
            h.oracle_crc_update.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
            h.oracle_crc_table.restype = ctypes.POINTER(ctypes.c_uint32)
            h.oracle_crc32_ragged.restype = None
            h.oracle_crc32_ragged.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_uint64, ctypes.c_void_p]
            h.oracle_crc32_uniform.restype = None
            h.oracle_crc32_uniform.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                               ctypes.c_uint64, ctypes.c_void_p]
            h.oracle_crc32_ragged_mt.restype = ctypes.c_int
            h.oracle_crc32_ragged_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
            h.oracle_crc32_uniform_mt.restype = ctypes.c_int
            h.oracle_crc32_uniform_mt.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                                  ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
            h.oracle_enet_verify.restype = ctypes.c_int
            h.oracle_enet_verify.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_uint32]
            h.oracle_enet_insert.restype = ctypes.c_uint32
            h.oracle_enet_insert.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(OracleIov),
                                             ctypes.c_size_t, ctypes.c_uint32]
            _lib = h
    return _lib


def _u8(b) -> np.ndarray:
    return b if isinstance(b, np.ndarray) else np.frombuffer(bytes(b), dtype=np.uint8)


def crc32(slices) -> int:
    arrs = [np.ascontiguousarray(_u8(s)) for s in slices]
    iov = (OracleIov * max(1, len(arrs)))()
    for i, a in enumerate(arrs):
        iov[i].data = a.ctypes.data if a.size else None
        iov[i].len = a.size
    return lib().oracle_crc32_iov(iov, len(arrs))


def crc32_ragged(data: np.ndarray, offsets: np.ndarray, lengths: np.ndarray, threads: int = 1) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    assert off.size == 0 or int((off + ln).max()) <= data.size
    out = np.empty(off.size, dtype=np.uint32)
    if threads > 1:
        assert lib().oracle_crc32_ragged_mt(data.ctypes.data, off.ctypes.data, ln.ctypes.data, off.size,
                                            out.ctypes.data, threads) == 0
    else:
        lib().oracle_crc32_ragged(data.ctypes.data, off.ctypes.data, ln.ctypes.data, off.size, out.ctypes.data)
    return out


def crc32_uniform(data: np.ndarray, stride: int, length: int, count: int, threads: int = 1) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    assert count == 0 or (count - 1) * stride + length <= data.size
    out = np.empty(count, dtype=np.uint32)
    if threads > 1:
        assert lib().oracle_crc32_uniform_mt(data.ctypes.data, stride, length, count, out.ctypes.data, threads) == 0
    else:
        lib().oracle_crc32_uniform(data.ctypes.data, stride, length, count, out.ctypes.data)
    return out


def table() -> list[int]:
    t = lib().oracle_crc_table()
    return [t[i] for i in range(256)]

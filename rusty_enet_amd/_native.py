"""ctypes binding of the C ABI in include/enet_crc_amd.h.

This is the Python equivalent of the cgo/JNI/Rust `extern "C"` stubs shown in
INTEGRATION.md.  It only loads the in-tree shared library
(rusty_enet_amd/lib/libenet_crc_amd.so, built by `make` / __graft_entry__.build()).
If that file is missing the import of the compute functions raises: there is no
Python or CPU fallback for the checksum.
"""
from __future__ import annotations

import ctypes
import os
import threading

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
# ENET_CRC_AMD_LIB points at another build of the same library (A/B timing runs).
LIB_PATH = os.environ.get("ENET_CRC_AMD_LIB") or os.path.join(LIB_DIR, "libenet_crc_amd.so")
INCLUDE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
HEADER_PATH = os.path.join(INCLUDE_DIR, "enet_crc_amd.h")
HEADER_PATHS = [HEADER_PATH, os.path.join(INCLUDE_DIR, "enet_range_amd.h")]

ENET_CRC_OK = 0
ENET_CRC_E_INVALID = -1
ENET_CRC_E_NO_DEVICE = -2
ENET_CRC_E_HIP = -3
ENET_CRC_E_NOMEM = -4
ENET_CRC_E_DEVICE = -5  # a batch kernel gave up on the device: outputs invalid (ABI 6)


class NativeLibraryMissing(RuntimeError):
    """The HIP extension was not built (run `make` or __graft_entry__.build())."""


class CrcError(RuntimeError):
    """A C-ABI call returned a negative status."""

    def __init__(self, status: int, where: str, hip_error: int = 0):
        self.status = status
        self.hip_error = hip_error
        msg = f"{where}: status {status}"
        if _lib is not None:
            msg += f" ({_lib.enet_crc_strerror(status).decode()})"
        if hip_error:
            msg += f", hipError {hip_error}"
        super().__init__(msg)


class Iov(ctypes.Structure):
    """enet_crc_iov == ENetBuffer {data, data_length} (reference src/c.rs:25-28)."""

    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_size_t)]


_lib = None
_lock = threading.Lock()

_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)

_SIGNATURES = {
    "enet_crc_abi_version": (ctypes.c_int, []),
    "enet_crc_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "enet_crc_last_hip_error": (ctypes.c_int, []),
    "enet_crc_device_count": (ctypes.c_int, []),
    "enet_crc_device_status": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    "enet_crc_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "enet_crc_ctx_create_multi": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_void_p)]),
    "enet_crc_ctx_destroy": (None, [ctypes.c_void_p]),
    "enet_crc_ctx_lanes": (ctypes.c_int, [ctypes.c_void_p]),
    "enet_crc_ctx_set_percall_mode": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "enet_crc_ctx_percall_mode": (ctypes.c_int, [ctypes.c_void_p]),
    "enet_crc_ctx_stop_server": (ctypes.c_int, [ctypes.c_void_p]),
    "enet_crc_shard_bounds": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]),
    "enet_crc32_shards_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]),
    "enet_crc32_iov": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Iov), ctypes.c_size_t, _u32p]),
    "enet_crc32_uniform_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                                 ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    "enet_crc32_ragged_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]),
    "enet_crc32_ragged_host": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]),
    "enet_crc32_verify_ragged_device": (ctypes.c_int, [ctypes.c_void_p] * 5 + [ctypes.c_uint64] +
                                        [ctypes.c_void_p] * 3),
    "enet_crc32_insert_ragged_device": (ctypes.c_int, [ctypes.c_void_p] * 5 + [ctypes.c_uint64] +
                                        [ctypes.c_void_p] * 2),
    "enet_crc32_slot_adjust": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_uint32]),
    "enet_crc32_combine": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]),
    "enet_crc_ring_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.POINTER(ctypes.c_void_p)]),
    "enet_crc_ring_destroy": (None, [ctypes.c_void_p]),
    "enet_crc_ring_slot": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32] + [ctypes.POINTER(ctypes.c_void_p)] * 4),
    "enet_crc_ring_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64]),
    "enet_crc_ring_wait": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32]),
    # include/enet_range_amd.h
    "enet_range_scratch_bytes": (ctypes.c_uint64, [ctypes.c_uint64]),
    "enet_range_compress_ragged_device": (ctypes.c_int, [ctypes.c_void_p] * 3 + [ctypes.c_uint64] +
                                          [ctypes.c_void_p] * 5 + [ctypes.c_uint64, ctypes.c_void_p]),
    "enet_range_decompress_ragged_device": (ctypes.c_int, [ctypes.c_void_p] * 3 + [ctypes.c_uint64] +
                                            [ctypes.c_void_p] * 5 + [ctypes.c_uint64, ctypes.c_void_p]),
    "enet_range_compress_iov": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Iov), ctypes.c_size_t, ctypes.c_size_t,
                                               ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    "enet_range_decompress": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                             ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]),
    "enet_range_compress_ragged_host": (ctypes.c_int, [ctypes.c_void_p] * 4 + [ctypes.c_uint64] + [ctypes.c_void_p] * 4),
    "enet_range_decompress_ragged_host": (ctypes.c_int, [ctypes.c_void_p] * 4 + [ctypes.c_uint64] +
                                          [ctypes.c_void_p] * 4),
}


class Shard(ctypes.Structure):
    """enet_crc_shard (include/enet_crc_amd.h)."""

    _fields_ = [("device", ctypes.c_int), ("d_base", ctypes.c_void_p), ("d_offsets", ctypes.c_void_p),
                ("d_lengths", ctypes.c_void_p), ("stride", ctypes.c_uint64), ("length", ctypes.c_uint32),
                ("count", ctypes.c_uint64), ("d_out", ctypes.c_void_p), ("hip_stream", ctypes.c_void_p)]


ENET_CRC_PERCALL_COPY = 0
ENET_CRC_PERCALL_ZEROCOPY = 1
ENET_CRC_PERCALL_PERSISTENT = 2

ABI_VERSION = 6


def lib() -> ctypes.CDLL:
    """Load (once) and return the native library; raise if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"{LIB_PATH} not found: build the HIP extension first (make, or "
                "python -c 'import __graft_entry__ as g; g.build()')")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (restype, argtypes) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = restype
            fn.argtypes = argtypes
        if handle.enet_crc_abi_version() != ABI_VERSION:
            raise NativeLibraryMissing("ABI version mismatch")
        _lib = handle
    return _lib


def check(status: int, where: str) -> None:
    if status != ENET_CRC_OK:
        raise CrcError(status, where, lib().enet_crc_last_hip_error())


def exported_symbols() -> list[str]:
    return list(_SIGNATURES)

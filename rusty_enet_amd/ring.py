"""Pinned receive ring over the ``enet_crc_ring_*`` C ABI.

The reference receives each datagram into ``host->packet_data`` and checksums it on the
spot (src/c/protocol.rs:1660-1665, :1499).  A ring gives the receive loop pinned slots
to receive into directly, and checksums a whole slot per submit: H2D copy, kernel and
D2H copy run on the slot's own stream, so one slot's transfers overlap the others'
work.  The slot arrays are numpy views of the pinned memory itself (no staging copy).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import check, lib


class ReceiveRing:
    def __init__(self, device: int = 0, nslots: int = 4, slot_bytes: int = 64 << 20, slot_packets: int = 1 << 16):
        handle = ctypes.c_void_p()
        check(lib().enet_crc_ring_create(device, nslots, slot_bytes, slot_packets, ctypes.byref(handle)),
              "enet_crc_ring_create")
        self._handle = handle
        self.nslots, self.slot_bytes, self.slot_packets = nslots, slot_bytes, slot_packets
        self._views = [self._map(i) for i in range(nslots)]

    def _map(self, i: int):
        ptrs = [ctypes.c_void_p() for _ in range(4)]
        check(lib().enet_crc_ring_slot(self._handle, i, *[ctypes.byref(p) for p in ptrs]), "enet_crc_ring_slot")

        def view(ptr, ctype, n, dtype):
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctype)), shape=(n,)).view(dtype)

        return (view(ptrs[0], ctypes.c_uint8, self.slot_bytes, np.uint8),
                view(ptrs[1], ctypes.c_uint64, self.slot_packets, np.uint64),
                view(ptrs[2], ctypes.c_uint32, self.slot_packets, np.uint32),
                view(ptrs[3], ctypes.c_uint32, self.slot_packets, np.uint32))

    def slot(self, i: int):
        """(data, offsets, lengths, crcs): numpy views of slot i's pinned memory."""
        return self._views[i]

    def submit(self, i: int, count: int) -> None:
        check(lib().enet_crc_ring_submit(self._handle, i, count), "enet_crc_ring_submit")

    def wait(self, i: int) -> None:
        check(lib().enet_crc_ring_wait(self._handle, i), "enet_crc_ring_wait")

    def close(self) -> None:
        if getattr(self, "_handle", None) is not None and self._handle.value:
            lib().enet_crc_ring_destroy(self._handle)
        self._handle = None
        self._views = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

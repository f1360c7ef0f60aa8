"""ENet datagram-level checksum handling, batched.

Mirrors the two places where jabuwu/rusty_enet v0.4.0 calls the checksum hook:

* receive (``enet_protocol_handle_incoming_commands``, src/c/protocol.rs:1395-1502):
  header = big-endian u16 peer id with flag/session bits (:1400-1406), header size 2,
  or 4 with the SENT_TIME flag (:1407-1411), plus 4 for the checksum slot (:1412-1415);
  the slot's u32 is the sender's checksum; it is replaced by ``peer.connect_id`` (0 when
  the peer id is PROTOCOL_MAXIMUM_PEER_ID = 4095) and the datagram is accepted iff its
  checksum equals the stored value (:1470-1502).
* send (``enet_protocol_send_outgoing_commands``, :2255-2293): the slot after the
  header takes connect_id (0 while outgoing_peer_id >= 4095), the datagram is
  checksummed and the checksum overwrites the slot.

The reference does this one datagram at a time, inside a loop of up to 256 receives
(:1652-1692).  Here a whole batch goes to the GPU in one call; for receive, the
connect_id is still read per datagram at processing time (an earlier CONNECT in the
batch can change it, :550) and applied with ``slot_adjust``, which transforms the
GPU checksum by linearity.
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import numpy as np

from .checksum import default_context, slot_adjust

# src/c/protocol.rs:53-57, src/consts.rs:2
HEADER_SESSION_SHIFT = 12
HEADER_SESSION_MASK = 0x3000
HEADER_FLAG_MASK = 0xC000
HEADER_FLAG_SENT_TIME = 0x8000
HEADER_FLAG_COMPRESSED = 0x4000
PROTOCOL_MAXIMUM_PEER_ID = 4095
PROTOCOL_MAXIMUM_MTU = 4096  # src/consts.rs:8; the receive buffers are [u8; 4096] (c/host.rs:37)


def parse_header(datagram, checksum: bool = True):
    """(peer_id, flags, header_size) of a received datagram, or None if shorter than 2
    bytes (protocol.rs:1396-1415).  header_size includes the 4-byte checksum slot."""
    if len(datagram) < 2:
        return None
    raw = (datagram[0] << 8) | datagram[1]
    flags = raw & HEADER_FLAG_MASK
    peer_id = raw & ~(HEADER_FLAG_MASK | HEADER_SESSION_MASK) & 0xFFFF
    header_size = 4 if flags & HEADER_FLAG_SENT_TIME else 2
    if checksum:
        header_size += 4
    return peer_id, flags, header_size


def verify_received(datagrams: Sequence, connect_id_of: Callable[[int], int], ctx=None,
                    compressor: Optional[bool] = None) -> list:
    """Receive-side checksum verdicts for a batch of datagrams, in arrival order.

    ``connect_id_of(peer_id)`` is called per datagram, in order, at the moment the
    reference would read ``peer.connect_id`` (protocol.rs:1483-1487); it is never called
    for peer id 4095 (slot value 0).  Returns one bool per datagram (True = accept);
    datagrams too short for their header are rejected, as the reference returns
    before reaching the checksum (:1396-1398, :1412-1415 with :1440-1450).

    Compressed datagrams (HEADER_FLAG_COMPRESSED, :1441-1469): with ``compressor``
    true (the host has the range coder installed) the payload after the header is
    decompressed first, on the GPU, into a window of 4096 - header_size bytes, and the
    checksum covers the header plus the decompressed bytes, as in the reference; a
    size of 0 or one past the window drops the datagram (:1456-1460).  Without a
    compressor a compressed datagram is dropped (:1442-1444).
    """
    ctx = ctx or default_context(0)
    n = len(datagrams)
    if n == 0:
        return []
    views = [bytes(d) for d in datagrams]
    hdrs = [parse_header(d) for d in views]
    # Decompress the flagged payloads in one batch (only those that reach :1442).
    comp = [i for i, (d, h) in enumerate(zip(views, hdrs))
            if h is not None and h[1] & HEADER_FLAG_COMPRESSED and compressor and h[2] <= len(d)]
    if comp:
        payloads = [views[i][hdrs[i][2]:] for i in comp]
        p_len = np.array([len(p) for p in payloads], dtype=np.uint32)
        p_off = np.zeros(len(comp), dtype=np.uint64)
        if len(comp) > 1:
            p_off[1:] = np.cumsum(p_len[:-1], dtype=np.uint64)
        limits = np.array([PROTOCOL_MAXIMUM_MTU - hdrs[i][2] for i in comp], dtype=np.uint32)
        blob = np.frombuffer(b"".join(payloads) or b"\0", dtype=np.uint8)
        out, o_off, sizes = ctx.range_ragged_host(True, blob, p_off, p_len, limits)
        for k, i in enumerate(comp):
            size = int(sizes[k])
            if size == 0 or size > int(limits[k]):
                views[i] = None
            else:
                start = int(o_off[k])
                views[i] = views[i][:hdrs[i][2]] + out[start:start + size].tobytes()
    lens = np.array([len(d) if d is not None else 0 for d in views], dtype=np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    if n > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    joined = b"".join(d for d in views if d is not None)
    buf = np.frombuffer(joined, dtype=np.uint8) if joined else np.zeros(1, np.uint8)
    crcs = ctx.crc32_ragged_host(buf, offs, lens)  # one GPU pass, slots as received
    out = []
    for i, (d, hdr) in enumerate(zip(views, hdrs)):
        if hdr is None or d is None or hdr[2] > len(d):
            out.append(False)
            continue
        peer_id, flags, h = hdr
        if flags & HEADER_FLAG_COMPRESSED and not compressor:
            out.append(False)
            continue
        desired = int.from_bytes(d[h - 4:h], "little")  # native-endian u32 (x86)
        v = 0 if peer_id == PROTOCOL_MAXIMUM_PEER_ID else (connect_id_of(peer_id) & 0xFFFFFFFF)
        out.append(slot_adjust(int(crcs[i]), desired, v, len(d) - h) == desired)
    return out


def insert_outgoing(datagrams: Sequence[bytearray], header_lens: Sequence[int], slot_values: Sequence[int],
                    ctx=None) -> list:
    """Send-side: write the checksum into each datagram's slot (in place).

    Datagram i is ``header_lens[i]`` header bytes (2 or 4), the 4-byte slot, then the
    commands (uncompressed, protocol.rs:2294-2299 swaps buffers only afterwards).
    ``slot_values[i]`` is connect_id, or 0 while outgoing_peer_id >= 4095.  Returns the
    checksums.  One GPU pass for the batch, then the slot correction per datagram.
    """
    ctx = ctx or default_context(0)
    n = len(datagrams)
    if n == 0:
        return []
    lens = np.array([len(d) for d in datagrams], dtype=np.uint32)
    for d, h in zip(datagrams, header_lens):
        if h + 4 > len(d):
            raise ValueError("datagram shorter than its header and checksum slot")
    offs = np.zeros(n, dtype=np.uint64)
    if n > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bytes(d) for d in datagrams), dtype=np.uint8)
    crcs = ctx.crc32_ragged_host(buf, offs, lens)
    out = []
    for i, (d, h, v) in enumerate(zip(datagrams, header_lens, slot_values)):
        stored = int.from_bytes(bytes(d[h:h + 4]), "little")
        crc = slot_adjust(int(crcs[i]), stored, v & 0xFFFFFFFF, len(d) - h - 4)
        d[h:h + 4] = crc.to_bytes(4, "little")
        out.append(crc)
    return out

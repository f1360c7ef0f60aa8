"""Pin the CPU oracle (oracle/crc32_oracle.c) before trusting it as the GPU checker.

Pins: the reference's own KATs (src/crc32.rs:49-57), the CRC-32 check value,
and the zlib-generated golden fixtures (tests/golden/make_golden.py).
"""
import zlib

import numpy as np
import pytest

import _oracle
from _data import packed_offsets, ragged_lengths, splitmix64_bytes


def _slices(case):
    return [splitmix64_bytes(s, n) for s, n in case["slices"]]


def test_reference_kats():
    # src/crc32.rs:52
    assert _oracle.crc32([bytes([1, 2, 3, 4, 5, 6, 7, 8])]) == 3314076223
    # src/crc32.rs:54-55 (two slices = concatenation)
    assert _oracle.crc32([bytes([1, 2, 3, 4, 5, 6, 7, 8]), bytes([8, 7, 6, 5, 4, 3, 2, 1])]) == 1712484799


def test_golden_kats(golden):
    for k in golden["kat"]:
        assert _oracle.crc32([bytes(s) for s in k["slices_bytes"]]) == k["expected"], k["name"]


def test_golden_cases(golden):
    assert len(golden["cases"]) >= 50
    for case in golden["cases"]:
        assert _oracle.crc32(_slices(case)) == case["expected"], case["name"]


def test_table_is_reflected_edb88320():
    # src/crc32.rs:1-34 is the reflected 0xEDB88320 table: spot values that zlib's
    # table must have (T[1], T[128], T[255]) and the defining recurrence.
    t = _oracle.table()
    assert t[0] == 0 and t[1] == 0x77073096 and t[128] == 0xEDB88320 and t[255] == 0x2D02EF8D
    # every single-byte register step agrees with zlib
    for b in range(256):
        reg = _oracle.lib().oracle_crc_update(0xFFFFFFFF, bytes([b]), 1)
        assert (~reg) & 0xFFFFFFFF == zlib.crc32(bytes([b]))


def test_ragged_and_uniform_drivers_match_single_calls():
    lengths = ragged_lengths(3, 500, lo=0, hi=300)
    offsets = packed_offsets(lengths)
    data = splitmix64_bytes(4, int(lengths.sum()) + 8)
    got = _oracle.crc32_ragged(data, offsets, lengths)
    for i in range(0, 500, 37):
        o, n = int(offsets[i]), int(lengths[i])
        assert got[i] == int.from_bytes(zlib.crc32(data[o:o + n].tobytes()).to_bytes(4, "little"), "big")
    uni = _oracle.crc32_uniform(data, 97, 64, 100)
    mt = _oracle.crc32_uniform(data, 97, 64, 100, threads=4)
    assert np.array_equal(uni, mt)
    assert uni[5] == _oracle.crc32([data[5 * 97:5 * 97 + 64]])


def test_enet_insert_and_verify(golden):
    lib = _oracle.lib()
    for d in golden["enet"]:
        header = bytes.fromhex(d["header_hex"])
        payload = splitmix64_bytes(*d["payload"])
        # send side, src/c/protocol.rs:2255-2293
        hbuf = (np.zeros(len(header) + 4, dtype=np.uint8))
        hbuf[:len(header)] = np.frombuffer(header, dtype=np.uint8)
        iov = (_oracle.OracleIov * 1)()
        iov[0].data = payload.ctypes.data if payload.size else None
        iov[0].len = payload.size
        crc = lib.oracle_enet_insert(hbuf.ctypes.data, len(header), iov, 1, d["slot_value"])
        assert crc == d["checksum"], d["name"]
        wire = np.concatenate([hbuf, payload])
        assert wire.size == d["wire_len"]
        # receive side, src/c/protocol.rs:1470-1502
        rx = wire.copy()
        assert lib.oracle_enet_verify(rx.ctypes.data, rx.size, d["header_size"], d["slot_value"]) == 1
        # the slot is left holding slot_value, as in the reference
        assert int.from_bytes(rx[d["header_size"] - 4:d["header_size"]].tobytes(), "little") == d["slot_value"]
        # wrong connect_id or one flipped bit -> dropped
        rx = wire.copy()
        assert lib.oracle_enet_verify(rx.ctypes.data, rx.size, d["header_size"], d["slot_value"] ^ 1) == 0
        rx = wire.copy()
        rx[-1 if rx.size > d["header_size"] else 0] ^= 0x10
        assert lib.oracle_enet_verify(rx.ctypes.data, rx.size, d["header_size"], d["slot_value"]) == 0


@pytest.mark.parametrize("n", [0, 1, 3, 4, 5, 17, 1200, 4099])
def test_oracle_vs_zlib_random(n):
    rng = np.random.default_rng(n)
    data = rng.integers(0, 256, n, dtype=np.uint8)
    want = int.from_bytes(zlib.crc32(data.tobytes()).to_bytes(4, "little"), "big")
    assert _oracle.crc32([data]) == want
    # any split into slices gives the same value (concatenation, src/crc32.rs:41-42)
    cuts = sorted(rng.integers(0, n + 1, 5)) if n else [0]
    parts, prev = [], 0
    for c in cuts:
        parts.append(data[prev:c])
        prev = c
    parts.append(data[prev:])
    assert _oracle.crc32(parts) == want

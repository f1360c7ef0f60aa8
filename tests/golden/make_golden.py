"""Generate tests/golden/crc32_golden.json (run once in the build container).

Expected values come from Python's zlib.crc32, an implementation independent
of both the reference and this repo: the reference's crc32() equals
bswap32(zlib.crc32(concatenation)) on little-endian hosts (its table is the
reflected-0xEDB88320 table, src/crc32.rs:1-34, and it returns (!crc).to_be(),
src/crc32.rs:46).  The two known answers of src/crc32.rs:52 and :54-55 are
included verbatim as values (they are data, not code).

Input bytes are not stored: each slice is (seed, length) into the splitmix64
stream of tests/_data.py, so the file stays small.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from _data import splitmix64_bytes  # noqa: E402


def ref_value(data: bytes) -> int:
    return int.from_bytes(zlib.crc32(data).to_bytes(4, "little"), "big")


def main() -> None:
    cases = []

    def add(name, slices):
        data = b"".join(bytes(splitmix64_bytes(s, n)) for s, n in slices)
        cases.append({"name": name, "slices": [[s, n] for s, n in slices], "expected": ref_value(data)})

    # Lengths called out by SURVEY.md §7 step 2 (edges of the 4/16/128-byte grids,
    # ENet MTU-derived sizes 1360/1392/1396, PROTOCOL_MAXIMUM_MTU 4096, 64 KiB).
    lengths = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 11, 12, 13, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128,
               129, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 1199, 1200, 1201, 1360, 1392, 1396,
               2047, 2048, 4095, 4096, 4097, 65535, 65536, 65537]
    for i, n in enumerate(lengths):
        add(f"len{n}", [(1000 + i, n)])
    # Multi-slice: the hook receives up to BUFFER_MAXIMUM = 65 slices (src/consts.rs:37),
    # some of them empty (src/c/protocol.rs:2275-2286).
    add("two_slices", [(7, 600), (8, 600)])
    add("empty_slices", [(9, 0), (10, 13), (11, 0), (12, 0), (13, 1187), (14, 0)])
    add("odd_splits", [(15, 1), (16, 2), (17, 3), (18, 5), (19, 7), (20, 1182)])
    add("slices65", [(100 + j, (j * 37) % 61) for j in range(65)])
    add("header_plus_fragment", [(21, 4), (22, 4), (23, 24), (24, 1360)])

    kat = [
        {"name": "crc32.rs:52", "slices_bytes": [list(range(1, 9))], "expected": 3314076223},
        {"name": "crc32.rs:54-55", "slices_bytes": [list(range(1, 9)), list(range(8, 0, -1))],
         "expected": 1712484799},
        {"name": "check-123456789", "slices_bytes": [list(b"123456789")], "expected": 0x2639F4CB},
        {"name": "empty", "slices_bytes": [], "expected": 0},
        {"name": "empty-slice", "slices_bytes": [[]], "expected": 0},
    ]
    for k in kat:
        data = b"".join(bytes(s) for s in k["slices_bytes"])
        assert ref_value(data) == k["expected"], k

    # ENet-shaped datagrams (src/c/protocol.rs): header = peer_id (u16 BE) [+ sent_time
    # (u16 BE)], then the 4-byte checksum slot, then commands.  Send side (:2255-2293):
    # slot := connect_id (LE, native-endian copy) or 0 while connecting, checksum over
    # header||slot||rest, slot := checksum (LE).  Receive side (:1470-1502) re-derives it.
    enet = []
    specs = [  # (peer_id field, sent_time?, connect_id, slot uses connect_id?, payload len)
        (0x0001, False, 0x12345678, True, 1360 + 24 + 4),
        (0x8002, True, 0xDEADBEEF, True, 48),
        (0x0FFF, False, 0, False, 40),          # peer_id 4095: connect, slot = 0 (:1483-1487)
        (0x4003, True, 0x00000001, True, 1),
        (0x0004, False, 0xFFFFFFFF, True, 0),
    ]
    for j, (pid, sent_time, cid, use_cid, plen) in enumerate(specs):
        header = pid.to_bytes(2, "big") + ((0x1234).to_bytes(2, "big") if sent_time else b"")
        slot_value = cid if use_cid else 0
        payload = bytes(splitmix64_bytes(5000 + j, plen))
        crc = ref_value(header + slot_value.to_bytes(4, "little") + payload)
        wire = header + crc.to_bytes(4, "little") + payload
        enet.append({"name": f"enet{j}", "header_hex": header.hex(), "payload": [5000 + j, plen],
                     "slot_value": slot_value, "header_size": len(header) + 4,
                     "checksum": crc, "wire_len": len(wire)})

    out = {
        "generator": "tests/golden/make_golden.py (Python zlib)",
        "prng": "splitmix64 little-endian, tests/_data.py",
        "convention": "reference value = bswap32(zlib.crc32(concat)) = (!crc).to_be() of src/crc32.rs:46",
        "kat": kat,
        "cases": cases,
        "enet": enet,
    }
    with open(os.path.join(HERE, "crc32_golden.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(f"wrote {len(kat)} KATs, {len(cases)} cases, {len(enet)} ENet datagrams")


if __name__ == "__main__":
    main()

"""Pin of CRC_TABLE (jabuwu/rusty_enet src/crc32.rs:1-34) for tests/test_table_pin.py.

Run in the build container, where /root/reference exists:
    python tests/golden/make_table_fixture.py
It reads the reference file as TEXT (nothing of the reference is executed), parses
the 256 integer literals of the `CRC_TABLE` array, and stores only their SHA-256
(over the little-endian u32 bytes) plus a few spot entries in
tests/golden/crc_table_fixture.json.  The table itself is not copied into the repo:
the oracle and the kernels generate theirs from the polynomial and the tests
compare hashes.
"""
import hashlib
import json
import os
import re
import struct
import sys

REF = os.environ.get("RUSTY_ENET_REF", "/root/reference")
SRC = os.path.join(REF, "src", "crc32.rs")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "crc_table_fixture.json")


def parse_table(text: str) -> list[int]:
    m = re.search(r"const\s+CRC_TABLE\s*:\s*\[u32;\s*256\]\s*=\s*\[(.*?)\];", text, re.S)
    if not m:
        raise SystemExit("CRC_TABLE literal not found")
    vals = [int(tok, 0) for tok in re.findall(r"0[xX][0-9a-fA-F]+|\d+", m.group(1))]
    if len(vals) != 256:
        raise SystemExit(f"expected 256 entries, found {len(vals)}")
    first_line = text[:m.start()].count("\n") + 1
    last_line = text[:m.end()].count("\n") + 1
    return vals, first_line, last_line


def table_sha256(vals) -> str:
    return hashlib.sha256(struct.pack("<256I", *vals)).hexdigest()


def main() -> None:
    with open(SRC) as f:
        vals, l0, l1 = parse_table(f.read())
    fixture = {"source": f"src/crc32.rs:{l0}-{l1}", "entries": len(vals), "sha256_le_u32": table_sha256(vals),
               "spot": {str(i): vals[i] for i in (0, 1, 128, 255)},
               "generator": "tests/golden/make_table_fixture.py (text parse, reference not executed)"}
    with open(OUT, "w") as f:
        json.dump(fixture, f, indent=1)
    print(json.dumps(fixture))


if __name__ == "__main__":
    sys.exit(main())

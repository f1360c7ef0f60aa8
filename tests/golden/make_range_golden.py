"""Regenerates tests/golden/range_golden.json from the range-coder oracle
(oracle/range_coder_oracle.c).  The reference ships no range-coder vectors, so
these pin the oracle against regressions of its own (and the GPU against it),
not against reference output: "parity unpinned" (DESIGN.md §11).

    python tests/golden/make_range_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import _range_oracle as ro  # noqa: E402
from _data import ENET_SEED, enet_like_bytes, splitmix64_bytes  # noqa: E402

cases = []


def add(name, slices, out_limit=None):
    comp = ro.compress(slices, out_limit=out_limit)
    cases.append({"name": name, "slices": [bytes(s).hex() for s in slices], "out_limit": out_limit,
                  "compressed": comp.hex()})


add("hello", [b"hello hello hello world"])
add("kat_bytes", [bytes([1, 2, 3, 4, 5, 6, 7, 8])])
add("two_slices", [bytes([1, 2, 3, 4, 5, 6, 7, 8]), bytes([8, 7, 6, 5, 4, 3, 2, 1])])
add("empty_middle_slice", [b"ab", b"", b"cd"])
add("empty_first_slice", [b"", b"abc"])
add("zeros_1392", [bytes(1392)])
add("enet_like_1200", [enet_like_bytes(ENET_SEED, 1200).tobytes()])
add("random_600", [splitmix64_bytes(ENET_SEED + 1, 600).tobytes()])
add("random_limit_600", [splitmix64_bytes(ENET_SEED + 1, 600).tobytes()], out_limit=600)
add("reset_crossing_3000", [enet_like_bytes(ENET_SEED + 2, 3000).tobytes()])
add("single_byte", [b"\x7f"])

with open(os.path.join(HERE, "range_golden.json"), "w") as f:
    json.dump({"generator": "tests/golden/make_range_golden.py", "source": "oracle/range_coder_oracle.c",
               "cases": cases}, f, indent=1)
print(len(cases), "cases")

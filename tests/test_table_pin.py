"""a1 pin: the CRC table of the oracle and of the kernels equals CRC_TABLE of
src/crc32.rs:1-34, compared by SHA-256 against tests/golden/crc_table_fixture.json
(written by tests/golden/make_table_fixture.py from the reference text)."""
import hashlib
import json
import os
import struct
import subprocess

import _oracle

HERE = os.path.dirname(os.path.abspath(__file__))


def _fixture():
    with open(os.path.join(HERE, "golden", "crc_table_fixture.json")) as f:
        return json.load(f)


def _sha(vals) -> str:
    return hashlib.sha256(struct.pack("<256I", *vals)).hexdigest()


def test_fixture_shape():
    fx = _fixture()
    assert fx["source"] == "src/crc32.rs:1-34" and fx["entries"] == 256


def test_oracle_table_matches_reference_text():
    fx = _fixture()
    t = _oracle.table()
    assert _sha(t) == fx["sha256_le_u32"]
    assert all(t[int(i)] == v for i, v in fx["spot"].items())


def test_kernel_tables_match_reference_text(tmp_path):
    exe = tmp_path / "table_dump"
    subprocess.check_call(["g++", "-std=c++20", "-O1", os.path.join(HERE, "cpp", "table_dump.cpp"), "-o", str(exe)])
    lines = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    vals = [int(x, 16) for x in lines]
    assert len(vals) == 512
    fx = _fixture()
    assert _sha(vals[:256]) == fx["sha256_le_u32"]  # kOpTables.sarwate (tail/byte steps)
    assert _sha(vals[256:]) == fx["sha256_le_u32"]  # op[0][3], the LDS copy the kernels read

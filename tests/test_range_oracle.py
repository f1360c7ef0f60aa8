"""Range coder on the CPU: the oracle (oracle/range_coder_oracle.c,
a restatement of src/c/compress.rs) and the gfx950 kernel's coder code run on the host
(tests/cpp/range_model.hip includes rusty_enet_amd/csrc/range_coder.hip, whose coder
functions are __host__ __device__).

Parity unpinned by reference vectors: the reference has no range-coder tests or
fixtures and cannot be built here (no rustc).  The oracle is pinned by following
compress.rs statement by statement and by the round-trip property below;
tests/golden/range_golden.json guards it against regressions.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import _range_oracle as ro
from _data import ENET_SEED, enet_like_bytes, splitmix64_bytes

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


def _inputs():
    rng = np.random.default_rng(7)
    for t in range(240):
        n = int(rng.integers(0, 2600))
        kind = t % 4
        if kind == 0:
            yield rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            yield rng.integers(0, 3, n, dtype=np.uint8).tobytes()
        elif kind == 2:
            yield bytes(n)
        else:
            yield enet_like_bytes(ENET_SEED + t, n).tobytes()


def test_oracle_round_trip():
    for x in _inputs():
        c = ro.compress([x])
        if len(x) == 0:
            assert c == b""
            continue
        assert c, len(x)
        assert ro.decompress(c, out_limit=len(x)) == x
        assert ro.decompress(c, out_limit=len(x) + 17) == x
        if len(x) > 1:  # short output window: the reference returns 0 (compress.rs:949-951)
            assert ro.decompress(c, out_limit=len(x) - 1) == b""


def test_oracle_low_entropy_compresses():
    assert len(ro.compress([bytes(1392)])) < 16
    x = enet_like_bytes(ENET_SEED, 1200).tobytes()
    assert len(ro.compress([x])) < len(x)


def test_output_limit_and_empty_calls():
    x = splitmix64_bytes(ENET_SEED, 600).tobytes()
    assert ro.compress([x], out_limit=len(x)) == b""  # incompressible: limit reached -> 0
    assert ro.compress([x], out_limit=0) == b""
    assert ro.compress([x], in_limit=0) == b""  # compress.rs:79
    assert ro.compress([]) == b""
    assert ro.compress([b""]) == b""
    assert ro.decompress(b"") == b""  # compress.rs:481


def test_slice_rule_matches_gather():
    """An empty slice after the first codes one 0 byte (compress.rs:110-126 with the
    dangling empty-slice pointer, c.rs:79-85); the host gather reproduces that."""
    from rusty_enet_amd.range_coder import gather_slices

    a, b = b"header", b"payload bytes"
    for slices in ([a, b""], [a, b"", b], [b"", a, b], [a, b"", b"", b], [b"", b""], [a, b]):
        assert ro.compress(slices, in_limit=1) == ro.compress([gather_slices(slices)], in_limit=1), slices
    assert ro.decompress(ro.compress([a, b"", b])) == a + b"\x00" + b


def test_golden_fixtures():
    with open(os.path.join(HERE, "golden", "range_golden.json")) as f:
        cases = json.load(f)["cases"]
    assert len(cases) >= 10
    for c in cases:
        slices = [bytes.fromhex(s) for s in c["slices"]]
        got = ro.compress(slices, out_limit=c["out_limit"])
        assert got.hex() == c["compressed"], c["name"]
        if got:
            from rusty_enet_amd.range_coder import gather_slices
            assert ro.decompress(got, out_limit=8192) == gather_slices(slices), c["name"]


def test_ragged_helpers_agree_with_single_calls():
    lens = np.array([0, 1, 17, 300, 1200, 64], np.uint32)
    data = enet_like_bytes(ENET_SEED, int(lens.sum()))
    off = np.zeros(lens.size, np.uint64)
    off[1:] = np.cumsum(lens[:-1])
    out_off = np.zeros(lens.size, np.uint64)
    out_off[1:] = np.cumsum(lens[:-1])
    out, sizes = ro.compress_ragged(data, off, lens, out_off, lens)
    for p in range(lens.size):
        x = data[int(off[p]):int(off[p]) + int(lens[p])].tobytes()
        want = ro.compress([x], out_limit=int(lens[p]))
        assert sizes[p] == len(want)
        assert out[int(out_off[p]):int(out_off[p]) + len(want)].tobytes() == want


def test_kernel_coder_code_on_host(tmp_path):
    """The kernel's own coder functions, compiled for the host, agree with the oracle
    byte for byte (compressed bytes, sizes, decodes, limit failures, malformed input)."""
    exe = tmp_path / "range_model"
    so_dir = os.path.dirname(ro.build())
    try:
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-std=c++20",
                               os.path.join(HERE, "cpp", "range_model.hip"), "-L" + so_dir,
                               "-l:liboracle_range.so", "-Wl,-rpath," + so_dir, "-o", str(exe)])
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f"hipcc host build unavailable: {e}")
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad=0" in out.stdout

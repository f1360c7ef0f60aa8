"""`make asan`: the host-side code of the C ABI (shard split, slot correction, merged
digest, staging-chunk plan; rusty_enet_amd/csrc/crc32_host.hpp) and the C oracle, built
with -fsanitize=address,undefined and checked against each other (tests/cpp/host_asan.cpp;
SURVEY.md §5).  CPU only."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_host_code_under_asan_and_ubsan():
    r = subprocess.run(["make", "-C", REPO, "-s", "asan"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "0 failed" in r.stdout

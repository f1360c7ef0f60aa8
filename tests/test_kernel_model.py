"""CPU model of the gfx950 kernel arithmetic (tests/cpp/kernel_sim.cpp) vs the oracle.

Validates the operator tables in rusty_enet_amd/csrc/crc32_ops.hpp and the
stream/combine decomposition the kernel uses, for G = 2, 4, 8, 16 lanes per
packet, on ~60k random (start, length) cases including unaligned starts,
lengths 0..600 exhaustively and buffers up to 300 KB.  No GPU needed.
"""
import os
import subprocess

import _oracle

HERE = os.path.dirname(os.path.abspath(__file__))


def test_kernel_arithmetic_model(tmp_path):
    exe = tmp_path / "kernel_sim"
    subprocess.check_call(["g++", "-O2", "-std=c++20", "-fconstexpr-ops-limit=200000000",
                           os.path.join(HERE, "cpp", "kernel_sim.cpp"), _oracle.build(),
                           "-Wl,-rpath," + os.path.dirname(_oracle.SO), "-pthread",
                           "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad=0" in out.stdout


def test_lds_layout_and_bank_conflicts(tmp_path):
    """The kernels' replicated-table addressing (crc32_layout.hpp) returns the right
    operator entries for every lane, and every lookup is bank-conflict-free."""
    exe = tmp_path / "layout_check"
    subprocess.check_call(["g++", "-O2", "-std=c++20", "-fconstexpr-ops-limit=200000000",
                           os.path.join(HERE, "cpp", "layout_check.cpp"), "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad=0 conflicts=0" in out.stdout

#!/usr/bin/env python3
"""How long the ragged jobs kernel's waves spin on their LDS flags (tooling; the
`ENET_CRC_SPIN_STAMPS` measurement build).

    python scripts/exp_spin.py rusty_enet_amd/lib/variants/libenet_crc_amd_spin.so [--configs g2,frag,r740]

Per config: 200 back-to-back launches of enet_crc32_ragged_device (through the power-management
transient), then one more whose per-wave cells are read with enet_crc_debug_spin: the loop's
shader cycles per round, and per wait kind (ready, consumed, freed) the waits that found their
flag unset per 100 rounds and the cycles they spun per round."""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--configs", default="g2,frag,r740")
    ap.add_argument("--launches", type=int, default=200)
    args = ap.parse_args()

    import torch

    from _data import ENET_SEED, packed_offsets, ragged_lengths

    lib = ctypes.CDLL(os.path.abspath(args.lib))
    f = lib.enet_crc32_ragged_device
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    spin = lib.enet_crc_debug_spin
    spin.restype = ctypes.c_int
    spin.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int, ctypes.c_int]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    stream = torch.cuda.current_stream(dev)
    waves = min(4096, torch.cuda.get_device_properties(dev).multi_processor_count * 16)
    out = {}
    for name in args.configs.split(","):
        if name == "g2":
            lengths = ragged_lengths(ENET_SEED, 1 << 20)
        elif name.startswith("r") and name[1:].isdigit():
            lengths = np.full(1 << 20, int(name[1:]), dtype=np.uint32)
        else:
            lengths = np.tile(np.array([1392] * 48 + [288], dtype=np.uint32), 32768)
        offsets = packed_offsets(lengths)
        total = int(lengths.sum())
        g = torch.Generator(device=dev)
        g.manual_seed(ENET_SEED + 11)
        data = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
        off = torch.from_numpy(offsets.astype(np.int64)).to(dev)
        ln = torch.from_numpy(lengths.astype(np.int32)).to(dev)
        o = torch.empty(lengths.size, dtype=torch.int32, device=dev)
        for _ in range(args.launches):
            if f(data.data_ptr(), off.data_ptr(), ln.data_ptr(), lengths.size, o.data_ptr(), stream.cuda_stream):
                raise SystemExit("launch failed")
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 8)()
        if spin(buf, waves, 1) != 0:
            raise SystemExit("debug_spin failed")
        f(data.data_ptr(), off.data_ptr(), ln.data_ptr(), lengths.size, o.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        if spin(buf, waves, 0) != 0:
            raise SystemExit("debug_spin failed")
        cyc, rounds = buf[0], max(1, buf[1])
        row = {"waves": waves, "rounds": rounds, "cycles_per_round": round(cyc / rounds, 1)}
        for i, kind in enumerate(("ready", "consumed", "freed")):
            n, c = buf[2 + 2 * i], buf[3 + 2 * i]
            row[kind] = {"spinning_waits_per_100_rounds": round(100.0 * n / rounds, 2),
                         "spin_cycles_per_round": round(c / rounds, 1),
                         "share_of_loop": round(c / max(1, cyc), 4)}
        out[name] = row
        print(name, json.dumps(row), flush=True)
        del data, off, ln, o
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Per-launch series of a rocprofv3 --kernel-trace --pmc run of scripts/exp_ramp_pmc.py (tooling).

    python scripts/ramp_pmc_summary.py <rocprofv3 -d dir> [--block 10]

Joins each ragged-kernel dispatch's counters with its kernel-trace duration and prints, per block
of launches: duration, GRBM_GUI_ACTIVE (summed over the 8 XCDs, so / 8 per XCD), the effective
GPU clock = GRBM_GUI_ACTIVE / 8 / duration, SQ_BUSY_CYCLES, and the UTCL1 / UTCL2 translation
counters per launch."""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--block", type=int, default=10)
    ap.add_argument("--filter", default="crc32_ragged_jobs")
    args = ap.parse_args()
    dur = {}
    for p in glob.glob(os.path.join(args.root, "**", "*kernel_trace*.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if args.filter in r.get("Kernel_Name", ""):
                    dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    ctr = defaultdict(dict)
    for p in glob.glob(os.path.join(args.root, "**", "*counter_collection*.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                if args.filter in r.get("Kernel_Name", ""):
                    d = ctr[r["Dispatch_Id"]]
                    d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(set(ctr) & set(dur), key=int)
    names = sorted({c for i in ids for c in ctr[i]})
    print(f"{len(ids)} dispatches with counters and durations; counters: {', '.join(names)}")
    hdr = f"{'launches':>10} {'us':>8} {'GHz(GUI/8/t)':>13}"
    for c in names:
        if c != "GRBM_GUI_ACTIVE":
            hdr += f" {c[:28]:>29}"
    print(hdr)
    for b in range(0, len(ids), args.block):
        blk = ids[b:b + args.block]
        t = sum(dur[i] for i in blk) / len(blk)
        gui = sum(ctr[i].get("GRBM_GUI_ACTIVE", 0.0) for i in blk) / len(blk)
        line = f"{b:>4}-{b + len(blk) - 1:<5} {t * 1e6:8.1f} {gui / 8 / t * 1e-9:13.3f}"
        for c in names:
            if c != "GRBM_GUI_ACTIVE":
                line += f" {sum(ctr[i].get(c, 0.0) for i in blk) / len(blk):29.4g}"
        print(line)


if __name__ == "__main__":
    main()

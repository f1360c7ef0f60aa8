#!/usr/bin/env python3
"""Per-launch durations of one kernel in a rocprofv3 --kernel-trace run, in blocks of 10
launches (mean, min, max per block), with the gap to the previous launch (tooling).

    python scripts/launch_series.py gpurun_out/<tag>/trace_ragged --kernel crc32_ragged_jobs_kernel"""
import argparse
import csv
import glob
import os
import statistics
import sys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--block", type=int, default=10)
    args = ap.parse_args()
    rows = []
    for p in glob.glob(os.path.join(args.trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    sel = [(s, e) for s, e, k in rows if args.kernel in k]
    if not sel:
        print("no launches of", args.kernel, file=sys.stderr)
        return 1
    print(f"{len(sel)} launches of {args.kernel}")
    for i in range(0, len(sel), args.block):
        blk = sel[i:i + args.block]
        d = [(e - s) / 1000.0 for s, e in blk]
        gap = (blk[0][0] - sel[i - 1][1]) / 1000.0 if i else 0.0
        print(f"launches {i:4d}-{i + len(blk) - 1:4d}: mean {statistics.fmean(d):7.1f} us  min {min(d):7.1f}  "
              f"max {max(d):7.1f}  gap before {gap:9.1f} us")
    return 0


if __name__ == "__main__":
    sys.exit(main())

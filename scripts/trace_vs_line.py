#!/usr/bin/env python3
"""One bench process under rocprofv3 --kernel-trace: the headline kernel's per-launch
durations against the bench line that process printed (tooling).

    python scripts/trace_vs_line.py gpurun_out/<tag>/trace_200_10 gpurun_out/<tag>/trace_200_10.json \
        [--csv profiles/r04/final/trace_200_10_kernel_trace.csv]

The timed launches are launches 1 + warmup .. warmup + steps of the headline kernel
(crc32_uniform_lines_kernel<10>, G1) in the trace (launch 0 is the verification step; since
round 5 the line's cold window follows the timed steps); their mean is compared with the line's
roofline.kernel_ms (HIP events around the same launches).  --csv writes the condensed
per-launch series (launch, kernel, duration_us) of the whole process."""
import argparse
import csv
import glob
import json
import os
import statistics
import sys

HEADLINE = "crc32_uniform_lines_kernel<10>"


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("line")
    ap.add_argument("--csv")
    args = ap.parse_args()
    paths = glob.glob(os.path.join(args.trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not paths:
        print(f"no kernel trace under {args.trace_dir}", file=sys.stderr)
        return 1
    rows = []
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    line = None
    with open(args.line) as f:
        for ln in f:
            ln = ln.strip()
            if ln.startswith("{"):
                line = json.loads(ln)
    if line is None:
        print(f"no JSON line in {args.line}", file=sys.stderr)
        return 1
    steps, warmup = int(line["steps"]), int(line["warmup"])
    head = [(e - s) / 1000.0 for s, e, k in rows if HEADLINE in k]
    timed = head[1 + warmup:1 + warmup + steps]
    mean = statistics.fmean(timed)
    line_us = float(line["roofline"]["kernel_ms"]) * 1000.0
    out = {"trace_dir": args.trace_dir, "headline_launches": len(head), "timed": len(timed),
           "trace_mean_us": round(mean, 2), "trace_median_us": round(statistics.median(timed), 2),
           "trace_min_us": round(min(timed), 2), "trace_max_us": round(max(timed), 2),
           "line_kernel_us": round(line_us, 2), "line_over_trace": round(line_us / mean, 4)}
    print(json.dumps(out))
    if args.csv:
        with open(args.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["launch", "kernel", "duration_us"])
            for i, (s, e, k) in enumerate(rows):
                w.writerow([i, k[:90], round((e - s) / 1000.0, 2)])
    return 0


if __name__ == "__main__":
    sys.exit(main())

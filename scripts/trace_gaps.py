#!/usr/bin/env python3
"""Per-kernel mean duration and the median idle gap before each kernel, from a
rocprofv3 --kernel-trace output directory (CRC kernels only)."""
import csv
import re
import glob
import statistics
import sys
from collections import defaultdict

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "crc32" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur, gap = defaultdict(list), defaultdict(list)
for i, r in enumerate(rows):
    name = re.search(r"(crc32_\w+)", r["Kernel_Name"]).group(1)[:40]
    dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if i:
        gap[name].append((int(r["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"])) / 1e3)
for name in dur:
    g = statistics.median(gap[name]) if gap[name] else float("nan")
    print(f"   {name:40s} n={len(dur[name]):4d} mean {statistics.mean(dur[name]):8.1f} us  gap before (median) {g:6.2f} us")

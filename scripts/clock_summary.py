"""Effective shader clock per kernel from rocprofv3 GRBM_GUI_ACTIVE (sum over 8 XCDs)."""
import collections
import csv
import glob
import statistics
import sys

for d in sys.argv[1:]:
    by = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            t = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            by[r["Kernel_Name"][:48]].append((float(r["Counter_Value"]), t))
    for n, v in by.items():
        if len(v) < 3:
            continue
        print(f"{d.rsplit('/', 1)[-1]:28s} {n:48s} n={len(v):3d} dur_us={statistics.median(t for _, t in v) / 1e3:8.1f} "
              f"GHz={statistics.median(c / 8 / (t * 1e-9) / 1e9 for c, t in v if t > 0):.2f}")

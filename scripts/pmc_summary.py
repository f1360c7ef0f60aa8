"""Summarise rocprofv3 --pmc CSVs: per-kernel mean of each counter over dispatches."""
import csv
import glob
import os
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
paths = [p for root in sys.argv[1:] for p in glob.glob(os.path.join(root, "**", "*counter_collection*.csv"),
                                                           recursive=True)]
for path in paths:
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row.get("Kernel_Name", "?")
            if not any(f in name for f in os.environ.get("PMC_FILTER", "crc32").split(",")):
                continue
            key = (row.get("Dispatch_Id"), row.get("Counter_Name"))
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, ctrs in acc.items():
    print(name[:100])
    for c, vals in sorted(ctrs.items()):
        print(f"  {c:24s} mean={sum(vals)/len(vals):.6g}  n={len(vals)}")

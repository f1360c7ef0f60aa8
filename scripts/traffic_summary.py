"""Per-kernel FETCH_SIZE (gfx950-corrected) and mean duration from one profile round.

    python scripts/traffic_summary.py gpurun_out/<tag> [--write profiles/pmc_traffic.json]

Each entry records the hash of the kernel sources it was measured on (bench.py
kernel_source_hash); bench.py reports the traffic only while that hash still matches.

FETCH_SIZE is reported in KiB and, on gfx950, counts half the bytes of 16-B-per-lane
streaming reads (MI355X_MICROARCH.md, HBM section): bytes = FETCH_SIZE * 1024 * 2.
"""
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_source_hash  # noqa: E402

root = sys.argv[1]
src_hash = kernel_source_hash()
out = {}
for cfg in ("uniform", "ragged", "large", "frag"):
    fetch, dur = {}, {}
    for path in glob.glob(os.path.join(root, f"pmc_{cfg}", "**", "*counter_collection*.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            m = re.search(r"(crc32_\w+)", r["Kernel_Name"])
            if m and r["Counter_Name"] == "FETCH_SIZE":
                fetch.setdefault(m.group(1), []).append(float(r["Counter_Value"]))
    for path in glob.glob(os.path.join(root, f"prof_{cfg}", "**", "*kernel_stats*.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            m = re.search(r"(crc32_\w+)", r["Name"])
            if m:
                dur[m.group(1)] = float(r["AverageNs"])
    if not fetch:
        continue
    kernels = {}
    for k, v in fetch.items():
        kernels[k] = {"hbm_bytes_per_launch": sum(v) / len(v) * 1024 * 2, "launches": len(v),
                      "mean_duration_ns": dur.get(k)}
    main = max(kernels, key=lambda k: kernels[k]["hbm_bytes_per_launch"])
    out[cfg] = {"kernel": main, "hbm_bytes_per_launch": kernels[main]["hbm_bytes_per_launch"],
                "kernels": kernels, "source": os.path.relpath(root), "source_hash": src_hash}
# Range coder (compress kernel): memory-side read and write requests per launch (random
# 16-B node read-modify-writes, each its own request; bench.py range_roofline turns them
# into a request rate).
req, wreq, dur = [], [], None
for path in glob.glob(os.path.join(root, "pmc_range", "**", "*counter_collection*.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        if "range_coder_kernel<false>" in r["Kernel_Name"] and r["Counter_Name"].startswith("TCC_EA0_RDREQ"):
            req.append(float(r["Counter_Value"]))
        if "range_coder_kernel<false>" in r["Kernel_Name"] and r["Counter_Name"].startswith("TCC_EA0_WRREQ"):
            wreq.append(float(r["Counter_Value"]))
for path in glob.glob(os.path.join(root, "prof_range", "**", "*kernel_stats*.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        if "range_coder_kernel<false>" in r["Name"]:
            dur = float(r["AverageNs"])
if req:
    out["range"] = {"kernel": "range_coder_kernel<false>", "read_requests_per_launch": sum(req) / len(req),
                    "write_requests_per_launch": sum(wreq) / len(wreq) if wreq else None,
                    "launches": len(req), "mean_duration_ns": dur, "source": os.path.relpath(root),
                    "source_hash": src_hash}
print(json.dumps(out, indent=1))
if "--write" in sys.argv:
    with open(sys.argv[sys.argv.index("--write") + 1], "w") as f:
        json.dump(out, f, indent=1)

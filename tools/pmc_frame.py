#!/usr/bin/env python3
"""Sums one rocprofv3 --pmc pass's counters over the dispatches of the sample kernel and divides by
the number of dispatches: counters per frame of an A/B run (tools/ab_libs.py under rocprofv3).

    python tools/pmc_frame.py gpurun_out/pmc_x/   (directory rocprofv3 -d wrote)
"""
import csv
import glob
import json
import sys

rows = []
for f in glob.glob(sys.argv[1].rstrip("/") + "/**/*counter_collection.csv", recursive=True):
    rows += [r for r in csv.DictReader(open(f)) if "sample_kernel" in r["Kernel_Name"]]
sums, disp = {}, set()
for r in rows:
    sums[r["Counter_Name"]] = sums.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    disp.add(r["Dispatch_Id"])
n = max(1, len(disp))
print(json.dumps({"dispatches": len(disp), "per_frame": {k: v / n for k, v in sums.items()}}))

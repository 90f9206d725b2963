#!/usr/bin/env python3
"""Print the PMC counters of the dominant kernel from a tools/pmc_sets.sh run (sums over its
dispatches).   python tools/pmc_show.py gpurun_out/pmc_<tag> [kernel-substring]"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
key = sys.argv[2] if len(sys.argv) > 2 else "sample_kernel"
vals = defaultdict(float)
durs = defaultdict(float)
for f in glob.glob(os.path.join(root, "*", "pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            vals[r["Counter_Name"]] += float(r["Counter_Value"])
            durs[r["Counter_Name"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k in sorted(vals):
    print(f"{k:28s} {vals[k]:20.4e}   dur {durs[k]:.3f} ms")

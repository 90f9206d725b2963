#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>/ and profiles/pmc_traffic.json.

Reads gpurun_out/prof_<tag>/: the kernel-trace stats and the separate PMC passes (FETCH_SIZE,
WRITE_SIZE, SQ/GRBM counters) of the bench command, keeps the rows of the dominant kernel
(sample_kernel) and writes
  profiles/<tag>/kernel_stats.csv, profiles/<tag>/pmc_<counter>.csv (dominant-kernel rows only),
  profiles/<tag>/summary.json, profiles/pmc_traffic.json (read by bench.py's roofline.traffic).
HBM bytes per launch = (FETCH_SIZE + WRITE_SIZE) x 1024 (rocprofv3 reports KiB).  Per
MI355X_MICROARCH.md, FETCH_SIZE reads half the bytes of 16-B-per-lane streaming reads on gfx950 and
WRITE_SIZE is exact for 16-B-per-lane stores; this kernel's HBM reads are negligible (scene in
L2/scalar cache) and its stores are 8-B-per-lane f64 sample colors, which we calibrate against the
algorithmic byte count (24 B per sample) instead of assuming a correction.
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL_KEY = "sample_kernel"


def timed_kernel(name):
    """The dominant kernel's production instantiation: the last template argument of the sample
    kernels is kProf, and bench.py runs one instrumented (kProf = true) frame before timing."""
    return KERNEL_KEY in name and not name.split("(")[0].endswith("true>")


def rows(path):
    with open(path) as f:
        return [r for r in csv.DictReader(f) if timed_kernel(r.get("Kernel_Name", ""))]


def main(tag, workload):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    summary = {"tag": tag, "workload": workload, "counters": {}}
    st = os.path.join(src, "trace", "trace_kernel_stats.csv")
    if os.path.exists(st):
        shutil.copy(st, os.path.join(dst, "kernel_stats.csv"))
        with open(st) as f:
            for r in csv.DictReader(f):
                if timed_kernel(r["Name"]):
                    summary["trace"] = {"kernel": r["Name"], "calls": int(r["Calls"]),
                                        "avg_ms": float(r["AverageNs"]) / 1e6,
                                        "percent": float(r["Percentage"])}
    for d in sorted(glob.glob(os.path.join(src, "pmc_*"))):
        if not os.path.isdir(d):
            continue
        f = os.path.join(d, "pmc_counter_collection.csv")
        if not os.path.exists(f):
            continue
        rr = rows(f)
        if not rr:
            continue
        with open(os.path.join(dst, os.path.basename(d) + ".csv"), "w", newline="") as out:
            w = csv.DictWriter(out, fieldnames=list(rr[0].keys()))
            w.writeheader()
            w.writerows(rr)
        for r in rr:
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            summary["counters"][r["Counter_Name"]] = {"value": float(r["Counter_Value"]), "dur_ms": dur,
                                                     "vgpr": r.get("VGPR_Count"), "sgpr": r.get("SGPR_Count")}
    c = summary["counters"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fetch = c["FETCH_SIZE"]["value"] * 1024
        write = c["WRITE_SIZE"]["value"] * 1024
        summary["hbm_bytes_per_launch"] = fetch + write
        summary["fetch_bytes"] = fetch
        summary["write_bytes"] = write
        json.dump({"workload": workload, "tag": tag, "hbm_bytes_per_launch": fetch + write,
                   "fetch_bytes": fetch, "write_bytes": write,
                   "source": f"profiles/{tag}/pmc_FETCH_SIZE.csv, pmc_WRITE_SIZE.csv (rocprofv3 --pmc, "
                             "separate passes, KiB x 1024)"},
                  open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w"), indent=1)
    if "GRBM_GUI_ACTIVE" in c:
        g = c["GRBM_GUI_ACTIVE"]
        summary["effective_clock_GHz"] = g["value"] / 8 / (g["dur_ms"] / 1e3) / 1e9
    json.dump(summary, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else
         "final-render 1200x800 500spp depth50 (485 spheres)")

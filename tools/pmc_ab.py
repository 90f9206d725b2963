#!/usr/bin/env python3
"""Per-build PMC counters of a tools/pmc_ab.sh run: the sample kernel's dispatches in order, build
b's k-th launch being dispatch k * n_builds + b (tools/ab_libs.py runs the builds round-robin).

    python tools/pmc_ab.py gpurun_out/pmcab_<tag> <n_builds> [names...]
"""
import csv
import glob
import json
import os
import sys

src, nb = sys.argv[1], int(sys.argv[2])
names = sys.argv[3:] or [f"build{b}" for b in range(nb)]
per = {n: {} for n in names}
for f in sorted(glob.glob(os.path.join(src, "p*", "**", "pmc_counter_collection.csv"), recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if "sample_kernel" in r["Kernel_Name"] and "true, true" not in r["Kernel_Name"]]
    disp = sorted({int(r["Dispatch_Id"]) for r in rows})
    for r in rows:
        k = disp.index(int(r["Dispatch_Id"]))
        if k < nb:
            continue  # round 0: warm-up
        n = names[k % nb]
        c = r["Counter_Name"]
        per[n].setdefault(c, []).append(float(r["Counter_Value"]))
        per[n].setdefault("_dur_" + c, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
out = {}
for n, d in per.items():
    g = {c: sum(v) / len(v) for c, v in d.items() if not c.startswith("_dur_")}
    dur = {c[5:]: sum(v) / len(v) for c, v in d.items() if c.startswith("_dur_")}
    o = {"counters": g}
    if "GRBM_GUI_ACTIVE" in g:
        t = dur["GRBM_GUI_ACTIVE"]
        o["kernel_ms"] = t * 1e3
        o["clock_GHz"] = g["GRBM_GUI_ACTIVE"] / 8 / t / 1e9
        if "SQ_ACTIVE_INST_VALU" in g:
            o["valu_active_frac"] = 4 * g["SQ_ACTIVE_INST_VALU"] / (1024 * g["GRBM_GUI_ACTIVE"] / 8)
        if "SQ_THREAD_CYCLES_VALU" in g:
            o["lanes_active"] = g["SQ_THREAD_CYCLES_VALU"] / g["SQ_ACTIVE_INST_VALU"]
        if "SQ_WAVE_CYCLES" in g:
            w = g["SQ_WAVE_CYCLES"]
            o["wave_split"] = {k: g[k] / w for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY") if k in g}
    out[n] = o
print(json.dumps(out, indent=1))

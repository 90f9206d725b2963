#!/usr/bin/env python3
"""Per-variant PMC summary of tools/walk_occupancy.hip runs (rocprofv3 --pmc counter CSVs).

    python tools/occ_pmc.py gpurun_out/occ_pmc1 gpurun_out/occ_pmc2 [--out profiles/r03_occupancy/pmc.json]

For each walk_kernel instantiation (block size, stack entry, waves per SIMD) it sums every counter
over the variant's last dispatch and derives the wave-cycle split the DESIGN cites for the product
kernel: issuing (SQ_ACTIVE_INST_ANY), ready but not issued (SQ_WAIT_INST_ANY), parked on s_waitcnt
(SQ_WAIT_ANY), each / SQ_WAVE_CYCLES, plus VALU lanes per instruction
(SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU) and waves per SIMD (SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / 4
SIMDs x 256 CUs ... reported raw).
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def load(dirs):
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = row["Kernel_Name"]
                if "walk_kernel" not in k:
                    continue
                key = (k, int(row["Dispatch_Id"]), d)
                per[key][row["Counter_Name"]] += float(row["Counter_Value"])
                meta[key] = (int(row["Workgroup_Size"]), int(row["VGPR_Count"]), int(row["LDS_Block_Size"]),
                             int(row["Start_Timestamp"]), int(row["End_Timestamp"]))
    return per, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out")
    a = ap.parse_args()
    per, meta = load(a.dirs)
    last = {}  # (kernel, dir) -> the variant's last dispatch in that pass
    for (k, disp, d) in per:
        if (k, d) not in last or disp > last[(k, d)]:
            last[(k, d)] = disp
    res = defaultdict(dict)
    for (k, d), disp in last.items():
        m = re.search(r"walk_kernel<(\d+), (int|short), (\d+)>", k) or re.search(r"walk_kernelILi(\d+)E([is])Li(\d+)E", k)
        name = f"w{m.group(3)}_{'i32' if m.group(2) in ('i', 'int') else 'i16'}_B{m.group(1)}" if m else k
        c = per[(k, disp, d)]
        res[name].update(c)
        wg, vgpr, lds, t0, t1 = meta[(k, disp, d)]
        res[name].update({"block": wg, "vgpr": vgpr, "lds_bytes": lds, f"kernel_ms_{os.path.basename(d)}": (t1 - t0) / 1e6})
    out = {}
    for name, c in sorted(res.items()):
        wc = c.get("SQ_WAVE_CYCLES")
        row = {k: v for k, v in c.items()}
        if wc:
            for key, label in (("SQ_ACTIVE_INST_ANY", "issuing"), ("SQ_WAIT_INST_ANY", "ready_not_issued"),
                               ("SQ_WAIT_ANY", "waitcnt")):
                if key in c:
                    row[f"frac_{label}"] = round(c[key] / wc, 4)
        if c.get("SQ_ACTIVE_INST_VALU"):
            row["valu_lanes_per_inst"] = round(c.get("SQ_THREAD_CYCLES_VALU", 0) / c["SQ_ACTIVE_INST_VALU"], 2)
        if c.get("SQ_BUSY_CYCLES"):
            row["waves_resident_per_busy_cycle"] = round(c.get("SQ_WAVE_CYCLES", 0) / c["SQ_BUSY_CYCLES"], 2)
        out[name] = row
    print(json.dumps(out, indent=1))
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Per-region instruction table of the shipped parity kernel.

1. Compiles rt_kernel.hip with -DRTZIG_MARKS=1: the path loop emits an assembly comment ";@R <name>"
   where each region starts (finalise, handout, seed, idle, trips, scatter_finish, walk_setup,
   walk_inner, leaf, shade, store) and ";@R rare" on the slow paths behind wave-uniform tests.  The
   markers emit no instruction (the marked kernel's size is within 0.2% of the shipped one).
2. Splits sample_kernel_bvh<true,false,false> into basic blocks, builds the CFG and gives every block
   the region of its first marker, or else the region its predecessors end in (a merge after a rare
   block takes the non-rare side).
3. Counts each region's instructions by class (f64 VALU, 32-bit VALU, SALU, LDS, VMEM, s_nop) on its
   common path (rare blocks apart) and weights them with the wave-level executions of one
   instrumented frame (tools/kprofile.py --spp 100 -> stats[7..10], [26..31]):
     finalise, handout, idle, store: once per loop iteration; seed: seeding blocks; trips: the three
     unrolled trips' blocks, each once per trip (region static count x trips / 3);
     scatter_finish: per iteration; walk_setup: walks started; walk_inner: the inner-step loop block
     per inner step, its other blocks per leaf round + walk start; leaf: per leaf round, with the
     sqrt/root blocks per candidate block; shade: shading blocks; fin_work (the ring fold of a unit
   whose predecessor chunk is done): per finalisation, its 8x-unrolled loop 6 times.
   Every block of a region is assumed to run whenever the region runs (a wave executes each branch
   some lane takes), so the estimate is an upper bound per region; the sum is compared with the
   PMC count of VALU instructions.

    python tools/region_table.py <kprof.json> [--spp-scale 5] [--pmc profiles/r03/summary.json] [--out F]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "raytracing-with-zig_amd", "csrc", "rt_kernel.hip")
KERNEL = "_ZN3rtk17sample_kernel_bvhILb1ELb0ELb0E"
F64 = re.compile(r"^v_(add|mul|fma|fmac)_f64|^v_(rsq|rcp|sqrt)_f64|^v_div_(scale|fmas|fixup)_f64|^v_cmp\w*_f64|^v_(min|max)_f64|^v_cvt_f64")


def asm(extra):
    out = os.path.join(tempfile.mkdtemp(prefix="rtzig_regions_"), "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-x", "hip", "--offload-arch=gfx950",
                    "--cuda-device-only", "-S", SRC, "-o", out, *extra], check=True, capture_output=True)
    return open(out).read().split("\n")


def blocks_of(lines, kernel):
    st = next(i for i, l in enumerate(lines) if l.startswith(kernel))
    en = st
    while not lines[en].startswith(".Lfunc_end"):
        en += 1
    blocks, cur = [], {"name": "entry", "ins": [], "marks": []}
    blocks.append(cur)
    for l in lines[st + 1:en]:
        t = l.strip()
        m = re.match(r"^(\.LBB\d+_\d+):", t) or re.match(r"^; %(bb\.\d+):", t)
        if m:
            cur = {"name": m.group(1), "ins": [], "marks": []}
            blocks.append(cur)
            continue
        if t.startswith(";@R "):
            cur["marks"].append((len(cur["ins"]), t[4:].strip()))
            continue
        if not t or t.startswith(";") or t.startswith("."):
            continue
        cur["ins"].append(t.split(";")[0].strip())
    return blocks


def klass(i):
    op = i.split()[0]
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("v_"):
        return "valu_f64" if F64.match(op) else "valu_32"
    if op.startswith("s_"):
        return "smem" if op.startswith("s_load") or op.startswith("s_buffer") else "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def regions(blocks):
    idx = {b["name"]: k for k, b in enumerate(blocks)}
    succ = collections.defaultdict(list)
    pred = collections.defaultdict(list)
    for k, b in enumerate(blocks):
        ends = b["ins"][-1] if b["ins"] else ""
        for i in b["ins"]:
            m = re.match(r"s_cbranch_\w+\s+(\.LBB\d+_\d+)|s_branch\s+(\.LBB\d+_\d+)", i)
            if m:
                tgt = m.group(1) or m.group(2)
                if tgt in idx:
                    succ[k].append(idx[tgt])
        if not ends.startswith("s_branch") and not ends.startswith("s_endpgm") and k + 1 < len(blocks):
            succ[k].append(k + 1)
    for k, ss in succ.items():
        for t in ss:
            pred[t].append(k)
    entry_r = {0: "prologue"}
    exit_r = {}
    # region at a block's exit: its last marker, else its entry region
    for _ in range(50):
        changed = False
        for k, b in enumerate(blocks):
            if b["marks"] and b["marks"][0][0] == 0:
                er = b["marks"][0][1]
            else:
                cands = [exit_r[p] for p in pred[k] if p in exit_r]
                if not cands:
                    er = entry_r.get(k)
                else:
                    non_rare = [c for c in cands if c != "rare"]
                    er = collections.Counter(non_rare or cands).most_common(1)[0][0]
            if er is None:
                continue
            xr = b["marks"][-1][1] if b["marks"] else er
            if entry_r.get(k) != er or exit_r.get(k) != xr:
                entry_r[k], exit_r[k] = er, xr
                changed = True
        if not changed:
            break
    # per-instruction region: entry region until the first marker inside the block
    per = []
    for k, b in enumerate(blocks):
        marks = dict(b["marks"])
        r = entry_r.get(k, "?")
        for j, ins in enumerate(b["ins"]):
            if j in marks:
                r = marks[j]
            per.append((k, r, ins))
    return per, succ


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kprof")
    ap.add_argument("--spp-scale", type=float, default=5.0, help="frame spp / kprof spp (500 / 100)")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r03", "summary.json"))
    ap.add_argument("--out", default=None)
    ap.add_argument("-D", action="append", default=[], help="extra -D for the build (variants)")
    args = ap.parse_args()
    raw = json.load(open(args.kprof))["variants"]["bvh"]["raw"]
    sc = args.spp_scale
    n = {"iter": raw[26] * sc, "trips": raw[27] * sc, "seed": raw[28] * sc, "wstart": raw[29] * sc, "shade": raw[30] * sc,
         "inner": raw[7] * sc, "leaf": raw[8] * sc, "cand": raw[9] * sc, "root2": raw[10] * sc, "fin": raw[31] * sc}
    blocks = blocks_of(asm(["-DRTZIG_MARKS=1"] + ["-D" + d for d in args.D]), KERNEL)
    per, succ = regions(blocks)
    static = collections.defaultdict(lambda: collections.Counter())
    inner_loop = {k for k, ss in succ.items() if k in ss and any(klass(i) == "lds" for i in blocks[k]["ins"])
                  and any(i.startswith("v_pk_fma") for i in blocks[k]["ins"])}
    cand_blocks = {k for k, b in enumerate(blocks) if any(i.startswith("v_rsq_f64") for i in b["ins"])}
    # blocks on a cycle that stays inside walk_setup: the always-list loop for more than 4 spheres
    ws_blocks = {k for k, r, _ in per if r == "walk_setup"}
    def reach(a):
        seen, todo = set(), [a]
        while todo:
            x = todo.pop()
            for y in succ.get(x, []):
                if y in ws_blocks and y not in seen:
                    seen.add(y)
                    todo.append(y)
        return seen
    ws_loop = {k for k in ws_blocks if k in reach(k)}
    dyn = collections.defaultdict(lambda: collections.Counter())
    for k, r, ins in per:
        c = klass(ins)
        static[r][c] += 1
        if r in ("rare", "prologue", "epilogue", "?"):
            continue
        if r == "walk_inner":
            w = n["inner"] if k in inner_loop else n["leaf"] + n["wstart"]
        elif r == "leaf":
            w = n["cand"] - 0.0 if k in cand_blocks else n["leaf"]
        elif r == "walk_setup":
            # the always-list loop for more than 4 spheres (self-loop blocks) does not run on a scene
            # with <= 4 always-list spheres (config 4: the ground and three r = 1 spheres)
            w = 0 if k in ws_loop else n["wstart"]
        elif r == "trips":
            # the region holds kRuvTrips = 3 unrolled trips: each trip's blocks run once per trip
            w = n["trips"] / 3
        elif r == "seed":
            w = n["seed"]
        elif r == "shade":
            w = n["shade"]
        elif r == "fin_work":
            # the ring fold: loop blocks once per 8 of the unit's <= 48 samples, the rest once
            w = n["fin"] * (6 if k in succ.get(k, []) else 1)
        else:
            w = n["iter"]
        dyn[r][c] += w
    order = ["finalise", "fin_work", "handout", "seed", "idle", "trips", "scatter_finish", "walk_setup", "walk_inner", "leaf", "shade",
             "store", "rare", "prologue", "epilogue", "?"]
    rows = []
    tot = collections.Counter()
    for r in order:
        if r not in static:
            continue
        d = dyn.get(r, collections.Counter())
        tot.update(d)
        issue = 2 * d["valu_32"] + 4 * d["valu_f64"]
        rows.append({"region": r, "static": dict(static[r]),
                     "executions_per_frame": None if r in ("rare", "prologue", "?") else None,
                     "dyn_valu": d["valu_32"] + d["valu_f64"], "dyn_valu_f64": d["valu_f64"], "dyn_salu": d["salu"],
                     "dyn_lds": d["lds"], "dyn_nop": d["nop"], "valu_issue_cycles_est": issue})
    res = {"kernel": "sample_kernel_bvh<true,false,false> (-DRTZIG_MARKS=1 build: " + str(len(per)) + " instructions)",
           "counts_per_frame": n, "rows": rows,
           "total_est": {"valu": tot["valu_32"] + tot["valu_f64"], "valu_f64": tot["valu_f64"], "salu": tot["salu"],
                         "lds": tot["lds"], "nop": tot["nop"]}}
    try:
        pm = json.load(open(args.pmc))["counters_per_frame"]
        res["pmc"] = {"valu": pm["SQ_INSTS_VALU"], "salu": pm["SQ_INSTS_SALU"], "lds": pm["SQ_INSTS_LDS"],
                      "valu_f64": pm["SQ_INSTS_VALU_ADD_F64"] + pm["SQ_INSTS_VALU_MUL_F64"] + pm["SQ_INSTS_VALU_FMA_F64"],
                      "source": args.pmc}
    except (OSError, KeyError):
        pass
    txt = json.dumps(res, indent=1)
    if args.out:
        open(args.out, "w").write(txt)
    print(f"{'region':16s} {'static V/S/LDS/nop':>22s} {'dyn VALU':>10s} {'f64':>9s} {'SALU':>9s} {'LDS':>9s} {'issue cyc':>10s}")
    for r in rows:
        s = r["static"]
        print(f"{r['region']:16s} {s.get('valu_32', 0) + s.get('valu_f64', 0):5d}/{s.get('salu', 0):4d}/{s.get('lds', 0):3d}/{s.get('nop', 0):3d}"
              f"       {r['dyn_valu']:10.3g} {r['dyn_valu_f64']:9.3g} {r['dyn_salu']:9.3g} {r['dyn_lds']:9.3g} {r['valu_issue_cycles_est']:10.3g}")
    print("total est", res["total_est"], "pmc", res.get("pmc"))


if __name__ == "__main__":
    main()

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
4. Prices every VALU instruction with its MEASURED issue cost on the MI355X (round 5:
   tools/peak_rates.hip, event-timed over every CU, profiles/r05_peak/issue_rates.json via
   tools/issue_rates.py): ~4.15 SIMD cycles per wave64 instruction for f64, 64-bit integer, packed
   f32, min/max, compare, cndmask, alignbit, mul, mad, bfi ops; ~2.2 for the "fast" 32-bit ops
   (add/sub/and/or/xor/not/mov/lshr/ashr, f32 add/sub/mul/fma, bitop3) when they read at most two
   distinct VGPRs and no SGPR, 4.15 otherwise; 8.1 for v_rcp_f32; 16.1 for v_rsq/rcp_f64.  (Round 4's
   s_memtime table, profiles/r04_valu_rates/, was off by 1.4-2x: its waves were not all co-resident.)

    python tools/region_table.py <kprof.json> [--spp-scale 5] [--pmc profiles/r04/summary.json] [--out F]
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


RATES = os.path.join(ROOT, "profiles", "r05_peak", "issue_rates.json")
import sys  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import issue_rates  # noqa: E402


def load_rates(path=RATES):
    """opcode -> SIMD cycles per wave64 instruction at 4 waves/SIMD (measured)."""
    out = {}
    for r in json.load(open(path))["results"]:
        op = r["op"].split()[0]
        if "(pair)" in r["op"]:  # a cmp + cndmask pair, not one opcode
            continue
        if op == "v_cndmask_b32":  # VOP2 form reading a VCC nothing wrote: an artifact (README); use the e64 rate
            continue
        out[op] = r["simd_cycles_per_instr_4waves"]
    out["v_cndmask_b32"] = out.get("v_cndmask_b32_e64", 3.12)
    return out


def rate(op, rates):
    """Issue cost of one opcode: exact match (encoding suffix dropped), else a measured sibling."""
    base = re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)
    if base in rates:
        return rates[base]
    sib = [("v_fmac_f64", "v_fma_f64"), ("v_fmac_f32", "v_fma_f32"), ("v_cmp", "v_cmp_lt_f64" if "f64" in base or "64" in base else "v_cmp_gt_f32"),
           ("v_cndmask", "v_cndmask_b32_e64"), ("v_min3", "v_max3_f32"), ("v_max3", "v_max3_f32"), ("v_min_f64", "v_max_f64"),
           ("v_or_b32", "v_xor_b32"), ("v_sub_", "v_sub_u32"), ("v_subrev", "v_sub_u32"), ("v_addc", "v_add_co_u32"),
           ("v_sub_co", "v_add_co_u32"), ("v_readlane", "v_mbcnt_lo_u32_b32"), ("v_readfirstlane", "v_mbcnt_lo_u32_b32"),
           ("v_writelane", "v_mbcnt_lo_u32_b32"), ("v_mbcnt", "v_mbcnt_lo_u32_b32"), ("v_cvt", "v_cvt_f32_f64"),
           ("v_rsq", "v_rsq_f64"), ("v_sqrt_f64", "v_rsq_f64"), ("v_div_", "v_fma_f64"), ("v_frexp", "v_ldexp_f64"),
           ("v_mul_f64", "v_mul_f64"), ("v_pk_", "v_pk_fma_f32"), ("v_mov", "v_mov_b32"), ("v_lshl_or", "v_and_or_b32"),
           ("v_or3", "v_and_or_b32"), ("v_ashrrev_i64", "v_lshrrev_b64"), ("v_min_u32", "v_max_u32"), ("v_min_i32", "v_max_i32")]
    for pre, tgt in sib:
        if base.startswith(pre) and tgt in rates:
            return rates[tgt]
    return 3.12 if base.startswith("v_") else 0.0


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
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "r05", "summary.json"))
    ap.add_argument("--asm", default=None, help="price this assembly file instead of compiling (RTZIG_MARKS build)")
    ap.add_argument("--out", default=None)
    ap.add_argument("-D", action="append", default=[], help="extra -D for the build (variants)")
    args = ap.parse_args()
    raw = json.load(open(args.kprof))["variants"]["bvh"]["raw"]
    sc = args.spp_scale
    lanes_ok = len(raw) >= 64 and raw[32] > 0
    n = {"iter": raw[26] * sc, "trips": raw[27] * sc, "seed": raw[28] * sc, "wstart": raw[29] * sc, "shade": raw[30] * sc,
         "inner": raw[7] * sc, "leaf": raw[8] * sc, "cand": raw[9] * sc, "root2": raw[10] * sc, "fin": raw[31] * sc}
    # Weights (wave-level executions) and mean active lanes per region.  Round 6: the instrumented
    # kernel also counts, per block, the lanes that execute it (stats[32..63], tools/kprofile.py
    # "lanes"), and the candidate blocks, scatter finish and shading branches carry markers of their
    # own, so each sub-region is weighted by its own executions (round 5 weighted every block of a
    # region by the region's executions: an upper bound).
    W, LN = {}, {}
    full = 64.0
    for r in ("finalise", "fin_work", "handout", "idle", "scatter_finish"):
        LN[r] = full
    if lanes_ok:
        g = lambda k: raw[k] * sc  # noqa: E731
        acw, acl = [g(54 + q) for q in range(4)], [g(58 + q) for q in range(4)]
        lcw, lcl = g(9) - sum(acw), g(52) - sum(acl)
        ratio = lambda l, w: l / w if w else 0.0  # noqa: E731
        if len(raw) > 65 and raw[64]:  # seed-window builds: fills at 64 lanes, take passes at the fresh lanes
            W.update({"win_fill": g(64), "seed": g(65)})
            LN.update({"win_fill": full})
        W.update({"walk_setup": g(38), "always": n["wstart"], "cam_finish": g(36), "scat_finish": g(34),
                  "sky": g(42), "lam_metal": g(44), "dielectric": g(46), "store": g(48), "aroot2N": 0.0, "acandN": 0.0})
        for q in range(4):
            W[f"acand{q}"] = acw[q]
            LN[f"acand{q}"] = ratio(acl[q], acw[q])
        LN.update({"seed": ratio(g(32), g(65) if len(raw) > 65 and raw[64] else g(28)), "trips": ratio(g(33), g(27)), "cam_finish": ratio(g(37), g(36)),
                   "scat_finish": ratio(g(35), g(34)), "walk_setup": ratio(g(39), g(38)), "always": ratio(g(40), g(29)),
                   "walk_inner": ratio(g(3), g(7)), "walk_inner_other": ratio(g(39), g(38)), "leaf": ratio(g(51), g(8)),
                   "lcand": ratio(lcl, lcw), "aroot2": ratio(g(63), g(62)), "lroot2": ratio(g(53) - g(63), g(10) - g(62)),
                   "shade": ratio(g(41), g(30)), "sky": ratio(g(43), g(42)), "lam_metal": ratio(g(45), g(44)),
                   "dielectric": ratio(g(47), g(46)), "store": ratio(g(49), g(48))})
        n.update({"lcand_total": lcw, "aroot2_total": g(62), "lroot2_total": g(10) - g(62), "walk_any": g(38)})
    lines = open(args.asm).read().split("\n") if args.asm else asm(["-DRTZIG_MARKS=1"] + ["-D" + d for d in args.D])
    blocks = blocks_of(lines, KERNEL)
    per, succ = regions(blocks)
    # copies of an inlined candidate block: marker occurrences (entry + the re-entry after the root2
    # branch for the candidate markers), so each copy gets its share of the region's executions
    nmarks = collections.Counter(m for b in blocks for _, m in b["marks"])
    copies = {"lcand": nmarks["lcand"] / 2, "aroot2": nmarks["aroot2"], "lroot2": nmarks["lroot2"]}
    if lanes_ok:
        W["lcand"] = n["lcand_total"] / max(1.0, copies["lcand"])
        W["aroot2"] = n["aroot2_total"] / max(1.0, copies["aroot2"])
        W["lroot2"] = n["lroot2_total"] / max(1.0, copies["lroot2"])
    static = collections.defaultdict(lambda: collections.Counter())
    inner_loop = {k for k, ss in succ.items() if k in ss and any(klass(i) == "lds" for i in blocks[k]["ins"])
                  and any(i.startswith("v_pk_fma") for i in blocks[k]["ins"])}
    cand_blocks = {k for k, b in enumerate(blocks) if any(i.startswith("v_rsq_f64") for i in b["ins"])}
    # blocks on a cycle that stays inside walk_setup: the always-list loop for more than 4 spheres
    ws_blocks = {k for k, r, _ in per if r in ("walk_setup", "always")}
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
    table = issue_rates.load(RATES)
    cyc = collections.Counter()    # measured-rate VALU issue cycles per region
    lcyc = collections.Counter()   # ... x mean active lanes (lane-cycles)
    other = collections.Counter()  # the ops outside the PMC's f64 add/mul/fma and transcendental classes
    opcyc = collections.Counter()  # ... per opcode (whole kernel)
    opcnt = collections.Counter()  # executions per opcode
    regop = collections.Counter()  # issue cycles per (region, opcode)
    unpriced = collections.Counter()
    pen = collections.Counter()    # cycles fast-form ops lose to an SGPR or third VGPR source
    for k, r, ins in per:
        c = klass(ins)
        static[r][c] += 1
        if r in ("rare", "prologue", "epilogue", "?"):
            continue
        lanes = LN.get(r, full)
        if r == "walk_inner":
            if k in inner_loop:
                w = n["inner"]
            else:
                w = n["leaf"] + (n["walk_any"] if lanes_ok else n["wstart"])
                lanes = LN.get("walk_inner_other", full)
        elif r in W:
            w = 0 if (r in ("walk_setup", "always") and k in ws_loop) else W[r]
        elif r == "leaf":
            w = n["cand"] if (k in cand_blocks and not lanes_ok) else n["leaf"]
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
        op = ins.split()[0]
        if op.startswith("v_"):
            rt = issue_rates.price(ins, table)
            base = re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)
            if base not in table["opcodes"] and base not in table["fast_rule"]["opcodes"]:
                unpriced[op] += w
            cyc[r] += w * rt
            lcyc[r] += w * rt * lanes
            dyn[r]["valu_lanes"] += w * lanes
            opcyc[op] += w * rt
            opcnt[op] += w
            regop[(r, op)] += w * rt
            why = issue_rates.fast_penalty(ins, table)
            if why and r not in ("rare", "prologue", "epilogue", "?"):
                pen[(r, op, why)] += w * (rt - table["fast_rule"]["fast"])
            if not re.match(r"^v_(add|mul|fma|fmac)_f64|^v_(rsq|rcp|sqrt|exp|log|sin|cos)_f(32|64)", op):
                other["n"] += w
                other["cyc"] += w * rt
    order = ["finalise", "fin_work", "handout", "seed", "win_fill", "idle", "trips", "scatter_finish", "cam_finish", "scat_finish",
             "walk_setup", "always", "acand0", "acand1", "acand2", "acand3", "acandN", "aroot2", "aroot2N", "walk_inner",
             "leaf", "lcand", "lroot2", "shade", "sky", "lam_metal", "dielectric", "store", "rare", "prologue", "epilogue", "?"]
    rows = []
    tot = collections.Counter()
    for r in order:
        if r not in static:
            continue
        d = dyn.get(r, collections.Counter())
        tot.update(d)
        valu = d["valu_32"] + d["valu_f64"]
        rows.append({"region": r, "static": dict(static[r]),
                     "dyn_valu": valu, "dyn_valu_f64": d["valu_f64"], "dyn_salu": d["salu"],
                     "dyn_lds": d["lds"], "dyn_nop": d["nop"], "valu_issue_cycles_est": cyc.get(r, 0.0),
                     "mean_active_lanes": round(lcyc[r] / cyc[r], 2) if cyc.get(r) else None})
    tcyc = sum(cyc[r["region"]] for r in rows)
    tval = tot["valu_32"] + tot["valu_f64"]
    for r in rows:
        c = r["valu_issue_cycles_est"]
        r["valu_issue_share"] = round(c / tcyc, 4) if tcyc else None
        if r["mean_active_lanes"] is not None and tcyc:
            # issue cycles spent on lanes that do nothing: share x (1 - lanes / 64)
            r["wasted_issue_share"] = round(c / tcyc * (1 - r["mean_active_lanes"] / 64), 4)
    res = {"kernel": "sample_kernel_bvh<true,false,false> (-DRTZIG_MARKS=1 build: " + str(len(per)) + " instructions)",
           "counts_per_frame": n, "lane_counts": lanes_ok, "region_copies": copies, "rows": rows,
           "total_est": {"valu": tval, "valu_f64": tot["valu_f64"], "salu": tot["salu"],
                         "lds": tot["lds"], "nop": tot["nop"], "valu_issue_cycles": tcyc,
                         "valu_cycles_per_instruction": tcyc / tval if tval else None,
                         "other_valu_cycles_per_instruction": other["cyc"] / other["n"] if other["n"] else None,
                         "mean_active_lanes_cycle_weighted": round(sum(lcyc.values()) / tcyc, 2) if tcyc else None,
                         "mean_active_lanes_instruction_weighted": round(tot["valu_lanes"] / tval, 2) if tval else None,
                         "wasted_issue_share": round(1 - sum(lcyc.values()) / tcyc / 64, 4) if tcyc else None},
           "rates": {"source": os.path.relpath(RATES, ROOT),
                     "model": "SIMD cycles per wave64 instruction, event-timed per opcode and operand form (round 5)"},
           "top_opcodes_by_issue_cycles": [{"op": o, "cycles": c, "share": round(c / tcyc, 4),
                                            "mean_rate": round(c / opcnt[o], 3)}
                                           for o, c in opcyc.most_common(25)],
           "top_region_opcodes": [{"region": k[0], "op": k[1], "share": round(c / tcyc, 4)}
                                  for k, c in regop.most_common(40)],
           "unpriced_opcodes (sibling rate used)": {o: c for o, c in unpriced.most_common(10)},
           "fast_form_penalty": {"total_share": round(sum(pen.values()) / tcyc, 4) if tcyc else None,
                                 "top": [{"region": k[0], "op": k[1], "why": k[2], "share": round(c / tcyc, 4)}
                                         for k, c in pen.most_common(20)]}}
    try:
        pm = json.load(open(args.pmc))["counters_per_frame"]
        res["pmc"] = {"valu": pm["SQ_INSTS_VALU"], "salu": pm["SQ_INSTS_SALU"], "lds": pm["SQ_INSTS_LDS"],
                      "valu_f64": pm["SQ_INSTS_VALU_ADD_F64"] + pm["SQ_INSTS_VALU_MUL_F64"] + pm["SQ_INSTS_VALU_FMA_F64"],
                      "source": os.path.relpath(args.pmc, ROOT),
                      "estimate_over_pmc_valu": round(tval / pm["SQ_INSTS_VALU"], 3)}
        if pm.get("SQ_ACTIVE_INST_VALU"):
            res["pmc"]["valu_lanes_active_of_64"] = round(pm["SQ_THREAD_CYCLES_VALU"] / pm["SQ_ACTIVE_INST_VALU"], 2)
    except (OSError, KeyError):
        pass
    txt = json.dumps(res, indent=1)
    if args.out:
        open(args.out, "w").write(txt)
    print(f"{'region':16s} {'static V/S/LDS/nop':>22s} {'dyn VALU':>10s} {'f64':>9s} {'SALU':>9s} {'LDS':>9s} {'issue cyc':>10s} share lanes wasted")
    for r in rows:
        s = r["static"]
        print(f"{r['region']:16s} {s.get('valu_32', 0) + s.get('valu_f64', 0):5d}/{s.get('salu', 0):4d}/{s.get('lds', 0):3d}/{s.get('nop', 0):3d}"
              f"       {r['dyn_valu']:10.3g} {r['dyn_valu_f64']:9.3g} {r['dyn_salu']:9.3g} {r['dyn_lds']:9.3g} {r['valu_issue_cycles_est']:10.3g}"
              f" {r['valu_issue_share'] or 0:.3f} {r['mean_active_lanes'] or 0:5.1f} {r.get('wasted_issue_share', 0):.3f}")
    print("total est", res["total_est"], "pmc", res.get("pmc"))


if __name__ == "__main__":
    main()

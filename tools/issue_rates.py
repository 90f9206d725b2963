#!/usr/bin/env python3
"""Issue-cost table of the MI355X VALU from the event-timed harness (tools/peak_rates.hip), the
cost model the region table (tools/region_table.py) and the PMC summary (tools/pmc_summary.py) price
the sample kernel with.

Each rate is SIMD cycles per wave64 instruction = 1024 SIMDs x in-kernel clock x hipEvent time /
wave-instructions, at 8 waves per SIMD (the SIMD saturates from 2 waves on; 4 and 8 agree within
3%).  What the tables show (profiles/r05_peak/):

  * ~4.1 cycles: every f64 op (add, mul, fma, max, compare, ldexp, cvt), every 64-bit integer op
    (shifts, lshl_add_u64, mov_b64, u64 compares), 32-bit min/max/min3/max3/med3, compares,
    cndmask, alignbit, bfi, add3, or3, lshl_add, lshlrev_b32, mul_lo/hi, mad_u64_u32, mad/mul_u24,
    mbcnt, ffbh, bfrev, cvt, dpp moves, and the packed f32 ops (pk_fma/pk_add/pk_mul/pk_mov);
  * ~2.2 cycles ("fast"): v_add/sub/subrev_u32, and/or/xor/not_b32, mov_b32, lshrrev_b32,
    ashrrev_i32, add/sub/mul_f32, fma_f32 and bitop3 — but ONLY when the instruction reads at most
    two distinct VGPRs and no SGPR (inline constants and literals are free): v_fma_f32 (x, b, x) 2.5,
    (x, 0.5, b) 2.25, (x, b, c) 4.2, (x, s, b) 4.2; v_xor_b32 (s, x) 4.2; v_bitop3 (x, b, x) 2.3,
    (x, b, c) 4.05;
  * 8.1: v_rcp_f32 (and the other f32 transcendentals); 16.1: v_rsq_f64, v_rcp_f64.

Round 4's s_memtime table (profiles/r04_valu_rates/) assumed all 4 waves of each launch were
co-resident on their SIMD; per-wave s_memtime counts show they were not (e.g. v_fma_f64: 16 ticks per
wave-instruction at "8 waves" = 4 co-resident waves x 4.2 cycles), so its per-SIMD rates were too low
by 1.4-2x for most ops.

    python tools/issue_rates.py > profiles/r05_peak/issue_rates.json
"""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "profiles", "r05_peak", f) for f in ("peak_table.json", "peak_table_operands.json")]
FAST = ["v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_not_b32", "v_mov_b32",
        "v_lshrrev_b32", "v_ashrrev_i32", "v_add_f32", "v_sub_f32", "v_subrev_f32", "v_mul_f32", "v_fma_f32",
        "v_fmac_f32", "v_bitop3_b32"]
FAST_RATE = 2.2
SLOW_RATE = 4.15


def build():
    rates, forms = {}, {}
    for f in SRC:
        for r in json.load(open(f))["results"]:
            if r["waves_per_simd"] != 8:
                continue
            name = r["op"]
            cyc = round(r["simd_cycles_per_wave_instr_event"], 3)
            forms[name] = cyc
            op = name.split()[0]
            if "(" in name or "pair" in name or op in rates:
                continue  # operand variants and pairs: listed under "forms" only
            rates[op] = cyc
    return {"source": [os.path.relpath(f, ROOT) for f in SRC],
            "unit": "SIMD cycles per wave64 instruction (event-timed, 8 waves per SIMD)",
            "opcodes": rates, "forms": forms,
            "fast_rule": {"opcodes": FAST, "fast": FAST_RATE, "otherwise": SLOW_RATE,
                          "condition": "at most 2 distinct VGPR sources and no SGPR source (constants free)"},
            "default": SLOW_RATE}


def load(path=os.path.join(ROOT, "profiles", "r05_peak", "issue_rates.json")):
    return json.load(open(path))


_VREG = re.compile(r"\bv\[?(\d+)(?::(\d+))?\]?")
_SREG = re.compile(r"(?<![\w])(s\[?\d+|vcc|exec|m0|ttmp)")


def fast_penalty(ins, table):
    """Why a fast-form opcode issues at the slow rate: "sgpr" (an SGPR source), "3vgpr" (a third
    distinct VGPR source), or None (not a fast-form opcode, or issued fast)."""
    parts = ins.split(None, 1)
    op = re.sub(r"_(e32|e64|sdwa|dpp)$", "", parts[0])
    if op not in table["fast_rule"]["opcodes"]:
        return None
    ops = [o.strip() for o in (parts[1] if len(parts) > 1 else "").split(",")]
    srcs = ops[1:] if not op.startswith("v_fmac") else ops
    if op.startswith("v_add_co") or op.startswith("v_sub_co"):
        srcs = ops[2:]
    vregs, sgpr = set(), False
    for s in srcs:
        s = s.split()[0] if s else s
        if s.startswith("v") and not s.startswith("vcc"):
            vregs.add(s.lstrip("-|"))
        elif re.match(r"^-?\|?(s\[|s\d|vcc|exec|m0|ttmp)", s):
            sgpr = True
    return "sgpr" if sgpr else ("3vgpr" if len(vregs) > 2 else None)


def price(ins, table):
    """Issue cost of one assembly instruction (opcode + operands) under the table's model."""
    parts = ins.split(None, 1)
    op = re.sub(r"_(e32|e64|sdwa|dpp)$", "", parts[0])
    if op in table["fast_rule"]["opcodes"]:
        ops = [o.strip() for o in (parts[1] if len(parts) > 1 else "").split(",")]
        srcs = ops[1:] if not op.startswith("v_fmac") else ops  # fmac reads its destination
        if op.startswith("v_add_co") or op.startswith("v_sub_co"):
            srcs = ops[2:]
        vregs, sgpr = set(), False
        for s in srcs:
            s = s.split()[0] if s else s
            if s.startswith("v") and not s.startswith("vcc"):
                vregs.add(s.lstrip("-|"))
            elif re.match(r"^-?\|?(s\[|s\d|vcc|exec|m0|ttmp)", s):
                sgpr = True
        return table["fast_rule"]["fast"] if len(vregs) <= 2 and not sgpr else table["fast_rule"]["otherwise"]
    if op in table["opcodes"]:
        return table["opcodes"][op]
    sib = [("v_fmac_f64", "v_fma_f64"), ("v_cmp", "v_cmp_lt_f64" if "64" in op else "v_cmp_gt_f32"),
           ("v_cndmask", "v_cndmask_b32_e64"), ("v_min3", "v_max3_f32"), ("v_max3", "v_max3_f32"),
           ("v_min_f64", "v_max_f64"), ("v_addc", "v_add_co_u32"), ("v_sub_co", "v_add_co_u32"),
           ("v_subb", "v_add_co_u32"), ("v_readlane", "v_mbcnt_lo_u32_b32"), ("v_readfirstlane", "v_mbcnt_lo_u32_b32"),
           ("v_writelane", "v_mbcnt_lo_u32_b32"), ("v_mbcnt", "v_mbcnt_lo_u32_b32"), ("v_cvt", "v_cvt_f32_f64"),
           ("v_rsq_f32", "v_rcp_f32"), ("v_sqrt_f32", "v_rcp_f32"), ("v_rsq", "v_rsq_f64"), ("v_sqrt_f64", "v_rsq_f64"),
           ("v_div_", "v_fma_f64"), ("v_frexp", "v_ldexp_f64"), ("v_pk_", "v_pk_fma_f32"), ("v_mov_b64", "v_mov_b64"),
           ("v_lshl_or", "v_and_or_b32"), ("v_ashrrev_i64", "v_lshrrev_b64"), ("v_min_u32", "v_max_u32"),
           ("v_min_i32", "v_max_i32"), ("v_med3", "v_med3_f32")]
    for pre, tgt in sib:
        if op.startswith(pre) and tgt in table["opcodes"]:
            return table["opcodes"][tgt]
    return table["default"] if op.startswith("v_") else 0.0


if __name__ == "__main__":
    print(json.dumps(build(), indent=1))

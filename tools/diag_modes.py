#!/usr/bin/env python3
"""Render-mode diagnostics over library builds (verdict r03 item 1): each build renders the launch
shapes a rank of a multi-GPU job and the 1-GPU bench run — direct mode (rank 0's rows of 8, 500 spp;
with and without the instrumented kernel and its 32-word stats), ring mode (the whole frame), the
f32 fast mode and the list walk (chapter 9) — through the device-resident C ABI, waits with
rt_context_sync (which reports the kernel's sticky error word: a hand-off give-up, or, in
-DRTZIG_BOUNDS=1 builds, an index out of range), and compares every output with the first build's
bit for bit.  The first build's direct-mode rows are also checked against oracle B on one row.

    python tools/diag_modes.py raytracing-with-zig_amd/librtzig.so ab/bounds.so ab/bounds_w3.so ...

Prints one JSON object per (build, case) and a summary line; exit status 1 on any mismatch or error.
The mean printed is that of the output after the sync (round 3's uncommitted script printed 0.0: it
ran against the in-kernel fold's no-fold timing ablation, which writes no output).
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-with-zig_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtzig  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--spp", type=int, default=500)
ap.add_argument("--oracle-row", action="store_true", help="check row 0 of the first build's direct rows against oracle B")
args = ap.parse_args()

final = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=args.spp)
full100 = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=100)
ch9 = rtzig.chapter9_camera(width=400, spp=100)
# (name, camera, row0, row_step, n_rows, precision, profile)
CASES = [
    ("direct_rank0_of_8", final, 0, 8, 100, 0, False),
    ("direct_rank0_of_8_prof", final, 0, 8, 100, 0, True),
    ("direct_rank7_of_8", final, 7, 8, 99, 0, False),
    ("ring_full_100spp", full100, 0, 1, full100.height, 0, False),
    ("fast_direct_rank0_of_8", final, 0, 8, 100, 1, False),
    ("list_ch9", ch9, 0, 1, ch9.height, 0, False),
]


def bind(path):
    L = C.CDLL(os.path.abspath(path))
    vp = C.c_void_p
    for name, res, argt in [("rt_context_create", C.c_int, [C.c_int, C.POINTER(vp)]),
                            ("rt_context_destroy", C.c_int, [vp]),
                            ("rt_context_set_scene", C.c_int, [vp, C.POINTER(rtzig.RtSphere), C.c_size_t]),
                            ("rt_context_set_precision", C.c_int, [vp, C.c_int]),
                            ("rt_context_enable_profile", C.c_int, [vp, C.c_int]),
                            ("rt_context_sync", C.c_int, [vp]),
                            ("rt_kernel_name", C.c_char_p, [vp]),
                            ("rt_render_rows_async", C.c_int, [vp, C.POINTER(rtzig.RtCamera), C.c_uint32, C.c_uint32,
                                                               C.c_uint32, C.c_uint32, vp, vp, vp]),
                            ("rt_last_error", C.c_char_p, [])]:
        getattr(L, name).restype = res
        getattr(L, name).argtypes = argt
    return L


ref = {}
bad = 0
for li, path in enumerate(args.libs):
    L = bind(path)
    ctx = C.c_void_p()
    assert L.rt_context_create(0, C.byref(ctx)) == 0, L.rt_last_error()
    scene_of = None
    for name, cam, row0, step, n, prec, prof in CASES:
        if scene_of is not cam.scene:
            assert L.rt_context_set_scene(ctx, cam.scene.world, len(cam.scene.world)) == 0, L.rt_last_error()
            scene_of = cam.scene
        L.rt_context_set_precision(ctx, prec)
        L.rt_context_enable_profile(ctx, int(prof))
        out = torch.zeros((n, cam.width, 3), dtype=torch.float64, device="cuda:0")
        stats = torch.zeros(rtzig.abi.RT_PROFILE_STATS_WORDS, dtype=torch.int64, device="cuda:0")
        rec = {"lib": path, "case": name}
        rc = L.rt_render_rows_async(ctx, C.byref(cam.cam), 0, row0, step, n, C.c_void_p(out.data_ptr()),
                                    C.c_void_p(stats.data_ptr()), None)
        if rc == 0:
            rc = L.rt_context_sync(ctx)
        rec["kernel"] = L.rt_kernel_name(ctx).decode()
        if rc != 0:
            rec["error"] = f"rc {rc}: {L.rt_last_error().decode()}"
            bad += 1
        else:
            img = out.cpu().numpy()
            st = stats.cpu().tolist()
            rec.update({"mean": float(img.mean()), "rays": st[0], "samples": st[1],
                        "samples_expected": n * cam.width * cam.cam.samples_per_pixel})
            if st[1] != rec["samples_expected"]:
                rec["error"] = "sample count"
                bad += 1
            if li == 0:
                ref[name] = img
            elif not np.array_equal(img, ref[name]):
                rec["error"] = f"differs from {args.libs[0]} in {int((img != ref[name]).any(-1).sum())} pixels"
                bad += 1
            else:
                rec["bit_exact_vs_first"] = True
        L.rt_context_enable_profile(ctx, 0)
        print(json.dumps(rec), flush=True)
    L.rt_context_destroy(ctx)
if args.oracle_row and "direct_rank0_of_8" in ref:
    from oracle_lib import Oracle
    row, _ = Oracle().render_b(final.cam, final.scene.world, row0=0, row_step=1, n_rows=1, threads=1)
    ok = bool(np.array_equal(ref["direct_rank0_of_8"][:1], row))
    print(json.dumps({"oracle_b_row0_bit_exact": ok}), flush=True)
    bad += 0 if ok else 1
print(json.dumps({"summary": "ok" if bad == 0 else f"{bad} failures", "libs": args.libs}), flush=True)
sys.exit(1 if bad else 0)

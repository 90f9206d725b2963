#!/usr/bin/env python3
"""Fixed per-launch overhead of the sample kernel: times one row set at several spp and fits
t(spp) = a + b * spp (HIP events, median of --reps); a = ramp + drain tail + (direct mode) reduce.

    python tools/overhead_fit.py --row-step 8 --spp 125 250 500
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-with-zig_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtzig  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--row-step", type=int, default=8)
ap.add_argument("--spp", type=int, nargs="+", default=[125, 250, 500])
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--bounce-max", type=int, default=50, help="diagnostics only (changes the image)")
args = ap.parse_args()

r = rtzig.DeviceRenderer(0)
res = {"row_step": args.row_step, "bounce_max": args.bounce_max, "points": {}}
for spp in args.spp:
    cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=spp, bounce_max=args.bounce_max)
    r.set_scene(cam.scene.world)
    r.enable_timing(True)
    n_rows = (cam.height + args.row_step - 1) // args.row_step
    out = torch.empty((n_rows, cam.width, 3), dtype=torch.float64, device="cuda:0")
    r.render_rows_async(cam.cam, out.data_ptr(), row0=0, row_step=args.row_step, n_rows=n_rows)
    ks, rs = [], []
    for _ in range(args.reps):
        r.render_rows_async(cam.cam, out.data_ptr(), row0=0, row_step=args.row_step, n_rows=n_rows)
        k, red = r.kernel_times()
        ks.append(k)
        rs.append(red)
    res["points"][spp] = {"sample_ms": statistics.median(ks), "reduce_ms": statistics.median(rs),
                          "kernel": r.kernel_name()}
x = np.array(args.spp, dtype=float)
y = np.array([res["points"][s]["sample_ms"] for s in args.spp])
b, a = np.polyfit(x, y, 1)
res["fit_sample_kernel"] = {"intercept_ms": round(float(a), 4), "ms_per_spp": round(float(b), 5)}
print(json.dumps(res))

#!/usr/bin/env python3
"""Msamples/s of the parity kernel on every BASELINE.json GPU config (one MI355X, sample + reduce
kernels by HIP events, inputs resident).  Config 5 (3840x2160, 10000 spp) runs at a bounded spp
(--stress-spp) so the run stays short; the rate is per sample, and at 10000 spp only the number
of units grows with spp (one launch per frame, in-kernel ordered accumulation).

    python tools/configs_bench.py [--stress-spp 200] [--out profiles/r02_configs.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-with-zig_amd"))
import torch  # noqa: E402

import rtzig  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--stress-spp", type=int, default=200)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--out", default=None)
args = ap.parse_args()

configs = [
    ("2: chapter9 two-sphere Lambertian", rtzig.chapter9_camera(width=400, spp=100)),
    ("3: chapter13 three-material + defocus", rtzig.chapter13_camera(width=1200, spp=500)),
    ("4: final random-sphere scene", rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=500)),
    ("4': final scene at the reference's 16:9", rtzig.final_scene_camera(width=1200, aspect_ratio=16 / 9, spp=500)),
    (f"5: final scene 3840x2160 (spp {args.stress_spp} of 10000)",
     rtzig.final_scene_camera(width=3840, aspect_ratio=16 / 9, spp=args.stress_spp)),
]
res = {"device": torch.cuda.get_device_name(0), "configs": {}}
for name, cam in configs:
    H, W = cam.height, cam.width
    spp = cam.cam.samples_per_pixel
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    out = torch.empty((H, W, 3), dtype=torch.float64, device="cuda:0")
    st = torch.zeros(2, dtype=torch.int64, device="cuda:0")
    r.render_rows_async(cam.cam, out.data_ptr())  # warm-up (BVH, workspace)
    torch.cuda.synchronize()
    r.enable_timing(True)
    for _ in range(args.reps):
        r.render_rows_async(cam.cam, out.data_ptr(), d_stats_ptr=st.data_ptr())
    s_ms, r_ms, launches = r.kernel_times_total()
    torch.cuda.synchronize()
    ms = (s_ms + r_ms) / args.reps
    rays = int(st[0]) // args.reps
    res["configs"][name] = {"width": W, "height": H, "spp": spp, "spheres": len(cam.scene.world),
                            "kernel": r.kernel_name(), "sample_launches_per_frame": launches // args.reps,
                            "ms_per_frame": round(ms, 3), "Msamples_s": round(W * H * spp / ms / 1e3, 1),
                            "rays_per_sample": round(rays / (W * H * spp), 4)}
    print(name, res["configs"][name], file=sys.stderr, flush=True)
    r.sync()  # raises if a wave reported a hand-off timeout
    r.close()
print(json.dumps(res))
if args.out:
    json.dump(res, open(args.out, "w"), indent=1)

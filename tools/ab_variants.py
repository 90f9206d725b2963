#!/usr/bin/env python3
"""A/B the sample-kernel variants IN ONE PROCESS, interleaved rounds (cdna guide rule 24).

    python tools/ab_variants.py --spp 100 --rounds 5                 # the walk variants
    python tools/ab_variants.py --env RTZIG_UNIT_MODE --variants "ring direct"
Each variant is selected through the --env variable (default RTZIG_KERNEL), set both while the
variant's scene is built and at every launch.  Prints one JSON line with
per-variant median/min sample-kernel ms (HIP events) and Msamples/s.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-with-zig_amd"))
import torch  # noqa: E402

import rtzig  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--width", type=int, default=1200)
ap.add_argument("--aspect", type=float, default=1.5)
ap.add_argument("--spp", type=int, default=100)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--env", default="RTZIG_KERNEL")
ap.add_argument("--variants", default=os.environ.get("RTZIG_VARIANTS", "bvh smem_u4 lds_u4"))
ap.add_argument("--row-step", type=int, default=1,
                help="render rank 0's interleaved row set of an N-rank job (rows 0, N, 2N, ...)")
args = ap.parse_args()

cam = rtzig.final_scene_camera(width=args.width, aspect_ratio=args.aspect, spp=args.spp)
H, W = cam.height, cam.width
R = (H + args.row_step - 1) // args.row_step
out = torch.empty((R, W, 3), dtype=torch.float64, device="cuda:0")
variants = args.variants.split()
# one renderer per variant, with the variable set while the scene (and its BVH) is built too, so
# the tool also A/Bs build-time knobs such as RTZIG_BVH_ALWAYS_AREA
renderers = {}
for v in variants:
    os.environ[args.env] = v
    renderers[v] = rtzig.DeviceRenderer(0)
    renderers[v].set_scene(cam.scene.world)
    renderers[v].enable_timing(True)
times = {v: [] for v in variants}
names = {}
ref = None
for rnd in range(args.rounds + 1):
    for v in variants:
        os.environ[args.env] = v
        r = renderers[v]
        r.render_rows_async(cam.cam, out.data_ptr(), row0=0, row_step=args.row_step, n_rows=R)
        torch.cuda.synchronize()
        sm, rm = r.kernel_times()
        sm += rm  # direct mode's reduce pass belongs to the frame
        names[v] = r.kernel_name()
        img = out.cpu()
        if ref is None:
            ref = img
        assert torch.equal(img, ref), f"variant {v} output differs"
        if rnd > 0:  # round 0 = warmup
            times[v].append(sm)
res = {}
for v in variants:
    med = statistics.median(times[v])
    res[v] = {"kernel": names[v], "median_ms": round(med, 3), "min_ms": round(min(times[v]), 3),
              "Msamples_s": round(W * R * args.spp / med / 1e3, 1),
              "workspace_bytes": renderers[v].workspace_bytes()}
print(json.dumps({"config": f"{W}x{H} {args.spp}spp, rows 0::{args.row_step} ({R} rows)", "env": args.env, "results": res}))

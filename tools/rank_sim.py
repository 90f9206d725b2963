#!/usr/bin/env python3
"""Strong-scaling rehearsal on one GPU: the sample + reduce kernel time of rank 0's row set
(rows 0, N, 2N, ...) for N = 1, 2, 4, 8, i.e. the per-rank work of `bench.py --gpus N`, so that
the scaling efficiency the 8-GPU driver will measure can be predicted without 8 GPUs.

    python tools/rank_sim.py --spp 500 --reps 3
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-with-zig_amd"))
import torch  # noqa: E402

import rtzig  # noqa: E402
from rtzig import dist as rdist  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=500)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--lib", default=None, help="alternative librtzig build (A/B)")
args = ap.parse_args()

cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=args.spp)
H, W = cam.height, cam.width
r = rtzig.DeviceRenderer(0)
r.set_scene(cam.scene.world)
r.enable_timing(True)
res = {"config": f"{W}x{H} {args.spp}spp", "ranks": {}}
base = None
for n in (1, 2, 4, 8):
    row0, step, n_rows = rdist.rank_rows(H, 0, n)
    out = torch.empty((n_rows, W, 3), dtype=torch.float64, device="cuda:0")
    r.render_rows_async(cam.cam, out.data_ptr(), row0=row0, row_step=step, n_rows=n_rows)
    torch.cuda.synchronize()
    ks = []
    for _ in range(args.reps):
        r.render_rows_async(cam.cam, out.data_ptr(), row0=row0, row_step=step, n_rows=n_rows)
        a, b = r.kernel_times()
        ks.append(a + b)
        red = b
    k = min(ks)
    # back-to-back frames without a host sync between them (GPU never idles): wall time per frame
    import time
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps * 2):
        r.render_rows_async(cam.cam, out.data_ptr(), row0=row0, row_step=step, n_rows=n_rows)
    torch.cuda.synchronize()
    bb = (time.perf_counter() - t0) * 1e3 / (args.reps * 2)
    base = base or k
    res["ranks"][n] = {"rows": n_rows, "kernel_ms": round(k, 3), "reduce_ms": round(red, 3), "back_to_back_ms": round(bb, 3),
                       "predicted_speedup": round(base / k, 3), "efficiency": round(base / k / n, 3)}
print(json.dumps(res))

# two-deep frame pipelining: two contexts (own workspace + queue), two streams, frames alternate
if os.environ.get("RANK_SIM_PIPE"):
    import time
    r2 = rtzig.DeviceRenderer(0)
    r2.set_scene(cam.scene.world)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    pipe = {}
    for n in (1, 2, 4, 8):
        row0, step, n_rows = rdist.rank_rows(H, 0, n)
        outs = [torch.empty((n_rows, W, 3), dtype=torch.float64, device="cuda:0") for _ in range(2)]
        for rr, ss, o in ((r, s1, outs[0]), (r2, s2, outs[1])):
            rr.render_rows_async(cam.cam, o.data_ptr(), row0=row0, row_step=step, n_rows=n_rows,
                                 stream_ptr=ss.cuda_stream)
        torch.cuda.synchronize()
        frames = args.reps * 4
        t0 = time.perf_counter()
        for f in range(frames):
            rr, ss, o = (r, s1, outs[0]) if f % 2 == 0 else (r2, s2, outs[1])
            rr.render_rows_async(cam.cam, o.data_ptr(), row0=row0, row_step=step, n_rows=n_rows,
                                 stream_ptr=ss.cuda_stream)
        torch.cuda.synchronize()
        pipe[n] = round((time.perf_counter() - t0) * 1e3 / frames, 3)
    print(json.dumps({"pipelined_ms_per_frame": pipe}))

# per-rank kernel times at N = 8 (the bench takes the max over ranks)
if os.environ.get("RANK_SIM_ALL"):
    per = {}
    for rank in range(8):
        row0, step, n_rows = rdist.rank_rows(H, rank, 8)
        out = torch.empty((n_rows, W, 3), dtype=torch.float64, device="cuda:0")
        ks = []
        for _ in range(args.reps + 1):
            r.render_rows_async(cam.cam, out.data_ptr(), row0=row0, row_step=step, n_rows=n_rows)
            a, b = r.kernel_times()
            ks.append(a + b)
        per[rank] = round(min(ks[1:]), 3)
    print(json.dumps({"n8_rank_ms": per, "max_over_min": round(max(per.values()) / min(per.values()), 4)}))

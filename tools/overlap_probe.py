#!/usr/bin/env python3
"""Probe: K frames back to back on one context (serial) against frames alternating between two
contexts on two HIP streams (frame k+1 starts on the CUs frame k's drain tail frees).  Wall time
per frame, one GPU; the row set of one rank of an N-rank job (--row-step N).

    python tools/overlap_probe.py --row-step 8 --frames 20
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-with-zig_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rtzig  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--row-step", type=int, default=8)
ap.add_argument("--spp", type=int, default=500)
ap.add_argument("--frames", type=int, default=20)
args = ap.parse_args()

cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=args.spp)
n_rows = (cam.height + args.row_step - 1) // args.row_step
ctxs = [rtzig.DeviceRenderer(0) for _ in range(2)]
for c in ctxs:
    c.set_scene(cam.scene.world)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
outs = [torch.empty((n_rows, cam.width, 3), dtype=torch.float64, device="cuda:0") for _ in range(2)]
for k in range(2):  # warm-up both (tree, workspace)
    ctxs[k].render_rows_async(cam.cam, outs[k].data_ptr(), row0=0, row_step=args.row_step, n_rows=n_rows,
                              stream_ptr=streams[k].cuda_stream)
torch.cuda.synchronize()


def run(n_ctx):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for f in range(args.frames):
        k = f % n_ctx
        ctxs[k].render_rows_async(cam.cam, outs[k].data_ptr(), row0=0, row_step=args.row_step, n_rows=n_rows,
                                  stream_ptr=streams[k].cuda_stream)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / args.frames


res = {"row_step": args.row_step, "spp": args.spp, "frames": args.frames}
res["serial_ms"] = [round(run(1), 3) for _ in range(3)]
res["two_contexts_ms"] = [round(run(2), 3) for _ in range(3)]
a, b = np.median(res["serial_ms"]), np.median(res["two_contexts_ms"])
res["gain"] = round(1 - b / a, 4)
a_img, b_img = outs[0].cpu().numpy(), outs[1].cpu().numpy()
res["images_equal"] = bool(np.array_equal(a_img, b_img))
print(json.dumps(res))

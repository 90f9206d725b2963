#!/usr/bin/env python3
"""Frames in flight: one context and one stream (frames back to back) against two contexts on two
streams (frame k+1's persistent grid takes the CUs frame k's tail waves free).

    python tools/inflight_ab.py [--steps 10] [--rounds 3] [--ranks 1,8] [--spp 500]

For each row set (--ranks N: rank 0's rows j = 0 mod N of the config-4 frame) it times K frames with
1 and with 2 frames in flight, alternating, and checks that both give the same image bits.  One JSON
line per (N, inflight, round) and a summary line.
"""
import argparse
import json
import os
import sys
import time

# HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default) round-robin; two contexts'
# upload streams, the null stream and the two render streams are five, and two streams sharing a
# queue serialise.  Set before HIP initialises.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-with-zig_amd"))
import rtzig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ranks", default="1,8")
    ap.add_argument("--spp", type=int, default=500)
    args = ap.parse_args()
    cam = rtzig.final_scene_camera(spp=args.spp)
    H, W = cam.height, cam.width
    rens = [rtzig.DeviceRenderer(0) for _ in range(2)]
    for r in rens:
        r.set_scene(cam.scene.world)
    streams = [torch.cuda.Stream() for _ in range(2)]
    summary = {}
    for N in [int(x) for x in args.ranks.split(",")]:
        rows = (H + N - 1) // N
        outs = [torch.zeros((rows, W, 3), dtype=torch.float64, device="cuda") for _ in range(2)]

        def frame(k, inflight):
            b = k % inflight
            rens[b].render_rows_async(cam.cam, outs[b].data_ptr(), row0=0, row_step=N, n_rows=rows,
                                      stream_ptr=streams[b].cuda_stream)

        for inflight in (1, 2):  # warm both contexts (tree training, workspace)
            for k in range(2):
                frame(k, inflight)
        torch.cuda.synchronize()
        ref = outs[0].clone()
        res = {1: [], 2: []}
        for rd in range(args.rounds):
            for inflight in (1, 2):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(args.steps):
                    frame(k, inflight)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / args.steps * 1e3
                same = all(torch.equal(outs[b], ref) for b in range(inflight))
                res[inflight].append(ms)
                print(json.dumps({"N": N, "rows": rows, "inflight": inflight, "round": rd, "ms_per_frame": round(ms, 4),
                                  "bit_exact": same}), flush=True)
                if not same:
                    raise SystemExit("inflight_ab: images differ")
        med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        summary[N] = {"rows": rows, "ms_inflight1": round(med[1], 4), "ms_inflight2": round(med[2], 4),
                      "speedup": round(med[1] / med[2], 4)}
    for r in rens:
        r.sync()
        r.close()
    print(json.dumps({"summary": summary, "steps": args.steps, "rounds": args.rounds, "spp": args.spp}), flush=True)


if __name__ == "__main__":
    main()

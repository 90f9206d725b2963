#!/usr/bin/env python3
"""Direct mode's reduce pass on the output stream (rt_render_rows_async_split) against the plain call,
in bench.py's N > 1 frame pipeline, emulated on one GPU for rank 0's rows of an N-rank job.

Both modes run K frames into two row buffers on a render stream, each frame's output consumed on a
second ("collective") stream that waits for it, as bench.py does around dist.gather:
  plain: sample kernel + reduce pass on the render stream; the collective stream waits for the frame;
  split: sample kernel on the render stream, reduce pass on the collective stream (two per-sample
         buffers in turn), so frame k's pass overlaps frame k+1's sample kernel.
Outputs must be bit-identical.  One JSON line per (row step, mode, round), then a summary.

    python tools/split_ab.py --steps 10 --rounds 3 --row-steps 8,4
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-with-zig_amd"))
import rtzig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--row-steps", default="8,4")
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--render-priority", type=int, default=0,
                    help="torch stream priority of the render stream (-1: high, ahead of the reduce pass)")
    args = ap.parse_args()
    cam = rtzig.final_scene_camera(spp=args.spp)
    H, W = cam.height, cam.width
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    render = torch.cuda.Stream(priority=args.render_priority)
    coll = torch.cuda.Stream()
    summary = {}
    for N in [int(x) for x in args.row_steps.split(",")]:
        rows = (H + N - 1) // N
        outs = [torch.zeros((rows, W, 3), dtype=torch.float64, device="cuda") for _ in range(2)]
        done = [torch.cuda.Event() for _ in range(2)]
        freed = [None, None]

        pend = [False]

        def frame(k, split):
            b = k % 2
            if split == "deferred":
                # kernel k folds frame k-1 into buffer (k-1) % 2, last read by frame k-3's consumer
                pb = (k - 1) % 2
                if pend[0] and freed[pb] is not None:
                    render.wait_event(freed[pb])
                r.render_rows_async(cam.cam, outs[b].data_ptr(), row0=0, row_step=N, n_rows=rows,
                                    stream_ptr=render.cuda_stream, out_stream_ptr=coll.cuda_stream, deferred=True)
                if pend[0]:
                    freed[pb] = torch.cuda.Event()
                    freed[pb].record(coll)  # frame k-1's output is complete on coll here
                pend[0] = r.fold_pending()
                if not pend[0]:
                    freed[b] = torch.cuda.Event()
                    freed[b].record(coll)
                return
            if freed[b] is not None:
                render.wait_event(freed[b])
            if split:
                r.render_rows_async(cam.cam, outs[b].data_ptr(), row0=0, row_step=N, n_rows=rows,
                                    stream_ptr=render.cuda_stream, out_stream_ptr=coll.cuda_stream)
            else:
                r.render_rows_async(cam.cam, outs[b].data_ptr(), row0=0, row_step=N, n_rows=rows,
                                    stream_ptr=render.cuda_stream)
                done[b].record(render)
                coll.wait_event(done[b])
            freed[b] = torch.cuda.Event()
            freed[b].record(coll)  # the consumer of this buffer (bench: dist.gather) has run

        modes = (False, True, "deferred")

        def finish(split):
            if split == "deferred":
                r.flush()  # the last frame's pass, on coll
                pend[0] = False
                freed[0] = freed[1] = None

        for split in modes:  # warm (tree, workspace of every mode)
            for k in range(2):
                frame(k, split)
            finish(split)
        torch.cuda.synchronize()
        ref = outs[0].clone()
        res = {m: [] for m in modes}
        for rd in range(args.rounds):
            for split in modes:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(args.steps):
                    frame(k, split)
                finish(split)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / args.steps * 1e3
                same = all(torch.equal(o, ref) for o in outs)
                res[split].append(ms)
                print(json.dumps({"row_step": N, "rows": rows, "split": split, "round": rd, "ms_per_frame": round(ms, 4),
                                  "bit_exact": same, "kernel": r.kernel_name()}), flush=True)
                if not same:
                    raise SystemExit("split_ab: outputs differ")
        med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        summary[N] = {"rows": rows, "ms_plain": round(med[False], 4), "ms_split": round(med[True], 4),
                      "ms_deferred": round(med["deferred"], 4), "speedup": round(med[False] / med[True], 4),
                      "speedup_deferred": round(med[False] / med["deferred"], 4)}
    r.sync()
    r.close()
    print(json.dumps({"summary": summary, "steps": args.steps, "rounds": args.rounds, "spp": args.spp,
                      "render_priority": args.render_priority}), flush=True)


if __name__ == "__main__":
    main()

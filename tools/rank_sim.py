#!/usr/bin/env python3
"""Strong-scaling rehearsal on one GPU: what `bench.py --gpus N` does per frame on each rank, for
N = 1, 2, 4, 8, so the efficiency the 8-GPU driver will measure can be predicted without 8 GPUs.

Per N:
  * kernel: the HIP-event time of the sample kernel (+ direct mode's reduce pass) for EVERY rank's
    interleaved row set (rows r, r+N, ...)
    — the bench takes the max over ranks, so the prediction does too;
  * gather: rank 0's share of `rdist.gather_image` — the assemble copy (measured here on rank 0's
    buffer of N x R x W x 3 f64) plus the transfer of the N-1 peers' rows over xGMI (modelled: each
    peer sends R*W*24 B over its own link at LINK_GBPS, concurrently, plus a fixed collective
    latency LAUNCH_US; both stated in the output, neither measurable with one GPU).
Prediction: frame(N) = max_rank kernel + gather; efficiency = frame(1) / (N * frame(N)).  Also
reported: the frame with the gather hidden behind the next render (bench.py's pipeline), max(kernel,
gather).

    python tools/rank_sim.py --spp 500 --reps 3
    python tools/rank_sim.py --width 3840 --aspect 1.7777777777777777 --spp 10000 --ns 1 8 --reps 1   # config 5
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-with-zig_amd"))
import torch  # noqa: E402

import rtzig  # noqa: E402
from rtzig import dist as rdist  # noqa: E402

LINK_GBPS = 64.0   # conservative per-direction xGMI rate of one peer link (the ~153 GB/s figure is bidirectional)
LAUNCH_US = 50.0   # fixed cost of one RCCL gather launch + completion (assumed)

ap = argparse.ArgumentParser()
ap.add_argument("--spp", type=int, default=500)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--width", type=int, default=1200)
ap.add_argument("--aspect", type=float, default=1.5)
ap.add_argument("--ns", type=int, nargs="+", default=[1, 2, 4, 8])
ap.add_argument("--pipe-frames", type=int, default=0,
                help="also time each rank's rows in bench.py's frame pipeline (two row buffers, render "
                     "stream, output completed on a second stream: rt_render_rows_async_split), this many "
                     "frames, wall clock per frame")
ap.add_argument("--row-buffers", type=int, default=3, help="row buffers the pipeline rotates through (bench.py)")
ap.add_argument("--pipe-mode", choices=["plain", "split", "deferred"], default="deferred",
                help="the pipeline's render call (bench.py --pipeline)")
args = ap.parse_args()

cam = rtzig.final_scene_camera(width=args.width, aspect_ratio=args.aspect, spp=args.spp)
H, W = cam.height, cam.width
r = rtzig.DeviceRenderer(0)
r.set_scene(cam.scene.world)
r.enable_timing(True)


def kernel_ms(row0, step, n_rows):
    out = torch.empty((n_rows, W, 3), dtype=torch.float64, device="cuda:0")
    r.render_rows_async(cam.cam, out.data_ptr(), row0=row0, row_step=step, n_rows=n_rows)  # warm-up
    ks = []
    for _ in range(args.reps):
        r.render_rows_async(cam.cam, out.data_ptr(), row0=row0, row_step=step, n_rows=n_rows)
        ks.append(sum(r.kernel_times()))  # sample kernel + direct mode's reduce pass
    return min(ks)


def pipeline_ms(row0, step, n_rows):
    """bench.py's N > 1 loop without the collective: frame k renders into buffer k % NB on the render
    stream with its output completed on the second stream, where the gather would run (split: the
    reduce pass there; deferred: folded by the next frame's drained waves, the last one flushed);
    wall clock per frame over args.pipe_frames frames."""
    render, coll = torch.cuda.Stream(), torch.cuda.Stream()
    NB = args.row_buffers
    outs = [torch.empty((n_rows, W, 3), dtype=torch.float64, device="cuda:0") for _ in range(NB)]
    freed = [None] * NB
    pend = [False]
    deferred = args.pipe_mode == "deferred"

    def frame(k):
        b, pb = k % NB, (k - 1) % NB
        # the kernel writes its own rows (outs[b]) and, with a pass pending, folds into outs[pb]
        for wb in ((b, pb) if pend[0] else (b,)):
            if freed[wb] is not None:
                render.wait_event(freed[wb])
        if args.pipe_mode == "plain":
            # one per-sample buffer: the reduce pass runs on the render stream after the sample
            # kernel; the collective stream waits for the frame
            r.render_rows_async(cam.cam, outs[b].data_ptr(), row0=row0, row_step=step, n_rows=n_rows,
                                stream_ptr=render.cuda_stream)
            done = torch.cuda.Event()
            done.record(render)
            coll.wait_event(done)
        else:
            r.render_rows_async(cam.cam, outs[b].data_ptr(), row0=row0, row_step=step, n_rows=n_rows,
                                stream_ptr=render.cuda_stream, out_stream_ptr=coll.cuda_stream, deferred=deferred)
        if pend[0]:
            freed[pb] = torch.cuda.Event()
            freed[pb].record(coll)
        pend[0] = deferred and r.fold_pending()
        if not pend[0]:
            freed[b] = torch.cuda.Event()
            freed[b].record(coll)

    def finish():
        if pend[0]:
            r.flush()
            pend[0] = False

    for k in range(2):
        frame(k)
    finish()
    torch.cuda.synchronize()
    best = None
    for _ in range(args.reps):
        freed[:] = [None] * NB
        t0 = time.perf_counter()
        for k in range(args.pipe_frames):
            frame(k)
        finish()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.pipe_frames * 1e3
        best = ms if best is None else min(best, ms)
    ws[0] = max(ws[0], r.workspace_bytes())
    # one more pass with HIP-event timing: the sample kernel (with the fold inside, deferred) and the
    # reduce / follow-up passes per frame, to split the frame into kernel time and what lies between
    r.enable_timing(True)
    freed[:] = [None] * NB
    for k in range(args.pipe_frames):
        frame(k)
    finish()
    torch.cuda.synchronize()
    s_ms, r_ms, _ = r.kernel_times_total()
    split[0] = (s_ms / args.pipe_frames, r_ms / args.pipe_frames)
    return best


ws = [0]  # the largest workspace a rank's pipeline held (rt_context_workspace_bytes)
split = [(0.0, 0.0)]  # the last pipeline's (sample kernel, reduce / follow-up pass) ms per frame
res = {"config": f"{W}x{H} {args.spp}spp", "unit_mode_env": os.environ.get("RTZIG_UNIT_MODE"),
       "pipe_mode": args.pipe_mode if args.pipe_frames else None, "link_GBps_model": LINK_GBPS, "launch_us_model": LAUNCH_US, "ranks": {}}
base = None
pipe_base = None
for n in args.ns:
    R = rdist.rows_per_rank(H, n)
    per_rank, per_rank_pipe, per_rank_split = [], [], []
    ws[0] = 0
    for rank in range(n):
        row0, step, n_rows = rdist.rank_rows(H, rank, n)
        per_rank.append(kernel_ms(row0, step, n_rows))
        if args.pipe_frames:
            per_rank_pipe.append(pipeline_ms(row0, step, n_rows))
            per_rank_split.append(split[0])
        print(f"N={n} rank {rank}: {per_rank[-1]:.3f} ms" +
              (f", pipelined {per_rank_pipe[-1]:.3f} ms per frame" if per_rank_pipe else ""), file=sys.stderr, flush=True)
    k = max(per_rank)
    gather = 0.0
    if n > 1:
        g = torch.randn((n, R, W, 3), dtype=torch.float64, device="cuda:0")
        rdist.assemble(g, H)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            rdist.assemble(g, H)
        torch.cuda.synchronize()
        asm = (time.perf_counter() - t0) * 1e3 / 10
        xfer = R * W * 24 / (LINK_GBPS * 1e9) * 1e3
        gather = asm + xfer + LAUNCH_US / 1e3
    frame = k + gather
    # bench.py overlaps frame k's gather (collective stream) with frame k+1's render (two row
    # buffers): the steady-state frame is then the longer of the two, if the gather's copies find the
    # GPU time they need beside the render (not measurable on one GPU; both figures are reported)
    frame_ovl = max(k, gather)
    base = base or frame
    res["ranks"][n] = {"rows_rank0": len(range(0, H, n)), "kernel_ms_max_over_ranks": round(k, 3),
                       "kernel_ms_min_over_ranks": round(min(per_rank), 3), "gather_ms": round(gather, 3),
                       "frame_ms": round(frame, 3), "predicted_speedup": round(base / frame, 3),
                       "efficiency": round(base / frame / n, 3),
                       "frame_ms_gather_overlapped": round(frame_ovl, 3),
                       "efficiency_gather_overlapped": round(base / frame_ovl / n, 3)}
    if per_rank_pipe:
        # the steady-state frame of the pipeline (gather hidden beside the next render, reduce pass on
        # the second stream), max over ranks, against the 1-rank pipeline's frame
        pf = max(max(per_rank_pipe), gather)
        pipe_base = pipe_base or pf
        res["ranks"][n].update({"pipelined_frame_ms_max_over_ranks": round(max(per_rank_pipe), 3),
                                "pipelined_frame_ms_min_over_ranks": round(min(per_rank_pipe), 3),
                                "efficiency_pipelined": round(pipe_base / pf / n, 3),
                                "workspace_GiB_max_over_ranks": round(ws[0] / 2**30, 3),
                                # the slowest rank's frame split by HIP events (one more timed pass)
                                "pipelined_sample_kernel_ms_slowest_rank": round(per_rank_split[per_rank_pipe.index(max(per_rank_pipe))][0], 3),
                                "pipelined_reduce_ms_slowest_rank": round(per_rank_split[per_rank_pipe.index(max(per_rank_pipe))][1], 3)})
print(json.dumps(res))

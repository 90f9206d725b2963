#!/usr/bin/env python3
"""Benchmark: Msamples/s of the per-pixel x per-sample hot path (Camera.render,
reference src/camera.zig:123-145) on the final random-sphere scene — BASELINE.json config 4:
1200x800, 500 spp, depth 50, 485 spheres (seed 0xdeadbeef), rows interleaved over N GPUs.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Without a launcher (WORLD_SIZE unset), --gpus N > 1 starts the N ranks itself: N fresh worker
processes (torch.multiprocessing spawn, before anything in this process touches the GPU), each
joining the process group on 127.0.0.1.  A rank count the devices cannot serve (nccl: one device
per rank) or a --gpus that disagrees with WORLD_SIZE is an error (non-zero exit), never a silent
1-GPU run.

A step = one full frame: every rank renders its rows (one HIP kernel launch via the C ABI, inputs
resident in HBM) and the rows are gathered to rank 0 over RCCL.  The image is fixed, so N>1 is
strong scaling.  Rank 0 prints ONE JSON line.

`roofline` is the dominant kernel's VALU roofline (bound "valu": no GEMM-shaped work on this path,
DESIGN.md §5): achieved = the FLOPs the sample kernel executes per frame (exact in-kernel counts of
one instrumented frame: 17 f64 FLOPs per ray-sphere candidate test, SURVEY §8(d)'s unit, plus 24 f32
FLOPs per BVH node visit counted at half weight: a packed f32 fma issues in the cycles of one f64 fma)
/ its HIP-event time, against the 78.6 TFLOP/s FP64 vector peak (69.3 measured, profiles/r05_peak/).
`roofline.issue` is the VALU-issue cycle model from the committed PMC summary (event-timed issue costs
per opcode and operand form): the kernel is VALU-issue-bound, so that fraction is the one that binds.
`cpu_baseline` times the oracle's sequential-stream port of the reference (single thread — the
reference's single RNG stream is inherently sequential) on a bounded sample of the same frame.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raytracing-with-zig_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import rtzig  # noqa: E402
from rtzig import dist as rdist  # noqa: E402

METRIC = "Msamples/sec (pixels×spp/s) on final-render scene; achieved HBM GB/s vs peak"
FP64_VALU_PEAK_TFLOPS = 78.6   # MI355X vector FP64 (spec): 16 lanes/clock/SIMD at 2.4 GHz
# the same measured with hipEvents over all CUs (v_fma_f64, 8 waves/SIMD, the chip at 2.20 GHz under
# that load): profiles/r05_peak/ (round 4's 2.12-cycle s_memtime rate was a residency artefact)
FP64_VALU_MEASURED_TFLOPS = 69.3
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (spec), MI355X_MICROARCH.md
SIMDS = 1024                   # 256 CUs x 4 SIMDs
FLOPS_PER_TEST = 17            # oc(3) + h(5) + |oc|^2(5) + -r^2(1) + h^2-a*c(3), SURVEY §8(d)
F32_FLOPS_PER_VISIT = 24       # BVH node visit: 2 child boxes x 3 axes x 2 planes x fma (2 FLOPs), f32


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _oracle():
    """Oracle A's CPU baseline build: SURVEY §8(d)'s flags (-O3 -march=native -ffp-contract=off),
    compiled here for this host's CPU; the portable build if that fails."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle
    d = tempfile.mkdtemp(prefix="rtzig_oracle_")
    try:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native", f"NATIVE_DIR={d}"],
                       check=True, capture_output=True, timeout=120)
        return Oracle(os.path.join(d, "liboracle.so")), "-O3 -march=native -ffp-contract=off (built on this host)"
    except Exception as e:  # noqa: BLE001
        log(f"native oracle build failed ({e}); using the portable build")
        return Oracle(), "-O3 -ffp-contract=off (portable build)"


def cpu_baseline(width, aspect, cpu_spp):
    """Oracle A (reference port, sequential Xoshiro stream, one thread) on a bounded sample:
    the full config-4 frame at `cpu_spp` samples per pixel."""
    from rtzig.abi import D3, RtCameraParams
    o, flags = _oracle()
    spheres, state = o.scene_final(0xDEADBEEF)
    p = RtCameraParams(image_width=width, samples_per_pixel=cpu_spp, bounce_max=50,
                       aspect_ratio=aspect, look_from=D3(13, 2, 3), look_at=D3(0, 0, 0),
                       v_up=D3(0, 1, 0), vfov=20, defocus_angle=0.6, focus_dist=10,
                       t_min=1e-3, t_max=float("inf"), seed=0xDEADBEEF)
    cam = o.camera_build(p)
    t0 = time.perf_counter()
    _, rays = o.render_a(cam, spheres, state)
    dt = time.perf_counter() - t0
    n = cam.image_width * cam.image_height * cpu_spp
    res = {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": 1, "kind": "port",
           "sample": f"oracle A (C restatement of the Zig reference, sequential RNG stream, {flags}) "
                     f"full {cam.image_width}x{cam.image_height} frame at {cpu_spp} spp "
                     f"({n} samples, {rays} rays) in {dt:.2f} s"}
    # context only: oracle B, the same arithmetic with per-(pixel, sample) streams,
    # parallel over rows with OpenMP on this job's share of the host cores (at most 16)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    t0 = time.perf_counter()
    o.render_b(cam, spheres, threads=threads)
    dtb = time.perf_counter() - t0
    res["multicore_context"] = {"value": round(n / dtb / 1e6, 4), "unit": "Msamples/s", "cores": threads,
                                "kind": "port (oracle B, OpenMP over rows)",
                                "sample": f"same frame, {dtb:.2f} s"}
    return res


def pmc_summary(workload):
    """Per-frame PMC figures of the timed sample kernel from the committed rocprofv3 summary
    (profiles/pmc_traffic.json, written by tools/pmc_summary.py from separate --pmc passes), or {}."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    except (OSError, ValueError):
        return {}
    return d if d.get("workload") == workload else {}


def dropin(cam, device):
    """The drop-in path's cost INSIDE this process: rt_render (n_gpus=1) of the same frame into host
    memory, three calls.  The first creates rt_render's cached context (streams, scene + BVH upload,
    workspace) in a process whose HIP runtime torch has already initialised — it is NOT a cold start
    (dropin_one_shot is); the later calls reuse the cached context and scene."""
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        rtzig.render(cam.cam, cam.scene.world, n_gpus=1, device=device)
        times.append((time.perf_counter() - t0) * 1e3)
    return times


def dropin_one_shot(width, spp, aspect, runs=3):
    """The drop-in as the reference runs it — ONE image per process (main.zig:14-36): the C harness
    of the Zig shim (tools/rt_render_c.c: rt_scene_final -> rt_camera_build -> rt_render(n_gpus = 0,
    RGB8) -> rt_ppm_save_p6) started as a fresh child process per run, timed from spawn to the P6 file
    written (tools/dropin_cold.py: the harness's CLOCK_MONOTONIC stamps and the library's phase
    trace).  Everything a fresh process pays is inside: exec, library load, HIP runtime init, context,
    scene + tree, the frame, the copy-out, the write."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import statistics
    import dropin_cold
    args = (str(width), str(spp), "0xdeadbeef", repr(aspect), "final")
    res = {"harness": "tools/rt_render_c (fresh child process per run, n_gpus = 0, RGB8, P6)",
           "args": {"width": width, "spp": spp, "aspect": aspect, "scene": "final"}}
    try:
        with tempfile.TemporaryDirectory() as d:
            rs = [dropin_cold.one_run(args, os.path.join(d, f"{k}.ppm")) for k in range(runs)]
    except (OSError, RuntimeError, subprocess.SubprocessError) as e:
        res["error"] = f"{type(e).__name__}: {str(e)[-300:]}"
        return res
    med = lambda xs: round(statistics.median(xs), 2)  # noqa: E731
    res.update({
        "spawn_to_file_written_ms": [round(r["to_file_written_ms"], 2) for r in rs],
        "median_spawn_to_file_written_ms": med([r["to_file_written_ms"] for r in rs]),
        "median_spawn_to_exit_ms": med([r["total_ms"] for r in rs]),
        "median_hip_runtime_init_ms": med([r["rt_render_phases_ms"].get("hip_init_device_map", 0.0) for r in rs]),
        "median_frame_kernel_ms": med([r["kernel_ms"][0] for r in rs if r["kernel_ms"]]),
    })
    return res


def all_devices_check(ndev, timeout=240):
    """The drop-in over every GPU of the node, as the Zig shim calls it: tools/rt_render_c (a child
    process; rt_scene_final -> rt_camera_build -> rt_render(n_gpus = 0) -> rt_ppm_save_p6) on the
    reference's golden configuration (400x225, 10 spp, seed 0xdeadbeef: main.zig:41-55), once over
    all visible devices and once on device 0 alone (RTZIG_DEVICE_MAP=0).  The RNG is keyed by the
    global pixel, so the two P6 files must be identical (the multi-device branch is
    otherwise rehearsed with logical devices on one GPU).  Runs after the timed region and the
    process group, so a failure is reported here and never touches `value`."""
    exe = os.path.join(ROOT, "raytracing-with-zig_amd", "rt_render_c")
    cfg = ["400", "10", "0xdeadbeef", repr(16 / 9), "final"]
    res = {"devices": ndev, "harness": "tools/rt_render_c (n_gpus = 0, RGB8, P6), golden config 400x225 10 spp"}
    files = []
    try:
        with tempfile.TemporaryDirectory() as d:
            for tag, extra in (("all", None), ("one", "0")):
                path = os.path.join(d, tag + ".ppm")
                env = {k: v for k, v in os.environ.items() if k != "RTZIG_DEVICE_MAP"}
                if extra is not None:
                    env["RTZIG_DEVICE_MAP"] = extra
                t0 = time.perf_counter()
                p = subprocess.run([exe, path] + cfg, env=env, capture_output=True, text=True, timeout=timeout)
                res[tag + "_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
                if p.returncode:
                    res["error"] = f"{tag}: exit {p.returncode}: {p.stderr.strip()[-300:]}"
                    return res
                files.append(open(path, "rb").read())
    except (OSError, subprocess.SubprocessError) as e:
        res["error"] = f"{type(e).__name__}: {e}"
        return res
    res["identical"] = files[0] == files[1]
    return res


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--aspect", type=float, default=1.5)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--output", choices=["linear", "rgb8"], default="linear")
    ap.add_argument("--cpu-spp", type=int, default=4, help="spp of the bounded CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fast", action="store_true", help="skip the f32 fast-mode side measurement")
    ap.add_argument("--no-dropin", action="store_true", help="skip the rt_render drop-in measurement")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL over xGMI, the product) or gloo (rehearsal: several ranks on one GPU)")
    ap.add_argument("--check", action="store_true",
                    help="after the timed region, compare rank 0's last gathered frame bit for bit with "
                         "a whole-image render on its own device (tests: the pipelined gather path)")
    ap.add_argument("--collective", action="store_true",
                    help="at --gpus 1, still join a (1-rank) process group on --dist-backend and run the "
                         "N>1 pipeline: the row buffers, the render stream, and each frame's dist.gather on "
                         "the collective stream (nccl: the RCCL gather on one GPU)")
    ap.add_argument("--pipeline", choices=["plain", "split", "deferred"], default="deferred",
                    help="N > 1 frame loop: 'plain' completes each frame on the render stream (one "
                         "per-sample buffer in direct mode: half the workspace, the reduce pass on the "
                         "critical path); 'split' completes each frame's output on the collective stream "
                         "(rt_render_rows_async_split); 'deferred' also leaves a direct-mode frame's reduce "
                         "pass to the next frame's drained waves (rt_render_rows_async_deferred), gathering "
                         "each frame once the next one is issued")
    ap.add_argument("--row-buffers", type=int, default=3, choices=[2, 3, 4],
                    help="N > 1: row buffers the frame loop rotates through (gather overlap)")
    ap.add_argument("--no-device-check", action="store_true",
                    help="at N > 1, skip rank 0's rt_render(n_gpus = 0) check over every visible GPU")
    ap.add_argument("--launch-check", action="store_true",
                    help="start the ranks and join the process group, print one line, render nothing")
    return ap.parse_args(argv)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _worker(rank, argv, world, port):
    """One rank started by main() (no external launcher): the env a launcher would set, then run()."""
    os.environ.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    run(parse_args(argv))


def main():
    argv = sys.argv[1:]
    args = parse_args(argv)
    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1 (got {args.gpus})")
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
        run(args)
    elif args.gpus == 1:
        run(args)
    else:
        # no launcher: start the ranks here.  spawn = fresh interpreters; this process has not
        # touched the GPU and does not exec anything itself.
        import torch.multiprocessing as mp
        try:
            mp.spawn(_worker, args=(argv, args.gpus, _free_port()), nprocs=args.gpus, join=True)
        except Exception as e:  # a rank failed: its traceback is on stderr
            sys.exit(f"bench.py: a rank failed ({type(e).__name__}: {e})")


def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:
        # rank plumbing only (CPU tests): join a gloo group, agree on the world size, print it
        if world > 1 or args.collective:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            dist.init_process_group("gloo", rank=rank, world_size=world)
            t = torch.tensor([1])
            dist.all_reduce(t)
            n = int(t.item())
            dist.destroy_process_group()
        else:
            n = 1
        if rank == 0:
            print(json.dumps({"launch_check": True, "n_gpus": n, "gpus_arg": args.gpus}), flush=True)
        return
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and ndev < world:
        raise SystemExit(f"bench.py: {world} ranks over nccl need {world} visible GPUs, found {ndev} "
                         "(use --dist-backend gloo to rehearse several ranks on one GPU)")
    # gloo rehearsal: ranks may share a device (local rank modulo the visible device count)
    local_dev = local if args.dist_backend == "nccl" else local % max(1, ndev)
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    # grouped: a process group exists (N > 1, or --collective at N = 1); the pipeline below (render
    # stream + collective stream, --row-buffers row buffers, dist.gather per frame) runs whenever it does
    grouped = world > 1 or args.collective
    if grouped and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
    if grouped:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)

    t_init = time.perf_counter()
    cam = rtzig.final_scene_camera(width=args.width, aspect_ratio=args.aspect, spp=args.spp)
    H, W, spp = cam.height, cam.width, args.spp
    n_spheres = len(cam.scene.world)
    row0, step, n_rows = rdist.rank_rows(H, rank, world)
    R = rdist.rows_per_rank(H, world)
    renderer = rtzig.DeviceRenderer(local_dev)
    renderer.set_scene(cam.scene.world)
    renderer.enable_timing(True)
    # Row buffers (--row-buffers, 3) and a render stream of their own: frame k renders into
    # outs[k % NB] on `stream` while the collective stream (the current one, which RCCL's gather
    # joins) still gathers earlier frames from the others — the gather overlaps the next frame's
    # render instead of adding to it.  A buffer is rendered into again only after its previous gather
    # has finished (`freed`); with three, that gather is two frames old, so a deferred frame's kernel
    # does not wait for the previous kernel's completion to travel through the collective stream.
    dt = torch.float64 if args.output == "linear" else torch.uint8
    NB = args.row_buffers
    outs = [torch.zeros((R, W, 3), dtype=dt, device=dev) for _ in range(NB)]
    out = outs[0]
    stats = torch.zeros(2, dtype=torch.int64, device=dev)
    coll = torch.cuda.current_stream()
    stream = torch.cuda.Stream(device=dev) if grouped else coll
    rendered = [torch.cuda.Event() for _ in range(NB)]
    freed = [None] * NB
    nframe = [0]
    torch.cuda.synchronize()
    init_ms = (time.perf_counter() - t_init) * 1e3

    def gather(buf=None):
        buf = out if buf is None else buf
        if args.dist_backend == "gloo" and grouped:
            return rdist.gather_image(buf.cpu(), H, rank, world, collective=grouped)  # gloo: host tensors
        return rdist.gather_image(buf, H, rank, world, collective=grouped)

    pend = [False]  # the last deferred frame's output is still pending (its reduce pass not yet run)

    def frame_deferred(stats_ptr=None):
        # rt_render_rows_async_deferred: frame j's kernel folds frame j-1's reduce pass into its row
        # buffer in the launch's tail, so frame j-1 is gathered after frame j is issued; a ring-mode
        # frame (nothing pending) is gathered at once, as with the split call
        j = nframe[0]
        nframe[0] += 1
        b, pb = j % NB, (j - 1) % NB
        # the kernel writes its own rows into outs[b] (a call that cannot fold the pending pass runs it
        # first and writes outs[b] directly), and with a pass pending it also folds into outs[pb]: both
        # buffers' last gathers must have finished (in steady state both events have long completed)
        for wb in ((b, pb) if pend[0] else (b,)):
            if freed[wb] is not None:
                stream.wait_event(freed[wb])
        img = None
        if n_rows:
            renderer.render_rows_async(cam.cam, outs[b].data_ptr(), row0=row0, row_step=step,
                                       n_rows=n_rows, output=args.output, d_stats_ptr=stats_ptr,
                                       stream_ptr=stream.cuda_stream, out_stream_ptr=coll.cuda_stream,
                                       deferred=True)
        else:
            rendered[b].record(stream)
            coll.wait_event(rendered[b])
        if pend[0]:
            img = gather(outs[pb])
            freed[pb] = torch.cuda.Event()
            freed[pb].record(coll)
        pend[0] = bool(n_rows) and renderer.fold_pending()
        if not pend[0]:
            img = gather(outs[b])
            freed[b] = torch.cuda.Event()
            freed[b].record(coll)
        return img

    def finish():
        """The deferred loop's last frame: run its pending pass and gather it."""
        if not pend[0]:
            return None
        renderer.flush()
        pend[0] = False
        b = (nframe[0] - 1) % NB
        img = gather(outs[b])
        freed[b] = torch.cuda.Event()
        freed[b].record(coll)
        return img

    def frame(stats_ptr=None):
        if stream is not coll and args.pipeline == "deferred":
            return frame_deferred(stats_ptr)
        b = nframe[0] % NB
        nframe[0] += 1
        buf = outs[b]
        if freed[b] is not None:
            stream.wait_event(freed[b])  # the gather that last read this buffer has finished
        if stream is coll:
            if n_rows:
                renderer.render_rows_async(cam.cam, buf.data_ptr(), row0=row0, row_step=step,
                                           n_rows=n_rows, output=args.output, d_stats_ptr=stats_ptr,
                                           stream_ptr=stream.cuda_stream)
            return gather(buf)
        if n_rows and args.pipeline == "plain":
            # one per-sample buffer: sample kernel and reduce pass both on the render stream
            renderer.render_rows_async(cam.cam, buf.data_ptr(), row0=row0, row_step=step,
                                       n_rows=n_rows, output=args.output, d_stats_ptr=stats_ptr,
                                       stream_ptr=stream.cuda_stream)
            rendered[b].record(stream)
            coll.wait_event(rendered[b])
        elif n_rows:
            # the output is completed on the collective stream (rt_render_rows_async_split): the
            # sample kernel runs on the render stream and a direct-mode launch's reduce pass on the
            # collective stream, ahead of this frame's gather, so it overlaps the next frame's
            # sample kernel (rank 0 of 8 on config 4: -1.5%, profiles/r04_split_ab/)
            renderer.render_rows_async(cam.cam, buf.data_ptr(), row0=row0, row_step=step,
                                       n_rows=n_rows, output=args.output, d_stats_ptr=stats_ptr,
                                       stream_ptr=stream.cuda_stream, out_stream_ptr=coll.cuda_stream)
        else:
            rendered[b].record(stream)
            coll.wait_event(rendered[b])
        img = gather(buf)
        freed[b] = torch.cuda.Event()
        freed[b].record(coll)
        return img

    # the first frame also pays the one-time BVH rebuild from sample rays of this camera (DESIGN.md
    # §5 "Ray-driven tree"): its wall time is reported as a fixed cost
    first_ms = None
    for w in range(args.warmup):
        t_w = time.perf_counter()
        frame()
        finish()
        torch.cuda.synchronize()
        if w == 0:
            first_ms = (time.perf_counter() - t_w) * 1e3
    # one untimed instrumented frame: exact executed-work counts (sphere tests, BVH node visits)
    pstats = torch.zeros(rtzig.abi.RT_PROFILE_STATS_WORDS, dtype=torch.int64, device=dev)
    if n_rows:
        renderer.enable_profile(True)
        renderer.render_rows_async(cam.cam, out.data_ptr(), row0=row0, row_step=step, n_rows=n_rows,
                                   output=args.output, d_stats_ptr=pstats.data_ptr(),
                                   stream_ptr=coll.cuda_stream)
        torch.cuda.synchronize()
        renderer.enable_profile(False)
    prof = [int(x) for x in pstats.cpu().tolist()]
    stats.zero_()
    # HIP events around every sample / reduce launch of the timed frames, on the launch streams; read
    # back once after the timed region, so no frame waits on the host
    renderer.enable_timing(True)

    if grouped:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    img = None
    for k in range(args.steps):
        got = frame(stats.data_ptr())
        img = got if got is not None else img
    last = finish()  # the deferred loop's last frame (inside the timed region)
    img = last if last is not None else img
    torch.cuda.synchronize()
    if grouped:
        dist.barrier()
    elapsed = time.perf_counter() - t0

    t = torch.tensor([elapsed], dtype=torch.float64,
                     device=dev if args.dist_backend == "nccl" else "cpu")
    if grouped:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max = float(t.item())
    kname = renderer.kernel_name()  # the timed (parity) kernel, before the fast-mode frames
    k_sum, r_sum, n_launch = renderer.kernel_times_total() if n_rows else (0.0, 0.0, 0)
    renderer.sync()  # raises if a wave of any timed frame gave up on a hand-off (sticky error word)
    check = None
    if args.check and rank == 0 and n_rows:
        # the last timed frame as gathered (row buffers in rotation, gather overlapped with the next render)
        # against one whole-image render on this device: the RNG is keyed by the global pixel, so
        # they must agree bit for bit
        whole = torch.empty((H, W, 3), dtype=dt, device=dev)
        renderer.render_rows_async(cam.cam, whole.data_ptr(), row0=0, row_step=1, n_rows=H, output=args.output,
                                   stream_ptr=coll.cuda_stream)
        torch.cuda.synchronize()
        got = img.cpu() if img is not None else None
        check = bool(got is not None and torch.equal(got, whole.cpu()))
        if not check:
            raise SystemExit("bench.py --check: the gathered frame differs from the whole-image render")
    # N > 1: the gather alone, K times, bracketed like the timed region (the frame's other part)
    coll_dev = dev if args.dist_backend == "nccl" else "cpu"
    gather_ms = 0.0
    if grouped:
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        for _ in range(args.steps):
            gather()
        torch.cuda.synchronize()
        dist.barrier()
        gather_ms = (time.perf_counter() - tg) / args.steps * 1e3
    mine = torch.tensor([float(rank), float(n_rows), k_sum / args.steps, r_sum / args.steps, gather_ms,
                         elapsed / args.steps * 1e3, float(renderer.workspace_bytes())],
                        dtype=torch.float64, device=coll_dev)
    if grouped:
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
    else:
        every = [mine]
    per_rank = [{"rank": int(v[0]), "rows": int(v[1]), "kernel_ms_per_frame": round(float(v[2]), 3),
                 "reduce_ms_per_frame": round(float(v[3]), 3), "gather_ms": round(float(v[4]), 3),
                 "ms_per_step": round(float(v[5]), 3),
                 "workspace_GiB": round(float(v[6]) / 2**30, 3)} for v in (x.cpu() for x in every)]
    st = stats.cpu().tolist()
    rays_per_frame = st[0] / max(1, args.steps)
    samples_per_frame = st[1] / max(1, args.steps)
    # side measurement (1 GPU only): RT_PRECISION_F32 fast mode on the same frame.  Statistical
    # parity only (tests/test_fast_mode.py), so it is reported beside `value`, never as it.
    fast = None
    if world == 1 and not args.no_fast and n_rows:
        renderer.set_precision("f32")
        frame()
        finish()
        torch.cuda.synchronize()
        renderer.enable_timing(True)
        tf0 = time.perf_counter()
        for _ in range(2):
            frame()
        finish()
        torch.cuda.synchronize()
        tf = (time.perf_counter() - tf0) / 2
        fast = {"value": round(W * H * spp / tf / 1e6, 3), "unit": "Msamples/s", "dtype": "f32",
                "kernel": renderer.kernel_name(), "kernel_ms_per_frame": round(renderer.kernel_times_total()[0] / 2, 3),
                "note": "RT_PRECISION_F32 fast mode (huge spheres in f64), statistical parity only; "
                        "not the headline value"}
        renderer.set_precision("f64")
    renderer.sync()
    renderer.close()

    group_size = dist.get_world_size() if grouped else 1
    if grouped:
        dist.destroy_process_group()
    # N > 1 on a multi-GPU node: the drop-in's own multi-device branch over every visible GPU
    # (rank 0 only, after the other ranks are done with their devices' work)
    device_check = None
    if rank == 0 and world > 1 and not args.no_device_check:
        device_check = all_devices_check(ndev) if ndev > 1 else {"devices": ndev, "skipped": "one visible device"}
    if rank == 0:
        total_samples = W * H * spp * args.steps
        value = total_samples / elapsed_max / 1e6
        launches_per_frame = n_launch / max(1, args.steps)
        k_frame_s = k_sum / args.steps / 1e3   # sample kernel time per frame (sum of its launches)
        workload = f"final-render {W}x{H} {spp}spp depth50 ({n_spheres} spheres)"
        pmc = pmc_summary(workload)
        tests, visits = prof[2], prof[3]
        exec_flops = FLOPS_PER_TEST * tests + F32_FLOPS_PER_VISIT * visits / 2   # f64-equivalent, per frame
        exec_tf = exec_flops / k_frame_s / 1e12
        alg_eq_tf = FLOPS_PER_TEST * n_spheres * rays_per_frame / k_frame_s / 1e12
        issue = None
        # the PMC passes profile the whole 1-GPU frame: at N > 1 a rank renders 1/N of it, so the
        # issue fraction is only reported for the 1-GPU line
        if world == 1 and pmc.get("valu_issue_cycles_per_frame") and pmc.get("clock_GHz"):
            cyc = pmc["valu_issue_cycles_per_frame"]
            issue = {"frac": round(cyc / (SIMDS * pmc["clock_GHz"] * 1e9 * k_frame_s), 4),
                     "valu_issue_cycles_per_frame": cyc, "clock_GHz": pmc["clock_GHz"],
                     "model": "PMC VALU counts x issue cycles per wave64 instruction MEASURED on the MI355X with "
                              "hipEvent timing (f64 add/mul/fma 4.17, rsq/rcp_f64 16.1, f32 transcendentals 8.1, "
                              "the other ops at the kernel's own operand-aware mix of 4.15-cycle and 2.2-cycle "
                              "forms), / (1024 SIMDs x clock x kernel time): the bound that binds",
                     "rates": pmc.get("valu_issue_model"),
                     "source": pmc.get("source")}
        # HBM: the algorithmic traffic of a frame is the f64 linear framebuffer W*H*24 (or W*H*3
        # bytes of RGB8) written once; the rest is the design's own: each sample's
        # 24-B color through the wave's ring (L2 / MALL when it stays there), the running sums'
        # write-through hand-off between sample chunks (24 B per pixel per chunk, both ways)
        alg_bytes = n_rows * W * (24 if args.output == "linear" else 3)
        frame_ms = elapsed_max / args.steps * 1e3
        # the committed PMC passes profile the 1-GPU frame (ring mode); a rank's smaller row set runs
        # in direct mode with different traffic, so N > 1 lines carry no PMC figure
        traffic = pmc.get("hbm_bytes_per_frame") if world == 1 else None
        assert img is not None and img.shape[0] == H
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": group_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(frame_ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic: final random-sphere scene generated in-process (Scene.generateWorld, "
                    "seed 0xdeadbeef), main.zig camera preset",
            "config": {"workload": workload, "width": W, "height": H, "spp": spp, "depth": 50,
                       "spheres": n_spheres, "output": args.output,
                       "parallelism": f"rows interleaved over {world} GPU(s)"
                           + ((", RCCL gather to rank 0" if args.dist_backend == "nccl" else
                               ", gloo gather to rank 0 (rehearsal: ranks share devices)")
                              + (" (1-rank group, --collective)" if world == 1 else "")
                              + (f", each frame's gather overlapped with the next frame's render ({NB} row buffers); "
                                 "a direct-mode frame's reduce pass folded inside the next frame's sample kernel "
                                 "(rt_render_rows_async_deferred)" if args.pipeline == "deferred" else
                                 f", each frame's gather overlapped with the next frame's render ({NB} row buffers); "
                                 "a direct-mode reduce pass on the render stream (one per-sample buffer)"
                                 if args.pipeline == "plain" else
                                 ", each frame's gather and a direct-mode reduce pass on the collective stream, "
                                 f"overlapped with the next frame's render ({NB} row buffers; "
                                 "rt_render_rows_async_split)")
                              if grouped else "")},
            "roofline": {
                "bound": "valu",
                "kernel": kname,
                "achieved": round(exec_tf, 3),
                "peak": FP64_VALU_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(exec_tf / FP64_VALU_PEAK_TFLOPS, 4),
                "peak_measured": {"TFLOP/s": FP64_VALU_MEASURED_TFLOPS,
                                  "frac": round(exec_tf / FP64_VALU_MEASURED_TFLOPS, 4),
                                  "source": "profiles/r05_peak/ (tools/peak_rates.hip: event-timed v_fma_f64 over "
                                            "all CUs; 4.16 SIMD cycles per wave64 instruction = the spec's "
                                            "16 lanes/clock at the 2.2 GHz the chip holds under that load)"},
                "traffic": traffic,
                "work": f"executed per frame (rank 0, {n_rows} rows; exact counts of one instrumented frame): "
                        f"{tests} f64 ray-sphere tests x {FLOPS_PER_TEST} FLOP (SURVEY §8(d) unit) + "
                        f"{visits} BVH node visits x {F32_FLOPS_PER_VISIT} f32 FLOP at 1/2 weight = "
                        f"{exec_flops:.4g} FLOP / {k_frame_s * 1e3:.3f} ms of sample kernel",
                "sphere_tests_per_ray": round(tests / max(1, prof[0]), 3),
                "node_visits_per_ray": round(visits / max(1, prof[0]), 3),
                "issue": issue,
                "algorithmic_equivalent": {
                    "TFLOP/s": round(alg_eq_tf, 3),
                    "note": f"SURVEY §8(d)'s list-walk work {FLOPS_PER_TEST} x {n_spheres} spheres x "
                            f"{rays_per_frame:.0f} rays per frame: the BVH returns the same bits while "
                            "executing ~1% of those tests, so this is not a roofline fraction"},
                "kernel_ms_per_frame": round(k_frame_s * 1e3, 3),
                "launches_per_frame": round(launches_per_frame, 3),
                "kernel_ms_avg": round(k_frame_s * 1e3 / max(1.0, launches_per_frame), 3),
                "unit_mode": "direct" if "direct" in kname else "ring",
                "reduce_ms_per_frame": round(r_sum / args.steps, 3),
                "reduce_ms_meaning": ("the follow-up fold pass only (--pipeline deferred: the part folded inside "
                                      "the next frame's sample kernel is in kernel_ms, the last frame's flush is "
                                      "not timed)")
                if (grouped and args.pipeline == "deferred" and "direct" in kname) else
                ("direct mode's reduce pass" if "direct" in kname else "none (ring mode accumulates in the kernel)"),
            },
            "hbm": {
                "algorithmic_bytes_per_frame": alg_bytes,
                "achieved_GBps": round(alg_bytes / (frame_ms / 1e3) / 1e9, 3),
                "peak_GBps": HBM_PEAK_GBS,
                "frac": round(alg_bytes / (frame_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 7),
                "pmc_bytes_per_frame": traffic,
                "traffic_over_algorithmic": round(traffic / alg_bytes, 1) if traffic else None,
                "overhead": ("the in-kernel ordered accumulation: each sample's 24-B color written to and read "
                             "back from its wave's ring (an upper bound of "
                             f"{n_rows * W * spp * 48 / 1e9:.2f} GB per frame if none of it stays in L2 / MALL), "
                             "and the running sums' write-through hand-off, 48 B per pixel per sample chunk")
                            if "direct" not in kname else
                            ("direct mode (small launch): every sample's 24-B color stored and read back once by "
                             f"the reduce pass, {n_rows * W * spp * 48 / 1e9:.2f} GB per frame"),
            },
            "ranks": per_rank,
            "rays_per_sample": round(rays_per_frame / max(1, samples_per_frame), 4),
            "fixed_costs_ms": {"context_and_scene_upload": round(init_ms, 2),
                               "first_frame_incl_bvh_training": round(first_ms, 2) if first_ms else None},
            "cpu_baseline": None,
            "fast_f32": fast,
            **({"check": "gathered frame == whole-image render, bit for bit"} if check else {}),
            **({"rt_render_all_devices": device_check} if device_check is not None else {}),
        }
        if world == 1 and not args.no_dropin and n_rows:
            times = dropin(cam, local_dev)
            one = dropin_one_shot(W, spp, args.aspect)
            res["dropin_ms"] = {
                "one_shot_process": one,
                "one_shot_over_frame": (round(one["median_spawn_to_file_written_ms"] / frame_ms, 2)
                                        if "median_spawn_to_file_written_ms" in one else None),
                "first_call_hip_initialised": round(times[0], 2),
                "warm": round(min(times[1:]), 2),
                "warm_over_frame": round(min(times[1:]) / frame_ms, 4),
                "note": "one_shot_process = a fresh process per image, spawn to the P6 file written (the "
                        "reference's own use, main.zig:14-36); first_call_hip_initialised = the first "
                        "rt_render(n_gpus=1) call inside this bench process, whose HIP runtime is already "
                        "up (context, scene + BVH upload, workspace, render, D2H of f64 linear); warm = "
                        "later calls on the cached context and scene"}
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(W, args.aspect, args.cpu_spp)
            res["speedup_vs_cpu_baseline"] = round(value / res["cpu_baseline"]["value"], 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

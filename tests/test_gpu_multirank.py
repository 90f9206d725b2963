"""The multi-rank path through the HIP kernel: 2 and 3 ranks in separate
processes share GPU 0, each renders its interleaved rows (rows j = rank + k*world) with the
DeviceRenderer (C ABI -> HIP kernel), and rtzig.dist gathers them to rank 0 over gloo.  The gathered
image must equal the 1-rank GPU image and oracle B bit for bit: the RNG is keyed by the global pixel,
so the partition cannot change a bit.  (bench.py runs the same partition over RCCL, one GPU per
rank.)"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WIDTH, SPP = 160, 6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q, mode):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RTZIG_UNIT_MODE"] = mode
    import torch
    import torch.distributed as dist

    import rtzig
    from rtzig import dist as rdist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        cam = rtzig.final_scene_camera(width=WIDTH, aspect_ratio=16 / 9, spp=SPP)
        H, W = cam.height, cam.width
        row0, step, n = rdist.rank_rows(H, rank, world)
        R = rdist.rows_per_rank(H, world)
        r = rtzig.DeviceRenderer(0)
        r.set_scene(cam.scene.world)
        local = torch.zeros((R, W, 3), dtype=torch.float64, device="cuda:0")
        if n:
            r.render_rows_async(cam.cam, local.data_ptr(), row0=row0, row_step=step, n_rows=n,
                                stream_ptr=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        img = rdist.gather_image(local.cpu(), H, rank, world)  # gloo gathers host tensors
        r.close()
        if rank == 0:
            q.put(img.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["ring", "direct"])
@pytest.mark.parametrize("world", [2, 3])
def test_hip_ranks_gather_equals_single_rank(oracle, world, mode):
    """Both unit modes on every rank (ring: in-kernel ordered accumulation; direct: stored samples
    + reduce pass, the mode a rank's rows of an 8-GPU job use)."""
    import rtzig
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        img = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    cam = rtzig.final_scene_camera(width=WIDTH, aspect_ratio=16 / 9, spp=SPP)
    single = rtzig.render(cam.cam, cam.scene.world, n_gpus=1)
    ref, _ = oracle.render_b(cam.cam, cam.scene.world, threads=16)
    assert img.shape == single.shape
    assert np.array_equal(img, single)
    assert np.array_equal(img, ref)


@pytest.mark.parametrize("pipeline", ["deferred", "split", "plain"])
def test_bench_pipelined_gather_bit_exact(pipeline):
    """bench.py's own timed loop over 2 ranks it starts itself (gloo rehearsal, both on GPU 0): two
    row buffers, a render stream and the collective stream, each frame's gather overlapped with the
    next frame's render, in each --pipeline (deferred: the default; split; plain: one per-sample
    buffer).  `--check` compares rank 0's last gathered frame with a whole-image render bit for bit
    (the pipelining must not let a render overwrite rows still being gathered)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = ["--gpus", "2", "--dist-backend", "gloo", "--check", "--steps", "4", "--warmup", "1", "--spp", "8",
            "--width", "240", "--no-cpu-baseline", "--no-fast", "--no-dropin", "--pipeline", pipeline]
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, capture_output=True, text=True,
                       timeout=110, cwd=root)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2
    assert line["check"].startswith("gathered frame == whole-image render")


def test_bench_rccl_gather_world1_bit_exact():
    """The RCCL collective path on one MI355X: bench.py --collective joins a 1-rank nccl group and
    runs the N>1 pipeline unchanged (two row buffers, render stream, dist.gather through
    ProcessGroupNCCL on the collective stream each frame).  `--check`: rank 0's last gathered frame
    equals a whole-image render bit for bit (reference: the row loop of camera.zig:128-140)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = ["--gpus", "1", "--collective", "--dist-backend", "nccl", "--check", "--steps", "4", "--warmup", "1",
            "--spp", "8", "--width", "240", "--no-cpu-baseline", "--no-fast", "--no-dropin"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, capture_output=True, text=True,
                       timeout=110, cwd=root, env=env)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 1
    assert "RCCL gather to rank 0 (1-rank group" in line["config"]["parallelism"]
    assert line["check"].startswith("gathered frame == whole-image render")


def test_bench_all_devices_check():
    """bench.py's post-run drop-in check (rank 0 at N > 1): tools/rt_render_c with rt_render(n_gpus
    = 0) over every visible GPU against the same call on device 0 alone — identical P6 files
    (camera.zig:123-145 through the C ABI).  Needs two physical GPUs: on one, both calls would use
    the same device and the check would compare a render with itself (the logical-device form of
    the multi-device branch is test_c_harness_end_to_end with RTZIG_DEVICE_MAP)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs >= 2 physical GPUs (one device would be compared with itself)")
    res = bench.all_devices_check(torch.cuda.device_count())
    assert res.get("identical") is True, res

"""N>1 path on CPU: world_size-2 (and 3) gloo process groups run the row-interleaved partition and
the final gather to rank 0.  Each rank renders its rows with a CPU stand-in (oracle B — tests only,
the product renders on the GPU); the gathered image must equal the single-rank image bit-for-bit."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rtzig import dist as rdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_lib
        import rtzig
        o = oracle_lib.Oracle()
        cam = rtzig.final_scene_camera(width=48, aspect_ratio=16 / 9, spp=2)
        H, W = cam.height, cam.width
        row0, step, n = rdist.rank_rows(H, rank, world)
        R = rdist.rows_per_rank(H, world)
        local = torch.zeros((R, W, 3), dtype=torch.float64)
        if n:
            rows, _ = o.render_b(cam.cam, cam.scene.world, row0=row0, row_step=step, n_rows=n)
            local[:n] = torch.from_numpy(rows)
        img = rdist.gather_image(local, H, rank, world)
        if rank == 0:
            q.put(img.numpy().copy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_row_interleave_gather(oracle, world):
    import rtzig
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    img = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    cam = rtzig.final_scene_camera(width=48, aspect_ratio=16 / 9, spp=2)
    ref, _ = oracle.render_b(cam.cam, cam.scene.world)
    assert img.shape == ref.shape
    assert np.array_equal(img, ref)


def test_partition_covers_every_row_once():
    for H in (1, 2, 7, 225, 800):
        for world in (1, 2, 3, 4, 8):
            seen = []
            for r in range(world):
                row0, step, n = rdist.rank_rows(H, r, world)
                seen += [row0 + k * step for k in range(n)]
                assert n <= rdist.rows_per_rank(H, world)
            assert sorted(seen) == list(range(H))


def test_assemble_order():
    H, world = 7, 3
    R = rdist.rows_per_rank(H, world)
    g = torch.full((world, R, 1, 1), -1.0)
    for r in range(world):
        for k in range(R):
            if r + k * world < H:
                g[r, k] = r + k * world
    assert rdist.assemble(g, H).flatten().tolist() == list(range(H))


def _bench(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, capture_output=True, text=True,
                       timeout=240, env=env, cwd=root)
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return p.returncode, lines, p.stderr


def test_bench_spawns_ranks_without_launcher():
    """`bench.py --gpus 2` with no launcher (no WORLD_SIZE) starts the 2 ranks itself and they form
    one process group (--launch-check: gloo, no rendering), instead of silently running 1 GPU."""
    rc, lines, err = _bench(["--gpus", "2", "--launch-check"])
    assert rc == 0, err[-2000:]
    assert lines == [{"launch_check": True, "n_gpus": 2, "gpus_arg": 2}]


def test_bench_refuses_what_it_cannot_run():
    """Mismatched --gpus vs a launcher's WORLD_SIZE, and nccl ranks without one device each (this
    container has none), exit non-zero instead of reporting a 1-GPU number."""
    rc, lines, _ = _bench(["--gpus", "2", "--launch-check"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"},
                          drop=())
    assert rc != 0 and lines == []
    if torch.cuda.device_count() < 2:
        rc, lines, err = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
        assert rc != 0 and lines == [] and "need 2 visible GPUs" in err


def _one_rank_collective(port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        H = 5
        local = torch.arange(H * 4 * 3, dtype=torch.float64).reshape(H, 4, 3)
        img = rdist.gather_image(local, H, 0, 1, collective=True)
        q.put((img.data_ptr() != local.data_ptr(), torch.equal(img, local)))
    finally:
        dist.destroy_process_group()


def test_world1_collective_gather_goes_through_the_group():
    """collective=True at world 1 (bench.py --collective): the rows travel through dist.gather on a
    1-rank group (a new buffer), not the world-1 shortcut that returns the local rows."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_one_rank_collective, args=(_free_port(), q))
    p.start()
    copied, equal = q.get(timeout=120)
    p.join(timeout=60)
    assert p.exitcode == 0 and copied and equal


def test_bench_collective_flag_forms_one_rank_group():
    rc, lines, err = _bench(["--gpus", "1", "--collective", "--launch-check"])
    assert rc == 0, err[-2000:]
    assert lines == [{"launch_check": True, "n_gpus": 1, "gpus_arg": 1}]


def test_bench_pipeline_options_parse():
    """bench.py's N > 1 loop options: the deferred pipeline over three row buffers by default;
    plain / split and 2-4 row buffers selectable; anything else refused."""
    import importlib
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    bench = importlib.import_module("bench")
    a = bench.parse_args([])
    assert a.pipeline == "deferred" and a.row_buffers == 3 and not a.no_device_check
    a = bench.parse_args(["--pipeline", "plain", "--row-buffers", "2", "--no-device-check"])
    assert a.pipeline == "plain" and a.row_buffers == 2 and a.no_device_check
    for bad in (["--row-buffers", "1"], ["--pipeline", "fused"]):
        with pytest.raises(SystemExit):
            bench.parse_args(bad)


def test_bench_device_check_reports_instead_of_raising(tmp_path, monkeypatch):
    """The post-run all-devices check (rank 0 at N > 1) turns any harness failure into an `error`
    field of the JSON line — it never raises, so the bench line is printed whatever happens
    (here: a harness that does not exist)."""
    import importlib
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    bench = importlib.import_module("bench")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    res = bench.all_devices_check(8, timeout=30)
    assert res["devices"] == 8 and "error" in res and "identical" not in res

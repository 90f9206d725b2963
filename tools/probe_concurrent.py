"""Probe: G contexts on GPU 0 rendering interleaved row sets concurrently (one stream each, as
rt_render's multi-device branch does); per-context stats vs oracle B, repeated."""
import os, sys
sys.path.insert(0, "raytracing-with-zig_amd"); sys.path.insert(0, "tests")
import numpy as np, torch
import rtzig
from oracle_lib import Oracle
o = Oracle()
cam = rtzig.final_scene_camera(width=200, aspect_ratio=16 / 9, spp=4)
H, W = cam.height, cam.width
mode = sys.argv[1] if len(sys.argv) > 1 else "concurrent"
for G in (2, 3, 8):
    exp = []
    for g in range(G):
        n = (H - g + G - 1) // G
        _, rg = o.render_b(cam.cam, cam.scene.world, row0=g, row_step=G, n_rows=n, threads=16)
        exp.append((rg, n * W * 4))
    rs = [rtzig.DeviceRenderer(0) for _ in range(G)]
    for r in rs:
        r.set_scene(cam.scene.world)
    ss = [torch.cuda.Stream() for _ in range(G)]
    bad = 0
    for it in range(12):
        outs, sts = [], []
        for g in range(G):
            n = (H - g + G - 1) // G
            buf = torch.empty((n, W, 3), dtype=torch.float64, device="cuda:0")
            st = torch.zeros(2, dtype=torch.int64, device="cuda:0")
            torch.cuda.synchronize()
            rs[g].render_rows_async(cam.cam, buf.data_ptr(), row0=g, row_step=G, n_rows=n, d_stats_ptr=st.data_ptr(),
                                    stream_ptr=ss[g].cuda_stream)
            if mode == "serial":
                torch.cuda.synchronize()
            outs.append(buf); sts.append(st)
        torch.cuda.synchronize()
        got = [tuple(int(x) for x in st.tolist()) for st in sts]
        if got != exp:
            bad += 1
            print(f"G={G} it={it} MISMATCH", [(g, got[g], exp[g]) for g in range(G) if got[g] != exp[g]], flush=True)
    print(f"G={G} mode={mode}: {bad}/12 iterations with wrong stats", flush=True)
    for r in rs:
        r.close()

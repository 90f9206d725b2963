import os, sys, ctypes as C
sys.path.insert(0, "raytracing-with-zig_amd"); sys.path.insert(0, "tests")
import numpy as np, torch
import rtzig
from oracle_lib import Oracle
o = Oracle()
cam = rtzig.final_scene_camera(width=200, aspect_ratio=16 / 9, spp=4)
ref, rays = o.render_b(cam.cam, cam.scene.world, threads=16)
print("oracle rays", rays, flush=True)
H, W = cam.height, cam.width
for G in (1, 2, 3):
    tot = 0
    for g in range(G):
        _, rg = o.render_b(cam.cam, cam.scene.world, row0=g, row_step=G, n_rows=(H - g + G - 1) // G, threads=16)
        tot += rg
    print("oracle partition G", G, "sum", tot, flush=True)
    r = rtzig.DeviceRenderer(0); r.set_scene(cam.scene.world)
    s = 0
    for g in range(G):
        n = (H - g + G - 1) // G
        buf = torch.empty((n, W, 3), dtype=torch.float64, device="cuda:0")
        st = torch.zeros(2, dtype=torch.int64, device="cuda:0")
        r.render_rows_async(cam.cam, buf.data_ptr(), row0=g, row_step=G, n_rows=n, d_stats_ptr=st.data_ptr())
        torch.cuda.synchronize()
        print("  gpu rows g", g, "stats", st.tolist(), flush=True)
        s += int(st[0])
    print("gpu partition G", G, "sum", s, flush=True)
    r.close()
for m in (None, "0", "0,0", "0,0,0"):
    if m is None: os.environ.pop("RTZIG_DEVICE_MAP", None)
    else: os.environ["RTZIG_DEVICE_MAP"] = m
    st = {}
    out = rtzig.render(cam.cam, cam.scene.world, n_gpus=0, stats=st)
    print("map", m, st, np.array_equal(out, ref), flush=True)

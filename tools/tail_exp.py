import sys, os, json
sys.path.insert(0, "raytracing-with-zig_amd")
import torch, rtzig
res = {}
for bm in (50, 8, 2):
    for spp in (500, 250):
        cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=spp, bounce_max=bm)
        H, W = cam.height, cam.width
        r = rtzig.DeviceRenderer(0); r.set_scene(cam.scene.world); r.enable_timing(True)
        out = torch.empty((100, W, 3), dtype=torch.float64, device="cuda:0")
        st = torch.zeros(24, dtype=torch.int64, device="cuda:0")
        ks = []
        for _ in range(4):
            r.render_rows_async(cam.cam, out.data_ptr(), row0=0, row_step=8, n_rows=100)
            ks.append(sum(r.kernel_times()))
        r.enable_profile(True)
        r.render_rows_async(cam.cam, out.data_ptr(), row0=0, row_step=8, n_rows=100, d_stats_ptr=st.data_ptr())
        torch.cuda.synchronize()
        s = [int(x) for x in st.cpu().tolist()]
        m = 2**64 - 1
        first_start, first_drain, last_end = (~s[13]) & m, (~s[14]) & m, s[15]
        res[f"bm{bm}_spp{spp}"] = {"ms": round(min(ks[1:]), 3), "rays": s[0],
                                   "drain_us": round((first_drain - first_start) / 100, 1),
                                   "tail_us": round((last_end - first_drain) / 100, 1)}
        r.close()
print(json.dumps(res))

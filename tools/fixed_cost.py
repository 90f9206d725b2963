"""Per-launch fixed cost of the sample kernel at the N = 8 row set (rank 0's 100 rows of config 4):
HIP-event kernel time and the instrumented timeline (first wave start -> first queue drain -> last
wave end, on the 100 MHz s_memrealtime clock) for small and large launches, full and capped depth.
    python tools/fixed_cost.py > gpurun_out/fixed_cost.json"""
import json
import sys

sys.path.insert(0, "raytracing-with-zig_amd")
import torch  # noqa: E402

import rtzig  # noqa: E402

res = {}
for bm in (50, 2):
    for spp in (1, 4, 32, 500):
        cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=spp, bounce_max=bm)
        W = cam.width
        r = rtzig.DeviceRenderer(0)
        r.set_scene(cam.scene.world)
        r.enable_timing(True)
        out = torch.empty((100, W, 3), dtype=torch.float64, device="cuda:0")
        st = torch.zeros(rtzig.abi.RT_PROFILE_STATS_WORDS, dtype=torch.int64, device="cuda:0")
        ks, rs = [], []
        for _ in range(5):
            r.render_rows_async(cam.cam, out.data_ptr(), row0=0, row_step=8, n_rows=100)
            t = r.kernel_times()
            ks.append(t[0])
            rs.append(t[1])
        r.enable_profile(True)
        r.render_rows_async(cam.cam, out.data_ptr(), row0=0, row_step=8, n_rows=100, d_stats_ptr=st.data_ptr())
        torch.cuda.synchronize()
        s = [int(x) for x in st.cpu().tolist()]
        m = 2**64 - 1
        first_start, first_drain, last_end = (~s[13]) & m, (~s[14]) & m, s[15]
        res[f"bm{bm}_spp{spp}"] = {"sample_ms": round(min(ks[1:]), 4), "reduce_ms": round(min(rs[1:]), 4),
                                   "rays": s[0],
                                   "prof_start_to_drain_us": round((first_drain - first_start) / 100, 1),
                                   "prof_drain_to_end_us": round((last_end - first_drain) / 100, 1)}
        r.close()
        print(json.dumps({f"bm{bm}_spp{spp}": res[f"bm{bm}_spp{spp}"]}), file=sys.stderr, flush=True)
print(json.dumps(res))

#!/usr/bin/env python3
"""In-kernel instrumentation report (rt_context_enable_profile): per-ray sphere tests and BVH node
visits (exact counts) and the wave-cycle split refill / walk / shade, for each walk variant.

    python tools/kprofile.py --spp 100 --variants "bvh smem_u4"
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-with-zig_amd"))
import torch  # noqa: E402

import rtzig  # noqa: E402

def lanes_of(s):
    """Mean active lanes per block (round 6, rt.h stats[32..63] beside the wave-level counts): for each
    block, its wave-level executions, lane-level executions and their ratio.  None for a kernel
    without lane counts (direct mode)."""
    if len(s) < 64 or not s[32]:
        return None
    acw, acl = s[54:58], s[58:62]

    def row(w, l):
        return {"waves": w, "lanes": l, "mean_lanes": round(l / w, 3) if w else None}
    return {
        "seed_and_getRay": row(s[28], s[32]),
        "rejection_trip": row(s[27], s[33]),
        "scatter_finish": row(s[34], s[35]),
        "defocus_camera_finish": row(s[36], s[37]),
        "walk_any (started + resumed)": row(s[38], s[39]),
        "walk_start (always-list tests, slab setup)": row(s[29], s[40]),
        "walk_inner_step": row(s[7], s[3]),
        "leaf_round": row(s[8], s[51]),
        "candidate_block_all": row(s[9], s[52]),
        "candidate_block_always_list": {f"q{q}": row(acw[q], acl[q]) for q in range(4)},
        "candidate_block_leaf": row(s[9] - sum(acw), s[52] - sum(acl)),
        "root2_all": row(s[10], s[53]),
        "root2_always_list": row(s[62], s[63]),
        "root2_leaf": row(s[10] - s[62], s[53] - s[63]),
        "shade": row(s[30], s[41]),
        "shade_sky": row(s[42], s[43]),
        "shade_lambertian_metal": row(s[44], s[45]),
        "shade_dielectric": row(s[46], s[47]),
        "store": row(s[48], s[49]),
        "lanes_holding_a_path_per_iteration": row(s[26], s[50]),
        **({"seed_window": {"fills": s[64], "take_passes": s[65], "fresh_lanes_per_take": round(s[32] / s[65], 3),
                            "samples_per_fill": round(s[1] / s[64], 3)}} if len(s) > 65 and s[64] else {}),
    }


res_waves = torch.cuda.get_device_properties(0).multi_processor_count * 16 if torch.cuda.is_available() else 4096  # persistent grid: 16 waves per CU
ap = argparse.ArgumentParser()
ap.add_argument("--width", type=int, default=1200)
ap.add_argument("--aspect", type=float, default=1.5)
ap.add_argument("--spp", type=int, default=100)
ap.add_argument("--variants", default="bvh smem_u4")
ap.add_argument("--rows", default=None, help="row0:step:n (rank rehearsal), default: the whole image")
ap.add_argument("--out", default=None)
ap.add_argument("--scene", choices=["final", "ch9", "ch13"], default="final")
args = ap.parse_args()

if args.scene == "ch9":
    cam = rtzig.chapter9_camera(width=args.width, spp=args.spp)
elif args.scene == "ch13":
    cam = rtzig.chapter13_camera(width=args.width, spp=args.spp)
else:
    cam = rtzig.final_scene_camera(width=args.width, aspect_ratio=args.aspect, spp=args.spp)
H, W = cam.height, cam.width
r = rtzig.DeviceRenderer(0)
r.set_scene(cam.scene.world)
r.enable_timing(True)
row0, step, n_rows = (0, 1, H) if args.rows is None else tuple(int(x) for x in args.rows.split(":"))
rows = dict(row0=row0, row_step=step, n_rows=n_rows)
out = torch.empty((n_rows, W, 3), dtype=torch.float64, device="cuda:0")
stats = torch.zeros(rtzig.abi.RT_PROFILE_STATS_WORDS, dtype=torch.int64, device="cuda:0")
res = {"config": f"{W}x{H} {args.spp}spp, {len(cam.scene.world)} spheres", "variants": {}}
for v in args.variants.split():
    os.environ["RTZIG_KERNEL"] = v
    r.enable_profile(False)
    r.render_rows_async(cam.cam, out.data_ptr(), **rows)  # warm-up (code object, BVH, workspace)
    r.render_rows_async(cam.cam, out.data_ptr(), **rows)
    torch.cuda.synchronize()
    plain_ms, _ = r.kernel_times()
    r.enable_profile(True)
    stats.zero_()
    r.render_rows_async(cam.cam, out.data_ptr(), d_stats_ptr=stats.data_ptr(), **rows)
    torch.cuda.synchronize()
    prof_ms, _ = r.kernel_times()
    s = [int(x) for x in stats.cpu().tolist()]
    cyc = s[4] + s[5] + s[6] + s[16]
    res["variants"][v] = {
        "kernel": r.kernel_name(), "sample_kernel_ms": round(plain_ms, 3), "instrumented_ms": round(prof_ms, 3),
        "rays": s[0], "samples": s[1], "rays_per_sample": round(s[0] / s[1], 4),
        "sphere_tests_per_ray": round(s[2] / s[0], 3), "node_visits_per_ray": round(s[3] / s[0], 3),
        "wave_inner_iters_per_wave_iter": round(s[7] / max(1, s[0] / 64), 3),
        "wave_leaf_rounds_per_wave_iter": round(s[8] / max(1, s[0] / 64), 3),
        "lane_util_inner": round(s[3] / max(1, s[7] * 64), 4),
        "wave_cand_blocks_per_wave_iter": round(s[9] / max(1, s[0] / 64), 3),
        "wave_root2_blocks_per_wave_iter": round(s[10] / max(1, s[0] / 64), 3),
        "camera_ray_node_visits": round(s[11] / max(1, s[1]), 3),
        "camera_ray_sphere_tests": round(s[12] / max(1, s[1]), 3),
        "secondary_ray_node_visits": round((s[3] - s[11]) / max(1, s[0] - s[1]), 3),
        "secondary_ray_sphere_tests": round((s[2] - s[12]) / max(1, s[0] - s[1]), 3),
        "timeline_us": {"first_wave_start_to_first_drain": round(((~s[14] & (2**64 - 1)) - (~s[13] & (2**64 - 1))) / 100, 1)
                        if s[14] else None,
                        "first_drain_to_last_wave_end": round((s[15] - (~s[14] & (2**64 - 1))) / 100, 1)
                        if s[14] else None,
                        "first_drain_to_last_drain": round((s[22] - (~s[14] & (2**64 - 1))) / 100, 1)
                        if s[14] and s[22] else None,
                        "wave_tail_avg (own drain to own end)": round(s[20] / 100 / max(1, res_waves), 1),
                        "wave_tail_max": round(s[21] / 100, 1)},
        "cycle_split": {"refill": round(s[4] / cyc, 4), "walk": round(s[5] / cyc, 4), "shade": round(s[6] / cyc, 4), "trips": round(s[16] / cyc, 4),
                        "refill_parts": {"finalise": round(s[23] / cyc, 4), "hand_out": round(s[24] / cyc, 4),
                                         "seed_and_getRay": round(s[25] / cyc, 4)}},
        "scheduler": {"idle_sleeps": s[17], "deferred_finalisations": s[18], "refills_without_free_slot": s[19]},
        # true wave-level executions per loop iteration (stats[26..31]; the *_per_wave_iter figures above
        # are per 64 rays)
        "wave_level": ({"iterations": s[26], "rays_per_iter": round(s[0] / s[26], 3),
                        "inner_steps_per_iter": round(s[7] / s[26], 3), "leaf_rounds_per_iter": round(s[8] / s[26], 3),
                        "cand_blocks_per_iter": round(s[9] / s[26], 3), "root2_blocks_per_iter": round(s[10] / s[26], 3),
                        "trips_per_iter": round(s[27] / s[26], 3), "seed_blocks_per_iter": round(s[28] / s[26], 3),
                        "walk_starts_per_iter": round(s[29] / s[26], 3), "shade_blocks_per_iter": round(s[30] / s[26], 3),
                        "finalisations": s[31], "samples_per_iter": round(s[1] / s[26], 3)} if s[26] else None),
        "lanes": lanes_of(s),
        "raw": s,
    }
    r.enable_profile(False)
print(json.dumps(res))
if args.out:
    json.dump(res, open(args.out, "w"), indent=1)

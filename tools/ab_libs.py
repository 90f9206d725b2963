#!/usr/bin/env python3
"""In-process A/B of whole library builds (cdna guide rule 24): loads several copies of
librtzig.so (built from different revisions by tools/build_variant.sh), renders the same frame
with each in interleaved rounds, checks the outputs are bit-identical, and reports the sample
kernel's median HIP-event time per build.

    python tools/ab_libs.py ab/base.so ab/new.so --spp 100 --rounds 5
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-with-zig_amd"))
import torch  # noqa: E402

import rtzig  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--width", type=int, default=1200)
ap.add_argument("--aspect", type=float, default=1.5)
ap.add_argument("--spp", type=int, default=100)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--scene", choices=["final", "ch13", "ch9", "big"], default="final")
ap.add_argument("--n-spheres", type=int, default=4000,
                help="--scene big: random spheres on the final scene's ground (the tree no longer fits LDS)")
ap.add_argument("--row-step", type=int, default=1,
                help="render rank 0's interleaved row set of an N-rank job (rows 0, N, 2N, ...)")
ap.add_argument("--no-check", action="store_true", help="ablation builds: skip the bit-equality check")
ap.add_argument("--precision", choices=["f64", "f32"], default="f64", help="f32: fast mode (RT_PRECISION_F32)")
args = ap.parse_args()

if args.scene == "final":
    cam = rtzig.final_scene_camera(width=args.width, aspect_ratio=args.aspect, spp=args.spp)
elif args.scene == "ch13":
    cam = rtzig.chapter13_camera(width=args.width, spp=args.spp)
elif args.scene == "ch9":
    cam = rtzig.chapter9_camera(width=args.width, spp=args.spp)
else:  # a scene too large for the LDS tree: the BVH kernel walks its tree in global memory
    import numpy as np
    from rtzig.abi import D3, RtSphere
    rng = np.random.default_rng(4242)
    n = args.n_spheres
    arr = (RtSphere * n)()
    arr[0] = RtSphere(center=D3(0, -1000, 0), radius=1000.0, material=0, albedo=D3(0.5, 0.5, 0.5))
    c = rng.uniform([-11, 0.05, -11], [11, 0.4, 11], (n, 3))
    rad = rng.uniform(0.05, 0.2, n)
    mats = rng.integers(0, 3, n)
    alb = rng.uniform(0, 1, (n, 3))
    for k in range(1, n):
        arr[k] = RtSphere(center=D3(*c[k]), radius=float(rad[k]), material=int(mats[k]), albedo=D3(*alb[k]),
                          fuzz=0.2, refraction_index=1.5)
    cam = rtzig.final_scene_camera(width=args.width, aspect_ratio=args.aspect, spp=args.spp)
    cam.scene.world = arr
H, W = cam.height, cam.width
NR = (H + args.row_step - 1) // args.row_step
out = torch.empty((NR, W, 3), dtype=torch.float64, device="cuda:0")
runs = []
envs = {}
for spec in args.libs:  # "lib.so" or "lib.so:VAR=VAL" (an environment variable set around its renders)
    path, _, env = spec.partition(":")
    envs[spec] = tuple(env.split("=", 1)) if env else None
    L = C.CDLL(os.path.abspath(path))
    vp = C.c_void_p
    for name, res, argt in [("rt_context_create", C.c_int, [C.c_int, C.POINTER(vp)]),
                            ("rt_context_set_scene", C.c_int, [vp, C.POINTER(rtzig.RtSphere), C.c_size_t]),
                            ("rt_context_enable_timing", C.c_int, [vp, C.c_int]),
                            ("rt_context_kernel_times", C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
                            ("rt_render_rows_async", C.c_int, [vp, C.POINTER(rtzig.RtCamera), C.c_uint32, C.c_uint32,
                                                               C.c_uint32, C.c_uint32, vp, vp, vp]),
                            ("rt_context_set_precision", C.c_int, [vp, C.c_int]),
                            ("rt_last_error", C.c_char_p, [])]:
        getattr(L, name).restype = res
        getattr(L, name).argtypes = argt
    ctx = C.c_void_p()
    assert L.rt_context_create(0, C.byref(ctx)) == 0, L.rt_last_error()
    if envs[spec]:  # build-time knobs (the BVH is built in set_scene) as well as render-time ones
        os.environ[envs[spec][0]] = envs[spec][1]
    assert L.rt_context_set_scene(ctx, cam.scene.world, len(cam.scene.world)) == 0, L.rt_last_error()
    if envs[spec]:
        del os.environ[envs[spec][0]]
    assert L.rt_context_enable_timing(ctx, 1) == 0
    assert L.rt_context_set_precision(ctx, 1 if args.precision == "f32" else 0) == 0, L.rt_last_error()
    runs.append((spec, L, ctx))
times = {p: [] for p, _, _ in runs}
rtimes = {p: [] for p, _, _ in runs}
wtimes = {p: [] for p, _, _ in runs}  # wall time of render + synchronize (sample + reduce kernels of older builds)
ref = None
for rnd in range(args.rounds + 1):
    for path, L, ctx in runs:
        if envs[path]:
            os.environ[envs[path][0]] = envs[path][1]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = L.rt_render_rows_async(ctx, C.byref(cam.cam), 0, 0, args.row_step, NR, C.c_void_p(out.data_ptr()), None, None)
        assert rc == 0, L.rt_last_error()
        torch.cuda.synchronize()
        tw = (time.perf_counter() - t0) * 1e3
        if envs[path]:
            del os.environ[envs[path][0]]
        a, b = C.c_double(), C.c_double()
        assert L.rt_context_kernel_times(ctx, C.byref(a), C.byref(b)) == 0
        img = out.cpu()
        if ref is None:
            ref = img
        if not args.no_check and not torch.equal(img, ref):
            d = (img != ref).any(dim=-1)
            idx = d.nonzero()[:8].tolist()
            raise AssertionError(f"{path} output differs in {int(d.sum())} pixels, e.g. (row, col) {idx}")
        if rnd > 0:
            times[path].append(a.value)
            rtimes[path].append(b.value)
            wtimes[path].append(tw)
res = {p: {"median_ms": round(statistics.median(t), 3), "min_ms": round(min(t), 3),
           "Msamples_s": round(W * NR * args.spp / statistics.median(t) / 1e3, 1),
           "reduce_median_ms": round(statistics.median(rtimes[p]), 4),
           "wall_median_ms": round(statistics.median(wtimes[p]), 3)} for p, t in times.items()}
print(json.dumps({"config": f"{args.scene} {W}x{H} {args.spp}spp rows 0::{args.row_step}", "results": res}))

#!/usr/bin/env python3
"""One-shot cost of the drop-in as the reference uses it: ONE image per process
(/root/reference/src/main.zig:14-36: Scene.init + generateWorld, CameraBuilder.build,
camera.render() -> camera.zig:123-145, ppm.saveBinary).  Runs the C harness that mirrors the Zig
shim (tools/rt_render_c.c, built next to librtzig.so) as a fresh process per run and splits its wall
time, from spawn to exit, into:

    exec_and_library_load   spawn -> main() (exec, ld.so: librtzig.so + the HIP runtime libraries)
    scene_host / camera     Scene generation / CameraBuilder.build through the ABI
    rt_render               the call, with the library's own phase trace (RTZIG_TRACE=1):
                            HIP runtime init, context, scene build + upload, tree training,
                            workspace, first launch (code-object load), device wait, copy-out
    p6_write                PPM.saveBinary
    exit                    process teardown (HIP runtime shutdown)

Both sides stamp CLOCK_MONOTONIC (Python's time.monotonic).  Usage on the GPU box:

    python tools/dropin_cold.py [--runs 3] [--configs 2,4,5] > gpurun_out/dropin_cold.json
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "raytracing-with-zig_amd", "rt_render_c")

# BASELINE.json configs as rt_render_c arguments: width, spp, seed, aspect, scene
CONFIGS = {
    "2": ("400", "100", "0xdeadbeef", repr(16 / 9), "ch9"),
    "3": ("1200", "500", "0xdeadbeef", repr(16 / 9), "ch13"),
    "4": ("1200", "500", "0xdeadbeef", "1.5", "final"),
    "4_16x9": ("1200", "500", "0xdeadbeef", repr(16 / 9), "final"),
    "5": ("3840", "10000", "0xdeadbeef", repr(16 / 9), "final"),
    "golden": ("400", "10", "0xdeadbeef", repr(16 / 9), "final"),
}


def one_run(args, out_path, extra_env=None):
    env = dict(os.environ)
    env["RTZIG_TRACE"] = "1"
    if extra_env:
        env.update(extra_env)
    t_spawn = time.monotonic()
    p = subprocess.run([EXE, out_path, *args], capture_output=True, text=True, env=env, timeout=600)
    t_exit = time.monotonic()
    if p.returncode != 0:
        raise RuntimeError(f"rt_render_c {args} rc={p.returncode}: {p.stderr[-2000:]}")
    stamps = trace = None
    for line in p.stdout.splitlines():
        if line.startswith("{") and "harness_stamps" in line:
            stamps = json.loads(line)
    for line in p.stderr.splitlines():
        if line.startswith("{") and "rt_render_trace" in line:
            trace = json.loads(line)["rt_render_trace"]
    if stamps is None or trace is None:
        raise RuntimeError(f"no stamps / trace in the output: {p.stdout[-500:]} {p.stderr[-500:]}")
    s = stamps["harness_stamps"]
    ms = lambda a, b: round((b - a) * 1e3, 3)  # noqa: E731
    return {
        "total_ms": ms(t_spawn, t_exit),
        "to_file_written_ms": ms(t_spawn, s["saved"]),
        "exec_and_library_load_ms": ms(t_spawn, s["main"]),
        "scene_host_ms": ms(s["main"], s["scene"]),
        "camera_ms": ms(s["scene"], s["camera"]),
        "rt_render_ms": ms(s["camera"], s["render"]),
        "p6_write_ms": ms(s["render"], s["saved"]),
        "exit_ms": ms(s["saved"], t_exit),
        "rt_render_phases_ms": {k: round(v, 3) for k, v in trace["phases_ms"].items()},
        "kernel_ms": [round(k, 3) for k in trace["kernel_ms"]],
        "rays": stamps["rays"],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--configs", default="2,4,5")
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE for the harness (A/B hooks)")
    a = ap.parse_args()
    extra = dict(kv.split("=", 1) for kv in a.env)
    res = {"harness": "tools/rt_render_c.c (n_gpus = 0, RGB8, P6)", "runs_per_config": a.runs, "env": extra,
           "configs": {}}
    with tempfile.TemporaryDirectory() as td:
        for c in a.configs.split(","):
            args = CONFIGS[c]
            runs = []
            for r in range(a.runs):
                runs.append(one_run(args, os.path.join(td, f"cfg{c}_{r}.ppm"), extra))
                print(json.dumps({"config": c, "run": r, **{k: runs[-1][k] for k in
                                  ("total_ms", "rt_render_ms", "kernel_ms")}}), file=sys.stderr, flush=True)
            keys = [k for k in runs[0] if k.endswith("_ms") and not isinstance(runs[0][k], (dict, list))]
            med = {k: round(statistics.median(r[k] for r in runs), 3) for k in keys}
            phases = {k: round(statistics.median(r["rt_render_phases_ms"].get(k, 0.0) for r in runs), 3)
                      for k in runs[0]["rt_render_phases_ms"]}
            med["rt_render_phases_ms"] = phases
            med["kernel_ms"] = round(statistics.median(r["kernel_ms"][0] for r in runs), 3)
            w, spp, _, aspect, scene = args
            res["configs"][c] = {"args": {"width": int(w), "spp": int(spp), "aspect": float(aspect), "scene": scene},
                                 "median": med, "runs": runs}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

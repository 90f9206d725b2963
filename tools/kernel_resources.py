#!/usr/bin/env python3
"""Register and LDS budget of every kernel in rt_kernel.hip as the compiler allocated it
(hipcc -Rpass-analysis=kernel-resource-usage, the same flags as csrc/Makefile), written to
profiles/<tag>/kernel_resources.json.  rocprofv3's VGPR_Count column is not this count (it reports
64 for the 127-VGPR parity kernel), so the summaries quote the compiler's figures from here.

    python tools/kernel_resources.py <tag> [-D...]
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "raytracing-with-zig_amd", "csrc", "rt_kernel.hip")


def resources(extra=()):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-x", "hip", "--offload-arch=gfx950",
           "--cuda-device-only", "-c", SRC, "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage", *extra]
    err = subprocess.run(cmd, capture_output=True, text=True, check=True).stderr
    out, cur = {}, None
    for line in err.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\d+)", line)
        if m and cur:
            out[cur][m.group(1).strip()] = int(m.group(2))
    return out


if __name__ == "__main__":
    tag = sys.argv[1]
    res = resources(sys.argv[2:])
    d = os.path.join(ROOT, "profiles", tag)
    os.makedirs(d, exist_ok=True)
    json.dump({"source": "hipcc -Rpass-analysis=kernel-resource-usage " + " ".join(sys.argv[2:]), "kernels": res},
              open(os.path.join(d, "kernel_resources.json"), "w"), indent=1)
    for k, v in res.items():
        if "sample_kernel_bvh" in k:
            print(k[:60], v.get("VGPRs"), v.get("TotalSGPRs"), v.get("Occupancy [waves/SIMD]"))

#!/usr/bin/env python3
"""Compact register / scratch table of rt_kernel.hip's kernels as the product Makefile builds them.

    python tools/kres.py [-DRTZIG_...=...]
"""
import os
import re
import subprocess
import sys

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raytracing-with-zig_amd", "csrc")
err = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-x", "hip",
                      "--offload-arch=gfx950", "-fno-gpu-rdc", "-c", "rt_kernel.hip", "-o", os.devnull,
                      "-Rpass-analysis=kernel-resource-usage", *sys.argv[1:]], cwd=SRC, capture_output=True, text=True).stderr
cur, rows = None, {}
for line in err.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = m.group(2)
for k, v in rows.items():
    name = re.sub(r"^_ZN3rtk\d+", "", k)[:34]
    print(f"{name:34s} vgpr={v.get('VGPRs')} scratch={v.get('ScratchSize [bytes/lane]')} "
          f"spill={v.get('VGPRs Spill', '0')} waves={v.get('Occupancy [waves/SIMD]')}")

"""The shipped kernels' register budget, checked at build time (CPU; hipcc cross-compiles gfx950):
no sample kernel uses scratch memory (a stray by-reference flag or dynamically indexed local array
puts per-lane state in scratch: slower, and a spilling kernel faulted on the MI355X in round 4,
profiles/r04_occupancy), and the uninstrumented BVH kernels keep 4 waves per SIMD (<= 128 VGPRs,
DESIGN §5.1)."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _resources():
    err = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-x", "hip",
                          "--offload-arch=gfx950", "-fno-gpu-rdc", "-c", "rt_kernel.hip", "-o", os.devnull,
                          "-Rpass-analysis=kernel-resource-usage"],
                         cwd=os.path.join(ROOT, "raytracing-with-zig_amd", "csrc"), capture_output=True, text=True,
                         check=True).stderr
    cur, rows = None, {}
    for line in err.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
        if m and cur:
            rows[cur][m.group(1)] = int(m.group(2))
    return rows


def test_no_scratch_and_bvh_kernels_at_four_waves():
    rows = _resources()
    samples = {k: v for k, v in rows.items() if "sample_kernel" in k}
    assert len(samples) == 24, sorted(samples)
    assert all(v["ScratchSize [bytes/lane]"] == 0 for v in samples.values()), \
        {k: v["ScratchSize [bytes/lane]"] for k, v in samples.items() if v["ScratchSize [bytes/lane]"]}
    # sample_kernel_bvh<kLdsScene, kProf = false, kDirect> and the fast twin: 4 waves per SIMD
    plain = {k: v for k, v in rows.items() if re.search(r"sample_kernel_(bvh|fast)ILb[01]ELb0E", k)}
    assert len(plain) == 8
    assert all(v["Occupancy [waves/SIMD]"] == 4 and v["VGPRs"] <= 128 for v in plain.values()), plain

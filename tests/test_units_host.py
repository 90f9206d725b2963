"""Host check of the unit scheduler's chunk table (csrc/rt_schedule.hpp), CPU only."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_chunk_schedule_tiles_every_spp(tmp_path):
    exe = tmp_path / "test_units"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-x", "hip", "--offload-arch=gfx950",
                    os.path.join(ROOT, "tests", "cpp", "test_units.cpp"), "-o", str(exe)],
                   check=True, capture_output=True, timeout=300)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout
    assert out.stdout.strip().endswith("OK")

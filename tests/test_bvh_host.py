"""Host BVH builder invariants (CPU): compiles tests/cpp/test_bvh.cpp against csrc/rt_bvh.cpp."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("leaf", [4, 1, 2, 8])
def test_bvh_builder_invariants(tmp_path, leaf):
    """Builder invariants for the shipped leaf size (2) and the RTZIG_LEAF build knob's values."""
    exe = tmp_path / "test_bvh"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", f"-DRTZIG_LEAF={leaf}",
                    os.path.join(ROOT, "tests", "cpp", "test_bvh.cpp"),
                    os.path.join(ROOT, "raytracing-with-zig_amd", "csrc", "rt_bvh.cpp"),
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    print(out.stdout)
    assert out.returncode == 0, out.stdout
    assert out.stdout.strip().endswith("OK")

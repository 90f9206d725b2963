"""Exact division by invariant integers used in the kernel's refill (csrc/rt_fastdiv.h), CPU."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fastdiv_exact(tmp_path):
    exe = tmp_path / "test_fastdiv"
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "cpp", "test_fastdiv.cpp"),
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout
    assert out.stdout.strip().endswith("OK")

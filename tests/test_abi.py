"""The C-ABI library loads, exports every symbol include/rt.h declares, and its struct layouts match
the header (checked by compiling a probe against the header with gcc).  No GPU compute calls."""
import ctypes as C
import os
import re
import subprocess

import pytest

import rtzig
from rtzig import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rt.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(rt_\w+)\s*\(", text, flags=re.M)))


def test_header_lists_all_exports():
    assert header_functions() == sorted(rtzig.EXPORTED)


def test_library_exports_every_symbol():
    lib = rtzig.load()
    for name in header_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", rtzig.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (rt_\w+)", out))
    assert set(header_functions()) <= exported


def test_abi_version_and_error_string():
    lib = rtzig.load()
    assert lib.rt_abi_version() == 3
    assert isinstance(lib.rt_last_error(), bytes)


def test_struct_layout_matches_header(tmp_path):
    probe = tmp_path / "probe.c"
    probe.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "rt.h"
int main(void) {
  printf("%zu %zu %zu %zu\n", sizeof(rt_sphere), sizeof(rt_camera), sizeof(rt_camera_params), sizeof(rt_options));
  printf("%zu %zu %zu\n", offsetof(rt_sphere, material), offsetof(rt_sphere, albedo), offsetof(rt_sphere, refraction_index));
  printf("%zu %zu %zu\n", offsetof(rt_camera, pixel_samples_scale), offsetof(rt_camera, defocus_angle), offsetof(rt_camera, seed));
  printf("%zu %zu\n", offsetof(rt_options, output_format), offsetof(rt_options, stats_out));
  return 0;
}
''')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), str(probe), "-o", str(exe)], check=True)
    lines = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    sizes = list(map(int, lines[0].split()))
    assert sizes == [C.sizeof(abi.RtSphere), C.sizeof(abi.RtCamera), C.sizeof(abi.RtCameraParams),
                     C.sizeof(abi.RtOptions)]
    assert sizes == [abi.SPHERE_SIZE, abi.CAMERA_SIZE, abi.CAMERA_PARAMS_SIZE, abi.OPTIONS_SIZE]
    assert list(map(int, lines[1].split())) == [abi.RtSphere.material.offset, abi.RtSphere.albedo.offset,
                                                abi.RtSphere.refraction_index.offset]
    assert list(map(int, lines[2].split())) == [abi.RtCamera.pixel_samples_scale.offset,
                                                abi.RtCamera.defocus_angle.offset, abi.RtCamera.seed.offset]
    assert list(map(int, lines[3].split())) == [abi.RtOptions.output_format.offset,
                                                abi.RtOptions.stats_out.offset]


def test_invalid_arguments_fail_without_gpu_work():
    """Argument validation happens before any device call (reference-side `catch unreachable` /
    @panic become error codes)."""
    lib = rtzig.load()
    cam = rtzig.RtCamera(image_width=0, image_height=10, samples_per_pixel=1)
    opts = rtzig.RtOptions()
    rc = lib.rt_render(C.byref(cam), (rtzig.RtSphere * 1)(), 1, C.byref(opts), C.c_void_p(1))
    assert rc == abi.RT_ERR_INVALID
    assert b"image_width" in lib.rt_last_error()
    cam = rtzig.RtCamera(image_width=4, image_height=4, samples_per_pixel=1)
    rc = lib.rt_render(C.byref(cam), None, 0, C.byref(opts), C.c_void_p(1))
    assert rc == abi.RT_ERR_INVALID
    bad = (rtzig.RtSphere * 1)(rtzig.RtSphere(radius=1.0, material=7))
    rc = lib.rt_render(C.byref(cam), bad, 1, C.byref(opts), C.c_void_p(1))
    assert rc == abi.RT_ERR_INVALID
    assert b"material" in lib.rt_last_error()
    cam.samples_per_pixel = 0
    rc = lib.rt_render(C.byref(cam), (rtzig.RtSphere * 1)(rtzig.RtSphere(radius=1.0)), 1,
                       C.byref(opts), C.c_void_p(1))
    assert rc == abi.RT_ERR_INVALID
    # non-finite camera vectors are rejected (t_max = +inf stays legal)
    cam.samples_per_pixel = 1
    cam.t_max = float("inf")
    cam.center[1] = float("nan")
    rc = lib.rt_render(C.byref(cam), (rtzig.RtSphere * 1)(rtzig.RtSphere(radius=1.0)), 1,
                       C.byref(opts), C.c_void_p(1))
    assert rc == abi.RT_ERR_INVALID and b"finite" in lib.rt_last_error()
    cam.center[1] = 0.0
    cam.t_min = float("inf")
    rc = lib.rt_render(C.byref(cam), (rtzig.RtSphere * 1)(rtzig.RtSphere(radius=1.0)), 1,
                       C.byref(opts), C.c_void_p(1))
    assert rc == abi.RT_ERR_INVALID


def test_single_hip_runtime_per_process():
    """rtzig loads torch's HIP runtime before librtzig (rtzig/lib.py), so a process that uses both
    maps ONE libamdhip64 — a second runtime breaks torch's GPU init once our kernels have run."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "import rtzig; rtzig.load()\n"
            "import torch\n"
            "paths = {l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}\n"
            "print(len(paths), sorted(paths))\n") % os.path.join(ROOT, "raytracing-with-zig_amd")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.startswith("1 "), out.stdout

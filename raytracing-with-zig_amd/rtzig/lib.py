"""Loader for librtzig.so (the HIP path tracer + C ABI of include/rt.h).

The product path has NO fallback: if the shared library is missing this module raises, and every
render call goes through the HIP kernel on a gfx950 device (rt_render / rt_render_rows_async).
"""
import ctypes as C
import os

from .abi import RtCamera, RtCameraParams, RtOptions, RtSphere

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "librtzig.so")

# Every symbol include/rt.h declares (tests/test_abi.py checks the header against this list).
EXPORTED = [
    "rt_render",
    "rt_context_create",
    "rt_context_destroy",
    "rt_context_set_scene",
    "rt_render_rows_async",
    "rt_render_rows_async_split",
    "rt_render_rows_async_deferred",
    "rt_context_flush",
    "rt_context_fold_pending",
    "rt_kernel_name",
    "rt_context_tree_info",
    "rt_context_workspace_bytes",
    "rt_context_enable_timing",
    "rt_context_kernel_times",
    "rt_context_kernel_times_total",
    "rt_context_enable_profile",
    "rt_context_set_precision",
    "rt_context_sync",
    "rt_release_cached_contexts",
    "rt_scene_final",
    "rt_scene_chapter13",
    "rt_camera_build",
    "rt_color_to_rgb8",
    "rt_ppm_p6_size",
    "rt_ppm_encode_p6",
    "rt_ppm_save_p6",
    "rt_ppm_p3_size",
    "rt_ppm_encode_p3",
    "rt_ppm_save_p3",
    "rt_sample_key",
    "rt_last_error",
    "rt_abi_version",
]


class RtError(RuntimeError):
    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


_lib = None


def _declare(lib):
    P = C.POINTER
    vp = C.c_void_p
    sigs = {
        "rt_render": (C.c_int, [P(RtCamera), P(RtSphere), C.c_size_t, P(RtOptions), vp]),
        "rt_context_create": (C.c_int, [C.c_int, P(vp)]),
        "rt_context_destroy": (C.c_int, [vp]),
        "rt_context_set_scene": (C.c_int, [vp, P(RtSphere), C.c_size_t]),
        "rt_render_rows_async": (C.c_int, [vp, P(RtCamera), C.c_uint32, C.c_uint32, C.c_uint32,
                                           C.c_uint32, vp, vp, vp]),
        "rt_render_rows_async_split": (C.c_int, [vp, P(RtCamera), C.c_uint32, C.c_uint32, C.c_uint32,
                                                 C.c_uint32, vp, vp, vp, vp]),
        "rt_render_rows_async_deferred": (C.c_int, [vp, P(RtCamera), C.c_uint32, C.c_uint32, C.c_uint32,
                                                    C.c_uint32, vp, vp, vp, vp]),
        "rt_context_flush": (C.c_int, [vp]),
        "rt_context_fold_pending": (C.c_int, [vp, P(C.c_int)]),
        "rt_kernel_name": (C.c_char_p, [vp]),
        "rt_context_tree_info": (C.c_int, [vp, P(C.c_uint32)]),
        "rt_context_workspace_bytes": (C.c_int, [vp, P(C.c_uint64)]),
        "rt_context_enable_timing": (C.c_int, [vp, C.c_int]),
        "rt_context_kernel_times": (C.c_int, [vp, P(C.c_double), P(C.c_double)]),
        "rt_context_kernel_times_total": (C.c_int, [vp, P(C.c_double), P(C.c_double), P(C.c_uint32)]),
        "rt_context_enable_profile": (C.c_int, [vp, C.c_int]),
        "rt_context_set_precision": (C.c_int, [vp, C.c_int]),
        "rt_context_sync": (C.c_int, [vp]),
        "rt_release_cached_contexts": (C.c_int, []),
        "rt_scene_final": (C.c_int, [C.c_uint64, P(RtSphere), C.c_size_t, P(C.c_size_t),
                                     P(C.c_uint64)]),
        "rt_scene_chapter13": (C.c_int, [P(RtSphere), C.c_size_t, P(C.c_size_t)]),
        "rt_camera_build": (C.c_int, [P(RtCameraParams), P(RtCamera)]),
        "rt_color_to_rgb8": (C.c_int, [P(C.c_double), C.c_size_t, C.c_uint32, P(C.c_uint8)]),
        "rt_ppm_p6_size": (C.c_size_t, [C.c_uint32, C.c_uint32]),
        "rt_ppm_encode_p6": (C.c_int, [P(C.c_uint8), C.c_uint32, C.c_uint32, P(C.c_uint8),
                                       C.c_size_t]),
        "rt_ppm_save_p6": (C.c_int, [C.c_char_p, P(C.c_uint8), C.c_uint32, C.c_uint32]),
        "rt_ppm_p3_size": (C.c_size_t, [P(C.c_uint8), C.c_uint32, C.c_uint32]),
        "rt_ppm_encode_p3": (C.c_int, [P(C.c_uint8), C.c_uint32, C.c_uint32, P(C.c_uint8),
                                       C.c_size_t]),
        "rt_ppm_save_p3": (C.c_int, [C.c_char_p, P(C.c_uint8), C.c_uint32, C.c_uint32]),
        "rt_sample_key": (C.c_uint64, [C.c_uint64, C.c_uint64, C.c_uint64]),
        "rt_last_error": (C.c_char_p, []),
        "rt_abi_version": (C.c_int, []),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def _bind_torch_hip_runtime():
    """One HIP runtime per process.  PyTorch-ROCm wheels bundle their own libamdhip64 (SONAME
    libamdhip64.so.7, the same as /opt/rocm's) plus their own libhsa-runtime64, and torch's
    libc10_hip NEEDs the unversioned name.  Loaded AFTER librtzig, torch therefore maps a second
    HIP + ROCr stack next to ours, and that stack fails to initialise once our kernels have run
    ("No HIP GPUs are available").  Loaded BEFORE, torch's runtime is the libamdhip64.so.7 the
    dynamic linker hands librtzig too: both share one runtime, one device context and its streams.
    Processes without torch (the Zig host, tools/rt_render_c) just use /opt/rocm's runtime."""
    try:
        import torch  # noqa: F401  (import only: maps torch's HIP runtime, does not init a GPU)
    except ImportError:
        pass


def load():
    """Load librtzig.so (raises if it has not been built — there is no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(make -C raytracing-with-zig_amd/csrc)")
        _bind_torch_hip_runtime()
        lib = C.CDLL(LIB_PATH)
        _declare(lib)
        _lib = lib
    return _lib


def check(fn_name, rc):
    if rc != 0:
        msg = load().rt_last_error()
        raise RtError(fn_name, rc, msg.decode() if msg else "")
    return rc

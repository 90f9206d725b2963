"""Python mirror of the reference's host API over the C ABI (names follow the Zig code).

    scene = Scene.init(0xdeadbeef)                      # Scene.zig:23
    scene.generateWorld()                               # Scene.zig:48
    camera = (Camera.builder(400, 16.0 / 9.0)           # camera.zig:109
              .setScene(scene).setDefocusAngle(0.6).setFocusDist(10)
              .setViewport((13, 2, 3), (0, 0, 0), 20).setSamplesPerPixel(10)
              .build())                                 # camera.zig:300
    ppm = camera.render()                               # camera.zig:123 -> rt_render (HIP)
    ppm.saveBinary("images/chapter14.ppm")              # ppm.zig:42

Scene generation and camera construction run in the C++ host mirror (csrc/rt_host.cpp); render()
runs the HIP kernel on gfx950 GPUs.  There is no CPU fallback.
"""
import ctypes as C
import math

import numpy as np

from . import abi
from .abi import D3, RtCamera, RtCameraParams, RtOptions, RtSphere
from .lib import check, load

INF = math.inf


class Scene:
    """Scene.zig:16-187: world (Hittable list), seed, interval."""

    def __init__(self, seed):
        self.seed = seed
        self.world = (RtSphere * 0)()
        self.interval = (1e-3, INF)  # Scene.zig:21
        self.prng_state = None       # Xoshiro256++ words after generateWorld (for oracle A)

    @staticmethod
    def init(seed=None):
        if seed is None:
            import secrets
            seed = secrets.randbits(64)  # std.posix.getrandom stand-in (Scene.zig:33-37)
        return Scene(seed)

    def generateWorld(self):
        lib = load()
        n = C.c_size_t()
        check("rt_scene_final", lib.rt_scene_final(self.seed, None, 0, C.byref(n), None))
        arr = (RtSphere * n.value)()
        st = (C.c_uint64 * 4)()
        check("rt_scene_final", lib.rt_scene_final(self.seed, arr, n.value, C.byref(n), st))
        self.world = _concat(self.world, arr)
        self.prng_state = list(st)
        return self

    def generateChapter13(self):
        lib = load()
        n = C.c_size_t()
        arr = (RtSphere * 8)()
        check("rt_scene_chapter13", lib.rt_scene_chapter13(arr, 8, C.byref(n)))
        self.world = _concat(self.world, (RtSphere * n.value).from_buffer_copy(arr))
        return self

    def add(self, center, radius, material, albedo=(1, 1, 1), fuzz=0.0, refraction_index=1.0):
        s = RtSphere(center=D3(*center), radius=max(0.0, radius), material=material,
                     albedo=D3(*albedo), fuzz=fuzz, refraction_index=refraction_index)
        self.world = _concat(self.world, (RtSphere * 1)(s))
        return self


def _concat(a, b):
    out = (RtSphere * (len(a) + len(b)))()
    C.memmove(out, a, C.sizeof(a))
    C.memmove(C.addressof(out) + C.sizeof(a), b, C.sizeof(b))
    return out


class CameraBuilder:
    """camera.zig:233-346 (defaults camera.zig:218-232)."""

    def __init__(self, width, aspect_ratio):
        self.p = RtCameraParams(image_width=width, samples_per_pixel=100, bounce_max=50,
                                aspect_ratio=aspect_ratio, look_from=D3(0, 0, 0),
                                look_at=D3(0, 0, -1), v_up=D3(0, 1, 0), vfov=90.0,
                                defocus_angle=0.0, focus_dist=10.0, t_min=1e-3, t_max=INF,
                                seed=0)
        self.scene = None

    def setScene(self, scene):
        self.scene = scene
        self.p.seed = scene.seed
        self.p.t_min, self.p.t_max = scene.interval
        return self

    def setFocusDist(self, d):
        self.p.focus_dist = d
        return self

    def setDefocusAngle(self, a):
        self.p.defocus_angle = a
        return self

    def setViewport(self, look_from, look_at, vfov):
        self.p.look_from = D3(*look_from)
        self.p.look_at = D3(*look_at)
        self.p.vfov = vfov
        return self

    def setSamplesPerPixel(self, spp):
        self.p.samples_per_pixel = spp
        return self

    def setBounceMax(self, b):
        self.p.bounce_max = b
        return self

    def setVUp(self, v):
        self.p.v_up = D3(*v)
        return self

    def build(self):
        cam = RtCamera()
        check("rt_camera_build", load().rt_camera_build(C.byref(self.p), C.byref(cam)))
        return Camera(cam, self.scene if self.scene is not None else Scene.init(None))


class Camera:
    """camera.zig:82-216.  `cam` holds the flattened fields that cross the C ABI."""

    def __init__(self, cam, scene):
        self.cam = cam
        self.scene = scene

    @staticmethod
    def builder(width, aspect_ratio):
        return CameraBuilder(width, aspect_ratio)

    @property
    def width(self):
        return self.cam.image_width

    @property
    def height(self):
        return self.cam.image_height

    def render(self, n_gpus=0, device=0, output="linear", stats=None, precision="f64"):
        """Camera.render (camera.zig:123-145) on the GPU(s).  Returns a PPM."""
        return PPM(self.width, self.height,
                   render(self.cam, self.scene.world, n_gpus=n_gpus, device=device,
                          output=output, stats=stats, precision=precision))


_PRECISION = {"f64": abi.RT_PRECISION_F64, "f32": abi.RT_PRECISION_F32}


def render(cam, spheres, n_gpus=0, device=0, output="linear", stats=None, precision="f64"):
    """rt_render: whole image into host memory.  linear -> (H, W, 3) f64; rgb8 -> (H, W, 3) u8.
    precision: "f64" (parity, bit-exact) or "f32" (fast mode, statistical parity)."""
    lib = load()
    W, H = cam.image_width, cam.image_height
    if output == "linear":
        out = np.zeros((H, W, 3), np.float64)
        fmt = abi.RT_OUT_LINEAR_F64
    elif output == "rgb8":
        out = np.zeros((H, W, 3), np.uint8)
        fmt = abi.RT_OUT_RGB8
    else:
        raise ValueError(output)
    st = (C.c_uint64 * 2)()
    opts = RtOptions(n_gpus=n_gpus, device=device, pixel_stride=3, output_format=fmt,
                     precision=_PRECISION[precision], stats_out=C.cast(st, C.POINTER(C.c_uint64)))
    n = len(spheres)
    arr = spheres if isinstance(spheres, C.Array) else (RtSphere * n)(*spheres)
    check("rt_render", lib.rt_render(C.byref(cam), arr, n, C.byref(opts),
                                     out.ctypes.data_as(C.c_void_p)))
    if stats is not None:
        stats["rays"] = st[0]
        stats["samples"] = st[1]
    return out


class DeviceRenderer:
    """Device-resident renderer for one GPU (rt_context): scene uploaded once, rows rendered into
    device memory (e.g. a torch tensor's data_ptr) on a caller-provided HIP stream."""

    def __init__(self, device=0):
        self.lib = load()
        self.ctx = C.c_void_p()
        check("rt_context_create", self.lib.rt_context_create(device, C.byref(self.ctx)))
        self.device = device

    def set_scene(self, spheres):
        n = len(spheres)
        check("rt_context_set_scene", self.lib.rt_context_set_scene(self.ctx, spheres, n))

    def render_rows_async(self, cam, d_out_ptr, row0=0, row_step=1, n_rows=None, output="linear",
                          d_stats_ptr=None, stream_ptr=None, out_stream_ptr=None, deferred=False):
        """out_stream_ptr: complete the output on that stream instead (rt_render_rows_async_split:
        direct mode's reduce pass runs there, over two per-sample buffers taken in turn, so it
        overlaps the next call's sample kernel on stream_ptr).  deferred (with out_stream_ptr):
        rt_render_rows_async_deferred — this call's output completes after the NEXT deferred call (or
        flush() / sync()), its reduce pass folded by that call's drained waves."""
        if n_rows is None:
            n_rows = (cam.image_height - row0 + row_step - 1) // row_step
        fmt = abi.RT_OUT_LINEAR_F64 if output == "linear" else abi.RT_OUT_RGB8
        if deferred:  # out_stream_ptr 0 is the HIP null stream (torch's default stream)
            check("rt_render_rows_async_deferred",
                  self.lib.rt_render_rows_async_deferred(self.ctx, C.byref(cam), fmt, row0, row_step, n_rows,
                                                         C.c_void_p(d_out_ptr), C.c_void_p(d_stats_ptr or 0),
                                                         C.c_void_p(stream_ptr or 0), C.c_void_p(out_stream_ptr or 0)))
            return
        if out_stream_ptr is not None:
            check("rt_render_rows_async_split",
                  self.lib.rt_render_rows_async_split(self.ctx, C.byref(cam), fmt, row0, row_step, n_rows,
                                                      C.c_void_p(d_out_ptr), C.c_void_p(d_stats_ptr or 0),
                                                      C.c_void_p(stream_ptr or 0), C.c_void_p(out_stream_ptr or 0)))
            return
        check("rt_render_rows_async",
              self.lib.rt_render_rows_async(self.ctx, C.byref(cam), fmt, row0, row_step, n_rows,
                                            C.c_void_p(d_out_ptr), C.c_void_p(d_stats_ptr or 0),
                                            C.c_void_p(stream_ptr or 0)))

    def flush(self):
        """Runs a pending deferred reduce pass (rt_context_flush)."""
        check("rt_context_flush", self.lib.rt_context_flush(self.ctx))

    def fold_pending(self):
        """True if the last deferred call left its output pending (its reduce pass not yet run)."""
        v = C.c_int()
        check("rt_context_fold_pending", self.lib.rt_context_fold_pending(self.ctx, C.byref(v)))
        return bool(v.value)

    def sync(self):
        """Waits for the last render; raises if the kernel recorded a failure."""
        check("rt_context_sync", self.lib.rt_context_sync(self.ctx))

    def set_precision(self, precision):
        """"f64" (parity kernel, default) or "f32" (fast mode) for later renders."""
        check("rt_context_set_precision", self.lib.rt_context_set_precision(self.ctx, _PRECISION[precision]))

    def kernel_name(self):
        return self.lib.rt_kernel_name(self.ctx).decode()

    def tree_info(self):
        """The walk the next render uses: {"bvh", "nodes", "leaves", "depth", "always", "trained"}."""
        info = (C.c_uint32 * 6)()
        check("rt_context_tree_info", self.lib.rt_context_tree_info(self.ctx, info))
        return dict(zip(("bvh", "nodes", "leaves", "depth", "always", "trained"), [int(x) for x in info]))

    def workspace_bytes(self):
        """Device bytes the context's render workspace holds (rt.h "Workspace")."""
        b = C.c_uint64()
        check("rt_context_workspace_bytes", self.lib.rt_context_workspace_bytes(self.ctx, C.byref(b)))
        return b.value

    def enable_timing(self, enable=True):
        check("rt_context_enable_timing", self.lib.rt_context_enable_timing(self.ctx, int(enable)))

    def enable_profile(self, enable=True):
        """Instrumented kernels: the stats buffer passed to render_rows_async must hold 32 u64."""
        check("rt_context_enable_profile", self.lib.rt_context_enable_profile(self.ctx, int(enable)))

    def kernel_times(self):
        """(sample_kernel_ms, reduce_kernel_ms) of the last render call (HIP events)."""
        a, b = C.c_double(), C.c_double()
        check("rt_context_kernel_times", self.lib.rt_context_kernel_times(self.ctx, C.byref(a), C.byref(b)))
        return a.value, b.value

    def kernel_times_total(self):
        """(sample_kernel_ms, reduce_kernel_ms, launches) summed since timing was enabled."""
        a, b, n = C.c_double(), C.c_double(), C.c_uint32()
        check("rt_context_kernel_times_total",
              self.lib.rt_context_kernel_times_total(self.ctx, C.byref(a), C.byref(b), C.byref(n)))
        return a.value, b.value, n.value

    def close(self):
        """rt_context_destroy: runs a pending deferred reduce pass and waits for every launch first."""
        if self.ctx:
            ctx, self.ctx = self.ctx, C.c_void_p()
            check("rt_context_destroy", self.lib.rt_context_destroy(ctx))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PPM:
    """ppm.zig:5-61: framebuffer + P6 (saveBinary) and P3 (save) writers."""

    def __init__(self, width, height, pixels):
        self.width, self.height, self.pixels = width, height, pixels

    def toRgb(self):
        if self.pixels.dtype == np.uint8:
            return self.pixels
        return to_rgb8(self.pixels)

    def encodeBinary(self):
        return encode_p6(self.toRgb(), self.width, self.height)

    def saveBinary(self, path):
        rgb = np.ascontiguousarray(self.toRgb())
        check("rt_ppm_save_p6", load().rt_ppm_save_p6(
            path.encode(), rgb.ctypes.data_as(C.POINTER(C.c_uint8)), self.width, self.height))

    def encode(self):
        return encode_p3(self.toRgb(), self.width, self.height)

    def save(self, path):
        """PPM.save (ppm.zig:25-39): the P3 ASCII file."""
        rgb = np.ascontiguousarray(self.toRgb())
        check("rt_ppm_save_p3", load().rt_ppm_save_p3(
            path.encode(), rgb.ctypes.data_as(C.POINTER(C.c_uint8)), self.width, self.height))


def to_rgb8(linear):
    """Color.toRgb (color.zig:63-80) over an (..., 3) f64 array (host C++)."""
    lin = np.ascontiguousarray(linear, dtype=np.float64)
    n = lin.size // 3
    rgb = np.zeros(lin.shape, np.uint8)
    check("rt_color_to_rgb8", load().rt_color_to_rgb8(
        lin.ctypes.data_as(C.POINTER(C.c_double)), n, 3, rgb.ctypes.data_as(C.POINTER(C.c_uint8))))
    return rgb


def encode_p6(rgb, width, height):
    lib = load()
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    size = lib.rt_ppm_p6_size(width, height)
    buf = (C.c_uint8 * size)()
    check("rt_ppm_encode_p6", lib.rt_ppm_encode_p6(rgb.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                   width, height, buf, size))
    return bytes(buf)


def encode_p3(rgb, width, height):
    lib = load()
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    ptr = rgb.ctypes.data_as(C.POINTER(C.c_uint8))
    size = lib.rt_ppm_p3_size(ptr, width, height)
    buf = (C.c_uint8 * size)()
    check("rt_ppm_encode_p3", lib.rt_ppm_encode_p3(ptr, width, height, buf, size))
    return bytes(buf)


def release_cached_contexts():
    """Frees rt_render's per-device cached contexts (the next render creates them again)."""
    check("rt_release_cached_contexts", load().rt_release_cached_contexts())


def sample_key(seed, pixel, sample):
    return load().rt_sample_key(seed, pixel, sample)


# ---- presets (BASELINE.json configs) --------------------------------------------------------------
def final_scene_camera(width=1200, aspect_ratio=1.5, spp=500, seed=0xDEADBEEF, bounce_max=50):
    """main.zig:20-31 preset on the final random-sphere scene (configs 4/5, and the golden test
    at width 400, aspect 16/9, spp 10)."""
    scene = Scene.init(seed).generateWorld()
    return (Camera.builder(width, aspect_ratio).setScene(scene).setDefocusAngle(0.6)
            .setFocusDist(10).setViewport((13, 2, 3), (0, 0, 0), 20).setSamplesPerPixel(spp)
            .setBounceMax(bounce_max).build())


def chapter13_camera(width=1200, aspect_ratio=16.0 / 9.0, spp=500, seed=0xDEADBEEF):
    """Config 3: generateChapter13 (Scene.zig:136-182) with the book's chapter-13 camera."""
    scene = Scene.init(seed).generateChapter13()
    return (Camera.builder(width, aspect_ratio).setScene(scene).setDefocusAngle(10.0)
            .setFocusDist(3.4).setViewport((-2, 2, 1), (0, 0, -1), 20).setSamplesPerPixel(spp)
            .build())


def chapter9_camera(width=400, aspect_ratio=16.0 / 9.0, spp=100, seed=0xDEADBEEF):
    """Config 2: two Lambertian spheres (albedo 0.5), vFov 90, no defocus, focus 1."""
    scene = Scene.init(seed)
    scene.add((0, 0, -1), 0.5, abi.RT_LAMBERTIAN, albedo=(0.5, 0.5, 0.5))
    scene.add((0, -100.5, -1), 100, abi.RT_LAMBERTIAN, albedo=(0.5, 0.5, 0.5))
    return (Camera.builder(width, aspect_ratio).setScene(scene).setDefocusAngle(0.0)
            .setFocusDist(1.0).setViewport((0, 0, 0), (0, 0, -1), 90).setSamplesPerPixel(spp)
            .build())

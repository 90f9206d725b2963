"""ctypes mirror of include/rt.h (the C ABI of the MI355X path tracer).

Struct layouts must stay byte-identical to rt.h; tests/test_abi.py checks sizes and offsets.
"""
import ctypes as C

RT_OK = 0
RT_ERR_INVALID = -1
RT_ERR_HIP = -2
RT_ERR_NO_DEVICE = -3
RT_ERR_CAPACITY = -4
RT_ERR_IO = -5

RT_LAMBERTIAN = 0
RT_METAL = 1
RT_DIELECTRIC = 2

RT_OUT_LINEAR_F64 = 0
RT_OUT_RGB8 = 1
RT_PRECISION_F64 = 0
RT_PRECISION_F32 = 1
RT_PROFILE_STATS_WORDS = 72  # uint64 words of an instrumented render's d_stats (rt.h)

D3 = C.c_double * 3


class RtSphere(C.Structure):
    """rt_sphere: one Hittable .sphere (sphere.zig:13-16) with its Material (material.zig:126)."""
    _fields_ = [
        ("center", D3),
        ("radius", C.c_double),
        ("material", C.c_uint32),
        ("reserved", C.c_uint32),
        ("albedo", D3),
        ("fuzz", C.c_double),
        ("refraction_index", C.c_double),
    ]


class RtCamera(C.Structure):
    """rt_camera: built Camera fields (camera.zig:82-103) + Scene.interval/seed (Scene.zig:19-21)."""
    _fields_ = [
        ("image_width", C.c_uint32),
        ("image_height", C.c_uint32),
        ("samples_per_pixel", C.c_uint32),
        ("bounce_max", C.c_uint32),
        ("pixel_samples_scale", C.c_double),
        ("center", D3),
        ("pixel0", D3),
        ("du", D3),
        ("dv", D3),
        ("defocus_disk_u", D3),
        ("defocus_disk_v", D3),
        ("defocus_angle", C.c_double),
        ("t_min", C.c_double),
        ("t_max", C.c_double),
        ("seed", C.c_uint64),
    ]


class RtOptions(C.Structure):
    _fields_ = [
        ("n_gpus", C.c_int32),
        ("device", C.c_int32),
        ("pixel_stride", C.c_uint32),
        ("output_format", C.c_uint32),
        ("precision", C.c_uint32),
        ("reserved", C.c_uint32),
        ("stats_out", C.POINTER(C.c_uint64)),
    ]


class RtCameraParams(C.Structure):
    """rt_camera_params: CameraBuilder inputs (camera.zig:233-251)."""
    _fields_ = [
        ("image_width", C.c_uint32),
        ("samples_per_pixel", C.c_uint32),
        ("bounce_max", C.c_uint32),
        ("reserved", C.c_uint32),
        ("aspect_ratio", C.c_double),
        ("look_from", D3),
        ("look_at", D3),
        ("v_up", D3),
        ("vfov", C.c_double),
        ("defocus_angle", C.c_double),
        ("focus_dist", C.c_double),
        ("t_min", C.c_double),
        ("t_max", C.c_double),
        ("seed", C.c_uint64),
    ]


SPHERE_SIZE = 80
CAMERA_SIZE = 200
CAMERA_PARAMS_SIZE = 144
OPTIONS_SIZE = 32


def sphere_array(n):
    return (RtSphere * n)()


def camera_to_dict(cam):
    out = {}
    for name, _ in RtCamera._fields_:
        v = getattr(cam, name)
        out[name] = list(v) if isinstance(v, C.Array) else v
    return out

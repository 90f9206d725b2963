"""ctypes wrapper around oracle/liboracle.so — the CPU parity checker (test infrastructure only).

Mode A = the reference's single sequential RNG stream (pinned to test-files/chapter14.ppm);
mode B = same arithmetic, per-(pixel, sample) streams (the GPU's RNG layout).
"""
import ctypes as C
import os

import numpy as np

from rtzig.abi import RtCamera, RtCameraParams, RtSphere

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")

P = C.POINTER
dp = P(C.c_double)


class Oracle:
    def __init__(self, path=ORACLE_SO):
        L = C.CDLL(path)
        L.oracle_scene_final.argtypes = [C.c_uint64, P(RtSphere), C.c_size_t, P(C.c_size_t), P(C.c_uint64)]
        L.oracle_scene_chapter13.argtypes = [P(RtSphere), C.c_size_t, P(C.c_size_t)]
        L.oracle_camera_build.argtypes = [P(RtCameraParams), P(RtCamera)]
        L.oracle_render_a.argtypes = [P(RtCamera), P(RtSphere), C.c_size_t, P(C.c_uint64), dp, P(C.c_uint64)]
        L.oracle_render_b.argtypes = [P(RtCamera), P(RtSphere), C.c_size_t, C.c_uint32, C.c_uint32,
                                      C.c_uint32, dp, P(C.c_uint64), C.c_int]
        L.oracle_to_rgb8.argtypes = [dp, C.c_size_t, P(C.c_uint8)]
        L.oracle_ppm_p6.argtypes = [P(C.c_uint8), C.c_uint32, C.c_uint32, P(C.c_uint8), C.c_size_t]
        L.oracle_ppm_p6.restype = C.c_size_t
        L.oracle_sample_key.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
        L.oracle_sample_key.restype = C.c_uint64
        L.oracle_sphere_hit.argtypes = [P(RtSphere), dp, dp, C.c_double, C.c_double, dp, dp, dp, P(C.c_int)]
        L.oracle_world_hit.argtypes = [P(RtSphere), C.c_size_t, dp, dp, C.c_double, C.c_double, dp]
        L.oracle_world_hit.restype = C.c_long
        L.oracle_random_doubles.argtypes = [C.c_uint64, C.c_size_t, dp]
        L.oracle_random_u64.argtypes = [C.c_uint64, C.c_size_t, P(C.c_uint64)]
        L.oracle_render_book.argtypes = [C.c_int, C.c_uint32, C.c_double, P(C.c_uint8), P(C.c_uint32)]
        L.oracle_reflect.argtypes = [dp, dp, dp]
        L.oracle_refract.argtypes = [dp, dp, C.c_double, dp]
        self.L = L

    # ---- scenes / camera ------------------------------------------------------------------------
    def scene_final(self, seed):
        n = C.c_size_t()
        self.L.oracle_scene_final(seed, None, 0, C.byref(n), None)
        arr = (RtSphere * n.value)()
        st = (C.c_uint64 * 4)()
        rc = self.L.oracle_scene_final(seed, arr, n.value, C.byref(n), st)
        assert rc == 0
        return arr, list(st)

    def scene_chapter13(self):
        arr = (RtSphere * 8)()
        n = C.c_size_t()
        assert self.L.oracle_scene_chapter13(arr, 8, C.byref(n)) == 0
        return (RtSphere * n.value).from_buffer_copy(arr)

    def camera_build(self, params):
        cam = RtCamera()
        assert self.L.oracle_camera_build(C.byref(params), C.byref(cam)) == 0
        return cam

    # ---- renders --------------------------------------------------------------------------------
    def render_a(self, cam, spheres, prng_state=None):
        W, H = cam.image_width, cam.image_height
        out = np.zeros((H, W, 3))
        rays = C.c_uint64()
        st = (C.c_uint64 * 4)(*prng_state) if prng_state is not None else None
        self.L.oracle_render_a(C.byref(cam), spheres, len(spheres), st,
                               out.ctypes.data_as(dp), C.byref(rays))
        return out, rays.value

    def render_b(self, cam, spheres, row0=0, row_step=1, n_rows=None, threads=1):
        W, H = cam.image_width, cam.image_height
        if n_rows is None:
            n_rows = (H - row0 + row_step - 1) // row_step
        out = np.zeros((n_rows, W, 3))
        rays = C.c_uint64()
        self.L.oracle_render_b(C.byref(cam), spheres, len(spheres), row0, row_step, n_rows,
                               out.ctypes.data_as(dp), C.byref(rays), threads)
        return out, rays.value

    def to_rgb8(self, lin):
        lin = np.ascontiguousarray(lin, np.float64)
        rgb = np.zeros(lin.shape, np.uint8)
        self.L.oracle_to_rgb8(lin.ctypes.data_as(dp), lin.size // 3, rgb.ctypes.data_as(P(C.c_uint8)))
        return rgb

    def ppm_p6(self, rgb, w, h):
        rgb = np.ascontiguousarray(rgb, np.uint8)
        size = self.L.oracle_ppm_p6(rgb.ctypes.data_as(P(C.c_uint8)), w, h, None, 0)
        buf = (C.c_uint8 * size)()
        self.L.oracle_ppm_p6(rgb.ctypes.data_as(P(C.c_uint8)), w, h, buf, size)
        return bytes(buf)

    def render_book(self, chapter, width=400, ratio=16.0 / 9.0):
        """BASELINE config 1 (book chapter 4/5 renderer): (H, W, 3) uint8."""
        h = max(1, int(width / ratio))
        rgb = np.zeros((h, width, 3), np.uint8)
        hh = C.c_uint32()
        self.L.oracle_render_book(chapter, width, ratio, rgb.ctypes.data_as(P(C.c_uint8)), C.byref(hh))
        assert hh.value == h
        return rgb

    # ---- KAT helpers ----------------------------------------------------------------------------
    def sample_key(self, seed, pixel, sample):
        return self.L.oracle_sample_key(seed, pixel, sample)

    def sphere_hit(self, sphere, orig, direction, t_min, t_max):
        o = (C.c_double * 3)(*orig)
        d = (C.c_double * 3)(*direction)
        t = C.c_double()
        pt = (C.c_double * 3)()
        nrm = (C.c_double * 3)()
        fr = C.c_int()
        hit = self.L.oracle_sphere_hit(C.byref(sphere), o, d, t_min, t_max, C.byref(t), pt, nrm, C.byref(fr))
        if not hit:
            return None
        return dict(t=t.value, point=list(pt), normal=list(nrm), front=bool(fr.value))

    def world_hit(self, spheres, orig, direction, t_min, t_max):
        o = (C.c_double * 3)(*orig)
        d = (C.c_double * 3)(*direction)
        t = C.c_double()
        k = self.L.oracle_world_hit(spheres, len(spheres), o, d, t_min, t_max, C.byref(t))
        return k, t.value

    def random_doubles(self, seed, n):
        out = np.zeros(n)
        self.L.oracle_random_doubles(seed, n, out.ctypes.data_as(dp))
        return out

    def random_u64(self, seed, n):
        out = np.zeros(n, np.uint64)
        self.L.oracle_random_u64(seed, n, out.ctypes.data_as(P(C.c_uint64)))
        return out

    def reflect(self, v, n):
        out = (C.c_double * 3)()
        self.L.oracle_reflect((C.c_double * 3)(*v), (C.c_double * 3)(*n), out)
        return list(out)

    def refract(self, v, n, eta):
        out = (C.c_double * 3)()
        self.L.oracle_refract((C.c_double * 3)(*v), (C.c_double * 3)(*n), eta, out)
        return list(out)


def read_ppm(data):
    """Parse a P6 byte string -> (W, H, (H, W, 3) uint8)."""
    parts = data.split(b"\n", 3)
    assert parts[0] == b"P6" and parts[2] == b"255"
    w, h = map(int, parts[1].split())
    body = parts[3]
    rgb = np.frombuffer(body[: w * h * 3], np.uint8).reshape(h, w, 3)
    return w, h, rgb

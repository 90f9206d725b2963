"""Host-side logic of the product (C++ mirror of Scene / CameraBuilder / Color / PPM behind the C
ABI) against the pinned oracle.  CPU only: no compute calls on a GPU."""
import math
import os

import numpy as np
import pytest

import rtzig
from rtzig.abi import D3, RT_LAMBERTIAN, RtCameraParams
from test_oracle import golden_params

INF = math.inf


def _bytes(arr):
    return bytes(memoryview(arr).cast("B"))


@pytest.mark.parametrize("seed", [0xDEADBEEF, 0xABADCAFE, 0, 1, 2**64 - 1])
def test_scene_final_matches_oracle(oracle, seed):
    mine = rtzig.Scene.init(seed).generateWorld()
    ref, state = oracle.scene_final(seed)
    assert len(mine.world) == len(ref)
    assert _bytes(mine.world) == _bytes(ref)  # bit-identical sphere list (Scene.zig:48-134)
    assert mine.prng_state == state           # same Xoshiro state handed to render()


def test_scene_chapter13_matches_oracle(oracle):
    mine = rtzig.Scene.init(7).generateChapter13()
    assert _bytes(mine.world) == _bytes(oracle.scene_chapter13())


@pytest.mark.parametrize("width,aspect,vfov,angle,focus,spp", [
    (400, 16 / 9, 20, 0.6, 10, 10),
    (1200, 1.5, 20, 0.6, 10, 500),
    (3840, 16 / 9, 20, 0.6, 10, 10000),
    (1200, 16 / 9, 20, 10.0, 3.4, 500),
    (400, 16 / 9, 90, 0.0, 1.0, 100),
    (1, 2.0, 45, 0.0, 1.0, 1),
])
def test_camera_build_matches_oracle(oracle, width, aspect, vfov, angle, focus, spp):
    p = RtCameraParams(image_width=width, samples_per_pixel=spp, bounce_max=50, aspect_ratio=aspect,
                       look_from=D3(13, 2, 3), look_at=D3(0, 0, 0), v_up=D3(0, 1, 0), vfov=vfov,
                       defocus_angle=angle, focus_dist=focus, t_min=1e-3, t_max=INF, seed=99)
    cam = rtzig.RtCamera()
    import ctypes as C
    rtzig.lib.check("rt_camera_build", rtzig.load().rt_camera_build(C.byref(p), C.byref(cam)))
    ref = oracle.camera_build(p)
    assert _bytes(cam) == _bytes(ref)


def test_builder_fluent_matches_main_preset(oracle):
    cam = rtzig.final_scene_camera(width=400, aspect_ratio=16 / 9, spp=10)
    ref = oracle.camera_build(golden_params())
    assert _bytes(cam.cam) == _bytes(ref)
    assert (cam.width, cam.height) == (400, 225)


def test_image_height_rules():
    """camera.zig:33-40 Image.init: H = trunc(W / ratio), at least 1; camera.zig:348-371."""
    cam = rtzig.Camera.builder(1, 2.0).setViewport((0, 0, 0), (0, 0, -1), 90).build()
    assert (cam.width, cam.height) == (1, 1)
    cam = rtzig.Camera.builder(400, 1.0).setViewport((0, 0, 0), (0, 0, -1), 90).build()
    assert cam.height == 400
    cam = rtzig.Camera.builder(1200, 1.5).setViewport((0, 0, 0), (0, 0, -1), 90).build()
    assert cam.height == 800


def test_to_rgb8_matches_oracle(oracle):
    rng = np.random.default_rng(5)
    lin = np.concatenate([rng.uniform(-0.5, 1.5, (1000, 3)),
                          np.array([[0, 0.5, 0.75], [0.998001, 0.998, 1.0], [np.nan, -0.0, np.inf]])])
    assert np.array_equal(rtzig.to_rgb8(lin), oracle.to_rgb8(lin))
    assert rtzig.to_rgb8(np.array([[0, 0.5, 0.75]])).tolist() == [[0, 181, 221]]


def test_ppm_encode(oracle, golden_dir):
    assert rtzig.encode_p6(np.zeros((1, 1, 3), np.uint8), 1, 1) == \
        open(os.path.join(golden_dir, "test-binary.ppm"), "rb").read()
    rgb = np.arange(4 * 3 * 3, dtype=np.uint8).reshape(3, 4, 3)
    assert rtzig.encode_p6(rgb, 4, 3) == oracle.ppm_p6(rgb, 4, 3)


def test_ppm_save(tmp_path, golden_dir):
    """ppm.zig:92-105 via the C++ writer (file path)."""
    ppm = rtzig.PPM(1, 1, np.zeros((1, 1, 3)))
    path = str(tmp_path / "test-binary.ppm")
    ppm.saveBinary(path)
    assert open(path, "rb").read() == open(os.path.join(golden_dir, "test-binary.ppm"), "rb").read()
    with pytest.raises(rtzig.RtError):
        ppm.saveBinary(str(tmp_path / "no-such-dir" / "x.ppm"))


def test_sample_key_matches_oracle(oracle):
    for seed in (0, 0xDEADBEEF, 2**64 - 1):
        for pixel, s in ((0, 0), (1, 0), (0, 1), (959999, 499), (2**32 - 1, 2**32 - 1)):
            assert rtzig.sample_key(seed, pixel, s) == oracle.sample_key(seed, pixel, s)


def test_scene_add_clamps_radius():
    """Sphere.init clamps the radius to >= 0 (sphere.zig:21)."""
    s = rtzig.Scene.init(1).add((0, 0, 0), -3.0, RT_LAMBERTIAN)
    assert s.world[0].radius == 0.0


def test_ppm_p3_one_pixel_kat():
    """ppm.zig:73-90: a 1x1 black image saved as P3."""
    assert rtzig.encode_p3(np.zeros((1, 1, 3), np.uint8), 1, 1) == b"P3\n1 1\n255\n0 0 0\n"


def test_ppm_p3_matches_reference_chapter2(golden_dir):
    """The P3 writer reproduces the reference's images/chapter2.ppm byte-for-byte from the book's
    chapter-2 gradient (r = trunc(255.999 i/(W-1)), g = trunc(255.999 j/(H-1)), b = 0)."""
    W = H = 256
    i = np.arange(W, dtype=np.float64)[None, :].repeat(H, 0)
    j = np.arange(H, dtype=np.float64)[:, None].repeat(W, 1)
    rgb = np.stack([(255.999 * (i / (W - 1))).astype(np.uint8), (255.999 * (j / (H - 1))).astype(np.uint8),
                    np.zeros((H, W), np.uint8)], axis=-1)
    ref = open(os.path.join(golden_dir, "chapter2.ppm"), "rb").read()
    assert rtzig.encode_p3(rgb, W, H) == ref


def test_ppm_p3_save_and_consistency_with_p6(tmp_path):
    """PPM.save writes the P3 stream; its numbers are exactly the P6 payload (same toRgb)."""
    rng = np.random.default_rng(3)
    lin = rng.random((7, 5, 3)) * 1.3 - 0.1
    ppm = rtzig.PPM(5, 7, lin)
    path = str(tmp_path / "a.ppm")
    ppm.save(path)
    data = open(path, "rb").read()
    assert data == ppm.encode()
    head, body = data.split(b"\n", 3)[:3], data.split(b"\n", 3)[3]
    assert head == [b"P3", b"5 7", b"255"]
    nums = np.array([int(x) for x in body.split()], np.uint8)
    p6 = ppm.encodeBinary()
    assert np.array_equal(nums, np.frombuffer(p6[len(b"P6\n5 7\n255\n"):-1], np.uint8))
    # 0..255 round trip, including 1-, 2- and 3-digit values
    allv = np.arange(256, dtype=np.uint8).repeat(3).reshape(16, 16, 3)
    txt = rtzig.encode_p3(allv, 16, 16)
    assert [int(x) for x in txt.split()[4:]] == list(allv.reshape(-1))

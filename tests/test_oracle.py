"""Pins the CPU oracle against the reference's own fixtures and known-answer tests.

The only end-to-end golden in the reference is test "main" (src/main.zig:41-55): final scene,
seed 0xdeadbeef, width 400, 16/9, 10 spp, byte-exact vs test-files/chapter14.ppm.  The KATs below
restate the reference's unit tests (file:line cited per test).
"""
import math
import os

import numpy as np
import pytest

from rtzig.abi import D3, RT_DIELECTRIC, RT_LAMBERTIAN, RT_METAL, RtCameraParams, RtSphere
from oracle_lib import read_ppm

INF = math.inf


def golden_params(width=400, aspect=16.0 / 9.0, spp=10, seed=0xDEADBEEF):
    # main.zig:24-31 preset
    return RtCameraParams(image_width=width, samples_per_pixel=spp, bounce_max=50,
                          aspect_ratio=aspect, look_from=D3(13, 2, 3), look_at=D3(0, 0, 0),
                          v_up=D3(0, 1, 0), vfov=20, defocus_angle=0.6, focus_dist=10,
                          t_min=1e-3, t_max=INF, seed=seed)


def test_golden_chapter14_byte_exact(oracle, golden_dir):
    """main.zig:41-55: render with the sequential stream == test-files/chapter14.ppm."""
    spheres, state = oracle.scene_final(0xDEADBEEF)
    assert len(spheres) == 485
    cam = oracle.camera_build(golden_params())
    assert (cam.image_width, cam.image_height) == (400, 225)
    lin, rays = oracle.render_a(cam, spheres, state)
    data = oracle.ppm_p6(oracle.to_rgb8(lin), 400, 225)
    gold = open(os.path.join(golden_dir, "chapter14.ppm"), "rb").read()
    assert len(data) == len(gold) == 270016
    assert data == gold
    assert rays == 2379984  # world.hit calls for this render (recorded by the pinned oracle)


def test_scene_counts(oracle):
    """Scene.zig:189-205: seed 0xabadcafe -> 1 + 3 + 22*22 - 3 objects."""
    spheres, _ = oracle.scene_final(0xABADCAFE)
    assert len(spheres) == 1 + 3 + 22 * 22 - 3
    spheres, _ = oracle.scene_final(0xDEADBEEF)
    kinds = np.array([s.material for s in spheres])
    assert len(spheres) == 485
    # 1 ground + 382 lambertian + 68 metal + 31 glass small spheres + 3 big
    assert (kinds == RT_LAMBERTIAN).sum() == 1 + 382 + 1
    assert (kinds == RT_METAL).sum() == 68 + 1
    assert (kinds == RT_DIELECTRIC).sum() == 31 + 1


def test_chapter13_scene(oracle):
    s = oracle.scene_chapter13()
    assert len(s) == 5
    assert list(s[3].center) == [-1, 0, -1] and s[3].radius == 0.4
    assert s[3].refraction_index == 1.0 / 1.5
    assert s[4].material == RT_METAL and s[4].fuzz == 1


def test_camera_kat(oracle):
    """camera.zig:516-535: 400 x 16/9, viewport((0,0,0),(0,0,-1),90), focus 10."""
    p = RtCameraParams(image_width=400, samples_per_pixel=100, bounce_max=50,
                       aspect_ratio=16.0 / 9.0, look_from=D3(0, 0, 0), look_at=D3(0, 0, -1),
                       v_up=D3(0, 1, 0), vfov=90, defocus_angle=0, focus_dist=10,
                       t_min=1e-3, t_max=INF, seed=1)
    cam = oracle.camera_build(p)
    assert cam.image_height == 225
    assert list(cam.du) == [8.888888888888888e-2, 0.0, 0.0]
    assert list(cam.dv) == [0.0, -8.888888888888888e-2, 0.0]
    assert list(cam.pixel0) == [-1.773333333333333e1, 9.955555555555554e0, -1e1]
    assert cam.pixel_samples_scale == 1 / 100
    assert list(cam.defocus_disk_u) == [0, 0, 0]


def test_color_kat(oracle):
    """color.zig:157-163 toRgb(0, 0.5, 0.75) = (0, 181, 221); color.zig:165-172 gamma."""
    rgb = oracle.to_rgb8(np.array([[0.0, 0.5, 0.75]]))
    assert rgb.tolist() == [[0, 181, 221]]
    rgb = oracle.to_rgb8(np.array([[1.0, 0.0, 1.0], [-1.0, 4.0, 1e9]]))
    assert rgb.tolist() == [[255, 0, 255], [0, 255, 255]]


def _sphere(center, radius, kind=RT_LAMBERTIAN, albedo=(1, 1, 1), fuzz=0.0, ior=1.0):
    return RtSphere(center=D3(*center), radius=radius, material=kind, albedo=D3(*albedo),
                    fuzz=fuzz, refraction_index=ior)


def test_sphere_hit_kat(oracle):
    """sphere.zig:76-98 hit() success; :100-117 out of range; :119-136 no hit."""
    s = _sphere((0, 0, -2), 1.0)
    rec = oracle.sphere_hit(s, (0, 0, 0), (0, 0, -1), 0.0, 3.0)
    assert rec is not None
    assert rec["t"] == 1 and rec["point"] == [0, 0, -1] and rec["normal"] == [0, 0, 1] and rec["front"]
    assert oracle.sphere_hit(s, (0, 0, 0), (0, 0, -1), 0.0, 0.0) is None
    assert oracle.sphere_hit(s, (0, 0, 0), (0, 0, 1), 0.0, 3.0) is None


def test_hittable_list_kat(oracle):
    """hittable.zig:185-209: 4 spheres on -z, interval (-6, 6) -> first sphere, t = 1."""
    arr = (RtSphere * 4)(*[_sphere((0, 0, -z), 1.0) for z in (2, 3, 4, 5)])
    k, t = oracle.world_hit(arr, (0, 0, 0), (0, 0, -1), -6, 6)
    assert k == 0 and t == 1
    # ties: a later sphere at exactly the same t never replaces the earlier one (strict <)
    arr = (RtSphere * 2)(_sphere((0, 0, -2), 1.0), _sphere((0, 0, -2), 1.0))
    k, t = oracle.world_hit(arr, (0, 0, 0), (0, 0, -1), 1e-3, INF)
    assert k == 0 and t == 1


def test_vec_kat(oracle):
    """material.zig:196-220 (metal fuzz 0 == reflect), :222-246 (dielectric refract eta 1/1.5)."""
    assert oracle.reflect((0, 0, -1), (0, 0, 1)) == [0, 0, 1]
    r = oracle.refract((0, 0, -1), (0, 0, 1), 1.0 / 1.5)
    assert r == [0, 0, -1]
    r = oracle.reflect((1, -1, 0), (0, 1, 0))
    assert r == [1, 1, 0]


def test_ppm_binary_fixture(oracle, golden_dir):
    """ppm.zig:92-105: 1x1 black P6 == test-files/test-binary.ppm."""
    data = oracle.ppm_p6(np.zeros((1, 1, 3), np.uint8), 1, 1)
    assert data == open(os.path.join(golden_dir, "test-binary.ppm"), "rb").read()
    assert data == b"P6\n1 1\n255\n\x00\x00\x00\n"


def test_rng_self_consistency(oracle):
    """util.zig:33-86: same seed -> same draws; draws in [0, 1)."""
    a = oracle.random_doubles(0xCAFEF00D, 1000)
    b = oracle.random_doubles(0xCAFEF00D, 1000)
    assert np.array_equal(a, b)
    assert a[0] != a[1]
    assert (a >= 0).all() and (a < 1).all()
    # Xoshiro256++ from SplitMix64(0): first word is a fixed published-algorithm value
    w = oracle.random_u64(0, 2)
    assert int(w[0]) == 0x53175D61490B23DF


def test_sample_key_bijective(oracle):
    keys = {oracle.sample_key(0xDEADBEEF, p, s) for p in range(64) for s in range(64)}
    assert len(keys) == 64 * 64


def test_oracle_b_statistically_matches_golden(oracle, golden_dir):
    """Parity ladder step 3: the per-sample-stream render (B) differs from the
    sequential-stream golden only by RNG noise.  Tolerance: |mean_B - mean_gold| <= 1.0 per channel
    (8-bit units); 8x8 box RMSE <= 2.0."""
    from oracle_lib import read_ppm
    spheres, _ = oracle.scene_final(0xDEADBEEF)
    cam = oracle.camera_build(golden_params())
    lin, _ = oracle.render_b(cam, spheres, threads=8)
    rgb = oracle.to_rgb8(lin).astype(np.float64)
    _, _, gold = read_ppm(open(os.path.join(golden_dir, "chapter14.ppm"), "rb").read())
    gold = gold.astype(np.float64)
    assert np.abs(rgb.mean(axis=(0, 1)) - gold.mean(axis=(0, 1))).max() <= 1.0
    box = lambda x: x[:224].reshape(28, 8, 50, 8, 3).mean(axis=(1, 3))
    assert np.sqrt(((box(rgb) - box(gold)) ** 2).mean()) <= 2.0


@pytest.mark.parametrize("chapter", [4, 5, 6])
def test_config1_book_chapter_byte_exact(oracle, golden_dir, chapter):
    """BASELINE config 1 (chapter5 single sphere, 400x225, 1 spp, CPU plumbing + PPM diff): the
    book renderer restated in the oracle + the P6 writer reproduce test-files/chapter{4,5}.ppm and
    the "normals" variant test-files/chapter6.ppm (sphere + ground, 0.5 * (normal + 1), walked by
    HittableList.hit / Sphere.hit on (0, inf))."""
    rgb = oracle.render_book(chapter)
    data = oracle.ppm_p6(rgb, 400, 225)
    assert data == open(os.path.join(golden_dir, f"chapter{chapter}.ppm"), "rb").read()
    import rtzig
    assert rtzig.encode_p6(rgb, 400, 225) == data  # the product's P6 writer too


def test_config1_normals_antialiased_statistical(oracle, golden_dir):
    """test-files/chapter7.ppm is the chapter-6 normals scene antialiased (jittered samples per
    pixel, Interval.clamp + 256 quantisation).  Its RNG stream is unknown, so it is compared
    statistically with the oracle's 100-spp render: per-channel mean |delta| <= 1.0 (8-bit units),
    mean absolute difference <= 0.6, 98% of pixels within 2 levels (the rest are silhouette pixels)."""
    rgb = oracle.render_book(7).astype(np.float64)
    _, _, gold = read_ppm(open(os.path.join(golden_dir, "chapter7.ppm"), "rb").read())
    gold = gold.astype(np.float64)
    assert np.abs(rgb.mean(axis=(0, 1)) - gold.mean(axis=(0, 1))).max() <= 1.0
    assert np.abs(rgb - gold).mean() <= 0.6
    assert (np.abs(rgb - gold).max(axis=2) <= 2).mean() >= 0.98


def _box_rmse(a, b):
    box = lambda x: x[:224].reshape(28, 8, 50, 8, 3).astype(np.float64).mean(axis=(1, 3))
    return float(np.sqrt(((box(a) - box(b)) ** 2).mean()))


@pytest.mark.parametrize("config", ["chapter9", "chapter13"])
def test_presets_statistically_match_reference_images(oracle, golden_dir, config):
    """Configs 2 and 3 have no byte-exact pin: the reference's images/chapter9.ppm and
    images/chapter13.ppm come from the book-chapter code at an unknown seed.  The presets
    (rtzig.chapter9_camera / chapter13_camera at 400x225, 100 spp) are pinned statistically with the
    SURVEY §8(c) ladder-3 rule: per-channel image-mean |delta| <= 1.0 and 8x8 box RMSE <= 1.5x the
    A-vs-B RMSE (oracle A's sequential stream vs oracle B's per-sample streams, same scene)."""
    import rtzig
    cam = rtzig.chapter9_camera(spp=100) if config == "chapter9" else rtzig.chapter13_camera(width=400, spp=100)
    a, _ = oracle.render_a(cam.cam, cam.scene.world)
    b, _ = oracle.render_b(cam.cam, cam.scene.world, threads=8)
    A, B = oracle.to_rgb8(a), oracle.to_rgb8(b)
    _, _, gold = read_ppm(open(os.path.join(golden_dir, f"{config}.ppm"), "rb").read())
    floor = _box_rmse(A, B)
    assert np.abs(B.astype(np.float64).mean(axis=(0, 1)) - gold.astype(np.float64).mean(axis=(0, 1))).max() <= 1.0
    assert _box_rmse(B, gold) <= 1.5 * floor, (_box_rmse(B, gold), floor)

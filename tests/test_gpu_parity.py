"""GPU parity: the HIP kernel (through the C ABI) against oracle B, bit-for-bit.

Oracle B = the reference arithmetic restated in C with the per-(pixel, sample) RNG layout the GPU
uses; oracle A (pinned byte-exact to the reference golden) differs from B only in the RNG stream,
so GPU-vs-golden is checked statistically.  Bar: f64 linear pixels identical bit-for-bit
(np.array_equal), RGB8 identical byte-for-byte.
"""
import ctypes as C
import math
import os

import numpy as np
import pytest

import rtzig
from rtzig.abi import D3, RT_DIELECTRIC, RT_LAMBERTIAN, RT_METAL, RtSphere
from test_oracle import golden_params

pytestmark = pytest.mark.gpu
INF = math.inf


def gpu_render(cam, spheres, **kw):
    stats = {}
    out = rtzig.render(cam.cam if hasattr(cam, "cam") else cam, spheres, stats=stats, **kw)
    return out, stats


def test_chapter9_full_image_bit_exact(oracle):
    """Config 2 scene (two Lambertian spheres) at 400x225, reduced spp: every pixel bit-exact."""
    cam = rtzig.chapter9_camera(spp=8)
    out, st = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, threads=8)
    assert np.array_equal(out, ref)
    assert st["rays"] == rays and st["samples"] == 400 * 225 * 8


def test_final_scene_golden_config_bit_exact(oracle):
    """The golden test's configuration (main.zig:41-55: 400x225, 10 spp, seed 0xdeadbeef, 485
    spheres, defocus): GPU == oracle B on every pixel."""
    cam = rtzig.final_scene_camera(width=400, aspect_ratio=16 / 9, spp=10)
    out, st = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, threads=8)
    assert np.array_equal(out, ref)
    assert st["rays"] == rays


def _box_rmse(a, b):
    box = lambda x: x[:224].reshape(28, 8, 50, 8, 3).astype(np.float64).mean(axis=(1, 3))
    return float(np.sqrt(((box(a) - box(b)) ** 2).mean()))


def _check_vs_chapter14(oracle, rgb, golden_dir):
    """SURVEY §8(c) ladder 3: GPU (per-sample streams) vs the reference's own chapter14.ppm
    (sequential stream), calibrated like configs 2/3: per-channel image-mean |delta| <= 1.0 (8-bit
    units) and 8x8 box RMSE <= 1.5x the A-vs-B RMSE.  Oracle A reproduces chapter14.ppm byte for
    byte (test_oracle.py), so the A side of the floor is the fixture itself; the B side is oracle B
    on the oracle's own scene and camera (golden_params)."""
    from oracle_lib import read_ppm
    _, _, gold = read_ppm(open(os.path.join(golden_dir, "chapter14.ppm"), "rb").read())
    spheres, _ = oracle.scene_final(0xDEADBEEF)
    b, _ = oracle.render_b(oracle.camera_build(golden_params()), spheres, threads=16)
    floor = _box_rmse(gold, oracle.to_rgb8(b))
    assert np.abs(rgb.astype(np.float64).mean(axis=(0, 1)) - gold.astype(np.float64).mean(axis=(0, 1))).max() <= 1.0
    assert _box_rmse(rgb, gold) <= 1.5 * floor, (_box_rmse(rgb, gold), floor)


def test_final_scene_statistically_matches_reference_golden(oracle, golden_dir):
    """The bench scene at the golden test's configuration (main.zig:41-55) vs chapter14.ppm, with
    the calibrated A-vs-B rule of _check_vs_chapter14."""
    cam = rtzig.final_scene_camera(width=400, aspect_ratio=16 / 9, spp=10)
    rgb, _ = gpu_render(cam, cam.scene.world, n_gpus=1, output="rgb8")
    _check_vs_chapter14(oracle, rgb, golden_dir)


def test_chapter13_crop_bit_exact(oracle):
    """Config 3 scene (three materials, bubble, fuzz-1 metal, defocus 10) on a row subset."""
    cam = rtzig.chapter13_camera(width=1200, spp=16)
    out, _ = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, _ = oracle.render_b(cam.cam, cam.scene.world, row0=300, row_step=37, n_rows=10, threads=8)
    assert np.array_equal(out[300:300 + 37 * 10:37], ref)


def test_final_1200x800_rows_bit_exact(oracle):
    """Config 4 geometry (1200x800, aspect 1.5) at reduced spp on interleaved rows."""
    cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=4)
    out, _ = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, _ = oracle.render_b(cam.cam, cam.scene.world, row0=5, row_step=97, n_rows=8, threads=8)
    assert np.array_equal(out[5:5 + 97 * 8:97], ref)


def test_rgb8_output_matches_to_rgb(oracle):
    """Fused Color.toRgb epilogue (color.zig:63-80) == oracle B's image through the oracle's toRgb."""
    cam = rtzig.final_scene_camera(width=400, aspect_ratio=16 / 9, spp=3)
    rgb, _ = gpu_render(cam, cam.scene.world, n_gpus=1, output="rgb8")
    ref, _ = oracle.render_b(cam.cam, cam.scene.world, threads=16)
    assert np.array_equal(rgb, oracle.to_rgb8(ref))


def test_row_partition_invariance():
    """Rows rendered in any interleaved partition are bit-identical to the full render."""
    import torch
    cam = rtzig.final_scene_camera(width=320, aspect_ratio=16 / 9, spp=4)
    full, _ = gpu_render(cam, cam.scene.world, n_gpus=1)
    H, W = cam.height, cam.width
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    for G in (2, 3, 8):
        for g in range(G):
            n_rows = (H - g + G - 1) // G
            buf = torch.empty((n_rows, W, 3), dtype=torch.float64, device="cuda:0")
            r.render_rows_async(cam.cam, buf.data_ptr(), row0=g, row_step=G, n_rows=n_rows,
                                stream_ptr=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            assert np.array_equal(buf.cpu().numpy(), full[g::G])
    r.close()


def test_deterministic_and_finite_at_config4_size():
    """Size-independent properties at the bench's config size (1200x800) with reduced spp:
    repeat renders identical, all values finite and in [0, 1]."""
    cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=8)
    a, sa = gpu_render(cam, cam.scene.world, n_gpus=1)
    b, sb = gpu_render(cam, cam.scene.world, n_gpus=1)
    assert np.array_equal(a, b) and sa == sb
    assert np.isfinite(a).all() and a.min() >= 0 and a.max() <= 1.0
    assert sa["samples"] == 1200 * 800 * 8
    assert 1.5 < sa["rays"] / sa["samples"] < 5


@pytest.mark.parametrize("bounce_max", [0, 1, 2, 50])
def test_bounce_max_edges(oracle, bounce_max):
    """rayColor's loop bound (camera.zig:153,181): 0 bounces -> black, 1 -> only sky survives."""
    cam = rtzig.final_scene_camera(width=64, aspect_ratio=16 / 9, spp=4, bounce_max=bounce_max)
    out, st = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, threads=8)
    assert np.array_equal(out, ref)
    assert st["rays"] == rays
    if bounce_max == 0:
        assert not out.any() and rays == 0


def test_single_pixel_image(oracle):
    cam = rtzig.Camera.builder(1, 2.0).setScene(rtzig.Scene.init(3).generateWorld()) \
        .setViewport((13, 2, 3), (0, 0, 0), 20).setSamplesPerPixel(7).build()
    out, _ = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, _ = oracle.render_b(cam.cam, cam.scene.world)
    assert out.shape == (1, 1, 3) and np.array_equal(out, ref)


def test_materials_and_degenerate_spheres(oracle):
    """Every material branch incl. inside-glass (front=False), fuzz>1 metal absorption, a
    zero-radius sphere (clamped negative radius, sphere.zig:21) and coincident spheres (tie)."""
    scene = rtzig.Scene.init(0x1234)
    scene.add((0, -100.5, -1), 100, RT_LAMBERTIAN, albedo=(0.8, 0.8, 0.0))
    scene.add((0, 0, -1.2), 0.5, RT_METAL, albedo=(0.9, 0.9, 0.9), fuzz=1.7)
    scene.add((-1, 0, -1), 0.5, RT_DIELECTRIC, refraction_index=1.5)
    scene.add((-1, 0, -1), 0.4, RT_DIELECTRIC, refraction_index=1.0 / 1.5)
    scene.add((1, 0, -1), 0.5, RT_METAL, albedo=(0.8, 0.6, 0.2), fuzz=0.0)
    scene.add((1, 0, -1), 0.5, RT_LAMBERTIAN, albedo=(0.1, 0.1, 0.9))  # exact duplicate: never wins
    scene.add((0, 1, -1), -0.3, RT_LAMBERTIAN)                          # radius clamps to 0
    cam = (rtzig.Camera.builder(160, 16 / 9).setScene(scene).setDefocusAngle(2.0).setFocusDist(1.5)
           .setViewport((0, 0.3, 0.5), (0, 0, -1), 70).setSamplesPerPixel(16).build())
    out, st = gpu_render(cam, scene.world, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, scene.world, threads=8)
    assert np.array_equal(out, ref) and st["rays"] == rays


def test_large_scene_global_memory_variant(oracle):
    """More spheres than the LDS capacity (2048) -> the global-memory kernel variant."""
    rng = np.random.default_rng(11)
    n = 2600
    arr = (RtSphere * n)()
    arr[0] = RtSphere(center=D3(0, -1000, 0), radius=1000, material=RT_LAMBERTIAN, albedo=D3(0.5, 0.5, 0.5))
    for k in range(1, n):
        arr[k] = RtSphere(center=D3(*rng.uniform([-30, 0.1, -30], [30, 3, 30])),
                          radius=float(rng.uniform(0.05, 0.3)), material=int(k % 3),
                          albedo=D3(*rng.uniform(0, 1, 3)), fuzz=float(rng.uniform(0, 0.5)),
                          refraction_index=1.5)
    scene = rtzig.Scene.init(77)
    scene.world = arr
    cam = (rtzig.Camera.builder(96, 16 / 9).setScene(scene).setDefocusAngle(0.6).setFocusDist(10)
           .setViewport((13, 2, 3), (0, 0, 0), 20).setSamplesPerPixel(2).build())
    out, st = gpu_render(cam, arr, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, arr, threads=8)
    assert np.array_equal(out, ref) and st["rays"] == rays


@pytest.mark.parametrize("device_map", ["0,0", "0,0,0", "0,0,0,0,0,0,0,0", None])
def test_multi_gpu_call_equals_single(oracle, device_map, monkeypatch):
    """rt_render over several devices (n_gpus=0: all of them) == oracle B, bit for bit: its multi-
    device branch (contexts created on host threads, one stream each, row j on device j mod G,
    host un-interleave, stats summed) with G = 2, 3 and 8 logical devices mapped onto GPU 0
    (RTZIG_DEVICE_MAP, rt_runtime.cpp), and over the real devices when there are several.  f64 with
    the Zig shim's stride 4, and the fused RGB8 output."""
    import torch
    if device_map is None:
        if torch.cuda.device_count() < 2:
            pytest.skip("one visible GPU: the mapped cases cover the multi-device branch")
        monkeypatch.delenv("RTZIG_DEVICE_MAP", raising=False)
        G = torch.cuda.device_count()
    else:
        monkeypatch.setenv("RTZIG_DEVICE_MAP", device_map)
        G = len(device_map.split(","))
    lib = rtzig.load()
    cam = rtzig.final_scene_camera(width=200, aspect_ratio=16 / 9, spp=4)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, threads=16)
    out = np.full((cam.height, cam.width, 4), -7.0)
    st = (C.c_uint64 * 2)()
    opts = rtzig.RtOptions(n_gpus=0, pixel_stride=4, output_format=0, stats_out=C.cast(st, C.POINTER(C.c_uint64)))
    rc = lib.rt_render(C.byref(cam.cam), cam.scene.world, len(cam.scene.world), C.byref(opts),
                       out.ctypes.data_as(C.c_void_p))
    assert rc == 0, lib.rt_last_error()
    assert np.array_equal(out[..., :3], ref) and (out[..., 3] == -7.0).all()
    one, st1 = gpu_render(cam, cam.scene.world, n_gpus=1)
    assert (st[0], st[1]) == (rays, cam.width * cam.height * 4), (list(st), rays, st1)
    rgb, _ = gpu_render(cam, cam.scene.world, n_gpus=0, output="rgb8")
    assert np.array_equal(rgb, oracle.to_rgb8(ref))
    if device_map is not None:  # the logical device count is what the map says
        with pytest.raises(rtzig.lib.RtError):
            gpu_render(cam, cam.scene.world, n_gpus=G + 1)


def test_multi_device_ring_mode_bit_exact(oracle, monkeypatch):
    """The multi-device branch with every context in ring mode (in-kernel ordered accumulation and
    its cross-wave hand-off; three 1.2 GB workspaces on GPU 0)."""
    monkeypatch.setenv("RTZIG_DEVICE_MAP", "0,0,0")
    monkeypatch.setenv("RTZIG_UNIT_MODE", "ring")
    cam = rtzig.final_scene_camera(width=160, aspect_ratio=1.5, spp=60)
    out, st = gpu_render(cam, cam.scene.world, n_gpus=0)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, threads=16)
    assert np.array_equal(out, ref) and st["rays"] == rays
    rtzig.release_cached_contexts()


def test_pixel_stride_4_matches_zig_vector_layout(oracle):
    """Zig's @Vector(3, f64) is 32 bytes: the shim passes pixel_stride=4 (compared with oracle B)."""
    lib = rtzig.load()
    cam = rtzig.final_scene_camera(width=64, aspect_ratio=16 / 9, spp=2)
    ref, _ = oracle.render_b(cam.cam, cam.scene.world, threads=16)
    out = np.full((cam.height, cam.width, 4), -7.0)
    opts = rtzig.RtOptions(n_gpus=1, pixel_stride=4, output_format=0)
    rc = lib.rt_render(C.byref(cam.cam), cam.scene.world, len(cam.scene.world), C.byref(opts),
                       out.ctypes.data_as(C.c_void_p))
    assert rc == 0
    assert np.array_equal(out[..., :3], ref) and (out[..., 3] == -7.0).all()


def test_camera_render_api(tmp_path, golden_dir):
    """Camera.render() -> PPM.saveBinary() round trip through the mirror API."""
    cam = rtzig.final_scene_camera(width=400, aspect_ratio=16 / 9, spp=10)
    ppm = cam.render(n_gpus=1)
    path = str(tmp_path / "chapter14.ppm")
    ppm.saveBinary(path)
    data = open(path, "rb").read()
    assert len(data) == 270016 and data.startswith(b"P6\n400 225\n255\n") and data.endswith(b"\n")


@pytest.mark.parametrize("device_map", ["0,0,0", "0", None])
def test_c_harness_end_to_end(oracle, golden_dir, tmp_path, device_map):
    """The drop-in exactly as the Zig shim calls it (reference main.zig:41-55 ->
    camera.zig:123-145 -> saveBinary): tools/rt_render_c.c builds the golden configuration (400x225,
    10 spp, seed 0xdeadbeef, 485 spheres) through the ABI and calls rt_render with the shim's
    n_gpus = 0 — with RTZIG_DEVICE_MAP=0,0,0 that is the multi-device branch over three contexts.
    Its P6 file must equal oracle B's P6 byte for byte, and match the reference's chapter14.ppm
    under the calibrated statistical rule."""
    import subprocess
    from oracle_lib import read_ppm
    exe = os.path.join(os.path.dirname(rtzig.LIB_PATH), "rt_render_c")
    out = str(tmp_path / "chapter14.ppm")
    env = dict(os.environ)
    env.pop("RTZIG_DEVICE_MAP", None)
    if device_map is not None:
        env["RTZIG_DEVICE_MAP"] = device_map
    subprocess.run([exe, out, "400", "10", "0xdeadbeef"], check=True, capture_output=True, timeout=300, env=env)
    cam = rtzig.final_scene_camera(width=400, aspect_ratio=16 / 9, spp=10)
    ref, _ = oracle.render_b(cam.cam, cam.scene.world, threads=16)
    data = open(out, "rb").read()
    assert data == oracle.ppm_p6(oracle.to_rgb8(ref), 400, 225)
    _, _, rgb = read_ppm(data)
    _check_vs_chapter14(oracle, rgb, golden_dir)


def test_c_harness_phase_trace(tmp_path):
    """RTZIG_TRACE=1 (the one-shot cost breakdown of profiles/r05_dropin/): the harness's rt_render
    prints one JSON line of phases — HIP init first, the return last, the host scene/tree thread as a
    note — with one sample-kernel time per logical device, and its P6 file equals the untraced one."""
    import json
    import subprocess
    exe = os.path.join(os.path.dirname(rtzig.LIB_PATH), "rt_render_c")
    files = []
    for trace in ("0", "1"):
        out = str(tmp_path / f"t{trace}.ppm")
        env = dict(os.environ, RTZIG_DEVICE_MAP="0,0,0", RTZIG_TRACE=trace)
        p = subprocess.run([exe, out, "400", "10", "0xdeadbeef"], check=True, capture_output=True, text=True,
                           timeout=300, env=env)
        files.append(open(out, "rb").read())
        lines = [json.loads(ln) for ln in p.stderr.splitlines() if ln.startswith('{"rt_render_trace"')]
        if trace == "0":
            assert not lines
            continue
        assert len(lines) == 1, p.stderr[-2000:]
        t = lines[0]["rt_render_trace"]
        phases = list(t["phases_ms"])
        assert phases[0] == "hip_init_device_map" and phases[-1] == "return", phases
        assert "[host_scene_and_tree_thread]" in phases
        assert len(t["kernel_ms"]) == 3 and all(k > 0 for k in t["kernel_ms"])
        timed = sum(v for k, v in t["phases_ms"].items() if not k.startswith("["))
        assert abs(timed - t["total_ms"]) <= 0.01 * t["total_ms"] + 0.1
    assert files[0] == files[1]


@pytest.mark.parametrize("mode", ["ring", "direct"])
@pytest.mark.parametrize("variant", ["bvh", "smem_u4", "lds_u4"])
def test_walk_variants_bit_exact(oracle, variant, mode, monkeypatch):
    """Every closest-hit walk (BVH and the linear list walks) gives oracle B's bits in both unit
    modes (separate kernel instantiations): golden config + the degenerate-materials scene."""
    monkeypatch.setenv("RTZIG_KERNEL", variant)
    monkeypatch.setenv("RTZIG_UNIT_MODE", mode)
    cam = rtzig.final_scene_camera(width=200, aspect_ratio=16 / 9, spp=6)
    out, st = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, threads=8)
    assert np.array_equal(out, ref) and st["rays"] == rays
    cam = rtzig.chapter13_camera(width=160, spp=8)
    out, _ = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, _ = oracle.render_b(cam.cam, cam.scene.world, threads=8)
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("always_area", [None, "0", "1e-6"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_bvh_random_scenes_bit_exact(oracle, seed, always_area, monkeypatch):
    """BVH culling stress: random sphere soups (overlapping, duplicated, tiny and huge spheres,
    negative radii) from random camera positions; the BVH walk must return the linear scan's bits.
    always_area: the builder's huge-sphere rule at its default, off, and nearly always on (the 4
    largest spheres leave the tree for the always-list)."""
    monkeypatch.setenv("RTZIG_KERNEL", "bvh")
    if always_area is not None:
        monkeypatch.setenv("RTZIG_BVH_ALWAYS_AREA", always_area)
    rng = np.random.default_rng(seed)
    n = int(rng.integers(2, 300))
    arr = (RtSphere * (n + 2))()
    for k in range(n):
        arr[k] = RtSphere(center=D3(*rng.normal(0, 3, 3)), radius=float(rng.choice([rng.uniform(-0.1, 0.01),
                          rng.uniform(0.01, 0.5), rng.uniform(0.5, 3)])),
                          material=int(rng.integers(0, 3)), albedo=D3(*rng.uniform(0, 1, 3)),
                          fuzz=float(rng.uniform(0, 1.2)), refraction_index=float(rng.uniform(0.5, 2.5)))
    arr[n] = arr[0]                      # exact duplicate of sphere 0 (tie: index 0 must win)
    arr[n + 1] = RtSphere(center=D3(0, -1000.5, 0), radius=1000.0, material=0, albedo=D3(0.5, 0.5, 0.5))
    scene = rtzig.Scene.init(seed)
    scene.world = arr
    look_from = tuple(rng.normal(0, 8, 3))
    cam = (rtzig.Camera.builder(96, 1.5).setScene(scene).setDefocusAngle(float(rng.uniform(0, 3)))
           .setFocusDist(float(rng.uniform(1, 10))).setViewport(look_from, (0, 0, 0), float(rng.uniform(20, 90)))
           .setSamplesPerPixel(4).build())
    out, st = gpu_render(cam, arr, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, arr, threads=8)
    assert np.array_equal(out, ref) and st["rays"] == rays


@pytest.mark.parametrize("seed", [4, 23, 61])
def test_trained_tree_random_scenes_bit_exact(oracle, seed, monkeypatch):
    """Ray-driven trees (RTZIG_BVH_TRAIN=1 forces training on these small launches): the tree built
    from the camera's sample rays must return the linear scan's bits on random soups."""
    monkeypatch.setenv("RTZIG_KERNEL", "bvh")
    monkeypatch.setenv("RTZIG_BVH_TRAIN", "1")
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(40, 300))
    arr = (RtSphere * (n + 1))()
    for k in range(n):
        arr[k] = RtSphere(center=D3(*rng.normal(0, 3, 3)), radius=float(rng.choice([rng.uniform(-0.1, 0.01),
                          rng.uniform(0.01, 0.5), rng.uniform(0.5, 3)])),
                          material=int(rng.integers(0, 3)), albedo=D3(*rng.uniform(0, 1, 3)),
                          fuzz=float(rng.uniform(0, 1.2)), refraction_index=float(rng.uniform(0.5, 2.5)))
    arr[n] = RtSphere(center=D3(0, -1000.5, 0), radius=1000.0, material=0, albedo=D3(0.5, 0.5, 0.5))
    scene = rtzig.Scene.init(seed)
    scene.world = arr
    cam = (rtzig.Camera.builder(96, 1.5).setScene(scene).setDefocusAngle(float(rng.uniform(0, 3)))
           .setFocusDist(float(rng.uniform(1, 10))).setViewport(tuple(rng.normal(0, 8, 3)), (0, 0, 0),
                                                               float(rng.uniform(20, 90)))
           .setSamplesPerPixel(4).build())
    out, st = gpu_render(cam, arr, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, arr, threads=8)
    assert np.array_equal(out, ref) and st["rays"] == rays


@pytest.mark.parametrize("mode", ["ring", "direct"])
def test_trained_tree_final_scene_bit_exact(oracle, mode, monkeypatch):
    """The bench's scene and camera with the tree trained on its rays (what config 4 runs), on a
    reduced image: every pixel bit-exact, in both unit modes."""
    monkeypatch.setenv("RTZIG_BVH_TRAIN", "1")
    monkeypatch.setenv("RTZIG_UNIT_MODE", mode)
    cam = rtzig.final_scene_camera(width=240, aspect_ratio=1.5, spp=6)
    out, st = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, threads=8)
    assert np.array_equal(out, ref) and st["rays"] == rays


def test_bvh_far_camera_rebuild(oracle, monkeypatch):
    """A camera far outside the scene's extent raises the BVH padding's origin bound (rebuild)."""
    monkeypatch.setenv("RTZIG_KERNEL", "bvh")
    cam = (rtzig.Camera.builder(64, 1.5).setScene(rtzig.Scene.init(5).generateWorld()).setDefocusAngle(0.1)
           .setFocusDist(5000).setViewport((5000, 300, 4000), (0, 0, 0), 1.0).setSamplesPerPixel(3).build())
    out, _ = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, _ = oracle.render_b(cam.cam, cam.scene.world, threads=8)
    assert np.array_equal(out, ref)


def test_config5_crop_bit_exact(oracle):
    """Config 5 geometry (3840x2160, 16/9, final scene) on a crop of rows at reduced spp."""
    cam = rtzig.final_scene_camera(width=3840, aspect_ratio=16 / 9, spp=2)
    assert (cam.width, cam.height) == (3840, 2160)
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    import torch
    rows = [0, 700, 1333, 2159]
    for j in rows:
        buf = torch.empty((1, 3840, 3), dtype=torch.float64, device="cuda:0")
        r.render_rows_async(cam.cam, buf.data_ptr(), row0=j, row_step=1, n_rows=1)
        torch.cuda.synchronize()
        ref, _ = oracle.render_b(cam.cam, cam.scene.world, row0=j, row_step=1, n_rows=1, threads=8)
        assert np.array_equal(buf.cpu().numpy(), ref), j
    r.close()


def _soup(seed, scale):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(20, 120))
    arr = (RtSphere * (n + 1))()
    for k in range(n):
        arr[k] = RtSphere(center=D3(*(rng.normal(0, 3, 3) * scale)),
                          radius=float(rng.choice([rng.uniform(0.01, 0.5), rng.uniform(0.5, 3)]) * scale),
                          material=int(rng.integers(0, 3)), albedo=D3(*rng.uniform(0, 1, 3)),
                          fuzz=float(rng.uniform(0, 1.2)), refraction_index=float(rng.uniform(0.5, 2.5)))
    arr[n] = RtSphere(center=D3(0, -1000.5 * scale, 0), radius=1000.0 * scale, material=0, albedo=D3(0.5, 0.5, 0.5))
    scene = rtzig.Scene.init(seed)
    scene.world = arr
    look_from = tuple(rng.normal(0, 8, 3) * scale)
    cam = (rtzig.Camera.builder(64, 1.5).setScene(scene).setDefocusAngle(float(rng.uniform(0, 3)))
           .setFocusDist(float(rng.uniform(1, 10)) * scale).setViewport(look_from, (0, 0, 0), float(rng.uniform(20, 90)))
           .setSamplesPerPixel(3).build())
    return arr, cam


@pytest.mark.parametrize("scale", [1e-70, 1e-40, 1e40, 1e70])
def test_extreme_scales_bit_exact(oracle, scale):
    """The exact fast paths of the kernel (unscaled sqrt, shared-reciprocal divisions, the leaf
    filter, f32 BVH boxes) are guarded by range checks; at these scales the discriminants, |dir|^2
    and the coordinates leave the guarded ranges (and f32's range), so the lanes take the full
    correctly rounded sequences and the always-list.  Bits must still equal oracle B."""
    arr, cam = _soup(11, scale)
    out, st = gpu_render(cam, arr, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, arr, threads=8)
    assert np.array_equal(out, ref) and st["rays"] == rays


@pytest.mark.parametrize("t_min", [0.0, -0.5, 1e-9, 0.25])
def test_interval_min_variants_bit_exact(oracle, t_min):
    """Scene.interval.min other than 1e-3 (zero, negative, tiny, large): the leaf filter's margins
    and the root selection (sphere.zig:35-41) must follow the reference for any t_min."""
    arr, cam = _soup(12, 1.0)
    cam.cam.t_min = t_min
    out, st = gpu_render(cam, arr, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, arr, threads=8)
    assert np.array_equal(out, ref) and st["rays"] == rays


def test_kernel_times_total_accumulates():
    """rt_context_kernel_times_total sums the HIP-event times of every launch since timing was
    enabled (bench.py reads it once after its timed region); per-call times stay available."""
    import torch
    cam = rtzig.final_scene_camera(width=120, aspect_ratio=1.5, spp=4)
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    out = torch.zeros((cam.height, cam.width, 3), dtype=torch.float64, device="cuda:0")
    r.enable_timing(True)
    per = []
    for _ in range(3):
        r.render_rows_async(cam.cam, out.data_ptr())
        per.append(r.kernel_times())
    s, red, n = r.kernel_times_total()
    assert n == 3
    assert abs(s - sum(a for a, _ in per)) < 1e-3 and abs(red - sum(b for _, b in per)) < 1e-3
    r.enable_timing(True)  # re-enabling restarts the totals
    r.render_rows_async(cam.cam, out.data_ptr())
    assert r.kernel_times_total()[2] == 1
    r.close()


@pytest.mark.parametrize("mode", ["ring", "direct"])
@pytest.mark.parametrize("spp", [1, 2, 3, 15, 16, 17, 31, 33, 47, 48, 49, 95, 97, 100])
def test_unit_schedule_sample_counts_bit_exact(oracle, spp, mode, monkeypatch):
    """Every chunk schedule shape of the unit scheduler (rt_kernel.h "Work units": chunks of up to kUnitS = 48
    samples, shrinking towards the end, rt_schedule.hpp) on an image whose pixel count is not a
    multiple of 64 (a partial last tile), in both modes: the ring's in-kernel ordered accumulation
    and direct mode's stored samples + reduce pass must give oracle B's bits."""
    monkeypatch.setenv("RTZIG_UNIT_MODE", mode)
    cam = rtzig.final_scene_camera(width=37, aspect_ratio=16 / 9, spp=spp)
    out, st = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, threads=16)
    assert (37 * cam.height) % 64 != 0
    assert np.array_equal(out, ref) and st["rays"] == rays and st["samples"] == 37 * cam.height * spp
    rgb, _ = gpu_render(cam, cam.scene.world, n_gpus=1, output="rgb8")
    assert np.array_equal(rgb, oracle.to_rgb8(ref))


@pytest.mark.parametrize("width,spp", [(8, 300), (64, 120), (1, 700)])
def test_running_sum_handoff_chains(oracle, width, spp, monkeypatch):
    """One or a few tiles with many sample chunks: consecutive units of the SAME tile are claimed
    back to back by different waves, so nearly every finalisation waits on the previous chunk's
    hand-off (write-through sums + per-tile flag, rt_units.h).  Ring mode forced (such small
    launches run in direct mode by default)."""
    monkeypatch.setenv("RTZIG_UNIT_MODE", "ring")
    cam = (rtzig.Camera.builder(width, 1.0).setScene(rtzig.Scene.init(0x5eed).generateWorld())
           .setDefocusAngle(0.6).setFocusDist(10).setViewport((13, 2, 3), (0, 0, 0), 20)
           .setSamplesPerPixel(spp).build())
    out, st = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, threads=16)
    assert np.array_equal(out, ref) and st["rays"] == rays


@pytest.mark.parametrize("n_big,ground,n_unbound", [(0, False, 0), (0, True, 0), (1, True, 0), (2, True, 0),
                                                    (3, True, 0), (4, True, 0), (3, True, 2)])
def test_always_list_sizes_bit_exact(oracle, n_big, ground, n_unbound):
    """The always-list (rt_bvh.cpp: huge / big / unboundable spheres tested by every ray before the
    walk) at every size the kernel distinguishes: 0 to 4 spheres take the unrolled path whose
    geometry and original index come by scalar loads at immediate offsets from the kernarg
    pointers; more than 4 (unboundable spheres beside the capped big ones) take the runtime loop.
    A grid of small spheres with n_big radius-1.2 spheres among them (box area >= 10x the median:
    big), an optional radius-1000 ground (huge) and n_unbound spheres centred at 2e30 (never hit,
    but tested)."""
    rng = np.random.default_rng(100 + 10 * n_big + n_unbound + (5 if ground else 0))
    sph = []
    for a in range(-4, 4):
        for b in range(-4, 4):
            sph.append(RtSphere(center=D3(a + 0.9 * rng.uniform(), 0.2, b + 0.9 * rng.uniform()), radius=0.2,
                                material=int(rng.integers(0, 3)), albedo=D3(*rng.uniform(0, 1, 3)),
                                fuzz=float(rng.uniform(0, 0.5)), refraction_index=1.5))
    for k in range(n_big):
        sph.append(RtSphere(center=D3(-3.0 + 2.0 * k, 1.2, 0.3 * k), radius=1.2, material=k % 3,
                            albedo=D3(0.7, 0.6, 0.5), fuzz=0.0, refraction_index=1.5))
    if ground:
        sph.insert(int(rng.integers(0, len(sph))), RtSphere(center=D3(0, -1000, 0), radius=1000.0, material=0,
                                                            albedo=D3(0.5, 0.5, 0.5)))
    for k in range(n_unbound):
        sph.insert(int(rng.integers(0, len(sph))), RtSphere(center=D3(2e30, 1.0 + k, 0), radius=1.0, material=0,
                                                            albedo=D3(0.5, 0.5, 0.5)))
    arr = (RtSphere * len(sph))(*sph)
    scene = rtzig.Scene.init(7)
    scene.world = arr
    cam = (rtzig.Camera.builder(64, 1.5).setScene(scene).setDefocusAngle(0.6).setFocusDist(10.0)
           .setViewport((13, 2, 3), (0, 0, 0), 20.0).setSamplesPerPixel(4).build())
    out, st = gpu_render(cam, arr, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, arr, threads=8)
    assert np.array_equal(out, ref) and st["rays"] == rays


@pytest.mark.parametrize("scale", [None, "0.0", "0.05"])
def test_far_origin_lanes_walk_without_culling(oracle, monkeypatch, scale):
    """Rays whose origin lies beyond the BVH padding's origin bound (rt_bvh.cpp) must not be culled
    by the f32 boxes: the kernel forces their box tests to "hit" (BvhArgs::origin_bound).
    Natural case: an unboundable (|c| + r >= 1e30) radius-2e30 sphere on the always-list that rays
    hit, so secondary rays start ~1e30 away.  Forced case (RTZIG_BVH_ORIGIN_SCALE): the bound is
    shrunk so that camera and secondary rays that DO hit small spheres take the no-culling walk."""
    monkeypatch.setenv("RTZIG_KERNEL", "bvh")
    if scale is not None:
        monkeypatch.setenv("RTZIG_BVH_ORIGIN_SCALE", scale)
    scene = rtzig.Scene.init(0xfa7).generateWorld()
    huge = RtSphere(center=D3(0, -2e30, 0), radius=2e30, material=RT_METAL, albedo=D3(0.7, 0.7, 0.7), fuzz=0.3)
    arr = (RtSphere * (len(scene.world) + 1))(*scene.world, huge)
    scene.world = arr
    cam = (rtzig.Camera.builder(96, 1.5).setScene(scene).setDefocusAngle(0.6).setFocusDist(10)
           .setViewport((13, 2, 3), (0, 0, 0), 20).setSamplesPerPixel(4).build())
    out, st = gpu_render(cam, arr, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, arr, threads=16)
    assert np.array_equal(out, ref) and st["rays"] == rays


def test_render_cache_scene_switch(oracle):
    """rt_render's cached per-device context: alternating scenes re-upload (bit-exact each time), a
    repeated scene reuses the upload, and releasing the cache is harmless."""
    a = rtzig.final_scene_camera(width=64, aspect_ratio=16 / 9, spp=3)
    b = rtzig.chapter13_camera(width=64, spp=3)
    ra, _ = oracle.render_b(a.cam, a.scene.world, threads=16)
    rb, _ = oracle.render_b(b.cam, b.scene.world, threads=16)
    for cam, ref in ((a, ra), (b, rb), (b, rb), (a, ra)):
        out, _ = gpu_render(cam, cam.scene.world, n_gpus=1)
        assert np.array_equal(out, ref)
    rtzig.release_cached_contexts()
    out, _ = gpu_render(a, a.scene.world, n_gpus=1)
    assert np.array_equal(out, ra)


def test_device_renderer_alternating_streams_and_cameras(oracle):
    """One context used from two HIP streams with different cameras: each call waits for the
    previous call's work before reusing the context's buffers (rt.h), so both images are exact."""
    import torch
    cam1 = rtzig.final_scene_camera(width=200, aspect_ratio=16 / 9, spp=9)
    cam2 = (rtzig.Camera.builder(200, 16 / 9).setScene(cam1.scene).setDefocusAngle(0.0).setFocusDist(4)
            .setViewport((-6, 3, 8), (0, 0.5, 0), 35).setSamplesPerPixel(7).build())
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam1.scene.world)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    o1 = torch.zeros((cam1.height, 200, 3), dtype=torch.float64, device="cuda:0")
    o2 = torch.zeros((cam2.height, 200, 3), dtype=torch.float64, device="cuda:0")
    for _ in range(2):
        r.render_rows_async(cam1.cam, o1.data_ptr(), stream_ptr=s1.cuda_stream)
        r.render_rows_async(cam2.cam, o2.data_ptr(), stream_ptr=s2.cuda_stream)
    torch.cuda.synchronize()
    ref1, _ = oracle.render_b(cam1.cam, cam1.scene.world, threads=16)
    ref2, _ = oracle.render_b(cam2.cam, cam1.scene.world, threads=16)
    assert np.array_equal(o1.cpu().numpy(), ref1)
    assert np.array_equal(o2.cpu().numpy(), ref2)
    r.close()


def test_trained_tree_retrains_per_camera_across_streams(oracle, monkeypatch):
    """RTZIG_BVH_TRAIN=1: every camera switch rebuilds the tree from that camera's rays and
    re-uploads it while the previous render (on another stream) may still walk the old one; the
    context waits for it first (quiesce), so both cameras' images stay exact on every pass."""
    import torch
    monkeypatch.setenv("RTZIG_BVH_TRAIN", "1")
    cam1 = rtzig.final_scene_camera(width=160, aspect_ratio=16 / 9, spp=6)
    cam2 = (rtzig.Camera.builder(160, 16 / 9).setScene(cam1.scene).setDefocusAngle(0.3).setFocusDist(6)
            .setViewport((-5, 1.5, 9), (0, 0.3, 0), 30).setSamplesPerPixel(5).build())
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam1.scene.world)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    o1 = torch.zeros((cam1.height, 160, 3), dtype=torch.float64, device="cuda:0")
    o2 = torch.zeros((cam2.height, 160, 3), dtype=torch.float64, device="cuda:0")
    ref1, _ = oracle.render_b(cam1.cam, cam1.scene.world, threads=16)
    ref2, _ = oracle.render_b(cam2.cam, cam1.scene.world, threads=16)
    for _ in range(3):
        r.render_rows_async(cam1.cam, o1.data_ptr(), stream_ptr=s1.cuda_stream)
        r.render_rows_async(cam2.cam, o2.data_ptr(), stream_ptr=s2.cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(o1.cpu().numpy(), ref1)
        assert np.array_equal(o2.cpu().numpy(), ref2)
    r.sync()
    r.close()


@pytest.mark.parametrize("profile", [False, True])
def test_direct_rows_instrumented_bit_exact(oracle, profile, monkeypatch):
    """The launch shape of round 3's unexplained fault (profiles/r04_diag): direct-mode BVH rows of
    an 8-rank job, plain and with the instrumented kernel writing its 32-word stats.  Bit-exact
    against oracle B; exact sample and ray counts (reference: the row loop camera.zig:128-138 that a
    rank's launch replaces)."""
    import torch
    monkeypatch.setenv("RTZIG_UNIT_MODE", "direct")
    cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=24)
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    r.enable_profile(profile)
    out = torch.zeros((12, 1200, 3), dtype=torch.float64, device="cuda:0")
    stats = torch.zeros(rtzig.abi.RT_PROFILE_STATS_WORDS, dtype=torch.int64, device="cuda:0")
    r.render_rows_async(cam.cam, out.data_ptr(), row0=3, row_step=8, n_rows=12, d_stats_ptr=stats.data_ptr())
    r.sync()
    assert "direct" in r.kernel_name() and ("prof" in r.kernel_name()) == profile
    r.close()
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, row0=3, row_step=8, n_rows=12, threads=16)
    st = stats.cpu().tolist()
    assert np.array_equal(out.cpu().numpy(), ref)
    assert st[0] == rays and st[1] == 12 * 1200 * 24


@pytest.mark.parametrize("mode", ["direct", "ring"])
def test_split_render_pipeline_bit_exact(oracle, mode, monkeypatch):
    """rt_render_rows_async_split (bench.py's N > 1 frame pipeline): the sample kernel on one stream,
    the output completed on a second one (direct mode: the reduce pass there, over two per-sample
    buffers taken in turn).  Four frames back to back into two row buffers, each consumed on the
    second stream, interleaved with a plain call: every frame bit-exact against oracle B with exact
    sample counts, and direct mode holds two per-sample buffers (reference: the row loop
    camera.zig:128-138 that a rank's launch replaces)."""
    import torch
    monkeypatch.setenv("RTZIG_UNIT_MODE", mode)
    cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=24)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, row0=5, row_step=8, n_rows=12, threads=16)
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    render, coll = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.zeros((12, 1200, 3), dtype=torch.float64, device="cuda:0") for _ in range(2)]
    stats = torch.zeros(2, dtype=torch.int64, device="cuda:0")
    got = []
    for k in range(4):
        buf = outs[k % 2]
        r.render_rows_async(cam.cam, buf.data_ptr(), row0=5, row_step=8, n_rows=12, d_stats_ptr=stats.data_ptr(),
                            stream_ptr=render.cuda_stream, out_stream_ptr=coll.cuda_stream)
        with torch.cuda.stream(coll):
            got.append(buf.clone())  # ordered after this frame's output on the second stream
        render.wait_stream(coll)  # the next frame into this buffer only after the copy
        if k == 1:
            direct_ws = r.workspace_bytes()
    plain = torch.zeros_like(outs[0])
    r.render_rows_async(cam.cam, plain.data_ptr(), row0=5, row_step=8, n_rows=12, stream_ptr=render.cuda_stream)
    torch.cuda.synchronize()
    r.sync()
    assert ("direct" in r.kernel_name()) == (mode == "direct")
    per_buf = 24 * 1200 * 12 * 24  # spp x pixels x 24 B
    if mode == "direct":
        assert direct_ws >= 2 * per_buf
    r.close()
    for img in got + [plain]:
        assert np.array_equal(img.cpu().numpy(), ref)
    st = stats.cpu().tolist()
    assert st[1] == 4 * 12 * 1200 * 24 and st[0] == 4 * rays


@pytest.mark.parametrize("mode", ["direct", "ring"])
@pytest.mark.parametrize("profile", [False, True])
def test_deferred_render_pipeline_bit_exact(oracle, mode, profile, monkeypatch):
    """rt_render_rows_async_deferred: a direct-mode call's reduce pass is left pending and folded by
    the next deferred call's waves (one wave per block first, then the drained waves; the
    instrumented kernels do not fold, so a follow-up pass runs it after them: `profile`); the last
    one by rt_context_flush.  Five frames into two row buffers, each taken on the second stream once
    it is complete (after the next call, or after the flush), interleaved with a plain call that must
    run the pending pass first: every frame bit-exact against oracle B, exact sample counts (reference:
    the row loop camera.zig:128-138 that a rank's launch replaces)."""
    import torch
    monkeypatch.setenv("RTZIG_UNIT_MODE", mode)
    cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=24)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, row0=5, row_step=8, n_rows=12, threads=16)
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    r.enable_profile(profile)
    render, coll = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.zeros((12, 1200, 3), dtype=torch.float64, device="cuda:0") for _ in range(2)]
    stats = torch.zeros(rtzig.abi.RT_PROFILE_STATS_WORDS, dtype=torch.int64, device="cuda:0")
    got = []
    pending = False
    for k in range(5):
        render.wait_stream(coll)  # the copies below have read the buffer this call may write
        r.render_rows_async(cam.cam, outs[k % 2].data_ptr(), row0=5, row_step=8, n_rows=12,
                            d_stats_ptr=stats.data_ptr(), stream_ptr=render.cuda_stream,
                            out_stream_ptr=coll.cuda_stream, deferred=True)
        with torch.cuda.stream(coll):
            if pending:
                got.append(outs[(k - 1) % 2].clone())  # frame k-1, completed by this call
        pending = r.fold_pending()
        assert pending == (mode == "direct")
        if not pending:
            with torch.cuda.stream(coll):
                got.append(outs[k % 2].clone())
        if k == 2:
            # a plain call in between runs the pending pass whole first
            plain = torch.zeros_like(outs[0])
            r.render_rows_async(cam.cam, plain.data_ptr(), row0=5, row_step=8, n_rows=12, stream_ptr=render.cuda_stream)
            assert not r.fold_pending()
            with torch.cuda.stream(coll):
                if pending:
                    got.append(outs[k % 2].clone())
            pending = False
            torch.cuda.synchronize()
            assert np.array_equal(plain.cpu().numpy(), ref)
    r.flush()
    with torch.cuda.stream(coll):
        if pending:
            got.append(outs[4 % 2].clone())
    torch.cuda.synchronize()
    r.sync()
    r.close()
    assert len(got) == 5
    for img in got:
        assert np.array_equal(img.cpu().numpy(), ref)
    st = stats.cpu().tolist()
    assert st[1] == 5 * 12 * 1200 * 24 and st[0] == 5 * rays


def test_split_and_deferred_on_the_null_stream(oracle, monkeypatch):
    """The output stream may be the HIP null stream (torch's default stream, handle 0 — the
    collective stream of bench.py): split and deferred calls then complete the output there, ordered
    after the sample kernel on the render stream.  Direct-mode rows, three frames each way, every
    frame bit-exact against oracle B."""
    import torch
    monkeypatch.setenv("RTZIG_UNIT_MODE", "direct")
    cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=24)
    ref, _ = oracle.render_b(cam.cam, cam.scene.world, row0=2, row_step=8, n_rows=12, threads=16)
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    render, null = torch.cuda.Stream(), torch.cuda.default_stream()
    assert null.cuda_stream == 0
    outs = [torch.zeros((12, 1200, 3), dtype=torch.float64, device="cuda:0") for _ in range(3)]
    for k in range(3):  # split
        r.render_rows_async(cam.cam, outs[k].data_ptr(), row0=2, row_step=8, n_rows=12,
                            stream_ptr=render.cuda_stream, out_stream_ptr=0)
    null.synchronize()  # the null stream alone: its order must cover the outputs
    got = [o.clone() for o in outs]
    torch.cuda.synchronize()
    outs = [torch.zeros_like(outs[0]) for _ in range(3)]
    for k in range(3):  # deferred
        r.render_rows_async(cam.cam, outs[k].data_ptr(), row0=2, row_step=8, n_rows=12,
                            stream_ptr=render.cuda_stream, out_stream_ptr=0, deferred=True)
    r.flush()
    null.synchronize()
    got += [o.clone() for o in outs]
    torch.cuda.synchronize()
    r.sync()
    r.close()
    for img in got:
        assert np.array_equal(img.cpu().numpy(), ref)


def test_destroy_completes_pending_deferred_output(oracle, monkeypatch):
    """rt_context_destroy with a deferred call's reduce pass still pending runs the pass and waits
    for it before freeing the context: the output is complete and bit-exact against oracle B once
    destroy returns (the reference's render always fills ppm.pixels, camera.zig:125,138)."""
    import torch
    monkeypatch.setenv("RTZIG_UNIT_MODE", "direct")
    cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=24)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, row0=3, row_step=8, n_rows=12, threads=16)
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    render, coll = torch.cuda.Stream(), torch.cuda.Stream()
    out = torch.zeros((12, 1200, 3), dtype=torch.float64, device="cuda:0")
    stats = torch.zeros(2, dtype=torch.int64, device="cuda:0")
    r.render_rows_async(cam.cam, out.data_ptr(), row0=3, row_step=8, n_rows=12, d_stats_ptr=stats.data_ptr(),
                        stream_ptr=render.cuda_stream, out_stream_ptr=coll.cuda_stream, deferred=True)
    assert r.fold_pending()
    r.close()  # destroy: must flush, not drop
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), ref)
    assert stats.cpu().tolist() == [rays, 12 * 1200 * 24]


def test_deferred_alternating_out_streams(oracle, monkeypatch):
    """Consecutive deferred calls on DIFFERENT out streams: the pending pass of call k is promised on
    call k's out stream, so call k+1 (another out stream) must not fold it on its own stream — it runs
    the pass whole on call k's stream first.  Each frame is read on its own out stream right after the
    next call is issued (rt.h's contract), four frames, every one bit-exact against oracle B."""
    import torch
    monkeypatch.setenv("RTZIG_UNIT_MODE", "direct")
    cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=24)
    ref, _ = oracle.render_b(cam.cam, cam.scene.world, row0=6, row_step=8, n_rows=12, threads=16)
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    render = torch.cuda.Stream()
    outs_s = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.zeros((12, 1200, 3), dtype=torch.float64, device="cuda:0") for _ in range(2)]
    got = []
    for k in range(4):
        for s in outs_s:
            render.wait_stream(s)  # the clones below have read the buffer this call may write
        r.render_rows_async(cam.cam, outs[k % 2].data_ptr(), row0=6, row_step=8, n_rows=12,
                            stream_ptr=render.cuda_stream, out_stream_ptr=outs_s[k % 2].cuda_stream, deferred=True)
        if k:
            with torch.cuda.stream(outs_s[(k - 1) % 2]):
                got.append(outs[(k - 1) % 2].clone())  # frame k-1: complete on ITS out stream now
    r.flush()
    with torch.cuda.stream(outs_s[3 % 2]):
        got.append(outs[3 % 2].clone())
    for s in outs_s:
        s.synchronize()
    imgs = [g.cpu().numpy() for g in got]
    r.sync()
    r.close()
    assert len(imgs) == 4
    for img in imgs:
        assert np.array_equal(img, ref)

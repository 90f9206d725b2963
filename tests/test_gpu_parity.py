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


def test_final_scene_statistically_matches_reference_golden(golden_dir):
    """Parity ladder step 3: GPU (per-sample streams) vs the reference's own chapter14.ppm
    (sequential stream).  Tolerance per north_star: per-channel image mean |delta| <= 1.0 (8-bit
    units) and 8x8 box-filtered RMSE <= 2.0."""
    from oracle_lib import read_ppm
    cam = rtzig.final_scene_camera(width=400, aspect_ratio=16 / 9, spp=10)
    rgb, _ = gpu_render(cam, cam.scene.world, n_gpus=1, output="rgb8")
    _, _, gold = read_ppm(open(os.path.join(golden_dir, "chapter14.ppm"), "rb").read())
    a, b = rgb.astype(np.float64), gold.astype(np.float64)
    assert np.abs(a.mean(axis=(0, 1)) - b.mean(axis=(0, 1))).max() <= 1.0
    box = lambda x: x[:224].reshape(28, 8, 50, 8, 3).mean(axis=(1, 3))
    assert np.sqrt(((box(a) - box(b)) ** 2).mean()) <= 2.0


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
    """Fused Color.toRgb epilogue == host toRgb of the linear output (color.zig:63-80)."""
    cam = rtzig.final_scene_camera(width=400, aspect_ratio=16 / 9, spp=3)
    lin, _ = gpu_render(cam, cam.scene.world, n_gpus=1)
    rgb, _ = gpu_render(cam, cam.scene.world, n_gpus=1, output="rgb8")
    assert np.array_equal(rgb, oracle.to_rgb8(lin))


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


def test_multi_gpu_call_equals_single(oracle):
    """rt_render over every visible device == one device (row interleave + host un-interleave)."""
    cam = rtzig.final_scene_camera(width=200, aspect_ratio=16 / 9, spp=4)
    one, _ = gpu_render(cam, cam.scene.world, n_gpus=1)
    many, _ = gpu_render(cam, cam.scene.world, n_gpus=0)
    assert np.array_equal(one, many)


def test_pixel_stride_4_matches_zig_vector_layout():
    """Zig's @Vector(3, f64) is 32 bytes: the shim passes pixel_stride=4."""
    lib = rtzig.load()
    cam = rtzig.final_scene_camera(width=64, aspect_ratio=16 / 9, spp=2)
    ref, _ = gpu_render(cam, cam.scene.world, n_gpus=1)
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


def test_c_harness_end_to_end(tmp_path):
    """tools/rt_render_c.c drives the ABI exactly like the Zig shim: its P6 file
    equals the Python path's fused-RGB8 render of the same preset."""
    import subprocess
    exe = os.path.join(os.path.dirname(rtzig.LIB_PATH), "rt_render_c")
    out = str(tmp_path / "chapter14.ppm")
    subprocess.run([exe, out, "400", "10", "0xdeadbeef"], check=True, capture_output=True, timeout=300)
    cam = rtzig.final_scene_camera(width=400, aspect_ratio=16 / 9, spp=10)
    rgb, _ = gpu_render(cam, cam.scene.world, output="rgb8")
    assert open(out, "rb").read() == rtzig.encode_p6(rgb, 400, 225)


@pytest.mark.parametrize("variant", ["bvh", "smem_u4", "smem_u1", "lds_u2", "lds_u4"])
def test_walk_variants_bit_exact(oracle, variant, monkeypatch):
    """Every closest-hit walk (BVH and the linear list walks) gives oracle B's bits: golden config
    + the degenerate-materials scene."""
    monkeypatch.setenv("RTZIG_KERNEL", variant)
    cam = rtzig.final_scene_camera(width=200, aspect_ratio=16 / 9, spp=6)
    out, st = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, threads=8)
    assert np.array_equal(out, ref) and st["rays"] == rays
    cam = rtzig.chapter13_camera(width=160, spp=8)
    out, _ = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, _ = oracle.render_b(cam.cam, cam.scene.world, threads=8)
    assert np.array_equal(out, ref)


@pytest.mark.parametrize("order", ["pixel", "tile"])
def test_work_orders_bit_exact(oracle, order, monkeypatch):
    """The optional work-item orders (RTZIG_ORDER: pixel-major, 8x8 tiles) hand out every (pixel,
    sample) exactly once and give oracle B's bits, including partial tiles (W, rows not multiples
    of 8) and interleaved row sets."""
    import torch
    monkeypatch.setenv("RTZIG_ORDER", order)
    cam = rtzig.final_scene_camera(width=203, aspect_ratio=16 / 9, spp=5)
    out, st = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, threads=8)
    assert np.array_equal(out, ref) and st["rays"] == rays
    H = cam.height
    for row0, step in [(0, 8), (3, 8), (1, 3)]:
        n = (H - row0 + step - 1) // step
        part, _ = oracle.render_b(cam.cam, cam.scene.world, row0=row0, row_step=step, n_rows=n, threads=8)
        assert np.array_equal(part, ref[row0::step])
        r = rtzig.DeviceRenderer(0)
        r.set_scene(cam.scene.world)
        d = torch.empty((n, cam.width, 3), dtype=torch.float64, device="cuda:0")
        r.render_rows_async(cam.cam, d.data_ptr(), row0=row0, row_step=step, n_rows=n)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), part)
        r.close()


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


@pytest.mark.parametrize("mb", [3, 5])
def test_sample_chunked_workspace_bit_exact(oracle, monkeypatch, mb):
    """A workspace budget smaller than one frame of per-sample colors (RTZIG_WORKSPACE_MB) splits
    the samples into several launches; the reduce kernel carries the running sums across them in
    sample order (camera.zig:133-136), so the image must not change."""
    monkeypatch.setenv("RTZIG_WORKSPACE_MB", str(mb))
    cam = rtzig.chapter9_camera(spp=7)
    out, st = gpu_render(cam, cam.scene.world, n_gpus=1)
    ref, rays = oracle.render_b(cam.cam, cam.scene.world, threads=8)
    assert np.array_equal(out, ref) and st["rays"] == rays and st["samples"] == 400 * 225 * 7
    rgb, _ = gpu_render(cam, cam.scene.world, n_gpus=1, output="rgb8")
    assert np.array_equal(rgb, oracle.to_rgb8(ref))


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

"""Size limits of the launch (rt_kernel.h "Work units"): the largest images render correctly, and a
launch whose work units would overflow the 32-bit unit counter is refused before anything runs."""
import numpy as np
import pytest
import torch

import rtzig
from rtzig.lib import RtError

pytestmark = pytest.mark.gpu


def test_too_many_units_is_refused():
    """16384 x 16384 pixels x 4 M spp: 4.2 M tiles x ~83 000 chunks (of up to kUnitS = 48 samples)
    > 2^32 units -> RT_ERR_CAPACITY, returned before any buffer is allocated or kernel launched (the
    context stays usable).  The output buffer is full-size, so a regression that launched anyway
    would run long, never write out of bounds."""
    big = rtzig.final_scene_camera(width=16384, aspect_ratio=1.0, spp=4_000_000)
    r = rtzig.DeviceRenderer(0)
    r.set_scene(big.scene.world)
    full = torch.empty((big.height, big.width, 3), dtype=torch.float64, device="cuda:0")
    with pytest.raises(RtError) as e:
        r.render_rows_async(big.cam, full.data_ptr())
    del full
    assert e.value.code == rtzig.abi.RT_ERR_CAPACITY
    small = rtzig.final_scene_camera(width=32, aspect_ratio=1.0, spp=2)
    out = torch.zeros((32, 32, 3), dtype=torch.float64, device="cuda:0")
    r.render_rows_async(small.cam, out.data_ptr())
    r.sync()
    assert torch.isfinite(out).all()
    r.close()


@pytest.mark.parametrize("mode", ["ring", "direct"])
def test_8k_image_rows_bit_exact(oracle, mode, monkeypatch):
    """An 8K frame (7680 x 4320, 2 spp: 66 M samples in one launch) equals oracle B on two crops of
    rows, and its rows equal the same rows rendered alone."""
    monkeypatch.setenv("RTZIG_UNIT_MODE", mode)
    cam = rtzig.final_scene_camera(width=7680, aspect_ratio=16 / 9, spp=2)
    H, W = cam.height, cam.width
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    full = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda:0")
    r.render_rows_async(cam.cam, full.data_ptr())
    r.sync()
    for row0 in (1000, 3999):
        ref, _ = oracle.render_b(cam.cam, cam.scene.world, row0=row0, row_step=1, n_rows=1, threads=16)
        assert np.array_equal(full[row0:row0 + 1].cpu().numpy(), ref)
    part = torch.zeros((2, W, 3), dtype=torch.float64, device="cuda:0")
    r.render_rows_async(cam.cam, part.data_ptr(), row0=1000, row_step=2999, n_rows=2)
    r.sync()
    assert torch.equal(part[0], full[1000]) and torch.equal(part[1], full[3999])
    r.close()


def test_huge_scene_linear_walk_ring_mode(oracle, monkeypatch):
    """70 000 spheres: more than the BVH's depth bound holds (2^15 two-sphere leaves), so the tree
    does not build and the kernel walks the whole list (smem_u4) for every ray — ~100x the final
    scene's per-segment cost.  Ring mode forced with 2 tiles x 40 spp, so units of the same tile
    are chained across waves and their hand-off waits span slow predecessor units.  The bound is per
    wave: one continuous wait on the wall clock (rt_units.h wait_clock), 40 s here (the host scales it
    by 40 s per 2^16 spheres of a list walk: 70 000 -> 80 s, rt_runtime.cpp stall_bound) against a
    whole launch of ~1 s on the MI355X, so the test fails only if a wait is ~80x longer than the whole
    render.  The bits must equal oracle B's linear scan."""
    from rtzig.abi import D3, RtSphere
    monkeypatch.setenv("RTZIG_UNIT_MODE", "ring")
    rng = np.random.default_rng(65537)
    n = 70_000
    arr = (RtSphere * n)()
    arr[0] = RtSphere(center=D3(0, -1000, 0), radius=1000.0, material=0, albedo=D3(0.5, 0.5, 0.5))
    c = rng.uniform([-40, 0.05, -40], [40, 2.5, 40], (n, 3))
    rad = rng.uniform(0.02, 0.12, n)
    mats = rng.integers(0, 3, n)
    alb = rng.uniform(0, 1, (n, 3))
    for k in range(1, n):
        arr[k] = RtSphere(center=D3(*c[k]), radius=float(rad[k]), material=int(mats[k]), albedo=D3(*alb[k]),
                          fuzz=0.2, refraction_index=1.5)
    scene = rtzig.Scene.init(99)
    scene.world = arr
    cam = (rtzig.Camera.builder(16, 2.0).setScene(scene).setDefocusAngle(0.6).setFocusDist(10.0)
           .setViewport((13, 2, 3), (0, 0, 0), 20.0).setSamplesPerPixel(40).build())
    assert cam.width * cam.height == 128
    r = rtzig.DeviceRenderer(0)
    r.set_scene(arr)
    out = torch.zeros((cam.height, cam.width, 3), dtype=torch.float64, device="cuda:0")
    stats = torch.zeros(2, dtype=torch.int64, device="cuda:0")
    r.render_rows_async(cam.cam, out.data_ptr(), d_stats_ptr=stats.data_ptr())
    r.sync()  # raises if a wave gave up waiting
    assert r.kernel_name() == "smem_u4"  # the list walk: no tree for this many spheres
    r.close()
    ref, rays = oracle.render_b(cam.cam, arr, threads=16)
    assert np.array_equal(out.cpu().numpy(), ref)
    assert int(stats[0]) == rays


def test_stalled_handoff_reports_error_and_recovers(oracle, monkeypatch):
    """The bounded hand-off wait's give-up path (rt_units.h).  With the bound shortened to 0 µs
    (test hook RTZIG_STALL_US) a wave that has to wait for a predecessor unit gives up on its second
    poll, sets the sticky error word and leaves; the launch must end (not hang) and report
    RT_ERR_HIP — through rt_context_sync after it, and through rt_render.  A report clears the word,
    so the next render with the normal bound succeeds and is bit-exact.  One pixel at 700 spp in
    ring mode: 700 one-sample units of one tile, finalised strictly in chain order, so many waves
    wait."""
    from rtzig.abi import RT_ERR_HIP
    monkeypatch.setenv("RTZIG_UNIT_MODE", "ring")
    cam = (rtzig.Camera.builder(1, 1.0).setScene(rtzig.Scene.init(0x5eed).generateWorld())
           .setDefocusAngle(0.6).setFocusDist(10).setViewport((13, 2, 3), (0, 0, 0), 20)
           .setSamplesPerPixel(700).build())
    ref, _ = oracle.render_b(cam.cam, cam.scene.world)
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    out = torch.zeros((1, 1, 3), dtype=torch.float64, device="cuda:0")
    monkeypatch.setenv("RTZIG_STALL_US", "0")
    r.render_rows_async(cam.cam, out.data_ptr())
    r.render_rows_async(cam.cam, out.data_ptr())  # a second failing frame before the report
    with pytest.raises(RtError) as e:
        r.sync()
    assert e.value.code == RT_ERR_HIP
    r.sync()  # reported once: the sticky word is clear again
    monkeypatch.delenv("RTZIG_STALL_US")
    r.render_rows_async(cam.cam, out.data_ptr())
    r.sync()
    assert np.array_equal(out.cpu().numpy(), ref)
    r.close()
    monkeypatch.setenv("RTZIG_STALL_US", "0")
    with pytest.raises(RtError) as e:
        rtzig.render(cam.cam, cam.scene.world, n_gpus=1)
    assert e.value.code == RT_ERR_HIP
    monkeypatch.delenv("RTZIG_STALL_US")
    assert np.array_equal(rtzig.render(cam.cam, cam.scene.world, n_gpus=1), ref)


def test_workspace_sized_to_the_launch(oracle):
    """The context's workspace follows the kernel it launches (rt.h "Workspace"): config 4's whole
    frame (ring mode, the BVH kernel's 16 resident waves per CU) holds at most 0.6 GiB; a rank's rows
    of an 8-GPU job (direct mode) hold their stored samples and no ring; back in ring mode the
    samples are given back.  The frame rendered last equals the first bit for bit, and a crop of
    both equals oracle B (reference: camera.zig:125 allocates only the W x H framebuffer)."""
    cam = rtzig.final_scene_camera(width=1200, aspect_ratio=1.5, spp=500)
    H, W = cam.height, cam.width
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    full = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda:0")
    r.render_rows_async(cam.cam, full.data_ptr())
    r.sync()
    ring_bytes = r.workspace_bytes()
    assert "direct" not in r.kernel_name()
    assert ring_bytes <= 0.6 * 2**30, ring_bytes
    rows = torch.zeros((100, W, 3), dtype=torch.float64, device="cuda:0")
    r.render_rows_async(cam.cam, rows.data_ptr(), row0=0, row_step=8, n_rows=100)
    r.sync()
    assert "direct" in r.kernel_name()
    direct_bytes = r.workspace_bytes()
    need = 100 * W * 500 * 24
    assert need <= direct_bytes <= need + 2**20, direct_bytes
    assert torch.equal(rows, full[0::8])
    again = torch.zeros_like(full)
    r.render_rows_async(cam.cam, again.data_ptr())
    r.sync()
    assert abs(r.workspace_bytes() - ring_bytes) <= 2**16  # the chunk table may differ by a few bytes
    assert torch.equal(again, full)
    r.close()
    ref, _ = oracle.render_b(cam.cam, cam.scene.world, row0=400, row_step=1, n_rows=1, threads=16)
    assert np.array_equal(full[400:401].cpu().numpy(), ref)

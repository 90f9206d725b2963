"""Fast mode (RT_PRECISION_F32, rt_kernel_fast.hip): the hot path in f32 arithmetic.

Parity ladder step 4: fast mode is checked statistically against the f64 parity
path and against the reference's own golden image, with the tolerance of the f64-vs-golden check:
per-channel image mean |delta| <= 1.0 (8-bit units), and an 8x8 box-filtered RMSE that stays within
1.5x the noise floor (two f64 renders that differ only in their seed) plus 0.25.
"""
import numpy as np
import pytest
import torch

import rtzig

pytestmark = pytest.mark.gpu


def box8(x):
    h, w = x.shape[0] // 8 * 8, x.shape[1] // 8 * 8
    return x[:h, :w].reshape(h // 8, 8, w // 8, 8, 3).mean(axis=(1, 3))


def rmse(a, b):
    return float(np.sqrt(((box8(a) - box8(b)) ** 2).mean()))


def render_rgb(cam, precision, seed=None):
    c = cam.cam
    if seed is not None:
        c.seed = seed
    out = rtzig.render(c, cam.scene.world, n_gpus=1, output="rgb8", precision=precision)
    return out.astype(np.float64)


def check_stat(cam):
    f64_a = render_rgb(cam, "f64", seed=0xDEADBEEF)
    f64_b = render_rgb(cam, "f64", seed=0x5EED5EED)
    f32_a = render_rgb(cam, "f32", seed=0xDEADBEEF)
    floor = rmse(f64_a, f64_b)
    mean_d = np.abs(f32_a.mean(axis=(0, 1)) - f64_a.mean(axis=(0, 1))).max()
    err = rmse(f32_a, f64_a)
    assert mean_d <= 1.0, (mean_d, floor, err)
    assert err <= 1.5 * floor + 0.25, (mean_d, floor, err)
    return floor, err


@pytest.mark.parametrize("mode", ["ring", "direct"])
def test_fast_final_scene_statistical(mode, monkeypatch):
    """Final random-sphere scene (485 spheres, defocus, all three materials), in both unit modes
    (rt_kernel.h "Work units"; direct is the default at this size)."""
    monkeypatch.setenv("RTZIG_UNIT_MODE", mode)
    check_stat(rtzig.final_scene_camera(width=480, aspect_ratio=1.5, spp=64))


def test_fast_chapter13_statistical():
    """Three materials, hollow glass bubble, fuzz-1 metal, defocus 10."""
    check_stat(rtzig.chapter13_camera(width=480, spp=64))


def test_fast_chapter9_statistical():
    """Two Lambertian spheres, no defocus (the ground r=100 sphere is on the f64 always-list)."""
    check_stat(rtzig.chapter9_camera(width=400, spp=64))


def test_fast_vs_reference_golden(golden_dir):
    """The golden test's configuration (main.zig:41-55) against test-files/chapter14.ppm with the
    tolerance of tests/test_gpu_parity.py's f64 check."""
    import os

    from oracle_lib import read_ppm
    cam = rtzig.final_scene_camera(width=400, aspect_ratio=16 / 9, spp=10)
    a = rtzig.render(cam.cam, cam.scene.world, n_gpus=1, output="rgb8", precision="f32").astype(np.float64)
    _, _, gold = read_ppm(open(os.path.join(golden_dir, "chapter14.ppm"), "rb").read())
    b = gold.astype(np.float64)
    assert np.abs(a.mean(axis=(0, 1)) - b.mean(axis=(0, 1))).max() <= 1.0
    assert rmse(a, b) <= 2.0


@pytest.mark.parametrize("mode", ["ring", "direct"])
def test_fast_counts_deterministic_and_row_invariant(mode, monkeypatch):
    """Every sample is written once; the image does not depend on the row partition or on the unit
    mode (both add each pixel's samples in sample order)."""
    monkeypatch.setenv("RTZIG_UNIT_MODE", mode)
    cam = rtzig.final_scene_camera(width=240, aspect_ratio=1.5, spp=16)
    H, W = cam.height, cam.width
    r = rtzig.DeviceRenderer(0)
    r.set_scene(cam.scene.world)
    r.set_precision("f32")
    full = torch.zeros((H, W, 3), dtype=torch.float64, device="cuda:0")
    st = torch.zeros(2, dtype=torch.int64, device="cuda:0")
    r.render_rows_async(cam.cam, full.data_ptr(), d_stats_ptr=st.data_ptr())
    torch.cuda.synchronize()
    assert "fast_f32" in r.kernel_name()
    assert int(st[1]) == H * W * 16
    assert int(st[0]) >= H * W * 16
    again = torch.zeros_like(full)
    r.render_rows_async(cam.cam, again.data_ptr())
    parts = []
    for rank in range(3):
        n = (H - rank + 2) // 3
        buf = torch.zeros((n, W, 3), dtype=torch.float64, device="cuda:0")
        r.render_rows_async(cam.cam, buf.data_ptr(), row0=rank, row_step=3, n_rows=n)
        parts.append(buf)
    torch.cuda.synchronize()
    assert torch.equal(full, again)
    for rank in range(3):
        assert torch.equal(full[rank::3], parts[rank])
    assert torch.isfinite(full).all()
    other = "direct" if mode == "ring" else "ring"
    monkeypatch.setenv("RTZIG_UNIT_MODE", other)
    again2 = torch.zeros_like(full)
    r.render_rows_async(cam.cam, again2.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(full, again2)
    r.close()

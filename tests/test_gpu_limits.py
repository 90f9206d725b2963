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

"""Checks derived by hand from the reference's source, independent of the oracle (oracle/ is a
restatement of the same code, so a mistake shared by it and the kernels would pass the parity
tests; these expected values come from reading engine.rs / object.rs / color.rs directly).

* BoundingBox::intersects (object.rs:327-379) with a loaded mesh's box, which is the degenerate
  (0,0,0)-(0,0,0) box (object.rs:101-186 never sets it).  For a camera at (0, 0, z) every slab
  entry/exit of x and y is (0 - 0) * invdir = 0 (or NaN where a direction component is +-0: 0 *
  inf), so neither early return fires and the final `t = txmin` is the z slab's positive entry:
  every camera ray passes, exactly as with the mesh's true box.  For a camera at (0.3, 0, z), a
  ray with dy != 0 has t_y = 0 and t_x = -0.3 / dx != 0 on one side of it, so `txmin > tymax` or
  `tymin > txmax` returns false; only a ray with dy == +0 (t_y = NaN, every comparison false)
  passes — the camera row y = H / 2 (y' = 0.5 makes the direction's y exactly 0, camera.rs:57-76).
* Engine::render's anti-aliasing (engine.rs:59-77): the pixel is (sum of the AA + 1 samples'
  colours) / AA, clamped; a ray that hits nothing contributes the single colour (0.1, 0.1, 0.2)
  (engine.rs:212), whose Color::sum is that colour (color.rs:82-87, reduce without a zero).
"""
import numpy as np
import pytest

from eray_amd import capi

pytestmark = pytest.mark.gpu

W, H = 160, 90


def _scene(gpu, cube, center, true_box):
    pos, nrm, uv = cube
    gpu.scene_reset()
    gpu.set_camera(capi.make_camera(center, (16.0, 9.0), W, 1.0))
    gpu.add_light(capi.make_light((0.0, 2.0, 0.0), "ambient", (1.0, 1.0, 1.0), 0.2))
    gpu.add_light(capi.make_light((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0))
    if true_box:
        p = pos.reshape(-1, 3)
        gpu.add_object(pos, nrm, uv, tuple(p.min(0)), tuple(p.max(0)))
    else:
        gpu.add_object(pos, nrm, uv)  # the loader's (0,0,0)-(0,0,0) box


def _render(gpu, flags=0, aa=0):
    rgb = gpu.empty((H, W, 3), np.float32)
    face = gpu.empty((H, W), np.int32)
    try:
        gpu.render(W, H, out_rgb=rgb.ptr, out_face=face.ptr, flags=flags, anti_aliasing=aa, aa_seed=7)
        gpu.synchronize()
        return rgb.numpy().copy(), face.numpy().copy()
    finally:
        rgb.free()
        face.free()


@pytest.mark.parametrize("flags", [capi.RENDER_DEFAULT, capi.RENDER_BRUTE_FORCE])
def test_degenerate_box_on_axis_camera_passes_every_ray(gpu, cube, flags):
    _scene(gpu, cube, (0.0, 0.0, 5.0), true_box=False)
    rgb_d, face_d = _render(gpu, flags)
    _scene(gpu, cube, (0.0, 0.0, 5.0), true_box=True)
    rgb_t, face_t = _render(gpu, flags)
    assert (face_d >= 0).sum() > 500
    assert np.array_equal(face_d, face_t)
    assert np.array_equal(rgb_d.view(np.uint32), rgb_t.view(np.uint32))


@pytest.mark.parametrize("flags", [capi.RENDER_DEFAULT, capi.RENDER_BRUTE_FORCE])
def test_degenerate_box_off_axis_camera_passes_only_the_centre_row(gpu, cube, flags):
    _scene(gpu, cube, (0.3, 0.0, 5.0), true_box=False)
    _, face_d = _render(gpu, flags)
    _scene(gpu, cube, (0.3, 0.0, 5.0), true_box=True)
    _, face_t = _render(gpu, flags)
    rows = np.flatnonzero((face_d >= 0).any(axis=1))
    assert rows.tolist() == [H // 2]
    # on that row the degenerate box lets every ray through: the hits are the true box's
    assert np.array_equal(face_d[H // 2], face_t[H // 2])
    assert (face_t >= 0).sum() > (face_d >= 0).sum() > 10


@pytest.mark.parametrize("aa", [1, 2, 3, 5])
def test_anti_aliasing_average_of_missed_rays(gpu, aa):
    gpu.scene_reset()
    gpu.set_camera(capi.make_camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0))
    rgb, face = _render(gpu, aa=aa)
    miss = np.array([0.1, 0.1, 0.2], np.float32)
    avg = miss.copy()  # the un-jittered ray's Color::sum
    for _ in range(aa):
        avg = (avg + miss).astype(np.float32)
    want = np.clip((avg / np.float32(aa)).astype(np.float32), 0.0, 1.0).astype(np.float32)
    assert (face == -1).all()
    assert np.array_equal(rgb.reshape(-1, 3).view(np.uint32), np.broadcast_to(want, (W * H, 3)).view(np.uint32))

"""Moving cameras: eray_render_camera_path (Scene::set_camera + Engine::render per frame,
scene.rs:39-54, engine.rs:46-81) runs every frame's camera setup on the device (setup.hip,
bins.hip) and reads it in the frame kernel (device-camera mode).  Every frame must be the frame
eray_render writes for that camera, bit for bit, and the oracle's."""
import math

import numpy as np
import pytest

from eray_amd import capi, meshgen
from eray_amd.frame import MainScene
from tests.helpers import assert_bit_equal

pytestmark = pytest.mark.gpu


def dolly(n, z=5.0, amp=1.5, fov=(16.0, 9.0), width=320):
    """n cameras moving along the z axis with a changing z_dist.  A loaded mesh's bounding box is
    the degenerate (0,0,0)-(0,0,0) box (object.rs:306-315, 327-379): only rays from x = y = 0 pass
    it, so a camera that leaves the axis sees nothing of it — the reference's semantics."""
    return [capi.make_camera((0.0, 0.0, z + amp * math.sin(2.0 * math.pi * k / n)), fov, width,
                             1.0 + 0.3 * math.cos(2.0 * math.pi * k / n)) for k in range(n)]


def orbit(n, radius=4.0, fov=(16.0, 9.0), width=160):
    """n off-axis cameras around the origin (for objects with real bounding boxes)."""
    return [capi.make_camera((1.3 * math.sin(2.0 * math.pi * k / n), 0.7 * math.cos(6.0 * math.pi * k / n),
                              radius + 0.8 * math.cos(2.0 * math.pi * k / n)), fov, width, 1.0) for k in range(n)]


class Out:
    def __init__(self, ctx, W, H):
        self.ctx, self.W, self.H = ctx, W, H
        self.rgb = ctx.empty((H, W, 3), np.float32)
        self.ppm = ctx.empty((H, W, 3), np.uint8)
        self.face = ctx.empty((H, W), np.int32)

    def clear(self):
        for a, v in ((self.rgb, 0), (self.ppm, 0), (self.face, 0x7F)):
            self.ctx.memset(a.ptr, v, a.nbytes)

    def kw(self):
        return dict(out_rgb=self.rgb.ptr, out_ppm=self.ppm.ptr, out_face=self.face.ptr)

    def get(self):
        self.ctx.synchronize()
        return self.rgb.numpy(), self.face.numpy(), self.ppm.numpy()

    def free(self):
        for a in (self.rgb, self.ppm, self.face):
            a.free()


def per_camera(ctx, out, cam, flags=0):
    ctx.set_camera(cam)
    out.clear()
    ctx.render(out.W, out.H, flags=flags, **out.kw())
    return [a.copy() for a in out.get()]


def check(got, ref, what):
    assert np.array_equal(got[1], ref[1]), f"{what}: faces"
    assert_bit_equal(got[0], ref[0], what)
    assert np.array_equal(got[2], ref[2]), f"{what}: ppm"


def test_cube_camera_path_equals_per_camera_renders(gpu, oracle, cube):
    W, H = 320, 180
    sc = MainScene(gpu, *cube, W, H, texture=256, fov=(16.0, 9.0))
    out = Out(gpu, W, H)
    cams = dolly(7, width=W)
    try:
        refs = [per_camera(gpu, out, c) for c in cams]
        gpu.set_camera(capi.make_camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0))
        assert len({r[1].tobytes() for r in refs}) == len(refs)  # the cameras see different frames
        for k in range(len(cams)):  # every prefix: its last frame is camera k's
            out.clear()
            ms = gpu.render_camera_path(cams[: k + 1], W, H, timed=True, **out.kw())
            assert ms > 0.0
            check(out.get(), refs[k], f"path frame {k}")
        # a long path (graph chunks of 64 + a remainder), cycling the cameras: ends on camera 69 % 7
        path = [cams[f % 7] for f in range(70)]
        out.clear()
        gpu.render_camera_path(path, W, H, **out.kw())
        check(out.get(), refs[69 % 7], "path of 70")
        # the same path again (the cached graphs re-read the cameras), now ending on another camera
        path[-1] = cams[2]
        out.clear()
        gpu.render_camera_path(path, W, H, **out.kw())
        check(out.get(), refs[2], "path of 70, replayed")
        # the scene camera is untouched and is set up again for the next render
        again = per_camera(gpu, out, capi.make_camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0))
        ref, ref_face, _ = oracle.render(oracle.main_rs_scene(*cube, texture=256),
                                         oracle.camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0), want_faces=True)
        assert np.array_equal(again[1], ref_face)
        assert_bit_equal(again[0], ref, "scene camera after paths")
        # one path camera against the oracle
        c = cams[3]
        ref, ref_face, _ = oracle.render(oracle.main_rs_scene(*cube, texture=256),
                                         oracle.camera(tuple(c.center), (16.0, 9.0), W, c.z_dist), want_faces=True)
        out.clear()
        gpu.render_camera_path([c], W, H, **out.kw())
        got = out.get()
        assert np.array_equal(got[1], ref_face)
        assert_bit_equal(got[0], ref, "path camera vs oracle")
    finally:
        out.free()
        sc.close()


def test_off_axis_path_with_bounding_boxes(gpu, oracle):
    """Objects with real bounding boxes seen from an off-axis orbit: every path frame equals the
    oracle's frame for its camera."""
    from tests.helpers import random_mesh
    rng = np.random.default_rng(21)
    W, H = 160, 90
    gpu.scene_reset()
    gpu.set_camera(capi.make_camera((0.0, 0.0, 4.0), (16.0, 9.0), W, 1.0))
    s = oracle.Scene()
    keep = []
    for k in range(3):
        pos, nrm, uv = random_mesh(rng, 60, scale=0.5, center=rng.uniform(-0.8, 0.8, 3))
        lo, hi = pos.reshape(-1, 3).min(0), pos.reshape(-1, 3).max(0)
        color = rng.uniform(0, 1, (8, 8, 3)).astype(np.float32)
        dc = gpu.to_device(color)
        keep.append(dc)
        gpu.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=dc.image())
        s.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=color)
    for pos, var, col, b in (((0.0, 2.0, 0.0), "ambient", (1.0, 1.0, 1.0), 0.2),
                             ((1.0, 1.0, 2.0), "point", (1.0, 0.8, 0.6), 1.0)):
        gpu.add_light(capi.make_light(pos, var, col, b))
        s.add_light(pos, var, col, b)
    out = Out(gpu, W, H)
    try:
        cams = orbit(6, width=W)
        for k in (0, 3, 5):
            out.clear()
            gpu.render_camera_path(cams[: k + 1], W, H, **out.kw())
            got = out.get()
            c = cams[k]
            ref, ref_face, _ = oracle.render(s, oracle.camera(tuple(c.center), (16.0, 9.0), W, 1.0), want_faces=True)
            assert (ref_face >= 0).sum() > 100
            assert np.array_equal(got[1], ref_face), f"orbit frame {k}"
            assert_bit_equal(got[0], ref, f"orbit frame {k}")
    finally:
        out.free()
        for a in keep:
            a.free()


def test_camera_path_rejects_a_different_camera_size(gpu, cube):
    W, H = 64, 36
    sc = MainScene(gpu, *cube, W, H, texture=16, fov=(16.0, 9.0))
    out = Out(gpu, W, H)
    try:
        with pytest.raises(capi.ErayError) as e:
            gpu.render_camera_path([capi.make_camera((0, 0, 5), (16.0, 9.0), 128, 1.0)], W, H, **out.kw())
        assert e.value.status == capi.E_INVALID_ARGUMENT
    finally:
        out.free()
        sc.close()


@pytest.fixture(scope="module")
def standin70k():
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(**meshgen.STANDIN_70K)
    return (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(n[fn].reshape(-1, 9)),
            np.ascontiguousarray(t[ft].reshape(-1, 6)))


@pytest.mark.parametrize("flags", [0, capi.RENDER_DENSE_DETAIL | capi.RENDER_SEPARATE_FILL,
                                   capi.RENDER_SHARED_DETAIL])
def test_binned_camera_path_equals_brute_force(gpu, standin70k, flags):
    """A 70k-face object: each path frame's bins are rebuilt on the device; the frame equals the
    brute-force scan for that camera.  RENDER_SHARED_DETAIL: the split detail list's
    light sub-blocks sit at the back of the list, so list positions must follow the setup's heavy
    count whatever the flag says about sharing work."""
    W, H = 480, 270
    sc = MainScene(gpu, *standin70k, W, H, texture=256, fov=(16.0, 9.0))
    out = Out(gpu, W, H)
    cams = dolly(5, width=W, z=4.5, amp=1.2)
    try:
        refs = [per_camera(gpu, out, c, flags=capi.RENDER_BRUTE_FORCE) for c in cams]
        for k in (0, 2, 4):
            out.clear()
            gpu.render_camera_path(cams[: k + 1], W, H, flags=flags, **out.kw())
            check(out.get(), refs[k], f"binned path frame {k}")
        path = [cams[f % 5] for f in range(67)]
        out.clear()
        gpu.render_camera_path(path, W, H, flags=flags, **out.kw())
        check(out.get(), refs[66 % 5], "binned path of 67")
    finally:
        out.free()
        sc.close()


def test_bin_overflow_falls_back_and_grows(gpu, standin70k):
    """Bins whose entries exceed the capacity are dropped for that camera (the frame scans the
    object through LDS tiles: same image); the host then grows the capacity."""
    W, H = 480, 270
    sc = MainScene(gpu, *standin70k, W, H, texture=256, fov=(16.0, 9.0))
    out = Out(gpu, W, H)
    L = capi.lib()
    try:
        cam = capi.make_camera((0.2, 0.1, 4.0), (16.0, 9.0), W, 1.0)
        ref = per_camera(gpu, out, cam, flags=capi.RENDER_BRUTE_FORCE)
        assert L.eray_debug_set_bin_capacity(gpu.handle, 16) == 0
        first = per_camera(gpu, out, cam)  # device-camera frame of an overflowed setup
        check(first, ref, "overflowed bins")
        out.clear()
        gpu.render(W, H, **out.kw())  # the count reached the host: capacity grown, set up again
        check(out.get(), ref, "after growth")
        assert L.eray_debug_bin_capacity(gpu.handle) > 16
        out.clear()
        gpu.render_camera_path([cam, cam], W, H, **out.kw())
        check(out.get(), ref, "path after growth")
    finally:
        out.free()
        sc.close()


def test_path_graph_not_replayed_after_bin_reallocation(gpu, standin70k):
    """A camera path captured while the bins overflowed, then a render that grows the capacity
    (every bin buffer reallocated), then the same path again: the path's cached graph holds the
    old buffers' addresses and must be captured anew (bins generation in the key)."""
    W, H = 480, 270
    sc = MainScene(gpu, *standin70k, W, H, texture=256, fov=(16.0, 9.0))
    out = Out(gpu, W, H)
    L = capi.lib()
    try:
        cam = capi.make_camera((0.1, -0.1, 4.2), (16.0, 9.0), W, 1.0)
        ref = per_camera(gpu, out, cam, flags=capi.RENDER_BRUTE_FORCE)
        assert L.eray_debug_set_bin_capacity(gpu.handle, 16) == 0
        for rep in range(2):
            out.clear()
            gpu.render_camera_path([cam, cam, cam], W, H, **out.kw())  # overflowed bins: LDS tiles
            check(out.get(), ref, f"overflowed path {rep}")
        out.clear()
        gpu.render(W, H, **out.kw())  # the count reached the host: capacity grown, buffers reallocated
        check(out.get(), ref, "render after growth")
        assert L.eray_debug_bin_capacity(gpu.handle) > 16
        for rep in range(2):
            out.clear()
            gpu.render_camera_path([cam, cam, cam], W, H, **out.kw())
            check(out.get(), ref, f"path after reallocation {rep}")
    finally:
        out.free()
        sc.close()

"""Frames in flight (eray_render_frames_ring / eray_render_camera_path_ring): several frames per
kernel launch, frame k into ring slot k % slots.  Every slot must hold exactly the frame eray_render
writes (engine.rs:46-81) for that frame's camera, bit for bit, whatever the frames per launch."""
import math

import numpy as np
import pytest

from eray_amd import capi
from eray_amd.dist import band_split
from eray_amd.frame import MainScene
from tests.helpers import assert_bit_equal

pytestmark = pytest.mark.gpu


class Ring:
    """`slots` contiguous output slots of rows x W (f32 RGB, PPM bytes, faces)."""

    def __init__(self, ctx, slots, rows, W):
        self.ctx, self.slots, self.rows, self.W = ctx, slots, rows, W
        self.rgb = ctx.empty((slots, rows, W, 3), np.float32)
        self.ppm = ctx.empty((slots, rows, W, 3), np.uint8)
        self.face = ctx.empty((slots, rows, W), np.int32)

    def clear(self):
        for a, v in ((self.rgb, 0), (self.ppm, 0), (self.face, 0x7F)):
            self.ctx.memset(a.ptr, v, a.nbytes)

    def kw(self):
        return dict(out_rgb=self.rgb.ptr, out_ppm=self.ppm.ptr, out_face=self.face.ptr)

    def ring(self, per_launch=0):
        return capi.frame_ring(self.slots, self.rows, self.W, per_launch)

    def get(self):
        self.ctx.synchronize()
        return self.rgb.numpy(), self.face.numpy(), self.ppm.numpy()

    def free(self):
        for a in (self.rgb, self.ppm, self.face):
            a.free()


def single(ctx, W, H, flags=0, **kw):
    rows = kw.get("rows", H)
    rgb = ctx.empty((rows, W, 3), np.float32)
    ppm = ctx.empty((rows, W, 3), np.uint8)
    face = ctx.empty((rows, W), np.int32)
    try:
        ctx.render(W, H, out_rgb=rgb.ptr, out_ppm=ppm.ptr, out_face=face.ptr, flags=flags, **kw)
        ctx.synchronize()
        return rgb.numpy(), face.numpy(), ppm.numpy()
    finally:
        for a in (rgb, ppm, face):
            a.free()


def check_slot(got, s, ref, what):
    assert np.array_equal(got[1][s], ref[1]), f"{what}: faces of slot {s}"
    assert_bit_equal(got[0][s], ref[0], f"{what}: rgb of slot {s}")
    assert np.array_equal(got[2][s], ref[2]), f"{what}: ppm of slot {s}"


@pytest.mark.parametrize("per_launch", [0, 1, 2, 4, 8])
def test_static_ring_every_slot_is_the_frame(gpu, cube, per_launch):
    W, H = 320, 180
    sc = MainScene(gpu, *cube, W, H, texture=256, fov=(16.0, 9.0))
    ring = Ring(gpu, 8, H, W)
    try:
        ref = single(gpu, W, H)
        assert (ref[1] >= 0).any()
        for frames in (8, 13, 64 + 6):  # whole rings, a partial launch, a graph chunk + remainder
            ring.clear()
            gpu.render_frames(frames, W, H, ring=ring.ring(per_launch), **ring.kw())
            got = ring.get()
            for s in range(min(frames, 8)):
                check_slot(got, s, ref, f"{frames} frames, {per_launch} per launch")
        ms = gpu.render_frames(16, W, H, ring=ring.ring(per_launch), timed=True, **ring.kw())
        assert ms > 0.0
    finally:
        ring.free()
        sc.close()


def test_ring_beyond_the_infinity_cache(gpu, cube):
    """A ring whose slots together exceed the 256 MiB Infinity Cache (16 slots of 1920x1080: 630 MB)
    takes the unpaced per-lane-coordinate fill (render.hip kLaunchRingBeyondCache): every slot is
    still the frame eray_render writes."""
    W, H = 1920, 1080
    sc = MainScene(gpu, *cube, W, H, texture=256, fov=(16.0, 9.0))
    ring = Ring(gpu, 16, H, W)
    try:
        ref = single(gpu, W, H)
        assert (ref[1] >= 0).any()
        ring.clear()
        gpu.render_frames(16, W, H, ring=ring.ring(8), **ring.kw())
        got = ring.get()
        for s in range(16):
            check_slot(got, s, ref, "16-slot ring")
    finally:
        ring.free()
        sc.close()


def test_static_ring_large_mesh_and_bands(gpu, standin70k_ring):
    """A binned 70k-face mesh (screen bins, detail list), whole frames and a 3-rank band share."""
    W, H = 480, 270
    sc = MainScene(gpu, *standin70k_ring, W, H, texture=256, fov=(16.0, 9.0))
    try:
        for split in (None, (1, 3)):
            kw = {}
            rows = H
            if split:
                sp = band_split(split[0], split[1], H)
                kw = dict(row0=sp["row0"], rows=sp["rows"], band_rows=sp["band_rows"], band_stride=sp["band_stride"])
                rows = sp["rows"]
            ref = single(gpu, W, H, **kw)
            assert (ref[1] >= 0).sum() > 500
            ring = Ring(gpu, 4, rows, W)
            try:
                for per_launch in (0, 2, 4):
                    ring.clear()
                    gpu.render_frames(9, W, H, ring=ring.ring(per_launch), **ring.kw(), **kw)
                    got = ring.get()
                    for s in range(4):
                        check_slot(got, s, ref, f"split {split}, {per_launch} per launch")
            finally:
                ring.free()
    finally:
        sc.close()


@pytest.fixture(scope="module")
def standin70k_ring():
    from eray_amd import meshgen
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(**meshgen.STANDIN_70K)
    return (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(n[fn].reshape(-1, 9)),
            np.ascontiguousarray(t[ft].reshape(-1, 6)))


def dolly(n, W):
    return [capi.make_camera((0.0, 0.0, 5.0 + 1.5 * math.sin(2.0 * math.pi * k / n)), (16.0, 9.0), W,
                             1.0 + 0.3 * math.cos(2.0 * math.pi * k / n)) for k in range(n)]


@pytest.mark.parametrize("per_launch", [0, 1, 4])
def test_camera_path_ring_every_slot_is_its_camera(gpu, cube, per_launch):
    """A moving camera, several frames per launch: slot s ends holding the last frame k of the
    path with k % slots == s, rendered for camera k."""
    W, H = 320, 180
    sc = MainScene(gpu, *cube, W, H, texture=256, fov=(16.0, 9.0))
    cams = dolly(70, W)  # a graph chunk (64) + a remainder
    ring = Ring(gpu, 8, H, W)
    try:
        refs = {}
        for k in range(len(cams) - 8, len(cams)):
            gpu.set_camera(cams[k])
            refs[k % 8] = single(gpu, W, H)
        gpu.set_camera(capi.make_camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0))
        assert len({r[1].tobytes() for r in refs.values()}) == 8
        for rep in range(2):
            ring.clear()
            ms = gpu.render_camera_path(cams, W, H, ring=ring.ring(per_launch), timed=(rep == 1), **ring.kw())
            if rep == 1:
                assert ms > 0.0
            got = ring.get()
            for s in range(8):
                check_slot(got, s, refs[s], f"path, {per_launch} per launch, rep {rep}")
    finally:
        ring.free()
        sc.close()


@pytest.mark.parametrize("per_launch", [0, 2, 8])
def test_binned_camera_path_ring_every_slot_is_its_camera(gpu, standin70k_ring, per_launch):
    """A moving camera over a binned 70k-face mesh, several frames per launch: the frames of one
    launch read their own cameras' slices of a multi-camera setup (culling records, descriptors,
    detail lists, occupancy).  Paths of several builds (16 cameras each), a graph chunk plus a
    remainder, a partial build, and a 3-rank band share."""
    W, H = 480, 270
    sc = MainScene(gpu, *standin70k_ring, W, H, texture=256, fov=(16.0, 9.0))
    # (on the view axis: a loaded mesh's box is the degenerate one at the origin, object.rs:306-315)
    cams = [capi.make_camera((0.0, 0.0, 4.6 + 1.1 * math.sin(0.3 * k)), (16.0, 9.0), W, 1.0 + 0.2 * math.cos(0.5 * k))
            for k in range(70)]
    scene_cam = capi.make_camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0)
    try:
        for split in (None, (2, 3)):
            kw, rows = {}, H
            if split:
                sp = band_split(split[0], split[1], H)
                kw = dict(row0=sp["row0"], rows=sp["rows"], band_rows=sp["band_rows"], band_stride=sp["band_stride"])
                rows = sp["rows"]
            ring = Ring(gpu, 8, rows, W)
            try:
                for n in ((70, 37) if split is None else (21,)):
                    refs = {}
                    for k in range(n - 8, n):
                        gpu.set_camera(cams[k])
                        refs[k % 8] = single(gpu, W, H, flags=capi.RENDER_BRUTE_FORCE, **kw)
                    assert len({r[1].tobytes() for r in refs.values()}) == 8
                    gpu.set_camera(scene_cam)
                    ring.clear()
                    gpu.render_camera_path(cams[:n], W, H, ring=ring.ring(per_launch), **ring.kw(), **kw)
                    got = ring.get()
                    for s in range(8):
                        check_slot(got, s, refs[s], f"binned path of {n}, split {split}, {per_launch} per launch")
            finally:
                ring.free()
    finally:
        sc.close()


def test_ring_arguments_are_checked(gpu, cube):
    W, H = 64, 36
    sc = MainScene(gpu, *cube, W, H, texture=64, fov=(16.0, 9.0))
    ring = Ring(gpu, 4, H, W)
    try:
        bad = [capi.FrameRing(3, 0, 12 * W * H, 3 * W * H, 4 * W * H),        # slots not a power of two
               capi.FrameRing(4, 8, 12 * W * H, 3 * W * H, 4 * W * H),        # more per launch than slots
               capi.FrameRing(4, 3, 12 * W * H, 3 * W * H, 4 * W * H),        # not a power of two
               capi.FrameRing(4, 0, 12 * W * H - 16, 3 * W * H, 4 * W * H),   # overlapping slots
               capi.FrameRing(4, 0, 12 * W * H, 3 * W * H + 8, 4 * W * H)]    # unaligned stride
        for r in bad:
            with pytest.raises(capi.ErayError) as e:
                gpu.render_frames(4, W, H, ring=r, **ring.kw())
            assert e.value.status == capi.E_INVALID_ARGUMENT
    finally:
        ring.free()
        sc.close()


def test_anti_aliased_ring_is_one_frame_per_launch(gpu, cube):
    """The general tracer renders one frame per launch, into the ring's slots all the same."""
    W, H = 128, 72
    sc = MainScene(gpu, *cube, W, H, texture=64, fov=(16.0, 9.0))
    ring = Ring(gpu, 2, H, W)
    try:
        rgb = gpu.empty((H, W, 3), np.float32)
        gpu.render(W, H, out_rgb=rgb.ptr, anti_aliasing=2, aa_seed=7)
        ref = rgb.numpy()
        rgb.free()
        ring.clear()
        gpu.render_frames(3, W, H, ring=ring.ring(0), anti_aliasing=2, aa_seed=7, **ring.kw())
        got = ring.get()
        for s in range(2):
            assert_bit_equal(got[0][s], ref, f"AA slot {s}")
    finally:
        ring.free()
        sc.close()

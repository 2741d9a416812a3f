"""GPU parity of the general tracer's binned camera rays (trace.hip first_face_binned, bins.hip
with SetupParams::keep_all): anti-aliasing on scenes with objects of more than kDirectMax (256)
faces, whose camera rays read the wave's screen bin instead of every face.

Bar: bit-identical f32 RGB, PPM bytes and first-ray faces, against the brute-force scan
(ERAY_RENDER_BRUTE_FORCE: every face per ray, the reference's loop) and the CPU oracle, which draws
the same Philox4x32-10 jitter (see test_gpu_trace.py).  Objects sit on the frame's first row and
column, whose jittered rays leave the viewport square [0, 1]^2 (the tracer's setup widens it to
[-1/W, 1] x [-1/H, 1]).
"""
import numpy as np
import pytest

from eray_amd import capi, meshgen
from eray_amd.frame import MainScene
from tests.helpers import assert_bit_equal, random_mesh

pytestmark = pytest.mark.gpu


def _trace(ctx, W, H, *, aa, seed, bounces=0, flags=capi.RENDER_DEFAULT, row0=0, rows=None, band_rows=0,
           band_stride=0):
    rows = H - row0 if rows is None else rows
    rgb = ctx.empty((rows, W, 3), np.float32)
    face = ctx.empty((rows, W), np.int32)
    ctx.memset(face.ptr, 0x7F, face.nbytes)
    ctx.render(W, H, row0=row0, rows=rows, out_rgb=rgb.ptr, out_face=face.ptr, bounces=bounces,
               anti_aliasing=aa, aa_seed=seed, flags=flags, band_rows=band_rows, band_stride=band_stride)
    out = rgb.numpy(), face.numpy()
    rgb.free()
    face.free()
    return out


def _corner_scene(gpu, oracle, rng, W, H, n_big, reflect):
    """One binned object (n_big random faces) across the corner of camera row 0 and column 0 (the
    viewport's bottom left: the view spans x in [-6, 6], y in [-4, 4] at the camera's distance 4),
    one across row 0, one small (unbinned) object in the middle; colour and reflection textures."""
    cam_center = (0.02, -0.01, 4.0)
    s = oracle.Scene()
    gpu.scene_reset()
    gpu.set_camera(capi.make_camera(cam_center, (3.0, 2.0), W, 1.0))
    keep = []
    for T, scale, c in ((n_big, 0.6, (-5.5, -3.6, 0.2)), (n_big // 2, 0.5, (1.0, -3.9, 0.0)),
                        (60, 0.4, (0.4, 0.2, -0.3))):
        pos, nrm, uv = random_mesh(rng, T, scale=scale, center=c)
        lo, hi = pos.reshape(-1, 3).min(0), pos.reshape(-1, 3).max(0)
        color = rng.uniform(0, 1.2, (5, 7, 3)).astype(np.float32)
        kw, okw = {}, {}
        d = [gpu.to_device(color)]
        if reflect:
            refl = rng.uniform(0, 0.9, (3, 4)).astype(np.float32)
            d.append(gpu.to_device(refl))
            kw["reflection"] = d[1].image()
            okw["reflection"] = refl
        keep += d
        gpu.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=d[0].image(), **kw)
        s.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=color, **okw)
    for p, var, col, b in [((0.0, 2.0, 0.0), "ambient", (0.9, 0.5, 1.0), 0.3),
                           ((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0)]:
        gpu.add_light(capi.make_light(p, var, col, b))
        s.add_light(p, var, col, b)
    return s, oracle.camera(cam_center, (3.0, 2.0), W, 1.0), keep


@pytest.mark.parametrize("seed,n_big,aa,bounces", [(61, 400, 4, 0), (62, 1500, 3, 1), (63, 5000, 2, 0)])
def test_binned_anti_aliasing_matches_brute_force_and_oracle(gpu, oracle, seed, n_big, aa, bounces):
    """Overlapping random faces: bins of every kind (short unsorted, 65..256 sorted, long
    unsorted), the frame's first row and column, reflected rays (bounces=1) and an unbinned object."""
    rng = np.random.default_rng(seed)
    W, H = 144, 96
    s, cam, keep = _corner_scene(gpu, oracle, rng, W, H, n_big, reflect=bounces > 0)
    try:
        rgb, face = _trace(gpu, W, H, aa=aa, seed=seed, bounces=bounces)
        brute, brute_face = _trace(gpu, W, H, aa=aa, seed=seed, bounces=bounces, flags=capi.RENDER_BRUTE_FORCE)
        # a row tile off the bins' phase, and interleaved bands
        tile, tile_face = _trace(gpu, W, H, aa=aa, seed=seed, bounces=bounces, row0=6, rows=50)
        bands, bands_face = _trace(gpu, W, H, aa=aa, seed=seed, bounces=bounces, row0=4, rows=44, band_rows=4,
                                   band_stride=8)
    finally:
        for a in keep:
            a.free()
    assert_bit_equal(rgb, brute, "binned vs brute force")
    assert np.array_equal(face, brute_face)
    assert_bit_equal(tile, rgb[6:56], "row tile")
    assert np.array_equal(tile_face, face[6:56])
    rows = np.array([4 + (j >> 2) * 8 + (j & 3) for j in range(44)])
    assert_bit_equal(bands, rgb[rows], "bands")
    assert np.array_equal(bands_face, face[rows])
    ref, ref_face, _ = oracle.render(s, cam, want_faces=True, bounces=bounces, anti_aliasing=aa, seed=seed)
    assert_bit_equal(rgb, ref, f"aa={aa}, bounces={bounces} vs oracle")
    assert np.array_equal(face, ref_face)
    assert (face[0] >= 0).any() and (face[:, 0] >= 0).any()  # the corner object reaches row 0 and column 0
    assert 0 < (face >= 0).sum() < face.size


def test_c3_anti_aliasing_frame_and_rows(gpu, oracle):
    """C3 (69,451-face stand-in, 1920x1080, main.rs's scene) with AA = 4: the binned frame equals the
    brute-force frame bit for bit, and the oracle on rows through the mesh centre and across its top
    silhouette."""
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(**meshgen.STANDIN_70K)
    mesh = (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(n[fn].reshape(-1, 9)),
            np.ascontiguousarray(t[ft].reshape(-1, 6)))
    W, H, seed = 1920, 1080, 2024
    sc = MainScene(gpu, *mesh, W, H, texture=1024, fov=(16.0, 9.0))
    try:
        rgb, face = _trace(gpu, W, H, aa=4, seed=seed)
        brute, brute_face = _trace(gpu, W, H, aa=4, seed=seed, flags=capi.RENDER_BRUTE_FORCE)
    finally:
        sc.close()
    assert (face >= 0).sum() > 30_000
    assert np.array_equal(face, brute_face)
    assert_bit_equal(rgb, brute, "c3 aa=4 binned vs brute force")
    hit_rows = np.nonzero((face >= 0).any(1))[0]
    top = int(hit_rows.min())
    s = oracle.main_rs_scene(*mesh, texture=1024)
    cam = oracle.camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0)
    for row0 in (540, top - 1, top + 2):
        ref, ref_face, _ = oracle.render(s, cam, row0=row0, rows=1, want_faces=True, anti_aliasing=4, seed=seed)
        assert np.array_equal(face[row0:row0 + 1], ref_face), row0
        assert_bit_equal(rgb[row0:row0 + 1], ref, f"c3 aa=4 row {row0} vs oracle")

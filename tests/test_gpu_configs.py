"""GPU parity at the BASELINE.json configurations' full sizes.

C4 (cube, 3840x2160, 4 GPUs) and C5 (1M faces, 7680x4320, 8 GPUs) are multi-GPU row-tile splits
(eray_amd/dist.py: rank r renders the r-th block of PPM file rows).  Every tile is rendered here on
one GPU exactly as its rank renders it (eray_render with row0 / rows), and the tiles must
concatenate into the full frame; the full frame is checked against the oracle (C4: the whole frame
and its committed digest; C5: the committed oracle pixel spans across the silhouette, the mesh
centre and the middle tile boundary) and, for the binned large-mesh path, against the GPU's own
brute-force scan (the reference's per-pixel loop, engine.rs:52-78, first hit by index,
object.rs:63-78) on row blocks at every tile boundary and through the mesh centre.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from eray_amd import capi, dist, meshgen
from eray_amd.dist import band_camera_rows, band_split
from eray_amd.frame import MainScene
from tests.helpers import assert_bit_equal

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


class Frame:
    """Device outputs of one W x H frame (or a row block of it), reused across renders."""

    def __init__(self, ctx, w, rows):
        self.ctx = ctx
        self.rgb = ctx.empty((rows, w, 3), np.float32)
        self.face = ctx.empty((rows, w), np.int32)
        self.ppm = ctx.empty((rows, w, 3), np.uint8)

    def render(self, W, H, row0=0, rows=None, flags=0):
        rows = H - row0 if rows is None else rows
        for a, v in ((self.rgb, 0), (self.face, 0x7F), (self.ppm, 0)):
            self.ctx.memset(a.ptr, v, a.nbytes)
        self.ctx.render(W, H, row0=row0, rows=rows, out_rgb=self.rgb.ptr, out_face=self.face.ptr,
                        out_ppm=self.ppm.ptr, flags=flags)
        n = rows * W
        rgb = self.rgb.numpy().reshape(-1)[: 3 * n].reshape(rows, W, 3)
        face = self.face.numpy().reshape(-1)[:n].reshape(rows, W)
        ppm = self.ppm.numpy().reshape(-1)[: 3 * n].reshape(rows, W, 3)
        return rgb, face, ppm

    def free(self):
        for a in (self.rgb, self.face, self.ppm):
            a.free()


def _mesh(triangles, seed):
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(triangles, seed)
    return (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(n[fn].reshape(-1, 9)),
            np.ascontiguousarray(t[ft].reshape(-1, 6)))


def _tiles_concatenate(fr, W, H, world, full):
    """Rank r of `world` renders the r-th block of PPM file rows (dist.row_block); its f32 rows,
    faces and file-order PPM rows must be the full frame's."""
    rgb, face, ppm = full
    rows = H // world
    got_ppm = []
    for r in range(world):
        row0, n = dist.row_block(r, world, rows)
        t_rgb, t_face, t_ppm = fr.render(W, H, row0=row0, rows=n)
        assert np.array_equal(t_face, face[row0:row0 + n]), f"tile {r} faces"
        assert_bit_equal(t_rgb, rgb[row0:row0 + n], f"tile {r} rgb")
        got_ppm.append(t_ppm.copy())
    # the gather on rank 0 is a concatenation in rank order = PPM file order
    assert np.array_equal(np.concatenate(got_ppm, 0), ppm), "gathered PPM body != full frame"


def _bands_assemble(gpu, W, H, world, full, band=dist.BAND_ROWS):
    """The interleaved-band split (dist.band_split): every rank's bands rendered with
    eray_render(row0, rows, band_rows, band_stride) must hold the full frame's pixels at its camera
    rows, and rank 0's reordering step of the banded gather (eray_debug_unband over the ranks'
    padded PPM blocks, as ncclGather leaves them) must give the full frame's PPM body."""
    rgb, face, ppm = full
    alloc = band_split(0, world, H, band)["alloc_rows"]
    staging = gpu.empty((world * alloc, W, 3), np.uint8)
    out = Frame(gpu, W, alloc)
    frame = gpu.empty((H, W, 3), np.uint8)
    try:
        gpu.memset(staging.ptr, 0, staging.nbytes)
        for r in range(world):
            sp = band_split(r, world, H, band)
            n = sp["rows"]
            for a, v in ((out.rgb, 0), (out.face, 0x7F), (out.ppm, 0)):
                gpu.memset(a.ptr, v, a.nbytes)
            gpu.render(W, H, row0=sp["row0"], rows=n, band_rows=sp["band_rows"], band_stride=sp["band_stride"],
                       out_rgb=out.rgb.ptr, out_face=out.face.ptr, out_ppm=out.ppm.ptr)
            cams = np.array(band_camera_rows(r, world, H, band))
            t_rgb = out.rgb.numpy().reshape(-1)[: 3 * n * W].reshape(n, W, 3)
            t_face = out.face.numpy().reshape(-1)[: n * W].reshape(n, W)
            assert np.array_equal(t_face, face[cams]), f"band rank {r} faces"
            assert_bit_equal(t_rgb, rgb[cams], f"band rank {r} rgb")
            gpu.copy_to_device(staging.ptr + r * alloc * W * 3, out.ppm.numpy().reshape(-1)[: 3 * n * W])
        assert capi.lib().eray_debug_unband(gpu.handle, staging.ptr, frame.ptr, H, W, band, world) == 0
        assert np.array_equal(frame.numpy(), ppm), "banded gather != full frame PPM"
        gpu.memset(frame.ptr, 0, frame.nbytes)  # the coded transport eray_gather_rows uses
        assert capi.lib().eray_debug_coded_unband(gpu.handle, staging.ptr, frame.ptr, H, W, band, world) == 0
        assert np.array_equal(frame.numpy(), ppm), "coded banded gather != full frame PPM"
    finally:
        out.free()
        staging.free()
        frame.free()


def test_c3_full_frame_binned_equals_brute_force(gpu):
    """C3 at 1920x1080 (69,451-face stand-in): the binned frame equals the brute-force scan over the
    whole frame, bit for bit, for both material paths."""
    mesh = _mesh(**meshgen.STANDIN_70K)
    W, H = 1920, 1080
    fr = Frame(gpu, W, H)
    try:
        for material in ("textures", "example"):
            sc = MainScene(gpu, *mesh, W, H, texture=1024, fov=(16.0, 9.0), material=material)
            a = [x.copy() for x in fr.render(W, H)]
            b = fr.render(W, H, flags=capi.RENDER_BRUTE_FORCE)
            sc.close()
            assert (a[1] >= 0).sum() > 30_000
            assert np.array_equal(a[1], b[1]), material
            assert_bit_equal(a[0], b[0], f"c3 full frame binned vs brute force ({material})")
            assert np.array_equal(a[2], b[2])
    finally:
        fr.free()


def test_c4_cube_4k_matches_oracle_and_row_tiles(gpu, oracle, cube):
    """C4: the cube at 3840x2160 against the oracle (live and its committed digest), and the
    4-GPU split's four row tiles concatenated into it."""
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        g = json.load(f)["c4"]
    W, H = 3840, 2160
    sc = MainScene(gpu, *cube, W, H, texture=1024, fov=(16.0, 9.0))
    fr = Frame(gpu, W, H)
    try:
        full = [x.copy() for x in fr.render(W, H)]
        rgb, face, ppm = full
        assert _sha(face.astype(np.int32)) == g["face_sha256"]
        assert _sha(rgb.astype(np.float32)) == g["rgb_f32_sha256"]
        assert _sha(ppm) == g["ppm_body_sha256"]
        assert hashlib.sha256(capi.ppm_header(W, H) + ppm.tobytes()).hexdigest() == g["ppm_file_sha256"]
        ref, ref_face, stats = oracle.render(oracle.main_rs_scene(*cube, texture=1024),
                                             oracle.camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0), want_faces=True)
        assert np.array_equal(face, ref_face)
        assert_bit_equal(rgb, ref, "c4 frame vs oracle")
        assert int((face >= 0).sum()) == stats["hit_pixels"] == g["hit_pixels"]
        _tiles_concatenate(fr, W, H, 4, full)
        _bands_assemble(gpu, W, H, 4, full)
    finally:
        fr.free()
        sc.close()


@pytest.fixture(scope="module")
def synth1m():
    """SURVEY.md §8(d) C5 mesh: the displaced sphere at 1,000,000 faces, permuted with seed 1234."""
    return _mesh(**meshgen.SYNTH_1M)


def test_c5_8k_1m_tiles_spans_and_brute_force(gpu, synth1m):
    """C5: 1M faces at 7680x4320.  The 8 row tiles of the 8-GPU split concatenate into the full
    binned frame; the frame matches the oracle's committed pixel spans; and the binned frame equals
    the GPU brute-force scan on 4-row blocks at every tile boundary and through the mesh centre
    (row blocks of every row phase, so the bins are rebuilt per phase)."""
    W, H = 7680, 4320
    sc = MainScene(gpu, *synth1m, W, H, texture=1024, fov=(16.0, 9.0))
    fr = Frame(gpu, W, H)
    blk = Frame(gpu, W, 8)
    try:
        full = [x.copy() for x in fr.render(W, H)]
        rgb, face, ppm = full
        assert (face >= 0).sum() > 400_000
        fx = np.load(os.path.join(GOLDEN, "c5_spans.npz"))
        for k, (y, x0, cols) in enumerate(fx["spans"].tolist()):
            assert np.array_equal(face[y, x0:x0 + cols], fx[f"face{k}"]), f"span {k} faces"
            assert_bit_equal(rgb[y, x0:x0 + cols], fx[f"rgb{k}"], f"span {k} ({y}, {x0}+{cols})")
        _tiles_concatenate(fr, W, H, 8, full)
        _bands_assemble(gpu, W, H, 8, full)
        boundaries = [540 * r for r in range(1, 8)]
        for y0, n in [(b - 2, 4) for b in boundaries] + [(2156, 8), (2161, 3), (1763, 5)]:
            for flags in (capi.RENDER_DEFAULT, capi.RENDER_BRUTE_FORCE):  # binned at row phase y0 % 4
                b_rgb, b_face, _ = blk.render(W, H, row0=y0, rows=n, flags=flags)
                assert np.array_equal(b_face, face[y0:y0 + n]), f"rows {y0}+{n} flags {flags}"
                assert_bit_equal(b_rgb, rgb[y0:y0 + n], f"c5 rows {y0}+{n} flags {flags}")
    finally:
        blk.free()
        fr.free()
        sc.close()

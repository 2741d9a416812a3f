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
import ctypes
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
    whole frame, bit for bit, for both material paths, and the oracle's whole C3 frame at main.rs's
    1024x1024 material (its committed digests: tests/golden/make_c3_digest.py, ~1.4e11 tests on the
    CPU)."""
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        g = json.load(f)["c3"]
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
            rgb, face, ppm = a
            assert int((face >= 0).sum()) == g["hit_pixels"], material
            assert _sha(face.astype(np.int32)) == g["face_sha256"], f"c3 faces vs oracle ({material})"
            assert _sha(rgb.astype(np.float32)) == g["rgb_f32_sha256"], f"c3 rgb vs oracle ({material})"
            assert _sha(ppm) == g["ppm_body_sha256"], f"c3 ppm vs oracle ({material})"
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


def test_north_star_4k_70k_full_frame_binned_equals_brute_force(gpu):
    """BASELINE north_star: the 69,451-face stand-in at 3840x2160.  The binned frame — the
    library's own launch choice (the dense 3-per-CU detail build and the heavy-first ordered
    detail list), the 2-per-CU build, and the dense build with the separate fill kernel — equals
    the brute-force scan over the whole frame, bit for bit (object.rs:63-78: first hit by index);
    so do two frames in flight per launch, the 4-band split's ranks and the scene-camera gather of
    their rows.  Against the oracle (not HIP against HIP): the committed rows of the frame through
    the mesh centre and its top and bottom silhouettes (tests/golden/ns_spans.npz)."""
    mesh = _mesh(**meshgen.STANDIN_70K)
    W, H = 3840, 2160
    sc = MainScene(gpu, *mesh, W, H, texture=1024, fov=(16.0, 9.0))
    fr = Frame(gpu, W, H)
    try:
        ref = [x.copy() for x in fr.render(W, H, flags=capi.RENDER_BRUTE_FORCE)]
        assert (ref[1] >= 0).sum() > 100_000
        fx = np.load(os.path.join(GOLDEN, "ns_spans.npz"))
        got = [x.copy() for x in fr.render(W, H)]  # the library's own launch choice
        for k, (y, x0, cols) in enumerate(fx["spans"].tolist()):
            for tag, fr_ in (("binned", got), ("brute force", ref)):
                assert np.array_equal(fr_[1][y, x0:x0 + cols], fx[f"face{k}"]), f"{tag} span {k} faces"
                assert_bit_equal(fr_[0][y, x0:x0 + cols], fx[f"rgb{k}"], f"{tag} span {k} ({y}, {x0}+{cols})")
        for flags in (capi.RENDER_DEFAULT, capi.RENDER_NO_DENSE_DETAIL, capi.RENDER_SHARED_DETAIL,
                      capi.RENDER_NO_DENSE_DETAIL | capi.RENDER_SHARED_DETAIL,
                      capi.RENDER_DENSE_DETAIL | capi.RENDER_SEPARATE_FILL):
            got = fr.render(W, H, flags=flags)
            assert np.array_equal(got[1], ref[1]), f"faces, flags {flags}"
            assert_bit_equal(got[0], ref[0], f"4k/70k binned vs brute force, flags {flags}")
            assert np.array_equal(got[2], ref[2]), f"ppm, flags {flags}"
        ring_rgb = gpu.empty((2, H, W, 3), np.float32)
        ring_ppm = gpu.empty((2, H, W, 3), np.uint8)
        try:
            gpu.memset(ring_rgb.ptr, 0, ring_rgb.nbytes)
            gpu.render_frames(2, W, H, out_rgb=ring_rgb.ptr, out_ppm=ring_ppm.ptr, ring=capi.frame_ring(2, H, W, 2))
            gpu.synchronize()
            rgb2, ppm2 = ring_rgb.numpy(), ring_ppm.numpy()
            for s in range(2):
                assert_bit_equal(rgb2[s], ref[0], f"frame {s} of two in flight")
                assert np.array_equal(ppm2[s], ref[2])
        finally:
            ring_rgb.free()
            ring_ppm.free()
        _bands_assemble(gpu, W, H, 4, ref)
        fr.render(W, H)  # the scene camera's whole frame: its setup's rectangles for the gather
        staging = gpu.to_device(_band_blocks(ref[2], H, W, 4, 4))
        out = gpu.empty((H, W, 3), np.uint8)
        try:
            assert capi.lib().eray_debug_scene_gather(gpu.handle, staging.ptr, out.ptr, H, W, 4, 4) == 0
            assert np.array_equal(out.numpy(), ref[2]), "scene-camera gather of the 4 bands"
        finally:
            staging.free()
            out.free()
    finally:
        fr.free()
        sc.close()


def _band_blocks(frame, H, W, band, world):
    """Each rank's padded local PPM rows (local file order) of a file-order frame in the band split."""
    cam = frame[::-1]
    rows_max = capi.band_rows(H, band, world, 0)
    blocks = np.zeros((world, rows_max, W, 3), np.uint8)
    for r in range(world):
        mine = [y for y in range(H) if (y // band) % world == r]
        blocks[r, :len(mine)] = cam[mine][::-1]
    return blocks


def test_c5_every_64th_row_block_equals_brute_force(gpu, synth1m):
    """C5 (1M faces, 7680x4320): every 64th 4-row block of the binned frame equals the GPU's
    brute-force scan of the same rows (~5e11 ray-triangle tests), where the culling margins are
    thinnest (tiny faces, 7680-pixel rows)."""
    W, H = 7680, 4320
    sc = MainScene(gpu, *synth1m, W, H, texture=1024, fov=(16.0, 9.0))
    fr = Frame(gpu, W, H)
    blk = Frame(gpu, W, 4)
    try:
        rgb, face, _ = [x.copy() for x in fr.render(W, H)]
        checked = 0
        for y0 in range(0, H, 64 * 4):
            b_rgb, b_face, _ = blk.render(W, H, row0=y0, rows=4, flags=capi.RENDER_BRUTE_FORCE)
            assert np.array_equal(b_face, face[y0:y0 + 4]), f"rows {y0}+4"
            assert_bit_equal(b_rgb, rgb[y0:y0 + 4], f"c5 rows {y0}+4")
            checked += int((b_face >= 0).sum())
        assert checked > 5_000
    finally:
        blk.free()
        fr.free()
        sc.close()


def _bin_entries(gpu, b, cap=1024):
    tri, mask, pad = (ctypes.c_uint32 * cap)(), (ctypes.c_uint64 * cap)(), (ctypes.c_uint32 * cap)()
    n = ctypes.c_uint32()
    assert capi.lib().eray_debug_bin_entries(gpu.handle, 0, b, tri, mask, pad, cap, ctypes.byref(n)) == 0
    m = min(n.value, cap)
    return (n.value, np.frombuffer(tri, np.uint32)[:m].copy(), np.frombuffer(mask, np.uint64)[:m].copy(),
            np.frombuffer(pad, np.uint32)[:m].copy())


def test_c5_sorted_bins_carry_later_chunk_masks(gpu, synth1m):
    """C5's bins (1M faces, 7680x4320) as render.hip first_hit_binned_wave relies on them
    (bins.hip bin_sort_kernel): every bin of 65..1024 entries lists its faces in increasing index —
    including those of more than 256 entries, sorted by a whole workgroup — and the first two
    entries of each chunk but the last hold the low and high half of the union of the masks of the
    later chunks; every other pad word is 0."""
    W, H = 7680, 4320
    sc = MainScene(gpu, *synth1m, W, H, texture=1024, fov=(16.0, 9.0))
    fr = Frame(gpu, W, H)
    try:
        fr.render(W, H)  # (the scene camera's full-frame setup: its bins)
        st = (ctypes.c_uint64 * 14)()
        assert capi.lib().eray_debug_bin_stats(gpu.handle, 0, st) == 0
        nbins = int(st[0])
        counts = np.zeros(nbins, np.uint32)
        nb = ctypes.c_uint32()
        assert capi.lib().eray_debug_bin_counts(gpu.handle, 0, counts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                                nbins, ctypes.byref(nb)) == 0
        heavy = np.nonzero(counts > 64)[0]
        assert len(heavy) > 1000 and counts.max() <= 1024
        big = np.nonzero(counts > 256)[0]
        assert len(big) > 0, "no bin for the workgroup sort"
        rng = np.random.default_rng(6)
        pick = np.concatenate([big, rng.choice(heavy, 200, replace=False), np.nonzero((counts > 0) & (counts <= 64))[0][:50]])
        for b in pick.tolist():
            n, tri, mask, pad = _bin_entries(gpu, b)
            assert n == counts[b]
            if n <= 64:
                assert not pad.any(), f"bin {b}: pads in an unsorted bin"
                continue
            assert (np.diff(tri.astype(np.int64)) > 0).all(), f"bin {b} ({n} entries) not in face order"
            nch = (n + 63) // 64
            want = np.zeros(n, np.uint32)
            for c in range(nch - 1):
                u = np.bitwise_or.reduce(mask[64 * (c + 1):])
                want[64 * c] = np.uint32(int(u) & 0xFFFFFFFF)
                want[64 * c + 1] = np.uint32(int(u) >> 32)
            assert np.array_equal(pad, want), f"bin {b} ({n} entries): later-chunk mask unions"
    finally:
        fr.free()
        sc.close()


def test_faces_grazing_the_view_leave_the_bins(gpu):
    """Hand-derived (primitives.rs:47-66: a hit needs det = -(d . n) >= 1e-6): 400 small faces
    tilted so that det lies between 0 and 1e-6 for every camera ray near them (n = e1 x e2 with
    e1 = (s, 0, 0), e2 = (0, s eps, -s): det ~ s^2 eps = 5e-7 at s = 0.01, eps = 0.005).  The
    culling records' det bound drops them — no bin entry, an empty object rectangle — and the
    frame is all background, as the brute-force scan finds; tilted 200x further the
    same faces are binned and hit (det ~ 1e-4: each face about a pixel tall), culled = brute force
    bit for bit."""
    W, H = 1920, 1080
    s = 0.01
    rng = np.random.default_rng(11)
    cx = rng.uniform(-0.5, 0.5, 400)
    cy = rng.uniform(-0.01, 0.01, 400)  # rays through them have |d.y| <~ 0.003: det stays in (0, 1e-6)
    results = {}
    for eps in (0.005, 1.0):
        pos = np.zeros((400, 9), np.float32)
        for i in range(400):
            a = np.array([cx[i], cy[i], 0.0])
            e1 = np.array([s, 0.0, 0.0])
            e2 = np.array([0.0, s * eps, -s])
            pos[i] = np.concatenate([a, a + e1, a + e2]).astype(np.float32)
        nrm = np.tile(np.array([0.0, 0.0, 1.0], np.float32), (400, 3))
        uv = rng.uniform(0.0, 1.0, (400, 6)).astype(np.float32)
        sc = MainScene(gpu, pos, nrm, uv, W, H, texture=64, fov=(16.0, 9.0))
        fr = Frame(gpu, W, H)
        try:
            a = [x.copy() for x in fr.render(W, H)]
            st = (ctypes.c_uint64 * 14)()
            assert capi.lib().eray_debug_bin_stats(gpu.handle, 0, st) == 0
            b = fr.render(W, H, flags=capi.RENDER_BRUTE_FORCE)
            assert np.array_equal(a[1], b[1]), f"faces, eps {eps}"
            assert_bit_equal(a[0], b[0], f"grazing faces, eps {eps}")
            assert np.array_equal(a[2], b[2])
            results[eps] = (int(st[1]), int((b[1] >= 0).sum()))
        finally:
            fr.free()
            sc.close()
    assert results[0.005] == (0, 0), results  # no entry, no hit
    assert results[1.0][0] > 100 and results[1.0][1] > 50, results


def test_faces_at_the_det_threshold_equal_brute_force(gpu):
    """Adversarial for the culling records' det bound: 4000 faces close to the camera (distance
    1.2-2) whose det along their centre ray is 0.6e-6..1.6e-6, so the reference's det >= 1e-6 test
    (primitives.rs:47-66) flips across their pixels.  With a = centre, e1 = s u, e2 = s (d + b w)
    (u, w perpendicular to the centre ray d): n = s^2 (b d - w) ... det = -(d . n) = -s^2 b.  The
    binned frame must equal the brute-force scan bit for bit, faces and all."""
    W, H = 1920, 1080
    rng = np.random.default_rng(12)
    nf = 4000
    C = np.array([0.0, 0.0, 5.0])
    pos = np.zeros((nf, 9), np.float32)
    for i in range(nf):
        dist = rng.uniform(1.2, 2.0)
        c = C + dist * np.array([rng.uniform(-0.8, 0.8), rng.uniform(-0.45, 0.45), -1.0]) / 1.0
        d = (c - C) / np.linalg.norm(c - C)
        u = np.cross(d, rng.normal(size=3))
        u /= np.linalg.norm(u)
        w = np.cross(d, u)
        s = rng.uniform(0.01, 0.04)
        det = rng.uniform(0.6e-6, 1.6e-6)
        e1 = s * u
        e2 = s * (d - (det / (s * s)) * w)
        pos[i] = np.concatenate([c, c + e1, c + e2]).astype(np.float32)
    nrm = rng.normal(size=(nf, 9)).astype(np.float32)
    uv = rng.uniform(0.0, 1.0, (nf, 6)).astype(np.float32)
    sc = MainScene(gpu, pos, nrm, uv, W, H, texture=64, fov=(16.0, 9.0))
    fr = Frame(gpu, W, H)
    try:
        a = [x.copy() for x in fr.render(W, H)]
        b = fr.render(W, H, flags=capi.RENDER_BRUTE_FORCE)
        assert np.array_equal(a[1], b[1]), "faces"
        assert_bit_equal(a[0], b[0], "faces at the det threshold: binned vs brute force")
        assert np.array_equal(a[2], b[2])
        assert (b[1] >= 0).sum() > 100  # (222 hit pixels of 215 such faces)
    finally:
        fr.free()
        sc.close()


def _corner_ray_point(W, H, ratio, x, y, t):
    """The point at parameter t along the (unnormalised) camera ray through pixel corner (x, y)
    of main.rs's camera (centre (0, 0, 5), z_dist 1, viewport 2*ratio x 2): camera.rs:57-76."""
    px = -ratio + 2.0 * ratio * x / W
    py = -1.0 + 2.0 * y / H
    return np.array([t * px, t * py, 5.0 - t], np.float64)


@pytest.mark.parametrize("faces", [200, 3000])
def test_culling_margins_on_pixel_corner_rays(gpu, faces):
    """Adversarial culling: triangles whose vertices lie on pixel-corner camera rays and whose
    edges pass through pixel corners (the exact rays the frame kernel traces, x/W and y/H), at
    W = 7680 where a pixel is 1/7680 of the viewport.  The culled frame (per-wave bounds for 200
    faces, screen bins for 3000) must equal the brute-force scan bit for bit."""
    W, H = 7680, 4320
    ratio = 16.0 / 9.0
    rng = np.random.default_rng(faces)
    pos = np.empty((faces, 9), np.float32)
    cx, cy = 3840, 2160  # around the frame centre (the degenerate bbox passes every camera ray)
    for i in range(faces):
        x0, y0 = cx + int(rng.integers(-300, 300)), cy + int(rng.integers(-160, 160))
        t = rng.uniform(4.0, 6.0, 3)
        if i % 2:  # a small triangle with all three vertices on pixel-corner rays
            pts = [_corner_ray_point(W, H, ratio, x0 + int(dx), y0 + int(dy), tt)
                   for (dx, dy), tt in zip([(0, 0), (int(rng.integers(1, 6)), 0), (0, int(rng.integers(1, 6)))], t)]
        else:  # an edge whose midpoint is on a pixel-corner ray: symmetric about that ray
            mid = _corner_ray_point(W, H, ratio, x0, y0, t[0])
            off = rng.normal(size=3) * 2e-3
            far = _corner_ray_point(W, H, ratio, x0 + int(rng.integers(-4, 5)), y0 + int(rng.integers(2, 6)), t[1])
            pts = [mid + off, mid - off, far]
        if rng.integers(2):
            pts = pts[::-1]  # both windings (backfaces are culled by the test)
        pos[i] = np.concatenate(pts).astype(np.float32)
    nrm = rng.normal(size=(faces, 9)).astype(np.float32)
    uv = rng.uniform(0.0, 1.0, (faces, 6)).astype(np.float32)
    rows, row0 = 336, 2160 - 168
    sc = MainScene(gpu, pos, nrm, uv, W, H, texture=64, fov=(16.0, 9.0))
    blk = Frame(gpu, W, rows)
    try:
        a = [x.copy() for x in blk.render(W, H, row0=row0, rows=rows)]
        b = blk.render(W, H, row0=row0, rows=rows, flags=capi.RENDER_BRUTE_FORCE)
        assert (b[1] >= 0).sum() > 100
        assert np.array_equal(a[1], b[1]), "faces"
        assert_bit_equal(a[0], b[0], "culled vs brute force on pixel-corner geometry")
        assert np.array_equal(a[2], b[2])
    finally:
        blk.free()
        sc.close()


def _all_bins(gpu):
    """Every bin of object 0 as built by the last setup: {bin: sorted [(face, mask)]}."""
    L = capi.lib()
    st = (ctypes.c_uint64 * 14)()
    assert L.eray_debug_bin_stats(gpu.handle, 0, st) == 0
    cap = 4096
    tri, mask, n = (ctypes.c_uint32 * cap)(), (ctypes.c_uint64 * cap)(), ctypes.c_uint32()
    out = {}
    for b in range(int(st[0])):
        assert L.eray_debug_bin_dump(gpu.handle, 0, b, tri, mask, cap, ctypes.byref(n)) == 0
        assert n.value <= cap
        if n.value:
            out[b] = sorted(zip(tri[: n.value], mask[: n.value]))
    return out, int(st[13])


def test_bin_segments_equal_rectangle_pairs(gpu):
    """The frame setups' pair pass over the faces' bin-rectangle rows (bins.hip
    bin_segments_kernel: per-row pixel ranges from bin_pixels' own double-precision lines) against
    the rectangle-pair form: every bin holds the same (face, pixel mask) entries — the segment form
    may add a few the pair form's f32 pre-test drops, never with another mask — at bin phase 0 and
    at phase 1 (a row tile from row 1), and the frames are bit-identical."""
    mesh = _mesh(**meshgen.STANDIN_70K)
    W, H = 1920, 1080
    sc = MainScene(gpu, *mesh, W, H, texture=1024, fov=(16.0, 9.0))
    fr = Frame(gpu, W, H)
    L = capi.lib()
    try:
        for row0 in (0, 1):
            got = []
            for rect in (1, 0):
                assert L.eray_debug_set_bin_form(gpu.handle, rect) == 0
                img = [x.copy() for x in fr.render(W, H, row0=row0)]
                bins, units = _all_bins(gpu)
                got.append((img, bins, units))
            (ia, ba, ua), (ib, bb, ub) = got
            assert np.array_equal(ia[1], ib[1]) and np.array_equal(ia[2], ib[2])
            assert_bit_equal(ia[0], ib[0], f"segments vs rectangle pairs, row0 {row0}")
            assert ub <= ua, (ub, ua)  # (rows of the rectangles, at most their bins)
            n_pairs = sum(len(v) for v in ba.values())
            assert n_pairs > 10_000
            extra = 0
            for b, seg in bb.items():
                pairs = dict(ba.get(b, []))
                seg_d = dict(seg)
                assert len(seg_d) == len(seg), f"bin {b}: a face twice"
                for f, m in pairs.items():
                    assert seg_d.get(f) == m, f"bin {b} face {f}: mask {seg_d.get(f)} vs {m} (row0 {row0})"
                extra += len(seg_d) - len(pairs)
            assert set(ba) <= set(bb)
            assert extra <= n_pairs // 20, (extra, n_pairs)
    finally:
        assert L.eray_debug_set_bin_form(gpu.handle, 0) == 0
        sc.close()
        fr.free()

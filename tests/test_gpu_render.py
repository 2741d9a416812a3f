"""GPU parity of the render path (eray_render through the C-ABI) against the CPU oracle.

Bar: bit-identical f32 RGB, identical first-hit face index per pixel, identical PPM bytes
(the kernels use the reference's exact f32 operation order).
"""
import os

import numpy as np
import pytest

from eray_amd import capi, meshgen
from eray_amd.frame import MainScene, fov_for
from tests.helpers import assert_bit_equal, mismatch_report, random_mesh

pytestmark = pytest.mark.gpu


def gpu_render(ctx, img_w, img_h, row0=0, rows=None, flags=0, ppm=True):
    rows = img_h - row0 if rows is None else rows
    rgb = ctx.empty((rows, img_w, 3), np.float32)
    face = ctx.empty((rows, img_w), np.int32)
    ctx.memset(rgb.ptr, 0, rgb.nbytes)
    ctx.memset(face.ptr, 0xFF, face.nbytes)
    out_ppm = ctx.empty((rows, img_w, 3), np.uint8) if ppm else None
    ctx.render(img_w, img_h, row0=row0, rows=rows, out_rgb=rgb.ptr, out_face=face.ptr,
               out_ppm=out_ppm.ptr if ppm else None, flags=flags)
    res = rgb.numpy(), face.numpy(), (out_ppm.numpy() if ppm else None)
    for a in (rgb, face, out_ppm):
        if a is not None:
            a.free()
    return res


def oracle_main_scene(oracle, mesh, W, H, texture=1024, rows=None, row0=0):
    s = oracle.main_rs_scene(*mesh, texture=texture)
    cam = oracle.camera((0.0, 0.0, 5.0), fov_for(W, H), W, 1.0)
    rgb, faces, stats = oracle.render(s, cam, row0=row0, rows=rows, want_faces=True)
    return rgb, faces, stats


@pytest.mark.parametrize("W,H", [(256, 256), (1920, 1080)])
def test_cube_frame_matches_oracle(gpu, oracle, cube, W, H):
    """C1 and C2: main.rs's scene, bit-exact frame, faces and PPM."""
    sc = MainScene(gpu, *cube, W, H)
    rgb, face, ppm = gpu_render(gpu, W, H)
    sc.close()
    ref, ref_face, stats = oracle_main_scene(oracle, cube, W, H)
    assert_bit_equal(rgb, ref, f"cube {W}x{H} rgb")
    assert np.array_equal(face, ref_face)
    body = oracle.ppm_bytes(ref)
    header = capi.ppm_header(W, H)
    assert body[: len(header)] == header
    assert ppm.tobytes() == body[len(header):]
    assert int((face >= 0).sum()) == stats["hit_pixels"]


def test_cube_centre_pixel_known_answer(gpu, cube):
    """pixel (W/2, H/2) hits face 1 and shades to ~(0.548175, 0.311178, 0.311178),
    bytes (139, 79, 79)."""
    sc = MainScene(gpu, *cube, 256, 256)
    rgb, face, ppm = gpu_render(gpu, 256, 256)
    sc.close()
    assert face[128, 128] == 1
    np.testing.assert_allclose(rgb[128, 128], [0.548175, 0.311178, 0.311178], atol=2e-6)
    assert tuple(ppm[255 - 128, 128]) == (139, 79, 79)


def test_brute_force_and_culled_agree_on_cube(gpu, cube):
    sc = MainScene(gpu, *cube, 1920, 1080)
    a = gpu_render(gpu, 1920, 1080)
    b = gpu_render(gpu, 1920, 1080, flags=capi.RENDER_BRUTE_FORCE)
    sc.close()
    assert_bit_equal(a[0], b[0], "culled vs brute force")
    assert np.array_equal(a[1], b[1])


@pytest.fixture(scope="module")
def sphere8k():
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(8000, 7)
    return (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(n[fn].reshape(-1, 9)),
            np.ascontiguousarray(t[ft].reshape(-1, 6)))


def test_displaced_sphere_matches_oracle(gpu, oracle, sphere8k):
    """A permuted non-convex mesh: first hits spread over the whole index range."""
    W, H = 256, 144
    sc = MainScene(gpu, *sphere8k, W, H, texture=256)
    rgb, face, ppm = gpu_render(gpu, W, H)
    rgb_b, face_b, _ = gpu_render(gpu, W, H, flags=capi.RENDER_BRUTE_FORCE)
    sc.close()
    ref, ref_face, stats = oracle_main_scene(oracle, sphere8k, W, H, texture=256)
    assert stats["hit_pixels"] > 300
    assert np.array_equal(face, ref_face)
    assert_bit_equal(rgb, ref, "sphere8k culled")
    assert_bit_equal(rgb_b, ref, "sphere8k brute force")


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_multi_object_scene(gpu, oracle, seed):
    """Several objects (general bounding boxes), coloured point/ambient lights, off-axis camera,
    random textures of different sizes: exercises closest-object selection, bbox gating and
    shadow rays that reach the triangle scan."""
    rng = np.random.default_rng(seed)
    W, H = 96, 64
    cam_center = tuple(rng.uniform(-0.7, 0.7, 3).astype(np.float32) + np.float32([0, 0, 4]))
    s = oracle.Scene()
    gpu.scene_reset()
    cam = capi.make_camera(cam_center, (3.0, 2.0), W, 1.0)
    gpu.set_camera(cam)
    keep = []
    for k in range(3):
        T = int(rng.integers(5, 300))
        pos, nrm, uv = random_mesh(rng, T, scale=float(rng.uniform(0.3, 1.2)),
                                   center=rng.uniform(-0.8, 0.8, 3))
        lo = pos.reshape(-1, 3).min(0) if k != 1 else np.zeros(3, np.float32)
        hi = pos.reshape(-1, 3).max(0) if k != 1 else np.zeros(3, np.float32)
        tw, th = int(rng.integers(1, 40)), int(rng.integers(1, 40))
        color = rng.uniform(0, 1.2, (th, tw, 3)).astype(np.float32)
        diffuse = rng.uniform(0, 1, (th + 1, tw + 2)).astype(np.float32) if k != 2 else None
        spec = rng.uniform(0, 1, (5, 7)).astype(np.float32) if k == 0 else None
        dc, dd = gpu.to_device(color), (gpu.to_device(diffuse) if diffuse is not None else None)
        ds = gpu.to_device(spec) if spec is not None else None
        keep += [x for x in (dc, dd, ds) if x is not None]
        gpu.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=dc.image(),
                       diffuse=dd.image() if dd else None, specular=ds.image() if ds else None)
        s.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=color, diffuse=diffuse, specular=spec)
    lights = [((0.0, 2.0, 0.0), "ambient", (0.9, 0.5, 1.0), 0.3),
              ((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0),
              ((-2.0, 0.5, 1.0), "point", (0.2, 0.9, 0.4), 0.7),
              ((0.0, -1.0, 0.5), "ambient", (1.0, 1.0, 1.0), 0.1)]
    for pos, var, col, b in lights:
        gpu.add_light(capi.make_light(pos, var, col, b))
        s.add_light(pos, var, col, b)
    rgb, face, _ = gpu_render(gpu, W, H)
    rgb_b, face_b, _ = gpu_render(gpu, W, H, flags=capi.RENDER_BRUTE_FORCE)
    ocam = oracle.camera(cam_center, (3.0, 2.0), W, 1.0)
    ref, ref_face, stats = oracle.render(s, ocam, want_faces=True)
    for a in keep:
        a.free()
    assert stats["shadow_tests"] > 0
    assert np.array_equal(face, ref_face)
    assert_bit_equal(rgb, ref, f"random scene {seed}")
    assert_bit_equal(rgb_b, ref, f"random scene {seed} brute")


def test_specular_power_textures_bit_exact(gpu, oracle):
    """A specular-power texture (engine.rs:164,171,174: powf not the identity): the frame kernel's
    restated glibc powf against the oracle's glibc powf, culled and brute force, bit for bit."""
    rng = np.random.default_rng(23)
    W, H = 128, 72
    gpu.scene_reset()
    cam_center = (0.05, -0.1, 3.5)
    gpu.set_camera(capi.make_camera(cam_center, (16.0, 9.0), W, 1.0))
    s = oracle.Scene()
    keep = []
    for k in range(2):
        pos, nrm, uv = random_mesh(rng, 200, scale=0.9, center=rng.uniform(-0.5, 0.5, 3))
        lo, hi = pos.reshape(-1, 3).min(0), pos.reshape(-1, 3).max(0)
        color = rng.uniform(0, 1, (6, 5, 3)).astype(np.float32)
        sp = rng.uniform(0.0, 40.0, (7, 9)).astype(np.float32)  # exponents 0 .. 40
        sp[0, :3] = [1.0, 0.5, 2.0]
        spec = rng.uniform(0, 1, (3, 3)).astype(np.float32)
        dc, dsp, ds = gpu.to_device(color), gpu.to_device(sp), gpu.to_device(spec)
        keep += [dc, dsp, ds]
        gpu.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=dc.image(), specular=ds.image(),
                       specular_power=dsp.image())
        s.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=color, specular=spec, specular_power=sp)
    for p, var, col, b in (((0.0, 2.0, 0.0), "ambient", (1.0, 1.0, 1.0), 0.2),
                           ((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0),
                           ((-1.5, 0.3, 1.5), "point", (0.6, 0.8, 1.0), 0.8)):
        gpu.add_light(capi.make_light(p, var, col, b))
        s.add_light(p, var, col, b)
    try:
        ref, ref_face, stats = oracle.render(s, oracle.camera(cam_center, (16.0, 9.0), W, 1.0), want_faces=True)
        assert stats["hit_pixels"] > 150
        for flags in (capi.RENDER_DEFAULT, capi.RENDER_BRUTE_FORCE):
            rgb, face, _ = gpu_render(gpu, W, H, flags=flags)
            assert np.array_equal(face, ref_face)
            assert_bit_equal(rgb, ref, f"specular power flags={flags}")
    finally:
        for a in keep:
            a.free()


def test_row_tiles_equal_full_frame(gpu, cube):
    W, H = 640, 360
    sc = MainScene(gpu, *cube, W, H)
    full_rgb, full_face, full_ppm = gpu_render(gpu, W, H)
    cuts = [0, 100, 101, 250, H]
    for a, b in zip(cuts[:-1], cuts[1:]):
        rgb, face, ppm = gpu_render(gpu, W, H, row0=a, rows=b - a)
        assert_bit_equal(rgb, full_rgb[a:b], f"rows {a}:{b}")
        assert np.array_equal(face, full_face[a:b])
        # PPM byte rows of a tile are the file rows H-b .. H-a-1
        assert np.array_equal(ppm, full_ppm[H - b:H - a])
    sc.close()


def test_engine_image_wider_than_camera(gpu, oracle, cube):
    """Image::set indexes with the engine image's width (image.rs:41-43)."""
    sc = MainScene(gpu, *cube, 128, 128)
    rgb, face, _ = gpu_render(gpu, 200, 150, rows=128, ppm=False)
    sc.close()
    s = oracle.main_rs_scene(*cube)
    ref, stats = oracle.render(s, oracle.camera(width=128), image_width=200, image_height=150)
    assert_bit_equal(rgb, ref, "stride")


def test_render_errors(gpu, cube):
    sc = MainScene(gpu, *cube, 64, 64)
    buf = gpu.empty((64, 64, 3), np.float32)
    with pytest.raises(capi.ErayError) as e:
        gpu.render(64, 64, row0=60, rows=10, out_rgb=buf.ptr)
    assert e.value.status == capi.E_INVALID_ARGUMENT
    with pytest.raises(capi.ErayError) as e:  # camera 64x64 does not fit a 64x32 engine image
        gpu.render(64, 32, rows=64, out_rgb=buf.ptr)
    assert e.value.status == capi.E_OUT_OF_BOUNDS
    buf.free()
    sc.close()


def test_empty_scene_and_empty_object(gpu, oracle):
    gpu.scene_reset()
    gpu.set_camera(capi.make_camera((0, 0, 5), (60, 60), 32, 1.0))
    gpu.add_light(capi.make_light((1, 1, 2), "point"))
    rgb, face, _ = gpu_render(gpu, 32, 32)
    assert np.all(face == -1)
    assert np.all(rgb == np.float32([0.1, 0.1, 0.2]))
    z = np.zeros((0, 9), np.float32)
    gpu.add_object(z, z, np.zeros((0, 6), np.float32))
    rgb2, face2, _ = gpu_render(gpu, 32, 32)
    assert_bit_equal(rgb2, rgb, "empty object")


def test_pack_ppm_matches_oracle(gpu, oracle):
    rng = np.random.default_rng(5)
    img = rng.uniform(-0.5, 1.5, (37, 53, 3)).astype(np.float32)
    img[0, 0] = [np.nan, np.inf, -np.inf]
    img[1, 1] = [1.0, 254.5 / 255.0, 0.0039215689]
    d = gpu.to_device(img)
    out = gpu.empty((37, 53, 3), np.uint8)
    gpu.pack_ppm(d.ptr, 53, 37, out.ptr)
    got = out.numpy().tobytes()
    d.free()
    out.free()
    ref = oracle.ppm_bytes(img)
    assert got == ref[len(capi.ppm_header(53, 37)):]


def test_many_objects_and_lights(gpu, oracle):
    """More objects and lights than travel inline in the kernel arguments."""
    rng = np.random.default_rng(11)
    W, H = 64, 48
    s = oracle.Scene()
    gpu.scene_reset()
    cam = capi.make_camera((0.1, -0.2, 4.5), (4.0, 3.0), W, 1.0)
    gpu.set_camera(cam)
    keep = []
    for k in range(6):
        pos, nrm, uv = random_mesh(rng, int(rng.integers(3, 40)), scale=0.6, center=rng.uniform(-1, 1, 3))
        color = rng.uniform(0, 1, (4, 4, 3)).astype(np.float32)
        dc = gpu.to_device(color)
        keep.append(dc)
        lo, hi = pos.reshape(-1, 3).min(0), pos.reshape(-1, 3).max(0)
        gpu.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=dc.image())
        s.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=color)
    for k in range(10):
        var = "ambient" if k % 3 == 0 else "point"
        p, c, b = tuple(rng.uniform(-2, 2, 3)), tuple(rng.uniform(0, 1, 3)), float(rng.uniform(0.1, 1))
        gpu.add_light(capi.make_light(p, var, c, b))
        s.add_light(p, var, c, b)
    rgb, face, _ = gpu_render(gpu, W, H)
    ref, ref_face, stats = oracle.render(s, oracle.camera((0.1, -0.2, 4.5), (4.0, 3.0), W, 1.0), want_faces=True)
    for a in keep:
        a.free()
    assert stats["hit_pixels"] > 0
    assert np.array_equal(face, ref_face)
    assert_bit_equal(rgb, ref, "many objects/lights")


def test_render_frames_graph_replay_matches_render(gpu, cube):
    """eray_render_frames replays a cached HIP graph (64 frames + plain launches for the rest);
    every replayed frame must be the frame eray_render writes, and a camera change must
    rebuild the plan (new culling records, new pixel rectangles)."""
    W, H = 320, 180
    sc = MainScene(gpu, *cube, W, H, texture=256, fov=(16.0, 9.0))
    ref = gpu_render(gpu, W, H)
    rgb = gpu.empty((H, W, 3), np.float32)
    ppm = gpu.empty((H, W, 3), np.uint8)
    face = gpu.empty((H, W), np.int32)
    try:
        for frames in (1, 70):
            gpu.memset(rgb.ptr, 0, rgb.nbytes)
            gpu.memset(face.ptr, 0x7F, face.nbytes)
            gpu.render_frames(frames, W, H, out_rgb=rgb.ptr, out_ppm=ppm.ptr, out_face=face.ptr,
                              prepare_only=True)
            ms = gpu.render_frames(frames, W, H, out_rgb=rgb.ptr, out_ppm=ppm.ptr, out_face=face.ptr,
                                   timed=True)
            assert ms > 0.0
            assert_bit_equal(rgb.numpy(), ref[0], f"render_frames({frames})")
            assert np.array_equal(face.numpy(), ref[1])
            assert np.array_equal(ppm.numpy(), ref[2])
        gpu.set_camera(capi.make_camera((0.4, -0.3, 4.0), (16.0, 9.0), W, 1.0))
        moved = gpu_render(gpu, W, H)
        assert not np.array_equal(moved[1], ref[1])
        gpu.memset(rgb.ptr, 0, rgb.nbytes)
        gpu.render_frames(70, W, H, out_rgb=rgb.ptr, out_ppm=ppm.ptr, out_face=face.ptr)
        gpu.synchronize()
        assert_bit_equal(rgb.numpy(), moved[0], "render_frames after a camera move")
        assert np.array_equal(face.numpy(), moved[1])
    finally:
        for a in (rgb, ppm, face):
            a.free()
        sc.close()


def test_every_pixel_written_and_rectangles_conservative(gpu, oracle):
    """Off-centre objects partly outside the frame, edge-sized images (not multiples of 16 / 4):
    the background fill and the detail sub-blocks must cover every pixel exactly as the oracle
    renders it, with culling on and off."""
    rng = np.random.default_rng(11)
    for W, H in ((101, 37), (64, 4), (17, 130)):
        s = oracle.Scene()
        gpu.scene_reset()
        cam = capi.make_camera((0.2, 0.1, 3.0), (float(W), float(H)), W, 1.0)
        gpu.set_camera(cam)
        keep = []
        for k in range(2):
            pos, nrm, uv = random_mesh(rng, 40, scale=0.8, center=rng.uniform(-1.5, 1.5, 3) * [1, 1, 0])
            color = rng.uniform(0, 1, (8, 8, 3)).astype(np.float32)
            dc = gpu.to_device(color)
            keep.append(dc)
            z = (0.0, 0.0, 0.0)
            gpu.add_object(pos, nrm, uv, z, z, color=dc.image())
            s.add_object(pos, nrm, uv, z, z, color=color)
        s.add_light((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0)
        gpu.add_light(capi.make_light((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0))
        if capi.camera_size(cam) != (W, H):
            continue
        ref, ref_face, _ = oracle.render(s, oracle.camera((0.2, 0.1, 3.0), (float(W), float(H)), W, 1.0),
                                         want_faces=True)
        for flags in (capi.RENDER_DEFAULT, capi.RENDER_BRUTE_FORCE):
            rgb, face, _ = gpu_render(gpu, W, H, flags=flags)
            assert np.array_equal(face, ref_face), (W, H, flags)
            assert_bit_equal(rgb, ref, f"{W}x{H} flags={flags}")
        for a in keep:
            a.free()


@pytest.fixture(scope="module")
def standin70k():
    """SURVEY.md §8(d) C3 mesh: the displaced-sphere stand-in, 69,451 faces, permuted (seed 42)."""
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(**meshgen.STANDIN_70K)
    return (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(n[fn].reshape(-1, 9)),
            np.ascontiguousarray(t[ft].reshape(-1, 6)))


DENSE = {"auto": 0, "0": capi.RENDER_NO_DENSE_DETAIL, "1": capi.RENDER_DENSE_DETAIL}
SEPARATE = {None: 0, "0": capi.RENDER_NO_SEPARATE_FILL, "1": capi.RENDER_SEPARATE_FILL}


@pytest.mark.parametrize("dense,separate", [("auto", None), ("0", None), ("1", "0"), ("1", "1")])
@pytest.mark.parametrize("material", ["textures", "example"])
def test_c3_binned_equals_brute_force(gpu, standin70k, material, dense, separate):
    """Screen bins (bins.hip) for a 70k-face object: bit-identical to the brute-force scan, with
    the large-mesh frame kernel at 2 and at 3 workgroups per CU (ERAY_RENDER_(NO_)DENSE_DETAIL)
    and the dense build with and without the separate fill kernel (ERAY_RENDER_(NO_)SEPARATE_FILL)."""
    flags = DENSE[dense] | SEPARATE[separate]
    W, H = 480, 270
    sc = MainScene(gpu, *standin70k, W, H, texture=256, fov=(16.0, 9.0), material=material)
    a = gpu_render(gpu, W, H, flags=flags)
    b = gpu_render(gpu, W, H, flags=capi.RENDER_BRUTE_FORCE)
    sc.close()
    assert (a[1] >= 0).sum() > 1000
    assert np.array_equal(a[1], b[1])
    assert_bit_equal(a[0], b[0], "c3 binned vs brute force")
    assert np.array_equal(a[2], b[2])


@pytest.mark.parametrize("separate", ["0", "1"])
def test_dense_frames_graph_replay(gpu, standin70k, separate):
    """The dense large-mesh build replayed from a HIP graph, with the fill in the same launch and
    as a second kernel on a forked stream (two parallel graph nodes joined by an event): every
    replayed frame equals eray_render's brute-force frame.  The flags are part of the launch-plan
    key, so each setting captures its own graph."""
    flags = capi.RENDER_DENSE_DETAIL | SEPARATE[separate]
    W, H = 480, 270
    sc = MainScene(gpu, *standin70k, W, H, texture=256, fov=(16.0, 9.0))
    ref = gpu_render(gpu, W, H, flags=capi.RENDER_BRUTE_FORCE)
    rgb = gpu.empty((H, W, 3), np.float32)
    ppm = gpu.empty((H, W, 3), np.uint8)
    face = gpu.empty((H, W), np.int32)
    try:
        for frames in (1, 9):
            gpu.memset(rgb.ptr, 0, rgb.nbytes)
            gpu.memset(ppm.ptr, 0, ppm.nbytes)
            gpu.memset(face.ptr, 0x7F, face.nbytes)
            gpu.render_frames(frames, W, H, out_rgb=rgb.ptr, out_ppm=ppm.ptr, out_face=face.ptr, flags=flags)
            gpu.synchronize()
            assert_bit_equal(rgb.numpy(), ref[0], f"dense render_frames({frames}) separate={separate}")
            assert np.array_equal(face.numpy(), ref[1])
            assert np.array_equal(ppm.numpy(), ref[2])
    finally:
        for a in (rgb, ppm, face):
            a.free()
        sc.close()


@pytest.mark.parametrize("dense,separate", [("0", "0"), ("1", "0"), ("1", "1")])
def test_c3_full_size_rows_match_oracle(gpu, oracle, standin70k, dense, separate):
    """C3 at 1920x1080 (bins built for the full camera) against the oracle on a row sample
    through the object, including row blocks rendered with a row phase (row0 % 4 != 0); the
    large-mesh kernel at 2 and at 3 workgroups per CU, the latter also beside the separate fill
    kernel."""
    flags = DENSE[dense] | SEPARATE[separate]
    W, H = 1920, 1080
    sc = MainScene(gpu, *standin70k, W, H, texture=256, fov=(16.0, 9.0))
    rgb, face, _ = gpu_render(gpu, W, H, flags=flags)
    osc = oracle.main_rs_scene(*standin70k, texture=256)
    ocam = oracle.camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0)
    for row0, rows in ((538, 3), (601, 2)):
        ref, ref_face, _ = oracle.render(osc, ocam, row0=row0, rows=rows, want_faces=True)
        assert np.array_equal(face[row0:row0 + rows], ref_face)
        assert_bit_equal(rgb[row0:row0 + rows], ref, f"c3 rows {row0}+{rows}")
        part, part_face, _ = gpu_render(gpu, W, H, row0=row0, rows=rows, flags=flags)
        assert np.array_equal(part_face, ref_face)
        assert_bit_equal(part, ref, f"c3 row block {row0}+{rows}")
    sc.close()


def test_binned_and_small_objects_row_tiles(gpu, oracle, cube):
    """A binned object (8k faces, general bounding box) beside small ones (the cube, a random
    mesh), rendered whole and in row tiles of every row phase: the detail sub-block list (non-empty
    bins + the small objects' rectangles) and its occupancy bitmap for the fill must give the
    brute-force frame bit for bit, and the oracle's on the tiles."""
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(8000, 3)
    big = (np.ascontiguousarray(v[fv].reshape(-1, 9)) * np.float32(0.6) + np.float32([-0.9, 0.3, 0.0] * 3),
           np.ascontiguousarray(n[fn].reshape(-1, 9)), np.ascontiguousarray(t[ft].reshape(-1, 6)))
    rng = np.random.default_rng(5)
    small = random_mesh(rng, 40, scale=0.3, center=(0.9, -0.4, 0.5))
    W, H = 320, 180
    cam_center = (0.1, -0.05, 4.0)
    gpu.scene_reset()
    gpu.set_camera(capi.make_camera(cam_center, (16.0, 9.0), W, 1.0))
    s = oracle.Scene()
    tex = rng.uniform(0, 1, (16, 16, 3)).astype(np.float32)
    dt = gpu.to_device(tex)
    cube_s = (cube[0] * np.float32(0.4) + np.float32([0.8, 0.5, -0.5] * 3), cube[1], cube[2])
    for pos, nrm, uv in (big, cube_s, small):
        lo, hi = pos.reshape(-1, 3).min(0), pos.reshape(-1, 3).max(0)
        gpu.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=dt.image())
        s.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=tex)
    for p, var, col, b in (((0.0, 2.0, 0.0), "ambient", (1.0, 1.0, 1.0), 0.2),
                           ((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0)):
        gpu.add_light(capi.make_light(p, var, col, b))
        s.add_light(p, var, col, b)
    full, full_face, _ = gpu_render(gpu, W, H)
    brute, brute_face, _ = gpu_render(gpu, W, H, flags=capi.RENDER_BRUTE_FORCE)
    assert (full_face >= 0).sum() > 800
    assert np.array_equal(full_face, brute_face)
    assert_bit_equal(full, brute, "binned + small vs brute force")
    ocam = oracle.camera(cam_center, (16.0, 9.0), W, 1.0)
    for row0, rows in ((0, 45), (45, 46), (91, 43), (134, 46), (61, 7)):
        part, part_face, _ = gpu_render(gpu, W, H, row0=row0, rows=rows, ppm=False)
        assert np.array_equal(part_face, full_face[row0:row0 + rows])
        assert_bit_equal(part, full[row0:row0 + rows], f"tile {row0}+{rows}")
    ref, ref_face, _ = oracle.render(s, ocam, row0=85, rows=12, want_faces=True)
    assert np.array_equal(full_face[85:97], ref_face)
    assert_bit_equal(full[85:97], ref, "binned + small vs oracle")
    dt.free()


def test_example_material_errors(gpu, cube):
    sc = MainScene(gpu, *cube, 64, 64, texture=16)
    with pytest.raises(capi.ErayError) as e:
        gpu.set_object_example_material(5, 16, 16, 1.0, 1.0, 1.0, 0.0, 0.0, 0.5)
    assert e.value.status == capi.E_INVALID_ARGUMENT
    with pytest.raises(capi.ErayError) as e:
        gpu.set_object_example_material(0, 0, 16, 1.0, 1.0, 1.0, 0.0, 0.0, 0.5)
    assert e.value.status == capi.E_OUT_OF_BOUNDS
    sc.close()

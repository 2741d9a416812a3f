"""GPU parity of the general tracer (trace.hip): Engine::render with anti-aliasing and reflection
bounces (engine.rs:59-77, 181-191) through the C-ABI, against the CPU oracle.

Bar: bit-identical f32 RGB, PPM bytes and first-ray faces.  The reference's anti-aliasing draws
from the OS-seeded rand::thread_rng, which no two runs reproduce; both sides here draw the same
Philox4x32-10 stream (key = aa_seed, counter = (x, y, sample, 0)) mapped to [-1, 1) as rand
0.8's gen_range does, so the comparison is exact.
"""
import numpy as np
import pytest

from eray_amd import capi
from eray_amd.frame import MainScene, fov_for
from tests.helpers import assert_bit_equal, random_mesh

pytestmark = pytest.mark.gpu


def gpu_trace(ctx, W, H, bounces=0, aa=0, seed=0, row0=0, rows=None, ppm=True):
    rows = H - row0 if rows is None else rows
    rgb = ctx.empty((rows, W, 3), np.float32)
    face = ctx.empty((rows, W), np.int32)
    out_ppm = ctx.empty((rows, W, 3), np.uint8) if ppm else None
    ctx.memset(rgb.ptr, 0, rgb.nbytes)
    ctx.render(W, H, row0=row0, rows=rows, out_rgb=rgb.ptr, out_face=face.ptr,
               out_ppm=out_ppm.ptr if ppm else None, bounces=bounces, anti_aliasing=aa, aa_seed=seed)
    res = rgb.numpy(), face.numpy(), (out_ppm.numpy() if ppm else None)
    for a in (rgb, face, out_ppm):
        if a is not None:
            a.free()
    return res


@pytest.mark.parametrize("aa,seed", [(1, 0), (2, 7), (4, 0x123456789ABCDEF)])
def test_cube_anti_aliasing_matches_oracle(gpu, oracle, cube, aa, seed):
    """main.rs's scene with Engine::new(.., 0, aa): jittered rays, (sum / aa).clamp()."""
    W, H = 128, 72
    sc = MainScene(gpu, *cube, W, H, texture=256)
    rgb, face, ppm = gpu_trace(gpu, W, H, aa=aa, seed=seed)
    sc.close()
    s = oracle.main_rs_scene(*cube, texture=256)
    ref, ref_face, _ = oracle.render(s, oracle.camera((0.0, 0.0, 5.0), fov_for(W, H), W, 1.0),
                                     want_faces=True, anti_aliasing=aa, seed=seed)
    assert_bit_equal(rgb, ref, f"aa={aa}")
    assert np.array_equal(face, ref_face)
    assert ppm.tobytes() == oracle.ppm_bytes(ref)[len(capi.ppm_header(W, H)):]
    assert float(ref.max()) <= 1.0 and float(ref.min()) >= 0.0  # clamped


def test_anti_aliasing_seed_changes_the_jitter(gpu, cube):
    W, H = 64, 64
    sc = MainScene(gpu, *cube, W, H, texture=256)
    a = gpu_trace(gpu, W, H, aa=2, seed=1)[0]
    b = gpu_trace(gpu, W, H, aa=2, seed=1)[0]
    c = gpu_trace(gpu, W, H, aa=2, seed=2)[0]
    sc.close()
    assert_bit_equal(a, b, "same seed")
    assert not np.array_equal(a, c)


def test_anti_aliasing_row_tiles(gpu, oracle, cube):
    """Row tiles (multi-GPU split) draw the same jitter: the counter is the camera pixel."""
    W, H = 96, 54
    sc = MainScene(gpu, *cube, W, H, texture=128)
    full = gpu_trace(gpu, W, H, aa=3, seed=5, ppm=False)[0]
    part = gpu_trace(gpu, W, H, aa=3, seed=5, row0=20, rows=17, ppm=False)[0]
    sc.close()
    assert_bit_equal(part, full[20:37], "row tile")


def reflective_scene(gpu, oracle, rng, W, H, with_refl=True):
    """Three objects with general bounding boxes (the reflected rays reach each other), random
    colour / diffuse / reflection textures (reflection 0 on part of every texture), coloured point
    and ambient lights, an off-axis camera."""
    cam_center = tuple(rng.uniform(-0.5, 0.5, 3).astype(np.float32) + np.float32([0, 0, 4]))
    s = oracle.Scene()
    gpu.scene_reset()
    gpu.set_camera(capi.make_camera(cam_center, (3.0, 2.0), W, 1.0))
    keep = []
    for k in range(3):
        T = int(rng.integers(4, 120))
        pos, nrm, uv = random_mesh(rng, T, scale=float(rng.uniform(0.4, 1.1)), center=rng.uniform(-0.7, 0.7, 3))
        lo, hi = pos.reshape(-1, 3).min(0), pos.reshape(-1, 3).max(0)
        tw, th = int(rng.integers(2, 30)), int(rng.integers(2, 30))
        color = rng.uniform(0, 1.2, (th, tw, 3)).astype(np.float32)
        diffuse = rng.uniform(0, 1, (th, tw)).astype(np.float32)
        refl = None
        if with_refl:
            refl = rng.uniform(0, 0.9, (7, 5)).astype(np.float32)
            refl[rng.uniform(size=refl.shape) < 0.3] = 0.0
        dev = [gpu.to_device(a) for a in (color, diffuse) + ((refl,) if refl is not None else ())]
        keep += dev
        gpu.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=dev[0].image(), diffuse=dev[1].image(),
                       reflection=dev[2].image() if refl is not None else None)
        s.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=color, diffuse=diffuse, reflection=refl)
    lights = [((0.0, 2.0, 0.0), "ambient", (0.9, 0.5, 1.0), 0.3),
              ((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0),
              ((-2.0, 0.5, 1.0), "point", (0.2, 0.9, 0.4), 0.7)]
    for p, var, col, b in lights:
        gpu.add_light(capi.make_light(p, var, col, b))
        s.add_light(p, var, col, b)
    return s, oracle.camera(cam_center, (3.0, 2.0), W, 1.0), keep


@pytest.mark.parametrize("seed,bounces", [(11, 1), (12, 2), (13, 3)])
def test_reflection_bounces_match_oracle(gpu, oracle, seed, bounces):
    """engine.rs:181-191: one reflected ray per point light and level, its lighting list
    flattened into the parent's times the reflection factor; the pixel is the left fold."""
    rng = np.random.default_rng(seed)
    W, H = 72, 48
    s, cam, keep = reflective_scene(gpu, oracle, rng, W, H)
    rgb, face, _ = gpu_trace(gpu, W, H, bounces=bounces, ppm=False)
    flat, _, _ = gpu_trace(gpu, W, H, bounces=0, ppm=False)
    for a in keep:
        a.free()
    ref, ref_face, _ = oracle.render(s, cam, want_faces=True, bounces=bounces)
    ref0, _ = oracle.render(s, cam, bounces=0)
    assert_bit_equal(rgb, ref, f"bounces={bounces}")
    assert np.array_equal(face, ref_face)
    assert_bit_equal(flat, ref0, "bounces=0 (frame kernel)")
    assert not np.array_equal(ref, ref0)  # the reflections do change the image


def test_bounces_and_anti_aliasing_together(gpu, oracle):
    rng = np.random.default_rng(21)
    W, H = 48, 32
    s, cam, keep = reflective_scene(gpu, oracle, rng, W, H)
    rgb, face, _ = gpu_trace(gpu, W, H, bounces=2, aa=2, seed=99, ppm=False)
    for a in keep:
        a.free()
    ref, ref_face, _ = oracle.render(s, cam, want_faces=True, bounces=2, anti_aliasing=2, seed=99)
    assert_bit_equal(rgb, ref, "bounces=2, aa=2")
    assert np.array_equal(face, ref_face)


def test_bounces_without_reflection_output_take_the_frame_kernel(gpu, oracle):
    """No material has a reflection output: bounces change nothing (reflection defaults to 0)."""
    rng = np.random.default_rng(31)
    W, H = 60, 40
    s, cam, keep = reflective_scene(gpu, oracle, rng, W, H, with_refl=False)
    a = gpu_trace(gpu, W, H, bounces=5, ppm=False)[0]
    for x in keep:
        x.free()
    ref, _ = oracle.render(s, cam, bounces=5)
    assert_bit_equal(a, ref, "bounces=5 without reflection")


def test_too_many_bounces_is_reported(gpu, oracle):
    rng = np.random.default_rng(41)
    s, cam, keep = reflective_scene(gpu, oracle, rng, 16, 16)
    out = gpu.empty((10, 16, 3), np.float32)
    with pytest.raises(capi.ErayError) as e:
        gpu.render(16, 10, out_rgb=out.ptr, bounces=17)
    assert e.value.status == capi.E_UNSUPPORTED
    gpu.render(16, 10, out_rgb=out.ptr, bounces=16, rows=1)  # the deepest supported walk
    out.free()
    for x in keep:
        x.free()


@pytest.mark.parametrize("seed,n_tris", [(51, 40), (52, 120), (53, 300)])
def test_background_skip_is_exact(gpu, oracle, seed, n_tris):
    """trace_kernel's background skip (waves no jittered camera ray of which can reach a face,
    from the culling records) against the brute-force scan (ERAY_RENDER_BRUTE_FORCE) and the
    oracle: small objects near the frame's corners and edges, so many waves sit next to a face
    within a jitter's reach.  300 faces exceed the skip's LDS table (plain scan)."""
    rng = np.random.default_rng(seed)
    W, H = 144, 96  # (Camera::size of fov 3 x 2)
    cam_center = (0.05, -0.03, 4.0)
    s = oracle.Scene()
    gpu.scene_reset()
    gpu.set_camera(capi.make_camera(cam_center, (3.0, 2.0), W, 1.0))
    keep = []
    for k, c in enumerate([(-1.35, 0.85, 0.3), (1.3, -0.9, 0.0), (0.0, 0.0, -0.5)]):
        T = n_tris // 3 + (n_tris % 3 if k == 0 else 0)
        pos, nrm, uv = random_mesh(rng, T, scale=0.12 + 0.05 * k, center=c)
        lo, hi = pos.reshape(-1, 3).min(0), pos.reshape(-1, 3).max(0)
        color = rng.uniform(0, 1.2, (5, 7, 3)).astype(np.float32)
        refl = rng.uniform(0, 0.9, (3, 4)).astype(np.float32)
        dev = [gpu.to_device(a) for a in (color, refl)]
        keep += dev
        gpu.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=dev[0].image(), reflection=dev[1].image())
        s.add_object(pos, nrm, uv, tuple(lo), tuple(hi), color=color, reflection=refl)
    for p, var, col, b in [((0.0, 2.0, 0.0), "ambient", (0.9, 0.5, 1.0), 0.3),
                           ((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0)]:
        gpu.add_light(capi.make_light(p, var, col, b))
        s.add_light(p, var, col, b)
    outs = []
    for flags in (capi.RENDER_DEFAULT, capi.RENDER_BRUTE_FORCE):
        rgb = gpu.empty((H, W, 3), np.float32)
        face = gpu.empty((H, W), np.int32)
        gpu.render(W, H, out_rgb=rgb.ptr, out_face=face.ptr, anti_aliasing=3, bounces=1, aa_seed=seed,
                   flags=flags)
        outs.append((rgb.numpy(), face.numpy()))
        rgb.free()
        face.free()
    for a in keep:
        a.free()
    (rgb, face), (brute, brute_face) = outs
    assert_bit_equal(rgb, brute, "skip vs brute force")
    assert np.array_equal(face, brute_face)
    ref, ref_face, _ = oracle.render(s, oracle.camera(cam_center, (3.0, 2.0), W, 1.0), want_faces=True,
                                     bounces=1, anti_aliasing=3, seed=seed)
    assert_bit_equal(rgb, ref, "aa=3, bounces=1")
    assert np.array_equal(face, ref_face)
    hit = face >= 0
    assert 0 < hit.sum() < hit.size // 4  # small objects: most waves are background

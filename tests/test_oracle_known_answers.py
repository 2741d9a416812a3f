"""Pins the CPU oracle against every known answer the reference's own tests hold for this
path, plus the answers SURVEY.md §8(c) derives (the oracle is the checker of all GPU tests)."""
import numpy as np
import pytest


def test_vector_dot_product(oracle):
    # vector.rs:259-270: (1,2,-3).(-1.5,2.3,0.1) == 2.8 (abs <= 1e-4)
    assert abs(oracle.vec_dot((1, 2, -3), (-1.5, 2.3, 0.1)) - 2.8) <= 1e-4


def test_vector_cross_product(oracle):
    # vector.rs:272-284: cross == (7.1, 4.4, 5.3), |got - expected|^2 < 1e-4
    got = oracle.vec_cross((1, 2, -3), (-1.5, 2.3, 0.1))
    assert float(((got - np.float32([7.1, 4.4, 5.3])) ** 2).sum()) < 1e-4


def test_vector_angle(oracle):
    # vector.rs:286-299: angle == 1.2949 (abs <= 1e-4)
    assert abs(oracle.vec_angle((1, 2, -3), (-1.5, 2.3, 0.1)) - 1.2949) <= 1e-4


def test_triangle_projection(oracle):
    # primitives.rs:88-112: exact equality
    got = oracle.triangle_project([-0.5, 0, -0.5, 0, 0, 0.5, 0.5, 0, -0.5], [0.2, 0.1, 0.0])
    assert got.tolist() == [np.float32(0.2), 0.0, 0.0]


def test_mod_get(oracle):
    # image.rs:201-213: mod_get(123, 12) on a 10x10 image == pixels[2*10+3]; the oracle's
    # mix node with factor 0 returns left.mod_get(x, y)
    left = np.zeros((10, 10, 3), np.float32)
    left[..., 0] = np.arange(100, dtype=np.float32).reshape(10, 10)
    out = oracle.node_mix_color(124, 13, left, np.zeros((1, 1, 3), np.float32), 0.0)
    assert out[12, 123, 0] == 23.0


def test_camera_size(oracle):
    # Fov(16,9) gives 1080/2160/4320 for 1920/3840/7680; Fov(106.66667,60) -> 1079
    for w, h in ((1920, 1080), (3840, 2160), (7680, 4320)):
        assert oracle.camera_size(oracle.camera(fov=(16.0, 9.0), width=w)) == (w, h)
    assert oracle.camera_size(oracle.camera(fov=(106.66667, 60.0), width=1920)) == (1920, 1079)
    assert oracle.camera_size(oracle.camera(width=256)) == (256, 256)


def test_centre_ray_is_minus_z(oracle):
    s, d = oracle.pixel_to_ray(oracle.camera(width=256), 0.5, 0.5)
    assert s.tolist() == [0.0, 0.0, 5.0] and d.tolist() == [0.0, 0.0, -1.0]


def test_centre_pixel_and_counts(oracle, cube):
    """face 1 at the centre, RGB ~ (0.548175, 0.311178,
    0.311178) -> bytes (139, 79, 79); 4,223 hit pixels at 256x256; 73,166 hit pixels and
    24,371,440 primary triangle tests at 1920x1080."""
    s = oracle.main_rs_scene(*cube)
    rgb, faces, st = oracle.render(s, oracle.camera(width=256), want_faces=True)
    assert faces[128, 128] == 1
    np.testing.assert_allclose(rgb[128, 128], [0.548175, 0.311178, 0.311178], atol=2e-6)
    assert tuple((rgb[128, 128] * np.float32(255)).astype(np.uint8)) == (139, 79, 79)
    assert st["hit_pixels"] == 4223
    rgb2, st2 = oracle.render(s, oracle.camera(fov=(16.0, 9.0), width=1920))
    assert st2["hit_pixels"] == 73166
    assert st2["primary_tests"] == 24371440


def test_texel_zero(oracle):
    # wave(0, 0) = |cos 0| = 1 -> mix((1,1,1), (1,0,0), 0.5) = (1, 0.5, 0.5) -> bytes (255,127,127)
    color, diffuse = oracle.example_material(8, 8)
    assert tuple(color[0, 0]) == (1.0, 0.5, 0.5) and diffuse[0, 0] == 1.0
    body = oracle.ppm_bytes(color)
    # texel (0,0) is in the LAST written row (rows are written bottom-up)
    assert body[-8 * 3:-8 * 3 + 3] == bytes([255, 127, 127])


def test_triangle_intersects_edge_semantics(oracle):
    # the centre ray hits face 1 of the cube exactly on the shared diagonal: u = 0.5, v = -0
    pos = [1, 1, 1, -1, -1, 1, 1, -1, 1]
    nrm = [0, 0, 1] * 3
    hit = oracle.triangle_intersects(pos, nrm, (0, 0, 5), (0, 0, -1))
    assert hit is not None
    p, n, b = hit
    assert p.tolist() == [0.0, 0.0, 1.0] and n.tolist() == [0.0, 0.0, 1.0]
    assert b[0] == 0.5 and b[1] == 0.0 and np.signbit(b[1])
    # backface: same triangle seen from behind
    assert oracle.triangle_intersects(pos, nrm, (0, 0, -5), (0, 0, 1)) is None


def test_philox_known_answers(oracle):
    """The anti-aliasing jitter stream: Philox4x32-10 against Random123's kat_vectors."""
    assert oracle.philox4x32_10([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert oracle.philox4x32_10([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6,
                                                                       0x6D5451FD]
    assert oracle.philox4x32_10([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]) == [
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_jitter_is_rand_gen_range(oracle):
    """rand 0.8 gen_range(-1.0..1.0) for f32: (word >> 9) as the mantissa of [1, 2), minus 1,
    times 2, minus 1 — the 2^23 outcomes are exactly -1 + k * 2^-22."""
    assert oracle.jitter(0) == -1.0
    assert oracle.jitter(0x1FF) == -1.0  # the low 9 bits are discarded
    assert oracle.jitter(0x200) == -1.0 + 2.0 ** -22
    assert oracle.jitter(0x80000000) == 0.0
    assert oracle.jitter(0xFFFFFFFF) == 1.0 - 2.0 ** -22


def test_anti_aliasing_zero_is_the_plain_render(oracle, cube):
    s = oracle.main_rs_scene(*cube, texture=64)
    cam = oracle.camera(width=24)
    a, _ = oracle.render(s, cam)
    b, _ = oracle.render(s, cam, anti_aliasing=0, seed=1234)
    c, _ = oracle.render(s, cam, anti_aliasing=1, seed=1234)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert not np.array_equal(a, c) and c.max() <= 1.0

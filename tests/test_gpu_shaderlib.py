"""GPU parity of the shaderlib node operators (src/shaderlib/*.rs) against the CPU oracle:
bit-identical images (the wave node's cosf is glibc's algorithm restated)."""
import numpy as np
import pytest

from eray_amd import capi
from tests.helpers import assert_bit_equal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("w,h,xf,yf", [(1024, 1024, 1.0, 1.0), (37, 19, 0.7, -1.3),
                                       (5, 300, 123.25, 0.001), (1, 1, 1.0, 1.0)])
def test_wave(gpu, oracle, w, h, xf, yf):
    out = gpu.empty((h, w), np.float32)
    gpu.node_wave(w, h, xf, yf, out.ptr)
    got = out.numpy()
    out.free()
    assert_bit_equal(got, oracle.node_wave(w, h, xf, yf), f"wave {w}x{h}")


def test_wave_huge_arguments(gpu, oracle):
    """x_fac large enough to take glibc's large-argument reduction path (|x| >= 120)."""
    out = gpu.empty((64, 64), np.float32)
    gpu.node_wave(64, 64, 1.0e6, -3.5e4, out.ptr)
    got = out.numpy()
    out.free()
    assert_bit_equal(got, oracle.node_wave(64, 64, 1.0e6, -3.5e4), "wave large")


def test_rgb_flat_mix(gpu, oracle):
    rng = np.random.default_rng(3)
    w, h = 33, 21
    r = rng.random((h, w), np.float32)
    g = rng.random((h + 2, w), np.float32)       # larger inputs are indexed with the output index
    b = rng.random((h, w + 5), np.float32)
    dr, dg, db = gpu.to_device(r), gpu.to_device(g), gpu.to_device(b)
    out = gpu.empty((h, w, 3), np.float32)
    gpu.node_rgb(w, h, dr.image(), dg.image(), db.image(), out.ptr)
    assert_bit_equal(out.numpy(), oracle.node_rgb(w, h, r, g, b), "rgb")

    flat = gpu.empty((h, w, 3), np.float32)
    gpu.node_flat_color(w, h, 0.25, -1.0, 3.5, flat.ptr)
    assert_bit_equal(flat.numpy(), oracle.node_flat_color(w, h, 0.25, -1.0, 3.5), "flat")

    left = rng.random((7, 11, 3), np.float32)     # mod_get wraps the smaller inputs
    right = rng.random((40, 3, 3), np.float32)
    dl, drr = gpu.to_device(left), gpu.to_device(right)
    mix = gpu.empty((h, w, 3), np.float32)
    gpu.node_mix_color(w, h, dl.image(), drr.image(), 0.3, mix.ptr)
    assert_bit_equal(mix.numpy(), oracle.node_mix_color(w, h, left, right, 0.3), "mix")
    for a in (dr, dg, db, out, flat, dl, drr, mix):
        a.free()


def test_mod_get_known_answer(gpu):
    """image.rs:201-213: on a 10x10 image, mod_get(123, 12) == pixels[2*10+3] — here through the
    mix node (factor 0 returns left.mod_get(x, y) exactly)."""
    left = np.zeros((10, 10, 3), np.float32)
    left[..., 0] = np.arange(100, dtype=np.float32).reshape(10, 10)
    right = np.zeros((1, 1, 3), np.float32)
    dl, dr = gpu.to_device(left), gpu.to_device(right)
    out = gpu.empty((13, 124, 3), np.float32)
    gpu.node_mix_color(124, 13, dl.image(), dr.image(), 0.0, out.ptr)
    got = out.numpy()
    for a in (dl, dr, out):
        a.free()
    assert got[12, 123, 0] == 23.0


def test_example_material(gpu, oracle):
    for w, h in [(1024, 1024), (129, 65)]:
        color = gpu.empty((h, w, 3), np.float32)
        diffuse = gpu.empty((h, w), np.float32)
        gpu.material_example(w, h, 1.0, 1.0, 1.0, 0.0, 0.0, 0.5, color.ptr, diffuse.ptr)
        c_ref, d_ref = oracle.example_material(w, h)
        assert_bit_equal(color.numpy(), c_ref, f"color {w}x{h}")
        assert_bit_equal(diffuse.numpy(), d_ref, f"diffuse {w}x{h}")
        color.free()
        diffuse.free()
    # texel (0, 0): w = |cos 0| = 1 -> colour (1, 0.5, 0.5)
    assert tuple(c_ref[0, 0]) == (1.0, 0.5, 0.5)


def test_node_errors(gpu):
    small = gpu.empty((2, 2), np.float32)
    out = gpu.empty((4, 4, 3), np.float32)
    with pytest.raises(capi.ErayError) as e:
        gpu.node_rgb(4, 4, small.image(), small.image(), small.image(), out.ptr)
    assert e.value.status == capi.E_OUT_OF_BOUNDS
    with pytest.raises(capi.ErayError) as e:
        gpu.node_mix_color(4, 4, capi.Image(None, 0, 0), small.image(), 0.5, out.ptr)
    assert e.value.status == capi.E_MISSING
    small.free()
    out.free()

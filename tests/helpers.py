"""Shared helpers for the parity tests."""
from __future__ import annotations

import numpy as np

# RGB tolerance stated by BASELINE.json's north star ("RGB within 1e-5 of CPU .ppm").  The
# kernels are built to be bit-exact; bitwise equality is asserted where the arithmetic is fully
# pinned (every op IEEE f32 in the reference's order, libm restated bit-exactly), and this
# tolerance is the documented fallback where a libm call is not restated (powf with exponent
# != 1).
RGB_TOL = 1e-5


def bit_equal(a: np.ndarray, b: np.ndarray) -> bool:
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def mismatch_report(a: np.ndarray, b: np.ndarray) -> str:
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    if a.shape != b.shape:
        return f"shape {a.shape} != {b.shape}"
    bad = a.view(np.uint32) != b.view(np.uint32)
    n = int(bad.sum())
    if not n:
        return "bit-identical"
    idx = np.argwhere(bad)[:5].tolist()
    diff = np.abs(a.astype(np.float64) - b.astype(np.float64))
    return f"{n} words differ; max |diff| {np.nanmax(diff):.3e}; first at {idx}"


def assert_bit_equal(a, b, what=""):
    assert bit_equal(a, b), f"{what}: {mismatch_report(a, b)}"


def random_mesh(rng: np.random.Generator, T: int, scale=1.0, center=(0.0, 0.0, 0.0)):
    """Random triangles around `center` with random per-vertex normals/uvs."""
    pos = (rng.uniform(-1, 1, (T, 9)) * scale + np.tile(center, 3)).astype(np.float32)
    nrm = rng.normal(size=(T, 9)).astype(np.float32)
    uv = rng.uniform(-0.5, 1.5, (T, 6)).astype(np.float32)
    return pos, nrm, uv

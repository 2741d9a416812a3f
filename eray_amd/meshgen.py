"""Deterministic synthetic meshes for the configs that name meshes absent from the reference.

BASELINE.json's C3 names the Stanford bunny (~70k triangles) and C5 a 1M-triangle synthetic
.obj; neither file exists (only objects/cube.obj ships with the reference).  SURVEY.md §8(d)
fixes the stand-in: a UV sphere of radius 0.9 with radial displacement
0.1*sin(5*theta)*sin(7*phi) (non-convex), faces randomly permuted with a fixed seed so the
first-hit index spreads over the whole range, fitted inside [-1, 1]^3 and written in the exact
.obj dialect the reference loader accepts.

    python -m eray_amd.meshgen --triangles 69451 --seed 42 -o objects/bunny_standin.obj
"""
from __future__ import annotations

import argparse
import math
import os

import numpy as np

from .objfile import write_obj


def _surface(theta, phi):
    r = 0.9 + 0.1 * np.sin(5.0 * theta) * np.sin(7.0 * phi)
    st = np.sin(theta)
    return np.stack([r * st * np.cos(phi), r * np.cos(theta), r * st * np.sin(phi)], axis=-1)


def displaced_sphere(triangles: int, seed: int):
    """Returns (vertices, normals, uvs, faces_v, faces_vt, faces_vn) with exactly `triangles`
    faces (a closed tessellation trimmed after the permutation when needed)."""
    if triangles < 8:
        raise ValueError("need at least 8 triangles")
    n_theta = max(3, int(round(math.sqrt(triangles / 4.0))) + 1)  # latitude bands
    n_phi = max(3, int(math.ceil(triangles / (2.0 * (n_theta - 1)))))
    # grid vertices (poles excluded) + 2 pole vertices
    th = np.linspace(0.0, math.pi, n_theta + 1)[1:-1]            # n_theta - 1 rings
    ph = np.linspace(0.0, 2.0 * math.pi, n_phi, endpoint=False)
    T, P = np.meshgrid(th, ph, indexing="ij")
    grid = _surface(T, P).reshape(-1, 3)
    north = _surface(np.array(0.0), np.array(0.0))[None]
    south = _surface(np.array(math.pi), np.array(0.0))[None]
    verts = np.concatenate([grid, north, south])
    # normals from the analytic surface by central differences
    eps = 1e-4
    dT = (_surface(T + eps, P) - _surface(T - eps, P)).reshape(-1, 3)
    dP = (_surface(T, P + eps) - _surface(T, P - eps)).reshape(-1, 3)
    nrm = np.cross(dP, dT)
    nrm = np.concatenate([nrm, [[0.0, 1.0, 0.0]], [[0.0, -1.0, 0.0]]])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    nrm[(nrm * verts).sum(axis=1) < 0] *= -1.0  # outward
    uvs = np.stack([(P / (2 * math.pi)).ravel(), (T / math.pi).ravel()], axis=1)
    uvs = np.concatenate([uvs, [[0.5, 0.0]], [[0.5, 1.0]]])
    rings = n_theta - 1
    ni, si = rings * n_phi, rings * n_phi + 1

    def vid(i, j):
        return i * n_phi + (j % n_phi)

    faces = []
    for j in range(n_phi):  # outward orientation: (b - a) x (c - a) points away from the centre
        faces.append((ni, vid(0, j + 1), vid(0, j)))
        faces.append((si, vid(rings - 1, j), vid(rings - 1, j + 1)))
    for i in range(rings - 1):
        for j in range(n_phi):
            a, b, c, d = vid(i, j), vid(i, j + 1), vid(i + 1, j), vid(i + 1, j + 1)
            faces.append((a, b, d))
            faces.append((a, d, c))
    F = np.array(faces, np.int64)
    # check and fix orientation per face against the outward direction
    v = verts[F]
    n = np.cross(v[:, 1] - v[:, 0], v[:, 2] - v[:, 0])
    out = (n * v.mean(axis=1)).sum(axis=1) < 0
    F[out] = F[out][:, [0, 2, 1]]
    rng = np.random.default_rng(seed)
    F = F[rng.permutation(len(F))][:triangles]
    # fit inside [-1, 1]^3 (already |r| <= 1); keep as is
    verts = verts.astype(np.float32)
    return verts, nrm.astype(np.float32), uvs.astype(np.float32), F, F, F


def generate(path: str, triangles: int, seed: int) -> str:
    v, n, t, fv, ft, fn = displaced_sphere(triangles, seed)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    write_obj(path, v, n, t, fv, ft, fn, name=f"displaced_sphere_{triangles}_{seed}")
    return path


# The configurations' meshes.
STANDIN_70K = dict(triangles=69451, seed=42)
SYNTH_1M = dict(triangles=1_000_000, seed=1234)


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--triangles", type=int, default=STANDIN_70K["triangles"])
    ap.add_argument("--seed", type=int, default=STANDIN_70K["seed"])
    ap.add_argument("-o", "--output", required=True)
    a = ap.parse_args()
    print(generate(a.output, a.triangles, a.seed))


if __name__ == "__main__":
    main()

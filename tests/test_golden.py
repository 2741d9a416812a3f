"""The committed golden fixtures (tests/golden/, made by tests/golden/make_golden.py from the
oracle): the CPU oracle must still reproduce them (CPU), and the HIP path must reproduce them bit
for bit (GPU), at C1 (256x256) directly and at C2 (1920x1080, the bench workload) through
SHA-256 digests of the PPM body, the f32 image and the face indices."""
import hashlib
import json
import os

import numpy as np
import pytest

from eray_amd import capi
from eray_amd.frame import MainScene

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _digests():
    with open(os.path.join(GOLDEN, "digests.json")) as f:
        return json.load(f)


def _sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("tag", ["c1", "c2", "c4"])
def test_oracle_reproduces_digests(oracle, cube, tag):
    g = _digests()[tag]
    scene = oracle.main_rs_scene(*cube, texture=1024)
    cam = oracle.camera((0.0, 0.0, 5.0), tuple(g["fov"]), g["width"], 1.0)
    rgb, face, stats = oracle.render(scene, cam, want_faces=True)
    full = oracle.ppm_bytes(rgb)
    assert full.startswith(g["ppm_header"].encode())
    assert hashlib.sha256(full).hexdigest() == g["ppm_file_sha256"]
    assert _sha(rgb.astype(np.float32)) == g["rgb_f32_sha256"]
    assert _sha(face.astype(np.int32)) == g["face_sha256"]
    assert stats == g["stats"]


def test_oracle_reproduces_c3_rows(oracle):
    """C3 (the 69,451-face stand-in at 1920x1080, main.rs's 1024x1024 material): two camera rows
    through the mesh centre, re-rendered by the oracle, equal the committed rows of the same run
    that produced digests["c3"] (make_c3_digest.py); the GPU test compares the whole frame with
    those digests."""
    from eray_amd import meshgen
    fx = np.load(os.path.join(GOLDEN, "c3_rows.npz"))
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(**meshgen.STANDIN_70K)
    mesh = (v[fv].reshape(-1, 9), n[fn].reshape(-1, 9), t[ft].reshape(-1, 6))
    scene = oracle.main_rs_scene(*mesh, texture=1024)
    row0 = int(fx["row0"])
    rgb, face, _ = oracle.render(scene, oracle.camera((0.0, 0.0, 5.0), (16.0, 9.0), 1920, 1.0), row0=row0,
                                 rows=fx["face"].shape[0], want_faces=True)
    assert (face >= 0).sum() > 300
    assert np.array_equal(face, fx["face"])
    assert np.array_equal(rgb.view(np.uint32), fx["rgb"].view(np.uint32))


def test_oracle_reproduces_c1_fixture(oracle, cube):
    fx = np.load(os.path.join(GOLDEN, "cube_c1_256.npz"))
    scene = oracle.main_rs_scene(*cube, texture=1024)
    rgb, face, _ = oracle.render(scene, oracle.camera((0.0, 0.0, 5.0), (60.0, 60.0), 256, 1.0), want_faces=True)
    assert np.array_equal(face, fx["face"].astype(np.int32))
    assert np.array_equal(rgb.reshape(-1, 3)[fx["hit_index"]], fx["hit_rgb"])
    body = oracle.ppm_bytes(rgb)[len(b"P6 256 256 255\n"):]
    assert np.array_equal(np.frombuffer(body, np.uint8).reshape(256, 256, 3), fx["ppm"])


def test_oracle_reproduces_c5_span_fixture(oracle):
    """Two of the C5 spans (1M faces at 7680x4320): the mesh centre and the right silhouette."""
    from tests.golden.make_golden import c5_mesh
    fx = np.load(os.path.join(GOLDEN, "c5_spans.npz"))
    scene = oracle.main_rs_scene(*c5_mesh(), texture=1024)
    cam = oracle.camera((0.0, 0.0, 5.0), (16.0, 9.0), 7680, 1.0)
    for k in (3, 4):
        y, x0, cols = (int(v) for v in fx["spans"][k])
        rgb, face, _ = oracle.render_span(scene, cam, y, 1, x0, cols)
        assert np.array_equal(face[0], fx[f"face{k}"])
        assert rgb[0].view(np.uint32).tobytes() == fx[f"rgb{k}"].view(np.uint32).tobytes()


def test_oracle_reproduces_north_star_span_fixture(oracle):
    """Two of the north_star spans (the 70k stand-in at 3840x2160): the top silhouette row and its
    neighbour above (tests/golden/make_golden.py ns)."""
    from tests.golden.make_golden import ns_mesh
    fx = np.load(os.path.join(GOLDEN, "ns_spans.npz"))
    scene = oracle.main_rs_scene(*ns_mesh(), texture=1024)
    cam = oracle.camera((0.0, 0.0, 5.0), (16.0, 9.0), 3840, 1.0)
    for k in (6, 7):
        y, x0, cols = (int(v) for v in fx["spans"][k])
        rgb, face, _ = oracle.render_span(scene, cam, y, 1, x0, cols)
        assert (face[0] >= 0).any() or k == 7
        assert np.array_equal(face[0], fx[f"face{k}"])
        assert rgb[0].view(np.uint32).tobytes() == fx[f"rgb{k}"].view(np.uint32).tobytes()


def test_oracle_reproduces_texture_fixture(oracle):
    fx = np.load(os.path.join(GOLDEN, "texture_8x4.npz"))
    color, diffuse = oracle.example_material(8, 4)
    assert np.array_equal(color, fx["color"]) and np.array_equal(diffuse, fx["diffuse"])


def _gpu_frame(gpu, cube, w, h, fov, material="textures"):
    sc = MainScene(gpu, *cube, w, h, texture=1024, fov=fov, material=material)
    rgb = gpu.empty((h, w, 3), np.float32)
    ppm = gpu.empty((h, w, 3), np.uint8)
    face = gpu.empty((h, w), np.int32)
    try:
        gpu.render(w, h, out_rgb=rgb.ptr, out_ppm=ppm.ptr, out_face=face.ptr)
        return rgb.numpy(), ppm.numpy(), face.numpy()
    finally:
        for a in (rgb, ppm, face):
            a.free()
        sc.close()


@pytest.mark.gpu
@pytest.mark.parametrize("material", ["textures", "example"])
def test_gpu_c1_matches_fixture(gpu, cube, material):
    fx = np.load(os.path.join(GOLDEN, "cube_c1_256.npz"))
    rgb, ppm, face = _gpu_frame(gpu, cube, 256, 256, (60.0, 60.0), material)
    assert np.array_equal(face, fx["face"].astype(np.int32))
    assert np.array_equal(ppm, fx["ppm"])
    got = rgb.reshape(-1, 3)[fx["hit_index"]]
    assert got.view(np.uint32).tobytes() == fx["hit_rgb"].view(np.uint32).tobytes()
    assert capi.ppm_header(256, 256) == b"P6 256 256 255\n"


@pytest.mark.gpu
@pytest.mark.parametrize("material", ["textures", "example"])
def test_gpu_c2_matches_digests(gpu, cube, material):
    """The bench workload at full size, bit for bit, against the oracle's committed digests —
    with the material sampled from its textures and evaluated per hit texel."""
    g = _digests()["c2"]
    rgb, ppm, face = _gpu_frame(gpu, cube, 1920, 1080, (16.0, 9.0), material)
    assert _sha(face.astype(np.int32)) == g["face_sha256"]
    assert _sha(rgb.astype(np.float32)) == g["rgb_f32_sha256"]
    assert _sha(ppm) == g["ppm_body_sha256"]
    assert hashlib.sha256(capi.ppm_header(1920, 1080) + ppm.tobytes()).hexdigest() == g["ppm_file_sha256"]
    assert int((face >= 0).sum()) == g["hit_pixels"]


@pytest.mark.gpu
def test_gpu_material_example_matches_fixture(gpu):
    fx = np.load(os.path.join(GOLDEN, "texture_8x4.npz"))
    color = gpu.empty((4, 8, 3), np.float32)
    diffuse = gpu.empty((4, 8), np.float32)
    try:
        gpu.material_example(8, 4, 1.0, 1.0, 1.0, 0.0, 0.0, 0.5, color.ptr, diffuse.ptr)  # main.rs inputs
        assert np.array_equal(color.numpy(), fx["color"]) and np.array_equal(diffuse.numpy(), fx["diffuse"])
    finally:
        color.free()
        diffuse.free()

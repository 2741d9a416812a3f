"""Generates the committed golden fixtures of tests/golden/ from the CPU oracle (oracle/, the
literal restatement of the reference's arithmetic, itself pinned by the reference's own known
answers in tests/test_oracle_known_answers.py).  The reference (Rust) cannot be built here
(SURVEY.md §8c), so these fixtures freeze the oracle's outputs: the GPU path and any later
oracle change are checked against the same bytes.

    python tests/golden/make_golden.py

Fixtures
  cube_c1_256.npz   C1 (cube.obj, 256x256, main.rs scene): the PPM body bytes (file order),
                    the hit face per pixel, and the f32 RGB of the hit pixels (indices + values)
  digests.json      SHA-256 of the PPM body and of the f32 image for C1, C2 (1920x1080), C4
                    (3840x2160) and main.rs's 1024x1024 output.ppm (with its color.ppm and rgb.ppm
                    debug files), the per-frame hit/test counters, and the P6 headers
  texture_8x4.npz   the example material graph (wave -> rgb -> mix with flat) at 8x4 texels:
                    color and diffuse images
  c5_spans.npz      C5 (the 1M-face synthetic mesh, meshgen seed 1234, at 7680x4320, main.rs
                    scene): pixel spans across the silhouette, the mesh centre and the row-tile
                    boundary of the 8-GPU split (oracle_render_span), f32 RGB and faces
  ns_spans.npz      north_star (the 69,451-face stand-in, meshgen seed 42, at 3840x2160, main.rs
                    scene): the two camera rows through the mesh centre in full, and spans across
                    the top and bottom silhouettes (the first and last hit rows of the centre
                    column and their neighbours), f32 RGB and faces — `python make_golden.py ns`
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from eray_amd import meshgen  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402
from oracle import pyoracle as O  # noqa: E402


def frame(mesh, w, h, fov):
    scene = O.main_rs_scene(*mesh, texture=1024)
    cam = O.camera((0.0, 0.0, 5.0), fov, w, 1.0)
    assert O.camera_size(cam) == (w, h)
    rgb, face, stats = O.render(scene, cam, want_faces=True)
    return rgb, face, stats


# C5 spans (camera row, first column, columns): the 8-GPU split's middle tile boundary (camera
# rows 2159 | 2160), the mesh centre, the left and right silhouettes, a row near the top of the
# mesh, and one row block at another tile boundary (all background there, 16 pixels)
C5_SPANS = [(2159, 3360, 48), (2160, 3360, 48), (2160, 3816, 48), (2160, 4252, 48), (2163, 3830, 20),
            (1812, 3800, 64), (2507, 3700, 40), (1620, 100, 4)]


def c5_mesh():
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(**meshgen.SYNTH_1M)
    return (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(n[fn].reshape(-1, 9)),
            np.ascontiguousarray(t[ft].reshape(-1, 6)))


def c5_spans() -> None:
    scene = O.main_rs_scene(*c5_mesh(), texture=1024)
    cam = O.camera((0.0, 0.0, 5.0), (16.0, 9.0), 7680, 1.0)
    assert O.camera_size(cam) == (7680, 4320)
    out = {"spans": np.array(C5_SPANS, np.int32)}
    for k, (y, x0, cols) in enumerate(C5_SPANS):
        rgb, face, _ = O.render_span(scene, cam, y, 1, x0, cols)
        out[f"rgb{k}"] = rgb[0]
        out[f"face{k}"] = face[0]
    np.savez_compressed(os.path.join(HERE, "c5_spans.npz"), **out)


NS_W, NS_H = 3840, 2160


def ns_mesh():
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(**meshgen.STANDIN_70K)
    return (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(n[fn].reshape(-1, 9)),
            np.ascontiguousarray(t[ft].reshape(-1, 6)))


def ns_spans() -> None:
    """north_star rows: the centre rows 1079 and 1080 whole (both silhouettes of the row), and
    the top and bottom silhouettes found on the centre column (its first and last hit rows),
    each with its neighbours as 640-pixel spans around the centre column."""
    import concurrent.futures as cf
    scene = O.main_rs_scene(*ns_mesh(), texture=1024)
    cam = O.camera((0.0, 0.0, 5.0), (16.0, 9.0), NS_W, 1.0)
    assert O.camera_size(cam) == (NS_W, NS_H)
    cx = NS_W // 2
    col = [O.render_span(scene, cam, y, 1, cx, 1)[1][0, 0] for y in range(NS_H // 2 - 320, NS_H // 2 + 320)]
    hit = [NS_H // 2 - 320 + i for i, f in enumerate(col) if f >= 0]
    y_lo, y_hi = min(hit), max(hit)
    spans = [(1079, 0, NS_W), (1080, 0, NS_W)]
    spans += [(y, cx - 320, 640) for y in (y_lo - 1, y_lo, y_lo + 1, y_hi - 1, y_hi, y_hi + 1)]
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:  # (ctypes drops the GIL)
        res = list(ex.map(lambda s: O.render_span(scene, cam, s[0], 1, s[1], s[2]), spans))
    out = {"spans": np.array(spans, np.int32)}
    for k, (rgb, face, _) in enumerate(res):
        out[f"rgb{k}"] = rgb[0]
        out[f"face{k}"] = face[0]
    np.savez_compressed(os.path.join(HERE, "ns_spans.npz"), **out)


def main() -> None:
    mesh = load_obj_file(os.path.join(ROOT, "objects", "cube.obj"))
    digests = {}
    configs = {"c1": (256, 256, (60.0, 60.0)), "c2": (1920, 1080, (16.0, 9.0)),
               "main_rs": (1024, 1024, (60.0, 60.0)),  # main.rs's own 1024x1024 render
               "c4": (3840, 2160, (16.0, 9.0))}
    for tag, (w, h, fov) in configs.items():
        rgb, face, stats = frame(mesh, w, h, fov)
        full = O.ppm_bytes(rgb)  # the whole P6 file: header + body
        header = f"P6 {w} {h} 255\n".encode()
        assert full.startswith(header)
        body = full[len(header):]
        digests[tag] = {
            "width": w, "height": h, "fov": list(fov),
            "ppm_header": f"P6 {w} {h} 255\n",
            "ppm_body_sha256": hashlib.sha256(body).hexdigest(),
            "ppm_file_sha256": hashlib.sha256(full).hexdigest(),
            "rgb_f32_sha256": hashlib.sha256(np.ascontiguousarray(rgb, np.float32).tobytes()).hexdigest(),
            "face_sha256": hashlib.sha256(np.ascontiguousarray(face, np.int32).tobytes()).hexdigest(),
            "hit_pixels": int((face >= 0).sum()),
            "stats": {k: int(v) for k, v in stats.items()},
        }
        if tag == "c1":
            hit = np.flatnonzero(face.reshape(-1) >= 0).astype(np.int32)
            np.savez_compressed(os.path.join(HERE, "cube_c1_256.npz"),
                                ppm=np.frombuffer(body, np.uint8).reshape(h, w, 3),
                                face=face.astype(np.int16),
                                hit_index=hit,
                                hit_rgb=rgb.reshape(-1, 3)[hit].astype(np.float32))
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(digests, f, indent=2, sort_keys=True)
    # main.rs's debug side-effect files at its 1024x1024 material: color.ppm (Material::update,
    # material.rs:41-50) and rgb.ppm (the rgb node, rgb.rs:96: rgb(wave, wave, wave))
    color, _ = O.example_material(1024, 1024)
    wave = O.node_wave(1024, 1024, 1.0, 1.0)
    rgb_img = O.node_rgb(1024, 1024, wave, wave, wave)
    digests["main_rs"]["color_ppm_sha256"] = hashlib.sha256(O.ppm_bytes(color)).hexdigest()
    digests["main_rs"]["rgb_ppm_sha256"] = hashlib.sha256(O.ppm_bytes(rgb_img)).hexdigest()
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(digests, f, indent=2, sort_keys=True)
    c5_spans()
    color, diffuse = O.example_material(8, 4)
    np.savez_compressed(os.path.join(HERE, "texture_8x4.npz"), color=color, diffuse=diffuse)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    if sys.argv[1:] == ["ns"]:
        ns_spans()
    else:
        main()

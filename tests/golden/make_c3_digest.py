"""Generates the C3 entry of tests/golden/digests.json from the CPU oracle: BASELINE.json configs[2]
(the 69,451-face stand-in, meshgen seed 42, at 1920x1080 with main.rs's scene and its 1024x1024
material).  The oracle scans every face per missed ray (~1.4e11 tests), so the frame's rows are
split over the host's cores (ctypes releases the GIL; the oracle keeps no global state).

    python tests/golden/make_c3_digest.py [--threads N]

Adds digests["c3"] with the same fields as the other frames (make_golden.py), and c3_rows.npz:
camera rows 540 and 541 (through the stand-in's centre) as f32 RGB and faces, which the CPU suite
re-renders with the oracle in about a second (tests/test_golden.py).  --rows-only writes just those.
"""
import argparse
import concurrent.futures as cf
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from eray_amd import meshgen  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

W, H, FOV = 1920, 1080, (16.0, 9.0)


def c3_mesh():
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(**meshgen.STANDIN_70K)
    return (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(n[fn].reshape(-1, 9)),
            np.ascontiguousarray(t[ft].reshape(-1, 6)))


ROWS = (540, 2)


def c3_rows(scene, cam) -> None:
    rgb, face, _ = O.render(scene, cam, row0=ROWS[0], rows=ROWS[1], want_faces=True)
    np.savez_compressed(os.path.join(HERE, "c3_rows.npz"), row0=ROWS[0], rgb=rgb, face=face)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 4)
    ap.add_argument("--rows-only", action="store_true")
    a = ap.parse_args()
    scene = O.main_rs_scene(*c3_mesh(), texture=1024)
    cam = O.camera((0.0, 0.0, 5.0), FOV, W, 1.0)
    assert O.camera_size(cam) == (W, H)
    c3_rows(scene, cam)
    if a.rows_only:
        return
    chunk = 8
    rgb = np.zeros((H, W, 3), np.float32)
    face = np.full((H, W), -1, np.int32)
    stats = {"primary_tests": 0, "shadow_tests": 0, "hit_pixels": 0}

    def part(row0):
        n = min(chunk, H - row0)
        r, f, st = O.render(scene, cam, row0=row0, rows=n, want_faces=True)
        return row0, n, r, f, st

    t0 = time.time()
    with cf.ThreadPoolExecutor(a.threads) as ex:
        for row0, n, r, f, st in ex.map(part, range(0, H, chunk)):
            rgb[row0:row0 + n] = r
            face[row0:row0 + n] = f
            for k in stats:
                stats[k] += st[k]
    full = O.ppm_bytes(rgb)
    header = f"P6 {W} {H} 255\n".encode()
    body = full[len(header):]
    path = os.path.join(HERE, "digests.json")
    with open(path) as f:
        digests = json.load(f)
    digests["c3"] = {
        "width": W, "height": H, "fov": list(FOV), "mesh": "meshgen.displaced_sphere(69451, seed 42)",
        "texture": 1024,
        "ppm_header": f"P6 {W} {H} 255\n",
        "ppm_body_sha256": hashlib.sha256(body).hexdigest(),
        "ppm_file_sha256": hashlib.sha256(full).hexdigest(),
        "rgb_f32_sha256": hashlib.sha256(np.ascontiguousarray(rgb, np.float32).tobytes()).hexdigest(),
        "face_sha256": hashlib.sha256(np.ascontiguousarray(face, np.int32).tobytes()).hexdigest(),
        "hit_pixels": int((face >= 0).sum()),
        "stats": stats,
    }
    with open(path, "w") as f:
        json.dump(digests, f, indent=2, sort_keys=True)
    print(f"c3: {digests['c3']['hit_pixels']} hit pixels, {stats['primary_tests']} tests, {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()

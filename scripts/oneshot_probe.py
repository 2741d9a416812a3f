"""Diagnostics: bench.one_shot's steps on a mesh, each timed, the host copy of the PPM body twice
(is the first copy's cost the copy, or something before it?)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from bench import TEXTURE, frame_camera_fov  # noqa: E402
from eray_amd import capi  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402


def main():
    path, W, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    for tag in ("cold", "warm"):
        t = [("start", time.perf_counter())]
        mesh = load_obj_file(path)
        t.append(("load_obj", time.perf_counter()))
        ctx = capi.Context(0)
        t.append(("context", time.perf_counter()))
        sc = MainScene(ctx, *mesh, W, H, texture=TEXTURE, fov=frame_camera_fov(W, H))
        ctx.synchronize()
        t.append(("upload_material", time.perf_counter()))
        ppm = ctx.empty((H, W, 3), np.uint8)
        t.append(("alloc_out", time.perf_counter()))
        ctx.render(W, H, out_ppm=ppm.ptr)
        t.append(("render_enqueue", time.perf_counter()))
        ctx.synchronize()
        t.append(("render_sync", time.perf_counter()))
        body = ppm.numpy()
        t.append(("ppm_to_host_1", time.perf_counter()))
        body = ppm.numpy()
        t.append(("ppm_to_host_2", time.perf_counter()))
        ctx.render(W, H, out_ppm=ppm.ptr)
        ctx.synchronize()
        t.append(("render_again", time.perf_counter()))
        ppm.free()
        sc.close()
        ctx.close()
        print(tag, {k: round((b - a) * 1e3, 3) for (_, a), (k, b) in zip(t, t[1:])}, flush=True)
        del body


if __name__ == "__main__":
    main()

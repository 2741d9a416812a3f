"""Diagnostics: a moving camera over a binned mesh (C3 by default) — device ms per frame of
eray_render_camera_path (setup + frame per camera), for the kernel timeline under rocprofv3."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from bench import dolly_path, frame_camera_fov  # noqa: E402
from eray_amd import capi, meshgen  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=64)
    a = ap.parse_args()
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(**meshgen.STANDIN_70K)
    mesh = (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(n[fn].reshape(-1, 9)),
            np.ascontiguousarray(t[ft].reshape(-1, 6)))
    W, H = a.width, a.height
    ctx = capi.Context(0)
    sc = MainScene(ctx, *mesh, W, H, texture=1024, fov=frame_camera_fov(W, H))
    rgb = ctx.empty((H, W, 3), np.float32)
    ppm = ctx.empty((H, W, 3), np.uint8)
    path = dolly_path(a.frames, frame_camera_fov(W, H), W)
    kw = dict(out_rgb=rgb.ptr, out_ppm=ppm.ptr)
    ctx.render_camera_path(path, W, H, **kw)
    ms = [ctx.render_camera_path(path, W, H, timed=True, **kw) for _ in range(3)]
    print(json.dumps({"frame": [W, H], "frames": a.frames, "device_ms_per_frame": [round(x, 4) for x in ms]}))
    rgb.free()
    ppm.free()
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()

"""A moving-camera frame loop alone (eray_render_camera_path), for rocprofv3 kernel statistics of
the per-frame camera setup: python scripts/moving_camera.py [--mesh M] [--width W] [--height H]."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from bench import dolly_path, frame_camera_fov  # noqa: E402
from eray_amd import capi  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mesh", default=os.path.join(ROOT, "objects", "cube.obj"))
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--frames", type=int, default=100)
a = ap.parse_args()
mesh = load_obj_file(a.mesh)
ctx = capi.Context(0)
fov = frame_camera_fov(a.width, a.height)
sc = MainScene(ctx, *mesh, a.width, a.height, texture=1024, fov=fov)
rgb = ctx.empty((a.height, a.width, 3), np.float32)
ppm = ctx.empty((a.height, a.width, 3), np.uint8)
path = dolly_path(a.frames, fov, a.width)
kw = dict(out_rgb=rgb.ptr, out_ppm=ppm.ptr)
ctx.render_camera_path(path, a.width, a.height, **kw)
ms = ctx.render_camera_path(path, a.width, a.height, timed=True, **kw)
st = ctx.render_frames(a.frames, a.width, a.height, timed=True, **kw)
print(f"{os.path.basename(a.mesh)} {a.width}x{a.height}: moving {ms * 1e3:.2f} us/frame, static {st * 1e3:.2f} us/frame")
rgb.free()
ppm.free()
sc.close()
ctx.close()

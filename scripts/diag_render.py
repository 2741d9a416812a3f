"""Diagnostic timings of the frame kernel on controlled scenes (not part of the product)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from eray_amd import capi  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402

W, H = 1920, 1080
mesh = load_obj_file(os.path.join(ROOT, "objects", "cube.obj"))
ctx = capi.Context(0)
rgb = ctx.empty((H, W, 3), np.float32)
ppm = ctx.empty((H, W, 3), np.uint8)


def timed(label, flags=0, frames=200, row0=0, rows=H, ppm_out=True):
    kw = dict(row0=row0, rows=rows, out_rgb=rgb.ptr, out_ppm=ppm.ptr if ppm_out else None, flags=flags)
    ctx.render_frames(frames, W, H, prepare_only=True, **kw)
    ctx.render_frames(20, W, H, **kw)
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.render_frames(frames, W, H, **kw)
    ctx.synchronize()
    wall = (time.perf_counter() - t0) / frames
    ms = ctx.render_frames(frames, W, H, timed=True, **kw)
    print(f"{label:48s} frame {wall * 1e6:8.2f} us   kernel {ms * 1e3:8.2f} us", flush=True)


sc = MainScene(ctx, *mesh, W, H, material="example")
timed("cube, material evaluated per hit")
sc.close()
sc = MainScene(ctx, *mesh, W, H)
timed("cube (main.rs scene)")
timed("cube, f32 image only (no PPM)", ppm_out=False)
timed("cube rows 300..780", row0=300, rows=480)
timed("cube rows 540..544 (one block row)", row0=540, rows=4)
timed("rows 0..4 (background only)", row0=0, rows=4)
timed("cube brute force", flags=capi.RENDER_BRUTE_FORCE)
ctx.set_camera(capi.make_camera((0.0, 0.0, 5.0), (16.0, 9.0), W, -1.0))
timed("cube out of view (fill only)")
ctx.scene_reset()
ctx.set_camera(capi.make_camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0))
timed("empty scene (fill only)")
sc.close()

"""A/B of eray_render_params flag sets on one workload (diagnostics): device us per frame (HIP
events over graph-replayed frames, one frame per launch into one buffer, as the bench's 4K line),
the sets interleaved over several rounds.  Usage: python scripts/ab_flags.py MESH W H FLAGS..."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from bench import frame_camera_fov  # noqa: E402
from eray_amd import capi  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402

mesh = load_obj_file(sys.argv[1])
W, H = int(sys.argv[2]), int(sys.argv[3])
sets = [int(x) for x in sys.argv[4:]] or [0]
ctx = capi.Context(0)
sc = MainScene(ctx, *mesh, W, H, fov=frame_camera_fov(W, H))
rgb = ctx.empty((H, W, 3), np.float32)
ppm = ctx.empty((H, W, 3), np.uint8)
K = 64
res = {f: [] for f in sets}
for f in sets:
    ctx.render_frames(K, W, H, out_rgb=rgb.ptr, out_ppm=ppm.ptr, flags=f, prepare_only=True)
for rnd in range(4):
    for f in sets:
        ctx.render_frames(K, W, H, out_rgb=rgb.ptr, out_ppm=ppm.ptr, flags=f)
        res[f].append(ctx.render_frames(K, W, H, out_rgb=rgb.ptr, out_ppm=ppm.ptr, flags=f, timed=True) * 1e3)
print(json.dumps({"mesh": os.path.basename(sys.argv[1]), "frame": [W, H],
                  "us_per_frame_by_flags": {f: [round(min(v), 3), round(float(np.median(v)), 3)] for f, v in res.items()}}))

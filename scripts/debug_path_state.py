"""Camera-path diagnostics: the setup state after each path (bin entries needed, overflow flag,
detail count, bin capacity) and the device time per frame, for a mesh at a frame size."""
import ctypes as C
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

mesh_path, W, H, frames = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
mesh = load_obj_file(mesh_path)
ctx = capi.Context(0)
fov = frame_camera_fov(W, H)
sc = MainScene(ctx, *mesh, W, H, texture=256, fov=fov)
rgb = ctx.empty((H, W, 3), np.float32)
ppm = ctx.empty((H, W, 3), np.uint8)
kw = dict(out_rgb=rgb.ptr, out_ppm=ppm.ptr)
L = capi.lib()
state = (C.c_uint32 * 64)()
rect = (C.c_int32 * 4)()


def show(tag):
    assert L.eray_debug_setup_state(ctx.handle, 0, state, rect) == 0
    print(f"{tag}: total_sub {state[9]}, bin_entries {state[10]}, overflow {state[11]}, "
          f"capacity {L.eray_debug_bin_capacity(ctx.handle)}", flush=True)


ms = ctx.render_frames(10, W, H, timed=True, **kw)
show(f"static {ms * 1e3:.1f} us/frame")
path = dolly_path(frames, fov, W)
for k in range(3):
    ms = ctx.render_camera_path(path, W, H, timed=True, **kw)
    show(f"path {k}: {ms * 1e3:.1f} us/frame")

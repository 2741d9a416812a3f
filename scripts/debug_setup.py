"""Diagnostics: device-camera vs args-mode frames and the setup state for a few cameras."""
import ctypes as C
import math
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from eray_amd import capi  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cube = load_obj_file(os.path.join(ROOT, "objects", "cube.obj"))
W, H = 320, 180
ctx = capi.Context(0)
sc = MainScene(ctx, *cube, W, H, texture=256, fov=(16.0, 9.0))
rgb = ctx.empty((H, W, 3), np.float32)
face = ctx.empty((H, W), np.int32)
L = capi.lib()
for k in range(4):
    a = 2.0 * math.pi * k / 7
    cam = capi.make_camera((1.1 * math.sin(a), 0.6 * math.cos(3 * a), 5.0 + 0.7 * math.cos(a)), (16.0, 9.0), W, 1.0)
    ctx.set_camera(cam)
    res = []
    for rep in range(2):
        ctx.memset(face.ptr, 0x7F, face.nbytes)
        ctx.render(W, H, out_rgb=rgb.ptr, out_face=face.ptr)
        f = face.numpy()
        res.append(f)
        st = (C.c_uint32 * 44)()
        rect = (C.c_int32 * 4)()
        assert L.eray_debug_setup_state(ctx.handle, 0, st, rect) == 0
        words = list(st)
        cam_f = np.frombuffer(bytes(st)[:20], np.float32)
        print(f"cam {k} rep {rep}: hits {(f >= 0).sum()} unset {(f == 0x7F7F7F7F).sum()} state cam {cam_f} "
              f"nrect {words[8]} total {words[9]} rects {words[12:16]} obj rect {list(rect)}")
    print("  equal:", np.array_equal(res[0], res[1]))

"""Phase timeline of the frame kernel (diagnostic build, `python -m eray_amd.build --trace`).

Renders the bench frame (cube, main.rs scene, 1920x1080) and prints, for workgroups
0, 16, ..., 1008, each wave's phase timestamps (s_memrealtime, 10 ns ticks) relative to the earliest
kernel-entry stamp: 0 entry, 1 caches ready, 2 primary hits, 3 material, 4 lighting,
5 sub-block stored, 7 detail done, 8 kernel end; 14 camera ray and bounding box, 15 shadow scan.
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["ERAY_LIB"] = os.path.join(ROOT, "eray_amd", "lib", "liberay_hip_trace.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from eray_amd import capi  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402

W, H = int(os.environ.get("ERAY_TRACE_W", 1920)), int(os.environ.get("ERAY_TRACE_H", 1080))
rows = int(sys.argv[1]) if len(sys.argv) > 1 else H
row0 = (H - rows) // 2
mesh = load_obj_file(sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "objects", "cube.obj"))
ctx = capi.Context(0)
rgb = ctx.empty((H, W, 3), np.float32)
ppm = ctx.empty((H, W, 3), np.uint8)
from bench import frame_camera_fov  # noqa: E402
sc = MainScene(ctx, *mesh, W, H, fov=frame_camera_fov(W, H))
for _ in range(30):
    ctx.render(W, H, row0=row0, rows=rows, out_rgb=rgb.ptr, out_ppm=ppm.ptr)
ctx.synchronize()
lib = capi.lib()
NS = 24
buf = (C.c_uint64 * (2 * 64 * 4 * NS))()
lib.eray_debug_trace.argtypes = [C.c_void_p, C.c_size_t]
assert lib.eray_debug_trace(buf, len(buf)) == 0
tt = np.frombuffer(buf, dtype=np.uint64).reshape(2, 64, 4, NS).astype(np.int64)
t, clk = tt[0], tt[1]
sel = (t[:, :, 0] > 0) & (t[:, :, 8] > 0)
if sel.any():
    ghz = ((clk[:, :, 8] - clk[:, :, 0])[sel] / ((t[:, :, 8] - t[:, :, 0])[sel] * 10.0)).mean()
    print(f"shader clock ~ {ghz:.2f} GHz (s_memtime / s_memrealtime)")
sel = (t[:, :, 1] > 0) & (t[:, :, 7] > 0)
if sel.any():
    ghz = ((clk[:, :, 7] - clk[:, :, 1])[sel] / ((t[:, :, 7] - t[:, :, 1])[sel] * 10.0)).mean()
    print(f"shader clock (detail waves) ~ {ghz:.2f} GHz")
t0 = t[:, :, 0][t[:, :, 0] > 0].min()
names = {16: "bin_in", 17: "bin_sync", 18: "bin_loop", 19: "bin_out", 20: "sh_in", 21: "sh_out", 0: "entry", 13: "issued", 12: "stored", 1: "caches", 9: "geom", 10: "cull", 11: "ray", 14: "bbox", 2: "primary", 3: "material", 15: "shadow", 4: "light", 5: "out",
         6: "repeat", 7: "detail", 8: "end"}
print(f"rows {row0}..{row0 + rows}; ticks of 10 ns from the first entry")
order = [0, 13, 12, 1, 16, 14, 17, 18, 19, 2, 3, 20, 21, 15, 4, 5, 7]
print("  wg.w " + " ".join(f"{names[k]:>8s}" for k in order))
for g in range(64):
    for w in range(4):
        row = t[g, w]
        if row[0] == 0:
            continue
        print(f"{16 * g:4d}.{w} " + " ".join(f"{(row[k] - t0) if row[k] else -1:8d}" for k in order)
              + f"   bin entries {row[23]:5d}")
print("shader cycles from each detail wave's entry (s_memtime)")
print("  wg.w " + " ".join(f"{names[k]:>8s}" for k in order))
for g in range(64):
    for w in range(4):
        row, ck = t[g, w], clk[g, w]
        if row[0] == 0 or row[1] == 0 or row[7] == 0:
            continue
        print(f"{16 * g:4d}.{w} " + " ".join(f"{(ck[k] - ck[0]) if ck[k] else -1:8d}" for k in order))

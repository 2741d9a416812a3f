"""Screen-bin statistics of a large mesh (diagnostics): bins, entries, (face, pixel) pairs."""
import ctypes as C
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
ctx = capi.Context(0)
sc = MainScene(ctx, *mesh, W, H, fov=frame_camera_fov(W, H))
rgb = ctx.empty((H, W, 3), np.float32)
face = ctx.empty((H, W), np.int32)
sc.render(out_rgb=rgb.ptr, out_face=face.ptr)
ctx.synchronize()
hits = int((face.numpy() >= 0).sum())
out = (C.c_uint64 * 14)()
lib = capi.lib()
lib.eray_debug_bin_stats.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
assert lib.eray_debug_bin_stats(ctx._h, 0, out) == 0
nb, n, pairs, most, nonempty, most_pairs = list(out)[:6]
rect = [C.c_int64(v).value for v in list(out)[6:10]]
print(f"{W}x{H} T={len(mesh[0])}: hits {hits}, bins {nb}, non-empty {nonempty}, entries {n} "
      f"({n / max(nonempty, 1):.1f}/bin, max {most}), pairs {pairs} ({pairs / max(n, 1):.2f}/entry, "
      f"{pairs / max(hits, 1):.1f}/hit px, max {most_pairs}/bin), object rect {rect}, rectangle pairs {out[13]}")

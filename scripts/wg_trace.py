"""Per-workgroup timeline of one frame_kernel launch (diagnostics; needs the trace build,
scripts/build_trace.sh, selected with ERAY_LIB=eray_amd/lib/liberay_hip_trace.so).
Usage: python scripts/wg_trace.py MESH W H"""
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
ppm = ctx.empty((H, W, 3), np.uint8)
lib = capi.lib()
lib.eray_debug_read_trace.argtypes = [C.c_void_p, C.c_size_t]
kw = dict(out_rgb=rgb.ptr, out_ppm=ppm.ptr)
ctx.render_frames(50, W, H, **kw)
ctx.synchronize()
n = 8192 * 16
for rep in range(3):
    assert lib.eray_debug_clear_trace() == 0
    ctx.render_frames(1, W, H, **kw)
    ctx.synchronize()
    buf = (C.c_uint64 * n)()
    assert lib.eray_debug_read_trace(buf, n) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 16).astype(np.int64)
    used = t[:, 0] > 0
    t = t[used]
    t0 = t[:, 0].min()
    us = lambda x: (x - t0) / 100.0  # 100 MHz -> us  # noqa: E731
    det = t[:, 1] > 0
    fil = t[:, 3] > 0
    end = np.maximum(t[:, 1], t[:, 3])
    print(f"rep {rep}: {len(t)} workgroups, span {us(end.max()):.2f} us; starts p50 {np.median(us(t[:, 0])):.2f} "
          f"max {us(t[:, 0]).max():.2f}")
    if det.any():
        d = us(t[det, 1]) - us(t[det, 0])
        print(f"  detail {det.sum()}: end p10 {np.percentile(us(t[det, 1]), 10):.2f} p50 {np.median(us(t[det, 1])):.2f} "
              f"p90 {np.percentile(us(t[det, 1]), 90):.2f} max {us(t[det, 1]).max():.2f}; duration p50 {np.median(d):.2f} "
              f"p90 {np.percentile(d, 90):.2f} max {d.max():.2f}")
        ph = t[det][:, 4:8] / 100.0
        ok = (ph > 0).all(axis=1)
        ph = ph[ok]
        print(f"  wave 0's latest sub-block: search p50 {np.median(ph[:, 1] - ph[:, 0]):.2f} us "
              f"(p90 {np.percentile(ph[:, 1] - ph[:, 0], 90):.2f}), shading p50 {np.median(ph[:, 2] - ph[:, 1]):.2f} "
              f"(p90 {np.percentile(ph[:, 2] - ph[:, 1], 90):.2f}), outputs p50 {np.median(ph[:, 3] - ph[:, 2]):.2f}, "
              f"to workgroup end p50 {np.median(t[det][ok, 1] / 100.0 - ph[:, 3]):.2f}; first start p50 "
              f"{np.median(us(t[det][ok, 4])):.2f}")
        P = t[det][ok]
        names = [(4, 8, "range+rays"), (8, 9, "barrier1"), (9, 10, "chunks"), (10, 11, "barrier2"),
                 (11, 12, "re-test"), (12, 5, "to object-loop end"), (5, 13, "hit records"), (13, 14, "shadow"),
                 (14, 6, "shading"), (6, 7, "outputs")]
        parts = []
        for a, b, nm in names:
            m = (P[:, a] > 0) & (P[:, b] > 0)
            if m.any():
                parts.append(f"{nm} {np.median((P[m, b] - P[m, a]) / 100.0):.2f}")
        print("  wave 0 phases p50 (us):", ", ".join(parts))
        hist, edges = np.histogram(us(t[det, 1]), bins=12)
        print("  detail end histogram:", " ".join(f"{e:.1f}:{h}" for e, h in zip(edges, hist)))
    if fil.any():
        f = us(t[fil, 3]) - us(t[fil, 2])
        print(f"  fill {fil.sum()}: start p50 {np.median(us(t[fil, 2])):.2f}, end p10 {np.percentile(us(t[fil, 3]), 10):.2f} "
              f"p50 {np.median(us(t[fil, 3])):.2f} p90 {np.percentile(us(t[fil, 3]), 90):.2f} max {us(t[fil, 3]).max():.2f}; "
              f"duration p50 {np.median(f):.2f} max {f.max():.2f}")

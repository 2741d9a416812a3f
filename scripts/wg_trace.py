"""Per-workgroup timeline of one frame_kernel launch (diagnostics; needs the trace build,
scripts/build_trace.sh, selected with ERAY_LIB=eray_amd/lib/liberay_hip_trace.so).
Usage: python scripts/wg_trace.py MESH W H [SLOTS [FRAMES]]   (SLOTS > 1: a ring of frame slots, one
frame per launch unless FRAMES (frames per launch, C2: 8 8), so that the traced frame's stores go to
HBM when the ring exceeds the Infinity Cache)"""
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
slots = int(sys.argv[4]) if len(sys.argv) > 4 else 1
frames = int(sys.argv[5]) if len(sys.argv) > 5 else 1
rgb = ctx.empty((slots, H, W, 3), np.float32)
ppm = ctx.empty((slots, H, W, 3), np.uint8)
lib = capi.lib()
lib.eray_debug_read_trace.argtypes = [C.c_void_p, C.c_size_t]
kw = dict(out_rgb=rgb.ptr, out_ppm=ppm.ptr)
if slots > 1:
    kw["ring"] = capi.frame_ring(slots, H, W, frames)
ctx.render_frames(50, W, H, **kw)
ctx.synchronize()
n = 8192 * 64  # (scripts/microbench/render_trace.hip kTraceSlots)
for rep in range(3):
    assert lib.eray_debug_clear_trace() == 0
    ctx.render_frames(frames, W, H, **kw)
    ctx.synchronize()
    buf = (C.c_uint64 * n)()
    assert lib.eray_debug_read_trace(buf, n) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 64).astype(np.int64)
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
        names = [(4, 16, "ObjGeom"), (16, 8, "rays+bbox"), (8, 9, "first chunk"), (9, 10, "chunks"),
                 (10, 5, "to object-loop end"), (5, 17, "MaterialDesc"), (17, 13, "hit records"), (13, 14, "shadow"),
                 (13, 18, "shadow: light read"), (18, 19, "shadow: ObjGeom read"), (19, 14, "shadow: skip or scan"),
                 (14, 6, "shading"), (6, 7, "outputs")]
        S = t[det]
        m = (S[:, 32 + 11] > 0) & (S[:, 32 + 12] > 0) & (S[:, 32 + 4] > 0)
        if m.any():
            print(f"  startup p50 (us): WG start -> list entry {np.median((S[m, 43] - S[m, 0]) / 100.0):.2f}, "
                  f"-> binned object {np.median((S[m, 44] - S[m, 43]) / 100.0):.2f}, "
                  f"-> first sub-block {np.median((S[m, 36] - S[m, 44]) / 100.0):.2f}")
        for label, off in (("first", 32), ("latest", 0)):
            P = t[det]
            ok = (P[:, off + 4] > 0) & (P[:, off + 7] > 0)
            P = P[ok]
            if not len(P):
                continue
            start = us(P[:, off + 4])
            total = (P[:, off + 7] - P[:, off + 4]) / 100.0
            parts = []
            for a, b, nm in names:
                m = (P[:, off + a] > 0) & (P[:, off + b] > 0)
                if m.any():
                    parts.append(f"{nm} {np.median((P[m, off + b] - P[m, off + a]) / 100.0):.2f}")
            ch = P[:, off + 15]
            print(f"  wave 0's {label} sub-block: start p50 {np.median(start):.2f}, length p50 {np.median(total):.2f} "
                  f"p90 {np.percentile(total, 90):.2f}; chunks p50 {np.median(ch):.0f} p90 {np.percentile(ch, 90):.0f} "
                  f"max {ch.max()}")
            print(f"    phases p50 (us): " + ", ".join(parts))
        S = t[det]
        print(f"  shadow point-box test (wave 0, any sub-block): skipped in {(S[:, 32 + 20] > 0).sum()} of {len(S)} "
              f"detail workgroups, scan ran in {(S[:, 32 + 21] > 0).sum()}")
        hist, edges = np.histogram(us(t[det, 1]), bins=12)
        print("  detail end histogram:", " ".join(f"{e:.1f}:{h}" for e, h in zip(edges, hist)))
    if fil.any():
        f = us(t[fil, 3]) - us(t[fil, 2])
        print(f"  fill {fil.sum()}: start p50 {np.median(us(t[fil, 2])):.2f}, end p10 {np.percentile(us(t[fil, 3]), 10):.2f} "
              f"p50 {np.median(us(t[fil, 3])):.2f} p90 {np.percentile(us(t[fil, 3]), 90):.2f} max {us(t[fil, 3]).max():.2f}; "
              f"duration p50 {np.median(f):.2f} max {f.max():.2f}")

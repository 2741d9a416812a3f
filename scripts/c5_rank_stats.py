"""Per-rank anatomy of C5's 8-GPU band split on one GPU (diagnostics): for
each rank's share (interleaved 4-row bands every 32 rows) its hit pixels, detail sub-blocks, heavy
sub-blocks (bins of more than one 64-entry chunk), bin entries and (face, pixel) pairs, and its
frame kernel's dispatch-timed duration at 1 and 4 frames per launch.

    python scripts/c5_rank_stats.py [--world 8] [--launches 20]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from bench import frame_camera_fov  # noqa: E402
from eray_amd import capi, meshgen  # noqa: E402
from eray_amd.dist import band_split  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402


class CamStateHead(C.Structure):  # internal.hpp CamState's leading fields
    _fields_ = [("cam", C.c_float * 8), ("nrect", C.c_uint32), ("total_sub", C.c_uint32),
                ("bin_entries", C.c_uint32), ("bin_overflow", C.c_uint32), ("heavy_sub", C.c_uint32),
                ("light_sub", C.c_uint32), ("rects", C.c_int32 * 32)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--faces", type=int, default=1_000_000)
    ap.add_argument("--seed", type=int, default=1234)
    a = ap.parse_args()
    W, H = 7680, 4320
    path = os.path.join(tempfile.gettempdir(), f"standin_{a.faces}_{a.seed}.obj")
    if not os.path.exists(path):
        meshgen.generate(path, a.faces, a.seed)
    mesh = load_obj_file(path)
    lib = capi.lib()
    lib.eray_debug_bin_stats.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p]
    lib.eray_debug_setup_state.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p]
    ctx = capi.Context(0)
    MainScene(ctx, *mesh, W, H, texture=1024, fov=frame_camera_fov(W, H))
    out = {"frame": [W, H], "faces": a.faces, "world": a.world, "ranks": []}
    for r in range(a.world):
        sp = band_split(r, a.world, H, 4)
        rows = sp["rows"]
        rgb = ctx.empty((4, sp["alloc_rows"], W, 3), np.float32)
        ppm = ctx.empty((4, sp["alloc_rows"], W, 3), np.uint8)
        face = ctx.empty((sp["alloc_rows"], W), np.int32)
        kw = dict(row0=sp["row0"], rows=rows, band_rows=sp["band_rows"], band_stride=sp["band_stride"])
        ctx.render(W, H, out_rgb=rgb.ptr, out_face=face.ptr, **kw)
        ctx.synchronize()
        hits = int((face.numpy()[:rows] >= 0).sum())
        st = (C.c_uint64 * 14)()
        assert lib.eray_debug_bin_stats(ctx._h, 0, st) == 0
        cs = CamStateHead()
        rect = (C.c_int32 * 4)()
        assert lib.eray_debug_setup_state(ctx._h, 0, C.byref(cs), rect) == 0
        # this rank's own bin rows (camera rows 4 r + 32 k .. + 3; at phase 0 camera row y is in bin
        # row y / 4 + 1, internal.hpp / render.hip's bin index)
        nb = C.c_uint32()
        cnt = np.zeros(st[0], np.uint32)
        assert lib.eray_debug_bin_counts(ctx._h, 0, cnt.ctypes.data_as(C.POINTER(C.c_uint32)), int(st[0]), C.byref(nb)) == 0
        bins_x = (W + 15) // 16
        rows_b = cnt.reshape(-1, bins_x)
        mine = rows_b[r + 1::a.world]
        heavy = mine[mine > 64]
        times = {}
        for F in (1, 4):
            rkw = dict(kw, out_rgb=rgb.ptr, out_ppm=ppm.ptr)
            if F > 1:
                rkw["ring"] = capi.frame_ring(4, sp["alloc_rows"], W, 4)
            ctx.time_frames(2 * F, W, H, **rkw)
            t = ctx.time_frames(a.launches * F, W, H, **rkw)
            times[f"F{F}_us_per_frame"] = round(t["launch_span_ms"] * 1e3 / F, 2)
        rec = {"rank": r, "rows": rows, "hit_pixels": hits, "detail_sub_blocks": cs.total_sub,
               "heavy_bins": int(st[11]), "bin_entries": int(st[1]), "pairs": int(st[2]),
               "nonempty_bins": int(st[4]), "most_entries_in_a_bin": int(st[3]),
               "own_bins": {"entries": int(mine.sum()), "nonempty": int((mine > 0).sum()), "max_entries": int(mine.max()),
                            "over_64": int(heavy.size), "over_256": int((mine > 256).sum()),
                            "chunks_of_heaviest_10": sorted((((mine.ravel() + 63) // 64)).tolist())[-10:]}, **times}
        out["ranks"].append(rec)
        print(json.dumps(rec), flush=True)
        for x in (rgb, ppm, face):
            x.free()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

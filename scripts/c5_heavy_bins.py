"""Where a C5 share's heavy bins end (diagnostics): for one rank of the 8-GPU
band split, rendered alone on one GPU, every own bin of more than one 64-entry chunk is dumped
(eray_debug_bin_dump: faces in bin order, pixel masks) and replayed on the host against the
frame's first-hit faces: the chunk after which render.hip first_hit_binned_wave's sorted-bin exit
fires (no pixel whose best position is still ahead is covered by a later chunk's mask), and what
holds it there — a pixel whose winning face sits late in the bin, or a pixel no face hits that a
later face's mask still covers.

    python scripts/c5_heavy_bins.py [--rank 2] [--world 8] [--top 12]
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

KBINW, KBINH, SORT_MAX = 16, 4, 1024


def replay(tri: np.ndarray, mask: np.ndarray, win: np.ndarray) -> dict:
    """The sorted-bin search of one bin: tri / mask in bin order, win[p] = pixel p's first-hit face
    (-1: none).  Returns the chunks processed and, at the exit, the pixels that kept it going."""
    n = len(tri)
    nch = (n + 63) // 64
    pos_of = {int(f): i for i, f in enumerate(tri)}
    best = np.full(64, 1 << 30, np.int64)  # a pixel's winning position once its chunk is done
    winpos = np.array([pos_of.get(int(f), -1) if f >= 0 else -1 for f in win], np.int64)
    bits = (mask[:, None] >> np.arange(64, dtype=np.uint64)[None, :]) & np.uint64(1)
    cover = bits.astype(bool)  # [entry, pixel]
    searching = cover.any(axis=0) | (winpos >= 0)
    best[~searching] = -1
    done = nch
    held = None  # the pixels that kept the search going into its last processed chunk
    for c in range(nch):
        hi = min(64 * (c + 1), n)
        hit_here = (winpos >= 64 * c) & (winpos < hi)
        best[hit_here] = winpos[hit_here]
        if c + 1 == nch:
            break
        keep = (best > hi) & cover[hi:].any(axis=0)
        if not keep.any():
            done = c + 1
            break
        held = keep
    late = int((held & (winpos >= 0)).sum()) if held is not None else 0
    miss = int((held & (winpos < 0)).sum()) if held is not None else 0
    return {"entries": n, "chunks": nch, "processed": done, "late_winner_px": late, "masked_miss_px": miss,
            "pixels_hit": int((winpos >= 0).sum()), "winner_not_in_bin": int(((win >= 0) & (winpos < 0)).sum())}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=2)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--top", type=int, default=12)
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
    lib.eray_debug_bin_dump.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint32,
                                        C.c_void_p]
    ctx = capi.Context(0)
    MainScene(ctx, *mesh, W, H, texture=1024, fov=frame_camera_fov(W, H))
    sp = band_split(a.rank, a.world, H, 4)
    rgb = ctx.empty((sp["alloc_rows"], W, 3), np.float32)
    face = ctx.empty((sp["alloc_rows"], W), np.int32)
    ctx.render(W, H, out_rgb=rgb.ptr, out_face=face.ptr, row0=sp["row0"], rows=sp["rows"], band_rows=sp["band_rows"],
               band_stride=sp["band_stride"])
    ctx.synchronize()
    fimg = face.numpy()[:sp["rows"]]
    nb = C.c_uint32()
    st = (C.c_uint64 * 14)()
    assert lib.eray_debug_bin_stats(ctx._h, 0, st) == 0
    cnt = np.zeros(int(st[0]), np.uint32)
    assert lib.eray_debug_bin_counts(ctx._h, 0, cnt.ctypes.data_as(C.POINTER(C.c_uint32)), int(st[0]), C.byref(nb)) == 0
    bins_x = (W + KBINW - 1) // KBINW
    own = []
    for b in np.nonzero(cnt > 64)[0]:
        by, bx = divmod(int(b), bins_x)
        y0 = (by - 1) * KBINH  # camera rows of bin row by (phase 0)
        if y0 < 0 or (y0 - sp["row0"]) % sp["band_stride"]:
            continue
        own.append((int(cnt[b]), int(b), bx, y0))
    own.sort(reverse=True)
    recs = []
    for n, b, bx, y0 in own:
        tri = np.zeros(n, np.uint32)
        mask = np.zeros(n, np.uint64)
        got = C.c_uint32()
        assert lib.eray_debug_bin_dump(ctx._h, 0, b, tri.ctypes.data, mask.ctypes.data, n, C.byref(got)) == 0
        j0 = (y0 - sp["row0"]) // sp["band_stride"] * 4
        win = fimg[j0:j0 + KBINH, bx * KBINW:(bx + 1) * KBINW].reshape(-1).astype(np.int64)
        r = replay(tri.astype(np.int64), mask, win) if n <= SORT_MAX else {"entries": n, "unsorted": True}
        r.update(bin=b, x=bx * KBINW, y=y0)
        recs.append(r)
    chunks = np.array([r["chunks"] for r in recs if "chunks" in r])
    proc = np.array([r["processed"] for r in recs if "chunks" in r])
    summary = {"rank": a.rank, "heavy_own_bins": len(recs), "chunks_total": int(chunks.sum()),
               "chunks_processed": int(proc.sum()), "max_chunks": int(chunks.max()), "max_processed": int(proc.max()),
               "top": recs[:a.top]}
    print(json.dumps(summary), flush=True)
    for x in (rgb, face):
        x.free()


if __name__ == "__main__":
    main()

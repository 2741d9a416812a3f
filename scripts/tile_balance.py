"""Per-rank frame-kernel time of a multi-GPU row split, measured tile by tile on ONE GPU: each
rank's row block (eray_amd/dist.py row_block) rendered alone, graph-replayed and timed with HIP
events (eray_render_frames), for the weak-scaling bench frames (C2 widened to 1920N x 1080) and
the strong splits of C4 (cube 3840x2160 / 4) and C5 (1M faces 7680x4320 / 8).  Prints one JSON
line per workload: tile ms, max / mean (the slowest rank sets the frame time)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from bench import frame_camera_fov  # noqa: E402
from eray_amd import capi, meshgen  # noqa: E402
from eray_amd.dist import band_split, row_block  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402


def tiles(ctx, mesh, label, W, H, N, frames, split="blocks"):
    sc = MainScene(ctx, *mesh, W, H, texture=1024, fov=frame_camera_fov(W, H))
    rows = H // N if split == "blocks" else band_split(0, N, H)["alloc_rows"]
    rgb = ctx.empty((rows, W, 3), np.float32)
    ppm = ctx.empty((rows, W, 3), np.uint8)
    ms = []
    for r in range(N):
        if split == "blocks":
            row0, n = row_block(r, N, rows)
            kw = dict(row0=row0, rows=n, out_rgb=rgb.ptr, out_ppm=ppm.ptr)
        else:
            sp = band_split(r, N, H)
            kw = dict(row0=sp["row0"], rows=sp["rows"], band_rows=sp["band_rows"], band_stride=sp["band_stride"],
                      out_rgb=rgb.ptr, out_ppm=ppm.ptr)
        ctx.render_frames(frames, W, H, prepare_only=True, **kw)
        ctx.render_frames(frames, W, H, **kw)
        ms.append(ctx.render_frames(frames, W, H, timed=True, **kw))
    rgb.free()
    ppm.free()
    sc.close()
    mean = sum(ms) / len(ms)
    print(json.dumps({"workload": label, "split": split, "frame": [W, H], "ranks": N, "rows_per_rank": rows,
                      "tile_ms": [round(v, 6) for v in ms], "max_over_mean": round(max(ms) / mean, 4),
                      "max_ms": round(max(ms), 6)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--with-1m", action="store_true")
    a = ap.parse_args()
    ctx = capi.Context(0)
    cube = load_obj_file(os.path.join(ROOT, "objects", "cube.obj"))
    for split in ("blocks", "bands"):
        for n in (2, 4, 8):
            tiles(ctx, cube, f"C2 widened x{n} (weak scaling)", 1920 * n, 1080, n, 200, split)
            tiles(ctx, cube, f"C2 1920x1080 / {n} (strong scaling)", 1920, 1080, n, 200, split)
        tiles(ctx, cube, "C4 cube 3840x2160 / 4", 3840, 2160, 4, 200, split)
    tiles(ctx, cube, "C2 (one GPU)", 1920, 1080, 1, 200)
    tiles(ctx, cube, "C4 cube 3840x2160 (one GPU)", 3840, 2160, 1, 200)
    if a.with_1m:
        v, nn, t, fv, ft, fn = meshgen.displaced_sphere(**meshgen.SYNTH_1M)
        mesh = (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(nn[fn].reshape(-1, 9)),
                np.ascontiguousarray(t[ft].reshape(-1, 6)))
        for split in ("blocks", "bands"):
            tiles(ctx, mesh, "C5 1M 7680x4320 / 8", 7680, 4320, 8, 20, split)
        tiles(ctx, mesh, "C5 1M 7680x4320 (one GPU)", 7680, 4320, 1, 10)
    ctx.close()


if __name__ == "__main__":
    main()

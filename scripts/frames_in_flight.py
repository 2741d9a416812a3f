"""Diagnostics: frames in flight.  Per-frame device time (HIP events around K graph-replayed
frames, eray_render_frames_ring) for 1, 2, 4, 8 frames per launch into an 8-slot ring, on the
BASELINE workloads and on one rank's share of a strong split (interleaved bands)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import frame_camera_fov  # noqa: E402
from eray_amd import capi  # noqa: E402
from eray_amd.dist import band_split  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402


def run(ctx, label, mesh, W, H, K, per_launch=((1, 1), (2, 2), (4, 4), (8, 8), (8, 16)), ranks=1, material="textures"):
    sc = MainScene(ctx, *mesh, W, H, texture=1024, fov=frame_camera_fov(W, H), material=material)
    kw = {}
    rows = H
    if ranks > 1:
        sp = band_split(0, ranks, H)
        kw = dict(row0=sp["row0"], rows=sp["rows"], band_rows=sp["band_rows"], band_stride=sp["band_stride"])
        rows = sp["rows"]
    most = max(s for _, s in per_launch)
    rgb = torch.empty((most, rows, W, 3), dtype=torch.float32, device="cuda")
    ppm = torch.empty((most, rows, W, 3), dtype=torch.uint8, device="cuda")
    out = {"workload": label, "frame": [W, H], "rows": rows, "ranks": ranks, "material": material,
           "us_per_frame [events, wall] by frames per launch / ring slots": {}}
    for F, slots in per_launch:
        ring = capi.frame_ring(slots, rows, W, F)
        args = dict(out_rgb=rgb.data_ptr(), out_ppm=ppm.data_ptr(), ring=ring, **kw)
        ctx.render_frames(K, W, H, prepare_only=True, **args)
        ctx.render_frames(K, W, H, **args)
        best = min(ctx.render_frames(K, W, H, timed=True, **args) for _ in range(3))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.render_frames(K, W, H, **args)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / K
        out["us_per_frame [events, wall] by frames per launch / ring slots"][f"{F}/{slots}"] = [
            round(best * 1e3, 3), round(wall * 1e6, 3)]
    print(json.dumps(out), flush=True)
    sc.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true", help="also the 70k-face stand-in")
    a = ap.parse_args()
    ctx = capi.Context(0)
    st = torch.cuda.Stream()
    ctx.set_stream(st.cuda_stream)
    torch.cuda.set_stream(st)
    cube = load_obj_file(os.path.join(ROOT, "objects", "cube.obj"))
    run(ctx, "C2", cube, 1920, 1080, 256)
    for n in (2, 4, 8):
        run(ctx, f"C2 / {n} (rank 0's bands)", cube, 1920, 1080, 256, ranks=n,
            per_launch=((1, 1), (4, 4), (8, 8), (16, 16), (32, 32)))
    run(ctx, "C4 cube 3840x2160 on one GPU", cube, 3840, 2160, 64, per_launch=((1, 1), (1, 8), (2, 2)))
    if a.big:
        big = load_obj_file("/tmp/eray_meshes/standin70k.obj")
        run(ctx, "C3", big, 1920, 1080, 128)
        run(ctx, "70k 3840x2160", big, 3840, 2160, 64, per_launch=((1, 1), (1, 8), (2, 2)))
    ctx.close()


if __name__ == "__main__":
    main()

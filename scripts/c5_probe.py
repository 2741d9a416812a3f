"""C5's frame on one GPU (1M-face stand-in, 7680x4320) and one rank's band share of the 8-GPU
split, timed per dispatch (eray_time_frames_ring: frame kernel, separate fill kernel, span), under
each launch shape the flags allow.  Diagnostics for DESIGN.md §5 / §7 (not the bench).

    python scripts/c5_probe.py [--faces 1000000] [--seed 1234] [--launches 10] [--shares 0,3,7]

The mesh is generated once into $TMPDIR (eray_amd.meshgen; SURVEY.md §8(d): seed 1234)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (one HIP runtime: torch's)

from eray_amd import capi, meshgen  # noqa: E402
from eray_amd.dist import band_split  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--faces", type=int, default=1_000_000)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--height", type=int, default=4320)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--shares", default="0,3,7")
    ap.add_argument("--no-full", action="store_true", help="skip the full frame (profiling one share)")
    ap.add_argument("--shapes", default="default,separate_fill,single_launch",
                    help="comma-separated launch shapes to time")
    ap.add_argument("--no-empty", action="store_true", help="skip the empty-scene fill")
    args = ap.parse_args()
    W, H = args.width, args.height
    path = os.path.join(tempfile.gettempdir(), f"standin_{args.faces}_{args.seed}.obj")
    t0 = time.perf_counter()
    if not os.path.exists(path):
        meshgen.generate(path, args.faces, args.seed)
    mesh = load_obj_file(path)
    gen = time.perf_counter() - t0
    ctx = capi.Context(0)
    st = torch.cuda.Stream()
    ctx.set_stream(st.cuda_stream)
    sc = MainScene(ctx, *mesh, W, H, texture=1024, fov=(16.0, 9.0))
    rgb = ctx.empty((H, W, 3), "float32")
    ppm = ctx.empty((H, W, 3), "uint8")
    out = {"mesh_s": round(gen, 2), "frame": [W, H], "faces": int(len(mesh[0]))}
    shapes = {"default": capi.RENDER_DEFAULT, "separate_fill": capi.RENDER_DENSE_DETAIL | capi.RENDER_SEPARATE_FILL,
              "single_launch": capi.RENDER_DENSE_DETAIL | capi.RENDER_NO_SEPARATE_FILL}
    shapes = {k: v for k, v in shapes.items() if k in args.shapes.split(",")}
    for name, flags in (() if args.no_full else shapes.items()):
        kw = dict(out_rgb=rgb.ptr, out_ppm=ppm.ptr, flags=flags)
        ctx.render(W, H, **kw)
        ctx.synchronize()
        out[f"full_{name}"] = ctx.time_frames(args.launches, W, H, **kw)
    for r in [int(x) for x in args.shares.split(",") if x]:
        sp = band_split(r, args.world, H, 4)
        for name, flags in shapes.items():
            kw = dict(row0=sp["row0"], rows=sp["rows"], band_rows=sp["band_rows"], band_stride=sp["band_stride"],
                      out_rgb=rgb.ptr, out_ppm=ppm.ptr, flags=flags)
            ctx.render(W, H, **kw)
            ctx.synchronize()
            out[f"share{r}of{args.world}_{name}"] = ctx.time_frames(args.launches, W, H, **kw)
    if not args.no_empty:
        empty = capi.Context(0)  # the same camera, no object: the fill alone (this kernel's write floor)
        empty.set_stream(st.cuda_stream)
        empty.set_camera(capi.make_camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0))
        empty.add_light(capi.make_light((1.0, 1.0, 2.0), "point"))
        empty.render(W, H, out_rgb=rgb.ptr, out_ppm=ppm.ptr)
        empty.synchronize()
        out["full_empty_scene"] = empty.time_frames(args.launches, W, H, out_rgb=rgb.ptr, out_ppm=ppm.ptr)
        empty.close()
    rgb.free()
    ppm.free()
    sc.close()
    ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

"""Camera-path frames against static frames on the same camera (diagnostics): a path of n copies
of the scene camera, the dolly path, and the static frames, through one ring slot — device ms per
frame (path: eray_render_camera_path_ring timed; static: graph-replayed frames).  Run each mode
in its own process under rocprofv3 --kernel-trace to read the frame kernel's own durations.

    python scripts/path_still_probe.py --mode still|dolly|static [--mesh 70k] [--frames 32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import dolly_path, frame_camera_fov  # noqa: E402
from eray_amd import capi  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from scripts.ab_probe import mesh_of  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("still", "dolly", "static"), required=True)
    ap.add_argument("--mesh", default="70k")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--frames", type=int, default=32)
    args = ap.parse_args()
    W, H, n = args.width, args.height, args.frames
    st = torch.cuda.Stream()
    ctx = capi.Context(0)
    ctx.set_stream(st.cuda_stream)
    fov = frame_camera_fov(W, H)
    sc = MainScene(ctx, *mesh_of(args.mesh), W, H, texture=1024, fov=fov)
    with torch.cuda.stream(st):
        rgb = torch.empty((1, H, W, 3), dtype=torch.float32, device="cuda")
        ppm = torch.empty((1, H, W, 3), dtype=torch.uint8, device="cuda")
    kw = dict(out_rgb=rgb.data_ptr(), out_ppm=ppm.data_ptr(), ring=capi.frame_ring(1, H, W, 1))
    if args.mode == "static":
        ctx.render_frames(n, W, H, **kw)
        ms = min(ctx.render_frames(n, W, H, timed=True, **kw) for _ in range(3))
    else:
        path = ([capi.make_camera((0.0, 0.0, 5.0), fov, W, 1.0) for _ in range(n)] if args.mode == "still"
                else dolly_path(n, fov, W))
        ctx.render_camera_path(path, W, H, **kw)
        ms = min(ctx.render_camera_path(path, W, H, timed=True, **kw) for _ in range(3))
    torch.cuda.synchronize()
    print(json.dumps({"mode": args.mode, "mesh": args.mesh, "frame": [W, H], "frames": n,
                      "device_us_per_frame": round(ms * 1e3, 2)}), flush=True)
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()

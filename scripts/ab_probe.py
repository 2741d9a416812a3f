"""Same-box A/B of library builds (diagnostics): each configuration's frame kernel timed per
dispatch (eray_time_frames_ring) with the library ERAY_LIB selects.  Run once per build, alternating
(scripts/ab_session.sh); prints one JSON line.

    ERAY_LIB=eray_amd/lib/liberay_hip_base.so python scripts/ab_probe.py [--configs c2,ns1,ns4]

Configs: c2 (cube 1920x1080, 8 frames per launch into 8 slots), c3 (70k stand-in 1920x1080, 4
per launch), ns1 / ns4 (70k stand-in 3840x2160, one frame per launch, 1 / 4 ring slots), c5
(1M faces 7680x4320), moving_ns (a moving camera over the 70k stand-in at 3840x2160), aa2 / aa_ns
(anti-aliasing = 4 through the general tracer: C2, the 70k stand-in at 3840x2160; graph-replayed
frames, device ms per frame), fill* (the same camera and lights, no object), ceil* (the
write ceiling of the fill* rings: eray_time_write_ceiling), mat (main.rs's
Material::update of a 1024 x 1024 texture, bench.py material_roofline)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import dolly_path, frame_camera_fov  # noqa: E402
from eray_amd import capi, meshgen  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402

MESHES = {"cube": None, "70k": (69451, 42), "1m": (1_000_000, 1234)}
CONFIGS = {"fill4k1": ("none", 3840, 2160, 1, 1), "fill4k4": ("none", 3840, 2160, 4, 1),
           "fill8k": ("none", 7680, 4320, 1, 1), "fillc2": ("none", 1920, 1080, 8, 8),
           # the plain block-strided store stream into the same rings (eray_time_write_ceiling)
           "ceil4k1": ("none", 3840, 2160, 1, 1), "ceil4k4": ("none", 3840, 2160, 4, 1),
           "ceilc2": ("none", 1920, 1080, 8, 8), "ceilc2b": ("none", 1920, 1080, 16, 8),
           "c2": ("cube", 1920, 1080, 8, 8), "c2b": ("cube", 1920, 1080, 16, 8), "c3": ("70k", 1920, 1080, 4, 4), "c3dense": ("70k", 1920, 1080, 4, 4), "c3nodense": ("70k", 1920, 1080, 4, 4), "ns1": ("70k", 3840, 2160, 1, 1),
           "ns4": ("70k", 3840, 2160, 4, 1), "c5": ("1m", 7680, 4320, 1, 1), "moving_ns": ("70k", 3840, 2160, 1, 1),
           "moving_c5": ("1m", 7680, 4320, 1, 1),
           "aa2": ("cube", 1920, 1080, 1, 1), "aa_ns": ("70k", 3840, 2160, 1, 1),
           "ns1sep": ("70k", 3840, 2160, 1, 1), "ns4sep": ("70k", 3840, 2160, 4, 1),
           "ns1ex": ("70k", 3840, 2160, 1, 1), "ns4ex": ("70k", 3840, 2160, 4, 1), "c2ex": ("cube", 1920, 1080, 8, 8),
           "mat": ("cube", 1920, 1080, 1, 1),
           # C5's 8-GPU split on one GPU: rank r's share (row0 = 4r, 4-row bands every 32 rows)
           **{f"c5s{r}": ("1m", 7680, 4320, 1, 1) for r in range(8)},
           # ... with frames in flight: 4 frames per launch into 4 slots (and the whole frame, 2 per launch)
           **{f"c5s{r}f4": ("1m", 7680, 4320, 4, 4) for r in range(8)}, "c5f2": ("1m", 7680, 4320, 2, 2)}
# launch-shape overrides (eray_render_params::flags) of the *sep configs: the dense build beside a
# separate fill kernel
SEPARATE = ("ns1sep", "ns4sep")


def mesh_of(kind):
    if kind == "cube":
        return load_obj_file(os.path.join(ROOT, "objects", "cube.obj"))
    faces, seed = MESHES[kind]
    path = os.path.join(tempfile.gettempdir(), f"standin_{faces}_{seed}.obj")
    if not os.path.exists(path):
        meshgen.generate(path, faces, seed)
    return load_obj_file(path)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c3,ns1,ns4")
    ap.add_argument("--launches", type=int, default=40)
    args = ap.parse_args()
    out = {"lib": os.path.basename(capi.LIB_PATH)}
    st = torch.cuda.Stream()
    for name in args.configs.split(","):
        kind, W, H, slots, F = CONFIGS[name]
        ctx = capi.Context(0)
        ctx.set_stream(st.cuda_stream)
        if kind == "none":  # the same camera and lights, no object: the fill alone
            from bench import empty_scene_context
            ctx.close()
            ctx = empty_scene_context(0, W, H, frame_camera_fov(W, H), st)
            sc = None
        else:
            # (*ex: main.rs's graph evaluated at the hit texel, eray_scene_set_object_example_material:
            # bit-identical frames, no texture reads)
            sc = MainScene(ctx, *mesh_of(kind), W, H, texture=1024, fov=frame_camera_fov(W, H),
                           material="example" if name.endswith("ex") else "textures")
        with torch.cuda.stream(st):
            rgb = torch.empty((slots, H, W, 3), dtype=torch.float32, device="cuda")
            ppm = torch.empty((slots, H, W, 3), dtype=torch.uint8, device="cuda")
        kw = dict(out_rgb=rgb.data_ptr(), out_ppm=ppm.data_ptr(), ring=capi.frame_ring(slots, H, W, F))
        if name.startswith("c5s"):
            from eray_amd.dist import band_split
            sp = band_split(int(name[3]), 8, H, 4)
            kw.update(row0=sp["row0"], rows=sp["rows"], band_rows=sp["band_rows"], band_stride=sp["band_stride"])
            if F == 1:
                del kw["ring"]
        if name in SEPARATE:
            kw["flags"] = capi.RENDER_DENSE_DETAIL | capi.RENDER_SEPARATE_FILL
        elif name.endswith("nodense"):  # launch-shape overrides: the 2-per-CU / dense detail builds
            kw["flags"] = capi.RENDER_NO_DENSE_DETAIL
        elif name.endswith("dense"):
            kw["flags"] = capi.RENDER_DENSE_DETAIL
        if name.startswith("ceil"):
            ctx.time_write_ceiling(2 * F, W, H, **kw)
            out[name] = ctx.time_write_ceiling(max(args.launches, 2) * F, W, H, **kw)
        elif name == "mat":
            from bench import material_roofline
            out[name] = {"frame_ms": min(material_roofline(sc, st, reps=50)["us_per_update"] for _ in range(3)) / 1e3}
        elif name.startswith("aa"):  # the general tracer, anti_aliasing = 4 (bench.py anti_aliasing_line)
            akw = dict(kw, anti_aliasing=4, aa_seed=12345)
            del akw["ring"]
            ctx.render_frames(20, W, H, prepare_only=True, **akw)
            out[name] = {"frame_ms": min(ctx.render_frames(20, W, H, timed=True, **akw) for _ in range(3))}
        elif name.startswith("moving"):
            path = dolly_path(32, frame_camera_fov(W, H), W)
            ctx.render_camera_path(path, W, H, **kw)
            out[name] = {"device_ms_per_frame": min(ctx.render_camera_path(path, W, H, timed=True, **kw)
                                                    for _ in range(3))}
        else:
            ctx.render_frames(max(slots, 4), W, H, **kw)
            ctx.time_frames(2 * F, W, H, **kw)  # (warm: a first launch after the setup can take ms)
            n = max(args.launches // (4 if name.startswith("c5") and "s" not in name else 1), 2) * F
            out[name] = ctx.time_frames(n, W, H, **kw)
        torch.cuda.synchronize()
        del rgb, ppm
        if sc:
            sc.close()
        ctx.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

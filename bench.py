#!/usr/bin/env python3
"""Benchmark of the eray ray-tracing hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]): objects/cube.obj with src/main.rs's scene
and material graph, 1920x1080 per GPU.  One step = one frame (camera rays, first-hit triangle
scan, shading with shadow rays) with the f32 image and the PPM bytes written by the fused kernel.

Multi-GPU (row tiles).  Default, weak scaling: N GPUs render a (1920*N) x 1080
frame — C2 widened at the same pixel pitch (the camera's Fov ratio grows with the width, the
viewport height and focal length stay main.rs's), so every rank renders 1080/N rows of 1920*N
pixels, the same 2,073,600 rays per GPU, and N = 1 is exactly C2.  --scaling strong splits one
fixed --width x --height frame (C4, C5) instead.  For N > 1 the job ends with the final RCCL
gather (xGMI) of the PPM rows to rank 0 inside the timed region (north_star: "a final RCCL
gather"); --gather-every-frame gathers after every frame instead.  Inputs (mesh, material
textures) are resident in HBM before timing; the material graph is evaluated once, as
Material::update is (reported separately).

The headline `value` replays frames of ONE camera (static camera: the per-camera setup — culling
records, pixel rectangles, screen bins — runs once before the timed region, as it would for a
serving loop that renders the same view).  `moving_camera` reports the same frames with a camera
that moves every frame (a dolly along the view axis: Scene::set_camera + Engine::render per
frame), every frame's setup on the device inside the timed frames (eray_render_camera_path).

--scaling weak widens the frame with N (C2's pixel pitch, not a BASELINE.json config); --scaling
strong splits BASELINE's fixed frames (C4: --width 3840 --height 2160, C5: 7680x4320).

Prints ONE JSON line on rank 0 (metric "Mrays/s": primary rays of all ranks / wall time).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (imported before the HIP library: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

from eray_amd import capi  # noqa: E402
from eray_amd.dist import BAND_ROWS, RowGather, band_split, gather_ppm_rows, row_block  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402

WIDTH, HEIGHT, TEXTURE = 1920, 1080, 1024  # C2 (defaults; --width / --height)
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_VALU_TOPS = 78.6  # non-FMA FP32 VALU: 256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz


def frame_camera_fov(width: int, height: int) -> tuple[float, float]:
    """Fov giving Camera::size() == (width, height) exactly: Fov(16, 9) for 16:9 frames (SURVEY.md
    §8), Fov(60, 60) for square ones, otherwise Fov(width, height) with fov1 nudged by a few ulps
    until (width as f32 / (fov0 / fov1)) as u32 == height."""
    cands = [(16.0, 9.0), (60.0, 60.0)]
    f1 = np.float32(height)
    for _ in range(8):
        cands += [(float(width), float(f1))]
        f1 = np.nextafter(f1, np.float32(np.inf))
    f1 = np.float32(height)
    for _ in range(8):
        f1 = np.nextafter(f1, np.float32(0))
        cands += [(float(width), float(f1))]
    for fov in cands:
        cam = capi.make_camera((0.0, 0.0, 5.0), fov, width, 1.0)
        if capi.camera_size(cam) == (width, height):
            return fov
    raise RuntimeError(f"no Fov gives a {width}x{height} camera")


def algorithmic_bytes(hit_pixels: int, pixels: int, triangles: int) -> int:
    """Bytes the render kernel must move per launch:
    15 B/pixel written (12 B f32 RGB + 3 B PPM), 16 B of texels read per hit (IColor 12 + IValue 4),
    and the triangle records once (48 B hot + 64 B culling + 64 B shading)."""
    return 15 * pixels + 16 * hit_pixels + (48 + 64 + 64) * triangles


def pmc_record(workload: dict):
    """The committed rocprofv3 counter summary of this workload's frame kernel
    (scripts/pmc_traffic.py): profiles/pmc_traffic*.json whose "workload" (mesh, frame, rows per
    GPU, GPUs) equals this run's, or None when no summary of this workload is committed."""
    # the newest round's summaries first (profiles/rNN/pmc_traffic*.json), then older ones
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic*.json")), reverse=True)
    for path in paths + sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic*.json"))):
        try:
            with open(path) as f:
                rec = json.load(f)
            if rec.get("workload") == workload and "frame_kernel" in rec:
                return rec["frame_kernel"]
        except (OSError, KeyError, ValueError):
            continue
    return None


def counter_figures(rec, kernel_ms: float) -> dict:
    """From a counter summary: HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, the gfx950
    correction of MI355X_MICROARCH.md), the HBM-read fraction (north_star's figure: corrected fetch
    bytes / kernel time / peak) and the VALU fraction (SURVEY.md §8(d)'s binding figure for the
    intersection: SQ_INSTS_VALU x 64 lanes / kernel time / the 78.6 T ops/s non-FMA FP32 peak; it
    counts every VALU instruction of the frame kernel — rays, tests, shading, fill addressing)."""
    if not rec:
        return {"traffic": None}
    out = {"traffic": int(rec["hbm_bytes_per_launch"])}
    sec = kernel_ms * 1e-3
    fetch = rec.get("fetch_bytes_corrected")
    if fetch is not None and sec > 0:
        gbs = fetch / sec / 1e9
        out["hbm_read"] = {"achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                           "frac": round(gbs / PEAK_HBM_GBS, 4), "bytes_per_launch": int(fetch)}
    valu = rec.get("counters_mean_per_dispatch", {}).get("SQ_INSTS_VALU")
    if valu is not None and sec > 0:
        tops = valu * 64 / sec / 1e12
        out["valu"] = {"achieved": round(tops, 2), "peak": PEAK_VALU_TOPS, "unit": "TOP/s",
                       "frac": round(tops / PEAK_VALU_TOPS, 4), "instructions_per_launch": int(valu)}
    return out


def host_cpu() -> tuple[int, str]:
    """(logical CPUs of this host, CPU model name) for the cpu_baseline record."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return os.cpu_count() or 0, model


def dolly_path(n: int, fov, width: int):
    """n cameras moving along the view axis (main.rs's camera at (0, 0, 5) +- 0.5, z_dist 1 +- 0.1):
    every frame a new camera with the same Camera::size.  A loaded mesh's bounding box is the
    degenerate (0,0,0) box (object.rs:306-315), which only rays from x = y = 0 pass, so the
    reference's own semantics keep the camera on the axis."""
    import math
    return [capi.make_camera((0.0, 0.0, 5.0 + 0.5 * math.sin(2.0 * math.pi * k / max(n, 1))), fov, width,
                             1.0 + 0.1 * math.cos(2.0 * math.pi * k / max(n, 1))) for k in range(n)]


def cpu_baseline(mesh, width: int, height: int, fov, seconds: float = 10.0) -> dict:
    """The single-threaded C++ restatement (oracle/, 'port') on this host, on the bench's own
    frame (width x height, same scene): whole frames (render + PPM byte pack) repeated for
    >= `seconds` when a frame takes under a second (the cube), otherwise a deterministic row
    sample — every 64th row, then the rows between — until `seconds` have passed."""
    from oracle import pyoracle as O

    scene = O.main_rs_scene(*mesh, texture=TEXTURE)
    cam = O.camera((0.0, 0.0, 5.0), fov, width, 1.0)
    t0 = time.perf_counter()
    rgb, _ = O.render(scene, cam, rows=1, row0=height // 2)  # one row: decide frames vs rows
    one_row = time.perf_counter() - t0
    if one_row * height < 1.0:
        frames, t0 = 0, time.perf_counter()
        while True:
            rgb, _ = O.render(scene, cam)
            O.ppm_bytes(rgb)
            frames += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
        rays = frames * width * height
        sample = f"{frames} full {width}x{height} frames (main.rs scene, render + PPM pack) in {el:.1f} s"
    else:
        order = [r for s in range(64) for r in range(s, height, 64)]
        done, t0 = 0, time.perf_counter()
        for r in order:
            O.render(scene, cam, row0=height - 1 - r, rows=1)
            done += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
        rays = done * width
        sample = (f"{done} of the {height} rows of the {width}x{height} frame (every 64th row first), "
                  f"render only, in {el:.1f} s")
    nproc, model = host_cpu()
    return {"value": rays / el / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "port",
            "nproc": nproc, "cpu_model": model,
            "sample": sample + ", single thread, oracle/eray_oracle.cpp (g++ -O2 -ffp-contract=off)"}


def mesh_label(path: str) -> str:
    """The mesh as the JSON line names it: repo-relative when it is in the tree, else the file name
    (meshes generated on the box by eray_amd.meshgen)."""
    rel = os.path.relpath(path, ROOT)
    return os.path.basename(path) if rel.startswith("..") else rel


def moving_camera(scene, args, width, height, render_args, world, allreduce) -> dict:
    """The bench's frames with a camera that moves every frame (dolly_path): eray_render_camera_path
    runs every frame's camera setup on the device inside the timed loop.  Returns the moving_camera record."""
    path = dolly_path(args.steps, frame_camera_fov(width, height), width)
    scene.ctx.render_camera_path(path, width, height, **render_args())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    m0 = time.perf_counter()
    scene.ctx.render_camera_path(path, width, height, **render_args())
    torch.cuda.synchronize()
    moving_s = time.perf_counter() - m0
    if world > 1:
        moving_s = float(allreduce(moving_s, torch.float64, dist.ReduceOp.MAX))
    device_ms = scene.ctx.render_camera_path(path, width, height, timed=True, **render_args())
    return {
        "frame_ms": round(moving_s / args.steps * 1e3, 6),
        "value": round(width * height * args.steps / moving_s / 1e6, 3),
        "unit": "Mrays/s",
        "device_ms_per_frame": round(device_ms, 6),
        "frames": args.steps,
        "camera": "dolly along the view axis, z 5 +- 0.5, z_dist 1 +- 0.1, a new camera every frame",
        "includes": "every frame's camera setup on the device (culling records, pixel rectangles, merged "
                    "detail rectangles: for scenes without meshes over 256 faces one launch sets up a graph "
                    "chunk's 64 cameras, one workgroup per camera; otherwise per frame, with the screen bins "
                    "and detail list) + frame",
    }


AA_SAMPLES = 4
AA_MAX_TRIANGLES = 4096  # the general tracer scans every face per ray: small scenes only


def anti_aliasing_line(scene, args, width, height, render_args) -> dict:
    """The general tracer (trace.hip: anti-aliasing, engine.rs:59-77) on the bench's frames:
    AA_SAMPLES jittered rays per pixel plus the centre ray, every face scanned per ray.  Device
    time per frame over graph-replayed frames; rays counted as the reference casts them."""
    frames = max(2, min(args.steps, 20))
    kw = dict(render_args(), anti_aliasing=AA_SAMPLES, aa_seed=12345)
    scene.ctx.render_frames(frames, width, height, prepare_only=True, **kw)
    ms = scene.ctx.render_frames(frames, width, height, timed=True, **kw)
    rays = width * height * (AA_SAMPLES + 1)
    return {"anti_aliasing": AA_SAMPLES, "frames": frames, "frame_ms": round(ms, 6),
            "value": round(rays / (ms * 1e-3) / 1e6, 3), "unit": "Mrays/s (all AA rays)",
            "kernel": "trace_kernel (eray_amd/csrc/trace.hip): waves no camera ray of which can reach a face skip the scan (culling records), the rest brute force per ray"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--mesh", default=os.path.join(ROOT, "objects", "cube.obj"))
    ap.add_argument("--width", type=int, default=WIDTH,
                    help="frame width per GPU (weak) or of the whole frame (strong); C2: 1920")
    ap.add_argument("--height", type=int, default=HEIGHT, help="frame height (C2: 1080)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="weak: a (width*N) x height frame; strong: one width x height frame split N ways")
    ap.add_argument("--brute-force", action="store_true", help="disable the exact wave culling")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-moving-camera", action="store_true", help="skip the moving-camera line (counter runs)")
    ap.add_argument("--split", choices=("bands", "blocks"), default="bands",
                    help="N > 1: interleaved 4-row bands (balanced, default) or contiguous row blocks")
    ap.add_argument("--gather-every-frame", action="store_true",
                    help="N > 1: gather the PPM rows to rank 0 after every frame (default: one final gather)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # ERAY_BENCH_REHEARSAL=1 rehearses the N > 1 path on ONE GPU: every rank on device 0, gloo
    # collectives through host memory (RCCL will not put two ranks on one device).  Never used
    # for a reported number.
    rehearsal = os.environ.get("ERAY_BENCH_REHEARSAL") == "1"
    device = 0 if rehearsal else local_rank
    torch.cuda.set_device(device)
    if world > 1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))

    def allreduce(value, dtype, op):
        t = torch.tensor([value], dtype=dtype, device="cpu" if rehearsal else "cuda")
        dist.all_reduce(t, op=op)
        return t.item()

    mesh = load_obj_file(args.mesh)
    ctx = capi.Context(device)
    stream = torch.cuda.Stream()  # one stream shared by the library, torch and RCCL
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    width = args.width * world if args.scaling == "weak" else args.width
    H_total = args.height
    if H_total % world:
        raise SystemExit(f"--height {H_total} does not split into {world} equal row tiles")
    per_gpu = H_total // world
    t_mat0 = time.perf_counter()
    scene = MainScene(ctx, *mesh, width, H_total, texture=TEXTURE, fov=frame_camera_fov(width, H_total))
    torch.cuda.synchronize()
    t_mat = time.perf_counter() - t_mat0

    # rank r renders interleaved 4-row bands r, r + N, ... (every rank an equal share of the scene
    # wherever it sits; tile timings in DESIGN.md §7) or, --split blocks, the r-th block of PPM file
    # rows: camera rows [H - (r+1)*h, H - r*h)
    bands = world > 1 and args.split == "bands"
    if bands:
        sp = band_split(rank, world, H_total, BAND_ROWS)
        row0, rows, alloc_rows = sp["row0"], sp["rows"], sp["alloc_rows"]
        band_args = dict(band_rows=sp["band_rows"], band_stride=sp["band_stride"])
    else:
        row0, rows = row_block(rank, world, per_gpu)
        alloc_rows, band_args = rows, {}
    rgb = torch.empty((alloc_rows, width, 3), dtype=torch.float32, device="cuda")
    ppm = torch.zeros((alloc_rows, width, 3), dtype=torch.uint8, device="cuda")
    face = torch.empty((alloc_rows, width), dtype=torch.int32, device="cuda")
    frame = torch.empty((H_total, width, 3), dtype=torch.uint8, device="cuda") if rank == 0 else None
    flags = capi.RENDER_BRUTE_FORCE if args.brute_force else capi.RENDER_DEFAULT
    # N > 1: the frame gather of the C-ABI (eray_gather_rows, RCCL ncclGather over xGMI); the
    # one-GPU rehearsal gathers through gloo instead
    band = BAND_ROWS if bands else 0
    if world > 1 and not rehearsal:
        rccl = RowGather(ctx, world, rank)

        def gather():
            rccl(ppm, frame, H_total, band)
    elif world > 1:
        def gather():
            gather_ppm_rows(ppm, frame, world, rank, band_rows=band)

    def render_args():
        return dict(row0=row0, rows=rows, out_rgb=rgb.data_ptr(), out_ppm=ppm.data_ptr(), flags=flags, **band_args)

    # one untimed instrumented frame: hit count for the algorithmic-bytes model; being the first
    # render of the camera it also builds the per-camera data (culling records, pixel
    # rectangles, screen bins of large meshes): reported as scene_setup_ms
    torch.cuda.synchronize()
    t_setup0 = time.perf_counter()
    face.fill_(-1)
    scene.ctx.render(width, H_total, out_rgb=rgb.data_ptr(), out_face=face.data_ptr(), row0=row0, rows=rows,
                     flags=flags, **band_args)
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t_setup0
    hits = int((face[:rows] >= 0).sum().item())

    # capture the frame-loop graph, then the W warmup frames through the same replayed path as
    # the timed ones (and the gather warmed) outside the timed region
    scene.ctx.render_frames(args.steps, width, H_total, prepare_only=True, **render_args())
    if args.warmup:
        scene.ctx.render_frames(args.warmup, width, H_total, **render_args())
    if world > 1:
        gather()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # every rank renders its row tile of each frame; the frame loop runs inside the library,
    # replayed from a HIP graph (no per-frame host round trip)
    if args.gather_every_frame and world > 1:
        for _ in range(args.steps):
            scene.render(**render_args())
            gather()
    else:
        scene.ctx.render_frames(args.steps, width, H_total, **render_args())
        if world > 1:  # the final RCCL gather of the PPM rows to rank 0 (file order)
            gather()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = float(allreduce(elapsed, torch.float64, dist.ReduceOp.MAX))
        hits_all = int(allreduce(hits, torch.int64, dist.ReduceOp.SUM))
    else:
        hits_all = hits
    # the frame kernel's duration: the same frames replayed once more, bracketed by HIP events on
    # the library's stream (back-to-back kernels: device time per frame)
    kernel_ms = scene.ctx.render_frames(args.steps, width, H_total, timed=True, **render_args())
    gather_ms = None
    rank_kernel_ms = [kernel_ms]
    if world > 1:  # one frame's gather, and every rank's frame-kernel time, for the record
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        gather()
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3
        got = [None] * world
        dist.all_gather_object(got, kernel_ms)
        rank_kernel_ms = got

    # moving camera: the same frames with a new camera every frame (the setup on the device,
    # inside each frame); one untimed pass captures the path's graphs
    moving = None if args.no_moving_camera else moving_camera(scene, args, width, H_total, render_args, world, allreduce)
    # the general tracer (anti-aliasing) on the same frames, rank 0 of one GPU, small scenes
    aa_line = None
    if world == 1 and not args.no_moving_camera and len(mesh[0]) <= AA_MAX_TRIANGLES:
        aa_line = anti_aliasing_line(scene, args, width, H_total, render_args)

    if rank == 0:
        # the workload a committed counter summary (profiles/pmc_traffic*.json) must match
        pmc_key = {"mesh": mesh_label(args.mesh), "frame": [width, H_total], "rows_per_gpu": rows,
                   "n_gpus": world, "brute_force": bool(args.brute_force)}
        is_c2 = (args.width, args.height, args.scaling) == (WIDTH, HEIGHT, "weak") and args.mesh.endswith(
            "objects/cube.obj") and not args.brute_force
        pixels = width * rows
        ms_per_step = elapsed / args.steps * 1e3
        rays = width * H_total * args.steps
        value = rays / elapsed / 1e6
        alg = algorithmic_bytes(hits, pixels, len(mesh[0]))
        achieved = alg / (kernel_ms * 1e-3) / 1e9
        result = {
            "metric": "Mrays/s",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 6),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": (f"synthetic scene of src/main.rs around {mesh_label(args.mesh)}"
                     + (" (the reference's own file)" if args.mesh.endswith("objects/cube.obj") else "")
                     + ", procedural material graph"),
            "config": {
                "workload": f"{'C2' + (f' widened x{world}' if world > 1 else '') + ': ' if is_c2 else ''}"
                            f"{os.path.basename(args.mesh)}, {width}x{H_total} frame, {width}x{per_gpu} rows per GPU, "
                            "main.rs scene + material graph; step = one frame (camera rays, first-hit scan, "
                            "shading + shadow rays, f32 image and PPM bytes); N > 1: interleaved 4-row bands "
                            "per GPU, final RCCL gather of the PPM rows to rank 0",
                "mesh": mesh_label(args.mesh),
                "triangles": int(len(mesh[0])),
                "frame": [width, H_total],
                "rows_per_gpu": rows,
                "texture": TEXTURE,
                "parallelism": (f"row tiles x{world} ({'interleaved 4-row bands' if bands else 'contiguous blocks'})"
                                if world > 1 else "single GPU"),
                "camera": "static (value); see moving_camera",
                **({"note": "weak scaling widens the frame to (1920 N) x 1080: not a BASELINE.json config"}
                   if world > 1 and args.scaling == "weak" else {}),
                "culling": not args.brute_force,
            },
            "rows_per_gpu_note": "rank 0's row count (bands: rows of its interleaved bands)" if bands else None,
            "frame_ms": round(ms_per_step, 6),
            "render_kernel_ms": round(kernel_ms, 6),
            "material_graph_s": round(t_mat, 4),
            "scene_setup_ms": round(t_setup * 1e3, 3),
            "gather_ms": None if gather_ms is None else round(gather_ms, 4),
            "rank_kernel_ms": [round(v, 6) for v in rank_kernel_ms],
            "moving_camera": moving,
            "anti_aliased": aa_line,
            "gather": ("every frame" if args.gather_every_frame else "final frame") if world > 1 else None,
            **({"rehearsal": "all ranks on GPU 0, gloo collectives: not a measurement"} if rehearsal else {}),
            "hit_pixels": hits_all,
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4),
                **counter_figures(pmc_record(pmc_key), kernel_ms),
                "kernel": "frame_kernel (eray_amd/csrc/render.hip)",
                "algorithmic_bytes_per_launch": alg,
                "kernel_ms": round(kernel_ms, 6),
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(mesh, width, H_total, frame_camera_fov(width, H_total), args.cpu_seconds)
        print(json.dumps(result), flush=True)

    if world > 1 and not rehearsal:
        rccl.close()
    scene.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

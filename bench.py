#!/usr/bin/env python3
"""Benchmark of the eray ray-tracing hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Metric (BASELINE.json): Mrays/s + frame ms at 1920x1080 cube.obj, 1/2/4/8-GPU tile scaling.
Workload (configs[1]): objects/cube.obj with src/main.rs's scene and material
graph, a 1920x1080 frame.  One step = one batch of frames (the single-GPU launch size, 8 frames at
C2; --frames-per-step), each frame: camera rays, first-hit triangle scan, shading with shadow rays,
the f32 image and the PPM bytes (fused), and for N > 1 the frame assembled on one GPU.  Inputs (mesh, material textures) are resident in HBM before timing; the material graph is
evaluated once, as Material::update is (reported separately).

Frames in flight: a serving loop renders a stream of independent frames, so the frames go
through a ring of output slots (eray_render_frames_ring) and several frames share one kernel
launch — the latency-bound shading chains of one frame overlap the others' background stores.
Every frame is rendered in full into its own slot.  `frame_latency_ms` reports one frame alone
per launch beside it.

Multi-GPU (row tiles), default --scaling strong: the same 1920x1080 frame split over
the N GPUs in interleaved 4-row bands (equal work wherever the cube sits); N = 1 is exactly C2.
Every frame is assembled whole on one GPU (eray_gather_frames): the ranks render batches of frames
into one half of a two-half ring while the previous batch's rows travel over xGMI (RCCL
point-to-point, only the objects' pixel rectangles: ERAY_GATHER_SCENE_CAMERA) on a second stream;
frame k of a batch is assembled on rank k % N (ERAY_GATHER_ROTATE_ROOT, default) or every frame on
rank 0 (--gather-root 0).  --scaling weak widens the frame to (1920 N) x 1080 instead (not a BASELINE config).
C4 (--width 3840 --height 2160) and C5 (7680x4320, a 1M-face mesh) are available by flag.

Prints ONE JSON line on rank 0 (metric "Mrays/s": primary rays of all frames / wall time).
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
from eray_amd.dist import BAND_ROWS, RowGather, band_split, frames_assembled, gather_ppm_rows, row_block  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402

WIDTH, HEIGHT, TEXTURE = 1920, 1080, 1024  # C2 (defaults; --width / --height)
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
ACHIEVABLE_HBM_GBS = 6290.0  # MI355X_MICROARCH.md: 6.29 TB/s measured (float4 copy)
PEAK_VALU_TOPS = 78.6  # non-FMA FP32 VALU: 256 CUs x 4 SIMDs x 32 lanes x 2.4 GHz
HIT_TEXEL_BYTES = 16  # Material::get per hit pixel: IColor 12 B + IValue 4 B (material.rs:56-94)
FACE_RECORD_BYTES = 48 + 64  # the first hit's intersection record (TriHot) + shading record (TriShade)


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


def algorithmic_bytes(pixels: int, hit_pixels: int, hit_faces: int) -> int:
    """Bytes one frame must move (DESIGN.md §5 roofline): the outputs, 15 B per pixel written
    (12 B f32 RGB + 3 B PPM); per hit pixel the two texels Material::get reads (16 B); per face
    that is some pixel's first hit its intersection and shading records (112 B).  Faces that are
    only candidates, the culling records and the screen bins are work of this implementation,
    not of the path, and are not counted."""
    return 15 * pixels + HIT_TEXEL_BYTES * hit_pixels + FACE_RECORD_BYTES * hit_faces


def pmc_record(workload: dict):
    """The committed rocprofv3 counter summary of this workload's frame kernel
    (scripts/pmc_traffic.py): profiles/rNN/pmc_traffic*.json whose "workload" equals this run's,
    or None when no summary of this workload is committed."""
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic*.json")), reverse=True)
    for path in paths:
        try:
            with open(path) as f:
                rec = json.load(f)
            if rec.get("workload") == workload and "frame_kernel" in rec:
                return rec["frame_kernel"]
        except (OSError, KeyError, ValueError):
            continue
    return None


def counter_figures(rec, launch_ms: float) -> dict:
    """From a counter summary (per launch of frames_per_launch frames): HBM bytes per launch
    (2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md), the HBM-read
    fraction (north_star's figure) and the VALU fraction (SQ_INSTS_VALU x 64 lanes / launch time /
    the 78.6 T ops/s non-FMA FP32 peak; every VALU instruction of the frame kernel), and the share
    of wave cycles spent waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES)."""
    if not rec:
        return {"traffic": None}
    out = {"traffic": int(rec["hbm_bytes_per_launch"])}
    sec = launch_ms * 1e-3
    fetch = rec.get("fetch_bytes_corrected")
    if fetch is not None and sec > 0:
        gbs = fetch / sec / 1e9
        out["hbm_read"] = {"achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                           "frac": round(gbs / PEAK_HBM_GBS, 4), "bytes_per_launch": int(fetch)}
    c = rec.get("counters_mean_per_dispatch", {})
    if c.get("SQ_INSTS_VALU") is not None and sec > 0:
        tops = c["SQ_INSTS_VALU"] * 64 / sec / 1e12
        out["valu"] = {"achieved": round(tops, 2), "peak": PEAK_VALU_TOPS, "unit": "TOP/s",
                       "frac": round(tops / PEAK_VALU_TOPS, 4), "instructions_per_launch": int(c["SQ_INSTS_VALU"])}
    if c.get("SQ_WAIT_ANY") and c.get("SQ_WAVE_CYCLES"):
        out["wave_wait_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
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


class Markers:
    """ROCTx ranges around the bench's legs (rocprofiler-sdk's roctx; a no-op without it), so that
    a `rocprofv3 --kernel-trace --marker-trace` run of this command attributes every dispatch to
    its leg and launch size (scripts/prof_legs.py): the committed per-leg profile rows are the
    ones the line's kernel figures must reproduce."""

    def __init__(self):
        self._lib = None
        import ctypes
        for name in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"):
            try:
                self._lib = ctypes.CDLL(name)
                self._lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                self._lib.roctxRangePushA(b"init")  # (the library's own first-call set-up, here)
                self._lib.roctxRangePop()
                break
            except (OSError, AttributeError):
                self._lib = None

    def range(self, name: str):
        import contextlib

        @contextlib.contextmanager
        def cm():
            if self._lib:
                self._lib.roctxRangePushA(name.encode())
            try:
                yield
            finally:
                if self._lib:
                    self._lib.roctxRangePop()
        return cm()


MARK = Markers()


def kernel_figures(kt: dict) -> dict:
    """eray_time_frames_ring's dispatch-timestamp durations (ms per launch) as line fields."""
    F = kt["frames_per_launch"]
    out = {"launches": kt["launches"], "frames_per_launch": F,
           "frame_kernel_ms_per_launch": round(kt["frame_kernel_ms"], 6),
           "frame_kernel_ms_min": round(kt["frame_kernel_min_ms"], 6),
           "frame_kernel_ms_max": round(kt["frame_kernel_max_ms"], 6),
           "frame_kernel_ms_per_frame": round(kt["frame_kernel_ms"] / F, 6)}
    if kt["fill_kernel_ms"] > 0:
        out["fill_kernel_ms_per_launch"] = round(kt["fill_kernel_ms"], 6)
        out["launch_span_ms"] = round(kt["launch_span_ms"], 6)
    return out


def write_ceiling_fields(ct: dict, launch_bytes: int, floor_ms: float) -> dict:
    """eray_time_write_ceiling's figures: the same launches' background bytes written by a plain
    block-strided store stream (one workgroup per CU, no other work) into the same ring slots, in
    this process — the chip's own write rate for the ring, against which the fill floor is read."""
    gbs = launch_bytes / (ct["frame_kernel_ms"] * 1e-3) / 1e9
    return {"kernel_ms_per_launch": round(ct["frame_kernel_ms"], 6), "kernel_ms_min": round(ct["frame_kernel_min_ms"], 6),
            "achieved_gbs": round(gbs, 1), "frac": round(gbs / PEAK_HBM_GBS, 4),
            "fill_floor_over_ceiling": round(floor_ms / ct["frame_kernel_ms"], 4),
            "kernel": "ceiling_fill_kernel (render.hip): 64x4 blocks, 1 workgroup per CU, unpaced write-through stores"}


def merge_times(parts: list) -> dict:
    """eray_kernel_times of several timed runs as one: launches summed, means weighted by launches."""
    n = sum(t["launches"] for t in parts)
    out = dict(parts[0])
    out["launches"] = n
    for k in ("frame_kernel_ms", "fill_kernel_ms", "launch_span_ms"):
        out[k] = sum(t[k] * t["launches"] for t in parts) / n
    out["frame_kernel_min_ms"] = min(t["frame_kernel_min_ms"] for t in parts)
    out["frame_kernel_max_ms"] = max(t["frame_kernel_max_ms"] for t in parts)
    return out


def floor_and_ceiling(empty, frames: int, W: int, H: int, tag: str, F: int, **kw) -> tuple:
    """The fill floor (the frame kernel with no object: eray_time_frames_ring) and the write ceiling
    (eray_time_write_ceiling) of the same launches into the same ring, measured in four alternating
    chunks each (ROCTx ranges {tag}fill_floor_F{F} / {tag}write_ceiling_F{F}), so that neither leg
    inherits the ring state the other or the frame leg before them left."""
    chunks = 4
    per = max(frames // chunks // F, 1) * F
    ceil_kw = {k: kw[k] for k in ("ring", "out_rgb", "out_ppm") if k in kw}
    fl, ce = [], []
    for _ in range(chunks):
        with MARK.range(f"{tag}fill_floor_F{F}"):
            fl.append(empty.time_frames(per, W, H, **kw))
        with MARK.range(f"{tag}write_ceiling_F{F}"):
            ce.append(empty.time_write_ceiling(per, W, H, **ceil_kw))
    return merge_times(fl), merge_times(ce)


def empty_scene_context(device: int, width: int, height: int, fov, stream) -> "capi.Context":
    """The same camera and lights with no object: every pixel is the miss colour (engine.rs:
    208-213), so its frame kernel is the fill alone — this kernel's write floor for the frame."""
    ctx = capi.Context(device)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_camera(capi.make_camera((0.0, 0.0, 5.0), fov, width, 1.0))
    ctx.add_light(capi.make_light((0.0, 2.0, 0.0), "ambient", (1.0, 1.0, 1.0), 0.2))
    ctx.add_light(capi.make_light((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0))
    return ctx


NS_FACES, NS_SEED, NS_WIDTH, NS_HEIGHT = 69451, 42, 3840, 2160  # north_star: 3840x2160 / 70k tris
MALL_BYTES = 256 << 20  # MI355X Infinity Cache (MI355X_MICROARCH.md)


def north_star_line(device: int, steps: int, slot_counts=None) -> dict:
    """BASELINE.json north_star's figure: the frame kernel at 3840x2160 over the 69,451-face
    stand-in (SURVEY.md §8(d) C3 mesh, generated here by eray_amd.meshgen, seed 42) with main.rs's
    scene and material, against 8 TB/s and against the same kernel's fill-alone floor (an empty
    scene: the frame's bytes with no detail work) at the same ring size.  Two ring sizes: one slot
    (each frame rewrites the same 124 MB, which the 256 MiB Infinity Cache absorbs) and the fewest
    slots whose bytes exceed the Infinity Cache (every frame's stores reach HBM)."""
    import tempfile

    from eray_amd import meshgen

    t0 = time.perf_counter()
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "standin_69451.obj")
        meshgen.generate(path, NS_FACES, NS_SEED)
        mesh = load_obj_file(path)
    gen_s = time.perf_counter() - t0
    W, H = NS_WIDTH, NS_HEIGHT
    fov = frame_camera_fov(W, H)
    frame_bytes = 15 * W * H
    big = 1
    while big * frame_bytes <= MALL_BYTES:
        big *= 2
    slot_counts = slot_counts or [1, big]
    stream = torch.cuda.Stream()
    ctx = capi.Context(device)
    ctx.set_stream(stream.cuda_stream)
    empty = empty_scene_context(device, W, H, fov, stream)
    scene = MainScene(ctx, *mesh, W, H, texture=TEXTURE, fov=fov)
    nmax = max(slot_counts)
    with torch.cuda.stream(stream):
        rgb = torch.empty((nmax, H, W, 3), dtype=torch.float32, device="cuda")
        ppm = torch.empty((nmax, H, W, 3), dtype=torch.uint8, device="cuda")
        face = torch.full((H, W), -1, dtype=torch.int32, device="cuda")
    ctx.render(W, H, out_rgb=rgb.data_ptr(), out_face=face.data_ptr())
    torch.cuda.synchronize()
    hit = face[face >= 0]
    hits, hit_faces = int(hit.numel()), int(torch.unique(hit).numel())
    del face
    alg = algorithmic_bytes(W * H, hits, hit_faces)
    steps = max(steps, 20)
    variants = {}
    for slots in slot_counts:
        ring = capi.frame_ring(slots, H, W, 1)
        out = dict(out_rgb=rgb.data_ptr(), out_ppm=ppm.data_ptr(), ring=ring)
        tag = f"ns_slots{slots}"
        ctx.render_frames(steps, W, H, prepare_only=True, **out)
        ctx.render_frames(steps, W, H, **out)  # warm
        torch.cuda.synchronize()
        with MARK.range(f"{tag}_replay_F1"):
            t1 = time.perf_counter()
            ctx.render_frames(steps, W, H, **out)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t1
        # dispatch-timed launches: 64 of them after two untimed ones (a plain launch after the
        # graph replays can take twice as long once)
        ctx.time_frames(2, W, H, **out)
        empty.time_frames(2, W, H, **out)
        with MARK.range(f"{tag}_timed_F1"):
            kt = ctx.time_frames(max(steps, 64), W, H, **out)
        ft, ct = floor_and_ceiling(empty, max(steps, 64), W, H, f"{tag}_", 1, **out)
        k_ms, f_ms = kt["frame_kernel_ms"], ft["frame_kernel_ms"]
        gbs = alg / (k_ms * 1e-3) / 1e9
        fill_gbs = 15 * W * H / (f_ms * 1e-3) / 1e9
        pmc_key = {"mesh": f"meshgen {NS_FACES} faces seed {NS_SEED}", "frame": [W, H], "rows_per_gpu": H,
                   "n_gpus": 1, "brute_force": False, "frames_per_launch": 1, "ring_slots": slots}
        variants[f"slots_{slots}"] = {
            "ring_slots": slots,
            "ring_bytes": slots * frame_bytes,
            "exceeds_infinity_cache": slots * frame_bytes > MALL_BYTES,
            "ms_per_step": round(wall / steps * 1e3, 6),
            "value": round(W * H * steps / wall / 1e6, 3),
            "unit": "Mrays/s",
            "kernel": kernel_figures(kt),
            "fill_floor": {"frame_kernel_ms": round(f_ms, 6),
                           "achieved_gbs": round(fill_gbs, 1),
                           "frac": round(fill_gbs / PEAK_HBM_GBS, 4),
                           "scene": "no objects: every pixel the miss colour, same kernel and ring",
                           "write_ceiling": write_ceiling_fields(ct, frame_bytes, f_ms)},
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(gbs / PEAK_HBM_GBS, 4),
                         "frac_of_fill_floor": round(f_ms / k_ms, 4),
                         **counter_figures(pmc_record(pmc_key), k_ms)},
        }
    del rgb, ppm
    scene.close()
    ctx.close()
    empty.close()
    return {"workload": f"north_star: {NS_FACES}-face stand-in (eray_amd.meshgen, seed {NS_SEED}), {W}x{H} frame, "
                        "main.rs scene + material graph, one frame per launch",
            "frame": [W, H], "triangles": int(len(mesh[0])), "hit_pixels": hits, "hit_faces": hit_faces,
            "algorithmic_bytes_per_frame": alg, "mesh_generation_s": round(gen_s, 3),
            "bytes_model": "15 B/pixel written + 16 B texels per hit pixel + 112 B records per hit face",
            "timing": "kernel = the frame kernel dispatch's own start / end timestamps (hipExtLaunchKernel events, "
                      "as rocprofv3's kernel trace); step = wall time of graph-replayed frames",
            "variants": variants}


def mesh_label(path: str) -> str:
    """The mesh as the JSON line names it: repo-relative when it is in the tree, else the file name
    (meshes generated on the box by eray_amd.meshgen)."""
    rel = os.path.relpath(path, ROOT)
    return os.path.basename(path) if rel.startswith("..") else rel


def moving_camera(scene, args, width, height, out, ring) -> dict:
    """The bench's frames with a camera that moves every frame (dolly_path), through the same ring:
    eray_render_camera_path_ring runs every frame's camera setup on the device inside the timed
    loop (small scenes: one launch sets up a graph chunk's 64 cameras, frames_per_launch frames
    per launch, each from its own setup slot).  One GPU."""
    path = dolly_path(args.steps, frame_camera_fov(width, height), width)
    scene.ctx.render_camera_path(path, width, height, ring=ring, **out)
    torch.cuda.synchronize()
    m0 = time.perf_counter()
    scene.ctx.render_camera_path(path, width, height, ring=ring, **out)
    torch.cuda.synchronize()
    moving_s = time.perf_counter() - m0
    device_ms = scene.ctx.render_camera_path(path, width, height, ring=ring, timed=True, **out)
    one = scene.ctx.render_camera_path(path, width, height, timed=True, **out)  # one frame per launch
    return {
        "frame_ms": round(moving_s / args.steps * 1e3, 6),
        "value": round(width * height * args.steps / moving_s / 1e6, 3),
        "unit": "Mrays/s",
        "device_ms_per_frame": round(device_ms, 6),
        "device_ms_per_frame_one_per_launch": round(one, 6),
        "frames": args.steps,
        "camera": "dolly along the view axis, z 5 +- 0.5, z_dist 1 +- 0.1, a new camera every frame",
        "includes": "every frame's camera setup on the device (culling records, pixel rectangles, merged "
                    "detail rectangles; for meshes over 256 faces the screen bins and detail list, built for "
                    "up to 16 cameras at once beside the previous cameras' frames) + frame",
    }


def one_shot(mesh_path: str, width: int, height: int) -> dict:
    """main.rs's own use (main.rs:17-70): load the mesh, build and update the material, set up the
    scene and render ONE frame to a PPM file's bytes on the host — each step timed, the first thing
    this process does on the GPU (so code-object loading and first allocations are inside), then
    the same steps again on a second context (the warm per-scene cost)."""
    out = {}
    for tag in ("cold", "warm"):
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        mesh = load_obj_file(mesh_path)  # Object::load_obj (object.rs:101-186)
        t.append(time.perf_counter())
        ctx = capi.Context(torch.cuda.current_device())
        t.append(time.perf_counter())
        sc = MainScene(ctx, *mesh, width, height, texture=TEXTURE, fov=frame_camera_fov(width, height))
        ctx.synchronize()  # upload + Material::update (the material graph on the device)
        t.append(time.perf_counter())
        ppm = ctx.empty((height, width, 3), np.uint8)
        ctx.render(width, height, out_ppm=ppm.ptr)  # per-camera setup + frame (Engine::render)
        ctx.synchronize()
        t.append(time.perf_counter())
        body = ppm.numpy()  # PPM body to the host (save_as_ppm's bytes, image.rs:48-74)
        t.append(time.perf_counter())
        ppm.free()
        sc.close()
        ctx.close()
        ms = [round((b - a) * 1e3, 3) for a, b in zip(t, t[1:])]
        out[tag] = {"load_obj_ms": ms[0], "context_ms": ms[1], "upload_and_material_ms": ms[2],
                    "setup_and_frame_ms": ms[3], "ppm_to_host_ms": ms[4], "total_ms": round((t[-1] - t[0]) * 1e3, 3)}
        del body
    out["note"] = ("cold: the process's first GPU work (HIP code-object load, first allocations); warm: a second "
                   "scene on a new context in the same process")
    return out


AA_SAMPLES = 4


def material_roofline(scene, stream, reps: int = 20) -> dict:
    """Material::update of main.rs's graph (shaderlib.hip material_example_kernel: wave -> rgb ->
    mix with flat, one fused pass) against the HBM roofline: 16 B written per texel (12 B IColor +
    4 B IValue), HIP events around `reps` back-to-back updates on the library's stream."""
    scene.evaluate_material()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    with torch.cuda.stream(stream):
        ev[0].record()
        for _ in range(reps):
            scene.evaluate_material()
        ev[1].record()
    ev[1].synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3 / reps
    texels = scene.texture * scene.texture
    gbs = texels * 16 / (us * 1e-6) / 1e9
    return {"kernel": "material_example_kernel (eray_amd/csrc/shaderlib.hip)", "texels": texels,
            "bytes_per_update": texels * 16, "us_per_update": round(us, 3), "achieved_gbs": round(gbs, 1),
            "peak_gbs": PEAK_HBM_GBS, "frac": round(gbs / PEAK_HBM_GBS, 4),
            "bound": "latency of the dependent double-precision glibc cosf chain per wave (8 waves per SIMD) "
                     "(a persistent grid of fewer waves is slower), neither VALU issue (~15 % of the chip's) nor HBM: 82 VALU "
                     "instructions per texel (18 % FP64), 0.48 of wave cycles waiting, WRITE_SIZE = the 16 B "
                     "per texel (profiles/r06/material_pmc.json)"}


def anti_aliasing_line(scene, args, width, height, out) -> dict:
    """The general tracer (trace.hip: anti-aliasing, engine.rs:59-77) on the bench's frames:
    AA_SAMPLES jittered rays per pixel plus the centre ray.  Device
    time per frame over graph-replayed frames; rays counted as the reference casts them."""
    frames = max(2, min(args.steps, 20))
    kw = dict(out, anti_aliasing=AA_SAMPLES, aa_seed=12345)
    scene.ctx.render_frames(frames, width, height, prepare_only=True, **kw)
    # (the best of three replays: the first after the plan is made carries one-time costs)
    ms = min(scene.ctx.render_frames(frames, width, height, timed=True, **kw) for _ in range(3))
    rays = width * height * (AA_SAMPLES + 1)
    return {"anti_aliasing": AA_SAMPLES, "frames": frames, "frame_ms": round(ms, 6),
            "value": round(rays / (ms * 1e-3) / 1e6, 3), "unit": "Mrays/s (all AA rays)",
            "kernel": "trace.hip: waves whose rays can reach no face skip the scan (culling records / bins and "
                      "object rectangles); with meshes over 256 faces the tracer's setup bins every face by the pixels "
                      "its jittered rays may hit, a wave searches its bin as (entry, pixel) pairs for all the pixel's "
                      "rays at once, heavy bins by a whole workgroup, fill roles write the background; shadow rays "
                      "every face"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--mesh", default=os.path.join(ROOT, "objects", "cube.obj"))
    ap.add_argument("--width", type=int, default=WIDTH,
                    help="frame width (strong) or width per GPU (weak); C2: 1920")
    ap.add_argument("--height", type=int, default=HEIGHT, help="frame height (C2: 1080)")
    ap.add_argument("--scaling", choices=("strong", "weak"), default="strong",
                    help="strong: one width x height frame split N ways (BASELINE); weak: a (width N) x height frame")
    ap.add_argument("--frames-per-step", type=int, default=0,
                    help="frames per step (0: the single-GPU launch size of the full frame, the same for every N)")
    ap.add_argument("--gather-root", choices=("rotate", "0"), default="rotate",
                    help="N > 1, scene gather: frame k assembled on rank k %% N (rotate) or all on rank 0")
    ap.add_argument("--frames-per-launch", type=int, default=0,
                    help="frames in flight per kernel launch (0: the library's choice, eray_frames_per_launch)")
    ap.add_argument("--brute-force", action="store_true", help="disable the exact wave culling")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-moving-camera", action="store_true",
                    help="skip the moving-camera, AA and one-frame latency lines (counter runs)")
    ap.add_argument("--split", choices=("bands", "blocks"), default="bands",
                    help="N > 1: interleaved 4-row bands (balanced, default) or contiguous row blocks")
    ap.add_argument("--gather", choices=("scene", "coded"), default="scene",
                    help="N > 1: only the objects' pixel rectangles travel (scene, sync-free) or the coded rows")
    ap.add_argument("--no-north-star", action="store_true", help="skip the north_star sub-record (N = 1)")
    ap.add_argument("--north-star-only", action="store_true",
                    help="print only the north_star sub-record (profiling runs); --ns-slots picks ring sizes")
    ap.add_argument("--ns-slots", default="", help="comma-separated ring sizes of the north_star leg")
    args = ap.parse_args()
    if args.north_star_only:
        torch.cuda.set_device(0)
        slots = [int(x) for x in args.ns_slots.split(",") if x] or None
        print(json.dumps({"north_star": north_star_line(0, args.steps, slots)}), flush=True)
        return

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

    # main.rs's one-shot use, before anything else touches the GPU (N = 1 only)
    oneshot = one_shot(args.mesh, args.width, args.height) if world == 1 and not args.no_moving_camera else None
    mesh = load_obj_file(args.mesh)
    ctx = capi.Context(device)
    stream = torch.cuda.Stream()  # the render stream: shared by the library and torch
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    width = args.width * world if args.scaling == "weak" else args.width
    H = args.height
    t_mat0 = time.perf_counter()
    scene = MainScene(ctx, *mesh, width, H, texture=TEXTURE, fov=frame_camera_fov(width, H))
    torch.cuda.synchronize()
    t_mat = time.perf_counter() - t_mat0
    material_line = material_roofline(scene, stream) if rank == 0 else None

    # this rank's rows: interleaved 4-row bands r, r + N, ... (every rank an equal share of the scene
    # wherever it sits) or, --split blocks, the r-th block of PPM file rows
    bands = world > 1 and args.split == "bands"
    if bands:
        sp = band_split(rank, world, H, BAND_ROWS)
        row0, rows, alloc_rows = sp["row0"], sp["rows"], sp["alloc_rows"]
        band_args = dict(band_rows=sp["band_rows"], band_stride=sp["band_stride"])
    else:
        if H % world:
            raise SystemExit(f"--height {H} does not split into {world} equal row blocks")
        row0, rows = row_block(rank, world, H // world)
        alloc_rows, band_args = rows, {}
    band = BAND_ROWS if bands else 0
    flags = capi.RENDER_BRUTE_FORCE if args.brute_force else capi.RENDER_DEFAULT

    # frames in flight: F frames per launch (the library's choice unless given); N = 1 renders into
    # a ring of F slots, N > 1 into two halves of G = F slots each (batch b renders into half b % 2
    # while batch b - 1 is gathered)
    F = args.frames_per_launch or ctx.frames_per_launch(width, H, rows=rows, slots=64)
    G = F
    slots = F if world == 1 else 2 * G
    # frames per step: one single-GPU launch of the full frame, so a step is the same work at every N
    fps = args.frames_per_step or ctx.frames_per_launch(args.width, H, rows=H, slots=64)
    n_timed = args.steps * fps
    slot_px = alloc_rows * width
    rgb = torch.empty((slots, alloc_rows, width, 3), dtype=torch.float32, device="cuda")
    ppm = torch.zeros((slots, alloc_rows, width, 3), dtype=torch.uint8, device="cuda")

    def ring_args(half=0, n=slots):
        return dict(row0=row0, rows=rows, flags=flags, out_rgb=rgb[half * G].data_ptr(),
                    out_ppm=ppm[half * G].data_ptr(), ring=capi.frame_ring(n, alloc_rows, width, min(F, n)),
                    **band_args)

    # one untimed instrumented frame: hit pixels and hit faces for the algorithmic-bytes model;
    # being the first render of the camera it also builds the per-camera data (culling records,
    # pixel rectangles, screen bins of large meshes): reported as scene_setup_ms
    face = torch.full((alloc_rows, width), -1, dtype=torch.int32, device="cuda")
    one_rgb = torch.empty((alloc_rows, width, 3), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    t_setup0 = time.perf_counter()
    ctx.render(width, H, out_rgb=one_rgb.data_ptr(), out_face=face.data_ptr(), row0=row0, rows=rows, flags=flags,
               **band_args)
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t_setup0
    hit = face[:rows][face[:rows] >= 0]
    hits, hit_faces = int(hit.numel()), int(torch.unique(hit).numel())
    del face, one_rgb

    gather = None
    frames_out = None
    rotate = False
    if world > 1:
        rotate = args.gather_root == "rotate" and args.gather == "scene" and not rehearsal
        # the frames this rank assembles per batch: k = rank, rank + N, ... (rotating roots) or all on rank 0
        n_out = frames_assembled(G, world, rank, rotate)
        frames_out = torch.empty((n_out, H, width, 3), dtype=torch.uint8, device="cuda") if n_out else None
        gstream = torch.cuda.Stream()
        if not rehearsal:
            rccl = RowGather(ctx, world, rank)

            def gather(half, n):  # frames of ring half `half` -> rank 0's frames, on the gather stream
                ctx.set_stream(gstream.cuda_stream)
                ctx.gather_frames(rccl.comm, ppm[half * G].data_ptr(), slot_px * 3,
                                  frames_out.data_ptr() if frames_out is not None else 0, H * width * 3, n, H, width,
                                  band_rows=band, scene_camera=args.gather == "scene", rotate_root=rotate)
                ctx.set_stream(stream.cuda_stream)
        else:
            def gather(half, n):  # plumbing only: gloo through host memory
                torch.cuda.synchronize()
                for k in range(n):
                    gather_ppm_rows(ppm[half * G + k], frames_out[k] if frames_out is not None else None, world, rank,
                                    band_rows=band)

    def run(nframes):
        """nframes frames through the ring (N > 1: batches of G, each gathered while the next renders)."""
        if world == 1:
            ctx.render_frames(nframes, width, H, **ring_args())
            return
        ev_r, ev_g = [], []
        b = 0
        for first in range(0, nframes, G):
            n = min(G, nframes - first)
            half = b % 2
            if b >= 2:  # the gather of batch b - 2 has read this half
                stream.wait_event(ev_g[b - 2])
            ctx.render_frames(n, width, H, **ring_args(half, G))
            e = torch.cuda.Event()
            e.record(stream)
            ev_r.append(e)
            gstream.wait_event(e)
            with torch.cuda.stream(gstream):
                gather(half, n)
                e2 = torch.cuda.Event()
                e2.record(gstream)
            ev_g.append(e2)
            b += 1
        stream.wait_event(ev_g[-1])

    # launch plans (graphs) of every batch size, the gather plan and buffers, then W warmup frames,
    # all outside the timed region
    sizes = {min(G, n_timed)} | ({n_timed % G} if world > 1 and n_timed % G else set())
    for n in sizes:
        ctx.render_frames(n, width, H, prepare_only=True, **(ring_args() if world == 1 else ring_args(0, G)))
    if world == 1:
        ctx.render_frames(n_timed, width, H, prepare_only=True, **ring_args())
    run(max(args.warmup, 1) * fps)
    if world > 1:
        for n in sizes:
            run(n)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    with MARK.range(f"steps_F{F}"):  # (pushed before, popped after the clock's two readings)
        t0 = time.perf_counter()
        run(n_timed)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = float(allreduce(elapsed, torch.float64, dist.ReduceOp.MAX))
        hits_all = int(allreduce(hits, torch.int64, dist.ReduceOp.SUM))
    else:
        hits_all = hits
    # the frame kernel's duration on this rank: launches of the line's size, each timed by its
    # dispatch's own start / end timestamps (eray_time_frames_ring); the same frames graph-replayed
    # between two events (launch gaps included); the latency of one frame alone per launch
    ring1 = ring_args() if world == 1 else ring_args(0, G)
    # dispatch-timed frames: 32 launches of 8 at C2 (8 left the mean to a launch or two: the
    # round-6 sessions' C2 launches spread 39.6-43.1 us)
    n_kt = max(256, F) // F * F
    with MARK.range(f"timed_F{F}"):
        kt = ctx.time_frames(n_kt, width, H, **ring1)
    kernel_ms = kt["frame_kernel_ms"] / F  # per frame
    with MARK.range(f"replay_F{F}"):  # the same frames graph-replayed, bracketed by two events
        replay_ms = ctx.render_frames(max(n_timed // F, 1) * F, width, H, timed=True, **ring1)
    latency = None
    fill_floor = None
    beyond = None
    if not args.no_moving_camera:  # (counter runs keep to the measured launches)
        lat_args = dict(ring1)
        lat_args["ring"] = capi.frame_ring(1, alloc_rows, width, 1)
        with MARK.range("latency_F1"):
            latency = ctx.time_frames(max(min(args.steps, 64), 2), width, H, **lat_args)
        if world == 1:  # the same frames with no object: the fill alone, this kernel's write floor
            empty = empty_scene_context(device, width, H, frame_camera_fov(width, H), stream)
            ft, ct = floor_and_ceiling(empty, n_kt, width, H, "", F, **ring1)
            fill_floor = {"frame_kernel_ms_per_launch": round(ft["frame_kernel_ms"], 6),
                          "frames_per_launch": ft["frames_per_launch"],
                          "achieved_gbs": round(15 * width * rows * ft["frames_per_launch"] / (ft["frame_kernel_ms"] * 1e-3)
                                                / 1e9, 1),
                          "scene": "no objects: every pixel the miss colour, same kernel, ring and launch size",
                          "write_ceiling": write_ceiling_fields(ct, 15 * width * rows * F, ft["frame_kernel_ms"])}
            # the same launches into a ring whose slots exceed the 256 MiB Infinity Cache: every
            # frame's stores reach HBM (the line's own ring of F slots may stay cache-resident)
            if slots * slot_px * 15 <= MALL_BYTES:
                big = slots
                while big * slot_px * 15 <= MALL_BYTES:
                    big *= 2
                with torch.cuda.stream(stream):
                    brgb = torch.empty((big, alloc_rows, width, 3), dtype=torch.float32, device="cuda")
                    bppm = torch.empty((big, alloc_rows, width, 3), dtype=torch.uint8, device="cuda")
                bkw = dict(row0=row0, rows=rows, flags=flags, out_rgb=brgb.data_ptr(), out_ppm=bppm.data_ptr(),
                           ring=capi.frame_ring(big, alloc_rows, width, F), **band_args)
                ctx.render_frames(big, width, H, **bkw)  # (the slots' pages touched once)
                with MARK.range(f"beyond_mall_timed_F{F}"):
                    bt = ctx.time_frames(n_kt, width, H, **bkw)
                bft, bct = floor_and_ceiling(empty, n_kt, width, H, "beyond_mall_", F, **bkw)
                del brgb, bppm
                b_ms = bt["frame_kernel_ms"]
                b_gbs = algorithmic_bytes(width * rows, hits, hit_faces) * F / (b_ms * 1e-3) / 1e9
                beyond = {"ring_slots": big, "ring_bytes": big * slot_px * 15, "kernel": kernel_figures(bt),
                          "achieved": round(b_gbs, 1), "frac": round(b_gbs / PEAK_HBM_GBS, 4),
                          "fill_floor_ms_per_launch": round(bft["frame_kernel_ms"], 6),
                          "frac_of_fill_floor": round(bft["frame_kernel_ms"] / b_ms, 4),
                          "write_ceiling": write_ceiling_fields(bct, 15 * width * rows * F, bft["frame_kernel_ms"])}
            empty.close()
    rank_kernel_ms = [kernel_ms]
    gather_ms = None
    if world > 1:
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        with torch.cuda.stream(gstream):
            gather(0, G)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3 / G
        got = [None] * world
        dist.all_gather_object(got, kernel_ms)
        rank_kernel_ms = got

    out1 = dict(row0=row0, rows=rows, flags=flags, out_rgb=rgb.data_ptr(), out_ppm=ppm.data_ptr(), **band_args)
    moving = None
    aa_line = None
    if world == 1 and not args.no_moving_camera:
        with MARK.range("moving_camera"):
            moving = moving_camera(scene, args, width, H, out1, capi.frame_ring(slots, alloc_rows, width, F))
        with MARK.range("anti_aliased"):
            aa_line = anti_aliasing_line(scene, args, width, H, out1)
    ns_line = None
    if world == 1 and not args.no_north_star:
        ns_line = north_star_line(device, args.steps)

    if rank == 0:
        # the workload a committed counter summary (profiles/rNN/pmc_traffic*.json) must match
        pmc_key = {"mesh": mesh_label(args.mesh), "frame": [width, H], "rows_per_gpu": rows, "n_gpus": world,
                   "brute_force": bool(args.brute_force), "frames_per_launch": F}
        is_c2 = (width, H) == (WIDTH, HEIGHT) and args.mesh.endswith("objects/cube.obj") and not args.brute_force
        pixels = width * rows
        ms_per_step = elapsed / args.steps * 1e3
        frame_ms = elapsed / n_timed * 1e3
        rays = width * H * n_timed
        value = rays / elapsed / 1e6
        alg = algorithmic_bytes(pixels, hits, hit_faces)
        gbs = alg / (kernel_ms * 1e-3) / 1e9
        launch_ms = kernel_ms * F
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
                "workload": f"{'C2: ' if is_c2 else ''}{os.path.basename(args.mesh)}, {width}x{H} frame, "
                            f"{width}x{rows} rows on rank 0, main.rs scene + material graph; step = {fps} frames, each: camera "
                            "rays, first-hit scan, shading + shadow rays, f32 image and PPM bytes"
                            + ((", assembled on rank k % N" if rotate else ", assembled on rank 0")
                               + ": scene-camera gather over RCCL point-to-point" if world > 1 else "")
                            + f"; {F} frames in flight per launch",
                "mesh": mesh_label(args.mesh),
                "triangles": int(len(mesh[0])),
                "frame": [width, H],
                "rows_per_gpu": rows,
                "texture": TEXTURE,
                "parallelism": (f"row tiles x{world} ({'interleaved 4-row bands' if bands else 'contiguous blocks'})"
                                if world > 1 else "single GPU"),
                "frames_per_step": fps,
                "frames_per_launch": F,
                "ring_slots": slots,
                "camera": "static (value); see moving_camera",
                **({"note": "weak scaling widens the frame to (1920 N) x 1080: not a BASELINE.json config"}
                   if world > 1 and args.scaling == "weak" else {}),
                "culling": not args.brute_force,
            },
            "frame_ms": round(frame_ms, 6),
            "render_kernel_ms": round(kernel_ms, 6),
            "frame_latency_ms": None if latency is None else round(latency["frame_kernel_ms"], 6),
            "graph_replay_ms_per_frame": round(replay_ms, 6),
            "material_graph_s": round(t_mat, 4),
            "material_update": material_line,
            "scene_setup_ms": round(t_setup * 1e3, 3),
            "gather": ({"kind": f"{args.gather}, every frame, batches of {G} overlapped with rendering, "
                                + ("frame k on rank k % N" if rotate else "every frame on rank 0"),
                        "ms_per_frame_alone": round(gather_ms, 5)} if world > 1 else None),
            "rank_kernel_ms": [round(v, 6) for v in rank_kernel_ms],
            "moving_camera": moving,
            "one_shot": oneshot,
            "anti_aliased": aa_line,
            **({"rehearsal": "all ranks on GPU 0, gloo collectives: not a measurement"} if rehearsal else {}),
            "hit_pixels": hits_all,
            "roofline": {
                "bound": "hbm",
                "achieved": round(gbs, 1),
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": round(gbs / PEAK_HBM_GBS, 4),
                "frac_of_achievable": round(gbs / ACHIEVABLE_HBM_GBS, 4),
                "achievable": ACHIEVABLE_HBM_GBS,
                **counter_figures(pmc_record(pmc_key), launch_ms),
                "kernel": "frame_kernel (eray_amd/csrc/render.hip)",
                "frames_per_launch": F,
                "algorithmic_bytes_per_frame": alg,
                "algorithmic_bytes_per_launch": alg * F,
                "bytes_model": "15 B/pixel written + 16 B texels per hit pixel + 112 B records per hit face",
                "hit_faces": hit_faces,
                "kernel_ms_per_frame": round(kernel_ms, 6),
                "kernel_ms_per_launch": round(launch_ms, 6),
                "timing": "the frame kernel dispatch's own start / end timestamps (hipExtLaunchKernel events, as "
                          "rocprofv3's kernel trace), mean over the launches of the line's launch size",
                "kernel_launches": kernel_figures(kt),
                **({"fill_floor": fill_floor, "frac_of_fill_floor": round(fill_floor["frame_kernel_ms_per_launch"] /
                                                                            launch_ms, 4)} if fill_floor else {}),
                "ring_slots": slots,
                "ring_bytes": slots * slot_px * 15,
                "exceeds_infinity_cache": slots * slot_px * 15 > MALL_BYTES,
                "beyond_infinity_cache": beyond,
            },
            "north_star": ns_line,
        }
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(mesh, width, H, frame_camera_fov(width, H), args.cpu_seconds)
        print(json.dumps(result), flush=True)

    if world > 1 and not rehearsal:
        torch.cuda.synchronize()
        rccl.close()
    scene.close()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""The multi-GPU decomposition (eray_amd/dist.py) on CPU: world_size-2 gloo ranks each render
their row block (with the CPU oracle standing in for the device: this checks the row split, the
file-order PPM rows and the gather, not the kernels), gather to rank 0, and rank 0's frame must
equal the single-process frame byte for byte.  The GPU path renders the same blocks with
eray_render(row0, rows, out_ppm) (tests/test_gpu_render.py::test_row_tiles_*)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from eray_amd.dist import row_block

W, ROWS = 48, 24  # 2 ranks x 24 rows = a 48x48 frame (Fov 60:60)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _render_block(row0, rows):
    from eray_amd.objfile import load_obj_file
    from oracle import pyoracle as O

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    mesh = load_obj_file(os.path.join(root, "objects", "cube.obj"))
    scene = O.main_rs_scene(*mesh, texture=64)
    cam = O.camera((0.0, 0.0, 5.0), (60.0, 60.0), W, 1.0)
    rgb, _ = O.render(scene, cam, row0=row0, rows=rows)
    body = O.ppm_bytes(rgb)
    header = f"P6 {W} {rows} 255\n".encode()
    return np.frombuffer(body[len(header):], np.uint8).reshape(rows, W, 3).copy()


def _render_rows(camera_rows):
    """The PPM bytes of the given camera rows, in local file order (last row first), as the
    fused out_ppm of a banded eray_render writes them."""
    rows = [_render_block(y, 1)[0] for y in camera_rows]
    return np.stack(rows[::-1]) if rows else np.zeros((0, W, 3), np.uint8)


def _worker(rank, world, port, out_path, bands):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eray_amd.dist import band_camera_rows, band_split, gather_ppm_rows

    H = world * ROWS
    if bands:
        sp = band_split(rank, world, H, bands)
        local = np.zeros((sp["alloc_rows"], W, 3), np.uint8)
        local[: sp["rows"]] = _render_rows(band_camera_rows(rank, world, H, bands))
        local = torch.from_numpy(local)
    else:
        row0, rows = row_block(rank, world, ROWS)
        local = torch.from_numpy(_render_block(row0, rows))
    frame = torch.empty((H, W, 3), dtype=torch.uint8) if rank == 0 else None
    gather_ppm_rows(local, frame, world, rank, band_rows=bands)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_band_split_covers_every_row_once():
    from eray_amd.dist import band_camera_rows, band_split
    for H, N, B in ((1080, 8, 4), (4320, 8, 4), (1081, 3, 4), (10, 3, 4), (2160, 4, 8)):
        rows = [y for r in range(N) for y in band_camera_rows(r, N, H, B)]
        assert sorted(rows) == list(range(H)), (H, N, B)
        assert max(band_split(r, N, H, B)["rows"] for r in range(N)) == band_split(0, N, H, B)["alloc_rows"]
    with pytest.raises(ValueError):
        band_split(0, 2, 100, 6)


def test_row_block_partition():
    assert row_block(0, 1, 1080) == (0, 1080)
    assert [row_block(r, 4, 540) for r in range(4)] == [(1620, 540), (1080, 540), (540, 540), (0, 540)]
    with pytest.raises(ValueError):
        row_block(2, 2, 10)


@pytest.mark.parametrize("bands", [0, 4, 8])
def test_two_rank_gather_equals_single_frame(tmp_path, bands):
    """Contiguous blocks and interleaved bands (band_split: every rank an equal share of the
    cube's rows) gather into the single-process frame."""
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(2, _free_port(), out, bands), nprocs=2, join=True, start_method="spawn")
    got = np.load(out)
    want = _render_block(0, 2 * ROWS)
    assert got.shape == want.shape and np.array_equal(got, want)


BG = np.array([25, 25, 51], np.uint8)  # the miss colour's PPM bytes (engine.rs:212)


def _rects_of(frame_file_order):
    """A conservative pixel rectangle of a frame (x0, x1, y0, y1 in camera rows): the bounding box
    of its non-background pixels — what the objects' rectangles (ObjGeom::rect) always contain."""
    cam = frame_file_order[::-1]
    ys, xs = np.nonzero((cam != BG).any(axis=2))
    return [(int(xs.min()), int(xs.max()), int(ys.min()), int(ys.max()))] if len(xs) else []


def _pack(local, lay, W):
    """A rank's per-frame pack in the library's layout (gather_pack_kernel restated): each
    rectangle's local rows l0..l1 (local PPM block row rows - 1 - j), columns 48 c0 .. 48 (c1 + 1)."""
    out = np.zeros(lay["bytes"], np.uint8)
    flat = local.reshape(local.shape[0], W * 3)
    for g in lay["rects"]:
        for j in range(g["l0"], g["l1"] + 1):
            at = g["off"] + (j - g["l0"]) * g["row_bytes"]
            out[at:at + g["row_bytes"]] = flat[lay["rows"] - 1 - j, 48 * g["c0"]:48 * (g["c1"] + 1)]
    return out


def _assemble(packs, lays, H, W, band, world):
    """Rank 0's frame from every rank's pack (gather_assemble_kernel restated): the background,
    except inside the owning rank's rectangles."""
    frame = np.empty((H, W * 3), np.uint8)
    frame[:] = np.tile(BG, W)
    for F in range(H):
        Y = H - 1 - F
        if band:
            r, j = (Y // band) % world, (Y // (world * band)) * band + Y % band
        else:
            h = H // world
            r = (H - 1 - Y) // h
            j = Y - (H - (r + 1) * h)
        for g in lays[r]["rects"]:
            if g["l0"] <= j <= g["l1"]:
                at = g["off"] + (j - g["l0"]) * g["row_bytes"]
                frame[F, 48 * g["c0"]:48 * (g["c1"] + 1)] = packs[r][at:at + g["row_bytes"]]
    return frame.reshape(H, W, 3)


def _scene_gather_worker(rank, world, port, out_path, bands):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eray_amd import capi
    from eray_amd.dist import band_camera_rows, band_split

    H = world * ROWS
    full = _render_block(0, H)  # every rank knows the camera's rectangles (here: from the frame)
    rects = _rects_of(full)
    lay = capi.gather_layout(rects, H, W, bands, world, rank)  # the library's own layout code
    if bands:
        sp = band_split(rank, world, H, bands)
        assert lay["rows"] == sp["rows"]
        local = np.zeros((sp["alloc_rows"], W, 3), np.uint8)
        local[: sp["rows"]] = _render_rows(band_camera_rows(rank, world, H, bands))
    else:
        row0, rows = row_block(rank, world, ROWS)
        local = _render_block(row0, rows)
    pack = _pack(local, lay, W)
    got = [None] * world
    dist.all_gather_object(got, (lay, pack))
    if rank == 0:
        frame = _assemble([p for _, p in got], [l for l, _ in got], H, W, bands, world)
        np.save(out_path, frame)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("bands", [0, 4, 8])
def test_two_rank_scene_camera_gather_layout(tmp_path, bands):
    """The scene-camera transport of eray_gather_frames across two gloo ranks: each rank's share
    laid out by the library's own layout code (eray_debug_gather_layout: rank rows, rectangles in
    local rows and column groups, pack offsets), packed and exchanged, assembled on rank 0 — equal
    to the single-process frame byte for byte.  (The kernels doing pack and assemble on the GPU
    are checked rank by rank in tests/test_gpu_gather.py.)"""
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_scene_gather_worker, args=(2, _free_port(), out, bands), nprocs=2, join=True,
                       start_method="spawn")
    got = np.load(out)
    want = _render_block(0, 2 * ROWS)
    assert (want != BG).any(axis=2).any()
    assert got.shape == want.shape and np.array_equal(got, want)


KEY = 0x1234_5678_9ABC_DEF0  # the frames' source key every rank's headers carry (kind 1: scene camera)


def _rotating_gather_worker(rank, world, port, out_dir, bands, B, rotate, fail_rank=-1, foreign_rank=-1):
    """Every rank packs B different frames (frame k: the rendered rows shifted by 37 k) where the
    library's schedule puts them, writes its transfer headers (the library's), runs the
    schedule's point-to-point transfers over gloo, and each root checks the headers it received
    (the library's assembly check) before it assembles its frames from its receive area.
    fail_rank: that rank cannot use its arguments (status ERAY_E_INVALID_ARGUMENT in its headers,
    no packs — the library's fail-safe path); foreign_rank: that rank's frames come from another
    source key.  Each rank saves the status it would return."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eray_amd import capi
    from eray_amd.dist import band_camera_rows, band_split

    H = world * ROWS
    rects = _rects_of(_render_block(0, H))
    lay = capi.gather_layout(rects, H, W, bands, world, rank)
    sp = band_split(rank, world, H, bands)
    local = np.zeros((sp["alloc_rows"], W, 3), np.uint8)
    local[: sp["rows"]] = _render_rows(band_camera_rows(rank, world, H, bands))
    lays = [None] * world
    dist.all_gather_object(lays, lay)
    nb = [l["bytes"] for l in lays]
    sched = capi.gather_schedule(nb, rank, B, rotate)
    buf = np.zeros(max(sched["need"], 1), np.uint8)
    status = capi.E_INVALID_ARGUMENT if rank == fail_rank else 0
    if not status:
        for k in range(B):
            at = sched["pack"][k]
            buf[at:at + lay["bytes"]] = _pack((local.astype(np.int32) + 37 * k).astype(np.uint8), lay, W)
    capi.gather_write_headers(nb, rank, B, rotate, buf, status=status, key=KEY + (rank == foreign_rank))
    t = torch.from_numpy(buf)
    reqs = [(dist.isend if op["send"] else dist.irecv)(t[op["off"]:op["off"] + op["bytes"]], int(op["peer"]))
            for op in sched["ops"]]
    for q in reqs:
        q.wait()
    if not status and sched["mine"]:
        status = capi.gather_check(nb, rank, B, rotate, buf, key=KEY)
    if not status:
        for j in range(sched["mine"]):
            packs = [buf[sched["recv"][q] + j * lays[q]["bytes"]:][:lays[q]["bytes"]] for q in range(world)]
            np.save(os.path.join(out_dir, f"r{rank}_f{j}.npy"), _assemble(packs, lays, H, W, bands, world))
    np.save(os.path.join(out_dir, f"status{rank}.npy"), np.array([status]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("B,rotate", [(3, True), (4, True), (3, False)])
def test_two_rank_gather_schedule_rotating_roots(tmp_path, B, rotate):
    """eray_gather_frames' batch schedule (the library's own: eray_debug_gather_schedule — pack
    offsets, receive areas, point-to-point transfers) across two gloo ranks: with
    ERAY_GATHER_ROTATE_ROOT frame k is assembled on rank k % 2 as its (k // 2)-th frame, else
    every frame on rank 0; each equals the frame restated from the ranks' packs in one process."""
    world, bands = 2, 4
    mp.start_processes(_rotating_gather_worker, args=(world, _free_port(), str(tmp_path), bands, B, rotate),
                       nprocs=world, join=True, start_method="spawn")
    from eray_amd import capi
    from eray_amd.dist import band_camera_rows, band_split
    H = world * ROWS
    full = _render_block(0, H)
    lays = [capi.gather_layout(_rects_of(full), H, W, bands, world, q) for q in range(world)]
    locals_ = []
    for q in range(world):
        sp = band_split(q, world, H, bands)
        loc = np.zeros((sp["alloc_rows"], W, 3), np.uint8)
        loc[: sp["rows"]] = _render_rows(band_camera_rows(q, world, H, bands))
        locals_.append(loc)
    for k in range(B):
        root, j = (k % world, k // world) if rotate else (0, k)
        got = np.load(str(tmp_path / f"r{root}_f{j}.npy"))
        packs = [_pack((locals_[q].astype(np.int32) + 37 * k).astype(np.uint8), lays[q], W) for q in range(world)]
        assert np.array_equal(got, _assemble(packs, lays, H, W, bands, world)), k
    assert np.array_equal(np.load(str(tmp_path / "r0_f0.npy")), full)
    assert all(np.load(str(tmp_path / f"status{q}.npy"))[0] == 0 for q in range(world))


@pytest.mark.parametrize("fail_rank,foreign_rank", [(1, -1), (0, -1), (-1, 1)])
def test_two_rank_gather_with_a_failed_rank(tmp_path, fail_rank, foreign_rank):
    """ADVICE r04 / VERDICT r04 item 5: a rank that cannot use its own arguments (null or unaligned
    buffers, frames it did not render) still takes part in the batch's transfers — its headers
    carry its error — and returns the error; the root of every frame finds the failed header
    (or, foreign_rank, a header of another source) and refuses the batch.  Both ranks return an
    error, no frame is written, and neither blocks (the gloo ranks join)."""
    world, bands, B = 2, 4, 3
    mp.start_processes(_rotating_gather_worker,
                       args=(world, _free_port(), str(tmp_path), bands, B, True, fail_rank, foreign_rank),
                       nprocs=world, join=True, start_method="spawn")
    from eray_amd import capi
    for q in range(world):
        assert np.load(str(tmp_path / f"status{q}.npy"))[0] == capi.E_INVALID_ARGUMENT, q
    assert not [f for f in os.listdir(tmp_path) if f.startswith("r")], "a root wrote a frame"


def _plan_verdict_worker(rank, world, port, out_dir, fail_rank, key_rank):
    """Each rank's record of a new plan exchange (status, kind, key), all-gathered over gloo, and
    the library's verdict on it (exchange_plan's)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eray_amd import capi
    status = capi.E_OUT_OF_MEMORY if rank == fail_rank else 0
    key = KEY + (rank == key_rank)
    rec = (status, 1, key & 0x7FFFFFFF, (key >> 32) & 0x7FFFFFFF)
    recs = [None] * world
    dist.all_gather_object(recs, rec)
    np.save(os.path.join(out_dir, f"verdict{rank}.npy"), np.array([capi.plan_verdict(recs, rank)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("fail_rank,key_rank,want", [(-1, -1, 0), (1, -1, "E_OUT_OF_MEMORY"),
                                                     (0, -1, "E_OUT_OF_MEMORY"), (-1, 0, "E_INVALID_ARGUMENT")])
def test_two_rank_plan_exchange_fails_together(tmp_path, fail_rank, key_rank, want):
    """A new plan's exchange (eray_gather_frames' first call after a new setup): one rank's own
    failure (an allocation, a frame lookup) or frames of another source makes every rank return
    the same kind of error; otherwise every rank accepts the plan."""
    world = 2
    mp.start_processes(_plan_verdict_worker, args=(world, _free_port(), str(tmp_path), fail_rank, key_rank),
                       nprocs=world, join=True, start_method="spawn")
    from eray_amd import capi
    expect = 0 if want == 0 else getattr(capi, want)
    assert [int(np.load(str(tmp_path / f"verdict{q}.npy"))[0]) for q in range(world)] == [expect] * world


def _replan_worker(rank, world, port, out_dir, null_rank):
    """Both ranks hold a cached plan for the old camera (kind 1, KEY), then render a new camera
    (the context's latest render: KEY + 7 on both, SPMD); rank `null_rank` passes local = NULL, so
    it cannot look its frames' source up.  Each rank decides with the library's own rule
    (eray_gather_frames' gather_replan) whether to exchange a new plan; the ranks that do exchange
    their records over gloo and take the library's verdict (exchange_plan's); a rank that would not
    exchange runs the cached plan's transfers instead (recorded as 'transfers')."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eray_amd import capi
    new_key = KEY + 7
    status = capi.E_INVALID_ARGUMENT if rank == null_rank else 0  # (null local: its own verdict)
    replan = capi.gather_replan(True, 1, KEY, 1, new_key)  # no input of this rank's buffers
    steps = [("exchange" if replan else "transfers")]
    steps_all = [None] * world
    dist.all_gather_object(steps_all, steps)  # (what each rank enters next; a mismatch would hang RCCL)
    verdict = None
    if replan and all(s == steps for s in steps_all):
        rec = (status, 1, new_key & 0x7FFFFFFF, (new_key >> 32) & 0x7FFFFFFF)
        recs = [None] * world
        dist.all_gather_object(recs, rec)
        verdict = capi.plan_verdict(recs, rank)
    np.save(os.path.join(out_dir, f"replan{rank}.npy"),
            np.array([int(replan), -1 if verdict is None else verdict, int(all(s == steps for s in steps_all))]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("null_rank", [1, 0])
def test_two_rank_new_camera_with_a_null_local_replans_together(tmp_path, null_rank):
    """VERDICT r05 W5 / ADVICE r05: the re-plan decision reads only state every rank shares (the
    cached plan, the context's latest render), so after both ranks set a new camera a rank passing
    local = NULL enters the same plan exchange as its peer — not the old plan's transfers — and
    both return the same error; neither blocks."""
    world = 2
    mp.start_processes(_replan_worker, args=(world, _free_port(), str(tmp_path), null_rank),
                       nprocs=world, join=True, start_method="spawn")
    from eray_amd import capi
    got = [np.load(str(tmp_path / f"replan{q}.npy")).tolist() for q in range(world)]
    assert got == [[1, capi.E_INVALID_ARGUMENT, 1]] * world, got


def test_gather_replan_rule():
    """The rule itself: a new plan when none is cached for the call's shared arguments or the
    context's latest render (kind, key) is not the plan's; the cached plan otherwise."""
    from eray_amd import capi
    assert capi.gather_replan(False, 1, KEY, 1, KEY)
    assert not capi.gather_replan(True, 1, KEY, 1, KEY)
    assert capi.gather_replan(True, 1, KEY, 1, KEY + 1)
    assert capi.gather_replan(True, 1, KEY, 2, KEY)  # a camera path after the scene camera


def test_gather_schedules_pair_up():
    """Host-only check of every rank's schedule for N = 1..8 ranks and batches of 1..12 frames:
    each send meets one receive of the same size from its peer, the packs of a rank's frames do
    not overlap and fit its buffer, and each rank roots the frames its rotation gives it."""
    from eray_amd import capi
    rng = np.random.default_rng(3)
    for N in range(1, 9):
        for B in (1, 2, 3, 7, 8, 12):
            for rotate in (False, True):
                nb = [int(48 * rng.integers(0, 40)) for _ in range(N)]
                S = [capi.gather_schedule(nb, r, B, rotate) for r in range(N)]
                for r in range(N):
                    assert S[r]["mine"] == (len(range(r, B, N)) if rotate else (B if r == 0 else 0))
                    spans = sorted((S[r]["pack"][k], S[r]["pack"][k] + nb[r]) for k in range(B))
                    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:])) and (not spans or spans[-1][1] <= S[r]["need"])
                    for op in S[r]["ops"]:
                        assert op["off"] + op["bytes"] <= S[r]["need"]
                        if op["send"]:
                            m = [o for o in S[op["peer"]]["ops"] if not o["send"] and o["peer"] == r]
                            assert len(m) == 1 and m[0]["bytes"] == op["bytes"], (N, B, rotate, r, op)
                    send_ops = [op for op in S[r]["ops"] if op["send"]]
                    # (every transfer ends with its sender's 16-B header)
                    assert sum(op["bytes"] for op in send_ops) == nb[r] * (B - S[r]["mine"]) + 16 * len(send_ops)
                    assert len(S[r]["headers"]) == len(send_ops) + (1 if S[r]["mine"] else 0)


def test_bench_frames_buffers_match_the_schedule():
    """bench.py sizes each rank's assembled-frames buffer with dist.frames_assembled; it must be
    what the library's schedule has the rank assemble (eray_debug_gather_schedule), for both
    root choices."""
    from eray_amd import capi
    from eray_amd.dist import frames_assembled
    for N in range(1, 9):
        for B in (1, 3, 8, 16, 32):
            for rotate in (False, True):
                for r in range(N):
                    assert frames_assembled(B, N, r, rotate) == capi.gather_schedule([48] * N, r, B, rotate)["mine"]

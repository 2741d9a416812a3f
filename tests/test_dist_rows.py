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

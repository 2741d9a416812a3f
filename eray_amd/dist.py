"""Multi-GPU decomposition of a frame: one process per GPU, row tiles, one gather.

Every pixel is independent (engine.rs:52-78), so rank r of n renders a block of `rows` camera rows
and the PPM body rows are gathered to rank 0.  The PPM body lists camera rows top-down
(image.rs:59-72: y = H-1 ... 0), so giving rank r the r-th block of FILE rows makes the gather a
plain concatenation in rank order: rank r owns camera rows [H - (r+1)*rows, H - r*rows), and the
library's fused PPM output of those rows is already in file order (eray_render_params.out_ppm).
No data-path collective other than that gather.  On the GPUs it is the library's own C-ABI gather
over an RCCL communicator (RowGather below; torch.distributed only carries the communicator's id
from rank 0 to the others):
  * eray_gather_rows, contiguous blocks: one ncclGather of the u8 rows to rank 0;
  * eray_gather_rows, interleaved bands (the default split): a coded transport — each rank encodes
    its rows (a uniform 64-pixel segment as one word), the packed counts are all-gathered and the
    host synchronises the stream once (point-to-point sizes must be known to post them), then
    grouped ncclSend / ncclRecv into rank 0 and one decode kernel — so this call blocks the host;
  * eray_gather_frames with ERAY_GATHER_SCENE_CAMERA (the bench's per-frame assembly): only the
    objects' pixel rectangles travel, with sizes fixed per camera (one exchange, one host
    synchronisation per camera setup), so batches of frames are gathered with no host round trip.
On CPU tests a gloo gather of the same blocks (gather_ppm_rows).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def row_block(rank: int, world: int, rows_per_rank: int) -> tuple[int, int]:
    """(row0, rows): the camera rows rank `rank` renders in a frame of world*rows_per_rank rows."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    height = world * rows_per_rank
    return height - (rank + 1) * rows_per_rank, rows_per_rank


BAND_ROWS = 4  # interleaved split: one 4-row sub-block band per turn (the finest the kernels take)


def band_split(rank: int, world: int, height: int, band: int = BAND_ROWS) -> dict:
    """Interleaved row bands (load balance): rank r renders camera-row bands r,
    r + world, ... of `band` rows — wherever the scene sits, every rank gets an equal share of it.
    Returns the eray_render_params fields (row0, rows, band_rows, band_stride) and `alloc_rows`,
    the rows each rank's local buffers hold for the gather (rank 0's count, the largest)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    if band < 4 or band & (band - 1):
        raise ValueError("bands must be a power of two of at least 4 rows")
    bands, tail = divmod(height, band)
    rows = (bands // world + (1 if rank < bands % world else 0)) * band + (tail if tail and bands % world == rank else 0)
    rows0 = (bands // world + (1 if 0 < bands % world else 0)) * band + (tail if tail and bands % world == 0 else 0)
    return dict(row0=rank * band, rows=rows, band_rows=band, band_stride=world * band, alloc_rows=rows0)


def frames_assembled(batch: int, world: int, rank: int, rotate: bool) -> int:
    """Frames of a batch of `batch` that `rank` assembles in eray_gather_frames' scene-camera
    gather: every frame on rank 0, or (ERAY_GATHER_ROTATE_ROOT) frames k = rank, rank + world, ...
    — the size of the frames buffer that rank passes."""
    if not rotate:
        return batch if rank == 0 else 0
    return max(0, (batch - rank + world - 1) // world)


def band_camera_rows(rank: int, world: int, height: int, band: int = BAND_ROWS) -> list[int]:
    """The camera rows of rank's local rows, in order (tests)."""
    sp = band_split(rank, world, height, band)
    return [sp["row0"] + (j // band) * sp["band_stride"] + j % band for j in range(sp["rows"])]


class RowGather:
    """The frame gather through the C-ABI (eray_gather_rows over an RCCL communicator made by
    eray_comm_init); `group` carries rank 0's unique id to the others (any backend)."""

    def __init__(self, ctx, world: int, rank: int):
        from . import capi
        self.ctx, self.world, self.rank = ctx, world, rank
        uid = [capi.comm_unique_id() if rank == 0 else None]
        if world > 1:
            dist.broadcast_object_list(uid, src=0)
        self.comm = ctx.comm_init(world, rank, uid[0])

    def __call__(self, local: torch.Tensor, frame: torch.Tensor | None, height: int, band_rows: int = 0) -> None:
        """local: this rank's fused PPM rows (bands: padded to band_split's alloc_rows); frame:
        rank 0's height x width x 3 PPM body."""
        width = local.shape[1]
        self.ctx.gather_rows(self.comm, local.data_ptr(), frame.data_ptr() if frame is not None else None,
                             height, width, band_rows)

    def close(self) -> None:
        from . import capi
        if self.comm:
            capi.comm_destroy(self.comm)
            self.comm = None


def gather_ppm_rows(local: torch.Tensor, frame: torch.Tensor | None, world: int, rank: int,
                    band_rows: int = 0) -> None:
    """Gather every rank's PPM rows into rank 0's (H, W, 3) uint8 `frame` (file order) with
    torch.distributed (the CPU tests' gloo path; GPU jobs use RowGather).  band_rows = 0: equal
    blocks of file rows in rank order; else interleaved bands (band_split), every rank's local
    buffer padded to alloc_rows, reordered on rank 0.  Other ranks pass frame=None."""
    if world == 1 and not band_rows:
        if frame is not None and frame.data_ptr() != local.data_ptr():
            frame.copy_(local)
        return
    host = local.cpu() if local.is_cuda else local
    if world == 1:
        parts = [host]
    else:
        parts = [torch.empty_like(host) for _ in range(world)] if rank == 0 else None
        dist.gather(host, parts, dst=0)
    if rank != 0:
        return
    if not band_rows:
        frame.copy_(torch.cat(parts, 0))
        return
    H = frame.shape[0]
    out = torch.empty_like(frame, device="cpu")
    for r in range(world):
        n = band_split(r, world, H, band_rows)["rows"]
        cams = band_camera_rows(r, world, H, band_rows)
        for k in range(n):  # block row k = local row n - 1 - k (local file order)
            out[H - 1 - cams[n - 1 - k]] = parts[r][k]
    frame.copy_(out)

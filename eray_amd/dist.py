"""Multi-GPU decomposition of a frame: one process per GPU, row tiles, one gather.

Every pixel is independent (engine.rs:52-78), so rank r of n renders a block of `rows` camera rows
and the PPM body rows are gathered to rank 0.  The PPM body lists camera rows top-down
(image.rs:59-72: y = H-1 ... 0), so giving rank r the r-th block of FILE rows makes the gather a
plain concatenation in rank order: rank r owns camera rows [H - (r+1)*rows, H - r*rows), and the
library's fused PPM output of those rows is already in file order (eray_render_params.out_ppm).
No data-path collective other than that gather: on the GPUs it is the library's own C-ABI gather
(eray_gather_rows, one RCCL ncclGather over xGMI; RowGather below — torch.distributed only carries
the communicator's id from rank 0 to the others), on CPU tests a gloo gather of the same blocks.
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

    def __call__(self, local: torch.Tensor, frame: torch.Tensor | None) -> None:
        rows, width = local.shape[0], local.shape[1]
        self.ctx.gather_rows(self.comm, local.data_ptr(), frame.data_ptr() if frame is not None else None,
                             rows, width)

    def close(self) -> None:
        from . import capi
        if self.comm:
            capi.comm_destroy(self.comm)
            self.comm = None


def gather_ppm_rows(local: torch.Tensor, frame: torch.Tensor | None, world: int, rank: int) -> None:
    """Gather every rank's (rows, W, 3) uint8 PPM rows into rank 0's (world*rows, W, 3) `frame`
    (file order).  Other ranks pass frame=None.  One collective, rank order = file order."""
    if world == 1:
        if frame is not None and frame.data_ptr() != local.data_ptr():
            frame.copy_(local)
        return
    if local.is_cuda and dist.get_backend() == "gloo":  # gloo gathers host tensors
        host = local.cpu()
        parts = [torch.empty_like(host) for _ in range(world)] if rank == 0 else None
        dist.gather(host, parts, dst=0)
        if rank == 0:
            frame.copy_(torch.cat(parts, 0))
        return
    dist.gather(local, list(frame.chunk(world, 0)) if rank == 0 else None, dst=0)

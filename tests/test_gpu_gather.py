"""The multi-GPU gather through the C-ABI (eray_gather_rows over an RCCL communicator from
eray_comm_init), on the one GPU of the box: a one-rank communicator gathers a rendered block into
the frame buffer (and in place).  More ranks need one GPU each (RCCL puts one rank per device):
the 2-rank split and gather order are covered on CPU (tests/test_dist_rows.py) and the tiles'
pixels on the GPU (tests/test_gpu_configs.py)."""
import numpy as np
import pytest

from eray_amd import capi
from eray_amd.frame import MainScene

pytestmark = pytest.mark.gpu


def test_one_rank_gather_through_rccl(gpu, cube):
    W, H = 256, 144
    sc = MainScene(gpu, *cube, W, H, texture=64, fov=(16.0, 9.0))
    local = gpu.empty((H, W, 3), np.uint8)
    frame = gpu.empty((H, W, 3), np.uint8)
    comm = None
    try:
        gpu.memset(frame.ptr, 0, frame.nbytes)
        gpu.render(W, H, out_ppm=local.ptr)
        comm = gpu.comm_init(1, 0, capi.comm_unique_id())
        gpu.gather_rows(comm, local.ptr, frame.ptr, H, W)
        gpu.synchronize()
        want = local.numpy()
        assert (want != 0).any()
        assert np.array_equal(frame.numpy(), want)
        gpu.gather_rows(comm, local.ptr, local.ptr, H, W)  # in place
        gpu.synchronize()
        assert np.array_equal(local.numpy(), want)
        with pytest.raises(capi.ErayError):
            gpu.gather_rows(comm, local.ptr, None, H, W)  # rank 0 needs the frame
    finally:
        if comm:
            capi.comm_destroy(comm)
        local.free()
        frame.free()
        sc.close()

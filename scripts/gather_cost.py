"""Cost of eray_gather_rows on a one-rank communicator (diagnostics): the contiguous gather (one
ncclGather) and the banded coded gather (encode, count all-gather + host sync, decode) of the C2
frame's PPM rows, and of a 7680x4320 frame."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import frame_camera_fov  # noqa: E402
from eray_amd import capi  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402

mesh = load_obj_file(os.path.join(ROOT, "objects", "cube.obj"))
ctx = capi.Context(0)
torch.cuda.init()
comm = ctx.comm_init(1, 0, capi.comm_unique_id())
for W, H in ((1920, 1080), (7680, 4320)):
    sc = MainScene(ctx, *mesh, W, H, texture=256, fov=frame_camera_fov(W, H))
    local = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
    frame = torch.empty((H, W, 3), dtype=torch.uint8, device="cuda")
    ctx.render(W, H, out_ppm=local.data_ptr())
    for band in (0, 4):
        for _ in range(3):
            ctx.gather_rows(comm, local.data_ptr(), frame.data_ptr(), H, W, band_rows=band)
        torch.cuda.synchronize()
        ts = []
        for _ in range(20):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.gather_rows(comm, local.data_ptr(), frame.data_ptr(), H, W, band_rows=band)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        assert torch.equal(frame, local)
        print(f"{W}x{H} band_rows={band}: {np.median(ts) * 1e6:.1f} us", flush=True)
    sc.close()
capi.comm_destroy(comm)

"""Diagnostics: the bench's timed-region shape at C2 (a plan prepared ahead, W warmup frames from
another plan, then K frames timed once) against repeated calls of the same plan: where the 20-step
wall time goes (call return, synchronize return), per attempt."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import frame_camera_fov  # noqa: E402
from eray_amd import capi  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402
from eray_amd.objfile import load_obj_file  # noqa: E402

W, H, K, WARM = 1920, 1080, int(os.environ.get("K", 20)), int(os.environ.get("WARM", 5))
mesh = load_obj_file(os.path.join(ROOT, "objects", "cube.obj"))
ctx = capi.Context(0)
torch.cuda.init()
sc = MainScene(ctx, *mesh, W, H, texture=1024, fov=frame_camera_fov(W, H))
F = ctx.frames_per_launch(W, H, slots=64)
rgb = torch.empty((F, H, W, 3), dtype=torch.float32, device="cuda")
ppm = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda")
kw = dict(out_rgb=rgb.data_ptr(), out_ppm=ppm.data_ptr(), ring=capi.frame_ring(F, H, W, F))
ctx.render_frames(min(F, K), W, H, prepare_only=True, **kw)
ctx.render_frames(K, W, H, prepare_only=True, **kw)
ctx.render_frames(WARM, W, H, **kw)
torch.cuda.synchronize()


def once(tag, pre=None):
    if pre:
        pre()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ctx.render_frames(K, W, H, **kw)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{tag:28s} call {(t1 - t0) * 1e6:7.1f} us  call+sync {(t2 - t0) * 1e6:7.1f} us  "
          f"per frame {(t2 - t0) * 1e6 / K:6.2f}", flush=True)


once("first launch of the plan")
once("second launch")
once("third launch")
time.sleep(0.05)
once("after 50 ms idle")
time.sleep(0.002)
once("after 2 ms idle")
once("after warm 5", lambda: ctx.render_frames(WARM, W, H, **kw))
once("after warm 5 (again)", lambda: ctx.render_frames(WARM, W, H, **kw))
busy = torch.empty(64 << 20, device="cuda")
once("after 256 MB fill", lambda: busy.fill_(1.0))
for i in range(3):
    once(f"back to back {i}")
d = ctx.render_frames(K, W, H, timed=True, **kw) * 1e3 * K
print(f"device {d:.1f} us for {K} frames (events)")

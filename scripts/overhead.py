"""Fixed cost of a timed bench region (diagnostics): wall time of render_frames(K) + synchronize
for several K at C2, and its host-side parts."""
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

W, H = 1920, 1080
mesh = load_obj_file(os.path.join(ROOT, "objects", "cube.obj"))
ctx = capi.Context(0)
torch.cuda.init()
sc = MainScene(ctx, *mesh, W, H, texture=1024, fov=frame_camera_fov(W, H))
F = ctx.frames_per_launch(W, H, slots=64)
rgb = torch.empty((F, H, W, 3), dtype=torch.float32, device="cuda")
ppm = torch.empty((F, H, W, 3), dtype=torch.uint8, device="cuda")
kw = dict(out_rgb=rgb.data_ptr(), out_ppm=ppm.data_ptr(), ring=capi.frame_ring(F, H, W, F))
print(f"frames per launch {F}")
for K in (1, 2, 5, 8, 16, 20, 24, 64, 200):
    ctx.render_frames(K, W, H, prepare_only=True, **kw)
    ctx.render_frames(K, W, H, **kw)
    torch.cuda.synchronize()
    ts = []
    for _ in range(30):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.render_frames(K, W, H, **kw)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ts.append((t1 - t0, t2 - t0))
    call = np.median([a for a, _ in ts]) * 1e6
    tot = np.median([b for _, b in ts]) * 1e6
    print(f"K={K:4d}: call {call:7.1f} us, call+sync {tot:8.1f} us, per frame {tot / K:6.2f} us", flush=True)
t = []
for _ in range(200):
    t0 = time.perf_counter()
    capi.lib().eray_abi_version()
    t.append(time.perf_counter() - t0)
print(f"ctypes call {np.median(t) * 1e6:.2f} us")
t = []
for _ in range(200):
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    t.append(time.perf_counter() - t0)
print(f"idle synchronize {np.median(t) * 1e6:.2f} us")
# device time of the 20-frame call (HIP events on the library's stream) vs its wall time
for K in (20, 200):
    d = np.median([ctx.render_frames(K, W, H, timed=True, **kw) for _ in range(10)]) * 1e3 * K
    print(f"K={K}: device {d:.1f} us (events around the graph launches)")

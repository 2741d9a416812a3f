"""Per-wave instruction counts of the C2 detail path (diagnostics, not part of the product).

Renders 20 single-launch frames of the cube's block row 538..542 (detail + fill waves), then 20 of
rows 0..4 (fill waves only); run under `rocprofv3 --pmc ... --kernel-include-regex frame_kernel`
the difference of the two dispatch groups' SQ counters is the detail waves' work.
`python scripts/pmc_detail.py report <dir>` prints it.
"""
import csv
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
N = 20


def render():
    import numpy as np
    import torch  # noqa: F401
    from eray_amd import capi
    from eray_amd.frame import MainScene
    from eray_amd.objfile import load_obj_file
    W, H = 1920, 1080
    mesh = load_obj_file(os.path.join(ROOT, "objects", "cube.obj"))
    ctx = capi.Context(0)
    rgb = ctx.empty((H, W, 3), np.float32)
    ppm = ctx.empty((H, W, 3), np.uint8)
    sc = MainScene(ctx, *mesh, W, H)
    for row0 in (538, 0):
        for _ in range(N):
            ctx.render(W, H, row0=row0, rows=4, out_rgb=rgb.ptr, out_ppm=ppm.ptr)
        ctx.synchronize()
    sc.close()


def report(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    by = {}
    for r in rows:
        by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(by)
    a, b = ids[:N], ids[N:2 * N]
    names = sorted(by[ids[0]])
    for n in names:
        va = sum(by[i].get(n, 0) for i in a) / len(a)
        vb = sum(by[i].get(n, 0) for i in b) / len(b)
        print(f"{n:24s} cube row {va:12.1f}  background {vb:12.1f}  detail {va - vb:12.1f}")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "report":
        report(sys.argv[2])
    else:
        render()

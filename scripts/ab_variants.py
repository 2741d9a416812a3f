"""A/B timing of frame-kernel design choices (diagnostics, not part of the product).

`python scripts/ab_variants.py build` compiles lib/liberay_hip_<name>.so for each variant below
(here, no GPU); `python scripts/ab_variants.py run` times the C2 frame (and a 4-row frame) with
each library in a child process on the GPU box.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VARIANTS = {
    "base": (),
    "batch4": ("ERAY_AB_BATCH_FIXED",),
    "lazyray": ("ERAY_AB_LAZY_RAY",),
    "lds_uniform": ("ERAY_AB_LDS_UNIFORM",),
    "sload_hot": ("ERAY_AB_SLOAD_HOT",),
    "global": ("ERAY_AB_NO_LDS_SCENE",),
    "x_noshadow": ("ERAY_AB_X_NO_SHADOW",),
    "x_notex": ("ERAY_AB_X_NO_TEXTURE",),
    "x_neither": ("ERAY_AB_X_NO_SHADOW", "ERAY_AB_X_NO_TEXTURE"),
    "x_nofill": ("ERAY_AB_X_NO_FILL",),
    "x_nodetail": ("ERAY_AB_X_NO_DETAIL",),
    "st_nt": ("ERAY_AB_STORE_NT",),
    "x_nowide": ("ERAY_AB_X_NO_WIDE",),
    "x_nopairs": ("ERAY_AB_X_NO_PAIRS",),
    "x_nobinwork": ("ERAY_AB_X_NO_WIDE", "ERAY_AB_X_NO_PAIRS"),
}

CHILD = r"""
import os, sys, time
sys.path.insert(0, os.environ["ROOT"])
import numpy as np, torch
from eray_amd import capi
from eray_amd.frame import MainScene
from eray_amd.objfile import load_obj_file
W, H = int(os.environ.get("ERAY_AB_W", 1920)), int(os.environ.get("ERAY_AB_H", 1080))
mesh = load_obj_file(os.environ.get("ERAY_AB_MESH") or os.path.join(os.environ["ROOT"], "objects", "cube.obj"))
ctx = capi.Context(0)
rgb = ctx.empty((H, W, 3), np.float32); ppm = ctx.empty((H, W, 3), np.uint8)
from bench import frame_camera_fov
sc = MainScene(ctx, *mesh, W, H, fov=frame_camera_fov(W, H))
out = []
for row0, rows in ((0, H), (H // 2 - 2, 4)):
    kw = dict(row0=row0, rows=rows, out_rgb=rgb.ptr, out_ppm=ppm.ptr)
    ctx.render_frames(64, W, H, prepare_only=True, **kw)
    ctx.render_frames(64, W, H, **kw); ctx.synchronize()
    best = min(ctx.render_frames(640, W, H, timed=True, **kw) for _ in range(5))
    out.append(f"{rows:5d} rows {best * 1e3:7.2f} us")
print(os.environ["ERAY_LIB"].split("_hip")[-1], " | ".join(out), flush=True)
"""


def build_head(rev="HEAD"):
    """lib/liberay_hip_head.so from the committed sources (the control of an A/B run)."""
    import shutil
    import tempfile
    from eray_amd import build as B
    tmp = tempfile.mkdtemp(prefix="eray_head_")
    subprocess.run(f"git -C {ROOT} archive {rev} eray_amd/csrc include | tar -x -C {tmp}", shell=True, check=True)
    csrc, inc = os.path.join(tmp, "eray_amd", "csrc"), os.path.join(tmp, "include")
    flags = [f if not f.startswith("-I") else "-I" + inc for f in B.CXXFLAGS]
    objs = []
    for src in B.SOURCES:
        o = os.path.join(tmp, src + ".o")
        lang = [] if src.endswith(".hip") else ["-x", "hip"]
        subprocess.run([B.hipcc(), *flags, *lang, "-c", os.path.join(csrc, src), "-o", o], check=True)
        objs.append(o)
    out = os.path.join(B.LIB_DIR, "liberay_hip_head.so")
    subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", out, *objs], check=True)
    shutil.rmtree(tmp)
    return out


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "run"
    names = sys.argv[2:] or list(VARIANTS)
    if mode == "build":
        from eray_amd.build import build
        for n in names:
            if n == "head":
                print(build_head(), flush=True)
                continue
            print(build(variant=n, defines=VARIANTS[n]), flush=True)
        return
    env = dict(os.environ, ROOT=ROOT)
    for n in names:
        env["ERAY_LIB"] = os.path.join(ROOT, "eray_amd", "lib", f"liberay_hip_{n}.so")
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, timeout=300)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()

"""Diagnostics: the general tracer on a binned mesh (C3 by default) — bin statistics of its setup
(keep_all bins) and device ms per frame for AA = 0 (frame kernel), 1, 2, 4."""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from eray_amd import capi, meshgen  # noqa: E402
from eray_amd.frame import MainScene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=10)
    a = ap.parse_args()
    v, n, t, fv, ft, fn = meshgen.displaced_sphere(**meshgen.STANDIN_70K)
    mesh = (np.ascontiguousarray(v[fv].reshape(-1, 9)), np.ascontiguousarray(n[fn].reshape(-1, 9)),
            np.ascontiguousarray(t[ft].reshape(-1, 6)))
    W, H = a.width, a.height
    ctx = capi.Context(0)
    sc = MainScene(ctx, *mesh, W, H, texture=1024, fov=(16.0, 9.0))
    rgb = ctx.empty((H, W, 3), np.float32)
    L = capi.lib()
    out = {"frame": [W, H]}
    for aa in (0, 1, 2, 4):
        kw = dict(out_rgb=rgb.ptr, anti_aliasing=aa, aa_seed=7)
        ctx.render(W, H, **kw)
        ctx.synchronize()
        st = (C.c_uint64 * 14)()
        L.eray_debug_bin_stats.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]
        L.eray_debug_bin_stats(ctx._h, 0, st)
        state = (C.c_uint8 * 176)()
        rect = (C.c_int32 * 4)()
        L.eray_debug_setup_state.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.POINTER(C.c_int32)]
        L.eray_debug_setup_state(ctx._h, 0, state, rect)
        words = np.frombuffer(bytes(state), np.uint32)
        ctx.render_frames(a.frames, W, H, prepare_only=True, **kw)
        ms = min(ctx.render_frames(a.frames, W, H, timed=True, **kw) for _ in range(3))
        heavy = int(st[10])
        cnt = C.c_uint32()
        tri = (C.c_uint32 * 4096)()
        msk = (C.c_uint64 * 4096)()
        L.eray_debug_bin_dump.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32),
                                          C.POINTER(C.c_uint64), C.c_uint32, C.POINTER(C.c_uint32)]
        L.eray_debug_bin_dump(ctx._h, 0, heavy, tri, msk, 4096, C.byref(cnt))
        pops = [bin(msk[i]).count("1") for i in range(min(cnt.value, 4096))]
        faces = [int(tri[i]) for i in range(min(cnt.value, 4096))]
        bins_x = (W + 15) // 16
        if aa == 4:
            np.savez(os.path.join(os.environ.get("PROBE_OUT", "/tmp"), "heavy_bin.npz"), faces=np.array(faces),
                     masks=np.array([int(msk[i]) for i in range(len(faces))], np.uint64), bin=heavy, bins_x=bins_x)
        out[f"aa{aa}"] = {"bins_over_64": int(st[11]), "bins_over_heavy_min": int(st[12]), "heavy_bin_xy": [16 * (heavy % bins_x), 4 * (heavy // bins_x) - 4],
                          "heavy_pop_hist": np.histogram(pops, bins=[0, 1, 2, 4, 8, 16, 32, 65])[0].tolist(),
                          "frame_ms": round(ms, 4), "bins": int(st[0]), "entries": int(st[1]),
                          "most_in_bin": int(st[3]), "nonempty_bins": int(st[4]), "rect": list(rect),
                          "state_bin_entries": int(words[10]), "overflow": int(words[11]),
                          "capacity": int(L.eray_debug_bin_capacity(ctx._h))}
        print(json.dumps(out[f"aa{aa}"]), flush=True)
    rgb.free()
    sc.close()
    ctx.close()


if __name__ == "__main__":
    main()

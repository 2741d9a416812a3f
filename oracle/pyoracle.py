"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.  It
loads oracle/_build/liberay_oracle.so, the literal C++ restatement of the reference
(oracle/eray_oracle.cpp), and never the product library.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liberay_oracle.so")

f32p = C.POINTER(C.c_float)


class Image(C.Structure):
    _fields_ = [("data", f32p), ("width", C.c_uint32), ("height", C.c_uint32)]


class Material(C.Structure):
    _fields_ = [("color", Image), ("diffuse", Image), ("specular", Image),
                ("specular_power", Image), ("reflection", Image)]


class Object(C.Structure):
    _fields_ = [("positions", f32p), ("normals", f32p), ("uvs", f32p),
                ("triangle_count", C.c_uint32), ("bbox_min", C.c_float * 3),
                ("bbox_max", C.c_float * 3), ("material", Material)]


class Camera(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("fov0", C.c_float), ("fov1", C.c_float),
                ("width", C.c_uint32), ("z_dist", C.c_float)]


class Light(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("variant", C.c_int32),
                ("color", C.c_float * 3), ("brightness", C.c_float)]


class Stats(C.Structure):
    _fields_ = [("primary_tests", C.c_uint64), ("shadow_tests", C.c_uint64),
                ("hit_pixels", C.c_uint64)]


def build() -> str:
    """Compile the oracle with its committed recipe (oracle/Makefile)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.oracle_cosf.restype = C.c_float
        L.oracle_cosf.argtypes = [C.c_float]
        L.oracle_powf.restype = C.c_float
        L.oracle_powf.argtypes = [C.c_float, C.c_float]
        L.oracle_ppm_header.restype = C.c_size_t
        L.oracle_jitter.restype = C.c_float
        L.oracle_jitter.argtypes = [C.c_uint32]
        _lib = L
    return _lib


def _fp(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(f32p)


def _img(a, w=0, h=0):
    if a is None:
        return Image(None, 0, 0)
    return Image(_fp(a), w, h)


# ---------------------------------------------------------------- small known answers ----
def vec_dot(a, b):
    out = C.c_float()
    lib().oracle_vec_dot((C.c_float * 3)(*a), (C.c_float * 3)(*b), C.byref(out))
    return out.value


def vec_cross(a, b):
    out = (C.c_float * 3)()
    lib().oracle_vec_cross((C.c_float * 3)(*a), (C.c_float * 3)(*b), out)
    return np.array(out[:], dtype=np.float32)


def vec_angle(a, b):
    out = C.c_float()
    lib().oracle_vec_angle((C.c_float * 3)(*a), (C.c_float * 3)(*b), C.byref(out))
    return out.value


def triangle_project(tri_pos, point):
    out = (C.c_float * 3)()
    lib().oracle_triangle_project((C.c_float * 9)(*tri_pos), (C.c_float * 3)(*point), out)
    return np.array(out[:], dtype=np.float32)


def triangle_intersects(pos, nrm, start, direction):
    p, n, b = (C.c_float * 3)(), (C.c_float * 3)(), (C.c_float * 3)()
    hit = lib().oracle_triangle_intersects((C.c_float * 9)(*pos), (C.c_float * 9)(*nrm),
                                           (C.c_float * 3)(*start), (C.c_float * 3)(*direction),
                                           p, n, b)
    if not hit:
        return None
    return (np.array(p[:], np.float32), np.array(n[:], np.float32), np.array(b[:], np.float32))


def camera(center=(0.0, 0.0, 5.0), fov=(60.0, 60.0), width=1024, z_dist=1.0):
    return Camera((C.c_float * 3)(*center), fov[0], fov[1], width, z_dist)


def camera_size(cam):
    w, h = C.c_uint32(), C.c_uint32()
    lib().oracle_camera_size(C.byref(cam), C.byref(w), C.byref(h))
    return w.value, h.value


def pixel_to_ray(cam, x, y):
    s, d = (C.c_float * 3)(), (C.c_float * 3)()
    lib().oracle_pixel_to_ray(C.byref(cam), C.c_float(x), C.c_float(y), s, d)
    return np.array(s[:], np.float32), np.array(d[:], np.float32)


def cosf(x):
    return lib().oracle_cosf(x)


def powf(x, y):
    return lib().oracle_powf(x, y)


# ---------------------------------------------------------------- shaderlib -------------
def node_wave(w, h, x_fac=1.0, y_fac=1.0):
    out = np.empty((h, w), np.float32)
    assert lib().oracle_node_wave(w, h, C.c_float(x_fac), C.c_float(y_fac), _fp(out)) == 0
    return out


def node_rgb(w, h, r, g, b):
    out = np.empty((h, w, 3), np.float32)
    st = lib().oracle_node_rgb(w, h, _img(r, r.shape[1], r.shape[0]), _img(g, g.shape[1], g.shape[0]),
                               _img(b, b.shape[1], b.shape[0]), _fp(out))
    if st:
        raise ValueError(f"oracle_node_rgb status {st}")
    return out


def node_flat_color(w, h, r, g, b):
    out = np.empty((h, w, 3), np.float32)
    lib().oracle_node_flat_color(w, h, C.c_float(r), C.c_float(g), C.c_float(b), _fp(out))
    return out


def node_mix_color(w, h, left, right, factor=0.5):
    out = np.empty((h, w, 3), np.float32)
    st = lib().oracle_node_mix_color(w, h, _img(left, left.shape[1], left.shape[0]),
                                     _img(right, right.shape[1], right.shape[0]), C.c_float(factor),
                                     _fp(out))
    if st:
        raise ValueError(f"oracle_node_mix_color status {st}")
    return out


def example_material(w=1024, h=1024, x_fac=1.0, y_fac=1.0, r=1.0, g=0.0, b=0.0, factor=0.5):
    """main.rs:22-42's inputs by default: returns (color HxWx3, diffuse HxW)."""
    color = np.empty((h, w, 3), np.float32)
    diffuse = np.empty((h, w), np.float32)
    st = lib().oracle_example_material(w, h, C.c_float(x_fac), C.c_float(y_fac), C.c_float(r),
                                       C.c_float(g), C.c_float(b), C.c_float(factor), _fp(color),
                                       _fp(diffuse))
    assert st == 0, st
    return color, diffuse


# ---------------------------------------------------------------- render ----------------
class Scene:
    """Holds numpy buffers alive while ctypes structs point into them."""

    def __init__(self):
        self.objects = []
        self.lights = []
        self._keep = []

    def add_object(self, positions, normals, uvs, bbox_min=(0, 0, 0), bbox_max=(0, 0, 0),
                   color=None, diffuse=None, specular=None, specular_power=None, reflection=None):
        P = np.ascontiguousarray(positions, np.float32).reshape(-1, 9)
        N = np.ascontiguousarray(normals, np.float32).reshape(-1, 9)
        U = np.ascontiguousarray(uvs, np.float32).reshape(-1, 6)
        imgs = []
        for a, ch in ((color, 3), (diffuse, 1), (specular, 1), (specular_power, 1), (reflection, 1)):
            if a is None:
                imgs.append(Image(None, 0, 0))
            else:
                a = np.ascontiguousarray(a, np.float32)
                self._keep.append(a)
                imgs.append(Image(_fp(a), a.shape[1], a.shape[0]))
        self._keep += [P, N, U]
        o = Object(_fp(P) if P.size else None, _fp(N) if N.size else None, _fp(U) if U.size else None,
                   P.shape[0], (C.c_float * 3)(*bbox_min), (C.c_float * 3)(*bbox_max), Material(*imgs))
        self.objects.append(o)
        return self

    def add_light(self, position, variant, color=(1.0, 1.0, 1.0), brightness=1.0):
        self.lights.append(Light((C.c_float * 3)(*position), 1 if variant in (1, "ambient") else 0,
                                 (C.c_float * 3)(*color), brightness))
        return self


def render(scene: Scene, cam: Camera, image_width=None, image_height=None, row0=0, rows=None,
           bounces=0, want_faces=False, anti_aliasing=0, seed=0):
    W, H = camera_size(cam)
    image_width = W if image_width is None else image_width
    image_height = H if image_height is None else image_height
    rows = H - row0 if rows is None else rows
    out = np.zeros((rows, image_width, 3), np.float32)
    faces = np.full((rows, image_width), -1, np.int32) if want_faces else None
    objs = (Object * max(1, len(scene.objects)))(*scene.objects)
    lights = (Light * max(1, len(scene.lights)))(*scene.lights)
    st = Stats()
    rc = lib().oracle_render_aa(objs, len(scene.objects), lights, len(scene.lights), C.byref(cam),
                                image_width, image_height, row0, rows, bounces, anti_aliasing,
                                C.c_uint64(seed), _fp(out),
                             faces.ctypes.data_as(C.POINTER(C.c_int32)) if want_faces else None,
                             None, C.byref(st))
    if rc:
        raise ValueError(f"oracle_render status {rc}")
    stats = dict(primary_tests=st.primary_tests, shadow_tests=st.shadow_tests, hit_pixels=st.hit_pixels)
    return (out, faces, stats) if want_faces else (out, stats)


def render_span(scene: Scene, cam: Camera, row0: int, rows: int, x0: int, cols: int):
    """Pixels [x0, x0+cols) x camera rows [row0, row0+rows) of the frame (AA = 0, no bounces):
    returns (rgb rows x cols x 3, faces rows x cols, stats)."""
    out = np.zeros((rows, cols, 3), np.float32)
    faces = np.full((rows, cols), -1, np.int32)
    objs = (Object * max(1, len(scene.objects)))(*scene.objects)
    lights = (Light * max(1, len(scene.lights)))(*scene.lights)
    st = Stats()
    rc = lib().oracle_render_span(objs, len(scene.objects), lights, len(scene.lights), C.byref(cam), row0, rows,
                                  x0, cols, _fp(out), faces.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(st))
    if rc:
        raise ValueError(f"oracle_render_span status {rc}")
    return out, faces, dict(primary_tests=st.primary_tests, shadow_tests=st.shadow_tests, hit_pixels=st.hit_pixels)


def philox4x32_10(ctr, key):
    """Philox4x32-10 block (the anti-aliasing jitter stream, oracle_render_aa)."""
    c, k, o = (C.c_uint32 * 4)(*ctr), (C.c_uint32 * 2)(*key), (C.c_uint32 * 4)()
    lib().oracle_philox4x32_10(c, k, o)
    return list(o)


def jitter(word: int) -> float:
    """rand 0.8 gen_range(-1.0..1.0) for f32 from one 32-bit word."""
    return lib().oracle_jitter(word)


def ppm_bytes(rgb: np.ndarray) -> bytes:
    rgb = np.ascontiguousarray(rgb, np.float32)
    h, w = rgb.shape[:2]
    out = np.empty(h * w * 3, np.uint8)
    lib().oracle_ppm_bytes(_fp(rgb), w, h, out.ctypes.data_as(C.POINTER(C.c_uint8)))
    buf = C.create_string_buffer(64)
    n = lib().oracle_ppm_header(w, h, buf, 64)
    return buf.raw[:n] + out.tobytes()


def load_obj(text: str | bytes):
    if isinstance(text, str):
        text = text.encode()
    P, N, U = f32p(), f32p(), f32p()
    T = C.c_uint32()
    err = C.create_string_buffer(256)
    rc = lib().oracle_load_obj(text, len(text), C.byref(P), C.byref(N), C.byref(U), C.byref(T), err, 256)
    if rc:
        raise ValueError(f"load_obj error {rc}: {err.value.decode()}")
    n = T.value
    try:
        pos = np.ctypeslib.as_array(P, shape=(max(n, 1) * 9,))[: n * 9].copy().reshape(n, 9)
        nrm = np.ctypeslib.as_array(N, shape=(max(n, 1) * 9,))[: n * 9].copy().reshape(n, 9)
        uv = np.ctypeslib.as_array(U, shape=(max(n, 1) * 6,))[: n * 6].copy().reshape(n, 6)
    finally:
        for p in (P, N, U):
            lib().oracle_free(p)
    return pos, nrm, uv


def main_rs_scene(positions, normals, uvs, texture=1024):
    """The scene of main.rs:17-65 around the given mesh, with the example material."""
    color, diffuse = example_material(texture, texture)
    s = Scene()
    s.add_object(positions, normals, uvs, color=color, diffuse=diffuse)
    s.add_light((0.0, 2.0, 0.0), "ambient", (1.0, 1.0, 1.0), 0.2)
    s.add_light((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0)
    return s

"""ctypes binding of include/eray_hip.h (the product C-ABI, eray_amd/lib/liberay_hip.so).

This is the Python host's view of the drop-in boundary: thin wrappers with the C names,
status codes turned into exceptions.  There is no CPU fallback anywhere: if the HIP library
is missing or no GPU is present, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_PKG = os.path.dirname(os.path.abspath(__file__))
# ERAY_LIB selects another build of the same ABI (diagnostics: lib/liberay_hip_trace.so)
LIB_PATH = os.environ.get("ERAY_LIB") or os.path.join(_PKG, "lib", "liberay_hip.so")

# eray_status (include/eray_hip.h)
OK = 0
E_INVALID_ARGUMENT = -1
E_HIP = -2
E_OUT_OF_MEMORY = -3
E_MISSING = -4
E_MISSING_MANY = -5
E_INVALID_TYPE = -6
E_OUT_OF_BOUNDS = -7
E_IO = -8
E_PARSE = -9
E_BUILD = -10
E_UNSUPPORTED = -11
E_CYCLE = -12

RENDER_DEFAULT = 0
RENDER_BRUTE_FORCE = 1
RENDER_DENSE_DETAIL = 2
RENDER_NO_DENSE_DETAIL = 4
RENDER_SEPARATE_FILL = 8
RENDER_NO_SEPARATE_FILL = 16
RENDER_SHARED_DETAIL = 32

GATHER_DEFAULT = 0
GATHER_SCENE_CAMERA = 1
GATHER_ROTATE_ROOT = 2

LIGHT_POINT = 0
LIGHT_AMBIENT = 1


class ErayError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"eray status {status}: {message}")
        self.status = status
        self.message = message


class Image(C.Structure):
    _fields_ = [("data", C.c_void_p), ("width", C.c_uint32), ("height", C.c_uint32)]


class Camera(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("fov", C.c_float * 2), ("width", C.c_uint32),
                ("z_dist", C.c_float)]


class Light(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("variant", C.c_int32), ("color", C.c_float * 3),
                ("brightness", C.c_float)]


class Material(C.Structure):
    _fields_ = [("color", Image), ("diffuse", Image), ("specular", Image),
                ("specular_power", Image), ("reflection", Image)]


class Object(C.Structure):
    _fields_ = [("positions", C.c_void_p), ("normals", C.c_void_p), ("uvs", C.c_void_p),
                ("triangle_count", C.c_uint32), ("bbox_min", C.c_float * 3),
                ("bbox_max", C.c_float * 3), ("material", Material)]


TEXEL_WAVE, TEXEL_RGB, TEXEL_FLAT_COLOR, TEXEL_MIX_COLOR = 0, 1, 2, 3


class TexelNode(C.Structure):  # eray_texel_node
    _fields_ = [("kind", C.c_uint32), ("width", C.c_uint32), ("height", C.c_uint32),
                ("param", C.c_float * 3), ("input", C.c_int32 * 3)]


class TexelGraph(C.Structure):  # eray_texel_graph
    _fields_ = [("nodes", C.POINTER(TexelNode)), ("count", C.c_uint32), ("color", C.c_int32),
                ("diffuse", C.c_int32), ("specular", C.c_int32), ("specular_power", C.c_int32),
                ("reflection", C.c_int32)]


def texel_node(kind, width, height, param=(0.0, 0.0, 0.0), inputs=(-1, -1, -1)) -> TexelNode:
    """One shaderlib node of a per-texel material graph (eray_texel_node)."""
    p = list(param) + [0.0] * (3 - len(param))
    q = list(inputs) + [-1] * (3 - len(inputs))
    return TexelNode(kind, width, height, (C.c_float * 3)(*p), (C.c_int32 * 3)(*q))


class ExampleMaterial(C.Structure):  # eray_material_example_params
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("x_fac", C.c_float), ("y_fac", C.c_float),
                ("r", C.c_float), ("g", C.c_float), ("b", C.c_float), ("factor", C.c_float)]


class RenderParams(C.Structure):
    _fields_ = [("image_width", C.c_uint32), ("image_height", C.c_uint32), ("row0", C.c_uint32),
                ("rows", C.c_uint32), ("bounces", C.c_uint32), ("anti_aliasing", C.c_uint32),
                ("out_rgb", C.c_void_p), ("out_ppm", C.c_void_p), ("out_face", C.c_void_p),
                ("flags", C.c_uint32), ("aa_seed", C.c_uint64), ("band_rows", C.c_uint32),
                ("band_stride", C.c_uint32)]


class FrameRing(C.Structure):  # eray_frame_ring
    _fields_ = [("slots", C.c_uint32), ("frames_per_launch", C.c_uint32), ("rgb_stride", C.c_uint64),
                ("ppm_stride", C.c_uint64), ("face_stride", C.c_uint64)]


def frame_ring(slots: int, rows: int, width: int, frames_per_launch: int = 0) -> FrameRing:
    """A ring of `slots` contiguous output slots of `rows` x `width` pixels (f32 RGB, PPM bytes,
    face indices: one slot's bytes as the stride; width a multiple of 16 keeps them 16-B aligned)."""
    px = rows * width
    return FrameRing(slots, frames_per_launch, 12 * px, 3 * px, 4 * px)


# Every exported symbol of include/eray_hip.h with its (restype, argtypes).
_P = C.c_void_p
_U = C.c_uint32
_F = C.c_float
class KernelTimes(C.Structure):  # eray_kernel_times
    _fields_ = [("launches", C.c_uint32), ("frames_per_launch", C.c_uint32), ("frame_kernel_ms", C.c_float),
                ("frame_kernel_min_ms", C.c_float), ("frame_kernel_max_ms", C.c_float), ("fill_kernel_ms", C.c_float),
                ("launch_span_ms", C.c_float)]


class ObjMesh(C.Structure):
    _fields_ = [("positions", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)),
                ("uvs", C.POINTER(C.c_float)), ("triangles", C.c_uint32)]


SIGNATURES = {
    "eray_abi_version": (C.c_int, []),
    "eray_obj_load": (C.c_int, [C.c_char_p, C.POINTER(ObjMesh)]),
    "eray_obj_free": (None, [C.POINTER(ObjMesh)]),
    "eray_ctx_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "eray_ctx_destroy": (C.c_int, [_P]),
    "eray_last_error": (C.c_char_p, [_P]),
    "eray_set_stream": (C.c_int, [_P, _P]),
    "eray_get_stream": (_P, [_P]),
    "eray_synchronize": (C.c_int, [_P]),
    "eray_device_alloc": (C.c_int, [_P, C.c_size_t, C.POINTER(_P)]),
    "eray_device_free": (C.c_int, [_P, _P]),
    "eray_memset": (C.c_int, [_P, _P, C.c_int, C.c_size_t]),
    "eray_copy_to_device": (C.c_int, [_P, _P, _P, C.c_size_t]),
    "eray_copy_to_host": (C.c_int, [_P, _P, _P, C.c_size_t]),
    "eray_node_wave": (C.c_int, [_P, _U, _U, _F, _F, _P]),
    "eray_node_rgb": (C.c_int, [_P, _U, _U, Image, Image, Image, _P]),
    "eray_node_flat_color": (C.c_int, [_P, _U, _U, _F, _F, _F, _P]),
    "eray_node_mix_color": (C.c_int, [_P, _U, _U, Image, Image, _F, _P]),
    "eray_material_example": (C.c_int, [_P, _U, _U, _F, _F, _F, _F, _F, _F, _P, _P]),
    "eray_scene_reset": (C.c_int, [_P]),
    "eray_scene_set_camera": (C.c_int, [_P, C.POINTER(Camera)]),
    "eray_scene_add_light": (C.c_int, [_P, C.POINTER(Light)]),
    "eray_scene_set_object_example_material": (C.c_int, [_P, _U, C.POINTER(ExampleMaterial)]),
    "eray_scene_set_object_texel_graph": (C.c_int, [_P, _U, C.POINTER(TexelGraph)]),
    "eray_scene_add_object": (C.c_int, [_P, C.POINTER(Object), C.POINTER(_U)]),
    "eray_camera_size": (C.c_int, [C.POINTER(Camera), C.POINTER(_U), C.POINTER(_U)]),
    "eray_render": (C.c_int, [_P, C.POINTER(RenderParams)]),
    "eray_render_frames": (C.c_int, [_P, C.POINTER(RenderParams), _U, C.POINTER(C.c_float)]),
    "eray_render_prepare": (C.c_int, [_P, C.POINTER(RenderParams), _U]),
    "eray_render_camera_path": (C.c_int, [_P, C.POINTER(RenderParams), C.POINTER(Camera), _U,
                                          C.POINTER(C.c_float)]),
    "eray_render_frames_ring": (C.c_int, [_P, C.POINTER(RenderParams), C.POINTER(FrameRing), _U,
                                          C.POINTER(C.c_float)]),
    "eray_render_prepare_ring": (C.c_int, [_P, C.POINTER(RenderParams), C.POINTER(FrameRing), _U]),
    "eray_frames_per_launch": (_U, [_P, C.POINTER(RenderParams), _U]),
    "eray_time_frames_ring": (C.c_int, [_P, C.POINTER(RenderParams), C.POINTER(FrameRing), _U,
                                        C.POINTER(KernelTimes)]),
    "eray_time_write_ceiling": (C.c_int, [_P, C.POINTER(RenderParams), C.POINTER(FrameRing), _U, _U,
                                          C.POINTER(KernelTimes)]),
    "eray_render_camera_path_ring": (C.c_int, [_P, C.POINTER(RenderParams), C.POINTER(FrameRing),
                                               C.POINTER(Camera), _U, C.POINTER(C.c_float)]),
    "eray_pack_ppm": (C.c_int, [_P, _P, _U, _U, _P]),
    "eray_comm_unique_id": (C.c_int, [_P]),
    "eray_comm_init": (C.c_int, [_P, C.c_int, C.c_int, _P, C.POINTER(_P)]),
    "eray_comm_destroy": (C.c_int, [_P]),
    "eray_gather_rows": (C.c_int, [_P, _P, _P, _P, _U, _U, _U]),
    "eray_gather_frames": (C.c_int, [_P, _P, _P, C.c_uint64, _P, C.c_uint64, _U, _U, _U, _U, _U]),
    "eray_band_rows": (_U, [_U, _U, _U, _U]),
    "eray_ppm_header": (C.c_int, [_U, _U, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
}

# Diagnostics exported beside the header's API (not part of include/eray_hip.h).
DEBUG_SIGNATURES = {
    "eray_debug_bin_stats": (C.c_int, [_P, _U, C.POINTER(C.c_uint64)]),
    "eray_debug_set_bin_form": (C.c_int, [_P, C.c_int]),
    "eray_debug_bin_dump": (C.c_int, [_P, _U, _U, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), _U,
                                      C.POINTER(C.c_uint32)]),
    "eray_debug_bin_entries": (C.c_int, [_P, _U, _U, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64),
                                         C.POINTER(C.c_uint32), _U, C.POINTER(C.c_uint32)]),
    "eray_debug_set_bin_capacity": (C.c_int, [_P, C.c_uint64]),
    "eray_debug_bin_counts": (C.c_int, [_P, _U, C.POINTER(C.c_uint32), _U, C.POINTER(C.c_uint32)]),
    "eray_debug_bin_capacity": (C.c_uint64, [_P]),
    "eray_debug_setup_state": (C.c_int, [_P, _U, _P, C.POINTER(C.c_int32)]),
    "eray_debug_unband": (C.c_int, [_P, _P, _P, _U, _U, _U, _U]),
    "eray_debug_coded_unband": (C.c_int, [_P, _P, _P, _U, _U, _U, _U]),
    "eray_debug_scene_gather": (C.c_int, [_P, _P, _P, _U, _U, _U, _U]),
    "eray_debug_gather_layout": (C.c_int, [C.POINTER(C.c_int32), _U, _U, _U, _U, _U, _U, C.POINTER(C.c_uint32)]),
    "eray_debug_scene_gather_batch": (C.c_int, [_P, _P, _P, _U, _U, _U, _U, _U, _U]),
    "eray_debug_gather_schedule": (C.c_int, [C.POINTER(C.c_uint32), _U, _U, _U, _U, C.POINTER(C.c_uint64), _U]),
    "eray_debug_gather_write_headers": (C.c_int, [C.POINTER(C.c_uint32), _U, _U, _U, _U, C.c_int32, _U, C.c_uint64,
                                                  _P]),
    "eray_debug_gather_check": (C.c_int, [C.POINTER(C.c_uint32), _U, _U, _U, _U, _U, C.c_uint64, _P]),
    "eray_debug_plan_verdict": (C.c_int, [C.POINTER(C.c_int32), _U, _U]),
    "eray_debug_gather_replan": (C.c_int, [_U, _U, C.c_uint64, _U, C.c_uint64]),
}

_lib = None


def _preload_hip_runtime() -> None:
    """Make sure exactly one HIP runtime serves this process.

    PyTorch ships its own libamdhip64.so.7; our library links the same SONAME.  Importing torch
    first makes the loader reuse torch's copy for us too, so device pointers and streams are
    shared.  ERAY_HIP_RUNTIME=rocm instead preloads /opt/rocm's runtime (then torch reuses it).
    """
    policy = os.environ.get("ERAY_HIP_RUNTIME", "torch")
    if policy == "rocm":
        for cand in ("/opt/rocm/lib/libamdhip64.so.7", "/opt/rocm/lib/libamdhip64.so"):
            if os.path.exists(cand):
                C.CDLL(cand, mode=C.RTLD_GLOBAL)
                break
    try:  # noqa: SIM105 - torch is optional for the C-ABI itself
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    """Load eray_amd/lib/liberay_hip.so (build it with `python -m eray_amd.build`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `python -m eray_amd.build` (no CPU fallback)")
        _preload_hip_runtime()
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        for name, (res, args) in DEBUG_SIGNATURES.items():
            if os.environ.get("ERAY_LIB") and not hasattr(L, name):
                continue  # (an older diagnostics build under A/B: debug entry points it predates)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error(ctx=None) -> str:
    msg = lib().eray_last_error(ctx)
    return msg.decode() if msg else ""


def check(status: int, ctx=None) -> None:
    if status != OK:
        raise ErayError(status, last_error(ctx))


def camera_size(cam: Camera) -> tuple[int, int]:
    w, h = _U(), _U()
    check(lib().eray_camera_size(C.byref(cam), C.byref(w), C.byref(h)))
    return w.value, h.value


def make_camera(center=(0.0, 0.0, 5.0), fov=(60.0, 60.0), width=1024, z_dist=1.0) -> Camera:
    return Camera((C.c_float * 3)(*center), (C.c_float * 2)(*fov), width, z_dist)


def make_light(position, variant, color=(1.0, 1.0, 1.0), brightness=1.0) -> Light:
    v = LIGHT_AMBIENT if variant in (LIGHT_AMBIENT, "ambient") else LIGHT_POINT
    return Light((C.c_float * 3)(*position), v, (C.c_float * 3)(*color), brightness)


COMM_ID_BYTES = 128


def comm_unique_id() -> bytes:
    """The id of a new RCCL communicator (eray_comm_unique_id), made on rank 0 and sent to the others."""
    buf = (C.c_uint8 * COMM_ID_BYTES)()
    check(lib().eray_comm_unique_id(buf))
    return bytes(buf)


def band_rows(height: int, band: int, nranks: int, rank: int) -> int:
    """Camera rows of `rank` in the interleaved band split (eray_band_rows)."""
    return lib().eray_band_rows(height, band, nranks, rank)


def gather_layout(rects, height: int, width: int, band_rows: int, nranks: int, rank: int) -> dict:
    """The library's layout of `rank`'s share in the scene-camera gather (eray_debug_gather_layout,
    host only): rows, bytes per frame and the rectangles (local rows l0..l1, 16-pixel column groups
    c0..c1, pack offset, row bytes) for the objects' pixel rectangles `rects` (x0, x1, y0, y1)."""
    flat = [int(v) for r in rects for v in r]
    arr = (C.c_int32 * max(1, len(flat)))(*flat)
    out = (C.c_uint32 * (4 + 8 * 8))()
    check(lib().eray_debug_gather_layout(arr, len(rects), height, width, band_rows, nranks, rank, out))
    rs = [dict(zip(("l0", "l1", "c0", "c1", "off", "row_bytes", "first"), out[4 + 8 * i: 4 + 8 * i + 7]))
          for i in range(out[1])]
    return {"rows": out[0], "bytes": out[2], "packed_rows": out[3], "rects": rs}


def gather_schedule(rank_bytes, rank: int, nframes: int, rotate: bool) -> dict:
    """The library's schedule of `rank` for a batch of `nframes` frames in the scene-camera gather
    (eray_debug_gather_schedule, host only) when rank q packs rank_bytes[q] bytes per frame: its
    buffer size, how many frames it assembles, each frame's pack offset, where each rank's packs
    start in its receive area, and its point-to-point transfers (peer, send, offset, bytes)."""
    n = len(rank_bytes)
    cap = 5 + nframes + 12 * n
    rb = (C.c_uint32 * n)(*[int(b) for b in rank_bytes])
    out = (C.c_uint64 * cap)()
    check(lib().eray_debug_gather_schedule(rb, n, rank, nframes, int(bool(rotate)), out, cap))
    v = list(out)
    k = 3 + nframes + n
    ops = [dict(zip(("peer", "send", "off", "bytes"), v[k + 4 * i: k + 4 * i + 4])) for i in range(v[2])]
    h = k + 4 * v[2]
    hdrs = v[h + 1:h + 1 + v[h]]
    peer_hdr = [None if x == 2 ** 64 - 1 else x for x in v[h + 1 + v[h]:h + 1 + v[h] + n]]
    return {"need": v[0], "mine": v[1], "pack": v[3:3 + nframes], "recv": v[3 + nframes:k], "ops": ops,
            "headers": hdrs, "peer_headers": peer_hdr}


def gather_write_headers(rank_bytes, rank: int, nframes: int, rotate: bool, buf: np.ndarray, status: int = 0,
                         kind: int = 1, key: int = 0) -> None:
    """Writes `rank`'s transfer headers (its verdict and its frames' source) into the host copy
    `buf` of its gather buffer (eray_debug_gather_write_headers, host only)."""
    n = len(rank_bytes)
    rb = (C.c_uint32 * n)(*[int(b) for b in rank_bytes])
    assert buf.dtype == np.uint8 and buf.flags.c_contiguous
    check(lib().eray_debug_gather_write_headers(rb, n, rank, nframes, int(bool(rotate)), status, kind, key,
                                                buf.ctypes.data))


def gather_check(rank_bytes, rank: int, nframes: int, rotate: bool, buf: np.ndarray, kind: int = 1,
                 key: int = 0) -> int:
    """A root's verdict on its received batch (the assembly's header check, eray_debug_gather_check,
    host only): E_OK or the error status; raises nothing."""
    n = len(rank_bytes)
    rb = (C.c_uint32 * n)(*[int(b) for b in rank_bytes])
    return lib().eray_debug_gather_check(rb, n, rank, nframes, int(bool(rotate)), kind, key, buf.ctypes.data)


def plan_verdict(records, rank: int) -> int:
    """A new gather plan's verdict on `rank` (exchange_plan's, eray_debug_plan_verdict, host only)
    from every rank's (status, kind, key low, key high): E_OK or the error status."""
    flat = [int(x) for r in records for x in r]
    arr = (C.c_int32 * len(flat))(*flat)
    return lib().eray_debug_plan_verdict(arr, len(records), rank)


def gather_replan(cached: bool, plan_kind: int, plan_key: int, cur_kind: int, cur_key: int) -> bool:
    """eray_gather_frames' re-plan decision (eray_debug_gather_replan, host only): from whether the
    cached plan fits the call's shared arguments, its source and the context's latest render."""
    return bool(lib().eray_debug_gather_replan(int(bool(cached)), plan_kind, plan_key, cur_kind, cur_key))


def comm_destroy(comm: int) -> None:
    check(lib().eray_comm_destroy(comm))


def ppm_header(width: int, height: int) -> bytes:
    buf = C.create_string_buffer(64)
    n = C.c_size_t()
    check(lib().eray_ppm_header(width, height, buf, 64, C.byref(n)))
    return buf.raw[: n.value]


def load_obj_native(path: str):
    """eray_obj_load (objload.cpp): Object::load_obj + build of the file at `path` as
    (positions (T, 9), normals (T, 9), uvs (T, 6)) float32.  Raises ErayError with the status
    (E_IO, E_PARSE, E_BUILD)."""
    m = ObjMesh()
    st = lib().eray_obj_load(os.fsencode(path), C.byref(m))
    if st:
        raise ErayError(st, last_error(None))
    try:
        T = m.triangles
        out = tuple(np.ctypeslib.as_array(ptr, (T, k)).copy() if T else np.zeros((0, k), np.float32)
                    for ptr, k in ((m.positions, 9), (m.normals, 9), (m.uvs, 6)))
    finally:
        lib().eray_obj_free(C.byref(m))
    return out


class DeviceArray:
    """A device allocation owned by a Context (numpy-like shape/dtype bookkeeping only)."""

    def __init__(self, ctx: "Context", shape, dtype):
        self.ctx = ctx
        self.shape = tuple(int(s) for s in shape)
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize
        self.ptr = ctx.alloc(self.nbytes)

    def numpy(self) -> np.ndarray:
        out = np.empty(self.shape, self.dtype)
        self.ctx.copy_to_host(out, self.ptr)
        return out

    def upload(self, a: np.ndarray) -> "DeviceArray":
        a = np.ascontiguousarray(a, self.dtype)
        assert a.nbytes == self.nbytes, (a.shape, self.shape)
        self.ctx.copy_to_device(self.ptr, a)
        return self

    def image(self) -> Image:
        h, w = self.shape[0], self.shape[1]
        return Image(self.ptr, w, h)

    def free(self) -> None:
        if self.ptr:
            self.ctx.free(self.ptr)
            self.ptr = None


class Context:
    """One eray_ctx (one GPU)."""

    def __init__(self, device: int = 0):
        self._h = _P()
        check(lib().eray_ctx_create(device, C.byref(self._h)))
        self.device = device

    @property
    def handle(self):
        return self._h

    def close(self) -> None:
        if self._h:
            lib().eray_ctx_destroy(self._h)
            self._h = _P()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, st: int) -> None:
        check(st, self._h)

    # memory ------------------------------------------------------------------------------
    def alloc(self, nbytes: int) -> int:
        p = _P()
        self._check(lib().eray_device_alloc(self._h, nbytes, C.byref(p)))
        return p.value

    def free(self, ptr: int) -> None:
        self._check(lib().eray_device_free(self._h, ptr))

    def empty(self, shape, dtype=np.float32) -> DeviceArray:
        return DeviceArray(self, shape, dtype)

    def to_device(self, a: np.ndarray) -> DeviceArray:
        a = np.ascontiguousarray(a)
        return DeviceArray(self, a.shape, a.dtype).upload(a)

    def memset(self, ptr: int, value: int, nbytes: int) -> None:
        self._check(lib().eray_memset(self._h, ptr, value, nbytes))

    def copy_to_device(self, dst: int, a: np.ndarray) -> None:
        self._check(lib().eray_copy_to_device(self._h, dst, a.ctypes.data, a.nbytes))

    def copy_to_host(self, a: np.ndarray, src: int) -> None:
        self._check(lib().eray_copy_to_host(self._h, a.ctypes.data, src, a.nbytes))

    def set_stream(self, stream_ptr) -> None:
        self._check(lib().eray_set_stream(self._h, stream_ptr))

    def synchronize(self) -> None:
        self._check(lib().eray_synchronize(self._h))

    # shaderlib ---------------------------------------------------------------------------
    def node_wave(self, w, h, x_fac, y_fac, out_ptr) -> None:
        self._check(lib().eray_node_wave(self._h, w, h, x_fac, y_fac, out_ptr))

    def node_rgb(self, w, h, r: Image, g: Image, b: Image, out_ptr) -> None:
        self._check(lib().eray_node_rgb(self._h, w, h, r, g, b, out_ptr))

    def node_flat_color(self, w, h, r, g, b, out_ptr) -> None:
        self._check(lib().eray_node_flat_color(self._h, w, h, r, g, b, out_ptr))

    def node_mix_color(self, w, h, left: Image, right: Image, factor, out_ptr) -> None:
        self._check(lib().eray_node_mix_color(self._h, w, h, left, right, factor, out_ptr))

    def material_example(self, w, h, x_fac, y_fac, r, g, b, factor, color_ptr, diffuse_ptr) -> None:
        self._check(lib().eray_material_example(self._h, w, h, x_fac, y_fac, r, g, b, factor,
                                                color_ptr, diffuse_ptr))

    # scene -------------------------------------------------------------------------------
    def scene_reset(self) -> None:
        self._check(lib().eray_scene_reset(self._h))

    def set_camera(self, cam: Camera) -> None:
        self._check(lib().eray_scene_set_camera(self._h, C.byref(cam)))

    def add_light(self, light: Light) -> None:
        self._check(lib().eray_scene_add_light(self._h, C.byref(light)))

    def set_object_example_material(self, index, width, height, x_fac, y_fac, r, g, b, factor) -> None:
        m = ExampleMaterial(width, height, x_fac, y_fac, r, g, b, factor)
        self._check(lib().eray_scene_set_object_example_material(self._h, index, C.byref(m)))

    def set_object_texel_graph(self, index, nodes, color=-1, diffuse=-1, specular=-1, specular_power=-1,
                               reflection=-1) -> None:
        """Material outputs of object `index` from a shaderlib graph evaluated per hit texel;
        nodes=None removes it."""
        if nodes is None:
            self._check(lib().eray_scene_set_object_texel_graph(self._h, index, None))
            return
        arr = (TexelNode * max(1, len(nodes)))(*nodes)
        g = TexelGraph(arr, len(nodes), color, diffuse, specular, specular_power, reflection)
        self._check(lib().eray_scene_set_object_texel_graph(self._h, index, C.byref(g)))

    def add_object(self, positions, normals, uvs, bbox_min=(0.0, 0.0, 0.0), bbox_max=(0.0, 0.0, 0.0),
                   color: Image | None = None, diffuse: Image | None = None,
                   specular: Image | None = None, specular_power: Image | None = None,
                   reflection: Image | None = None) -> int:
        P = np.ascontiguousarray(positions, np.float32).reshape(-1, 9)
        N = np.ascontiguousarray(normals, np.float32).reshape(-1, 9)
        U = np.ascontiguousarray(uvs, np.float32).reshape(-1, 6)
        if not (P.shape[0] == N.shape[0] == U.shape[0]):
            raise ValueError("positions/normals/uvs disagree on the triangle count")
        none = Image(None, 0, 0)
        mat = Material(color or none, diffuse or none, specular or none, specular_power or none,
                       reflection or none)
        obj = Object(P.ctypes.data, N.ctypes.data, U.ctypes.data, P.shape[0],
                     (C.c_float * 3)(*bbox_min), (C.c_float * 3)(*bbox_max), mat)
        idx = _U()
        self._check(lib().eray_scene_add_object(self._h, C.byref(obj), C.byref(idx)))
        return idx.value

    def render(self, image_width, image_height, row0=0, rows=None, out_rgb=None, out_ppm=None,
               out_face=None, bounces=0, anti_aliasing=0, flags=RENDER_DEFAULT, aa_seed=0, band_rows=0,
               band_stride=0) -> None:
        if rows is None:
            rows = image_height - row0
        p = RenderParams(image_width, image_height, row0, rows, bounces, anti_aliasing,
                         out_rgb or None, out_ppm or None, out_face or None, flags, aa_seed, band_rows, band_stride)
        self._check(lib().eray_render(self._h, C.byref(p)))

    def render_frames(self, frames, image_width, image_height, row0=0, rows=None, out_rgb=None,
                      out_ppm=None, out_face=None, flags=RENDER_DEFAULT, timed=False, prepare_only=False,
                      bounces=0, anti_aliasing=0, aa_seed=0, band_rows=0, band_stride=0, ring=None):
        """`frames` back-to-back renders (replayed from a cached HIP graph); returns the mean
        device ms per frame when `timed`.  `prepare_only` builds the launch plan and returns.
        ring (FrameRing): frame k into slot k % slots, several frames per launch."""
        if rows is None:
            rows = image_height - row0
        p = RenderParams(image_width, image_height, row0, rows, bounces, anti_aliasing, out_rgb or None,
                         out_ppm or None, out_face or None, flags, aa_seed, band_rows, band_stride)
        rg = C.byref(ring) if ring is not None else None
        if prepare_only:
            self._check(lib().eray_render_prepare_ring(self._h, C.byref(p), rg, frames))
            return None
        ms = C.c_float()
        self._check(lib().eray_render_frames_ring(self._h, C.byref(p), rg, frames, C.byref(ms) if timed else None))
        return ms.value if timed else None

    def time_frames(self, frames, image_width, image_height, row0=0, rows=None, out_rgb=None, out_ppm=None,
                    out_face=None, flags=RENDER_DEFAULT, band_rows=0, band_stride=0, ring=None) -> dict:
        """eray_time_frames_ring: the frames as plain launches, each frame kernel's dispatch timed by
        its own start / end timestamps.  Returns the eray_kernel_times fields (ms per launch)."""
        if rows is None:
            rows = image_height - row0
        p = RenderParams(image_width, image_height, row0, rows, 0, 0, out_rgb or None, out_ppm or None,
                         out_face or None, flags, 0, band_rows, band_stride)
        t = KernelTimes()
        self._check(lib().eray_time_frames_ring(self._h, C.byref(p), C.byref(ring) if ring is not None else None,
                                                frames, C.byref(t)))
        return {name: getattr(t, name) for name, _ in KernelTimes._fields_}

    def time_write_ceiling(self, frames, image_width, image_height, out_rgb=None, out_ppm=None, out_face=None,
                           ring=None, wgs_per_cu=1) -> dict:
        """eray_time_write_ceiling: the same launches' background bytes as a plain block-strided
        store stream (wgs_per_cu workgroups per CU), dispatch-timed; eray_kernel_times fields."""
        p = RenderParams(image_width, image_height, 0, image_height, 0, 0, out_rgb or None, out_ppm or None,
                         out_face or None, 0, 0, 0, 0)
        t = KernelTimes()
        self._check(lib().eray_time_write_ceiling(self._h, C.byref(p), C.byref(ring) if ring is not None else None,
                                                  frames, wgs_per_cu, C.byref(t)))
        return {name: getattr(t, name) for name, _ in KernelTimes._fields_}

    def frames_per_launch(self, image_width, image_height, rows=None, slots=64, anti_aliasing=0, bounces=0) -> int:
        """The frames per launch the library picks for a ring of `slots` (eray_frames_per_launch)."""
        p = RenderParams(image_width, image_height, 0, image_height if rows is None else rows, bounces,
                         anti_aliasing, None, None, None, 0, 0, 0, 0)
        return lib().eray_frames_per_launch(self._h, C.byref(p), slots)

    def render_camera_path(self, cameras, image_width, image_height, row0=0, rows=None, out_rgb=None,
                           out_ppm=None, out_face=None, flags=RENDER_DEFAULT, timed=False, bounces=0,
                           anti_aliasing=0, aa_seed=0, band_rows=0, band_stride=0, ring=None):
        """One frame per camera (Scene::set_camera + Engine::render each), the per-camera setup on
        the device; returns the mean device ms per frame (setup included) when `timed`."""
        if rows is None:
            rows = image_height - row0
        p = RenderParams(image_width, image_height, row0, rows, bounces, anti_aliasing, out_rgb or None,
                         out_ppm or None, out_face or None, flags, aa_seed, band_rows, band_stride)
        cams = (Camera * max(1, len(cameras)))(*cameras)
        ms = C.c_float()
        self._check(lib().eray_render_camera_path_ring(self._h, C.byref(p), C.byref(ring) if ring is not None else None,
                                                       cams, len(cameras), C.byref(ms) if timed else None))
        return ms.value if timed else None

    def comm_init(self, nranks: int, rank: int, uid: bytes) -> int:
        """An RCCL communicator for this context's GPU (eray_comm_init): every rank passes the id
        rank 0 got from comm_unique_id().  Returns the ncclComm_t handle."""
        if len(uid) != COMM_ID_BYTES:
            raise ValueError("unique id must be 128 bytes")
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        comm = _P()
        self._check(lib().eray_comm_init(self._h, nranks, rank, buf, C.byref(comm)))
        return comm.value

    def gather_rows(self, comm: int, local_ptr, frame_ptr, height: int, width: int, band_rows: int = 0) -> None:
        """eray_gather_rows: every rank's PPM rows into rank 0's height x width frame (file order):
        equal blocks in rank order (band_rows = 0) or interleaved bands of band_rows rows."""
        self._check(lib().eray_gather_rows(self._h, comm, local_ptr, frame_ptr or None, height, width, band_rows))

    def gather_frames(self, comm: int, local_ptr, local_stride: int, frames_ptr, frame_stride: int, nframes: int,
                      height: int, width: int, band_rows: int = 0, scene_camera: bool = False,
                      rotate_root: bool = False) -> None:
        """eray_gather_frames: `nframes` frames' rows (local + k * local_stride) into rank 0's frames
        (frames + k * frame_stride); scene_camera: only the objects' pixel rectangles travel;
        rotate_root (with scene_camera): frame k is assembled on rank k % N, at its frames + (k // N)
        * frame_stride."""
        flags = (GATHER_SCENE_CAMERA if scene_camera else GATHER_DEFAULT) | (GATHER_ROTATE_ROOT if rotate_root else 0)
        self._check(lib().eray_gather_frames(self._h, comm, local_ptr, local_stride, frames_ptr or None, frame_stride,
                                             nframes, height, width, band_rows, flags))

    def pack_ppm(self, rgb_ptr, w, h, out_ptr) -> None:
        self._check(lib().eray_pack_ppm(self._h, rgb_ptr, w, h, out_ptr))

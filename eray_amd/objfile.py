"""Wavefront .obj reading/writing in exactly the dialect eray's loader accepts.

`load_obj_file` reads files through the C-ABI loader (eray_obj_load); `load_obj` is the same
dialect stated in Python for in-memory text, and the check the native loader is tested against.

`load_obj` restates Object::load_obj + Object::build (src/lib/object.rs:101-230,
396-421) for the Python host; every input that panics in the reference raises ObjError
with the matching status (E_PARSE for panics, E_BUILD for build()'s Err).  The result is
three arrays per face, in file order (faces store vertex copies, object.rs:160-186):
positions (T, 9), normals (T, 9), uvs (T, 6), float32.

Floats are parsed like Rust's `str::parse::<f32>` (correctly rounded straight to f32):
Python parses to double first, and the rare double-rounding case (a double that lands
exactly on an f32 midpoint) is re-parsed with libc's strtof.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import re

import numpy as np

from .capi import E_BUILD, E_IO, E_PARSE

_FLOAT_RE = re.compile(r"^[+-]?(?:(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?|inf|infinity|nan)$",
                       re.IGNORECASE)
_USIZE_RE = re.compile(r"^\+?\d+$")
_libc = None


class ObjError(ValueError):
    def __init__(self, status: int, message: str):
        super().__init__(message)
        self.status = status


def _strtof(tok: str) -> np.float32:
    global _libc
    if _libc is None:
        _libc = ctypes.CDLL(ctypes.util.find_library("c"))
        _libc.strtof.restype = ctypes.c_float
        _libc.strtof.argtypes = [ctypes.c_char_p, ctypes.c_void_p]
    return np.float32(_libc.strtof(tok.encode(), None))


# char::is_whitespace (Unicode White_Space), the separators of str::split_whitespace — not
# Python's str.split(), which also splits on U+001C-U+001F
_RUST_WS = re.compile("[\t\n\x0b\x0c\r \x85\xa0\u1680\u2000-\u200a\u2028\u2029\u202f\u205f\u3000]+")


def _parse_f32(tokens: list[str], line: int) -> np.ndarray:
    for t in tokens:
        if not _FLOAT_RE.match(t):
            raise ObjError(E_PARSE, f"Failed to parse coords, should be an f32: {t} (line {line})")
    d = np.array([float(t) for t in tokens], dtype=np.float64)
    f = d.astype(np.float32)
    # double rounding: d exactly halfway between f and its neighbour toward d
    nb = np.nextafter(f, np.where(d > f.astype(np.float64), np.float32(np.inf), np.float32(-np.inf)))
    mid = (f.astype(np.float64) + nb.astype(np.float64)) / 2.0
    bad = np.isfinite(d) & (d != f.astype(np.float64)) & (d == mid)
    for i in np.nonzero(bad)[0]:
        f[i] = _strtof(tokens[i])
    return f


def load_obj(text: str | bytes):
    """Parse an .obj text; returns (positions (T,9), normals (T,9), uvs (T,6)) float32."""
    if isinstance(text, (bytes, bytearray)):
        try:  # std::fs::read_to_string: io::ErrorKind::InvalidData on invalid UTF-8
            text = bytes(text).decode("utf-8", errors="strict")
        except UnicodeDecodeError as e:
            raise ObjError(E_IO, f"stream did not contain valid UTF-8: {e}") from None
    verts: list[np.ndarray] = []
    norms: list[np.ndarray] = []
    uvs: list[np.ndarray] = []
    faces: list[tuple[int, int, int, int, int, int, int, int, int]] = []
    lines = text.split("\n")
    if lines and lines[-1] == "":
        lines.pop()
    for line_no, raw in enumerate(lines):
        line = raw[:-1] if raw.endswith("\r") else raw
        if not line or line[0] == "#":
            continue
        tok = [t for t in _RUST_WS.split(line) if t]  # str::split_whitespace
        if not tok:
            raise ObjError(E_PARSE, f"line {line_no}: whitespace-only line (tokens.next().unwrap())")
        m = tok[0]
        if m in ("o", "g"):
            if len(tok) < 2:
                raise ObjError(E_PARSE, f"line {line_no}: `{m}` without a name")
        elif m == "s":
            if len(tok) < 2 or tok[1] not in ("1", "on", "0", "off"):
                raise ObjError(E_PARSE, f"Unhandled smooth shading setting (line {line_no})")
        elif m in ("v", "vn", "vt"):
            c = _parse_f32(tok[1:], line_no)
            if not 2 <= len(c) < 4:
                raise ObjError(E_PARSE, f"Invalid coordinate count at line {line_no}: {len(c)}")
            if m == "vt":
                uvs.append(c[:2])
            else:
                if len(c) < 3:
                    raise ObjError(E_PARSE, f"line {line_no}: coords[0..=2] out of range")
                (verts if m == "v" else norms).append(c[:3])
        elif m == "f":
            idx = []
            for t in tok[1:]:
                parts = t.split("/")
                trip = []
                for k, (arr, what) in enumerate(((verts, "vertex"), (uvs, "uv"), (norms, "normal"))):
                    if k >= len(parts) or not _USIZE_RE.match(parts[k]):
                        raise ObjError(E_PARSE, f"line {line_no}: missing {what} index in `{t}`")
                    i = int(parts[k])
                    if i == 0 or i > len(arr):
                        raise ObjError(E_PARSE, f"line {line_no}: {what} index {i} out of range")
                    trip.append(i - 1)
                idx.append(trip)
            if len(idx) != 3:
                raise ObjError(E_PARSE, f"Invalid vertex count for face at line {line_no} "
                                        f"(should be 3, is {len(idx)})")
            faces.append(tuple(x for trip in idx for x in trip))
        else:
            raise ObjError(E_PARSE, f"Unhandled marker {m}")
    if not verts:
        raise ObjError(E_BUILD, "Missing vertices")
    if not norms:
        raise ObjError(E_BUILD, "Missing normals")
    V = np.array(verts, np.float32).reshape(-1, 3)
    N = np.array(norms, np.float32).reshape(-1, 3)
    U = np.array(uvs, np.float32).reshape(-1, 2)
    F = np.array(faces, np.int64).reshape(-1, 9)
    pos = V[F[:, [0, 3, 6]]].reshape(-1, 9)
    nrm = N[F[:, [2, 5, 8]]].reshape(-1, 9)
    uv = U[F[:, [1, 4, 7]]].reshape(-1, 6) if len(U) else np.zeros((len(F), 6), np.float32)
    return np.ascontiguousarray(pos), np.ascontiguousarray(nrm), np.ascontiguousarray(uv)


def load_obj_file(path: str):
    """The .obj file at `path` through the C-ABI loader (eray_obj_load, objload.cpp: the same
    dialect in one native pass); its statuses as ObjError (E_PARSE, E_BUILD) or OSError (E_IO)."""
    from . import capi

    try:
        return capi.load_obj_native(path)
    except capi.ErayError as e:
        if e.status in (E_PARSE, E_BUILD):
            raise ObjError(e.status, str(e)) from None
        if e.status == capi.E_IO:
            raise OSError(str(e)) from None
        raise


def _fmt(a: np.ndarray) -> list[str]:
    # repr of an f32 round-trips through a correctly rounded f32 parse
    return [np.format_float_positional(x, unique=True, trim="-") if np.isfinite(x) else str(x)
            for x in a.astype(np.float32)]


def write_obj(path: str, vertices: np.ndarray, normals: np.ndarray, uvs: np.ndarray,
              faces_v: np.ndarray, faces_vt: np.ndarray, faces_vn: np.ndarray, name="mesh") -> None:
    """Write an .obj in the strict dialect (o, v, vn, vt, s, f v/vt/vn; 1-based indices)."""
    out = [f"# eray_amd synthetic mesh", f"o {name}"]
    for tag, arr in (("v", vertices), ("vn", normals), ("vt", uvs)):
        arr = np.asarray(arr, np.float32)
        cols = [_fmt(arr[:, k]) for k in range(arr.shape[1])]
        out.extend(f"{tag} " + " ".join(c) for c in zip(*cols))
    out.append("s 0")
    fv, ft, fn = (np.asarray(x, np.int64) + 1 for x in (faces_v, faces_vt, faces_vn))
    for a, b, c in zip(fv, ft, fn):
        out.append("f " + " ".join(f"{a[k]}/{b[k]}/{c[k]}" for k in range(3)))
    with open(path, "w") as f:
        f.write("\n".join(out) + "\n")

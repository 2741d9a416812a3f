"""Checks derived by hand from the reference's source, independent of the oracle (oracle/ is a
restatement of the same code, so a mistake shared by it and the kernels would pass the parity
tests; these expected values come from reading engine.rs / object.rs / color.rs directly).

* BoundingBox::intersects (object.rs:327-379) with a loaded mesh's box, which is the degenerate
  (0,0,0)-(0,0,0) box (object.rs:101-186 never sets it).  For a camera at (0, 0, z) every slab
  entry/exit of x and y is (0 - 0) * invdir = 0 (or NaN where a direction component is +-0: 0 *
  inf), so neither early return fires and the final `t = txmin` is the z slab's positive entry:
  every camera ray passes, exactly as with the mesh's true box.  For a camera at (0.3, 0, z), a
  ray with dy != 0 has t_y = 0 and t_x = -0.3 / dx != 0 on one side of it, so `txmin > tymax` or
  `tymin > txmax` returns false; only a ray with dy == +0 (t_y = NaN, every comparison false)
  passes — the camera row y = H / 2 (y' = 0.5 makes the direction's y exactly 0, camera.rs:57-76).
* Engine::render's anti-aliasing (engine.rs:59-77): the pixel is (sum of the AA + 1 samples'
  colours) / AA, clamped; a ray that hits nothing contributes the single colour (0.1, 0.1, 0.2)
  (engine.rs:212), whose Color::sum is that colour (color.rs:82-87, reduce without a zero).
"""
import numpy as np
import pytest

from eray_amd import capi

pytestmark = pytest.mark.gpu

W, H = 160, 90


def _scene(gpu, cube, center, true_box):
    pos, nrm, uv = cube
    gpu.scene_reset()
    gpu.set_camera(capi.make_camera(center, (16.0, 9.0), W, 1.0))
    gpu.add_light(capi.make_light((0.0, 2.0, 0.0), "ambient", (1.0, 1.0, 1.0), 0.2))
    gpu.add_light(capi.make_light((1.0, 1.0, 2.0), "point", (1.0, 1.0, 1.0), 1.0))
    if true_box:
        p = pos.reshape(-1, 3)
        gpu.add_object(pos, nrm, uv, tuple(p.min(0)), tuple(p.max(0)))
    else:
        gpu.add_object(pos, nrm, uv)  # the loader's (0,0,0)-(0,0,0) box


def _render(gpu, flags=0, aa=0):
    rgb = gpu.empty((H, W, 3), np.float32)
    face = gpu.empty((H, W), np.int32)
    try:
        gpu.render(W, H, out_rgb=rgb.ptr, out_face=face.ptr, flags=flags, anti_aliasing=aa, aa_seed=7)
        gpu.synchronize()
        return rgb.numpy().copy(), face.numpy().copy()
    finally:
        rgb.free()
        face.free()


@pytest.mark.parametrize("flags", [capi.RENDER_DEFAULT, capi.RENDER_BRUTE_FORCE])
def test_degenerate_box_on_axis_camera_passes_every_ray(gpu, cube, flags):
    _scene(gpu, cube, (0.0, 0.0, 5.0), true_box=False)
    rgb_d, face_d = _render(gpu, flags)
    _scene(gpu, cube, (0.0, 0.0, 5.0), true_box=True)
    rgb_t, face_t = _render(gpu, flags)
    assert (face_d >= 0).sum() > 500
    assert np.array_equal(face_d, face_t)
    assert np.array_equal(rgb_d.view(np.uint32), rgb_t.view(np.uint32))


@pytest.mark.parametrize("flags", [capi.RENDER_DEFAULT, capi.RENDER_BRUTE_FORCE])
def test_degenerate_box_off_axis_camera_passes_only_the_centre_row(gpu, cube, flags):
    _scene(gpu, cube, (0.3, 0.0, 5.0), true_box=False)
    _, face_d = _render(gpu, flags)
    _scene(gpu, cube, (0.3, 0.0, 5.0), true_box=True)
    _, face_t = _render(gpu, flags)
    rows = np.flatnonzero((face_d >= 0).any(axis=1))
    assert rows.tolist() == [H // 2]
    # on that row the degenerate box lets every ray through: the hits are the true box's
    assert np.array_equal(face_d[H // 2], face_t[H // 2])
    assert (face_t >= 0).sum() > (face_d >= 0).sum() > 10


@pytest.mark.parametrize("aa", [1, 2, 3, 5])
def test_anti_aliasing_average_of_missed_rays(gpu, aa):
    gpu.scene_reset()
    gpu.set_camera(capi.make_camera((0.0, 0.0, 5.0), (16.0, 9.0), W, 1.0))
    rgb, face = _render(gpu, aa=aa)
    miss = np.array([0.1, 0.1, 0.2], np.float32)
    avg = miss.copy()  # the un-jittered ray's Color::sum
    for _ in range(aa):
        avg = (avg + miss).astype(np.float32)
    want = np.clip((avg / np.float32(aa)).astype(np.float32), 0.0, 1.0).astype(np.float32)
    assert (face == -1).all()
    assert np.array_equal(rgb.reshape(-1, 3).view(np.uint32), np.broadcast_to(want, (W * H, 3)).view(np.uint32))


# ---------------------------------------------------------------------------------------------
# Round 4: known answers worked out from the Rust source with a few lines of numpy f32 written
# here, not with oracle/ (every op below is one IEEE f32 operation in the reference's order).
F32 = np.float32


def _v(*a):
    return np.array(a, np.float32)


def _dot(a, b):  # vector.rs:188-193: fold from 0
    acc = F32(0.0)
    for i in range(3):
        acc = F32(acc + F32(a[i] * b[i]))
    return acc


def _cross(s, o):  # vector.rs:198-206
    return _v(F32(o[2] * s[1]) - F32(s[2] * o[1]), F32(o[0] * s[2]) - F32(s[0] * o[2]),
              F32(o[1] * s[0]) - F32(s[1] * o[0]))


def _normalize(v):  # vector.rs:150-158: v / sqrt(len_sq), a division per component
    n = F32(np.sqrt(_dot(v, v)))
    return _v(*(F32(x / n) for x in v))


def _clamp01(x):  # f32::clamp keeps NaN
    return x if np.isnan(x) else F32(min(max(x, F32(0.0)), F32(1.0)))


def _rmin(a, b):  # f32::min drops NaN
    return b if np.isnan(a) else a if np.isnan(b) else F32(min(a, b))


def _tri_hit(a, b, c, o, d):  # primitives.rs:41-72: (t, u, v) or None
    e1, e2 = b - a, c - a
    n = _cross(e1, e2)
    if _dot(n, d) > 0:
        return None
    det = F32(-_dot(d, n))
    inv = F32(F32(1.0) / det)
    ao = o - a
    dao = _cross(ao, d)
    u = F32(_dot(e2, dao) * inv)
    v = F32(F32(-_dot(e1, dao)) * inv)
    t = F32(_dot(ao, n) * inv)
    ok = det >= F32(1e-6) and t >= 0 and u >= 0 and v >= 0 and F32(u + v) <= 1.0
    return (t, u, v) if ok else None


TRI = (_v(-3.0, -3.0, 1.0), _v(3.0, -3.0, 1.0), _v(0.0, 3.0, 1.0))  # faces the camera (n.z > 0)
CAM = _v(0.0, 0.0, 5.0)
POINT = (_v(1.0, 1.0, 2.0), _v(1.0, 1.0, 1.0), F32(1.0))  # main.rs:53-65's point light
AMB = (_v(1.0, 1.0, 1.0), F32(0.2))


def _centre_dir():
    """Camera::pixel_to_ray of pixel (W/2, H/2) (camera.rs:57-76): x' = y' = 0.5."""
    ratio = F32(F32(16.0) / F32(9.0))
    vw = F32(ratio * F32(2.0))
    hor, ver = _v(vw, 0.0, 0.0), _v(0.0, 2.0, 0.0)
    bl = ((CAM - hor / F32(2.0)) - ver / F32(2.0)) - _v(0.0, 0.0, 1.0)
    return _normalize(((bl + hor * (F32(W // 2) / F32(W))) + ver * (F32(H // 2) / F32(H))) - CAM)


def _mesh(tris, normals):
    pos = np.concatenate([np.concatenate(t) for t in tris]).reshape(-1, 9).astype(np.float32)
    nrm = np.concatenate([np.concatenate(n) for n in normals]).reshape(-1, 9).astype(np.float32)
    uv = np.tile(np.array([0.0, 0.0, 1.0, 0.0, 0.5, 1.0], np.float32), (len(tris), 1))
    return pos, nrm, uv


def _textures(gpu, color, diffuse):
    c = gpu.to_device(np.array(color, np.float32).reshape(1, 1, 3))
    k = gpu.to_device(np.array([diffuse], np.float32).reshape(1, 1))
    return c, k


def _render_centre(gpu, objects, point=True, ambient=AMB):
    """Renders the scene (objects: (pos, nrm, uv, color texel, diffuse texel)); returns the centre
    pixel's RGB, its PPM bytes and face index, and the face map."""
    gpu.scene_reset()
    gpu.set_camera(capi.make_camera(tuple(CAM), (16.0, 9.0), W, 1.0))
    if ambient is not None:
        gpu.add_light(capi.make_light((0.0, 2.0, 0.0), "ambient", tuple(ambient[0]), float(ambient[1])))
    if point:
        gpu.add_light(capi.make_light(tuple(POINT[0]), "point", tuple(POINT[1]), float(POINT[2])))
    texs = []
    for pos, nrm, uv, col, kd in objects:
        c, k = _textures(gpu, col, kd)
        texs += [c, k]
        p = pos.reshape(-1, 3)
        gpu.add_object(pos, nrm, uv, tuple(p.min(0)), tuple(p.max(0)), color=c.image(), diffuse=k.image())
    rgb = gpu.empty((H, W, 3), np.float32)
    ppm = gpu.empty((H, W, 3), np.uint8)
    face = gpu.empty((H, W), np.int32)
    try:
        gpu.render(W, H, out_rgb=rgb.ptr, out_ppm=ppm.ptr, out_face=face.ptr)
        gpu.synchronize()
        y, x = H // 2, W // 2
        return rgb.numpy()[y, x], ppm.numpy()[H - 1 - y, x], int(face.numpy()[y, x]), face.numpy()
    finally:
        for a in [rgb, ppm, face] + texs:
            a.free()


def _shade(P, N, d, color, kd, point=True, ambient=AMB):
    """engine.rs:127-208 for one hit whose shadow ray reaches the light (a lone front face)."""
    out = []
    if point:
        Lp, lc, lb = POINT
        LmP = Lp - P
        prod = _clamp01(_dot(N, LmP))
        if np.isnan(prod):
            prod = F32(0.0)
        falloff = F32(F32(1.0) / F32(np.sqrt(_dot(LmP, LmP))))
        diff = [F32(F32(F32(F32(F32(color[i] * lc[i]) * kd) * prod) * lb) * falloff) for i in range(3)]
        refl = d - (N * F32(2.0)) * _dot(d, N)
        res = _clamp01(F32(F32(F32(0.5) * lb) * _dot(_normalize(refl), _normalize(LmP))))
        spec = F32(res * _clamp01(falloff))
        out.append([F32(diff[i] + spec) for i in range(3)])
    if ambient is not None:
        out.append([F32(F32(_rmin(ambient[0][i], F32(color[i])) * F32(kd)) * ambient[1]) for i in range(3)])
    acc = out[0]
    for c in out[1:]:
        acc = [F32(acc[i] + c[i]) for i in range(3)]
    return np.array(acc, np.float32)


def _ppm(c):  # color.rs:31-37: (c * 255.) as u8, saturating, NaN -> 0
    out = []
    for x in c:
        y = F32(x * F32(255.0))
        out.append(0 if np.isnan(y) or y <= 0 else 255 if y >= 255 else int(y))
    return np.array(out, np.uint8)


def test_first_hit_by_index_not_distance(gpu):
    """object.rs:63-78 returns the FIRST face in index order whose test passes: face 0 far (z = -1)
    and face 1 near (z = 0.5) both cover the centre, so face 0 wins inside one object; as two
    objects, cast_ray keeps the closer object (engine.rs:119-126) — the near face's — told apart by
    their diffuse texels (ambient light only: pixel = min(1, colour) kd 0.2)."""
    far = tuple(p * _v(1.0, 1.0, 0.0) + _v(0.0, 0.0, -1.0) for p in TRI)
    near = tuple(p * _v(0.5, 0.5, 0.0) + _v(0.0, 0.0, 0.5) for p in TRI)
    up = (_v(0.0, 0.0, 1.0),) * 3
    pos, nrm, uv = _mesh([far, near], [up, up])
    rgb, _, f, faces = _render_centre(gpu, [(pos, nrm, uv, (0.5, 0.5, 0.5), 0.25)], point=False)
    assert f == 0
    d = _centre_dir()
    assert _tri_hit(*far, CAM, d) is not None and _tri_hit(*near, CAM, d) is not None
    # where only the near (smaller) face is missed the far one still wins; nowhere does face 1
    assert (faces == 0).sum() > 1000 and not (faces == 1).any()
    # two objects, far first: the closer object (near) wins
    pf, nf, uf = _mesh([far], [up])
    pn, nn, un = _mesh([near], [up])
    rgb2, _, f2, _ = _render_centre(gpu, [(pf, nf, uf, (0.5, 0.5, 0.5), 0.25), (pn, nn, un, (0.5, 0.5, 0.5), 0.75)],
                                    point=False)
    want_near = _shade(None, None, d, (0.5, 0.5, 0.5), F32(0.75), point=False)
    assert f2 == 0 and np.array_equal(rgb2.view(np.uint32), want_near.view(np.uint32))
    assert np.array_equal(rgb.view(np.uint32), _shade(None, None, d, (0.5, 0.5, 0.5), F32(0.25), point=False).view(np.uint32))


def test_normal_interpolates_with_t(gpu):
    """primitives.rs:67: N = normalize(na u + nb v + nc t) — the third weight is the ray distance t,
    not 1 - u - v.  With distinct vertex normals the centre pixel's shading (one point light, its
    shadow ray unblocked, and the ambient light) is predicted from the Rust source bit for bit."""
    na, nb, nc = _v(0.0, 0.0, 1.0), _v(0.0, 1.0, 0.0), _v(0.6, 0.0, 0.8)
    pos, nrm, uv = _mesh([TRI], [(na, nb, nc)])
    color, kd = (0.8, 0.3, 0.3), F32(0.6)
    rgb, ppm, f, _ = _render_centre(gpu, [(pos, nrm, uv, color, kd)])
    d = _centre_dir()
    t, u, v = _tri_hit(*TRI, CAM, d)
    P = CAM + d * t
    N = _normalize((na * u + nb * v) + nc * t)
    want = _shade(P, N, d, color, kd)
    w = F32(F32(F32(1.0) - u) - v)
    wrong = _shade(P, _normalize((na * u + nb * v) + nc * w), d, color, kd)  # the barycentric reading
    assert f == 0
    assert not np.array_equal(want, wrong)
    assert np.array_equal(rgb.view(np.uint32), want.view(np.uint32)), (rgb, want)
    assert np.array_equal(ppm, _ppm(want))


def test_zero_normals_give_a_nan_pixel(gpu):
    """All-zero vertex normals: N = normalize(0) = NaN (0 / 0).  prod is NaN and is set to 0
    (engine.rs:147-149), but the specular term keeps NaN (f32::clamp keeps NaN, engine.rs:165-174),
    so the pixel's colour is NaN — and its PPM bytes 0 (a saturating `as u8`, color.rs:31-37)."""
    z = _v(0.0, 0.0, 0.0)
    pos, nrm, uv = _mesh([TRI], [(z, z, z)])
    rgb, ppm, f, _ = _render_centre(gpu, [(pos, nrm, uv, (0.8, 0.3, 0.3), 0.6)])
    assert f == 0
    assert np.isnan(rgb).all(), rgb
    assert ppm.tolist() == [0, 0, 0]
    rgb_a, ppm_a, _, _ = _render_centre(gpu, [(pos, nrm, uv, (0.8, 0.3, 0.3), 0.6)], point=False)
    want = _shade(None, None, None, (0.8, 0.3, 0.3), F32(0.6), point=False)  # no point light: finite
    assert np.array_equal(rgb_a.view(np.uint32), want.view(np.uint32)) and np.array_equal(ppm_a, _ppm(want))


def test_ambient_min_drops_nan_and_bytes_saturate(gpu):
    """engine.rs:197-208 with the ambient light alone: min(ambient colour, texel colour) drops a NaN
    texel channel (f32::min), so a NaN colour channel reads the light's; the raw sum is stored
    unclamped (AA = 0) and its PPM bytes saturate: a negative channel -> 0, above 1 -> 255."""
    up = (_v(0.0, 0.0, 1.0),) * 3
    pos, nrm, uv = _mesh([TRI], [up])
    for color, amb in (((float("nan"), 0.3, -2.0), AMB),
                       ((10.0, 0.5, float("nan")), (_v(20.0, 20.0, 20.0), F32(0.2)))):
        rgb, ppm, f, _ = _render_centre(gpu, [(pos, nrm, uv, color, 0.6)], point=False, ambient=amb)
        want = _shade(None, None, None, color, F32(0.6), point=False, ambient=amb)
        assert f == 0 and not np.isnan(want).any()
        assert np.array_equal(rgb.view(np.uint32), want.view(np.uint32)), (rgb, want)
        assert np.array_equal(ppm, _ppm(want)), (ppm, want)
    assert _ppm(np.array([-0.24, 1.2, 2.4], np.float32)).tolist() == [0, 255, 255]

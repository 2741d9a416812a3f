// hit.hpp — per-ray pieces of the reference's intersection and material lookup shared by the
// frame kernel (render.hip) and the general tracer (trace.hip).  Same f32 operations, in the
// same order, as the Rust source each function cites (compile with -ffp-contract=off).
#pragma once

#include "device_math.hpp"
#include "internal.hpp"

namespace eray {
namespace gpu {
namespace {

using namespace eray::dev;

// Triangle::intersects (primitives.rs:41-72) with e1/e2/n precomputed.  The conjunction is
// evaluated det-first so culled lanes skip the division; the outcome is the same conjunction.
__device__ __forceinline__ bool exact_test(const TriHot& r, f3 o, f3 d, float& u, float& v,
                                           float& t) {
    const f3 e1 = mk3(r.q0.x, r.q0.y, r.q0.z), e2 = mk3(r.q0.w, r.q1.x, r.q1.y);
    const f3 n = mk3(r.q1.z, r.q1.w, r.q2.x), a = mk3(r.q2.y, r.q2.z, r.q2.w);
    if (dot0(n, d) > 0.0f) return false;  // backface culling
    const float det = -dot0(d, n);
    if (!(det >= 1e-6f)) return false;
    const float invdet = 1.0f / det;
    const f3 ao = sub(o, a);
    const f3 dao = cross(ao, d);
    u = dot0(e2, dao) * invdet;
    v = -dot0(e1, dao) * invdet;
    t = dot0(ao, n) * invdet;
    return t >= 0.0f && u >= 0.0f && v >= 0.0f && (u + v) <= 1.0f;
}

// BoundingBox::intersects (object.rs:327-379), general box.
__device__ __forceinline__ bool bbox_hit(const ObjGeom& ob, f3 s, f3 d) {
    const float ix = 1.0f / d.x, iy = 1.0f / d.y, iz = 1.0f / d.z;
    const bool sx = ix < 0.0f, sy = iy < 0.0f, sz = iz < 0.0f;
    float txmin = ((sx ? ob.bb_hi[0] : ob.bb_lo[0]) - s.x) * ix;
    float txmax = ((sx ? ob.bb_lo[0] : ob.bb_hi[0]) - s.x) * ix;
    const float tymin = ((sy ? ob.bb_hi[1] : ob.bb_lo[1]) - s.y) * iy;
    const float tymax = ((sy ? ob.bb_lo[1] : ob.bb_hi[1]) - s.y) * iy;
    if ((txmin > tymax) || (tymin > txmax)) return false;
    if (tymin > txmin) txmin = tymin;
    if (tymax < txmax) txmax = tymax;
    const float tzmin = ((sz ? ob.bb_hi[2] : ob.bb_lo[2]) - s.z) * iz;
    const float tzmax = ((sz ? ob.bb_lo[2] : ob.bb_hi[2]) - s.z) * iz;
    if (tzmin > txmin) txmin = tzmin;
    if (tzmax < txmax) txmax = tzmax;
    if (txmin < 0.0f) {
        if (txmax < 0.0f) return false;
    }
    return true;
}

// i % n for the texture sizes of Image::mod_get (image.rs:36-38); n is wave-uniform and a power
// of two in practice, where the modulo is a mask
__device__ __forceinline__ uint32_t mod_size(uint32_t i, uint32_t n) {
    return (n & (n - 1)) == 0 ? (i & (n - 1)) : i % n;
}

// Image::mod_get's texel (image.rs:36-38) for uv (x, y) of a `comps`-float texture, or nullptr
// when the material has no such output (Material::get's default then stands).
__device__ __forceinline__ const float* texel(const TexView& tv, float x, float y, uint32_t comps) {
    if (!tv.data) return nullptr;
    const uint32_t ix = mod_size(sat_u32(x * (float)tv.w), tv.w);
    const uint32_t iy = mod_size(sat_u32(y * (float)tv.h), tv.h);
    return tv.data + comps * ((size_t)iy * tv.w + ix);
}
}  // namespace
}  // namespace gpu
}  // namespace eray

// hit.hpp — per-ray pieces of the reference's intersection and material lookup shared by the
// frame kernel (render.hip) and the general tracer (trace.hip).  Same f32 operations, in the
// same order, as the Rust source each function cites (compile with -ffp-contract=off).
#pragma once

#include "device_math.hpp"
#include "glibc_cosf.hpp"
#include "internal.hpp"

namespace eray {
namespace gpu {
namespace {

using namespace eray::dev;

// Frame outputs are written once and never read back by the kernel: 16-byte buffer stores with
// the sc1 (write-through) policy.  An sc1 store leaves no dirty line in the XCD's L2 (the line is
// dropped once written), so (a) the next dependent kernel boundary does not write back ~31 MB of
// dirty frame lines (MI355X_MICROARCH.md 'boundary': + B / 6 TB/s), and (b) the frame does not
// evict the scene and the textures the next frame reads.  Measured at C2: 10.5 -> 8.6 us per
// frame vs non-temporal stores (which keep the line).  `base` is the wave-uniform output array
// (the buffer resource); byte offsets fit 32 bits (FrameParams::aligned requires it).
//
// Round 5: a launch whose outputs exceed the 256 MiB Infinity Cache (C5's 7680x4320 frame, 498 MB)
// adds the NT (streaming) policy — measured, C5's launch span 156 -> 123 us: its frame lines no
// longer push the bins and records the detail waves read out of the Infinity Cache — while frames
// that fit it keep plain sc1 (with NT the 3840x2160 / 70k frame in one ring slot 19.9 -> 26.3 us:
// a frame rewritten in place is absorbed by the cache).  FrameParams::store_nt, chosen per launch.
using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
constexpr int kStoreSc1 = 16;  // CPol::SC1 (buffer instruction aux bits on gfx940+)
constexpr int kStoreNt = 2;    // CPol::NT
template <bool kNt, typename B>
__device__ __forceinline__ void stream16_pol(B* base, uint32_t voff, uint32_t soff, uint4 v) {
    const u32x4 w{v.x, v.y, v.z, v.w};
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, -1, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(w, r, voff, soff, kNt ? (kStoreSc1 | kStoreNt) : kStoreSc1);
}
template <typename B>
__device__ __forceinline__ void stream16(B* base, const void* dst, uint4 v, bool nt = false) {
    const uint32_t off = (uint32_t)(reinterpret_cast<const char*>(dst) - reinterpret_cast<const char*>(base));
    if (nt)
        stream16_pol<true>(base, off, 0u, v);
    else
        stream16_pol<false>(base, off, 0u, v);
}
template <typename B>
__device__ __forceinline__ void stream16(B* base, const void* dst, float4 v, bool nt = false) {
    stream16(base, dst, make_uint4(__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)),
             nt);
}

// A wave-uniform record read through the constant address space: scalar loads (the data was
// written by an earlier kernel; the scalar cache is invalidated at each kernel's start).
template <typename T>
__device__ __forceinline__ T load_const(const T* base, size_t i) {
    static_assert(sizeof(T) % 4 == 0, "dword-sized records only");
    using cu32 = const __attribute__((address_space(4))) uint32_t;
    cu32* src = (cu32*)(base + i);
    T out;
    uint32_t* dst = reinterpret_cast<uint32_t*>(&out);
#pragma unroll
    for (size_t k = 0; k < sizeof(T) / 4; ++k) dst[k] = src[k];
    return out;
}

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

// --------------------------------------------------------------------- exact test ----------
// The same test without branches: every quantity is computed (a failed det check may divide
// by zero; its u, v, t are then discarded) and the outcome is the same conjunction, so several
// tests can be interleaved by the compiler.
__device__ __forceinline__ bool exact_test_flat(const TriHot& r, f3 o, f3 d, float& u, float& v,
                                                float& t) {
    const f3 e1 = mk3(r.q0.x, r.q0.y, r.q0.z), e2 = mk3(r.q0.w, r.q1.x, r.q1.y);
    const f3 n = mk3(r.q1.z, r.q1.w, r.q2.x), a = mk3(r.q2.y, r.q2.z, r.q2.w);
    const float nd = dot0(n, d);
    const float det = -dot0(d, n);
    const float invdet = 1.0f / det;
    const f3 ao = sub(o, a);
    const f3 dao = cross(ao, d);
    u = dot0(e2, dao) * invdet;
    v = -dot0(e1, dao) * invdet;
    t = dot0(ao, n) * invdet;
    return !(nd > 0.0f) & (det >= 1e-6f) & (t >= 0.0f) & (u >= 0.0f) & (v >= 0.0f) & ((u + v) <= 1.0f);
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

// BoundingBox::intersects' first early return (object.rs:345-347) for a box that is a point in
// x and y (the loaded meshes' (0,0,0) box), decided without the shadow ray's direction.  With
// S = P + N * 0.1, w = Lp - P, d = normalize(w) and a = box - S, the test computes
// tx = a.x * (1 / d.x) and ty = a.y * (1 / d.y) and rejects when tx != ty (neither NaN).  Both
// carry the same positive factor |w| and at most ~3 roundings each: tx = (a.x / w.x) |w| (1 + dx)
// with |dx| <= 3.01 * 2^-24 while no value is subnormal or infinite.  q = a / w by the hardware
// reciprocal (1 ulp) and a product is within 3 * 2^-24 of a.x / w.x, so |qx - qy| above
// (|qx| + |qy|) * 2^-20 proves tx != ty.  Returns true only when bbox_hit(ob, S, d) is certainly
// false; false means undecided (the caller runs the exact test).
__device__ __forceinline__ bool point_box_rejects(const ObjGeom& ob, f3 S, f3 w) {
    const float ax = ob.bb_lo[0] - S.x, ay = ob.bb_lo[1] - S.y;
    const float wx = __builtin_fabsf(w.x), wy = __builtin_fabsf(w.y), ws = wx + wy + __builtin_fabsf(w.z);
    auto sane = [](float a) { return a == 0.0f || (__builtin_fabsf(a) >= 0x1p-60f && __builtin_fabsf(a) <= 0x1p20f); };
    const bool ok = ws >= 0x1p-60f && ws <= 0x1p60f && wx >= ws * 0x1p-100f && wy >= ws * 0x1p-100f && sane(ax) && sane(ay);
    const float qx = ax * __builtin_amdgcn_rcpf(w.x), qy = ay * __builtin_amdgcn_rcpf(w.y);
    return ok && __builtin_fabsf(qx - qy) > (__builtin_fabsf(qx) + __builtin_fabsf(qy)) * 0x1p-20f;
}
__device__ __forceinline__ bool point_box_xy(const ObjGeom& ob) {
    return ob.bb_lo[0] == ob.bb_hi[0] && ob.bb_lo[1] == ob.bb_hi[1];
}

// Wave-wide min and max of six floats at once (lanes that must not count pass +inf / -inf):
// the floats as order-preserving integer keys, DPP row shifts and row broadcasts (an invalid
// source lane reads the identity), the six reductions interleaved; results in SGPRs.
__device__ __forceinline__ int32_t float_key(float x) {
    const int32_t b = __float_as_int(x);
    return b ^ ((b >> 31) & 0x7fffffff);  // signed order of keys = numeric order of floats
}
__device__ __forceinline__ float key_float(int32_t k) { return __int_as_float(k ^ ((k >> 31) & 0x7fffffff)); }
template <int kCtrl, int kRowMask>
__device__ __forceinline__ void dpp_minmax_step(int32_t (&v)[6]) {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int32_t id = i < 3 ? 0x7fffffff : (int32_t)0x80000000;  // identity: fuses into v_min/max_dpp
        const int32_t o = __builtin_amdgcn_update_dpp(id, v[i], kCtrl, kRowMask, 0xf, false);
        v[i] = i < 3 ? min(v[i], o) : max(v[i], o);
    }
}
// v[0..2]: values to minimise, v[3..5]: values to maximise
__device__ __forceinline__ void wave_minmax6(const float (&in)[6], float (&out)[6]) {
    int32_t v[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) v[i] = float_key(in[i]);
    dpp_minmax_step<0x111, 0xf>(v);  // row_shr:1
    dpp_minmax_step<0x112, 0xf>(v);  // row_shr:2
    dpp_minmax_step<0x114, 0xf>(v);  // row_shr:4
    dpp_minmax_step<0x118, 0xf>(v);  // row_shr:8: lane 15 of each row holds the row's
    dpp_minmax_step<0x142, 0xa>(v);  // row_bcast:15
    dpp_minmax_step<0x143, 0xc>(v);  // row_bcast:31: lane 63 holds the wave's
#pragma unroll
    for (int i = 0; i < 6; ++i) out[i] = key_float(__builtin_amdgcn_readlane(v[i], 63));
}

// The box of the wave's hit points P (lanes with a hit), for the shadow rays' face bounds.
struct HitBox {
    float lo[3], hi[3];
    bool ok;  // some lane has a hit and every hit lane's P and N are finite
};
__device__ __forceinline__ HitBox hit_box(bool have, f3 P, f3 N) {
    const float inf = __builtin_inff();
    const bool finite = __builtin_isfinite(P.x) && __builtin_isfinite(P.y) && __builtin_isfinite(P.z) &&
                        __builtin_isfinite(N.x) && __builtin_isfinite(N.y) && __builtin_isfinite(N.z);
    const bool use = have && finite;
    const float in[6] = {use ? P.x : inf, use ? P.y : inf, use ? P.z : inf,
                         use ? P.x : -inf, use ? P.y : -inf, use ? P.z : -inf};
    float out[6];
    wave_minmax6(in, out);
    HitBox b;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        b.lo[k] = out[k];
        b.hi[k] = out[3 + k];
    }
    b.ok = __any(have) && !__any(have && !finite);
    return b;
}

// Can a shadow ray Ray::new(P + N * 0.1, Lp - P) of a hit point P in box `b` pass this face's
// det and t conditions (primitives.rs:47-66)?  det >= 1e-6 needs dot(P - Lp, n) > 0 and t >= 0
// needs dot(S - a, n) >= 0 for the origin S, which lies within 0.1 (|N| = 1) of the box; both
// are linear, so their maxima over the box decide.  The tolerance (1e-4 of the terms'
// magnitudes) dwarfs the f32 rounding of every quantity involved, so a face some lane's exact
// test accepts is never dropped; non-finite bounds keep the face.
__device__ __forceinline__ bool shadow_box_may_hit(const TriHot& r, f3 Lp, const HitBox& b) {
    const float n[3] = {r.q1.z, r.q1.w, r.q2.x}, a[3] = {r.q2.y, r.q2.z, r.q2.w};
    const float lp[3] = {Lp.x, Lp.y, Lp.z};
    const float g = 0.1001f;
    float m1 = 0.0f, m2 = 0.0f, mag = 0.0f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const bool pos = n[k] >= 0.0f;
        m1 += n[k] * ((pos ? b.hi[k] : b.lo[k]) - lp[k]);
        m2 += n[k] * ((pos ? b.hi[k] + g : b.lo[k] - g) - a[k]);
        mag += __builtin_fabsf(n[k]) *
               (__builtin_fabsf(b.lo[k]) + __builtin_fabsf(b.hi[k]) + __builtin_fabsf(lp[k]) + __builtin_fabsf(a[k]) + 1.0f);
    }
    const float tol = 1e-4f * mag + 1e-30f;
    return ((m1 >= -tol) & (m2 >= -tol)) | !(mag < 1e30f);
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

// Material output `out` (0 color .. 4 reflection) of a texel program (MaterialDesc::prog) at uv:
// the value Material::get would read from the texture Graph::run makes (material.rs:56-94).
// Returns false when the output is not a program output.  First the texel of every tree node,
// top-down (the root's is Material::get's mod_get texel), then the values, bottom-up:
//   wave  |cos((x as f32 * x_fac + y as f32 * y_fac) / 10)|     (wave.rs:127)
//   rgb   (red[i], green[i], blue[i]) at the node's own index  (rgb.rs:89-95)
//   flat  (r, g, b)                                            (flat_color.rs:88)
//   mix   l * (1 - factor) + r * factor per channel            (mix_color.rs:85-91)
__device__ __noinline__ bool texel_program(const uint32_t* prog, uint32_t out, float u, float v, float (&val)[3]) {
    const uint32_t first = prog[out], n = prog[5 + out];
    if (!n) return false;
    const TexelInstr* ins = reinterpret_cast<const TexelInstr*>(prog + kTexelHeaderWords) + first;
    uint32_t cx[kTexelMaxNodes], cy[kTexelMaxNodes];
    float vr[kTexelMaxNodes], vg[kTexelMaxNodes], vb[kTexelMaxNodes];
    cx[0] = mod_size(sat_u32(u * (float)ins[0].w), ins[0].w);
    cy[0] = mod_size(sat_u32(v * (float)ins[0].h), ins[0].h);
    for (uint32_t k = 1; k < n; ++k) {
        const TexelInstr& t = ins[k];
        const uint32_t q = t.parent;
        if (t.xform == kTexelMod) {
            cx[k] = cx[q] % t.w;
            cy[k] = cy[q] % t.h;
        } else {
            const uint64_t i = (uint64_t)cy[q] * ins[q].w + cx[q];
            cx[k] = (uint32_t)(i % t.w);
            cy[k] = (uint32_t)(i / t.w);
        }
    }
    for (uint32_t k = n; k-- > 0;) {
        const TexelInstr& t = ins[k];
        if (t.kind == 0) {  // wave
            vr[k] = __builtin_fabsf(libm::cosf_glibc(libm::div10_f32((float)cx[k] * t.p[0] + (float)cy[k] * t.p[1])));
        } else if (t.kind == 1) {  // rgb
            vr[k] = vr[t.c[0]];
            vg[k] = vr[t.c[1]];
            vb[k] = vr[t.c[2]];
        } else if (t.kind == 2) {  // flat_color
            vr[k] = t.p[0];
            vg[k] = t.p[1];
            vb[k] = t.p[2];
        } else {  // mix_color
            const float f = t.p[0];
            const uint32_t l = t.c[0], r = t.c[1];
            vr[k] = vr[l] * (1.0f - f) + vr[r] * f;
            vg[k] = vg[l] * (1.0f - f) + vg[r] * f;
            vb[k] = vb[l] * (1.0f - f) + vb[r] * f;
        }
    }
    val[0] = vr[0];
    val[1] = vg[0];
    val[2] = vb[0];
    return true;
}
}  // namespace
}  // namespace gpu
}  // namespace eray

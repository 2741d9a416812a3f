// device_math.hpp — f32 arithmetic with the reference's exact semantics, for gfx950 kernels.
//
// The whole library is compiled with -ffp-contract=off (no a*b+c -> v_fma fusion), with
// hipcc's default correctly rounded f32 division and sqrt and f32 denormals preserved, so
// each helper below performs the same IEEE operations, in the same order, as the Rust
// source it cites.  That is what makes GPU results bit-identical to the reference semantics.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "glibc_powf.hpp"

namespace eray {
namespace dev {

struct f3 {
    float x, y, z;
};

__device__ __forceinline__ f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
// Vector +/- Vector, Vector */÷ scalar: element-wise (vector.rs:73-125)
__device__ __forceinline__ f3 add(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 mul(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ f3 divs(f3 a, float s) { return f3{a.x / s, a.y / s, a.z / s}; }
// Vector::dot_product folds from TYPE::default() = 0 (vector.rs:188-193).  The leading
// `0.0f +` only matters for the sign of a zero result, but it is kept so results match bitwise.
__device__ __forceinline__ float dot0(f3 a, f3 b) {
    float acc = 0.0f;
    acc = acc + a.x * b.x;
    acc = acc + a.y * b.y;
    acc = acc + a.z * b.z;
    return acc;
}
// The same sum without the leading zero: equal to dot0 except possibly for the sign of a
// zero result.  Only used where the value feeds comparisons against non-zero thresholds
// or the sign of zero provably cannot matter.
__device__ __forceinline__ float dot_nz(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ float len_sq(f3 a) { return dot0(a, a); }
__device__ __forceinline__ float len(f3 a) { return __builtin_sqrtf(len_sq(a)); }
__device__ __forceinline__ f3 normalize(f3 a) { return divs(a, len(a)); }  // vector.rs:156-158
// cross_product(self, other) (vector.rs:198-206)
__device__ __forceinline__ f3 cross(f3 s, f3 o) {
    return f3{o.z * s.y - s.z * o.y, o.x * s.z - s.x * o.z, o.y * s.x - s.y * o.x};
}

struct rgb {
    float r, g, b;
};
__device__ __forceinline__ rgb cadd(rgb a, rgb b) { return rgb{a.r + b.r, a.g + b.g, a.b + b.b}; }
__device__ __forceinline__ rgb cmul(rgb a, float s) { return rgb{a.r * s, a.g * s, a.b * s}; }
__device__ __forceinline__ rgb cmulc(rgb a, rgb b) { return rgb{a.r * b.r, a.g * b.g, a.b * b.b}; }

// Rust f32::min on x86-64 (llvm.minnum lowering): isnan(a) ? b : (b < a ? b : a).
__device__ __forceinline__ float rust_min(float a, float b) {
    if (a != a) return b;
    return (b < a) ? b : a;
}
// Rust f32::clamp: NaN propagates.
__device__ __forceinline__ float rust_clamp(float x, float lo, float hi) {
    if (x < lo) x = lo;
    if (x > hi) x = hi;
    return x;
}
// `x as u32` / `x as u8`: saturating, NaN -> 0, truncation toward zero.
__device__ __forceinline__ uint32_t sat_u32(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xffffffffu;
    return (uint32_t)f;
}
__device__ __forceinline__ uint32_t sat_u8(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 255.0f) return 255u;
    return (uint32_t)f;
}

// powf as used by the specular term (engine.rs:171,174): the restated glibc powf
// (glibc_powf.hpp, bit-identical to the host's).  powf(x, 1) == x for every non-NaN x (checked
// exhaustively against glibc: tests/test_libm_restatement.py), which the kernels use when no
// material has a specular-power output (specular_power defaults to 1: engine.rs:164).
__device__ __forceinline__ float powf_ref(float x, float y) {
    if (y == 1.0f) return x;
    return libm::powf_glibc(x, y);
}

}  // namespace dev
}  // namespace eray

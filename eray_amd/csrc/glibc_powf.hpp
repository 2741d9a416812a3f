// glibc_powf.hpp — f32 power bit-identical to the reference's `f32::powf` on x86-64 Linux.
//
// The reference's specular term (src/lib/engine.rs:171,174) calls Rust's f32::powf, which lowers
// to the platform libm's `powf`.  On the reference's platform (x86-64 glibc, here 2.35) that is
// the ARM optimized-routines single-precision pow (glibc sysdeps/ieee754/flt-32/e_powf.c,
// e_powf_log2_data.c, e_exp2f_data.c; in glibc since 2.28), selected through its FMA ifunc
// variant on FMA-capable hosts.  Its published algorithm, all in double:
//   log2(x):  x = 2^k z with z in [0x3f330000, 2 * 0x3f330000) (exact), c the centre of z's
//             1/16 subinterval: log2(x) = k + log2(c) + P(z/c - 1), P a degree-5 polynomial of
//             log1p(r)/ln2 (tabulated 1/c and log2(c));
//   exp2(y log2 x): y log2 x = k/32 + r, 2^(k/32) from a 32-entry table (exponent added to the
//             bits), 2^r by a cubic;
//   special cases: zero / inf / NaN arguments, negative x with integer y (sign), subnormal x
//             (normalised), overflow / underflow thresholds on |y log2 x| >= 126.
// GCC contracts every a * b + c of the polynomials into an FMA in the ifunc variant the host
// runs (__powf_fma), so this restatement does too.  The tables were checked against the bytes of
// the host's libm.so.6 and the function bit-for-bit against the host glibc powf
// (tests/test_libm_restatement.py).
#pragma once

#include <stdint.h>
#include <string.h>

#include "glibc_cosf.hpp"  // ERAY_HD, fma_d, f32_bits

namespace eray {
namespace libm {

struct PowfLog2 {
    double invc, logc;
};

// e_powf_log2_data.c: 1/c and log2(c) for the 16 subintervals of [0x3f330000, 2 * 0x3f330000)
ERAY_HD inline const PowfLog2* powf_log2_tab() {
    static const PowfLog2 kTab[16] = {
        {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
        {0x1.49539f0f010bp+0, -0x1.7418b0a1fb77bp-2},  {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
        {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8eap+0, -0x1.97c1d1b3b7afp-3},
        {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
        {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1p+0, 0x0p+0},
        {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4},  {0x1.ca4b31f026aap-1, 0x1.476a9543891bap-3},
        {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
        {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2},  {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2},
    };
    return kTab;
}

// e_exp2f_data.c: tab[i] = bits of 2^(i/32) minus i << 47 (the exponent is added at use)
ERAY_HD inline const uint64_t* exp2f_tab() {
    static const uint64_t kTab[32] = {
        0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
        0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
        0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
        0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
        0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
        0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
        0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
        0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull,
    };
    return kTab;
}

ERAY_HD inline double f64_from_bits(uint64_t u) {
    double d;
    memcpy(&d, &u, 8);
    return d;
}
ERAY_HD inline uint64_t f64_bits(double d) {
    uint64_t u;
    memcpy(&u, &d, 8);
    return u;
}
ERAY_HD inline float f32_from_bits(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

// e_powf.c log2_inline: log2 of the (normalised, positive) bit pattern ix
ERAY_HD inline double powf_log2_inline(uint32_t ix) {
    const uint32_t kOff = 0x3f330000u;
    const uint32_t tmp = ix - kOff;
    const int i = (int)((tmp >> (23 - 4)) % 16u);
    const uint32_t top = tmp & 0xff800000u;
    const uint32_t iz = ix - top;
    const int k = (int32_t)top >> 23;  // arithmetic shift
    const PowfLog2 e = powf_log2_tab()[i];
    const double z = (double)f32_from_bits(iz);
    // log2(x) = log1p(z/c - 1)/ln2 + log2(c) + k
    const double r = fma_d(z, e.invc, -1.0);
    const double y0 = e.logc + (double)k;
    const double A0 = 0x1.27616c9496e0bp-2, A1 = -0x1.71969a075c67ap-2, A2 = 0x1.ec70a6ca7baddp-2,
                 A3 = -0x1.7154748bef6c8p-1, A4 = 0x1.71547652ab82bp0;
    const double r2 = r * r;
    double y = fma_d(A0, r, A1);
    const double p = fma_d(A2, r, A3);
    const double r4 = r2 * r2;
    double q = fma_d(A4, r, y0);
    q = fma_d(p, r2, q);
    y = fma_d(y, r4, q);
    return y;
}

// e_powf.c exp2_inline (no round-to-int intrinsics on x86-64: the shift trick)
ERAY_HD inline float powf_exp2_inline(double xd, uint32_t sign_bias) {
    const double kShift = 0x1.8p+47;  // 0x1.8p52 / 32
    double kd = xd + kShift;          // rounding to double precision is required
    const uint64_t ki = f64_bits(kd);
    kd -= kShift;  // k/32
    const double r = xd - kd;
    // exp2(x) = 2^(k/32) * 2^r ~= s * (C0 r^3 + C1 r^2 + C2 r + 1)
    uint64_t t = exp2f_tab()[ki % 32u];
    const uint64_t ski = ki + sign_bias;
    t += ski << (52 - 5);
    const double s = f64_from_bits(t);
    const double C0 = 0x1.c6af84b912394p-5, C1 = 0x1.ebfce50fac4f3p-3, C2 = 0x1.62e42ff0c52d6p-1;
    const double z = fma_d(C0, r, C1);
    const double r2 = r * r;
    double y = fma_d(C2, r, 1.0);
    y = fma_d(z, r2, y);
    y = y * s;
    return (float)y;
}

// 0: not an integer, 1: odd integer, 2: even integer (iy: a non-zero finite float's bits)
ERAY_HD inline int powf_checkint(uint32_t iy) {
    const int e = (int)(iy >> 23 & 0xff);
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1u)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}
ERAY_HD inline bool powf_zeroinfnan(uint32_t ix) { return 2u * ix - 1u >= 2u * 0x7f800000u - 1u; }
ERAY_HD inline bool issignaling_f32(uint32_t ix) { return 2u * (ix ^ 0x00400000u) > 2u * 0x7fc00000u; }

ERAY_HD inline float powf_glibc(float x, float y) {
    const uint32_t kSignBias = 1u << (5 + 11);
    uint32_t sign_bias = 0;
    uint32_t ix = f32_bits(x);
    const uint32_t iy = f32_bits(y);
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || powf_zeroinfnan(iy)) {
        // either (x < 0x1p-126 or inf or nan) or (y is 0 or inf or nan)
        if (powf_zeroinfnan(iy)) {
            if (2u * iy == 0) return issignaling_f32(ix) ? x + y : 1.0f;
            if (ix == 0x3f800000u) return issignaling_f32(iy) ? x + y : 1.0f;
            if (2u * ix > 2u * 0x7f800000u || 2u * iy > 2u * 0x7f800000u) return x + y;
            if (2u * ix == 2u * 0x3f800000u) return 1.0f;
            if ((2u * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;  // |x|<1 && y==inf or |x|>1 && y==-inf
            return y * y;
        }
        if (powf_zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000u) && powf_checkint(iy) == 1) x2 = -x2;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        // x and y are non-zero finite
        if (ix & 0x80000000u) {  // finite x < 0
            const int yint = powf_checkint(iy);
            if (yint == 0) return (x - x) / (x - x);  // __math_invalidf: NaN
            if (yint == 1) sign_bias = kSignBias;
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {  // normalise subnormal x so the exponent becomes negative
            ix = f32_bits(x * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    const double logx = powf_log2_inline(ix);
    const double ylogx = (double)y * logx;  // cannot overflow: y is single precision
    if ((f64_bits(ylogx) >> 47 & 0xffff) >= f64_bits(126.0) >> 47) {
        // |y * log(x)| >= 126
        if (ylogx > 0x1.fffffffd1d571p+6) {  // __math_oflowf
            const float h = sign_bias ? -0x1p97f : 0x1p97f;
            return h * 0x1p97f;
        }
        if (ylogx <= -150.0) {  // __math_uflowf
            const float h = sign_bias ? -0x1p-95f : 0x1p-95f;
            return h * 0x1p-95f;
        }
        if (ylogx < -149.0) {  // __math_may_uflowf (WANT_ERRNO_UFLOW)
            const float h = sign_bias ? -0x1.4p-75f : 0x1.4p-75f;
            return h * 0x1.4p-75f;
        }
    }
    return powf_exp2_inline(ylogx, sign_bias);
}

}  // namespace libm
}  // namespace eray

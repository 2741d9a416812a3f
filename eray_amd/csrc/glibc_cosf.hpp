// glibc_cosf.hpp — f32 cosine bit-identical to the reference's `f32::cos` on x86-64 Linux.
//
// The reference's wave node (src/shaderlib/wave.rs:127) calls Rust's f32::cos, which lowers
// to the platform libm's `cosf`.  On the reference's platform (x86-64 glibc, here 2.35) that is
// the ARM optimized-routines single-precision sin/cos (glibc sysdeps/ieee754/flt-32/s_cosf.c,
// sincosf.h, sincosf_data.c; in glibc since 2.28).  Its published algorithm:
//   |x| < pi/4         : cos polynomial in double (1 for |x| < 2^-12)
//   |x| < 120          : n = round(x * 2/pi) via a 2^24-scaled multiply, r = x - n*pi/2
//   |x| < inf          : Payne-Hanek style reduction with a 4/pi bit table (reduce_large)
//   then sin or cos polynomial of r (selected and signed by the quadrant), rounded to float.
// All intermediate arithmetic is double.  GCC contracts the polynomial steps and the reduction
// into FMAs on FMA-capable hosts (the __cosf_fma ifunc variant); the float result was checked
// to be identical with and without contraction, and this restatement was checked bit-for-bit
// against the host glibc over every finite float (tests/test_libm_restatement.py).
//
// The 4/pi table is the binary expansion of 4/pi in sliding 32-bit windows (8 new bits per
// entry), kept here as the packed bit string (inv_pio4_word); it is derived from first principles
// in tests/test_libm_restatement.py.
#pragma once

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define ERAY_HD __host__ __device__
#else
#include <math.h>
#define ERAY_HD
#endif

namespace eray {
namespace libm {

// The published coefficient tables (sincosf_data.c): the sin/cos polynomials' coefficients, 2/pi
// scaled by 2^24 and pi/2.  The library's second table (quadrants with bit 1 set) differs from the
// first only in the cos coefficients' signs; every cos-polynomial step is an FMA or a product, and
// fma(a, -b, -c) == -fma(a, b, c) and (float)-v == -(float)v exactly (round-to-nearest is
// symmetric; a cos value on [-pi/4, pi/4] is never 0), so the second table's result is the first's
// negated.  Immediates here, not a table in memory: on the GPU a per-lane table pointer made every
// coefficient a dependent vector load.
constexpr double kHpiInv = 0x1.45F306DC9C883p+23;  // 2/pi * 2^24
constexpr double kHpi = 0x1.921FB54442D18p0;       // pi/2
constexpr double kC0 = 0x1p0, kC1 = -0x1.ffffffd0c621cp-2, kC2 = 0x1.55553e1068f19p-5,
                 kC3 = -0x1.6c087e89a359dp-10, kC4 = 0x1.99343027bf8c3p-16;
constexpr double kS1 = -0x1.555545995a603p-3, kS2 = 0x1.1107605230bc4p-7, kS3 = -0x1.994eb3774cf24p-13;

// the table's sign[q & 3] = {1, -1, -1, 1}: negative when bits 0 and 1 of q differ
ERAY_HD inline double quadrant_sign(int q) { return ((q ^ (q >> 1)) & 1) ? -1.0 : 1.0; }

// The published 24-entry table (sincosf_data.c __inv_pio4): entry i holds the 32 bits at bit 8i
// of the string "24 zero bits, then 4/pi's bits".  That string as 32-bit words, selected by
// index (immediates: a per-lane table index made every large-argument reduction three dependent
// vector loads on the GPU); checked against 4/pi derived from first principles in
// tests/test_libm_restatement.py.
ERAY_HD inline uint32_t inv_pio4_word(int j) {  // j in 0..6
    return j == 0 ? 0x000000a2u
         : j == 1 ? 0xf9836e4eu
         : j == 2 ? 0x441529fcu
         : j == 3 ? 0x2757d1f5u
         : j == 4 ? 0x34ddc0dbu
         : j == 5 ? 0x6295993cu
                  : 0x439041feu;
}
// the 32 bits at bit 8 * (4j + q) of the string (words j, j + 1; q in 0..3): table entry 4j + q
ERAY_HD inline uint32_t inv_pio4_window(uint32_t hi, uint32_t lo, int q) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (32 - 8 * q));
}

ERAY_HD inline uint32_t f32_bits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
ERAY_HD inline uint32_t abstop12(float f) { return (f32_bits(f) >> 20) & 0x7ff; }

ERAY_HD inline double fma_d(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_fma(a, b, c);
#else
    return fma(a, b, c);
#endif
}

// sin (n even) or cos (n odd) polynomial of the reduced argument, rounded to float; `neg`: the
// second coefficient table (the cos result negated, see above).
ERAY_HD inline float sincos_poly(double x, double x2, int n, bool neg) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = fma_d(x2, kS3, kS2);
        double x7 = x3 * x2;
        double s = fma_d(x3, kS1, x);
        return (float)fma_d(x7, s1, s);
    }
    double x4 = x2 * x2;
    double c2 = fma_d(x2, kC4, kC3);
    double c1 = fma_d(x2, kC1, kC0);
    double x6 = x4 * x2;
    double c = fma_d(x4, kC2, c1);
    const float f = (float)fma_d(x6, c2, c);
    return neg ? -f : f;
}

// Reduction of |x| >= 120 with 4/pi to 96 significant bits: returns r in [-pi/4, pi/4]
// (before the final scaling) and the quadrant.
ERAY_HD inline double reduce_large(uint32_t xi, int* np) {
    int base = (int)((xi >> 26) & 15);
    int shift = (int)((xi >> 23) & 7);
    xi = (xi & 0xffffffu) | 0x800000u;
    xi <<= shift;
    // the table's entries base, base + 4 and base + 8 (base <= 15: words up to 6)
    uint32_t t0, t4, t8;
    auto entries = [&](int b) {
        const int j = b >> 2, q = b & 3;
        const uint32_t w0 = inv_pio4_word(j), w1 = inv_pio4_word(j + 1), w2 = inv_pio4_word(j + 2),
                       w3 = inv_pio4_word(j + 3);
        t0 = inv_pio4_window(w0, w1, q);
        t4 = inv_pio4_window(w1, w2, q);
        t8 = inv_pio4_window(w2, w3, q);
    };
#if defined(__HIP_DEVICE_COMPILE__)
    // a wave whose lanes share the row (main.rs's arguments 120..205 all do) selects it with
    // scalar instructions (kept apart from the per-lane path, which the compiler would merge)
    const int ub = __builtin_amdgcn_readfirstlane(base);
    if (__all(base == ub)) {
        entries(ub);
        asm volatile("" : "+s"(t0), "+s"(t4), "+s"(t8));
    } else
#endif
    {
        entries(base);
    }
    uint64_t res0 = (uint64_t)(uint32_t)(xi * t0);
    uint64_t res1 = (uint64_t)xi * t4;
    uint64_t res2 = (uint64_t)xi * t8;
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    uint64_t n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * 0x1.921FB54442D18p-62;
}

// a / 10.0f, correctly rounded (wave.rs:127's `/ 10.`): for biased exponents 32..254 a product
// by 0.1f and one FMA correction (q0 = a * 0.1f, r = a - 10 q0 exactly, q0 + r * 0.1f) equals the
// IEEE quotient — checked for every float of that range in tests/test_libm_restatement.py (it
// differs only for subnormal-range and non-finite inputs, which take the division)
ERAY_HD inline float div10_f32(float a) {
    const uint32_t e = (f32_bits(a) >> 23) & 0xffu;
    if (e >= 32u && e <= 254u) {
#if defined(__HIP_DEVICE_COMPILE__)
        const float q0 = a * 0x1.99999ap-4f;
        return __builtin_fmaf(__builtin_fmaf(-q0, 10.0f, a), 0x1.99999ap-4f, q0);
#else
        const float q0 = a * 0x1.99999ap-4f;
        return fmaf(fmaf(-q0, 10.0f, a), 0x1.99999ap-4f, q0);
#endif
    }
    return a / 10.0f;
}

// cosf(y) as computed by the reference platform's libm.
ERAY_HD inline float cosf_glibc(float y) {
    double x = y;
    int n;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {  // |y| < pi/4
        double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sincos_poly(x, x2, 1, false);
    } else if (abstop12(y) < abstop12(120.0f)) {
        double r = x * kHpiInv;
        n = ((int32_t)r + 0x800000) >> 24;
        x = fma_d(-(double)n, kHpi, x);
        return sincos_poly(x * quadrant_sign(n), x * x, n ^ 1, (n & 2) != 0);
    } else if (abstop12(y) < abstop12(__builtin_inff())) {
        uint32_t xi = f32_bits(y);
        int sign = (int)(xi >> 31);
        x = reduce_large(xi, &n);
        const int q = n + sign;
        return sincos_poly(x * quadrant_sign(q), x * x, n ^ 1, (q & 2) != 0);
    }
    return (y - y) / (y - y);  // inf or NaN -> NaN
}

}  // namespace libm
}  // namespace eray

// int_div.hpp — unsigned 32-bit division by a divisor fixed for a whole launch, as a multiply-high
// and two shifts (Granlund & Montgomery, "Division by invariant integers using multiplication",
// PLDI 1994, figure 4.1): the host derives (m, s1, s2) once; q = (t + ((n - t) >> s1)) >> s2 with
// t = mulhi(m, n) equals n / d for every 32-bit n (tests/test_int_div.py).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define ERAY_HD_DIV __host__ __device__
#else
#define ERAY_HD_DIV
#endif

namespace eray {

struct DivU32 {
    uint32_t m, s1, s2;
};

inline DivU32 make_div_u32(uint32_t d) {  // d >= 1
    uint32_t l = 0;
    while ((1ull << l) < d) ++l;  // ceil(log2 d)
    const uint64_t m = (((1ull << l) - d) << 32) / d + 1;
    return DivU32{(uint32_t)m, l < 1u ? l : 1u, l > 0u ? l - 1u : 0u};
}

ERAY_HD_DIV inline uint32_t div_u32(uint32_t n, DivU32 v) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t t = __umulhi(v.m, n);
#else
    const uint32_t t = (uint32_t)(((uint64_t)v.m * n) >> 32);
#endif
    return (t + ((n - t) >> v.s1)) >> v.s2;
}

}  // namespace eray

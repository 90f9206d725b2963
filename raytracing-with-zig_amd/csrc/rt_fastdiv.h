// rt_fastdiv.h — exact unsigned 32-bit division by a launch-invariant divisor (Granlund &
// Montgomery 1994, "Division by invariant integers using multiplication", Fig. 4.1 / Thm. 4.2).
//
// The work-queue refill splits a 32-bit item index into (sample, pixel) and a pixel into (row,
// column): two divisions by runtime values per new path.  A hardware-less 32-bit divide is ~30
// VALU instructions on CDNA; with the host-computed pair (m, l) it is one v_mul_hi_u32, a 64-bit
// add and a shift.  Exact for every 0 <= n < 2^32 and 1 <= d < 2^32 (tests/cpp/test_fastdiv.cpp).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define RT_FD_HD __host__ __device__ __forceinline__
#else
#define RT_FD_HD inline
#endif

namespace rtk {

struct FastDiv {
    uint32_t m;  // floor(2^32 (2^l - d) / d) + 1
    uint32_t l;  // ceil(log2 d)
};

inline FastDiv fastdiv_make(uint32_t d) {
    if (d == 0) d = 1;  // callers never divide by 0; keep the pair well-defined anyway
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < d) ++l;
    const uint64_t m = (((1ull << 32) * ((1ull << l) - d)) / d) + 1;  // < 2^32 + 1 by construction
    return FastDiv{(uint32_t)m, l};
}

RT_FD_HD uint32_t fastdiv(uint32_t n, FastDiv f) {
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t t = __umulhi(n, f.m);
#else
    const uint32_t t = (uint32_t)(((uint64_t)n * f.m) >> 32);
#endif
    return (uint32_t)(((uint64_t)t + n) >> f.l);
}

}  // namespace rtk

// CPU test of rt_fastdiv.h: fastdiv(n, fastdiv_make(d)) == n / d for edge and random (n, d),
// including every divisor 1..4096 and divisors near powers of two up to 2^32 - 1.
#include <cstdio>
#include <random>
#include <vector>

#include "../../raytracing-with-zig_amd/csrc/rt_fastdiv.h"

int main() {
    std::mt19937_64 rng(11);
    std::vector<uint32_t> ds;
    for (uint32_t d = 1; d <= 4096; d++) ds.push_back(d);
    for (int k = 1; k < 32; k++)
        for (int e = -2; e <= 2; e++) ds.push_back((uint32_t)((1ull << k) + e));
    ds.push_back(0xffffffffu);
    ds.push_back(1200u * 800u);
    for (int k = 0; k < 2000; k++) ds.push_back((uint32_t)rng() | 1u);
    long fails = 0, checks = 0;
    for (uint32_t d : ds) {
        if (d == 0) continue;
        const rtk::FastDiv f = rtk::fastdiv_make(d);
        std::vector<uint32_t> ns = {0u, 1u, d - 1, d, d + 1, 2 * d - 1, 0x7fffffffu, 0x80000000u,
                                    0xfffffffeu, 0xffffffffu, 0xffffffffu - d, 0xffffffffu / d * d};
        for (int k = 0; k < 2000; k++) ns.push_back((uint32_t)rng());
        for (uint32_t n : ns) {
            ++checks;
            if (rtk::fastdiv(n, f) != n / d) {
                if (fails++ < 10) std::printf("FAIL n=%u d=%u got %u\n", n, d, rtk::fastdiv(n, f));
            }
        }
    }
    std::printf("%ld checks, %ld fails\n%s\n", checks, fails, fails ? "FAILED" : "OK");
    return fails ? 1 : 0;
}

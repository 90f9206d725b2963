// Host check of the unit scheduler's chunk schedule (rt_kernel.h "Work units", chunk_range) and of
// the runtime's planning (rt_runtime.cpp unit_schedule, restated here): for every spp the chunks
// tile [0, spp) contiguously in order, main chunks have kUnitS samples, the tail halves down to
// one sample, and the unit count matches.  Built with hipcc (host code only; no GPU needed).
#include <cstdio>
#include <cstdlib>

#include "../../raytracing-with-zig_amd/csrc/rt_kernel.h"

static void plan(uint32_t spp, rtk::UnitArgs& ua) {  // == unit_schedule in rt_runtime.cpp
    ua.n_main = spp > rtk::kUnitS ? (spp - rtk::kUnitS) / rtk::kUnitS : 0;
    ua.tail_r = spp - ua.n_main * rtk::kUnitS;
    uint32_t t = 0;
    while ((1u << t) < ua.tail_r) ++t;
    ua.tail_t = t;
    ua.n_chunks = ua.n_main + t + 1;
}

int main() {
    for (uint32_t spp = 1; spp <= 20000; ++spp) {
        rtk::UnitArgs ua{};
        plan(spp, ua);
        uint32_t next = 0, prev_n = 0xffffffffu;
        for (uint32_t k = 0; k < ua.n_chunks; ++k) {
            uint32_t s0 = 0, n = 0;
            rtk::chunk_range(ua, k, &s0, &n);
            if (s0 != next || n == 0) { std::printf("spp %u chunk %u: s0 %u n %u (expected s0 %u)\n", spp, k, s0, n, next); return 1; }
            if (k < ua.n_main && n != rtk::kUnitS) { std::printf("spp %u main chunk %u has %u samples\n", spp, k, n); return 1; }
            if (k >= ua.n_main && n > prev_n) { std::printf("spp %u tail chunk %u grows (%u > %u)\n", spp, k, n, prev_n); return 1; }
            if (k >= ua.n_main) prev_n = n;
            if (n > rtk::kUnitS) { std::printf("spp %u chunk %u: %u samples > ring slot\n", spp, k, n); return 1; }
            next = s0 + n;
        }
        if (next != spp) { std::printf("spp %u: chunks cover %u samples\n", spp, next); return 1; }
        if (prev_n != 1) { std::printf("spp %u: last chunk has %u samples\n", spp, prev_n); return 1; }
    }
    std::printf("OK\n");
    return 0;
}

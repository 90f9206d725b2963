// Host check of the unit scheduler's chunk table (csrc/rt_schedule.hpp, read by rt_kernel.h
// chunk_range): for every spp and launch size the chunks tile [0, spp) contiguously in order, never
// exceed a ring slot (kUnitS), shrink monotonically towards the end (the first chunk is the
// remainder and may be smaller), end with a 1-sample chunk, and
// obey the drain bound S <= max(1, pixels / (kSchedDiv lanes) * samples_after).  Built with hipcc (host code
// only; no GPU needed).
#include <cstdio>
#include <cstdlib>

#include "../../raytracing-with-zig_amd/csrc/rt_kernel.h"
#include "../../raytracing-with-zig_amd/csrc/rt_schedule.hpp"

static int check(uint32_t spp, uint64_t pixels, uint64_t lanes) {
    const std::vector<uint32_t> t = rtk::chunk_schedule(spp, pixels, lanes, rtk::kUnitS);
    const size_t n_chunks = t.size() - 1;
    if (t.empty() || t[0] != 0 || t[n_chunks] != spp || n_chunks > spp) {
        std::printf("spp %u pixels %llu: bad table ends (%zu chunks)\n", spp, (unsigned long long)pixels, n_chunks);
        return 1;
    }
    const double ratio = (double)pixels / (rtk::kSchedDiv * (double)lanes);
    uint32_t prev = 0xffffffffu;
    for (size_t k = 0; k < n_chunks; ++k) {
        const uint32_t n = t[k + 1] - t[k], after = spp - t[k + 1];
        const double bound = ratio * after < 1.0 ? 1.0 : ratio * after;
        if (n == 0 || n > rtk::kUnitS || (k > 1 && n > prev) || (double)n > bound) {
            std::printf("spp %u pixels %llu chunk %zu: %u samples (prev %u, bound %.2f)\n", spp,
                        (unsigned long long)pixels, k, n, prev, bound);
            return 1;
        }
        prev = n;
    }
    if (prev != 1) { std::printf("spp %u: last chunk has %u samples\n", spp, prev); return 1; }
    return 0;
}

int main() {
    const uint64_t lanes = 256ull * 16 * 64;  // MI355X: 256 CUs x 16 waves
    const uint64_t sizes[] = {1, 37, 1200, 1200 * 100, 1200 * 800, 3840ull * 2160};
    for (uint64_t px : sizes)
        for (uint32_t spp = 1; spp <= 3000; ++spp)
            if (check(spp, px, lanes)) return 1;
    for (uint64_t px : sizes)
        if (check(10000, px, lanes)) return 1;
    // the bench launch: 960000 pixels at 500 spp keeps kUnitS-sample chunks up to the last few samples
    const std::vector<uint32_t> big = rtk::chunk_schedule(500, 1200 * 800, lanes, rtk::kUnitS);
    if (big.size() - 1 > 500 / rtk::kUnitS + 12) { std::printf("bench launch: %zu chunks\n", big.size() - 1); return 1; }
    std::printf("OK\n");
    return 0;
}

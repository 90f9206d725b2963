// rt_schedule.hpp — the sample-chunk schedule of a launch (host side; rt_kernel.h "Work units").
//
// A unit of S samples keeps its wave's lanes busy for about S path lengths.  When the claim counter
// runs dry, the units still in flight must not outlast the work that remains after them, or the
// launch ends in a long drain tail with most lanes idle; but small units cost lane utilisation (a
// ring slot frees only when the slowest of its paths ends).  So chunk sizes shrink towards the end
// of the launch: built backwards from the last chunk (1 sample), a chunk may hold S samples only if
// S <= ratio * (samples after it), ratio = pixels / (6 * resident lanes), and S <= kUnitS (a ring
// slot).  The divisor is measured: 8 with 16-sample units (config 4, rows 0::N, N = 1, 4, 8: 2, 3,
// 6, 16 slower), 6 with the 48 x 2 ring (4, 8, 12, 16 slower).
// The full frame gets kUnitS-sample chunks up to the last few samples; a rank's rows of an 8-GPU
// job taper off over the last ~250 samples.
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

namespace rtk {

constexpr double kSchedDiv = 6.0;  // drain divisor: ratio = pixels / (kSchedDiv * resident lanes)

// s0 of every chunk plus a final entry == spp (chunk k covers samples [s0[k], s0[k + 1])).
inline std::vector<uint32_t> chunk_schedule(uint32_t spp, uint64_t pixels, uint64_t lanes, uint32_t max_chunk) {
    const double ratio = (double)pixels / (kSchedDiv * (double)std::max<uint64_t>(lanes, 1));
    std::vector<uint32_t> rev;
    uint32_t after = 0;
    while (after < spp) {
        uint64_t s = (uint64_t)(ratio * (double)after);
        s = std::max<uint64_t>(1, std::min<uint64_t>(s, max_chunk));
        s = std::min<uint64_t>(s, spp - after);
        rev.push_back((uint32_t)s);
        after += (uint32_t)s;
    }
    std::vector<uint32_t> s0(rev.size() + 1);
    uint32_t acc = 0;
    for (size_t k = 0; k < rev.size(); ++k) {
        s0[k] = acc;
        acc += rev[rev.size() - 1 - k];
    }
    s0[rev.size()] = acc;
    return s0;
}

}  // namespace rtk

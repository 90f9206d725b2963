// CPU test of the host BVH builder (raytracing-with-zig_amd/csrc/rt_bvh.cpp): structural
// invariants the GPU walk's exactness relies on.  Built and run by tests/test_bvh_host.py.
//   * every boundable sphere appears in exactly one leaf slot, unboundable ones in the always-list
//   * every leaf has exactly kLeafMax slots (sentinel-padded)
//   * each child box (f32) contains the f64 box of every sphere below it, padded by
//     2^-17 (|c| + r) + 2^-21 * origin_bound
//   * depth <= kMaxDepth, refs in range
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../raytracing-with-zig_amd/csrc/rt_bvh.hpp"

static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { std::printf("FAIL %s:%d ", __FILE__, __LINE__); std::printf(__VA_ARGS__); std::printf("\n"); ++fails; } } while (0)

struct Box { double lo[3], hi[3]; };

static void collect(const rtbvh::Bvh& b, int32_t ref, std::vector<uint32_t>& out, int depth, int& maxd) {
    if (depth > maxd) maxd = depth;
    if (ref < 0) {
        const uint32_t leaf = (uint32_t)(~ref);
        const uint32_t first = b.n_always + leaf * rtbvh::kLeafMax;
        CHECK(first + rtbvh::kLeafMax <= b.slot_to_sphere.size(), "leaf %u out of range", leaf);
        for (uint32_t i = 0; i < (uint32_t)rtbvh::kLeafMax; i++) out.push_back(b.slot_to_sphere.at(first + i));
        return;
    }
    CHECK((size_t)ref < b.nodes.size(), "node ref %d", ref);
    const rtbvh::Node& nd = b.nodes[ref];
    collect(b, nd.ref0, out, depth + 1, maxd);
    collect(b, nd.ref1, out, depth + 1, maxd);
}

static void check_boxes(const rtbvh::Bvh& b, const std::vector<rt_sphere>& s, int32_t ref) {
    if (ref < 0) return;
    const rtbvh::Node& nd = b.nodes[ref];
    for (int c = 0; c < 2; c++) {
        std::vector<uint32_t> below;
        int d = 0;
        collect(b, c ? nd.ref1 : nd.ref0, below, 0, d);
        const float* lo = c ? nd.lo1 : nd.lo0;
        const float* hi = c ? nd.hi1 : nd.hi0;
        for (uint32_t k : below) {
            if (k == rtbvh::kSentinel) continue;
            const double r = s[k].radius > 0 ? s[k].radius : 0.0;
            double cmax = 0;
            for (int a = 0; a < 3; a++) cmax = std::fmax(cmax, std::fabs(s[k].center[a]));
            const double pad = std::ldexp(cmax + r, -17) + std::ldexp(b.origin_bound, -21);
            for (int a = 0; a < 3; a++) {
                CHECK((double)lo[a] <= s[k].center[a] - r - pad, "sphere %u axis %d lo", k, a);
                CHECK((double)hi[a] >= s[k].center[a] + r + pad, "sphere %u axis %d hi", k, a);
            }
        }
        check_boxes(b, s, c ? nd.ref1 : nd.ref0);
    }
}

static void run(const std::vector<rt_sphere>& s, const char* name) {
    const double ext = rtbvh::scene_extent(s.data(), s.size());
    const rtbvh::Bvh b = rtbvh::build(s.data(), s.size(), ext);
    CHECK(b.ok, "%s: build failed", name);
    if (!b.ok) return;
    std::vector<uint32_t> seen;
    int maxd = 0;
    collect(b, 0, seen, 1, maxd);
    CHECK(maxd <= rtbvh::kMaxDepth, "%s: depth %d", name, maxd);
    std::vector<int> count(s.size(), 0);
    for (uint32_t q = 0; q < b.n_always; q++) count.at(b.slot_to_sphere[q])++;
    for (uint32_t k : seen)
        if (k != rtbvh::kSentinel) count.at(k)++;
    for (size_t k = 0; k < s.size(); k++) CHECK(count[k] == 1, "%s: sphere %zu appears %d times", name, k, count[k]);
    check_boxes(b, s, 0);
    std::printf("%s: n=%zu nodes=%zu slots=%zu always=%u depth=%d\n", name, s.size(), b.nodes.size(),
                b.slot_to_sphere.size(), b.n_always, maxd);
}

int main() {
    std::mt19937_64 rng(7);
    std::normal_distribution<double> N(0, 5);
    std::uniform_real_distribution<double> U(0, 1);
    auto sph = [](double x, double y, double z, double r) {
        rt_sphere s{};
        s.center[0] = x; s.center[1] = y; s.center[2] = z;
        s.radius = r;
        return s;
    };
    {  // tiny scenes, including the single-sphere and two-sphere roots
        run({sph(0, 0, -1, 0.5)}, "one");
        run({sph(0, 0, -1, 0.5), sph(0, -100.5, -1, 100)}, "two");
    }
    {  // soup with duplicates, zero/negative radii, a huge sphere and an unboundable one
        std::vector<rt_sphere> s;
        for (int k = 0; k < 777; k++) s.push_back(sph(N(rng), N(rng), N(rng), U(rng) < 0.1 ? -U(rng) : U(rng)));
        s.push_back(s[3]);
        s.push_back(sph(0, -1000, 0, 1000));
        s.push_back(sph(INFINITY, 0, 0, 1));
        run(s, "soup");
    }
    {  // large scene (15000 full leaves): depth bound must hold (median splits take over)
        std::vector<rt_sphere> s;
        for (int k = 0; k < 15000 * rtbvh::kLeafMax; k++) s.push_back(sph(N(rng) * 10, N(rng), N(rng) * 10, 0.1));
        run(s, "large");
    }
    std::printf(fails ? "FAILED %d\n" : "OK\n", fails);
    return fails ? 1 : 0;
}

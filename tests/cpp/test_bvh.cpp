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
#include <cstring>
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

// a pinhole camera at `from` looking at the origin, 160x90 pixels (training-ray sampler input)
static rt_camera look_at(double fx, double fy, double fz) {
    rt_camera c{};
    c.image_width = 160; c.image_height = 90; c.samples_per_pixel = 1; c.bounce_max = 50;
    const double f[3] = {fx, fy, fz};
    double w[3], l = std::sqrt(fx * fx + fy * fy + fz * fz);
    for (int a = 0; a < 3; a++) w[a] = f[a] / l;
    double u[3] = {w[2], 0, -w[0]};  // cross((0,1,0), w)
    const double lu = std::sqrt(u[0] * u[0] + u[2] * u[2]);
    for (double& x : u) x /= lu;
    const double v[3] = {w[1] * u[2] - w[2] * u[1], w[2] * u[0] - w[0] * u[2], w[0] * u[1] - w[1] * u[0]};
    for (int a = 0; a < 3; a++) {
        c.center[a] = f[a];
        c.du[a] = 0.01 * u[a];
        c.dv[a] = -0.01 * v[a];
        c.pixel0[a] = f[a] - 10 * w[a] - 0.8 * u[a] + 0.45 * v[a];
    }
    c.t_min = 1e-3; c.t_max = INFINITY;
    return c;
}

static void run(const std::vector<rt_sphere>& s, const char* name, bool trained = false) {
    const double ext = std::fmax(rtbvh::scene_extent(s.data(), s.size()), 25.0);
    std::vector<rtbvh::TrainRay> rays;
    if (trained) {
        const rtbvh::Bvh sah = rtbvh::build(s.data(), s.size(), ext);
        rays = rtbvh::sample_rays(s.data(), s.size(), look_at(13, 2, 3), sah, 3000, 1);
        CHECK(rays.size() >= 3000, "%s: %zu training rays", name, rays.size());
    }
    const rtbvh::Bvh b = rtbvh::build(s.data(), s.size(), ext, trained ? &rays : nullptr);
    // the builder runs subtrees and axis pricing on threads: the tree must not depend on timing
    for (int rep = 0; rep < 3; rep++) {
        const rtbvh::Bvh b2 = rtbvh::build(s.data(), s.size(), ext, trained ? &rays : nullptr);
        CHECK(b2.ok == b.ok && b2.nodes.size() == b.nodes.size() && b2.slot_to_sphere == b.slot_to_sphere &&
                  (b.nodes.empty() || std::memcmp(b2.nodes.data(), b.nodes.data(), b.nodes.size() * sizeof(rtbvh::Node)) == 0),
              "%s: rebuild %d differs", name, rep);
    }
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
    // the host traversal (training-ray sampler) finds the linear scan's closest sphere
    std::mt19937_64 rng(11);
    std::normal_distribution<double> N(0, 4);
    for (int q = 0; q < 2000; q++) {
        const double o[3] = {N(rng), N(rng), N(rng)}, d[3] = {N(rng), N(rng), N(rng)};
        double t_tree, t_lin = INFINITY;
        const int k_tree = rtbvh::closest_hit(b, s.data(), o, d, 1e-3, &t_tree);
        int k_lin = -1;
        rtbvh::Bvh flat;  // always-list only: a linear scan through the same arithmetic
        flat.ok = true;
        for (uint32_t k = 0; k < s.size(); k++) flat.slot_to_sphere.push_back(k);
        flat.n_always = (uint32_t)s.size();
        k_lin = rtbvh::closest_hit(flat, s.data(), o, d, 1e-3, &t_lin);
        CHECK(k_tree == k_lin && (k_tree < 0 || t_tree == t_lin), "%s: ray %d tree %d lin %d", name, q, k_tree, k_lin);
    }
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
        s.pop_back();  // the sampler needs finite geometry to trace; the tree still takes any
        run(s, "soup_trained", true);
    }
    {  // a final-scene-like field: small spheres on a ground sphere, a ray-driven (trained) tree
        std::vector<rt_sphere> s{sph(0, -1000, 0, 1000)};
        for (int a = -11; a < 11; a++)
            for (int c = -11; c < 11; c++) s.push_back(sph(a + 0.9 * U(rng), 0.2, c + 0.9 * U(rng), 0.2));
        s.push_back(sph(0, 1, 0, 1));
        run(s, "field_trained", true);
    }
    {  // degenerate training input: zero and negative radii, coincident spheres (NaN normals in the
       // sampler's scatter) must still give a valid tree
        std::vector<rt_sphere> s;
        for (int k = 0; k < 200; k++) s.push_back(sph(N(rng) * 0.3, N(rng) * 0.3, N(rng) * 0.3, k % 3 ? 0.0 : -1.0));
        for (int k = 0; k < 100; k++) s.push_back(sph(0.5, 0.5, 0.5, 0.3));
        s.push_back(sph(0, -1000, 0, 1000));
        run(s, "degenerate_trained", true);
    }
    {  // large scene (15000 full leaves): depth bound must hold (median splits take over)
        std::vector<rt_sphere> s;
        for (int k = 0; k < 15000 * rtbvh::kLeafMax; k++) s.push_back(sph(N(rng) * 10, N(rng), N(rng) * 10, 0.1));
        run(s, "large");
    }
    std::printf(fails ? "FAILED %d\n" : "OK\n", fails);
    return fails ? 1 : 0;
}

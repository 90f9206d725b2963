// rt_bvh.cpp — host-side SAH BVH builder (see rt_bvh.hpp for the exactness argument).
//
// Padding rules (all f32 box bounds are rounded OUTWARD from the padded f64 bounds):
//   pad_k = 2^-17 * (|c_k|_inf + r_k) + 2^-21 * origin_bound + 2^-60
// The kernel's slab test computes t = fma(bound, inv32, -(o32 * inv32)) in f32, inv32 = v_rcp_f32
// of the f32 direction (1 ulp = 2^-23 relative).  Its position-space error on each axis is below
// 2^-24 * (4|bound| + 5|o|) (o -> f32, d -> f32, o*inv and the fma: one rounding of 2^-24 each;
// the reciprocal: 2^-23).  The |bound| part is covered by 2^-17 (|c| + r) and the |o| part by
// 2^-21 * origin_bound (= 8 * 2^-24 * bound >= 5 * 2^-24 |o|, a 1.6x margin).  A sphere's f64 root t_k is a point within ~1e-13 *
// (|c|+r) of the true surface, hence inside the padded box, so its leaf is never culled while
// t_k <= closest; the kernel also widens its `closest` bound by 2^-20 before comparing.
#include "rt_bvh.hpp"

#include <algorithm>
#include <cstdlib>
#include <utility>
#include <vector>
#include <cmath>
#include <limits>
#include <numeric>

namespace rtbvh {

namespace {

struct Prim {
    double lo[3], hi[3];  // padded bounds (f64)
    double c[3];          // centroid
    uint32_t sphere;      // original index
};

struct Builder {
    std::vector<Prim> prims;
    std::vector<Node> nodes;
    std::vector<uint32_t> slots;  // leaf slots (after the always-list)
    uint32_t slot_base = 0;
    int max_depth = 0;
    bool failed = false;

    static float down(double x) {
        float f = (float)x;
        if ((double)f > x) f = std::nextafterf(f, -std::numeric_limits<float>::infinity());
        return f;
    }
    static float up(double x) {
        float f = (float)x;
        if ((double)f < x) f = std::nextafterf(f, std::numeric_limits<float>::infinity());
        return f;
    }
    static double area(const double lo[3], const double hi[3]) {
        const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return dx * dy + dy * dz + dz * dx;
    }
    void bounds(size_t b, size_t e, double lo[3], double hi[3]) const {
        for (int a = 0; a < 3; a++) {
            lo[a] = std::numeric_limits<double>::infinity();
            hi[a] = -std::numeric_limits<double>::infinity();
        }
        for (size_t i = b; i < e; i++)
            for (int a = 0; a < 3; a++) {
                lo[a] = std::min(lo[a], prims[i].lo[a]);
                hi[a] = std::max(hi[a], prims[i].hi[a]);
            }
    }
    void set_box(float* flo, float* fhi, size_t b, size_t e) const {
        double lo[3], hi[3];
        bounds(b, e, lo, hi);
        for (int a = 0; a < 3; a++) {
            flo[a] = down(lo[a]);
            fhi[a] = up(hi[a]);
        }
    }

    // Leaves are padded to exactly kLeafMax slots with sentinels (kSentinel: never-hit geometry,
    // see rt_kernel.h), so the kernel tests every leaf with one fixed, unrolled block.
    int32_t leaf(size_t b, size_t e) {
        const uint32_t index = (uint32_t)(slots.size() / kLeafMax);
        for (size_t i = b; i < e; i++) slots.push_back(prims[i].sphere);
        for (size_t i = e - b; i < (size_t)kLeafMax; i++) slots.push_back(kSentinel);
        return ~(int32_t)index;
    }

    // returns the ref of the subtree over prims[b, e) at `depth` (root = 1)
    int32_t build(size_t b, size_t e, int depth) {
        max_depth = std::max(max_depth, depth);
        const size_t n = e - b;
        if (n <= (size_t)kLeafMax) return leaf(b, e);
        // levels a median-split subtree of n prims still needs below this node
        const int need = (int)std::ceil(std::log2((double)(n + kLeafMax - 1) / kLeafMax));
        if (depth + need > kMaxDepth) {
            failed = true;
            return leaf(b, b);
        }
        const bool median_only = depth + need + 2 > kMaxDepth;
        int best_axis = 0;
        size_t best_split = b + n / 2;
        double best_cost = std::numeric_limits<double>::infinity();
        std::vector<double> left_area(n);
        for (int ax = 0; ax < 3; ax++) {
            std::sort(prims.begin() + b, prims.begin() + e, [ax](const Prim& x, const Prim& y) {
                return x.c[ax] < y.c[ax] || (x.c[ax] == y.c[ax] && x.sphere < y.sphere);
            });
            if (median_only) {
                double lo[3], hi[3];
                bounds(b, e, lo, hi);
                const double ext = hi[ax] - lo[ax];
                if (-ext < best_cost) {  // widest axis
                    best_cost = -ext;
                    best_axis = ax;
                    best_split = b + n / 2;
                }
                continue;
            }
            double lo[3], hi[3];
            for (int a = 0; a < 3; a++) { lo[a] = prims[b].lo[a]; hi[a] = prims[b].hi[a]; }
            for (size_t i = b + 1; i < e; i++) {
                left_area[i - b] = area(lo, hi) * (double)(i - b);
                for (int a = 0; a < 3; a++) {
                    lo[a] = std::min(lo[a], prims[i].lo[a]);
                    hi[a] = std::max(hi[a], prims[i].hi[a]);
                }
            }
            for (int a = 0; a < 3; a++) { lo[a] = prims[e - 1].lo[a]; hi[a] = prims[e - 1].hi[a]; }
            for (size_t i = e - 1; i > b; i--) {
                const double cost = left_area[i - b] + area(lo, hi) * (double)(e - i);
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = ax;
                    best_split = i;
                }
                for (int a = 0; a < 3; a++) {
                    lo[a] = std::min(lo[a], prims[i - 1].lo[a]);
                    hi[a] = std::max(hi[a], prims[i - 1].hi[a]);
                }
            }
        }
        const int ax = best_axis;
        std::sort(prims.begin() + b, prims.begin() + e, [ax](const Prim& x, const Prim& y) {
            return x.c[ax] < y.c[ax] || (x.c[ax] == y.c[ax] && x.sphere < y.sphere);
        });
        const size_t me = nodes.size();
        nodes.emplace_back();
        const int32_t r0 = build(b, best_split, depth + 1);
        const int32_t r1 = build(best_split, e, depth + 1);
        Node& nd = nodes[me];
        set_box(nd.lo0, nd.hi0, b, best_split);
        set_box(nd.lo1, nd.hi1, best_split, e);
        nd.ref0 = r0;
        nd.ref1 = r1;
        nd.pad[0] = nd.pad[1] = 0;
        return (int32_t)me;
    }
};

bool boundable(const rt_sphere& s) {
    const double r = s.radius > 0 ? s.radius : 0.0;
    double m = r;
    for (int a = 0; a < 3; a++) {
        if (!std::isfinite(s.center[a])) return false;
        m = std::max(m, std::fabs(s.center[a]) + r);
    }
    return std::isfinite(r) && m < 1e30;
}

}  // namespace

double scene_extent(const rt_sphere* s, size_t n) {
    double m = 0;
    for (size_t k = 0; k < n; k++) {
        if (!boundable(s[k])) continue;
        const double r = s[k].radius > 0 ? s[k].radius : 0.0;
        for (int a = 0; a < 3; a++) m = std::max(m, std::fabs(s[k].center[a]) + r);
    }
    return m;
}

Bvh build(const rt_sphere* spheres, size_t n, double origin_bound) {
    Bvh out;
    out.origin_bound = origin_bound;
    Builder B;
    std::vector<uint32_t> always;
    const double e_origin = std::ldexp(origin_bound, -21);
    for (size_t k = 0; k < n; k++) {
        if (!boundable(spheres[k])) {
            always.push_back((uint32_t)k);
            continue;
        }
        Prim p;
        const double r = spheres[k].radius > 0 ? spheres[k].radius : 0.0;
        double cmax = 0;
        for (int a = 0; a < 3; a++) cmax = std::max(cmax, std::fabs(spheres[k].center[a]));
        const double pad = std::ldexp(cmax + r, -17) + e_origin + 0x1p-60;
        for (int a = 0; a < 3; a++) {
            p.c[a] = spheres[k].center[a];
            p.lo[a] = spheres[k].center[a] - r - pad;
            p.hi[a] = spheres[k].center[a] + r + pad;
        }
        p.sphere = (uint32_t)k;
        B.prims.push_back(p);
    }
    // Huge and big spheres go to the always-list.  A huge sphere (the final scene's radius-1000
    // ground) spans the scene: in the tree it costs a leaf round for most rays and inflates every
    // ancestor box.  A big one (its three radius-1 spheres among radius-0.2 ones) inflates the
    // boxes of every node above the small spheres it overlaps.  Tested up front in lockstep, each
    // costs one sphere test per ray and hands the traversal a tight `closest` to cull against.
    // Criterion: box surface area >= kAlwaysArea x the area of the box of all boundable spheres,
    // or >= kAlwaysRel x the median sphere box area; at most kMaxBig of them, largest first.
    // (Config 4: node visits per ray 8.86 -> 6.97, kernel -2%.)
    if (B.prims.size() > (size_t)kLeafMax) {
        double lo[3], hi[3];
        B.bounds(0, B.prims.size(), lo, hi);
        const double total = Builder::area(lo, hi);
        double frac = kAlwaysArea, rel = kAlwaysRel;
        if (const char* e = std::getenv("RTZIG_BVH_ALWAYS_AREA")) frac = std::atof(e);  // A/B knobs
        if (const char* e = std::getenv("RTZIG_BVH_ALWAYS_REL")) rel = std::atof(e);
        std::vector<double> areas(B.prims.size());
        for (size_t i = 0; i < B.prims.size(); i++) areas[i] = Builder::area(B.prims[i].lo, B.prims[i].hi);
        std::vector<double> sorted = areas;
        std::nth_element(sorted.begin(), sorted.begin() + (long)(sorted.size() / 2), sorted.end());
        const double median = sorted[sorted.size() / 2];
        std::vector<std::pair<double, size_t>> big;
        for (size_t i = 0; i < B.prims.size(); i++) {
            const double a = areas[i];
            if ((frac > 0 && a >= frac * total) || (rel > 0 && a >= rel * median)) big.push_back({-a, i});
        }
        std::sort(big.begin(), big.end());
        if (big.size() > (size_t)kMaxBig) big.resize(kMaxBig);
        std::vector<char> drop(B.prims.size(), 0);
        for (auto& bg : big) drop[bg.second] = 1;
        std::vector<Prim> keep;
        for (size_t i = 0; i < B.prims.size(); i++) {
            if (drop[i]) always.push_back(B.prims[i].sphere);
            else keep.push_back(B.prims[i]);
        }
        B.prims.swap(keep);
    }
    B.slot_base = (uint32_t)always.size();
    const size_t m = B.prims.size();
    if (m <= (size_t)kLeafMax) {
        // root with one leaf holding everything and one empty leaf (count 0)
        B.nodes.emplace_back();
        const int32_t r0 = B.leaf(0, m);
        Node& nd = B.nodes[0];
        if (m) {
            B.set_box(nd.lo0, nd.hi0, 0, m);
        } else {
            for (int a = 0; a < 3; a++) nd.lo0[a] = nd.hi0[a] = 3e38f;
        }
        for (int a = 0; a < 3; a++) nd.lo1[a] = nd.hi1[a] = 3e38f;
        nd.ref0 = r0;
        nd.ref1 = B.leaf(0, 0);  // all-sentinel leaf
        nd.pad[0] = nd.pad[1] = 0;
        B.max_depth = 2;
    } else {
        B.build(0, m, 1);
    }
    if (B.failed) return out;  // ok = false: the runtime falls back to the linear walk
    out.nodes = std::move(B.nodes);
    out.slot_to_sphere = always;
    out.slot_to_sphere.insert(out.slot_to_sphere.end(), B.slots.begin(), B.slots.end());
    out.n_always = (uint32_t)always.size();
    out.depth = B.max_depth;
    out.ok = true;
    return out;
}

}  // namespace rtbvh

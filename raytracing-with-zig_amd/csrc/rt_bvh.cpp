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
#include <exception>
#include <cstdlib>
#include <utility>
#include <vector>
#include <cmath>
#include <limits>
#include <numeric>
#include <thread>

namespace rtbvh {

namespace {

constexpr int kParDepth = 2;       // subtrees below nodes at depth <= this are built on their own threads
constexpr size_t kParMin = 64;     // ... when the node holds at least this many spheres

// f on its own thread while the caller goes on; join() rethrows what f threw, and the destructor
// joins, so no exception leaves a thread running or escapes one
struct Task {
    std::exception_ptr err;
    std::thread t;
    template <class F>
    explicit Task(F f) : t([this, f] {
        try {
            f();
        } catch (...) {
            err = std::current_exception();
        }
    }) {}
    Task(const Task&) = delete;
    Task& operator=(const Task&) = delete;
    void join() {
        if (t.joinable()) t.join();
        if (err) std::rethrow_exception(err);
    }
    ~Task() {
        if (t.joinable()) t.join();
    }
};

struct Prim {
    double lo[3], hi[3];  // padded bounds (f64)
    double c[3];          // centroid
    uint32_t sphere;      // original index
};

// a sample segment with its inverse direction (zero components flagged: those slabs test the
// origin instead)
struct Seg {
    double o[3], inv[3], tmax;
    unsigned zero;  // bit a: d[a] == 0
};

struct Builder {
    std::vector<Prim> prim_store;
    std::vector<Prim>& prims;     // shared with the sub-builders of parallel subtrees (disjoint ranges)
    std::vector<Seg> seg_store;
    const std::vector<Seg>& segs; // training segments (read-only once set)
    const std::vector<TrainRay>* train = nullptr;
    std::vector<Node> nodes;
    std::vector<uint32_t> slots;  // leaf slots (after the always-list)
    uint32_t slot_base = 0;
    int max_depth = 0;
    bool failed = false;

    Builder() : prims(prim_store), segs(seg_store) {}
    // a builder for one subtree of `p`'s tree: same primitives and segments, its own nodes and
    // leaves (merged back by append())
    explicit Builder(Builder& p) : prims(p.prims), segs(p.segs), train(p.train), slot_base(p.slot_base) {}

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

    void set_train(const std::vector<TrainRay>* t) {
        train = t;
        if (!t) return;
        seg_store.resize(t->size());
        for (size_t i = 0; i < t->size(); i++) {
            const TrainRay& r = (*t)[i];
            Seg& g = seg_store[i];
            g.zero = 0;
            g.tmax = r.tmax;
            for (int a = 0; a < 3; a++) {
                g.o[a] = r.o[a];
                g.inv[a] = r.d[a] == 0 ? 0.0 : 1.0 / r.d[a];
                if (r.d[a] == 0) g.zero |= 1u << a;
            }
        }
    }

    // does the sample segment [t_min, tmax] enter the box?  (f64 slabs)
    static bool seg_hits(const Seg& r, const double lo[3], const double hi[3]) {
        double t0 = 1e-3, t1 = r.tmax;
        for (int a = 0; a < 3; a++) {
            if (r.zero >> a & 1u) {
                if (r.o[a] < lo[a] || r.o[a] > hi[a]) return false;
                continue;
            }
            double ta = (lo[a] - r.o[a]) * r.inv[a], tb = (hi[a] - r.o[a]) * r.inv[a];
            if (ta > tb) std::swap(ta, tb);
            t0 = std::max(t0, ta);
            t1 = std::min(t1, tb);
        }
        return t0 <= t1;
    }

    // Ray-driven split cost over prims[b, e) sorted on one axis, for every split i (left = first i):
    // cost[i] = (segments entering the left box) * i^e + (segments entering the right box) * (n - i)^e
    // with e = kRayCostExp: the work a segment does below a box it enters grows with the box's
    // sphere count, but (a near-first walk stops early) much slower than linearly.
    // The left boxes grow with i and the right boxes shrink, so each segment's first entering left
    // split and last entering right split are found by bisection.
    // P: the node's n primitives, sorted on the axis being priced
    void ray_costs(const Prim* P, size_t n, const std::vector<uint32_t>& rays, std::vector<double>& cost) const {
        std::vector<double> L(6 * n), R(6 * n);  // L[i]: box of the first i prims, R[i]: of prims i..n-1
        double lo[3], hi[3];
        for (int a = 0; a < 3; a++) { lo[a] = P[0].lo[a]; hi[a] = P[0].hi[a]; }
        for (size_t i = 1; i < n; i++) {
            for (int a = 0; a < 3; a++) { L[6 * i + a] = lo[a]; L[6 * i + 3 + a] = hi[a]; }
            for (int a = 0; a < 3; a++) {
                lo[a] = std::min(lo[a], P[i].lo[a]);
                hi[a] = std::max(hi[a], P[i].hi[a]);
            }
        }
        for (int a = 0; a < 3; a++) { lo[a] = P[n - 1].lo[a]; hi[a] = P[n - 1].hi[a]; }
        for (size_t i = n - 1; i >= 1; i--) {
            for (int a = 0; a < 3; a++) { R[6 * i + a] = lo[a]; R[6 * i + 3 + a] = hi[a]; }
            for (int a = 0; a < 3; a++) {
                lo[a] = std::min(lo[a], P[i - 1].lo[a]);
                hi[a] = std::max(hi[a], P[i - 1].hi[a]);
            }
        }
        std::vector<double> first_l(n + 1, 0.0), last_r(n + 1, 0.0);  // histograms
        for (uint32_t ri : rays) {
            const Seg& r = segs[ri];
            if (seg_hits(r, &L[6 * (n - 1)], &L[6 * (n - 1) + 3])) {
                size_t l = 1, h = n - 1;  // smallest i with a hit
                while (l < h) {
                    const size_t m = (l + h) / 2;
                    if (seg_hits(r, &L[6 * m], &L[6 * m + 3])) h = m; else l = m + 1;
                }
                first_l[l] += 1;
            }
            if (seg_hits(r, &R[6], &R[9])) {
                size_t l = 1, h = n - 1;  // largest i with a hit
                while (l < h) {
                    const size_t m = (l + h + 1) / 2;
                    if (seg_hits(r, &R[6 * m], &R[6 * m + 3])) l = m; else h = m - 1;
                }
                last_r[l] += 1;
            }
        }
        cost.assign(n, std::numeric_limits<double>::infinity());
        double hl = 0, hr = 0;
        std::vector<double> hits_r(n + 1, 0.0);
        for (size_t i = n - 1; i >= 1; i--) { hr += last_r[i]; hits_r[i] = hr; }
        for (size_t i = 1; i < n; i++) {
            hl += first_l[i];
            cost[i] = hl * std::pow((double)i, kRayCostExp) + hits_r[i] * std::pow((double)(n - i), kRayCostExp);
        }
    }

    // appends sub-builder c's nodes and leaves after this builder's; returns c's ref `ref` remapped
    int32_t append(const Builder& c, int32_t ref) {
        const int32_t noff = (int32_t)nodes.size(), loff = (int32_t)(slots.size() / kLeafMax);
        auto remap = [&](int32_t r) { return r >= 0 ? r + noff : ~(~r + loff); };
        for (Node nd : c.nodes) {
            nd.ref0 = remap(nd.ref0);
            nd.ref1 = remap(nd.ref1);
            nodes.push_back(nd);
        }
        slots.insert(slots.end(), c.slots.begin(), c.slots.end());
        max_depth = std::max(max_depth, c.max_depth);
        failed = failed || c.failed;
        return remap(ref);
    }

    // returns the ref of the subtree over prims[b, e) at `depth` (root = 1); `rays`: the sample
    // segments that enter this subtree's box
    int32_t build(size_t b, size_t e, int depth, const std::vector<uint32_t>& rays = {}) {
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
            if (ax > 0 && !median_only && train && rays.size() >= kMinTrain) break;  // all axes priced at ax 0
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
            if (train && rays.size() >= kMinTrain) {
                if (ax == 0) {
                    // price the three axes (on their own threads at the top of the tree, each on a
                    // copy of the primitives sorted on its axis), then pick in the serial order
                    std::vector<double> cost[3];
                    auto price = [&](int a, std::vector<Prim>* copy) {
                        const Prim* P = &prims[b];
                        if (copy) {
                            copy->assign(prims.begin() + b, prims.begin() + e);
                            std::sort(copy->begin(), copy->end(), [a](const Prim& x, const Prim& y) {
                                return x.c[a] < y.c[a] || (x.c[a] == y.c[a] && x.sphere < y.sphere);
                            });
                            P = copy->data();
                        }
                        ray_costs(P, n, rays, cost[a]);
                    };
                    if (depth <= kParDepth + 1 && n >= kParMin) {
                        std::vector<Prim> c1, c2;
                        Task t1([&] { price(1, &c1); });
                        Task t2([&] { price(2, &c2); });
                        price(0, nullptr);  // prims[b, e) is sorted on axis 0 here
                        t1.join();
                        t2.join();
                    } else {
                        price(0, nullptr);
                        for (int a = 1; a < 3; a++) {
                            std::sort(prims.begin() + b, prims.begin() + e, [a](const Prim& x, const Prim& y) {
                                return x.c[a] < y.c[a] || (x.c[a] == y.c[a] && x.sphere < y.sphere);
                            });
                            price(a, nullptr);
                        }
                    }
                    for (int a = 0; a < 3; a++)
                        for (size_t i = 1; i < n; i++)
                            if (cost[a][i] < best_cost) {
                                best_cost = cost[a][i];
                                best_axis = a;
                                best_split = b + i;
                            }
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
        std::vector<uint32_t> rays0, rays1;
        if (train && rays.size() >= kMinTrain) {
            double lo[3], hi[3];
            bounds(b, best_split, lo, hi);
            for (uint32_t ri : rays)
                if (seg_hits(segs[ri], lo, hi)) rays0.push_back(ri);
            bounds(best_split, e, lo, hi);
            for (uint32_t ri : rays)
                if (seg_hits(segs[ri], lo, hi)) rays1.push_back(ri);
        }
        int32_t r0, r1;
        if (depth <= kParDepth && n >= kParMin) {
            // the two subtrees are independent (disjoint primitive ranges): build them concurrently
            // and append them in the serial order (left, then right), so the tree is identical
            Builder L(*this), R(*this);
            Task t([&] { r0 = L.build(b, best_split, depth + 1, rays0); });
            r1 = R.build(best_split, e, depth + 1, rays1);
            t.join();
            r0 = append(L, r0);
            r1 = append(R, r1);
        } else {
            r0 = build(b, best_split, depth + 1, rays0);
            r1 = build(best_split, e, depth + 1, rays1);
        }
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

Bvh build(const rt_sphere* spheres, size_t n, double origin_bound, const std::vector<TrainRay>* train) {
    Bvh out;
    out.origin_bound = origin_bound;
    Builder B;
    B.set_train(train);
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
        std::vector<uint32_t> rays;
        if (train) {
            double lo[3], hi[3];
            B.bounds(0, m, lo, hi);
            for (size_t i = 0; i < train->size(); i++)
                if (Builder::seg_hits(B.segs[i], lo, hi)) rays.push_back((uint32_t)i);
        }
        B.build(0, m, 1, rays);
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

namespace {

double sphere_root(const rt_sphere& s, const double o[3], const double d[3], double t_min, double closest) {
    const double r = s.radius > 0 ? s.radius : 0.0;
    double oc[3], a = 0, h = 0, c = 0;
    for (int k = 0; k < 3; k++) {
        oc[k] = s.center[k] - o[k];
        a += d[k] * d[k];
        h += d[k] * oc[k];
        c += oc[k] * oc[k];
    }
    c -= r * r;
    const double disc = h * h - a * c;
    if (!(disc >= 0)) return std::numeric_limits<double>::infinity();
    const double sq = std::sqrt(disc);
    double t = (h - sq) / a;
    if (!(t_min < t && t < closest)) {
        t = (h + sq) / a;
        if (!(t_min < t && t < closest)) return std::numeric_limits<double>::infinity();
    }
    return t;
}

bool box_enter(const float* lo, const float* hi, const double o[3], const double inv[3], double t0, double t1,
               double* tn) {
    for (int a = 0; a < 3; a++) {
        double ta = ((double)lo[a] - o[a]) * inv[a], tb = ((double)hi[a] - o[a]) * inv[a];
        if (ta > tb) std::swap(ta, tb);
        if (ta > t0) t0 = ta;  // NaN (0 * inf) keeps the box: permissive
        if (tb < t1) t1 = tb;
    }
    *tn = t0;
    return t0 <= t1;
}

// SplitMix64-driven uniform doubles in [0, 1) (training only; not the reference's stream)
struct TrainRng {
    uint64_t x;
    double next() {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return (double)((z ^ (z >> 31)) >> 11) * 0x1p-53;
    }
};

}  // namespace

int closest_hit(const Bvh& tree, const rt_sphere* spheres, const double o[3], const double d[3], double t_min,
                double* t_out) {
    double closest = std::numeric_limits<double>::infinity();
    int best = -1;
    auto test = [&](uint32_t k) {
        if (k == kSentinel) return;
        const double t = sphere_root(spheres[k], o, d, t_min, closest);
        if (t < closest || (t == closest && best >= 0 && (int)k < best)) {
            closest = t;
            best = (int)k;
        }
    };
    for (uint32_t q = 0; q < tree.n_always; q++) test(tree.slot_to_sphere[q]);
    if (!tree.nodes.empty()) {
        double inv[3];
        for (int a = 0; a < 3; a++) inv[a] = 1.0 / (d[a] == 0 ? 1e-300 : d[a]);
        int32_t stack[kMaxDepth + 2];
        int sp = 0;
        int32_t cur = 0;
        while (true) {
            if (cur >= 0) {
                const Node& nd = tree.nodes[(size_t)cur];
                double n0, n1;
                const bool h0 = box_enter(nd.lo0, nd.hi0, o, inv, t_min, closest, &n0);
                const bool h1 = box_enter(nd.lo1, nd.hi1, o, inv, t_min, closest, &n1);
                if (h0 && h1) {
                    stack[sp++] = n0 <= n1 ? nd.ref1 : nd.ref0;
                    cur = n0 <= n1 ? nd.ref0 : nd.ref1;
                    continue;
                }
                if (h0 || h1) {
                    cur = h0 ? nd.ref0 : nd.ref1;
                    continue;
                }
            } else {
                const size_t base = tree.n_always + (size_t)kLeafMax * (size_t)(~cur);
                for (int u = 0; u < kLeafMax; u++) test(tree.slot_to_sphere[base + (size_t)u]);
            }
            if (sp == 0) break;
            cur = stack[--sp];
        }
    }
    *t_out = closest;
    return best;
}

std::vector<TrainRay> sample_rays(const rt_sphere* spheres, size_t n, const rt_camera& cam, const Bvh& tree,
                                  size_t n_samples, uint64_t seed) {
    std::vector<TrainRay> out;
    if (!tree.ok || n == 0 || cam.image_width == 0 || cam.image_height == 0) return out;
    TrainRng g{seed};
    // pixel grid with ~n_samples points, stride s in both directions
    const double area = (double)cam.image_width * (double)cam.image_height;
    const uint32_t s = (uint32_t)std::max(1.0, std::floor(std::sqrt(area / (double)std::max<size_t>(n_samples, 1))));
    const uint32_t bounce_max = std::min<uint32_t>(cam.bounce_max, 50);
    auto unit_vec = [&](double v[3]) {  // Vec.randomUnitVec (vec.zig:71-80) by rejection
        while (true) {
            double l = 0;
            for (int k = 0; k < 3; k++) {
                v[k] = 2 * g.next() - 1;
                l += v[k] * v[k];
            }
            if (1e-160 < l && l <= 1) {
                const double sl = std::sqrt(l);
                for (int k = 0; k < 3; k++) v[k] /= sl;
                return;
            }
        }
    };
    for (uint32_t j = 0; j < cam.image_height; j += s)
        for (uint32_t i = 0; i < cam.image_width; i += s) {
            const double pi = (double)i + s * g.next() - 0.5, pj = (double)j + s * g.next() - 0.5;
            double o[3], d[3];
            double px = 0, py = 0;
            if (cam.defocus_angle > 0) {
                do {
                    px = 2 * g.next() - 1;
                    py = 2 * g.next() - 1;
                } while (px * px + py * py >= 1);
            }
            for (int k = 0; k < 3; k++) {
                const double ps = cam.pixel0[k] + cam.du[k] * pi + cam.dv[k] * pj;
                o[k] = cam.center[k] + (cam.defocus_angle > 0 ? cam.defocus_disk_u[k] * px + cam.defocus_disk_v[k] * py : 0.0);
                d[k] = ps - o[k];
            }
            for (uint32_t b = 0; b < bounce_max; b++) {
                double t;
                const int k = closest_hit(tree, spheres, o, d, cam.t_min, &t);
                TrainRay r;
                for (int a = 0; a < 3; a++) {
                    r.o[a] = o[a];
                    r.d[a] = d[a];
                }
                r.tmax = k >= 0 ? t : std::numeric_limits<double>::infinity();
                out.push_back(r);
                if (k < 0) break;
                const rt_sphere& S = spheres[k];
                const double rad = S.radius > 0 ? S.radius : 0.0;
                double p[3], nr[3], dn = 0;
                for (int a = 0; a < 3; a++) {
                    p[a] = o[a] + d[a] * t;
                    nr[a] = (p[a] - S.center[a]) / rad;
                    dn += d[a] * nr[a];
                }
                if (dn >= 0)
                    for (int a = 0; a < 3; a++) nr[a] = -nr[a];
                double v[3];
                if (S.material == RT_LAMBERTIAN) {
                    unit_vec(v);
                    for (int a = 0; a < 3; a++) d[a] = nr[a] + v[a];
                } else if (S.material == RT_METAL) {
                    double rf[3], l = 0, dd = 0;
                    for (int a = 0; a < 3; a++) dd += d[a] * nr[a];
                    for (int a = 0; a < 3; a++) {
                        rf[a] = d[a] - 2 * dd * nr[a];
                        l += rf[a] * rf[a];
                    }
                    unit_vec(v);
                    double dot_n = 0;
                    for (int a = 0; a < 3; a++) {
                        d[a] = rf[a] / std::sqrt(l) + S.fuzz * v[a];
                        dot_n += d[a] * nr[a];
                    }
                    if (!(dot_n > 0)) break;
                } else {
                    const double ri = dn < 0 ? 1.0 / S.refraction_index : S.refraction_index;
                    double u[3], l = 0, c = 0;
                    for (int a = 0; a < 3; a++) l += d[a] * d[a];
                    for (int a = 0; a < 3; a++) {
                        u[a] = d[a] / std::sqrt(l);
                        c -= u[a] * nr[a];
                    }
                    c = std::min(c, 1.0);
                    const double sn = std::sqrt(std::max(0.0, 1 - c * c));
                    double r0 = (1 - ri) / (1 + ri);
                    r0 *= r0;
                    if (ri * sn > 1 || r0 + (1 - r0) * std::pow(1 - c, 5) > g.next()) {
                        double un = 0;
                        for (int a = 0; a < 3; a++) un += u[a] * nr[a];
                        for (int a = 0; a < 3; a++) d[a] = u[a] - 2 * un * nr[a];
                    } else {
                        double perp[3], pl = 0;
                        for (int a = 0; a < 3; a++) {
                            perp[a] = ri * (u[a] + c * nr[a]);
                            pl += perp[a] * perp[a];
                        }
                        const double par = -std::sqrt(std::fabs(1 - pl));
                        for (int a = 0; a < 3; a++) d[a] = perp[a] + par * nr[a];
                    }
                }
                for (int a = 0; a < 3; a++) o[a] = p[a];
            }
        }
    return out;
}

}  // namespace rtbvh

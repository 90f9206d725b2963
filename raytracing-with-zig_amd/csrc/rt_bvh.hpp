// rt_bvh.hpp — bounding-volume hierarchy over the sphere list for the BVH walk of the hot path.
//
// Why this is exact (DESIGN.md §5 "BVH walk"): HittableList.hit (hittable.zig:64-77) accepts
// sphere k iff its root t_k (root1 if root1 > t_min, else root2 if root2 > t_min — independent of
// the running `closest`, because root2 >= root1) is strictly below the running closest.  The scan
// therefore returns argmin_k t_k with the LOWEST index winning ties.  Any traversal that (1) runs
// the identical f64 quadratic on every sphere it visits, (2) keeps min t with lowest-index ties, and
// (3) only skips spheres whose t_k provably exceeds the current closest, returns the same bits.
// (3) holds because node boxes are f32 boxes padded outward by more than every rounding error of
// the f32 slab test (see pad rules in rt_bvh.cpp), for every ray origin |o| <= origin_bound.
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/rt.h"

namespace rtbvh {

#ifndef RTZIG_LEAF
#define RTZIG_LEAF 2
#endif
constexpr int kLeafMax = RTZIG_LEAF;   // spheres per leaf (build knob; A/B on config 4: 2 < 4 < 3 ms, 1 and 8 clearly slower)
constexpr int kMaxDepth = 16; // tree depth bound == per-lane stack size in the kernel
constexpr double kAlwaysArea = 0.25;  // box-area fraction above which a sphere is tested always
constexpr double kAlwaysRel = 10.0;   // ... or box area above this multiple of the median sphere's
constexpr int kMaxBig = 4;           // at most this many such spheres
constexpr uint32_t kSentinel = 0xffffffffu;  // slot_to_sphere value of a padding slot
constexpr size_t kMinTrain = 64;             // ray-driven splits need at least this many segments
#ifndef RTZIG_RAYCOST_EXP
#define RTZIG_RAYCOST_EXP 0.4
#endif
constexpr double kRayCostExp = RTZIG_RAYCOST_EXP;  // ray-driven split cost: segments x spheres^kRayCostExp (build knob)

// Internal node: the boxes of both children (f32, padded outward) and their refs.
// ref >= 0: internal node index; ref < 0: leaf index ~ref.  Leaf L holds slots
// [n_always + kLeafMax*L, n_always + kLeafMax*(L+1)) (sentinel-padded to exactly kLeafMax).
struct alignas(16) Node {
    float lo0[3], hi0[3];
    float lo1[3], hi1[3];
    int32_t ref0, ref1;
    int32_t pad[2];
};  // 64 B
static_assert(sizeof(Node) == 64, "node layout");

struct Bvh {
    std::vector<Node> nodes;        // nodes[0] is the root
    std::vector<uint32_t> slot_to_sphere;  // leaf/always slot -> original sphere index
    uint32_t n_always = 0;          // slots [0, n_always) are tested for every ray (unboundable + huge spheres)
    int depth = 0;
    double origin_bound = 0;        // rays with max|o_i| <= origin_bound are covered by the padding
    bool ok = false;
};

// A sample ray segment [t_min, tmax] of the workload, for the ray-driven split cost (below).
struct TrainRay {
    double o[3], d[3];
    double tmax;  // the segment's end: its closest hit (or +inf)
};

// Builds the BVH.  `origin_bound`: bound on |ray origin| components the padding must cover
// (at least the scene's own extent; the runtime raises it for far-away cameras).
// `train` (optional): sample rays of the workload.  Each split then minimises the number of sample
// segments that enter each child box times the child's sphere count (the SAH's surface area is the
// same probability for uniformly distributed lines); nodes reached by fewer than kMinTrain
// segments use the SAH.
Bvh build(const rt_sphere* spheres, size_t n, double origin_bound, const std::vector<TrainRay>* train = nullptr);

// Closest hit of the ray (o, d) beyond t_min over the tree: a host traversal in plain f64, used to
// sample training rays (not the kernel's exact arithmetic).  Returns the sphere index or -1; *t =
// its root.
int closest_hit(const Bvh& tree, const rt_sphere* spheres, const double o[3], const double d[3], double t_min,
                double* t);

// Training segments for the ray-driven build: the paths of about `n_samples` camera samples spread
// over the whole image (a jittered pixel grid), traced through `tree` with the reference's camera
// and scatter rules (camera.zig:148-215, material.zig:27-110) and a local generator; every segment
// with its closest hit.  Deterministic for a given seed.
std::vector<TrainRay> sample_rays(const rt_sphere* spheres, size_t n, const rt_camera& cam, const Bvh& tree,
                                  size_t n_samples, uint64_t seed);

// Max |coordinate| of any sphere's bounding box (finite spheres only).
double scene_extent(const rt_sphere* spheres, size_t n);

}  // namespace rtbvh

// walk_occupancy.hip — does the closest-hit walk get faster with more resident waves?
// (VERDICT r02 "Next" #3)  A walk-only microkernel: the product's own BvhWalker
// (rt_kernel.hip, included below: the same while-while traversal of the LDS tree, the same f64 leaf
// rounds with the exact candidate filter, dynamic fetch at K = RTZIG_REFETCH_K) replays recorded
// ray segments of the config-4 workload at 4, 5, 6 and 8 waves per SIMD.  Nothing else runs in
// the kernel: no shading, RNG or scheduler, so the walk's dependent LDS chain is covered only by
// the other waves' walks.
//
// Occupancy is set by the block size B with two blocks per CU (each block stages the tree: 52.7 KB
// for the trained final-scene tree); the per-lane stacks use 16-bit entries (every ref of a tree
// that fits the LDS is < 2^15), so 2 x (tree + depth x B x 2 B) fits the CU's 160 KiB up to
// B = 1024 (8 waves per SIMD).  The 4-wave case is also run with the product's int32 stack.
// Every variant's (sphere, t) results must be bit-identical to each other and to a host linear scan
// of the reference's f64 quadratic on a sample of the segments.
//
// Segments: rtbvh::sample_rays (the library's path sampler: the reference's camera and scatter
// rules, a local generator) over the final scene with the main.zig camera at 1200x800, ~1.2 M
// camera samples.  Order: as sampled (each path's segments consecutive, paths on a jittered pixel
// grid), like the persistent kernel's neighbouring pixels.
//
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I include tools/walk_occupancy.hip \
//       raytracing-with-zig_amd/csrc/rt_bvh.cpp raytracing-with-zig_amd/csrc/rt_host.cpp -o walk_occ
//   ./walk_occ [samples=1200000] [reps=5]          (prints one JSON object)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../raytracing-with-zig_amd/csrc/rt_kernel.hip"
#include "../raytracing-with-zig_amd/csrc/rt_bvh.hpp"

// rt_host.cpp's Camera::render calls the GPU entry point; this tool never does
extern "C" int rt_render(const rt_camera*, const rt_sphere*, size_t, const rt_options*, void*) { return -1; }

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

namespace occ {
using namespace rtk;

struct Segs {  // SoA of the recorded segments, replayed: segment j of the launch is recorded one j % n
    const double *ox, *oy, *oz, *dx, *dy, *dz;
    uint32_t n;       // recorded segments
    uint32_t total;   // segments traced by the launch (n x replays)
    const uint32_t* path0;  // [n_paths + 1]: path p's segments are [path0[p], path0[p + 1]) (raster order)
    uint32_t n_paths;       // recorded paths (one camera sample each)
    uint32_t total_paths;   // paths traced by the launch (n_paths x replays)
};

// Static assignment: lane g of the grid (G lanes) traces segments g, g + G, g + 2G, ... (a shared
// claim counter would bound the launch at its ~100 atomics per µs, as round 2 measured).
// The argument order matters: BvhWalker reads the always-list pointers and count from the kernarg
// segment at BvhArgs's offset in the product kernels (KernelParams first, 336 B, then BvhArgs), so
// this kernel takes an (unused) KernelParams first as well.
template <int B, class StackT, int kWaves>
__global__ __launch_bounds__(B) __attribute__((amdgpu_waves_per_eu(kWaves, kWaves))) void walk_kernel(
    KernelParams kp_unused, BvhArgs b, Segs sg, double t_min, int32_t* __restrict__ out_k,
    double* __restrict__ out_t, unsigned long long* __restrict__ ctr, unsigned long long* __restrict__ sum) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const size_t scene_bytes = (size_t)bvh_leaves_offset(b.n_nodes) + (size_t)b.n_leaves * sizeof(BvhLeaf);
    StackT* stack = (StackT*)(lds_raw + scene_bytes);
    using W = BvhWalker<true, B, StackT>;
    stack[threadIdx.x] = (StackT)W::kEnd;
    BvhNode* ln = (BvhNode*)lds_raw;
    BvhLeaf* ll = (BvhLeaf*)(lds_raw + bvh_leaves_offset(b.n_nodes));
    for (uint32_t k = threadIdx.x; k < b.n_nodes; k += blockDim.x) ln[k] = b.nodes[k];
    for (uint32_t k = threadIdx.x; k < b.n_leaves; k += blockDim.x) ll[k] = b.leaves[k];
    __syncthreads();
    const W walk{ln, ll, b.always_geo, b.always_sid, b.n_always, stack + threadIdx.x, b.origin_bound, nullptr, 0};
    const uint32_t lane = lane_id();
    const uint32_t G = gridDim.x * blockDim.x;
    uint32_t next = blockIdx.x * blockDim.x + threadIdx.x;  // this lane's next segment
    bool active = false, susp = false;
    uint32_t mine = 0;
    Ray r;
    typename W::State ws;
    Prof<false> pr;
    bool drained = false;
    uint64_t check = 0;  // replays: a sum of the results (keeps their work live), compared across variants
    while (true) {
        if (!active && !drained) {
            const uint32_t j = next;
            if (j < sg.total) {
                const uint32_t i = j < sg.n ? j : j % sg.n;
                mine = j;
                r.orig = mk(sg.ox[i], sg.oy[i], sg.oz[i]);
                r.dir = mk(sg.dx[i], sg.dy[i], sg.dz[i]);
                active = true;
                susp = false;
                next = j + G < j ? 0xffffffffu : j + G;
            } else {
                drained = true;
            }
        }
        if (__ballot(active) == 0) break;
        if (active) {
            __builtin_amdgcn_s_setprio(2);
            double t;
            const int k = walk.template run<(kRefetchK > 0)>(r, t_min, __builtin_inf(), &t, pr, ws, susp);
            __builtin_amdgcn_s_setprio(0);
            susp = k == kSuspended;
            if (!susp) {
                if (mine < sg.n) {
                    out_k[mine] = k;
                    out_t[mine] = t;
                } else {
                    check += (uint64_t)(k + 1) + __builtin_bit_cast(uint64_t, t);
                }
                active = false;
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) check += __shfl_xor(check, off, 64);
    if (lane == 0) atomicAdd(sum, (unsigned long long)check);
}
// Path-ordered variant (round 4): the lanes of a wave trace whole PATHS the way
// the megakernel's lanes do — wave w owns a contiguous range of paths (raster order, so its lanes start
// on neighbouring pixels' camera rays), a lane walks its path's segments one after another, and a
// lane whose path has ended takes the wave's next path (ballot + mbcnt, no atomics).  Dynamic fetch as
// in the product.  The static-stride kernel above gives neighbouring lanes consecutive segments of ONE
// path (a camera ray next to its own bounces), which the megakernel never does.
template <int B, class StackT, int kWaves, bool kPrefetch = false>
__global__ __launch_bounds__(B) __attribute__((amdgpu_waves_per_eu(kWaves, kWaves))) void walk_kernel_paths(
    KernelParams kp_unused, BvhArgs b, Segs sg, double t_min, int32_t* __restrict__ out_k,
    double* __restrict__ out_t, unsigned long long* __restrict__ ctr, unsigned long long* __restrict__ sum) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const size_t scene_bytes = (size_t)bvh_leaves_offset(b.n_nodes) + (size_t)b.n_leaves * sizeof(BvhLeaf);
    StackT* stack = (StackT*)(lds_raw + scene_bytes);
    using W = BvhWalker<true, B, StackT>;
    stack[threadIdx.x] = (StackT)W::kEnd;
    BvhNode* ln = (BvhNode*)lds_raw;
    BvhLeaf* ll = (BvhLeaf*)(lds_raw + bvh_leaves_offset(b.n_nodes));
    for (uint32_t k = threadIdx.x; k < b.n_nodes; k += blockDim.x) ln[k] = b.nodes[k];
    for (uint32_t k = threadIdx.x; k < b.n_leaves; k += blockDim.x) ll[k] = b.leaves[k];
    __syncthreads();
    const W walk{ln, ll, b.always_geo, b.always_sid, b.n_always, stack + threadIdx.x, b.origin_bound, nullptr, 0};
    const uint32_t lane = lane_id();
    const uint32_t waves = gridDim.x * (blockDim.x / 64);
    const uint32_t wave = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
    const uint32_t per = (sg.total_paths + waves - 1) / waves;
    uint32_t pnext = wave * per;                                        // wave-uniform
    const uint32_t pend = pnext + per < sg.total_paths ? pnext + per : sg.total_paths;
    bool active = false, susp = false, has_path = false;
    uint32_t seg = 0, seg_end = 0, rep = 0;  // the lane's current segment, its path's end, replay round
    Ray r, nr;                               // nr: the next segment, prefetched (kPrefetch)
    bool pf_ok = false;                      // nr holds segment seg's ray
    typename W::State ws;
    Prof<false> pr;
    uint64_t check = 0;
    while (true) {
        // lanes without a segment: the next segment of their path, or a new path from the wave's range
        const uint64_t need = __ballot(!has_path);
        if (need != 0 && pnext < pend) {
            const uint32_t rk = rank_in(need);
            if (!has_path && pnext + rk < pend) {
                const uint32_t pg = pnext + rk, p = pg % sg.n_paths;
                rep = pg / sg.n_paths;
                seg = sg.path0[p];
                seg_end = sg.path0[p + 1];
                has_path = true;
            }
            const uint32_t got = (uint32_t)__popcll(need);
            pnext = pnext + got < pend ? pnext + got : pend;
        }
        if (has_path && !active) {
            if constexpr (kPrefetch) {
                // the ray was loaded into nr while the previous segment walked (the megakernel has
                // it in registers from shading); a new path's first segment is loaded here
                if (!pf_ok) {
                    nr.orig = mk(sg.ox[seg], sg.oy[seg], sg.oz[seg]);
                    nr.dir = mk(sg.dx[seg], sg.dy[seg], sg.dz[seg]);
                }
                r = nr;
                if (seg + 1 < seg_end) {
                    nr.orig = mk(sg.ox[seg + 1], sg.oy[seg + 1], sg.oz[seg + 1]);
                    nr.dir = mk(sg.dx[seg + 1], sg.dy[seg + 1], sg.dz[seg + 1]);
                }
                pf_ok = seg + 1 < seg_end;
            } else {
                r.orig = mk(sg.ox[seg], sg.oy[seg], sg.oz[seg]);
                r.dir = mk(sg.dx[seg], sg.dy[seg], sg.dz[seg]);
            }
            active = true;
            susp = false;
        }
        if (__ballot(active) == 0) break;
        if (active) {
            __builtin_amdgcn_s_setprio(2);
            double t;
            const int k = walk.template run<(kRefetchK > 0)>(r, t_min, __builtin_inf(), &t, pr, ws, susp);
            __builtin_amdgcn_s_setprio(0);
            susp = k == kSuspended;
            if (!susp) {
                if (rep == 0) {
                    out_k[seg] = k;
                    out_t[seg] = t;
                } else {
                    check += (uint64_t)(k + 1) + __builtin_bit_cast(uint64_t, t);
                }
                active = false;
                if (++seg == seg_end) {
                    has_path = false;
                    pf_ok = false;
                }
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) check += __shfl_xor(check, off, 64);
    if (lane == 0) atomicAdd(sum, (unsigned long long)check);
}
}  // namespace occ

namespace {

// device tree of rt_runtime.cpp's set_tree (tools keep their own copy of the conversion)
struct DevTree {
    std::vector<rtk::BvhNode> nodes;
    std::vector<rtk::BvhLeaf> leaves;
    std::vector<rtk::GeoRec> ageo;
    std::vector<uint32_t> asid;
    uint32_t depth = 0;
};
int32_t dref(int32_t ref) {
    if (ref >= 0) return (int32_t)(ref * (int64_t)sizeof(rtk::BvhNode));
    return ~(int32_t)((int64_t)(~ref) * (int64_t)sizeof(rtk::BvhLeaf));
}
rtk::GeoRec geo(const rt_sphere* s) {
    if (!s) return rtk::GeoRec{0, 0, 0, -INFINITY};
    const double r = s->radius > 0 ? s->radius : 0.0;
    return rtk::GeoRec{s->center[0], s->center[1], s->center[2], r * r};
}
DevTree convert(const rtbvh::Bvh& t, const std::vector<rt_sphere>& sp) {
    DevTree d;
    auto sph = [&](uint32_t k) { return k == rtbvh::kSentinel ? nullptr : &sp[k]; };
    for (const rtbvh::Node& s : t.nodes) {
        rtk::BvhNode n{};
        for (int a = 0; a < 3; a++) {
            n.c0[a][0] = n.c0[a][3] = s.lo0[a];
            n.c0[a][1] = n.c0[a][2] = s.hi0[a];
            n.c1[a][0] = n.c1[a][3] = s.lo1[a];
            n.c1[a][1] = n.c1[a][2] = s.hi1[a];
        }
        n.ref0 = dref(s.ref0);
        n.ref1 = dref(s.ref1);
        d.nodes.push_back(n);
    }
    const size_t na = t.n_always, nl = (t.slot_to_sphere.size() - na) / rtk::kLeafBvh;
    for (size_t l = 0; l < nl; l++) {
        rtk::BvhLeaf L{};
        for (int u = 0; u < rtk::kLeafBvh; u++) {
            const uint32_t k = t.slot_to_sphere[na + l * rtk::kLeafBvh + u];
            const rtk::GeoRec g = geo(sph(k));
            L.g[u] = rtk::LeafGeo{g.cx, g.cy, g.cz, g.r2};
            L.sid[u] = k;
        }
        d.leaves.push_back(L);
    }
    for (size_t q = 0; q < na; q++) {
        d.ageo.push_back(geo(sph(t.slot_to_sphere[q])));
        d.asid.push_back(t.slot_to_sphere[q]);
    }
    if (d.ageo.empty()) { d.ageo.push_back(geo(nullptr)); d.asid.push_back(0); }
    d.depth = (uint32_t)std::max(2, std::min(t.depth, rtk::kMaxDepthBvh));
    return d;
}

// the reference's linear scan (hittable.zig:64-77, sphere.zig:26-41) in plain f64, for the check
int scan(const std::vector<rt_sphere>& sp, const double* o, const double* d, double t_min, double* t_out) {
    double closest = INFINITY;
    int best = -1;
    const double a = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
    for (size_t k = 0; k < sp.size(); k++) {
        const double r = sp[k].radius > 0 ? sp[k].radius : 0.0;
        const double ocx = sp[k].center[0] - o[0], ocy = sp[k].center[1] - o[1], ocz = sp[k].center[2] - o[2];
        const double h = (d[0] * ocx + d[1] * ocy) + d[2] * ocz;
        const double c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - r * r;
        const double disc = h * h - a * c;
        if (disc < 0) continue;
        const double sq = std::sqrt(disc);
        double root = (h - sq) / a;
        if (!(t_min < root && root < closest)) {
            root = (h + sq) / a;
            if (!(t_min < root && root < closest)) continue;
        }
        closest = root;
        best = (int)k;
    }
    *t_out = closest;
    return best;
}

template <class T>
T* upload(const std::vector<T>& v) {
    T* p = nullptr;
    CK(hipMalloc(&p, std::max<size_t>(1, v.size()) * sizeof(T)));
    CK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return p;
}

struct Result {
    const char* name;
    int block, waves_per_simd, stack_bytes;
    double ms, ns_per_seg;
    uint32_t resident_blocks_per_cu;
};

}  // namespace

int main(int argc, char** argv) {
    const size_t n_samples = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 1200000;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const uint32_t replays = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 40;  // passes over the recorded set per launch
    std::vector<rt_sphere> sp(600);
    size_t n = 0;
    rt_scene_final(0xDEADBEEF, sp.data(), sp.size(), &n, nullptr);
    sp.resize(n);
    rt_camera_params p{};
    p.image_width = 1200; p.samples_per_pixel = 500; p.bounce_max = 50; p.aspect_ratio = 1.5;
    p.look_from[0] = 13; p.look_from[1] = 2; p.look_from[2] = 3;
    p.v_up[1] = 1; p.vfov = 20; p.defocus_angle = 0.6; p.focus_dist = 10; p.t_min = 1e-3; p.t_max = INFINITY;
    rt_camera cam;
    rt_camera_build(&p, &cam);
    // the runtime's tree for config 4: SAH, then trained on 6000 camera samples (rt_runtime.cpp)
    const double bound = rtbvh::scene_extent(sp.data(), n) * (1.0 + 0x1p-20) + 1e-300;
    const rtbvh::Bvh sah = rtbvh::build(sp.data(), n, bound);
    const auto train = rtbvh::sample_rays(sp.data(), n, cam, sah, 6000, 0x7261792d74726565ull);
    const rtbvh::Bvh tree = rtbvh::build(sp.data(), n, bound, &train);
    const DevTree dt = convert(tree, sp);
    // the replayed workload: a different sample of the same camera's paths
    const auto segs = rtbvh::sample_rays(sp.data(), n, cam, sah, n_samples, 0x0cc0ffee);
    const uint32_t ns = (uint32_t)segs.size();
    // path boundaries: sample_rays records each path's segments consecutively, starting with its
    // camera ray (origin within the defocus disk around the camera center)
    std::vector<uint32_t> path0;
    for (uint32_t i = 0; i < ns; i++) {
        double d2 = 0;
        for (int a = 0; a < 3; a++) d2 += (segs[i].o[a] - cam.center[a]) * (segs[i].o[a] - cam.center[a]);
        if (d2 < 1.0) path0.push_back(i);  // the disk radius is 10 * tan(0.3 deg) = 0.052
    }
    path0.push_back(ns);
    const uint32_t n_paths = (uint32_t)path0.size() - 1;
    std::vector<double> h[6];
    for (auto& v : h) v.reserve(ns);
    for (const auto& s : segs)
        for (int a = 0; a < 3; a++) {
            h[a].push_back(s.o[a]);
            h[3 + a].push_back(s.d[a]);
        }
    occ::Segs sg{upload(h[0]), upload(h[1]), upload(h[2]), upload(h[3]), upload(h[4]), upload(h[5]), ns,
                 (uint32_t)std::min<uint64_t>((uint64_t)ns * replays, 0xffffffffull), upload(path0), n_paths,
                 (uint32_t)std::min<uint64_t>((uint64_t)n_paths * replays, 0xffffffffull)};
    rtk::BvhArgs b{};
    b.nodes = upload(dt.nodes);
    b.leaves = upload(dt.leaves);
    b.always_geo = upload(dt.ageo);
    b.always_sid = upload(dt.asid);
    b.n_nodes = (uint32_t)dt.nodes.size();
    b.n_leaves = (uint32_t)dt.leaves.size();
    b.n_always = tree.n_always;
    b.stack_depth = dt.depth;
    b.origin_bound = (float)bound;
    if ((double)b.origin_bound > bound) b.origin_bound = std::nextafterf(b.origin_bound, 0.0f);
    const size_t scene_bytes = (size_t)rtk::bvh_leaves_offset(b.n_nodes) + (size_t)b.n_leaves * sizeof(rtk::BvhLeaf);
    rtk::KernelParams kp;
    std::memset(&kp, 0, sizeof kp);
    static_assert(sizeof(rtk::KernelParams) == 336, "BvhArgs's kernarg offset (rt_kernel.hip test_always_c)");
    int32_t* d_k = nullptr;
    double* d_t = nullptr;
    unsigned long long* d_ctr = nullptr;
    unsigned long long* d_sum = nullptr;
    CK(hipMalloc(&d_sum, sizeof(unsigned long long)));
    unsigned long long ref_sum = 0;
    CK(hipMalloc(&d_k, ns * sizeof(int32_t)));
    CK(hipMalloc(&d_t, ns * sizeof(double)));
    CK(hipMalloc(&d_ctr, sizeof(unsigned long long)));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::fprintf(stderr, "%u segments (%zu samples), tree %u nodes %u leaves depth %u always %u, scene %zu B, %d CUs\n",
                 ns, n_samples, b.n_nodes, b.n_leaves, b.stack_depth, b.n_always, scene_bytes, cus);

    std::vector<int32_t> ref_k;
    std::vector<double> ref_t;
    std::vector<Result> res;
    bool all_equal = true;
    auto run = [&](auto kernel, const char* name, int B, int waves, int entry) {
        const size_t shmem = scene_bytes + (size_t)b.stack_depth * B * entry;
        CK(hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem));
        int per_cu = 0;
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, B, shmem));
        const uint32_t grid = (uint32_t)(cus * per_cu);
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        std::vector<float> ms;
        for (int r = 0; r <= reps; r++) {
            CK(hipMemset(d_ctr, 0, sizeof(unsigned long long)));
            CK(hipMemset(d_sum, 0, sizeof(unsigned long long)));
            CK(hipMemset(d_k, 0xff, ns * sizeof(int32_t)));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(kernel, dim3(grid), dim3(B), shmem, 0, kp, b, sg, 1e-3, d_k, d_t, d_ctr, d_sum);
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r) ms.push_back(t);  // the first launch is a warm-up
        }
        std::sort(ms.begin(), ms.end());
        std::vector<int32_t> k(ns);
        std::vector<double> t(ns);
        CK(hipMemcpy(k.data(), d_k, ns * sizeof(int32_t), hipMemcpyDeviceToHost));
        CK(hipMemcpy(t.data(), d_t, ns * sizeof(double), hipMemcpyDeviceToHost));
        unsigned long long sum = 0;
        CK(hipMemcpy(&sum, d_sum, sizeof sum, hipMemcpyDeviceToHost));
        if (ref_k.empty()) {
            ref_k = k;
            ref_t = t;
            ref_sum = sum;
        } else if (k != ref_k || std::memcmp(t.data(), ref_t.data(), ns * sizeof(double)) != 0 || sum != ref_sum) {
            all_equal = false;
        }
        const double med = ms[ms.size() / 2];
        res.push_back({name, B, (int)(per_cu * B / 64 / 4), entry, med, med * 1e6 / sg.total, (uint32_t)per_cu});
        std::fprintf(stderr, "%-12s B=%4d blocks/CU=%d waves/SIMD=%d  %.3f ms  %.4f ns/segment\n", name, B, per_cu,
                     per_cu * B / 256, med, med * 1e6 / sg.total);
    };
    // 8 waves per SIMD (B = 1024) is not run: it needs 64 VGPRs and spills ~23 of them to scratch in
    // this build, and its launch faulted on the MI355X in round 4 (an aperture violation); round 3's
    // build (11 spilled) ran it +3.6% slower than 4 waves
    const char* mode = std::getenv("WALK_OCC_MODE");  // "stride" (round 3), "paths" (round 4), default both
    if (!mode || std::strcmp(mode, "paths") != 0) {
        run(occ::walk_kernel<512, int32_t, 4>, "w4_i32", 512, 4, 4);
        run(occ::walk_kernel<512, int16_t, 4>, "w4_i16", 512, 4, 2);
        run(occ::walk_kernel<640, int16_t, 5>, "w5_i16", 640, 5, 2);
        run(occ::walk_kernel<768, int16_t, 6>, "w6_i16", 768, 6, 2);
    }
    if (!mode || std::strcmp(mode, "stride") != 0) {
        run(occ::walk_kernel_paths<512, int32_t, 4>, "paths_w4_i32", 512, 4, 4);
        run(occ::walk_kernel_paths<512, int16_t, 4>, "paths_w4_i16", 512, 4, 2);
        run(occ::walk_kernel_paths<640, int16_t, 5>, "paths_w5_i16", 640, 5, 2);
        run(occ::walk_kernel_paths<768, int16_t, 6>, "paths_w6_i16", 768, 6, 2);
        run(occ::walk_kernel_paths<512, int32_t, 4, true>, "paths_pf_w4_i32", 512, 4, 4);
        run(occ::walk_kernel_paths<640, int16_t, 5, true>, "paths_pf_w5_i16", 640, 5, 2);
        // (6 waves with prefetch needs 94 VGPRs of 80 and spills 14 to scratch: not run, as w8 above)
    }

    // host check of a sample against the reference's linear scan
    uint32_t checked = 0, mism = 0;
    for (uint32_t i = 0; i < ns; i += 97, checked++) {
        double t;
        const int k = scan(sp, segs[i].o, segs[i].d, 1e-3, &t);
        if (k != ref_k[i] || (k >= 0 && std::memcmp(&t, &ref_t[i], sizeof t) != 0)) mism++;
    }
    std::printf("{\"segments_per_launch\": %u, \"recorded_segments\": %u, \"recorded_paths\": %u, \"samples\": %zu, \"refetch_k\": %d, \"variants_bit_identical\": %s, "
                "\"host_scan_checked\": %u, \"host_scan_mismatches\": %u, \"results\": [",
                sg.total, ns, n_paths, n_samples, rtk::kRefetchK, all_equal ? "true" : "false", checked, mism);
    for (size_t i = 0; i < res.size(); i++)
        std::printf("%s{\"variant\": \"%s\", \"block\": %d, \"blocks_per_cu\": %u, \"waves_per_simd\": %d, "
                    "\"stack_entry_bytes\": %d, \"ms\": %.4f, \"ns_per_segment\": %.4f}",
                    i ? ", " : "", res[i].name, res[i].block, res[i].resident_blocks_per_cu, res[i].waves_per_simd,
                    res[i].stack_bytes, res[i].ms, res[i].ns_per_seg);
    std::printf("]}\n");
    return (all_equal && mism == 0) ? 0 : 1;
}

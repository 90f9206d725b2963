// rt_kernel.h — device data layout shared by the kernels (rt_kernel.hip) and the host runtime.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_fastdiv.h"

namespace rtk {

constexpr int kBlock = 256;                // 4 waves of 64 lanes
constexpr uint32_t kMaxLdsSpheres = 2048;  // 64 KiB of LDS geometry; above this, read from global
#ifndef RTZIG_CHUNK
#define RTZIG_CHUNK 2048
#endif
constexpr uint32_t kChunk = RTZIG_CHUNK;          // work items a wave claims per queue fetch (at most: guided_chunk)
#ifndef RTZIG_QUEUE_HOME
#define RTZIG_QUEUE_HOME 0  // 1: segment (block / kQueues) % kQueues (A/B knob)
#endif
#ifndef RTZIG_QUEUES
#define RTZIG_QUEUES 8
#endif
// Work-queue counters: the items of a launch are split into kQueues contiguous segments, one
// counter each (kQueueStride u64 apart, separate 256-B lines); a wave claims from the segment of
// its block (blockIdx % kQueues) and moves on to the next segments once that one is exhausted.
// One counter serves ~88 claims per µs; 8 of them let the claims shrink to 64 items at the end of a
// launch (A/B, profiles/r01_chunk: chapter 9 -8%, rank 0's N = 8 rows -1%, final frame -0.5%).
constexpr uint32_t kQueues = RTZIG_QUEUES;
constexpr uint32_t kQueueStride = 32;
constexpr size_t kQueueBytes = (size_t)kQueues * kQueueStride * sizeof(unsigned long long);
constexpr size_t kQueueBufferBytes = 4096;  // allocated by rt_runtime.cpp
static_assert(kQueues >= 1 && kQueueBytes <= kQueueBufferBytes, "queue counters exceed the queue buffer");
// Wave-uniform claim state of the segmented work queue (path_loop, path_loop_fast).  claim()
// fetches a new window [cur, end) of item numbers: a guided claim from the wave's current segment,
// sized from an estimate of that segment's position (this wave's previous claim plus one such claim
// by every other wave of the segment since, rtk::guided_chunk); an exhausted segment sends the wave
// on to the next one, where it claims RTZIG_MIN_CHUNK items at a time.  After kQueues failed claims
// (one per segment) it returns false for good, so every wave reaches the drained state.
struct WorkQueue {
    uint64_t total, seg_waves;
    uint64_t cur = 0, end = 0, qend = 0, last_chunk = 0;
    uint32_t qcur, qmoves = 0;
    __device__ WorkQueue(uint64_t total_, uint64_t nwaves, uint32_t block)
        : total(total_), seg_waves(nwaves / kQueues > 0 ? nwaves / kQueues : 1),
          qcur(kQueues == 1 ? 0 : (RTZIG_QUEUE_HOME ? block / kQueues : block) % kQueues) {}
    __device__ __forceinline__ bool claim(unsigned long long* __restrict__ queue, uint32_t lane) {
        while (qmoves < kQueues) {
            const uint32_t q = qcur;
            const uint64_t s0 = kQueues == 1 ? 0 : total * q / kQueues;
            const uint64_t s1 = kQueues == 1 ? total : total * (q + 1) / kQueues;
            const uint64_t chunk = qmoves == 0 ? guided_chunk(s1 - s0, qend + seg_waves * last_chunk, seg_waves, kChunk)
                                               : (uint64_t)RTZIG_MIN_CHUNK;
            last_chunk = chunk;
            unsigned long long base = 0;
            if (lane == 0) base = atomicAdd(queue + (size_t)q * kQueueStride, (unsigned long long)chunk);
            base = __shfl(base, 0, 64);
            if (base < s1 - s0) {
                qend = base + chunk < s1 - s0 ? base + chunk : s1 - s0;
                cur = s0 + base;
                end = s0 + qend;
                return true;
            }
            ++qmoves;
            qcur = qcur + 1 == kQueues ? 0 : qcur + 1;
        }
        return false;
    }
};

constexpr uint32_t kPad = 4;               // sphere list padded to a multiple of this (sentinels)
#ifndef RTZIG_RUV_TRIPS
#define RTZIG_RUV_TRIPS 3
#endif
#ifndef RTZIG_TRIP_DEFER
#define RTZIG_TRIP_DEFER 0  // >0: skip trips 2.. when at most this many lanes still need a draw
#endif
constexpr int kRuvTrips = RTZIG_RUV_TRIPS;  // randomUnitVec rejection trips per loop iteration (path_loop)
constexpr const char* kDefaultVariant = "smem_u4";  // see variant_choice() in rt_kernel.hip

// Geometry walked by every lane for every ray: 32 B, one LDS broadcast pair per sphere.
// Padding entries are sentinels {0, 0, 0, -inf}: c = |oc|^2 + inf = +inf, so disc = -inf (or NaN
// for a zero direction) and the sentinel never passes `disc >= 0`.
struct alignas(32) GeoRec {
    double cx, cy, cz;  // Sphere.center
    double r2;          // radius * radius (hoisted from sphere.zig:30; same bits)
};

// Material + shading constants, read only for the winning sphere.
struct alignas(16) MatRec {
    double albedo[3];
    double fuzz;
    double ior;
    double inv_r;   // 1.0 / radius, as Vec.divScalar computes it (vec.zig:44, sphere.zig:45)
    // Dielectric constants, computed on the host with the device's IEEE operations (same bits):
    double inv_ior;   // 1.0 / ior: ri of a front-face hit (material.zig:86)
    double r0_front;  // Schlick r0 = ((1 - ri) / (1 + ri))^2 for ri = inv_ior (material.zig:106-108)
    double r0_back;   // ... for ri = ior
    uint32_t kind;  // 0 lambertian, 1 metal, 2 dielectric
    uint32_t pad;
};

// Arguments of the sample kernel (by value).  One launch renders the samples
// [s_begin, s_begin + s_count) of the rows j = row0 + k*row_step, k < n_rows.
// Work item t in [0, s_count * n_rows * W): sample s_begin + t / P of local pixel q = t % P
// (P = n_rows * W); its color goes to samples[3*t .. 3*t+2].
struct KernelParams {
    uint32_t width, height, spp, bounce_max;
    double scale;  // pixelSamplesScale
    double center[3], pixel0[3], du[3], dv[3], ddu[3], ddv[3];
    double defocus_angle, t_min, t_max;
    uint64_t seed_mix;  // sm_mix(seed), hoisted from sample_key
    uint32_t row0, row_step, n_rows, n_spheres;
    uint32_t n_pad;  // n_spheres rounded up to kPad (sentinel-padded)
    uint32_t s_begin, s_count;
    uint32_t prof;   // 1: instrumented build, stats has 8 entries (see rt_context_enable_profile)
    uint32_t order;  // work-item order: 0 sample-major, 1 pixel-major, 2 sample-major over 8x8 tiles (RTZIG_ORDER)
    uint32_t pad2;
    FastDiv div_layer;  // / (n_rows * width): item -> (sample, pixel) in the refill
    FastDiv div_width;  // / width: pixel -> (row, column)
    // f32 copies of the camera constants for the fast (RT_PRECISION_F32) kernel, read by scalar
    // loads at use: center, pixel0, du, dv, defocusDiskU, defocusDiskV (3 each), defocus_angle
    float fcam[20];
};

// BVH (rt_bvh.hpp).  Node = both child boxes (f32, padded outward) + child refs; on the device a
// ref >= 0 is the BYTE offset of a node, ref < 0 is ~(byte offset of a leaf block).
// Each axis of each child box is stored as {lo, hi, hi, lo}: a lane reads the 8-B pair at +0
// (lo, hi) when its ray direction on that axis is >= 0 and at +8 (hi, lo) when it is < 0, so one
// ds_read_b64 delivers (near plane, far plane) in ray order and the slab test needs no per-axis
// min/max (rt_kernel.hip, BvhWalker).  Node stride 104 B = 26 dwords: consecutive nodes start
// on 32 different banks of the 64 (gcd(26, 64) = 2), so per-lane random ds_read_b64 gathers
// spread over the whole bank row.  Leaves (2 slots: 80 B = 5 x 16, read as ds_read_b128) start
// at the next 16-B boundary after the nodes.
constexpr int kBlockBvh = 512;     // 8 waves; 2 blocks per CU share the LDS budget
constexpr int kMaxDepthBvh = 16;   // == rtbvh::kMaxDepth: bound on per-lane LDS stack entries (entry 0: "done")
#ifndef RTZIG_LEAF
#define RTZIG_LEAF 2
#endif
#ifndef RTZIG_LEAF_FILTER
#define RTZIG_LEAF_FILTER 1  // 0: every slot with disc >= 0; 1: drop spheres behind; 2: also beyond closest
#endif
constexpr int kLeafBvh = RTZIG_LEAF;       // == rtbvh::kLeafMax: slots per (sentinel-padded) leaf
struct alignas(8) BvhNode {
    float c0[3][4];   // child 0: per axis {lo, hi, hi, lo}
    float c1[3][4];   // child 1
    int32_t ref0, ref1;
};  // 104 B
struct alignas(16) LeafGeo {
    double cx, cy, cz, r2;    // as GeoRec, 16-B aligned so that a 2-slot leaf packs to 80 B
};
struct alignas(16) BvhLeaf {
    LeafGeo g[kLeafBvh];      // slot geometry (sentinels: {0,0,0,-inf})
    uint32_t sid[kLeafBvh];   // original sphere index per slot (0xffffffff for sentinels)
};  // 80 B for 2 slots (RTZIG_LEAF=4: 144 B)
static_assert(sizeof(BvhNode) == 104 && sizeof(BvhLeaf) % 32 == 16, "BVH node / leaf strides (bank spread)");
struct BvhArgs {
    const BvhNode* nodes;
    const BvhLeaf* leaves;
    const GeoRec* always_geo;    // spheres tested for every ray (unboundable)
    const uint32_t* always_sid;
    uint32_t n_nodes, n_leaves, n_always;
    uint32_t stack_depth;  // per-lane stack entries the tree needs: its depth (root = 1), <= kMaxDepthBvh
};
// LDS layout of the BVH kernel: [nodes, padded to 16 B][leaves][stacks: stack_depth x kBlockBvh x 4 B]
__host__ __device__ inline uint32_t bvh_leaves_offset(uint32_t n_nodes) {
    return (n_nodes * (uint32_t)sizeof(BvhNode) + 15u) & ~15u;
}

// Arguments of the ordered reduction: pixel q's running sum += samples[s][q] for s = 0..s_count-1
// (exactly the reference's sequential `pixelColor += rayColor(ray)`, camera.zig:133-136).
struct ReduceParams {
    uint32_t n_pixels, s_count;
    uint32_t first, last;   // first chunk starts from 0; last chunk scales and writes the output
    uint32_t out_format;    // 0 linear f64 (3 doubles per pixel), 1 rgb8
    uint32_t pad;
    double scale;
};

}  // namespace rtk

// Launch wrappers (rt_kernel.hip); all asynchronous on `stream`.
extern "C" hipError_t rtk_launch_samples(const rtk::KernelParams* p, const rtk::GeoRec* geo,
                                         const rtk::MatRec* mat, double* samples, void* queue,
                                         void* stats, hipStream_t stream, const char** name);
extern "C" hipError_t rtk_launch_samples_bvh(const rtk::KernelParams* p, const rtk::BvhArgs* b,
                                             const rtk::GeoRec* geo, const rtk::MatRec* mat, double* samples,
                                             void* queue, void* stats, hipStream_t stream, const char** name);
extern "C" hipError_t rtk_launch_reduce(const rtk::ReduceParams* p, const double* samples,
                                        double* sums, void* out, hipStream_t stream);
// Fast mode (rt_kernel_fast.hip): the same persistent path loop and BVH in f32 arithmetic, with
// the always-list (huge / unboundable) spheres tested in f64.  Statistical parity only.
extern "C" hipError_t rtk_launch_samples_fast(const rtk::KernelParams* p, const rtk::BvhArgs* b, const rtk::GeoRec* geo,
                                              const rtk::MatRec* mat, double* samples, void* queue, void* stats,
                                              hipStream_t stream, const char** name);
// Resident blocks of `kernel` on the current device (CUs x occupancy), cached (rt_kernel.hip).
extern "C" hipError_t rtk_resident_blocks(const void* kernel, int block, size_t shmem, uint32_t* blocks);

// rt_kernel.h — device data layout shared by the kernels (rt_kernel.hip) and the host runtime.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_fastdiv.h"

namespace rtk {

constexpr int kBlock = 256;                // 4 waves of 64 lanes
constexpr uint32_t kMaxLdsSpheres = 2048;  // 64 KiB of LDS geometry; above this, read from global
// ------------------------------------------------------------------------------------------------
// Work units and the ordered in-kernel accumulation.
//
// The reference sums a pixel's samples strictly in sample order (camera.zig:133-136:
// pixelColor += rayColor(ray), then * pixelSamplesScale at :137), so the f64 result depends on that
// order.  A work UNIT is (tile, chunk): the 64 consecutive pixels q = 64 * tile + l (l = 0..63) of
// the launch's rows x the samples [s0, s0 + S) of chunk k.  Units are claimed from one counter in
// chunk-major order (all tiles' chunk 0, then chunk 1, ...), so the 64 lanes of a wave trace
// neighbouring pixels.  A wave holds up to kSlots units at once and hands their S x 64 items to its
// lanes in sample-major order (item m: sample s0 + m / 64 of pixel 64 * tile + m % 64); a lane whose
// path ends stores its color into the unit's slot of the wave's private ring [slot][m][3] and takes
// the next item.  When every item of a unit has ended, the wave FINALISES it: lane l adds the ring's
// S colors of pixel l, in sample order, to the pixel's running sum — after the unit of the previous
// chunk of the same tile has been finalised (per-tile flag) — and writes the sum back (write-through
// sc1 stores, drained, then the flag: MI355X hand-off recipe, any XCD), or, for the last chunk,
// writes the framebuffer (scale + optional Color.toRgb).  No per-sample buffer and no reduce pass.
// Chunks: kUnitS samples each, shrinking towards the end of the launch (rt_schedule.hpp).
//
// DIRECT mode, for small launches (P x spp x 24 B within kDirectBytes: a rank's rows of a
// multi-GPU job, the short book scenes): the items are numbered flat and sample-major,
// t = s * P + q, and split into kSegs contiguous queue segments with a counter each; a wave claims a
// run from its home segment with one atomic (guided: 1/8 of an even share of what the segment has
// left, 64 to 2048 items), then from the other segments 64 at a time; a lane stores its color at
// samples[t], and nothing waits on anything; reduce_kernel then adds every pixel's stored colors
// in sample order.  Small launches have few
// tiles: (tile, chunk) units would either be large (a long drain) or so many that the claim
// counter's rate (≈88 claims per µs) bounds the launch.
// ------------------------------------------------------------------------------------------------
#ifndef RTZIG_UNIT_S
#define RTZIG_UNIT_S 48
#endif
#ifndef RTZIG_SLOTS
#define RTZIG_SLOTS 2
#endif
constexpr uint32_t kUnitS = RTZIG_UNIT_S;  // samples per unit of the main chunks (ring slot size)
constexpr uint32_t kSlots = RTZIG_SLOTS;   // units a wave holds at once (48 x 2 measured best)
constexpr uint32_t kSlotMask = (1u << kSlots) - 1;
constexpr uint32_t kRingSlotDoubles = kUnitS * 64 * 3;
constexpr uint32_t kRingWaveDoubles = kSlots * kRingSlotDoubles;  // 144 KiB of f64 per wave
// counters: ring mode's claim counter ctr[0]; direct mode one per queue segment, each on its own
// 128-B line, ctr[kCtrStride * seg] — zeroed per launch (the first kCtrLaunchBytes) — then the
// STICKY error word ctr[kErrWord]: set by a wave that gave up waiting (rt_units.h), cleared only by
// the host after it has reported it (rt_context_sync / rt_render), so a failure in any frame of a
// run is seen.
constexpr uint32_t kSegs = 8;
constexpr uint32_t kCtrStride = 16;
constexpr uint32_t kErrWord = kSegs * kCtrStride;
constexpr unsigned long long kErrStall = 1;   // error-word bits: a hand-off wait gave up (rt_units.h)
constexpr unsigned long long kErrBounds = 2;  // ... an index out of range (RTZIG_BOUNDS debug builds)
constexpr size_t kCtrLaunchBytes = (size_t)kErrWord * sizeof(unsigned long long);
constexpr size_t kCtrBytes = (kErrWord + kCtrStride) * sizeof(unsigned long long);
// bound on one hand-off wait (rt_units.h wait_clock): units of 256 ticks of the 100 MHz clock
constexpr double kStallUnitUs = 2.56;
constexpr uint32_t kStallUnitsPerSec = 390625;  // 1 s / 2.56 µs
constexpr uint32_t kStallBaseSec = 40;          // default bound; list walks scale it (rt_runtime.cpp)
constexpr uint32_t kStallMaxSec = 10000;        // < 2^32 units
constexpr uint64_t kDirectBytes = 2ull << 30;  // direct mode when P x spp x 24 B fits

// Deferred reduce pass (rt_render_rows_async_deferred): the previous direct-mode call's stored
// samples, folded by this launch's waves once the item queue has run dry (the launch's tail, where
// CUs otherwise idle behind a few long paths); chunks of 64 pixels claimed from `ctr` (zeroed before
// the launch); a follow-up pass (fold_rest_kernel) takes the chunks left unclaimed.
struct FoldArgs {
    const double* samples;     // [spp][P][3]; nullptr: nothing to fold
    void* out;                 // [P][3] f64 linear or u8 RGB
    unsigned long long* ctr;   // chunk claim counter
    uint32_t P, spp, format, n_chunks;
    double scale;
};

struct UnitArgs {
    double* ring;              // [waves][kSlots][kUnitS * 64][3] wave-private sample colors
    double* sums;              // [P][3] running per-pixel sums (write-through hand-off between waves)
    uint32_t* flags;           // [n_tiles] chunks finalised per tile (zeroed per launch)
    void* out;                 // [P][3] f64 linear or u8 RGB (the last chunk's finalisation)
    unsigned long long* ctr;   // kCtrBytes: claim counters, [kErrWord] error word
    FastDiv div_tiles;         // u -> (chunk, tile)
    const uint32_t* chunk_s0;  // [n_chunks + 1]: chunk k covers samples [chunk_s0[k], chunk_s0[k + 1])
    double* samples;           // direct mode: [spp][P][3] every sample's color (reduce_kernel sums them)
    FastDiv div_p;             // direct mode: / P, item t -> (sample, pixel)
    uint32_t n_tiles, n_units; // n_units = n_tiles * n_chunks < 2^32 (direct mode: the P * spp items)
    uint32_t n_chunks, spp;
    uint32_t P, out_format;    // pixels of the launch; 0 linear f64, 1 rgb8
    uint32_t ring_waves;       // ring capacity in waves (the launch never has more)
    uint32_t stall_ticks;      // bound on one continuous hand-off wait, wait_clock units (2.56 µs, rt_units.h)
    double scale;              // pixelSamplesScale
    FoldArgs fold;             // direct mode: a previous call's samples to fold in the tail (may be empty)
};

// samples [*s0, *s0 + *n) of chunk k (the table is read-only: scalar loads)
__device__ __forceinline__ void chunk_range(const UnitArgs& u, uint32_t k, uint32_t* s0, uint32_t* n) {
    const uint32_t a = u.chunk_s0[k], b = u.chunk_s0[k + 1];
    *s0 = a;
    *n = b - a;
}

constexpr uint32_t kPad = 4;               // sphere list padded to a multiple of this (sentinels)
#ifndef RTZIG_RUV_TRIPS
#define RTZIG_RUV_TRIPS 3
#endif
constexpr int kRuvTrips = RTZIG_RUV_TRIPS;  // randomUnitVec rejection trips per loop iteration (path_loop; 2, 4 slower)
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

// Arguments of the sample kernel (by value).  One launch renders every sample of the rows
// j = row0 + k*row_step, k < n_rows (P = n_rows * W launch-local pixels q, row k = q / W); the
// work decomposition (units or direct items) is UnitArgs's.
struct KernelParams {
    uint32_t width, height, spp, bounce_max;
    double scale;  // pixelSamplesScale
    double center[3], pixel0[3], du[3], dv[3], ddu[3], ddv[3];
    double defocus_angle, t_min, t_max;
    uint64_t seed_mix;  // sm_mix(seed), hoisted from sample_key
    uint32_t row0, row_step, n_rows, n_spheres;
    uint32_t n_pad;  // n_spheres rounded up to kPad (sentinel-padded)
    uint32_t s_begin, s_count;  // unused by the unit scheduler (kept for the kernarg layout)
    uint32_t prof;   // 1: instrumented build, stats holds RT_PROFILE_STATS_WORDS entries (rt.h)
    uint32_t pad2[2];
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
#ifndef RTZIG_BVH_BLOCK
#define RTZIG_BVH_BLOCK 1024
#endif
#ifndef RTZIG_STACK16
#define RTZIG_STACK16 0
#endif
constexpr int kBlockBvh = RTZIG_BVH_BLOCK;  // threads of the BVH kernels' blocks (build knob)
// per-lane stack entry of the BVH walk (build knob: int16 holds every ref of a tree whose nodes and
// leaves each span < 32 KiB, rt_kernel.hip StackOps)
#if RTZIG_STACK16
typedef int16_t StackEntry;
#else
typedef int32_t StackEntry;
#endif
// Seed window (RTZIG_SEED_WIN): a wave seeds the generators and pixel sample points
// of 64 items at once, all lanes busy, into an LDS window its fresh lanes then read — instead of each
// fresh lane seeding its own (≈21 of 64 lanes active).  Per wave: 14 dword planes of 64 lanes
// (Xoshiro s0..s3 after sampleSquare's two draws, the pixel sample point): 3.5 KiB.
#ifndef RTZIG_SEED_WIN
#define RTZIG_SEED_WIN 1
#endif
constexpr bool kSeedWin = RTZIG_SEED_WIN != 0;
constexpr uint32_t kSeedWinPlanes = 14;
constexpr uint32_t kSeedWinBytes = kSeedWinPlanes * 64 * 4 + 16;  // + the window's key (16-B aligned)
// LDS of one block: its share of a CU's 160 KiB at 16 waves per CU (2 blocks of 512 threads, or one
// of 1024), less its waves' seed windows; the rest holds the tree + stacks when they fit
constexpr size_t kLdsBlockShare = (size_t)160 * 1024 * (size_t)kBlockBvh / 1024;
constexpr size_t kSeedWinBlockBytes = kSeedWin ? (size_t)(kBlockBvh / 64) * kSeedWinBytes : 0;
constexpr size_t kLdsSceneBudget = kLdsBlockShare - kSeedWinBlockBytes;  // tree + stacks of one block
// The instrumented BVH kernels (kProf) run 512-thread blocks whatever kBlockBvh is: their counters
// need more than the 128 VGPRs a 1024-thread block allows (4 waves per SIMD) and would spill to
// scratch; at 512 threads they keep 3 waves per SIMD.  Their LDS budget is a whole CU's, less their
// seed windows (one block per CU when the tree is in LDS).
constexpr int kBlockBvhProf = 512;
constexpr size_t kSeedWinProfBytes = kSeedWin ? (size_t)(kBlockBvhProf / 64) * kSeedWinBytes : 0;
constexpr size_t kLdsSceneBudgetProf = (size_t)160 * 1024 - kSeedWinProfBytes;
__host__ __device__ constexpr int bvh_block(bool prof) { return prof ? kBlockBvhProf : kBlockBvh; }
constexpr int kMaxDepthBvh = 16;   // == rtbvh::kMaxDepth: bound on per-lane LDS stack entries (entry 0: "done")
#ifndef RTZIG_LEAF
#define RTZIG_LEAF 2
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
    // The f32 box padding covers ray origins with max|o_i| <= the builder's origin bound; this is
    // that bound rounded down to f32.  A lane whose f32 origin lies beyond it (a secondary ray
    // leaving an unboundable always-list sphere far out) skips the tree and walks the whole list.
    float origin_bound;
    uint32_t pad;
};
// LDS layout of the BVH kernel: [nodes, padded to 16 B][leaves][stacks: stack_depth x kBlockBvh x sizeof(StackEntry)]
__host__ __device__ inline uint32_t bvh_leaves_offset(uint32_t n_nodes) {
    return (n_nodes * (uint32_t)sizeof(BvhNode) + 15u) & ~15u;
}

}  // namespace rtk

// Launch wrappers (rt_kernel.hip); asynchronous on `stream`.  The caller zeroes ua->ctr
// (kCtrLaunchBytes) and ua->flags (n_tiles x 4 B) before every launch.  `direct`: direct mode
// (ua->samples set).  With plan_waves != nullptr nothing is launched: *plan_waves receives the waves
// of the persistent grid the launch would run (resident capacity of the chosen kernel, or fewer for a
// small launch), before the ring's bound — the runtime sizes the ring to it (ua may be null then).
// Direct mode's second pass: per pixel, the stored colors added in sample order, scaled, written.
extern "C" hipError_t rtk_launch_reduce(const rtk::UnitArgs* ua, hipStream_t stream);
extern "C" hipError_t rtk_launch_fold_rest(const rtk::FoldArgs* f, hipStream_t stream);
extern "C" hipError_t rtk_launch_samples(const rtk::KernelParams* p, const rtk::GeoRec* geo,
                                         const rtk::MatRec* mat, const rtk::UnitArgs* ua,
                                         void* stats, hipStream_t stream, const char** name, bool direct,
                                         uint32_t* plan_waves);
extern "C" hipError_t rtk_launch_samples_bvh(const rtk::KernelParams* p, const rtk::BvhArgs* b,
                                             const rtk::GeoRec* geo, const rtk::MatRec* mat, const rtk::UnitArgs* ua,
                                             void* stats, hipStream_t stream, const char** name, bool direct,
                                             uint32_t* plan_waves);
// Fast mode: the same persistent path loop and BVH walk instantiated in f32 arithmetic, with
// the always-list (huge / unboundable) spheres tested in f64.  Statistical parity only.
extern "C" hipError_t rtk_launch_samples_fast(const rtk::KernelParams* p, const rtk::BvhArgs* b, const rtk::GeoRec* geo,
                                              const rtk::MatRec* mat, const rtk::UnitArgs* ua, void* stats,
                                              hipStream_t stream, const char** name, bool direct,
                                              uint32_t* plan_waves);
// Resident blocks of `kernel` on the current device (CUs x occupancy), cached (rt_kernel.hip).
extern "C" hipError_t rtk_resident_blocks(const void* kernel, int block, size_t shmem, uint32_t* blocks);

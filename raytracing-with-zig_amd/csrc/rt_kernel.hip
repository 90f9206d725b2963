// rt_kernel.hip — the per-pixel x per-sample hot path on gfx950 (CDNA4).
//
// Replaces the loop nest of Camera.render (reference src/camera.zig:123-145):
//   for j, for i, for s: getRay (camera.zig:187-215) -> rayColor (camera.zig:148-183)
//     -> HittableList.hit (hittable.zig:64-77) -> Sphere.hit (sphere.zig:26-54)
//     -> Material.scatter (material.zig:145-151)
//
// One persistent launch per frame, plus a reduce pass in direct mode:
//
// sample_kernel_bvh (parity, default), sample_kernel (the reference's linear list walk, tiny scenes)
//   and sample_kernel_fast (RT_PRECISION_F32) all run path_loop below: persistent waves take work
//   items (one item = one sample of one pixel) from the unit scheduler of rt_units.h; every lane
//   traces one ray segment per loop iteration (rayColor's loop body), and a lane whose path ends
//   (miss / absorb / bounceMax) stores the sample's colour and takes the next item, so no lane idles
//   behind a long glass path and no CU idles behind a slow block.  Ring mode (large launches)
//   accumulates each pixel's samples in sample order inside the kernel (wave rings + running sums
//   handed from wave to wave); direct mode (small launches) stores every sample for the reduce pass.
//   The closest hit is HittableList.hit's first-wins argmin, found by a BVH walk over an LDS-resident
//   tree (BvhWalker) or the reference's list walk (LinearWalker) with the same f64 quadratic.  New
//   items are seeded 64 at a time by the whole wave into an LDS seed window (kSeedWin, path_loop).
//
// reduce_kernel — direct mode only: per pixel, adds the stored sample colours in sample order
//   (camera.zig:135 `pixelColor += rayColor(ray)`, the same sequence of roundings as the reference's
//   loop), then scales by pixelSamplesScale (camera.zig:137) and writes linear f64 or the fused
//   Color.toRgb bytes (color.zig:63-80).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstddef>
#include <cstdlib>
#include <climits>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>

#include "rt_device.h"
#include "rt_kernel.h"
#include "rt_units.h"

#pragma clang fp contract(off)

namespace rtk {

struct Ray {
    v3 orig, dir;
};

// The camera constants of getRay (center, pixel0, du, dv, defocusDiskU/V, defocusAngle: 38
// dwords of KernelParams) are read from the kernarg segment by scalar loads at each use instead of
// being held in SGPRs for the whole persistent loop: held, they pushed the kernel past 102 SGPRs
// and the compiler spilled uniform values to VGPR lanes, reloading them with ~50 v_readlane (VALU)
// per loop iteration.  The asm is volatile so the loads stay where they are used.
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
static_assert(offsetof(KernelParams, center) == 24 && offsetof(KernelParams, pixel0) == 48 &&
                  offsetof(KernelParams, du) == 72 && offsetof(KernelParams, dv) == 96 &&
                  offsetof(KernelParams, ddu) == 120 && offsetof(KernelParams, ddv) == 144 &&
                  offsetof(KernelParams, defocus_angle) == 168,
              "camera constants: kernarg offsets used by camera_start / camera_finish");
__device__ __forceinline__ double dw2d(uint32_t lo, uint32_t hi) {
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// getRay (camera.zig:187-200) in two parts around the defocus disk's rejection loop.
// camera_start: sampleSquare (:203-209) and the pixel sample point.  Without defocus the ray is
// complete; with defocus r.orig holds the camera center and r.dir the pixel sample point until
// camera_finish adds the disk sample (defocusDiskSample, :212-215) drawn by path_loop's trip loop.
// Camera constants are read from the kernarg segment by scalar loads at each use (KernelParams
// must be the kernel's first argument).
__device__ __forceinline__ bool camera_start(uint32_t i, uint32_t j, Rng& g, Ray& r) {
    u32x16 A;  // dwords 6..21 of KernelParams: center, pixel0, du.x, du.y
    u32x8 B;   // dwords 22..29: du.z, dv
    u32x2 C;   // dwords 42..43: defocus_angle
    const uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile(
        "s_load_dwordx16 %0, %3, 24\n\t"
        "s_load_dwordx8 %1, %3, 88\n\t"
        "s_load_dwordx2 %2, %3, 168\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=s"(A), "=s"(B), "=s"(C)
        : "s"(kp));
    const v3 center = mk(dw2d(A[0], A[1]), dw2d(A[2], A[3]), dw2d(A[4], A[5]));
    const v3 p0 = mk(dw2d(A[6], A[7]), dw2d(A[8], A[9]), dw2d(A[10], A[11]));
    const v3 du = mk(dw2d(A[12], A[13]), dw2d(A[14], A[15]), dw2d(B[0], B[1]));
    const v3 dv = mk(dw2d(B[2], B[3]), dw2d(B[4], B[5]), dw2d(B[6], B[7]));
    const double defocus_angle = dw2d(C[0], C[1]);
    const double ox = g.uniform() - 0.5;
    const double oy = g.uniform() - 0.5;
    const v3 ps = (p0 + muls(du, (double)i + ox)) + muls(dv, (double)j + oy);
    r.orig = center;
    if (defocus_angle <= 0) {
        r.dir = ps - center;
        return false;
    }
    r.dir = ps;
    return true;  // the disk sample is pending
}
// The seed window's half of camera_start: sampleSquare's draws and the pixel sample point
// (camera.zig:190-193, 203-209), the same operations as above.
__device__ __forceinline__ v3 pixel_sample_point(uint32_t i, uint32_t j, Rng& g) {
    u32x16 A;  // dwords 12..27 of KernelParams: pixel0, du, dv.x, dv.y
    u32x2 B;   // dwords 28..29: dv.z
    const uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile(
        "s_load_dwordx16 %0, %2, 48\n\t"
        "s_load_dwordx2 %1, %2, 112\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=s"(A), "=s"(B)
        : "s"(kp));
    const v3 p0 = mk(dw2d(A[0], A[1]), dw2d(A[2], A[3]), dw2d(A[4], A[5]));
    const v3 du = mk(dw2d(A[6], A[7]), dw2d(A[8], A[9]), dw2d(A[10], A[11]));
    const v3 dv = mk(dw2d(A[12], A[13]), dw2d(A[14], A[15]), dw2d(B[0], B[1]));
    const double ox = g.uniform() - 0.5;
    const double oy = g.uniform() - 0.5;
    return (p0 + muls(du, (double)i + ox)) + muls(dv, (double)j + oy);
}
// ... and the rest of camera_start: the ray's direction from the camera center (with defocus, the
// sample point itself, until camera_finish adds the disk sample) and whether the disk sample is
// pending; the window stores the direction, a fresh lane takes the origin
__device__ __forceinline__ v3 camera_center(bool& defocus) {
    u32x8 A;  // dwords 6..13: center (+2 unused)
    u32x2 C;  // dwords 42..43: defocus_angle
    const uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile(
        "s_load_dwordx8 %0, %2, 24\n\t"
        "s_load_dwordx2 %1, %2, 168\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=s"(A), "=s"(C)
        : "s"(kp));
    defocus = !(dw2d(C[0], C[1]) <= 0);
    return mk(dw2d(A[0], A[1]), dw2d(A[2], A[3]), dw2d(A[4], A[5]));
}
// rayOrigin = defocusDiskSample() = (center + defocusDiskU * p.x) + defocusDiskV * p.y;
// rayDirection = pixelSample - rayOrigin
__device__ __forceinline__ void camera_finish(double px, double py, Ray& r) {
    u32x8 A;   // dwords 6..13: center (+2 unused)
    u32x16 B;  // dwords 30..45: defocusDiskU, defocusDiskV (+4 unused)
    const uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile(
        "s_load_dwordx8 %0, %2, 24\n\t"
        "s_load_dwordx16 %1, %2, 120\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=s"(A), "=s"(B)
        : "s"(kp));
    const v3 center = mk(dw2d(A[0], A[1]), dw2d(A[2], A[3]), dw2d(A[4], A[5]));
    const v3 ddu = mk(dw2d(B[0], B[1]), dw2d(B[2], B[3]), dw2d(B[4], B[5]));
    const v3 ddv = mk(dw2d(B[6], B[7]), dw2d(B[8], B[9]), dw2d(B[10], B[11]));
    const v3 origin = (center + muls(ddu, px)) + muls(ddv, py);
    r.dir = r.dir - origin;
    r.orig = origin;
}

// ------------------------------------------------------------------------------------------------
// Fast mode (RT_PRECISION_F32, statistical parity only; DESIGN.md "Fast mode"): the same path loop,
// walk and scheduler instantiated with kF32 = true, shading, sampling and leaf tests in f32 with
// single-instruction v_rcp_f32 / v_rsq_f32 / v_sqrt_f32 and FMA allowed (the pragma in each helper).
// A uniform is 24 bits of the same per-(pixel, sample) Xoshiro256++ stream; paired draws take both
// 32-bit halves of one word.
// ------------------------------------------------------------------------------------------------
namespace fm {
struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ f3 neg(f3 a) { return f3{-a.x, -a.y, -a.z}; }
__device__ __forceinline__ f3 muls(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float dot(f3 a, f3 b) {
#pragma clang fp contract(fast)
    return a.x * b.x + a.y * b.y + a.z * b.z;
}
__device__ __forceinline__ float len_sq(f3 a) { return dot(a, a); }
__device__ __forceinline__ f3 unit(f3 a) { return muls(a, __builtin_amdgcn_rsqf(len_sq(a))); }
__device__ __forceinline__ f3 reflect(f3 v, f3 n) { return sub(v, muls(n, 2.0f * dot(v, n))); }
__device__ __forceinline__ f3 refract(f3 v, f3 n, float eta) {
#pragma clang fp contract(fast)
    const float cos_t = __builtin_fminf(-dot(v, n), 1.0f);
    const f3 r_perp = muls(add(v, muls(n, cos_t)), eta);
    return sub(r_perp, muls(n, __builtin_sqrtf(__builtin_fabsf(1.0f - len_sq(r_perp)))));
}
__device__ __forceinline__ bool near_zero(f3 v) { return v.x < 1e-8f && v.y < 1e-8f && v.z < 1e-8f; }  // vec.zig:26-29
__device__ __forceinline__ v3 to64(f3 a) { return v3{a.x, a.y, a.z}; }
// U[0, 1) from the top 24 bits of one Xoshiro256++ word (exact in f32); uniform2 takes two from one
// word (the top 24 bits of each 32-bit half), halving the generator work of paired draws
__device__ __forceinline__ float uniform(Rng& g) { return (float)(uint32_t)(g.next() >> 40) * 0x1p-24f; }
__device__ __forceinline__ void uniform2(Rng& g, float& a, float& b) {
    const uint64_t w = g.next();
    a = (float)(uint32_t)(w >> 40) * 0x1p-24f;
    b = (float)((uint32_t)w >> 8) * 0x1p-24f;
}
__device__ __forceinline__ float pm1(float u) { return __builtin_fmaf(2.0f, u, -1.0f); }
struct Ray {
    f3 orig, dir;
};
}  // namespace fm

// getRay (camera.zig:187-215) in f32 from KernelParams::fcam (kernarg scalar loads at use, like the
// f64 form below); the defocus disk sample is drawn by the trip loop as in parity mode
constexpr int kFcam = (int)offsetof(KernelParams, fcam);
static_assert(kFcam % 4 == 0, "fcam kernarg offset");
__device__ __forceinline__ float fw(uint32_t w) { return __builtin_bit_cast(float, w); }
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bool camera_start(uint32_t i, uint32_t j, Rng& g, fm::Ray& r) {
#pragma clang fp contract(fast)
    u32x16 A;  // fcam[0..15]
    u32x4 B;   // fcam[16..19]
    const uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile(
        "s_load_dwordx16 %0, %2, %3\n\t"
        "s_load_dwordx4 %1, %2, %4\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=s"(A), "=s"(B)
        : "s"(kp), "i"(kFcam), "i"(kFcam + 64));
    const fm::f3 center = fm::mk(fw(A[0]), fw(A[1]), fw(A[2]));
    const fm::f3 p0 = fm::mk(fw(A[3]), fw(A[4]), fw(A[5]));
    const fm::f3 du = fm::mk(fw(A[6]), fw(A[7]), fw(A[8]));
    const fm::f3 dv = fm::mk(fw(A[9]), fw(A[10]), fw(A[11]));
    const float defocus_angle = fw(B[2]);
    float ox, oy;
    fm::uniform2(g, ox, oy);
    ox -= 0.5f;
    oy -= 0.5f;
    const fm::f3 ps = fm::add(fm::add(p0, fm::muls(du, (float)i + ox)), fm::muls(dv, (float)j + oy));
    r.orig = center;
    if (defocus_angle <= 0) {
        r.dir = fm::sub(ps, center);
        return false;
    }
    r.dir = ps;
    return true;
}
// fast mode's camera center and defocus flag (fcam), for a fresh lane given its seed-window entry
__device__ __forceinline__ fm::f3 camera_center_f32(bool& defocus) {
    u32x4 B;  // fcam[16..19]
    u32x4 A;  // fcam[0..3]
    const uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile(
        "s_load_dwordx4 %0, %2, %3\n\t"
        "s_load_dwordx4 %1, %2, %4\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=s"(A), "=s"(B)
        : "s"(kp), "i"(kFcam), "i"(kFcam + 64));
    defocus = !(fw(B[2]) <= 0);
    return fm::mk(fw(A[0]), fw(A[1]), fw(A[2]));
}
__device__ __forceinline__ void camera_finish(float px, float py, fm::Ray& r) {
#pragma clang fp contract(fast)
    u32x16 A;
    u32x4 B;
    const uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile(
        "s_load_dwordx16 %0, %2, %3\n\t"
        "s_load_dwordx4 %1, %2, %4\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=s"(A), "=s"(B)
        : "s"(kp), "i"(kFcam), "i"(kFcam + 64));
    const fm::f3 center = fm::mk(fw(A[0]), fw(A[1]), fw(A[2]));
    const fm::f3 ddu = fm::mk(fw(A[12]), fw(A[13]), fw(A[14]));
    const fm::f3 ddv = fm::mk(fw(A[15]), fw(B[0]), fw(B[1]));
    const fm::f3 origin = fm::add(fm::add(center, fm::muls(ddu, px)), fm::muls(ddv, py));
    r.dir = fm::sub(r.dir, origin);
    r.orig = origin;
}

// HittableList.hit over Sphere.hit with the exact arithmetic of sphere.zig:27-41.
// Walks `n_pad` entries (the list padded to a multiple of kPad with never-hit sentinels, see
// GeoRec) U spheres at a time: the U discriminants are independent, so their f64 chains and LDS
// reads interleave; the hit tests then run in list order, so `closest` evolves exactly as in the
// reference.  Returns the winning sphere index (or -1); *t_hit = its root.
template <int U>
__device__ __forceinline__ int world_hit(const GeoRec* __restrict__ geo, uint32_t n_pad, const Ray& r,
                                         double t_min, double t_max, double* t_hit) {
    const double a = len_sq(r.dir);  // loop-invariant Vec.lenSquared(ray.dir)
    double closest = t_max;
    int best = -1;
    for (uint32_t k = 0; k < n_pad; k += U) {
        double h[U], disc[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const GeoRec s = geo[k + u];
            const double ocx = s.cx - r.orig.x;
            const double ocy = s.cy - r.orig.y;
            const double ocz = s.cz - r.orig.z;
            h[u] = (r.dir.x * ocx + r.dir.y * ocy) + r.dir.z * ocz;
            const double c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - s.r2;
            disc[u] = h[u] * h[u] - a * c;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (disc[u] >= 0) {  // !(disc < 0); a NaN disc rejects either way
                const double sq = sqrt_g(disc[u]);
                double root = (h[u] - sq) / a;
                bool ok = t_min < root && root < closest;
                if (!ok) {
                    root = (h[u] + sq) / a;
                    ok = t_min < root && root < closest;
                }
                if (ok) {
                    closest = root;
                    best = (int)(k + u);
                }
            }
        }
    }
    *t_hit = closest;
    return best;
}

// x / l for several numerators x sharing one denominator l, bit-identical to the compiler's
// correctly rounded f64 division (v_div_scale, v_rcp_f64, two Newton steps, q0 = x*y,
// r = fma(-l, q0, x), v_div_fmas = fma(r, y, q0), v_div_fixup) whenever that sequence does not
// scale: the reciprocal part depends on l alone, so it is computed once.  Valid (no scaling, no
// fixup) for l in [2^-300, 1] and |x| in {0} U [2^-53, l]; Vec.randomUnitVec (vec.zig:71-80)
// guarantees both: |p|^2 in (1e-160, 1], so l in (1e-80, 1]; each component is -1 + 2u with u a
// Random.float(f64) (granularity <= 2^-54 below 0.5), so it is 0 or at least 2^-53 in magnitude,
// and |x| <= l.  x == 0 gives +0 both ways (fixup of 0 / l).
__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
// number of set bits of `mask` below this lane
__device__ __forceinline__ uint32_t rank_in(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// ------------------------------------------------------------------------------------------------
// Optional instrumentation (KernelParams::prof != 0 launches the kProf instantiation): executed
// sphere tests, BVH node visits and per-wave shader-clock cycles spent in refill / walk / shade.
// The counts are deterministic functions of the inputs; the cycles are diagnostics only.
// ------------------------------------------------------------------------------------------------
// kLevel 1: exact counts (sphere tests, node visits) and wave-level executions; kLevel 2 (the
// instrumented ring-mode kernel, round 6) adds lane-level counts: every lane that executes a block
// counts itself, so a block's lane count / its wave count is the mean number of active lanes (exec)
// its instructions run with.  Per-lane counters are 32-bit (a launch's per-lane counts stay far below
// 2^32).  The instrumented direct-mode kernel keeps level 1: the lane counters would cost it scratch.
template <int kLevel>
struct Prof {
    __device__ __forceinline__ void tests(uint32_t) {}
    __device__ __forceinline__ void visit() {}
    __device__ __forceinline__ void inner_iter() {}
    __device__ __forceinline__ void leaf_iter() {}
    template <int Q>
    __device__ __forceinline__ void cand_block() {}
    template <int Q>
    __device__ __forceinline__ void root2_block() {}
};
template <>
struct Prof<1> {
    uint32_t n_tests = 0, n_visits = 0;      // n_visits: lane-level inner steps
    uint32_t cam_visits = 0, cam_tests = 0;  // of camera rays (bounce 0)
    uint32_t w_inner = 0, w_leaf = 0;  // wave-level iterations (counted by the first active lane)
    uint32_t w_cand = 0, w_root2 = 0;  // wave-level candidate blocks (sqrt + root1 division) / root2 divisions
    __device__ __forceinline__ void tests(uint32_t n) { n_tests += n; }
    __device__ __forceinline__ void visit() { ++n_visits; }
    __device__ __forceinline__ static uint32_t leader() {
        const uint64_t m = __ballot(1);
        return (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) == 0 ? 1u : 0u;
    }
    __device__ __forceinline__ void inner_iter() { w_inner += leader(); }
    __device__ __forceinline__ void leaf_iter() { w_leaf += leader(); }
    template <int Q>
    __device__ __forceinline__ void cand_block() { w_cand += leader(); }
    template <int Q>
    __device__ __forceinline__ void root2_block() { w_root2 += leader(); }
};
template <>
struct Prof<2> : Prof<1> {
    uint32_t l_leaf = 0, l_cand = 0, l_root2 = 0;  // lane-level leaf rounds, candidate blocks, root2 divisions
    // the always-list's share: candidate blocks per always-list sphere q < 4 (wave / lane level), and
    // their second-root divisions
    uint32_t w_acand[4] = {0, 0, 0, 0}, l_acand[4] = {0, 0, 0, 0}, w_aroot2 = 0, l_aroot2 = 0;
    __device__ __forceinline__ void leaf_iter() {
        w_leaf += leader();
        ++l_leaf;
    }
    template <int Q>
    __device__ __forceinline__ void cand_block() {
        const uint32_t ld = leader();
        w_cand += ld;
        ++l_cand;
        if constexpr (Q >= 0 && Q < 4) {
            w_acand[Q] += ld;
            ++l_acand[Q];
        }
    }
    template <int Q>
    __device__ __forceinline__ void root2_block() {
        const uint32_t ld = leader();
        w_root2 += ld;
        ++l_root2;
        if constexpr (Q >= -1) {
            w_aroot2 += ld;
            ++l_aroot2;
        }
    }
};

// Region markers of the candidate block (RTZIG_MARKS builds, tools/region_table.py): Q = 0..3 the
// unrolled always-list spheres, -1 the always-list loop (more than 4), -2 a leaf round.
template <int Q>
__device__ __forceinline__ void mark_cand() {
    if constexpr (Q == 0) RTK_MARK("acand0");
    else if constexpr (Q == 1) RTK_MARK("acand1");
    else if constexpr (Q == 2) RTK_MARK("acand2");
    else if constexpr (Q == 3) RTK_MARK("acand3");
    else if constexpr (Q == -1) RTK_MARK("acandN");
    else RTK_MARK("lcand");
}
template <int Q>
__device__ __forceinline__ void mark_root2() {
    if constexpr (Q >= 0) RTK_MARK("aroot2");
    else if constexpr (Q == -1) RTK_MARK("aroot2N");
    else RTK_MARK("lroot2");
}
template <int Q>
__device__ __forceinline__ void mark_caller() {
    if constexpr (Q >= -1) RTK_MARK("always");
    else RTK_MARK("leaf");
}

// ------------------------------------------------------------------------------------------------
// Closest-hit walkers.  Both return the ORIGINAL list index of the winning sphere (or -1) and its
// root in *t_hit, bit-identical to HittableList.hit.
// ------------------------------------------------------------------------------------------------

// The reference's linear walk over the whole list (hittable.zig:68-74).
template <int U>
struct LinearWalker {
    const GeoRec* __restrict__ geo;
    uint32_t n_pad;
    uint32_t n_real;
    static constexpr bool kCanSuspend = false;
    struct State {};
    template <class PR>
    __device__ __forceinline__ int operator()(const Ray& r, double t_min, double t_max, double* t, PR& pr) const {
        pr.tests(n_real);
        return world_hit<U>(geo, n_pad, r, t_min, t_max, t);
    }
    template <bool kSusp, class PR>
    __device__ __forceinline__ int run(const Ray& r, double t_min, double t_max, double* t, PR& pr, State&, bool,
                                       bool = true) const {
        return (*this)(r, t_min, t_max, t, pr);
    }
};

// Slab-interval ends: max(x, y, z, lower) and min(x, y, z, upper) as hardware v_max3/v_min3 +
// v_max/v_min.  With IEEE mode on (the default) these return the non-NaN operand for quiet NaNs —
// exactly fmaxf/fminf on every value this walk produces (arithmetic never yields signaling NaNs) —
// but written as builtins the compiler re-canonicalizes the loop-carried bounds every iteration.
#ifndef RTZIG_WALK_FORM
#define RTZIG_WALK_FORM 0
#endif
#if RTZIG_WALK_FORM == 4
__device__ __forceinline__ float slab_near(float x, float y, float z, float lower) {
    float t, r;
    asm("v_max_f32 %0, %1, %2" : "=v"(t) : "v"(z), "v"(lower));
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(t));
    return r;
}
__device__ __forceinline__ float slab_far(float x, float y, float z, float upper) {
    float t, r;
    asm("v_min_f32 %0, %1, %2" : "=v"(t) : "v"(z), "v"(upper));
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(t));
    return r;
}
#elif RTZIG_WALK_FORM >= 1
__device__ __forceinline__ float slab_near(float x, float y, float z, float lower) {
    return __builtin_fmaxf(__builtin_fmaxf(x, y), __builtin_fmaxf(z, lower));
}
__device__ __forceinline__ float slab_far(float x, float y, float z, float upper) {
    return __builtin_fminf(__builtin_fminf(x, y), __builtin_fminf(z, upper));
}
#else
__device__ __forceinline__ float slab_near(float x, float y, float z, float lower) {
    float t, r;
    asm volatile("v_max_f32 %0, %1, %2" : "=v"(t) : "v"(z), "v"(lower));
    asm volatile("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(t));
    return r;
}
__device__ __forceinline__ float slab_far(float x, float y, float z, float upper) {
    float t, r;
    asm volatile("v_min_f32 %0, %1, %2" : "=v"(t) : "v"(z), "v"(upper));
    asm volatile("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(t));
    return r;
}
#endif

// v_cndmask_b32 on a wave mask held in SGPRs: lanes whose bit of `m` is set get `t`, others `f`
__device__ __forceinline__ int32_t sel_mask(int32_t f, int32_t t, uint64_t m) {
    int32_t r;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
    return r;
}

// BVH walk (rt_bvh.hpp): per-lane, near-child-first, stack in LDS.  Every visited sphere runs the
// same f64 quadratic as the linear walk; the candidate root of sphere k is
//   t_k = root1 if t_min < root1, else root2 if t_min < root2   (sphere.zig:38-41),
// and it wins iff t_k < closest, or t_k == closest and k is lower (the linear scan's first-wins).
constexpr int32_t kDone = INT32_MIN;  // walk finished (stack entry 0)
// Dynamic fetch (RTZIG_REFETCH_K > 0): after a leaf round, once at least K lanes of the wave are
// free (walk over, or not walking), the walk returns kSuspended for the lanes still walking; they
// keep their walk state (BvhWalker::State, the stack stays in LDS) and resume in the next
// iteration, while the free lanes shade and start their next segment.
#ifndef RTZIG_REFETCH_K
#define RTZIG_REFETCH_K 52
#endif
constexpr int kRefetchK = RTZIG_REFETCH_K;
// Drain mode (RTZIG_DRAIN, default 0: an A/B knob, measured within noise and not adopted): once a
// wave's claims find the launch's items exhausted, its walks stop suspending for refills (nothing is
// left to fetch) and its rejection loops run until every lane has its sample instead of kRuvTrips
// trips per iteration, so the paths still in flight at the end of a launch take fewer loop
// iterations (the drain tail).  Results unchanged.
#ifndef RTZIG_DRAIN
#define RTZIG_DRAIN 0
#endif
// Waves per block that start the deferred fold before tracing (path_loop; 0: only drained waves fold)
#ifndef RTZIG_FOLD_HEAD
#define RTZIG_FOLD_HEAD 1
#endif
constexpr int kFoldHead = RTZIG_FOLD_HEAD;  // (1 measured best: 2 / 4, or 1 in every 2nd / 4th block, fold slower)
constexpr bool kDrainMode = RTZIG_DRAIN != 0;     // drained walks do not suspend
constexpr bool kDrainTrips = RTZIG_DRAIN == 1;    // drained trips are not capped (RTZIG_DRAIN=2: walks only)
#ifndef RTZIG_REFILL_MIN
#define RTZIG_REFILL_MIN 0
#endif
constexpr int kRefillMin = RTZIG_REFILL_MIN;
constexpr int kSuspended = -2;
typedef float f2 __attribute__((ext_vector_type(2)));
// {b.x * m.x + a.x, b.y * m.x + a.x}: v_pk_fma_f32 with the second and third operands' low halves
// broadcast to the high lane (op_sel_hi:[1,0,0]); their high halves are never read
// Forms of the inner step (A/B knob): 0 the shipped one (inline-asm v_pk_fma_f32 with a
// broadcast operand, volatile-asm v_max3/v_min3, asm ds_read_b64); 1 builtin packed fma and
// min/max; 2 form 1 with plain LDS loads (ds_read2_b64); 4 form 0 with the slab min/max as
// non-volatile asm (schedulable); 5 form 0 with builtin min/max.
#if RTZIG_WALK_FORM == 4 || RTZIG_WALK_FORM == 5
#define RTK_PK_ASM 1
#else
#define RTK_PK_ASM (RTZIG_WALK_FORM == 0)
#endif
__device__ __forceinline__ f2 pk_fma_lo(f2 b, f2 m, f2 a) {
#if !RTK_PK_ASM
    const f2 mm = {m.x, m.x}, aa = {a.x, a.x};
    return __builtin_elementwise_fma(b, mm, aa);
#else
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(b), "v"(m), "v"(a));
    return r;
#endif
}
typedef int32_t i2 __attribute__((ext_vector_type(2)));

// LDS reads issued as single instructions (the caller waits with s_waitcnt lgkmcnt(0), naming the
// results as operands so nothing reads them earlier).  `addr` is an LDS byte address.
template <class T>
__device__ __forceinline__ void lds_b64(T& v, uint32_t addr, int off) {
    static_assert(sizeof(T) == 8, "b64");
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
}
__device__ __forceinline__ void lds_b32(int32_t& v, uint32_t addr, int off) {
    asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// Exact candidate filter for the leaf round.  With s = fl(sqrt(disc)), the reference's roots are
// root1 = fl(fl(h - s) / a) <= root2 = fl(fl(h + s) / a), and the candidate of a sphere is root1 if
// t_min < root1, else root2 if t_min < root2 (sphere.zig:35-41).  behind(h, disc) proves
// root2 <= t_min, so the sphere yields no candidate.  It is evaluated with explicit fma and margins
// of 2^-30 relative (plus a * 2^-600 absolute) that dominate every rounding error of the comparison
// (a few ulps), so it never rejects a sphere the exact candidate() would accept; NaN or inf operands
// make the test false (keep the sphere).  Proof: Z = (t_min*a - margins) - h - 2^-30|h|;
// Z > 0 and Z*Z > disc*(1 + 2^-30) give s < Z, hence h + s < t_min*a by more than the rounding of
// fl(h + s), so fl(h + s) / a < t_min and root1 <= root2 <= t_min.  The filter needs a within
// [2^-400, 2^400] (else it never rejects).  Typical catch: the sphere a secondary ray starts on
// (c ~ 0, h < 0), whose candidate otherwise costs a sqrt and two divisions for the whole wave.
struct LeafFilter {
    double a_tiny;  // a * 2^-600
    double tm_lim;  // t_min * a lowered by the margins
    bool on;
    __device__ __forceinline__ static LeafFilter make(double a, double t_min) {
        LeafFilter f;
        f.on = a > 0x1p-400 && a < 0x1p400;
        f.a_tiny = a * 0x1p-600;
        const double pm = t_min * a;
        f.tm_lim = __builtin_fma(-__builtin_fabs(pm), 0x1p-30, pm) - f.a_tiny;
        return f;
    }
    __device__ __forceinline__ bool behind(double h, double disc) const {
        const double z = __builtin_fma(-__builtin_fabs(h), 0x1p-30, tm_lim - h);
        return on && z > 0 && __builtin_fma(z, z, -(disc * (1 + 0x1p-30))) > 0;
    }
};

// Stack entries are StackT (int32; int16 holds every ref of a tree that fits the LDS: byte offsets
// < 2^15) strided by kStride (the block size: element i of a lane at stack[i * kStride]); the
// product kernel uses <int32_t, kBlockBvh>, tools/walk_occupancy.hip other combinations.
template <class StackT>
struct StackOps;
template <>
struct StackOps<int32_t> {
    static constexpr int32_t kEnd = kDone;
    __device__ __forceinline__ static void read(int32_t& v, const int32_t* p) { lds_b32(v, lds_addr(p), 0); }
};
template <>
struct StackOps<int16_t> {
    static constexpr int32_t kEnd = INT16_MIN;  // sign-extended by ds_read_i16
    __device__ __forceinline__ static void read(int32_t& v, const int16_t* p) {
        asm volatile("ds_read_i16 %0, %1" : "=v"(v) : "v"(lds_addr(p)));
    }
};

template <bool kLdsNodes, int kStride = kBlockBvh, class StackT = int32_t, bool kF32 = false>
struct BvhWalker {
    static constexpr int32_t kEnd = StackOps<StackT>::kEnd;  // "walk finished" (stack entry 0)
    static constexpr bool kFast = kF32;  // fast mode: f32 ray, f32 leaf tests (huge spheres in f64)
    using RayT = std::conditional_t<kF32, fm::Ray, Ray>;
    using Real = std::conditional_t<kF32, float, double>;
    const BvhNode* __restrict__ nodes;
    const BvhLeaf* __restrict__ leaves;
    const GeoRec* __restrict__ ageo;     // always-list geometry
    const uint32_t* __restrict__ asid;   // always-list original indices
    uint32_t n_always;
    StackT* stack;                       // LDS, element i of this lane at stack[i * kStride]
    float origin_bound;                  // BvhArgs::origin_bound
    const GeoRec* __restrict__ geo_all;  // the whole list in original order (far-origin lanes)
    uint32_t n_pad;
#if RTZIG_BOUNDS
#ifndef RTZIG_BOUNDS_SELFTEST
#define RTZIG_BOUNDS_SELFTEST 0  // 1: the tree's last node counts as out of range (the check must report it)
#endif
    uint32_t node_bytes, leaf_bytes, depth;  // debug builds: the tree's extent, the stack's entries
    unsigned long long* err;                 // UnitArgs::ctr (the error word, rt_units.h bounds_ok)
    __device__ __forceinline__ bool node_ok(int32_t& cur, StackT* top) const {
        // at an internal node the lane's stack holds entries 0..sp and the push writes entry sp + 1,
        // which must lie below `depth` (the tree's depth bounds the pushes on any root path)
        const bool ok = (uint32_t)cur < node_bytes - RTZIG_BOUNDS_SELFTEST * (uint32_t)sizeof(BvhNode) &&
                        top >= stack && top + kStride < stack + depth * kStride;
        if (!bounds_ok(ok, err)) cur = kEnd;
        return ok;
    }
    __device__ __forceinline__ bool leaf_ok(int32_t cur) const { return bounds_ok((uint32_t)(~cur) < leaf_bytes, err); }
#else
    __device__ __forceinline__ bool node_ok(int32_t&, StackT*) const { return true; }
    __device__ __forceinline__ bool leaf_ok(int32_t) const { return true; }
#endif

    // always-list sphere q: geometry + original index from global memory (uniform address,
    // read-only data: scalar loads; the compiler emits per-lane vector loads, since it cannot prove
    // the kernel's stores do not alias it)
    template <class PR>
    __device__ __forceinline__ void test_always(uint32_t q, const Ray& r, double a, const RayDiv& ad, double t_min, const LeafFilter& lfilt,
                                                double& closest, uint32_t& best, bool& found, PR& pr) const {
        u32x8 w;
        asm volatile("s_load_dwordx8 %0, %1, 0\n\ts_waitcnt lgkmcnt(0)" : "=s"(w) : "s"(ageo + q));
        test_always_geo<-1>(w, asid[q], r, a, ad, t_min, lfilt, closest, best, found, pr);
    }
    // the same for a compile-time Q < 4 (the unrolled common case): the always-list pointers are
    // re-read from the kernarg segment (BvhArgs, the kernel's second argument) and the sphere sits
    // at an immediate offset, so no per-sphere address is held in SGPRs across the walk (held,
    // they were spilled to VGPR lanes and reloaded with v_readlane)
    template <int Q, class PR>
    __device__ __forceinline__ void test_always_c(const Ray& r, double a, const RayDiv& ad, double t_min, const LeafFilter& lfilt,
                                                  double& closest, uint32_t& best, bool& found, PR& pr) const {
        static_assert(sizeof(KernelParams) == 336 && offsetof(BvhArgs, always_geo) == 16 &&
                          offsetof(BvhArgs, always_sid) == 24,
                      "kernarg offsets of BvhArgs::always_geo / always_sid");
        constexpr int kGeoPtr = 336 + 16, kSidPtr = 336 + 24;
        const uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
        uint64_t pg, ps;
        asm volatile("s_load_dwordx2 %0, %2, %3\n\ts_load_dwordx2 %1, %2, %4\n\ts_waitcnt lgkmcnt(0)"
                     : "=s"(pg), "=s"(ps) : "s"(kp), "i"(kGeoPtr), "i"(kSidPtr));
        u32x8 w;
        uint32_t sid;
        asm volatile("s_load_dwordx8 %0, %2, %3\n\ts_load_dword %1, %4, %5\n\ts_waitcnt lgkmcnt(0)"
                     : "=s"(w), "=s"(sid) : "s"(pg), "i"(Q * 32), "s"(ps), "i"(Q * 4));
        test_always_geo<Q>(w, sid, r, a, ad, t_min, lfilt, closest, best, found, pr);
    }
    __device__ __forceinline__ static uint32_t n_always_now() {
        static_assert(offsetof(BvhArgs, n_always) == 40, "kernarg offset of BvhArgs::n_always");
        const uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
        uint32_t n;
        asm volatile("s_load_dword %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=s"(n) : "s"(kp), "i"(336 + 40));
        return n;
    }
    template <int Q, class PR>  // Q: the always-list slot when compile-time (instrumented counts), else -1
    __device__ __forceinline__ static void test_always_geo(const u32x8& w, uint32_t sid, const Ray& r, double a, const RayDiv& ad,
                                                           double t_min, const LeafFilter& lfilt, double& closest,
                                                           uint32_t& best, bool& found, PR& pr) {
        const GeoRec s{dw2d(w[0], w[1]), dw2d(w[2], w[3]), dw2d(w[4], w[5]), dw2d(w[6], w[7])};
        const double ocx = s.cx - r.orig.x;
        const double ocy = s.cy - r.orig.y;
        const double ocz = s.cz - r.orig.z;
        const double h = (r.dir.x * ocx + r.dir.y * ocy) + r.dir.z * ocz;
        const double c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - s.r2;
        const double disc = h * h - a * c;
        // the ground sphere is "behind" every ray that leaves it: no sqrt / second-root division
        if (disc >= 0 && !lfilt.behind(h, disc)) candidate<Q>(sid, h, disc, ad, t_min, closest, best, found, pr);
    }

    // root selection of sphere.zig:35-41 for a sphere with disc >= 0, then the first-wins argmin.
    // The argmin is order-independent (ties go to the lower original index), so candidates may be
    // taken in any order.  (A branch-free form that computes both roots for every lane measured 4%
    // slower.)
    // Q: the always-list slot 0..3, -1 (always-list loop) or -2 (a leaf round): instrumented counts
    // and region markers only
    template <int Q, class PR>
    __device__ __forceinline__ static void candidate(uint32_t k, double h, double disc, const RayDiv& a, double t_min,
                                                     double& closest, uint32_t& best, bool& found, PR& pr) {
        mark_cand<Q>();
        pr.template cand_block<Q>();
        const double sq = sqrt_g(disc);
        double ts = a.div(h - sq);
        bool cand = t_min < ts;
        if (!cand) {
            mark_root2<Q>();
            pr.template root2_block<Q>();
            ts = a.div(h + sq);
            cand = t_min < ts;
            mark_cand<Q>();
        }
        if (cand && (ts < closest || (found && ts == closest && k < best))) {
            closest = ts;
            best = k;
            found = true;
        }
        mark_caller<Q>();
    }

    static constexpr bool kCanSuspend = true;
    struct State {  // a suspended walk (dynamic fetch)
        int32_t cur;
        StackT* top;
        Real closest;
        uint32_t best;
        bool found;
    };
    // fast mode's always-list: big spheres (radius < 100 near the origin) in f32, huge ones (the
    // final scene's r = 1000 ground) in f64 — in f32 a point on a radius-1000 sphere is known only to
    // ~6e-5 along its normal, so rays leaving it would re-hit it at grazing angles
    __device__ __forceinline__ void always_f32(const fm::Ray& r, float t_min, float t_max, float& closest, uint32_t& best,
                                               bool& found) const {
#pragma clang fp contract(fast)
        const double ox = r.orig.x, oy = r.orig.y, oz = r.orig.z;
        const double dx = r.dir.x, dy = r.dir.y, dz = r.dir.z;
        const double a = (dx * dx + dy * dy) + dz * dz;
        const float fa = fm::len_sq(r.dir);
        double cl = (double)t_max;
        for (uint32_t q = 0; q < n_always; ++q) {
            const GeoRec s = ageo[q];
            if (s.r2 < 1e4 && __builtin_fabs(s.cx) + __builtin_fabs(s.cy) + __builtin_fabs(s.cz) < 1e4) {
                const float fx = (float)s.cx - r.orig.x, fy = (float)s.cy - r.orig.y, fz = (float)s.cz - r.orig.z;
                const float h = r.dir.x * fx + r.dir.y * fy + r.dir.z * fz;
                const float c = (fx * fx + fy * fy + fz * fz) - (float)s.r2;
                const float disc = h * h - fa * c;
                if (disc >= 0) {
                    const float sq = __builtin_sqrtf(disc), ia = __builtin_amdgcn_rcpf(fa);
                    float ts = (h - sq) * ia;
                    if (!(t_min < ts)) ts = (h + sq) * ia;
                    if (t_min < ts && (double)ts < cl) {
                        cl = ts;
                        best = asid[q];
                        found = true;
                    }
                }
                continue;
            }
            const double cx = s.cx - ox, cy = s.cy - oy, cz = s.cz - oz;
            const double h = (dx * cx + dy * cy) + dz * cz;
            const double c = ((cx * cx + cy * cy) + cz * cz) - s.r2;
            const double disc = h * h - a * c;
            if (disc >= 0) {
                const double sq = __builtin_sqrt(disc);
                double ts = (h - sq) / a;
                if (!(t_min < ts)) ts = (h + sq) / a;
                if (t_min < ts && ts < cl) {
                    cl = ts;
                    best = asid[q];
                    found = true;
                }
            }
        }
        closest = found ? (float)cl : t_max;
    }
    // fast mode's leaf: kLeafBvh f32 quadratics with the reciprocal of a
    __device__ __forceinline__ void leaf_f32(const BvhLeaf* lf, const fm::Ray& r, float t_min, float inv_a, float a,
                                             float& closest, uint32_t& best, bool& found) const {
#pragma clang fp contract(fast)
#pragma unroll
        for (int u = 0; u < kLeafBvh; ++u) {
            const LeafGeo s = lf->g[u];
            const float cx = (float)s.cx - r.orig.x, cy = (float)s.cy - r.orig.y, cz = (float)s.cz - r.orig.z;
            const float h = r.dir.x * cx + r.dir.y * cy + r.dir.z * cz;
            const float c = (cx * cx + cy * cy + cz * cz) - (float)s.r2;
            const float disc = h * h - a * c;
            if (disc >= 0) {
                const float sq = __builtin_sqrtf(disc);
                float ts = (h - sq) * inv_a;
                if (!(t_min < ts)) ts = (h + sq) * inv_a;
                if (t_min < ts && ts < closest) {
                    closest = ts;
                    best = lf->sid[u];
                    found = true;
                }
            }
        }
    }

    template <class PR>
    __device__ __forceinline__ int operator()(const RayT& r, Real t_min, Real t_max, Real* t_hit, PR& pr) const {
        State s;
        return run<false>(r, t_min, t_max, t_hit, pr, s, false);
    }
    // refetch (wave-uniform): suspend walks for a shading batch (dynamic fetch); false once the
    // launch's items are all handed out — there is nothing left to fetch, so walks run to the end
    template <bool kSusp, class PR>
    __device__ __forceinline__ int run(const RayT& r, Real t_min, Real t_max, Real* t_hit, PR& pr, State& st,
                                       const bool resume, const bool refetch = true) const {
        if constexpr (kF32) {
            return run_f32<kSusp>(r, t_min, t_max, t_hit, pr, st, resume, refetch);
        } else {
            return run_f64<kSusp>(r, t_min, t_max, t_hit, pr, st, resume, refetch);
        }
    }

    // The traversal shared by both precisions: lanes advance through internal nodes until each holds a
    // leaf or is done (cur, top: the lane's walk state; lower / upper: its f32 [t_min, closest]).
    template <class PR>
    __device__ __forceinline__ void descend(int32_t& cur, StackT*& top, uint32_t ax, uint32_t ay, uint32_t az,
                                            f2 inv_x, f2 inv_y, f2 inv_z, f2 noi_x, f2 noi_y, f2 noi_z, float lower,
                                            float upper, PR& pr) const {
        while (cur >= 0) {
            if (!node_ok(cur, top)) break;
            pr.visit();
            pr.inner_iter();
            f2 bx0, by0, bz0, bx1, by1, bz1;
            int32_t ref0, ref1, popped;
            if constexpr (kLdsNodes && RTZIG_WALK_FORM != 2 && RTZIG_WALK_FORM != 3) {
                // nodes start at LDS address 0: the ref is the address.  Seven ds_read_b64
                // (2 LDS cycles each); left to itself the compiler pairs them into
                // ds_read2_b64 (8 cycles for the same 16 B) behind extra base adds.
                const uint32_t a = (uint32_t)cur;
                i2 refs;
                lds_b64(bx0, a + ax, 0); lds_b64(bx1, a + ax, 48);
                lds_b64(by0, a + ay, 0); lds_b64(by1, a + ay, 48);
                lds_b64(bz0, a + az, 0); lds_b64(bz1, a + az, 48);
                lds_b64(refs, a, 96);
                StackOps<StackT>::read(popped, top);
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(bx0), "+v"(bx1), "+v"(by0), "+v"(by1), "+v"(bz0), "+v"(bz1), "+v"(refs),
                               "+v"(popped));
                ref0 = refs.x;
                ref1 = refs.y;
            } else if constexpr (kLdsNodes) {
                // the same reads as plain LDS loads (form 2): the compiler pairs each axis's two planes
                // into one ds_read2_b64 and waits for them one by one.  Nodes start at LDS address 0, so
                // the ref is the address itself.
                typedef const __attribute__((address_space(3))) char* lds_cp;
                const lds_cp nb = (lds_cp)(uintptr_t)(uint32_t)cur;
                bx0 = *(const __attribute__((address_space(3))) f2*)(nb + ax);
                by0 = *(const __attribute__((address_space(3))) f2*)(nb + ay);
                bz0 = *(const __attribute__((address_space(3))) f2*)(nb + az);
                bx1 = *(const __attribute__((address_space(3))) f2*)(nb + 48 + ax);
                by1 = *(const __attribute__((address_space(3))) f2*)(nb + 48 + ay);
                bz1 = *(const __attribute__((address_space(3))) f2*)(nb + 48 + az);
                const i2 refs = *(const __attribute__((address_space(3))) i2*)(nb + 96);
                ref0 = refs.x;
                ref1 = refs.y;
                popped = *top;
            } else {
                const char* nb = (const char*)nodes + cur;  // byte-offset ref
                bx0 = *(const f2*)(nb + ax); by0 = *(const f2*)(nb + ay); bz0 = *(const f2*)(nb + az);
                bx1 = *(const f2*)(nb + 48 + ax); by1 = *(const f2*)(nb + 48 + ay); bz1 = *(const f2*)(nb + 48 + az);
                ref0 = *(const int32_t*)(nb + 96);
                ref1 = *(const int32_t*)(nb + 100);
                popped = *top;
            }
            const f2 tx0 = pk_fma_lo(bx0, inv_x, noi_x);
            const f2 ty0 = pk_fma_lo(by0, inv_y, noi_y);
            const f2 tz0 = pk_fma_lo(bz0, inv_z, noi_z);
            const f2 tx1 = pk_fma_lo(bx1, inv_x, noi_x);
            const f2 ty1 = pk_fma_lo(by1, inv_y, noi_y);
            const f2 tz1 = pk_fma_lo(bz1, inv_z, noi_z);
            const float n0 = slab_near(tx0.x, ty0.x, tz0.x, lower), f0 = slab_far(tx0.y, ty0.y, tz0.y, upper);
            const float n1 = slab_near(tx1.x, ty1.x, tz1.x, lower), f1 = slab_far(tx1.y, ty1.y, tz1.y, upper);
            // both hit: descend into the nearer child and push the farther one (the store
            // always happens; it only counts when sp advances); one hit: descend; none: pop.
            // The three compares are taken as wave masks and combined on the scalar unit, and
            // the selects are v_cndmask on those masks: 3 compares + 5 selects (the compiler's
            // form of the same logic re-compared a negated mask on the VALU).
#if RTZIG_WALK_FORM == 3
            const bool h0 = n0 <= f0, h1 = n1 <= f1, nf = n0 <= n1;
            const bool p0 = h0 && (!h1 || nf);
            const int32_t near = p0 ? ref0 : ref1, far = p0 ? ref1 : ref0;
            top[kStride] = (StackT)far;
            cur = (h0 || h1) ? near : popped;
            top += (h0 && h1) ? kStride : ((h0 || h1) ? 0 : -kStride);
#else
            const uint64_t m0 = __ballot(n0 <= f0), m1 = __ballot(n1 <= f1), mf = __ballot(n0 <= n1);
            const uint64_t pick0 = m0 & (~m1 | mf);  // both: nearer; one: that one
            const uint64_t any = m0 | m1, both = m0 & m1;
            const int32_t near = sel_mask(ref1, ref0, pick0), far = sel_mask(ref0, ref1, pick0);
            top[kStride] = (StackT)far;
            cur = sel_mask(popped, near, any);
            // the stack step in bytes: one v_add_u32 (2.2 cycles) instead of the element step's
            // v_lshl_add_u32 (4.15, profiles/r05_peak/)
            constexpr int32_t kStep = kStride * (int32_t)sizeof(StackT);
            top = (StackT*)((char*)top + sel_mask(sel_mask(-kStep, 0, any), kStep, both));
#endif
        }
    }

    template <bool kSusp, class PR>
    __device__ __forceinline__ int run_f32(const fm::Ray& r, float t_min, float t_max, float* t_hit, PR& pr, State& st,
                                           const bool resume, const bool refetch) const {
        const float a = fm::len_sq(r.dir);
        const float inv_a = __builtin_amdgcn_rcpf(a);
        float closest = t_max;
        uint32_t best = 0;
        bool found = false;
        if (kSusp && resume) {
            closest = st.closest;
            best = st.best;
            found = st.found;
        } else {
            always_f32(r, t_min, t_max, closest, best, found);
            pr.tests(n_always);
        }
        const float ox = r.orig.x, oy = r.orig.y, oz = r.orig.z;
        const float ix = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(r.dir.x), -1e30f, 1e30f);
        const float iy = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(r.dir.y), -1e30f, 1e30f);
        const float iz = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(r.dir.z), -1e30f, 1e30f);
        const uint32_t ax = ix < 0 ? 8u : 0u, ay = 16u + (iy < 0 ? 8u : 0u), az = 32u + (iz < 0 ? 8u : 0u);
        // origins beyond the boxes' origin bound walk the whole list (exact f64 scan, as in parity mode)
        const bool far = !(kSusp && resume) &&
                         __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(ox), __builtin_fabsf(oy)), __builtin_fabsf(oz)) >
                             origin_bound;
        if (__builtin_expect(__ballot(far) != 0, 0)) {
            if (far) {
                double t;
                const Ray r64{fm::to64(r.orig), fm::to64(r.dir)};
                const int k = world_hit<1>(geo_all, n_pad, r64, (double)t_min, (double)t_max, &t);
                pr.tests(n_pad);
                found = k >= 0;
                best = found ? (uint32_t)k : 0u;
                closest = (float)t;
            }
        }
        f2 inv_x, inv_y, inv_z, noi_x, noi_y, noi_z;
        inv_x.x = ix; inv_y.x = iy; inv_z.x = iz;
        noi_x.x = -(ox * ix); noi_y.x = -(oy * iy); noi_z.x = -(oz * iz);
        float lower = t_min;
        lower = lower - __builtin_fabsf(lower) * 0x1p-20f - 1e-30f;
        float upper = closest + __builtin_fabsf(closest) * 0x1p-20f;
        StackT* top = stack;
        int32_t cur = far ? kEnd : 0;
        if (kSusp && resume) {
            top = st.top;
            cur = st.cur;
        }
        while (cur != kEnd) {
            descend(cur, top, ax, ay, az, inv_x, inv_y, inv_z, noi_x, noi_y, noi_z, lower, upper, pr);
            if (cur != kEnd && !leaf_ok(cur)) cur = kEnd;
            if (cur != kEnd) {
                pr.leaf_iter();
                leaf_f32((const BvhLeaf*)((const char*)leaves + (uint32_t)(~cur)), r, t_min, inv_a, a, closest, best, found);
                pr.tests(kLeafBvh);
                upper = closest + __builtin_fabsf(closest) * 0x1p-20f;
                cur = *top;
                top -= kStride;
            }
            if constexpr (kSusp) {
                const uint64_t walking = __ballot(cur != kEnd);
                if (refetch && walking != 0 && 64 - __popcll(walking) >= kRefetchK) break;
            }
        }
        if constexpr (kSusp) {
            if (cur != kEnd) {
                st.cur = cur;
                st.top = top;
                st.closest = closest;
                st.best = best;
                st.found = found;
                return kSuspended;
            }
        }
        *t_hit = closest;
        return found ? (int)best : -1;
    }

    template <bool kSusp, class PR>
    __device__ __forceinline__ int run_f64(const Ray& r, double t_min, double t_max, double* t_hit, PR& pr, State& st,
                                           const bool resume, const bool refetch) const {
        const double a = len_sq(r.dir);
        double closest = t_max;
        uint32_t best = 0;
        bool found = false;
        if constexpr (kSusp) {
            if (resume) {
                closest = st.closest;
                best = st.best;
                found = st.found;
            }
        }
        const LeafFilter lfilt = LeafFilter::make(a, t_min);
        const RayDiv ad(a);
        RTK_MARK("always");
        if (kSusp && resume) {
            // the always-list and the far-origin check ran when this walk started
        } else if (n_always <= 4) {
            // the common case (the ground and up to three big spheres), unrolled so that closest /
            // best / found are not loop-carried through a runtime-bounded loop
            // n_always is re-read from the kernarg segment at each test (a held copy of each
            // `n_always > q` was kept as a spilled lane mask)
            if (n_always_now() > 0) test_always_c<0>(r, a, ad, t_min, lfilt, closest, best, found, pr);
            if (n_always_now() > 1) test_always_c<1>(r, a, ad, t_min, lfilt, closest, best, found, pr);
            if (n_always_now() > 2) test_always_c<2>(r, a, ad, t_min, lfilt, closest, best, found, pr);
            if (n_always_now() > 3) test_always_c<3>(r, a, ad, t_min, lfilt, closest, best, found, pr);
        } else {
            for (uint32_t q = 0; q < n_always; ++q) test_always(q, r, a, ad, t_min, lfilt, closest, best, found, pr);
        }
        if (!(kSusp && resume)) pr.tests(n_always);
        RTK_MARK("walk_setup");

        // f32 ray for the conservative slab tests (error budget: rt_bvh.cpp)
        const float ox = (float)r.orig.x, oy = (float)r.orig.y, oz = (float)r.orig.z;
        const float dx = (float)r.dir.x, dy = (float)r.dir.y, dz = (float)r.dir.z;
        // v_rcp_f32 (1 ulp) instead of three correctly rounded f32 divisions (~11 ops each), then
        // clamped to +-1e30 by one v_med3 per axis: the inverse of a component clamped to
        // +-1e-30 (rcp(+-0) = +-inf keeps its sign), one op instead of compare + copysign + select
        const float ix = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(dx), -1e30f, 1e30f);
        const float iy = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(dy), -1e30f, 1e30f);
        const float iz = __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(dz), -1e30f, 1e30f);
        // slab planes as t = fma(bound, inv, -o*inv): one op per plane.  Error (position space,
        // per axis) <= 2^-24 (4|bound| + 5|o|), inside the padding of rt_bvh.cpp.  fma is monotone
        // in `bound`, so for inv > 0 the lo plane is the near one and for inv < 0 the hi plane: the
        // lane reads its (near, far) pair per axis at byte +0 or +8 of the axis's {lo, hi, hi, lo}
        // (rtk::BvhNode) and both planes of an axis come out of one packed fma.  inv is finite, and
        // nonzero unless the f32 component overflowed (then every point of the ray past t_min lies
        // beyond any boundable box, and the [0, 0] slab culls it correctly), and NaN only for a NaN
        // direction (whose f64 sphere tests never pass), so the pick matches the min/max of the
        // two planes exactly; an
        // overflowed plane is +-inf in ray order, and NaN arises only from a NaN origin, which
        // v_max3/v_min3 drop (the box is kept: permissive, never a wrong cull).
        const uint32_t ax = ix < 0 ? 8u : 0u, ay = 16u + (iy < 0 ? 8u : 0u), az = 32u + (iz < 0 ? 8u : 0u);
        // A lane whose origin lies outside the box padding's origin bound (rt_bvh.cpp) must not be
        // culled by the f32 boxes: it walks the whole list linearly instead (the reference's own
        // scan, exact) and skips the tree.  Only rays leaving an unboundable always-list sphere get
        // there, so the common path pays one compare and one ballot per ray.  (A NaN origin fails
        // every sphere test anyway; the max drops it.)
        const bool far = !(kSusp && resume) &&
                         __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(ox), __builtin_fabsf(oy)), __builtin_fabsf(oz)) >
                             origin_bound;
        if (__builtin_expect(__ballot(far) != 0, 0)) {
            if (far) {
                RTK_MARK("rare");
                double t;
                const int k = world_hit<1>(geo_all, n_pad, r, t_min, t_max, &t);
                pr.tests(n_pad);
                found = k >= 0;
                best = found ? (uint32_t)k : 0u;
                closest = t;
            }
        }
        // per-axis constants live in the low half of a register pair; pk_fma_lo broadcasts them to
        // both lanes of the packed fma (op_sel_hi), so they are not duplicated with v_mov
        f2 inv_x, inv_y, inv_z, noi_x, noi_y, noi_z;
        inv_x.x = ix; inv_y.x = iy; inv_z.x = iz;
        noi_x.x = -(ox * ix); noi_y.x = -(oy * iy); noi_z.x = -(oz * iz);
        float lower = (float)t_min;
        lower = lower - __builtin_fabsf(lower) * 0x1p-20f - 1e-30f;
        float upper = (float)closest;
        upper = upper + __builtin_fabsf(upper) * 0x1p-20f;

        // stack: entry 0 holds kEnd (written once per lane at kernel start), entries 1..sp the
        // pushed far children; a pop reads entry sp, so popping the empty stack yields kEnd
        StackT* top = stack;  // this lane's stack entry sp (entry i at stack[i * kStride])
        int32_t cur = far ? kEnd : 0;  // root
        if constexpr (kSusp) {
            if (resume) {
                top = st.top;
                cur = st.cur;
            }
        }
        // while-while (Aila & Laine 2009): every lane advances through internal nodes until it
        // holds a leaf (or is done); then the lanes with a leaf test its spheres together, so the
        // f64 leaf work runs with most lanes active instead of whenever any one lane hits a leaf.
        RTK_MARK("walk_inner");
        while (cur != kEnd) {
            descend(cur, top, ax, ay, az, inv_x, inv_y, inv_z, noi_x, noi_y, noi_z, lower, upper, pr);
            if (cur != kEnd && !leaf_ok(cur)) cur = kEnd;
            RTK_MARK("leaf");
            if (cur != kEnd) {
                pr.leaf_iter();
                // leaf: exactly kLeafBvh slots (sentinel-padded); the kLeafBvh discriminant chains
                // are independent, the candidate updates then run in slot order
                const BvhLeaf* lf = (const BvhLeaf*)((const char*)leaves + (uint32_t)(~cur));
                double h[kLeafBvh], disc[kLeafBvh];
#pragma unroll
                for (int u = 0; u < kLeafBvh; ++u) {
                    const LeafGeo s = lf->g[u];
                    const double ocx = s.cx - r.orig.x;
                    const double ocy = s.cy - r.orig.y;
                    const double ocz = s.cz - r.orig.z;
                    h[u] = (r.dir.x * ocx + r.dir.y * ocy) + r.dir.z * ocz;
                    const double c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - s.r2;
                    disc[u] = h[u] * h[u] - a * c;
                }
                // Compacted candidates: a wave pays a candidate block (sqrt + division) whenever ANY
                // of its lanes needs it, so each lane first drops the slots that provably cannot
                // win (LeafFilter) and then feeds its viable slots through ONE block per round,
                // nearest-looking (smallest h) first; a second round runs only for lanes with a
                // second slot still viable after `closest` has shrunk.
                if constexpr (kLeafBvh == 2) {
                    // the same rounds written out for two slots, so the viability flags stay lane
                    // masks (the generic form keeps them as 0/1 VGPRs and re-compares them)
                    const bool v0 = disc[0] >= 0 && !lfilt.behind(h[0], disc[0]);
                    const bool v1 = disc[1] >= 0 && !lfilt.behind(h[1], disc[1]);
                    const bool p1 = v1 && (!v0 || h[1] < h[0]);  // round 1 takes slot 1
                    const uint32_t s0 = lf->sid[0], s1 = lf->sid[1];
                    if (v0 || v1)
                        candidate<-2>(p1 ? s1 : s0, p1 ? h[1] : h[0], p1 ? disc[1] : disc[0], ad, t_min, closest, best,
                                  found, pr);
                    if (v0 && v1)  // round 2: the other slot
                        candidate<-2>(p1 ? s0 : s1, p1 ? h[0] : h[1], p1 ? disc[0] : disc[1], ad, t_min, closest, best,
                                  found, pr);
                } else {
                bool v[kLeafBvh];
                uint32_t sid[kLeafBvh];
#pragma unroll
                for (int u = 0; u < kLeafBvh; ++u) {
                    sid[u] = lf->sid[u];
                    v[u] = disc[u] >= 0 && !lfilt.behind(h[u], disc[u]);
                }
#pragma unroll
                for (int rd = 0; rd < kLeafBvh; ++rd) {
                    bool any = false;
                    double hb = 0, db = 0;
                    uint32_t kb = 0;
                    int pb = 0;
#pragma unroll
                    for (int u = 0; u < kLeafBvh; ++u) {
                        const bool take = v[u] && (!any || h[u] < hb);
                        hb = take ? h[u] : hb;
                        db = take ? disc[u] : db;
                        kb = take ? sid[u] : kb;
                        pb = take ? u : pb;
                        any = any || v[u];
                    }
                    if (!any) break;
                    candidate<-2>(kb, hb, db, ad, t_min, closest, best, found, pr);
                    if (rd + 1 < kLeafBvh) {
#pragma unroll
                        for (int u = 0; u < kLeafBvh; ++u) {
                            v[u] = v[u] && u != pb;
                        }
                    }
                }
                }
                pr.tests(kLeafBvh);
                upper = (float)closest;
                upper = upper + __builtin_fabsf(upper) * 0x1p-20f;
                cur = *top;  // pop (entry 0: kEnd)
                top -= kStride;
            }
            if constexpr (kSusp) {
                // wave-uniform: enough free lanes to make a shading batch worthwhile
                const uint64_t walking = __ballot(cur != kEnd);
                if (refetch && walking != 0 && 64 - __popcll(walking) >= kRefetchK) break;
            }
        }
        if constexpr (kSusp) {
            if (cur != kEnd) {
                st.cur = cur;
                st.top = top;
                st.closest = closest;
                st.best = best;
                st.found = found;
                return kSuspended;
            }
        }
        *t_hit = closest;
        return found ? (int)best : -1;
    }
};

// Fast mode's pieces of the path loop (the parity forms are written inline there).
template <class W, class = void>
struct WalkerPrecision {
    static constexpr bool kF32 = false;
};
template <class W>
struct WalkerPrecision<W, std::void_t<decltype(W::kFast)>> {
    static constexpr bool kF32 = W::kFast;
};
// one trip of the shared rejection loop: randomUnitVec (3 draws) or randomInUnitDisk (2 draws)
__device__ __forceinline__ void trip_f32(Rng& g, bool wr, float& ux, float& uy, float& uz, float& uls, bool& got,
                                         bool& dgot) {
#pragma clang fp contract(fast)
    fm::uniform2(g, ux, uy);
    ux = fm::pm1(ux);
    uy = fm::pm1(uy);
    const float xy = ux * ux + uy * uy;
    if (wr) {
        uz = fm::pm1(fm::uniform(g));
        uls = xy + uz * uz;
    }
    // the flags are assigned by value on both sides: stores into got OR dgot through a selected
    // address kept both in scratch memory (8 bytes per lane, scratch_store_byte per trip)
    const bool acc = wr ? (1e-30f < uls && uls <= 1.0f) : xy < 1.0f;
    got = wr ? acc : got;
    dgot = wr ? dgot : acc;
}
// the accepted randomUnitVec finishes a Lambertian / Metal scatter (material.zig:27-68)
__device__ __forceinline__ void scatter_f32(float ux, float uy, float uz, float uls, bool sc_metal, fm::f3 sc_nrm,
                                            fm::f3 sc_refl, float sc_fuzz, bool& pending, bool& done, fm::Ray& r,
                                            uint32_t& bounce) {
#pragma clang fp contract(fast)
    const fm::f3 ruv = fm::muls(fm::mk(ux, uy, uz), __builtin_amdgcn_rsqf(uls));
    fm::f3 dir;
    bool absorbed = false;
    if (!sc_metal) {
        dir = fm::add(sc_nrm, ruv);
        if (fm::near_zero(dir)) dir = sc_nrm;
    } else {
        dir = fm::add(sc_refl, fm::muls(ruv, sc_fuzz));
        absorbed = !(fm::dot(dir, sc_nrm) > 0);
    }
    pending = false;
    if (absorbed) {
        done = true;
    } else {
        r.dir = dir;
        ++bounce;
    }
}
// rayColor's loop body after the walk (camera.zig:157-177) in f32
__device__ __forceinline__ void shade_f32(int k, float t, const GeoRec* __restrict__ geo_orig,
                                          const MatRec* __restrict__ mat_g, Rng& g, fm::Ray& r, fm::f3& att, fm::f3& col,
                                          bool& done, bool& pending, bool& sc_metal, float& sc_fuzz, fm::f3& sc_nrm,
                                          fm::f3& sc_refl, uint32_t& bounce) {
#pragma clang fp contract(fast)
    // as the parity path (path_loop): every shaded lane computes the hit record (sky lanes on
    // sphere 0's records, never used), the metal reflection replaces ray.dir in place, and the
    // scatter state is written unconditionally (read only while pending)
    const bool hit = k >= 0;
    const uint32_t kk = hit ? (uint32_t)k : 0u;
    const GeoRec sg = geo_orig[kk];
    const MatRec m = mat_g[kk];
    const uint32_t kind = m.kind;
    const fm::f3 pt = fm::add(r.orig, fm::muls(r.dir, t));
    const fm::f3 outward = fm::muls(fm::sub(pt, fm::mk((float)sg.cx, (float)sg.cy, (float)sg.cz)), (float)m.inv_r);
    const bool front = fm::dot(r.dir, outward) < 0;
    const fm::f3 nrm = front ? outward : fm::neg(outward);
    if (hit && kind == 1) r.dir = fm::reflect(r.dir, nrm);
    const fm::f3 u = fm::unit(r.dir);
    sc_nrm = nrm;
    sc_refl = u;
    sc_fuzz = (float)m.fuzz;
    sc_metal = kind == 1;
    r.orig = pt;
    if (!hit) {
        const float a = 0.5f * (u.y + 1.0f);
        col = fm::mul(att, fm::add(fm::muls(fm::mk(1, 1, 1), 1.0f - a), fm::muls(fm::mk(0.5f, 0.7f, 1.0f), a)));
        done = true;
    } else if (kind <= 1) {
        att = fm::mul(att, fm::mk((float)m.albedo[0], (float)m.albedo[1], (float)m.albedo[2]));
        pending = true;
    } else {
        const float ri = front ? (float)m.inv_ior : (float)m.ior;
        const float cos_t = __builtin_fminf(-fm::dot(u, nrm), 1.0f);
        const float sin_t = __builtin_sqrtf(__builtin_fmaxf(1.0f - cos_t * cos_t, 0.0f));
        const bool cannot = ri * sin_t > 1.0f;
        const float r0 = front ? (float)m.r0_front : (float)m.r0_back;
        const float x1 = 1.0f - cos_t, x2 = x1 * x1;
        const float approx = r0 + (1.0f - r0) * (x1 * (x2 * x2));
        r.dir = (cannot || approx > fm::uniform(g)) ? fm::reflect(u, nrm) : fm::refract(u, nrm, ri);
        ++bounce;
    }
}

// Direct mode's reduce pass for one pixel (reduce_kernel, and the deferred fold below).
__device__ __forceinline__ void reduce_pixel(const double* __restrict__ samples, uint32_t P, uint32_t spp, uint32_t q,
                                             void* out, uint32_t format, double scale) {
    const double* src = samples + 3 * (size_t)q;
    const size_t stride = 3 * (size_t)P;
    double x = 0.0, y = 0.0, z = 0.0;
#pragma unroll 8
    for (uint32_t s = 0; s < spp; ++s) {
        x = x + src[0];
        y = y + src[1];
        z = z + src[2];
        src += stride;
    }
    if (format == 0) {
        double* o = (double*)out + 3 * (size_t)q;
        o[0] = x * scale;
        o[1] = y * scale;
        o[2] = z * scale;
    } else {
        uint8_t* o = (uint8_t*)out + 3 * (size_t)q;
        o[0] = to_byte(x * scale);
        o[1] = to_byte(y * scale);
        o[2] = to_byte(z * scale);
    }
}

// The deferred reduce pass: a wave claims chunks of 64 pixels until none is left (the same sums as
// reduce_kernel, lane l one pixel).  Run by the drained waves of the next direct-mode launch and by
// fold_rest_kernel for what they left.
__device__ __forceinline__ void fold_chunks(const FoldArgs& f, uint32_t lane) {
    while (true) {
        uint32_t c = 0;
        if (lane == 0) c = (uint32_t)atomicAdd(f.ctr, 1ull);
        c = __builtin_amdgcn_readfirstlane(__shfl(c, 0, 64));
        if (c >= f.n_chunks) break;
        const uint32_t q = c * 64 + lane;
        if (q < f.P) reduce_pixel(f.samples, f.P, f.spp, q, f.out, f.format, f.scale);
    }
}

// ------------------------------------------------------------------------------------------------
// The path state machine shared by every kernel variant: unit refill (rt_units.h) + one ray segment
// per lane per iteration (rayColor's loop body, camera.zig:153-177) + ring stores of finished
// samples + the ordered finalisation of finished units.
// `geo_orig` is the geometry in original list order (hit-record center of the winner).
// ------------------------------------------------------------------------------------------------
// kWin: fresh lanes take their generator and pixel sample point from the wave's seed window in LDS
// (`win`: its address; kSeedWin builds of the f64 BVH kernel).
template <bool kProf, bool kDirect, bool kWin = false, class Walker>
__device__ __forceinline__ void path_loop(const KernelParams& p, const Walker& walk, const GeoRec* __restrict__ geo_orig,
                                          const MatRec* __restrict__ mat_g, const UnitArgs& ua,
                                          unsigned long long* __restrict__ stats, uint32_t win = 0) {
    const uint32_t W = p.width;
    const uint32_t lane = lane_id();
    UnitSched<kDirect> us(ua, blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);
    // precision of the walk's instantiation: f64 parity, or fast mode (f32; walkers without the
    // member are f64)
    constexpr bool kF32 = WalkerPrecision<Walker>::kF32;
    using RayT = std::conditional_t<kF32, fm::Ray, Ray>;
    using Real = std::conditional_t<kF32, float, double>;
    using V = std::conditional_t<kF32, fm::f3, v3>;

    // per-lane path state
    bool active = false;
    uint32_t myslot = 0, mi = 0;  // the unit slot and item of the lane's path (its ring position)
    Rng g;
    RayT r;
    V att = V{1, 1, 1};
    uint32_t bounce = 0;
    // pending Lambertian/Metal scatter (waiting for its randomUnitVec), see below
    bool pending = false, sc_metal = false;
    bool dpend = false;  // camera ray waiting for its defocus-disk sample (camera_start)
    Real sc_fuzz = 0;
    V sc_nrm = V{0, 0, 0}, sc_refl = V{0, 0, 0};
    constexpr bool kSusp = kRefetchK > 0 && Walker::kCanSuspend;
    typename Walker::State ws;  // a suspended walk (dynamic fetch, kSusp only)
    bool susp = false;          // this lane's walk is suspended
    uint64_t rays = 0, nsamples = 0;
    constexpr bool kLanes = kProf && !kDirect;  // lane-level counts (ring mode only, see Prof)
    Prof<kLanes ? 2 : (kProf ? 1 : 0)> pr;
    uint64_t cyc_refill = 0, cyc_walk = 0, cyc_shade = 0, cyc_trips = 0;  // wave-uniform (kProf only)
    uint64_t cyc_fin = 0, cyc_hand = 0, cyc_seed = 0;  // parts of cyc_refill: finalise, hand-out, seed + getRay
    // wave-level executions (kProf only; scalar, wave-uniform): loop iterations, trip-loop trips, seeding
    // blocks, walks started (always-list tests), shading blocks, finalisations — with the per-step counts
    // of Prof they weight the static instruction counts of each region (tools/region_table.py)
    uint32_t n_iter = 0, n_trip = 0, n_seed = 0, n_wstart = 0, n_shade = 0, n_fin = 0;
    // lane-level executions (kProf only; wave-uniform sums of ballot popcounts): with the wave-level
    // counts they give each block's mean active lanes (stats[32..63], tools/region_table.py)
    uint32_t l_seed = 0, l_trip = 0, w_scat = 0, l_scat = 0, w_camf = 0, l_camf = 0, w_walk = 0, l_walk = 0,
             l_wstart = 0, l_shade = 0, w_sky = 0, l_sky = 0, w_lm = 0, l_lm = 0, w_di = 0, l_di = 0, w_store = 0,
             l_store = 0, l_busy = 0;
    uint32_t sh_kind = 3;  // kProf: this iteration's shading branch (0 sky, 1 Lambertian / metal, 2 dielectric, 3 none)
    uint32_t n_fill = 0, n_take = 0;  // kLanes: seed-window fills / take passes (stats[64], [65])
    uint64_t rt_start = 0, rt_drain = 0;  // s_memrealtime (100 MHz) at start / first empty claim (kProf only)
    // the seed window's key, {t, s}: the 64 pixels 64 * t + l of the launch at sample s, kept in LDS
    // after the window's planes (held in SGPRs, the pair pushed other uniform values into spills)
    typedef __attribute__((address_space(3))) uint32_t lds_u32;
    lds_u32* const wkey = (lds_u32*)(uintptr_t)(win + kSeedWinPlanes * 256);
    if constexpr (kWin) {
        if (lane == 0) {
            wkey[0] = ~0u;
            wkey[1] = ~0u;
        }
    }
    if constexpr (kProf) rt_start = __builtin_amdgcn_s_memrealtime();

    // Head fold: the previous deferred call's reduce pass (rt_render_rows_async_deferred) is started
    // by the first kFoldHead waves of every block before they trace, while the block's other waves
    // trace; the drained waves at the end take what is left (below).  Left to the drained waves
    // alone, most of it waited for waves to finish their last long paths and ran after the tail.
    if constexpr (kDirect && !kProf) {
        if (kFoldHead > 0 && ua.fold.samples != nullptr && threadIdx.x / 64 < (uint32_t)kFoldHead) fold_chunks(ua.fold, lane);
    }

    while (true) {
        uint64_t t_top = 0;
        if constexpr (kProf) t_top = __builtin_amdgcn_s_memtime();
        // ---- finalise one unit whose samples have all ended (rt_units.h) --------------------------
        RTK_MARK("finalise");
        __builtin_amdgcn_s_setprio(2);  // the hand-off's dependent loads (see the walk below)
        const bool progressed = us.finalize_one(us.ready_mask(active, myslot), lane);
        if constexpr (kProf) {
            ++n_iter;
            n_fin += progressed ? 1u : 0u;
        }
        __builtin_amdgcn_s_setprio(0);
        uint64_t t_fin = 0;
        if constexpr (kProf) {
            t_fin = __builtin_amdgcn_s_memtime();
            cyc_fin += t_fin - t_top;
        }
        // ---- hand new items to lanes without a path (wave-uniform control flow) ----------------
        RTK_MARK("handout");
        bool fresh = false;
        uint32_t fq = 0, fs = 0;  // pixel (launch-local) and sample of a freshly handed item
        const bool was_drained = us.drained;
        // RTZIG_REFILL_MIN (A/B knob, default 0): hand out items only once at least that many lanes
        // are free (or the wave has no path left), so seeding / getRay run with fuller waves
        if (kRefillMin == 0 || __popcll(__ballot(!active)) >= kRefillMin || __ballot(active) == 0)
            us.refill(active, fresh, myslot, mi, fq, fs, lane);
        uint64_t t_ref = 0;
        if constexpr (kProf) {
            if (us.drained && !was_drained) rt_drain = __builtin_amdgcn_s_memrealtime();
            t_ref = __builtin_amdgcn_s_memtime();
            cyc_hand += t_ref - t_fin;
        }
        // the lanes handed an item above start their path: seeding and getRay run once, outside
        // the claim loop, so the generator state and ray are not loop-carried through it
        if constexpr (kProf) n_seed += __ballot(fresh) != 0 ? 1u : 0u;
        if constexpr (kLanes) {
            l_seed += (uint32_t)__popcll(__ballot(fresh));
            l_busy += (uint32_t)__popcll(__ballot(active));
        }
        RTK_MARK("seed");
        if constexpr (kWin) {
            // Seed window: the fresh lanes' items are (pixel fq, sample fs); the window holds the
            // generators (after sampleSquare's draws) and pixel sample points of the 64 pixels
            // 64 * win_t + l at sample win_s, computed by all 64 lanes at once.  Each pass serves
            // the fresh lanes of one (pixel group, sample) key, refilling the window first when it
            // holds another: a hand-out that crosses a sample layer or a unit takes two passes.
            // Every lane's generator is seeded and drawn exactly as camera_start does, so the bits
            // are unchanged.
            lds_u32* wp = (lds_u32*)(uintptr_t)win;
            uint64_t todo = __ballot(fresh);
            while (todo != 0) {
                const uint32_t ld = (uint32_t)__builtin_ctzll(todo);
                const uint32_t kt = __builtin_amdgcn_readlane(fq >> 6, ld);
                const uint32_t ks = __builtin_amdgcn_readlane(fs, ld);
                const uint32_t ht = __builtin_amdgcn_readfirstlane(wkey[0]), hs = __builtin_amdgcn_readfirstlane(wkey[1]);
                if (kt != ht || ks != hs) {
                    RTK_MARK("win_fill");
                    if constexpr (kLanes) ++n_fill;
                    if (lane == 0) {
                        wkey[0] = kt;
                        wkey[1] = ks;
                    }
                    const uint32_t q = kt * 64 + lane;  // past the launch's last pixel: computed, never read
                    const uint32_t row_local = fastdiv(q, p.div_width);
                    const uint32_t i = q - row_local * W;
                    const uint32_t j = p.row0 + row_local * p.row_step;
                    Rng gw;
                    gw.seed(sample_key(p.seed_mix, (uint64_t)j * W + i, ks));
                    uint64_t w[7];
                    if constexpr (kF32) {  // fast mode: camera_start's f32 ray direction (2 planes unused)
                        fm::Ray rw;
                        (void)camera_start(i, j, gw, rw);
                        w[4] = (uint64_t)__builtin_bit_cast(uint32_t, rw.dir.x) |
                               ((uint64_t)__builtin_bit_cast(uint32_t, rw.dir.y) << 32);
                        w[5] = __builtin_bit_cast(uint32_t, rw.dir.z);
                        w[6] = 0;
                    } else {
                        const v3 ps = pixel_sample_point(i, j, gw);
                        bool defocus;
                        const v3 center = camera_center(defocus);
                        const v3 dir = defocus ? ps : ps - center;  // camera_start's ray.dir
                        w[4] = __builtin_bit_cast(uint64_t, dir.x);
                        w[5] = __builtin_bit_cast(uint64_t, dir.y);
                        w[6] = __builtin_bit_cast(uint64_t, dir.z);
                    }
                    w[0] = gw.s0;
                    w[1] = gw.s1;
                    w[2] = gw.s2;
                    w[3] = gw.s3;
#pragma unroll
                    for (int k = 0; k < 7; ++k) {
                        wp[(2 * k) * 64 + lane] = (uint32_t)w[k];
                        wp[(2 * k + 1) * 64 + lane] = (uint32_t)(w[k] >> 32);
                    }
                    RTK_MARK("seed");
                }
                if constexpr (kLanes) ++n_take;
                const bool mine = fresh && (fq >> 6) == kt && fs == ks;
                if (mine) {
                    const uint32_t e = fq & 63;
                    uint64_t w[7];
#pragma unroll
                    for (int k = 0; k < 7; ++k)
                        w[k] = (uint64_t)wp[(2 * k) * 64 + e] | ((uint64_t)wp[(2 * k + 1) * 64 + e] << 32);
                    g.s0 = w[0];
                    g.s1 = w[1];
                    g.s2 = w[2];
                    g.s3 = w[3];
                    bool defocus;
                    if constexpr (kF32) {
                        r.orig = camera_center_f32(defocus);
                        r.dir = fm::mk(__builtin_bit_cast(float, (uint32_t)w[4]), __builtin_bit_cast(float, (uint32_t)(w[4] >> 32)),
                                       __builtin_bit_cast(float, (uint32_t)w[5]));
                    } else {
                        r.orig = camera_center(defocus);
                        r.dir = mk(__builtin_bit_cast(double, w[4]), __builtin_bit_cast(double, w[5]),
                                   __builtin_bit_cast(double, w[6]));
                    }
                    dpend = defocus;
                    att = V{1, 1, 1};
                    bounce = 0;
                }
                todo &= ~__ballot(mine);
            }
        } else if (fresh) {
            const uint32_t row_local = fastdiv(fq, p.div_width);
            const uint32_t i = fq - row_local * W;
            const uint32_t j = p.row0 + row_local * p.row_step;
            const uint64_t pixel = (uint64_t)j * W + i;
            g.seed(sample_key(p.seed_mix, pixel, fs));
            dpend = camera_start(i, j, g, r);
            att = V{1, 1, 1};
            bounce = 0;
        }
        if constexpr (kProf) cyc_seed += __builtin_amdgcn_s_memtime() - t_ref;
        RTK_MARK("idle");
        const bool idle = __ballot(active) == 0;
        if (idle) {
            // nothing to trace: finish (no unit left, none held), or claim again next iteration
            if (us.busy == 0 && us.drained) break;
            // a wave that can neither finalise nor claim waits for the previous chunk of a tile
            // another wave holds
            if (!progressed && !us.can_claim() && !us.wait(lane)) break;
            // else: the rest of the iteration runs with every lane idle (no back edge of its own:
            // one measured 17 extra VGPRs)
        }
        uint64_t t_walk0 = 0, t_walk1 = 0;
        if constexpr (kProf) {
            t_walk0 = __builtin_amdgcn_s_memtime();
            cyc_refill += t_walk0 - t_top;
        }

        // ---- rejection loops, at most kRuvTrips trips per iteration ------------------------------
        RTK_MARK("trips");
        // Two rejection samplers draw from a lane's stream: Vec.randomUnitVec (vec.zig:71-80) for a
        // pending Lambertian / Metal scatter (3 draws a trip, mean 1.91 trips) and randomInUnitDisk
        // (vec.zig:82-92) for a new camera ray's defocus sample (2 draws a trip, mean 1.27 trips).
        // A wave pays the maximum trip count over its lanes, so both share ONE capped loop: a lane
        // still rejected after kRuvTrips trips stays pending, skips the next walk and continues
        // drawing where it stopped.  Every lane consumes its own stream in the reference's order,
        // so the bits do not change.
        bool done = false;
        V col = V{0, 0, 0};
        Real ux = 0, uy = 0, uz = 0, uls = 1;
        bool got = false, dgot = false;
        // One trip for the lanes still drawing; leaves the loop when no lane of the wave is.  (A macro:
        // written as a lambda or a function taking the flags by reference, got / dgot went to
        // scratch memory.)
#define RTK_TRIP_BODY                                                                   \
    const bool wr = pending && !got, wd = dpend && !dgot;                               \
    const uint64_t trip_m = __ballot(wr || wd);                                         \
    if (trip_m == 0) break;                                                             \
    if constexpr (kProf) ++n_trip;                                                      \
    if constexpr (kLanes) l_trip += (uint32_t)__popcll(trip_m);                         \
    if constexpr (kF32) {                                                               \
        if (wr || wd) trip_f32(g, wr, ux, uy, uz, uls, got, dgot);                      \
    } else if (wr || wd) {                                                              \
        ux = g.range_pm1();                                                             \
        uy = g.range_pm1();                                                             \
        const double xy = ux * ux + uy * uy;                                            \
        if (wr) {                                                                       \
            uz = g.range_pm1();                                                         \
            uls = xy + uz * uz;                                                         \
        }                                                                               \
        /* Vec.lenSquared of (x, y, 0) for the disk; flags assigned by value (see trip_f32) */ \
        const bool acc = wr ? (1e-160 < uls && uls <= 1) : xy + 0.0 * 0.0 < 1;         \
        got = wr ? acc : got;                                                           \
        dgot = wr ? dgot : acc;                                                         \
    }
#pragma unroll
        for (int k = 0; k < kRuvTrips; ++k) {
            RTK_TRIP_BODY
        }
        if constexpr (kDrainTrips) {
            // drained: no lane will take a new item, so a lane left pending would only cost the wave
            // another pass of the whole loop — draw until every lane has its sample
            if (us.drained)
                while (true) {
                    RTK_TRIP_BODY
                }
        }
#undef RTK_TRIP_BODY
        RTK_MARK("scatter_finish");
        if constexpr (kLanes) {
            const uint64_t mg = __ballot(got), md = __ballot(dgot);
            w_scat += mg != 0 ? 1u : 0u;
            l_scat += (uint32_t)__popcll(mg);
            w_camf += md != 0 ? 1u : 0u;
            l_camf += (uint32_t)__popcll(md);
        }
        if (dgot) {
            RTK_MARK("cam_finish");
            camera_finish(ux, uy, r);
            dpend = false;
            RTK_MARK("scatter_finish");
        }
        if constexpr (kF32) {
            if (got) scatter_f32(ux, uy, uz, uls, sc_metal, sc_nrm, sc_refl, sc_fuzz, pending, done, r, bounce);
        } else if (got) {  // finish the scatter
            RTK_MARK("scat_finish");
            const double l = sqrt_normal(uls);  // |p|^2 in (1e-160, 1] (vec.zig:76)
            const SharedRcp rl(l);
            const v3 ruv = mk(rl.div(ux), rl.div(uy), rl.div(uz));  // p / sqrt(|p|^2), true divisions
            // the new direction is written in place: an absorbed ray's direction is never read again
            bool absorbed = false;
            if (!sc_metal) {
                r.dir = sc_nrm + ruv;
                if (near_zero(r.dir)) r.dir = sc_nrm;
            } else {
                r.dir = sc_refl + muls(ruv, sc_fuzz);  // unit(reflect(ray.dir, n)) + fuzz * ruv
                absorbed = !(dot(r.dir, sc_nrm) > 0);  // absorbed -> black
            }
            pending = false;
            if (absorbed) {
                done = true;
            } else {
                ++bounce;
            }
        }
        // ---- trace one ray segment per ready lane (rayColor's loop body, camera.zig:153-177) ---
        RTK_MARK("walk_setup");
        // Lambertian and Metal scatters draw their randomUnitVec in the next iteration's trip loop
        if constexpr (kProf) {  // the trip loop counts as shading
            const uint64_t t = __builtin_amdgcn_s_memtime();
            cyc_trips += t - t_walk0;
            t_walk0 = t;
        }
        bool shaded = false;  // kProf: this lane ran the shading below
        if constexpr (kProf) {
            const bool walks = active && !done && !pending && !dpend && bounce < p.bounce_max;
            const uint64_t ms = __ballot(walks && !susp);
            n_wstart += ms != 0 ? 1u : 0u;
            if constexpr (kLanes) {
                const uint64_t mw = __ballot(walks);
                l_wstart += (uint32_t)__popcll(ms);
                w_walk += mw != 0 ? 1u : 0u;
                l_walk += (uint32_t)__popcll(mw);
                sh_kind = 3;
            }
        }
        if (active && !done && !pending && !dpend) {
            if (bounce >= p.bounce_max) {
                done = true;  // too many bounces -> black (camera.zig:181)
            } else {
                Real t;
                if (!susp) ++rays;
                uint64_t v0 = 0, t0 = 0;
                if constexpr (kProf) { v0 = pr.n_visits; t0 = pr.n_tests; }
                // The walk is a chain of dependent LDS reads: raised issue priority lets a wave whose
                // node data has arrived issue its next step ahead of the co-resident waves' shading
                // and sampling work (-0.8% kernel time; the finalisation above likewise, -0.2%; a
                // raised priority everywhere but the trip loop was slower).  The shading that follows
                // (dependent loads of the hit sphere's records) runs at priority 1 (chapter 13 -1.3%).
                __builtin_amdgcn_s_setprio(2);
                int k;
                if constexpr (kSusp) {
                    k = walk.template run<true>(r, (Real)p.t_min, (Real)p.t_max, &t, pr, ws, susp,
                                                !(kDrainMode && us.drained));
                    susp = k == kSuspended;
                } else {
                    k = walk(r, (Real)p.t_min, (Real)p.t_max, &t, pr);
                }
                __builtin_amdgcn_s_setprio(1);
                RTK_MARK("shade");
                if constexpr (kProf) {
                    if (bounce == 0) { pr.cam_visits += pr.n_visits - v0; pr.cam_tests += pr.n_tests - t0; }
                }
                if constexpr (kProf) {
                    t_walk1 = __builtin_amdgcn_s_memtime();
                    shaded = !susp;
                }
                if constexpr (kF32) {
                    if (k >= 0 && !bounds_ok((uint32_t)k < p.n_spheres, ua.ctr)) k = -1;
                    if (!susp) shade_f32(k, t, geo_orig, mat_g, g, r, att, col, done, pending, sc_metal, sc_fuzz, sc_nrm,
                                         sc_refl, bounce);
                } else if (!susp) {  // a suspended walk resumes next iteration; nothing to shade yet
                // Three branches below need a unit vector: the sky (unit(ray.dir).y), the
                // dielectric (unit(ray.dir)) and the metal (unit(reflect(ray.dir, n))).  Each is a
                // correctly rounded sqrt and division, and a wave executes every branch some lane
                // takes; so each lane selects its vector first and one unit() serves all three.
                // The hit record and material are computed by EVERY shaded lane, the sky lanes on
                // sphere 0's records (their values are never used): a wave runs this block whenever
                // any lane hit, so the sky lanes cost no extra issue, and without the divergent
                // `if (k >= 0)` there is no merge of the hit values with placeholder ones (the
                // compiler zeroed 12 registers per iteration for it, and copied ray.dir).
                if (k >= 0 && !bounds_ok((uint32_t)k < p.n_spheres, ua.ctr)) k = -1;
                const bool hit = k >= 0;
                const uint32_t kk = hit ? (uint32_t)k : 0u;
                const GeoRec sg = geo_orig[kk];
                const MatRec m = mat_g[kk];
                // hit record (sphere.zig:44-53); a sky lane's t is t_max (inf): its values are unused
                const v3 pt = r.orig + muls(r.dir, t);
                const v3 outward = muls(pt - mk(sg.cx, sg.cy, sg.cz), m.inv_r);
                const bool front = dot(r.dir, outward) < 0;
                const v3 nrm = front ? outward : -outward;
                const uint32_t kind = m.kind;
                const double ri = front ? m.inv_ior : m.ior;        // dielectric: 1.0 / ior precomputed (same bits)
                const double r0 = front ? m.r0_front : m.r0_back;   // Schlick ((1-ri)/(1+ri))^2, host
                // a metal lane's ray.dir is not read again before its scatter finishes (it then
                // takes sc_refl + fuzz * ruv), so the reflected direction replaces it in place
                if (hit && kind == 1) r.dir = reflect(r.dir, nrm);
                if constexpr (kLanes) sh_kind = hit ? (kind <= 1 ? 1u : 2u) : 0u;
                const v3 u = unit(r.dir);
                // The scatter state is read only while `pending`, and a shaded lane was not
                // pending: every shaded lane takes it (and the hit point as its next origin; a sky
                // lane's path ends here), so these are plain writes, not copies under a branch.
                sc_nrm = nrm;
                sc_refl = u;
                sc_fuzz = m.fuzz;
                sc_metal = kind == 1;
                r.orig = pt;
                if (!hit) {
                    // sky gradient (camera.zig:171-177)
                    RTK_MARK("sky");
                    const double a = 0.5 * (u.y + 1.0);
                    const v3 sky = muls(mk(1, 1, 1), 1.0 - a) + muls(mk(0.5, 0.7, 1), a);
                    col = att * sky;
                    done = true;
                } else if (kind <= 1) {
                    // Lambertian (material.zig:27-39) / Metal (:55-68): attenuation = albedo.  A
                    // metal ray that ends up absorbed returns black whatever `att` is, so the
                    // product can be taken now.
                    RTK_MARK("lam_metal");
                    att = att * mk(m.albedo[0], m.albedo[1], m.albedo[2]);
                    pending = true;
                } else {  // Dielectric.scatter (material.zig:82-110), attenuation (1,1,1)
                    RTK_MARK("dielectric");
                    const v3 ud = u;
                    const double cos_t = __builtin_fmin(dot(-ud, nrm), 1.0);
                    const double sin_t = sqrt_g(1.0 - cos_t * cos_t);
                    const bool cannot = ri * sin_t > 1.0;
                    const double approx = r0 + (1 - r0) * zig_pow5(1 - cos_t);
                    // short-circuit `or` (material.zig:94): draw only if refraction is possible
                    const v3 dir = (cannot || approx > g.uniform()) ? reflect(ud, nrm) : refract(ud, nrm, ri);
                    r.dir = dir;
                    ++bounce;
                }
                RTK_MARK("shade");
                }
            }
        }
        __builtin_amdgcn_s_setprio(0);
        if constexpr (kProf) n_shade += __ballot(shaded) != 0 ? 1u : 0u;
        if constexpr (kLanes) {
            l_shade += (uint32_t)__popcll(__ballot(shaded));
            const uint64_t m0 = __ballot(shaded && sh_kind == 0), m1 = __ballot(shaded && sh_kind == 1),
                           m2 = __ballot(shaded && sh_kind == 2), md = __ballot(done);
            w_sky += m0 != 0 ? 1u : 0u;
            l_sky += (uint32_t)__popcll(m0);
            w_lm += m1 != 0 ? 1u : 0u;
            l_lm += (uint32_t)__popcll(m1);
            w_di += m2 != 0 ? 1u : 0u;
            l_di += (uint32_t)__popcll(m2);
            w_store += md != 0 ? 1u : 0u;
            l_store += (uint32_t)__popcll(md);
        }
        RTK_MARK("store");
        if (done) {
            us.store(myslot, mi, col.x, col.y, col.z);
            ++nsamples;
            active = false;
        }
        if constexpr (kProf) {
            // s_memtime is a scalar op: every lane sees the same stamps; lanes that skipped the
            // walk this iteration have t_walk1 == 0 and contribute nothing via the max-reduce below
            const uint64_t t_end = __builtin_amdgcn_s_memtime();
            uint64_t w1 = t_walk1;
            for (int off = 32; off > 0; off >>= 1) {
                const uint64_t o = __shfl_xor(w1, off, 64);
                w1 = o > w1 ? o : w1;
            }
            if (w1 != 0) {
                cyc_walk += w1 - t_walk0;
                cyc_shade += t_end - w1;
            } else {
                cyc_shade += t_end - t_walk0;
            }
        }
    }

    // the previous direct-mode call's reduce pass, taken up by the waves that ran out of items while a
    // few long paths finish elsewhere (rt_render_rows_async_deferred; empty otherwise)
    if constexpr (kDirect && !kProf) {
        if (ua.fold.samples != nullptr) fold_chunks(ua.fold, lane);
    }
    RTK_MARK("epilogue");
    if (stats) {
        // wave-level reduction, one atomic pair per wave (all lanes converged here)
        for (int off = 32; off > 0; off >>= 1) {
            rays += __shfl_xor(rays, off, 64);
            nsamples += __shfl_xor(nsamples, off, 64);
        }
        if (lane == 0) {
            atomicAdd(&stats[0], (unsigned long long)rays);
            atomicAdd(&stats[1], (unsigned long long)nsamples);
        }
        if constexpr (kProf) {
            uint64_t nt = pr.n_tests, nv = pr.n_visits;
            for (int off = 32; off > 0; off >>= 1) {
                nt += __shfl_xor(nt, off, 64);
                nv += __shfl_xor(nv, off, 64);
            }
            uint64_t cv = pr.cam_visits, ct = pr.cam_tests;
            for (int off = 32; off > 0; off >>= 1) {
                cv += __shfl_xor(cv, off, 64);
                ct += __shfl_xor(ct, off, 64);
            }
            if (lane == 0) {
                atomicAdd(&stats[11], (unsigned long long)cv);
                atomicAdd(&stats[12], (unsigned long long)ct);
                // kernel timeline on the constant 100 MHz clock: earliest wave start, earliest queue
                // drain, latest wave end (the host reads [13..15]; 0 = unset, so min via max of ~x)
                const uint64_t rt_end = __builtin_amdgcn_s_memrealtime();
                atomicMax(&stats[13], (unsigned long long)~rt_start);
                atomicMax(&stats[14], (unsigned long long)~rt_drain);
                atomicMax(&stats[15], (unsigned long long)rt_end);
                // drain-tail shape: sum and max over waves of (own end - own drain), last drain
                const uint64_t own_tail = rt_drain ? rt_end - rt_drain : 0;
                atomicAdd(&stats[20], (unsigned long long)own_tail);
                atomicMax(&stats[21], (unsigned long long)own_tail);
                atomicMax(&stats[22], (unsigned long long)rt_drain);
            }
            uint64_t wi = pr.w_inner, wl = pr.w_leaf, wc = pr.w_cand, w2 = pr.w_root2;
            for (int off = 32; off > 0; off >>= 1) {
                wi += __shfl_xor(wi, off, 64);
                wl += __shfl_xor(wl, off, 64);
                wc += __shfl_xor(wc, off, 64);
                w2 += __shfl_xor(w2, off, 64);
            }
            if (lane == 0) {
                atomicAdd(&stats[2], (unsigned long long)nt);
                atomicAdd(&stats[3], (unsigned long long)nv);
                atomicAdd(&stats[7], (unsigned long long)wi);
                atomicAdd(&stats[8], (unsigned long long)wl);
                atomicAdd(&stats[9], (unsigned long long)wc);
                atomicAdd(&stats[10], (unsigned long long)w2);
                atomicAdd(&stats[4], (unsigned long long)cyc_refill);
                atomicAdd(&stats[5], (unsigned long long)cyc_walk);
                atomicAdd(&stats[6], (unsigned long long)cyc_shade);
                atomicAdd(&stats[16], (unsigned long long)cyc_trips);
                atomicAdd(&stats[17], (unsigned long long)us.spins);       // idle-wave sleeps
                atomicAdd(&stats[18], (unsigned long long)us.n_dep_wait);  // deferred finalisations
                atomicAdd(&stats[19], (unsigned long long)us.n_no_slot);   // refills without a free slot
                atomicAdd(&stats[23], (unsigned long long)cyc_fin);        // parts of stats[4]
                atomicAdd(&stats[24], (unsigned long long)cyc_hand);
                atomicAdd(&stats[25], (unsigned long long)cyc_seed);
                atomicAdd(&stats[26], (unsigned long long)n_iter);
                atomicAdd(&stats[27], (unsigned long long)n_trip);
                atomicAdd(&stats[28], (unsigned long long)n_seed);
                atomicAdd(&stats[29], (unsigned long long)n_wstart);
                atomicAdd(&stats[30], (unsigned long long)n_shade);
                atomicAdd(&stats[31], (unsigned long long)n_fin);
            }
        }
        if constexpr (kLanes) {
            if (lane == 0) {
                const uint32_t wu[19] = {l_seed, l_trip, w_scat, l_scat, w_camf, l_camf, w_walk, l_walk, l_wstart,
                                         l_shade, w_sky, l_sky, w_lm, l_lm, w_di, l_di, w_store, l_store, l_busy};
#pragma unroll
                for (int k = 0; k < 19; ++k) atomicAdd(&stats[32 + k], (unsigned long long)wu[k]);
                atomicAdd(&stats[64], (unsigned long long)n_fill);
                atomicAdd(&stats[65], (unsigned long long)n_take);
            }
            // the walker's per-lane counts (leaf rounds, candidate blocks, always-list parts), summed
            // over the wave: stats[51..63]
            uint32_t pl[13] = {pr.l_leaf, pr.l_cand, pr.l_root2, pr.w_acand[0], pr.w_acand[1], pr.w_acand[2],
                               pr.w_acand[3], pr.l_acand[0], pr.l_acand[1], pr.l_acand[2], pr.l_acand[3], pr.w_aroot2,
                               pr.l_aroot2};
#pragma unroll
            for (int k = 0; k < 13; ++k) {
                for (int off = 32; off > 0; off >>= 1) pl[k] += __shfl_xor(pl[k], off, 64);
                if (lane == 0) atomicAdd(&stats[51 + k], (unsigned long long)pl[k]);
            }
        }
    }
}

// Linear-walk kernel: geometry in LDS (kLds) or read by scalar loads from global memory.
template <bool kLds, int U, int kWaves, bool kProf, bool kDirect>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kWaves))) void sample_kernel(
    KernelParams p, const GeoRec* __restrict__ geo_g, const MatRec* __restrict__ mat_g, UnitArgs ua,
    unsigned long long* __restrict__ stats) {
    extern __shared__ GeoRec lds_geo[];
    const GeoRec* geo = geo_g;
    if constexpr (kLds) {
        for (uint32_t k = threadIdx.x; k < p.n_pad; k += blockDim.x) lds_geo[k] = geo_g[k];
        __syncthreads();
        geo = lds_geo;
    }
    // the waves' seed windows after the LDS geometry (kSeedWin; rtk_launch_samples sizes the LDS)
    const uint32_t win = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)(
        (unsigned char*)lds_geo + (kLds ? (size_t)p.n_pad * sizeof(GeoRec) : 0) + (threadIdx.x / 64) * kSeedWinBytes);
    path_loop<kProf, kDirect, kSeedWin>(p, LinearWalker<U>{geo, p.n_pad, p.n_spheres}, geo, mat_g, ua, stats, win);
}

// BVH-walk kernel: nodes + slot geometry + slot ids staged in LDS (kLdsScene) or read from global
// memory; the per-lane traversal stack always lives in LDS.
// The uninstrumented kernels are held to 4 waves per SIMD (128 VGPRs): the LDS-tree kernels fit by
// themselves (127, 125), the global-tree ring kernel (large scenes) took 133 VGPRs, i.e. 3 waves,
// and fits 128 with no spill under the bound.  The instrumented ones (kProf, ~160 VGPRs) keep 3.
// Build knob RTZIG_BVH_WAVES overrides the bound.
#ifdef RTZIG_BVH_WAVES
#define RTK_BVH_WAVES __attribute__((amdgpu_waves_per_eu(RTZIG_BVH_WAVES)))
#else
#define RTK_BVH_WAVES __attribute__((amdgpu_waves_per_eu(kProf ? 3 : 4)))
#endif
// The kernel body, pasted into both entry points below: shared through a __device__ function taking
// the kernel arguments by reference (or by value) the parity kernel compiled to 51 more instructions
// (SGPR constants rematerialised in the loop), 0.6% slower.
#if RTZIG_BOUNDS
#define RTK_BOUNDS_ARGS \
    , b.n_nodes * (uint32_t)sizeof(BvhNode), (uint32_t)(b.n_leaves * sizeof(BvhLeaf)), b.stack_depth, ua.ctr
#else
#define RTK_BOUNDS_ARGS
#endif
#define RTK_BVH_BODY(kF32) \
    /* LDS: [nodes][leaves] (kLdsScene) at address 0, so a node's byte-offset ref IS its LDS */ \
    /* address; then the per-lane stacks [stack_depth][kB]; then the waves' seed windows */ \
    constexpr int kB = bvh_block(kProf); \
    extern __shared__ __align__(16) unsigned char lds_raw[]; \
    const size_t scene_bytes = \
        kLdsScene ? (size_t)bvh_leaves_offset(b.n_nodes) + (size_t)b.n_leaves * sizeof(BvhLeaf) : 0; \
    /* the int16 stack (RTZIG_STACK16) needs every ref in LDS range: the global-memory tree uses int32 */ \
    using Stack = std::conditional_t<kLdsScene, StackEntry, int32_t>; \
    using Walker = BvhWalker<kLdsScene, kB, Stack, kF32>; \
    Stack* stack = (Stack*)(lds_raw + scene_bytes); \
    stack[threadIdx.x] = (Stack)Walker::kEnd;  /* entry 0 of this lane's stack: popping it ends the walk */ \
    const BvhNode* nodes = b.nodes; \
    const BvhLeaf* leaves = b.leaves; \
    if constexpr (kLdsScene) { \
        BvhNode* ln = (BvhNode*)lds_raw; \
        BvhLeaf* ll = (BvhLeaf*)(lds_raw + bvh_leaves_offset(b.n_nodes)); \
        for (uint32_t k = threadIdx.x; k < b.n_nodes; k += blockDim.x) ln[k] = b.nodes[k]; \
        for (uint32_t k = threadIdx.x; k < b.n_leaves; k += blockDim.x) ll[k] = b.leaves[k]; \
        __syncthreads(); \
        nodes = ln; \
        leaves = ll; \
    } \
    /* the wave's seed window after the stacks (kSeedWin: the kernels with the tree in LDS; the */ \
    /* global-memory tree kernels for large scenes keep per-lane seeding, which fits 128 VGPRs) */ \
    const uint32_t win = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)( \
        lds_raw + ((scene_bytes + (size_t)b.stack_depth * kB * sizeof(Stack) + 15) & ~(size_t)15) + \
        (threadIdx.x / 64) * kSeedWinBytes); \
    path_loop<kProf, kDirect, kSeedWin && kLdsScene>(p, Walker{nodes, leaves, b.always_geo, b.always_sid, b.n_always, \
                                         stack + threadIdx.x, b.origin_bound, geo_g, p.n_pad RTK_BOUNDS_ARGS}, geo_g, \
                              mat_g, ua, stats, win);

template <bool kLdsScene, bool kProf, bool kDirect>
__global__ __launch_bounds__(bvh_block(kProf)) RTK_BVH_WAVES void sample_kernel_bvh(KernelParams p, BvhArgs b,
                                                               const GeoRec* __restrict__ geo_g,
                                                               const MatRec* __restrict__ mat_g, UnitArgs ua,
                                                               unsigned long long* __restrict__ stats) {
    RTK_BVH_BODY(false)
}
// Fast mode (RT_PRECISION_F32): the same body in f32, under the same wave bound as the parity kernel
// (4 waves per SIMD; left alone its ring-mode instantiation takes 131 VGPRs, i.e. 3 waves; the
// instrumented builds 3, as for the parity kernel; RTZIG_BVH_WAVES overrides both)
template <bool kLdsScene, bool kProf, bool kDirect>
__global__ __launch_bounds__(bvh_block(kProf)) RTK_BVH_WAVES void sample_kernel_fast(
    KernelParams p, BvhArgs b, const GeoRec* __restrict__ geo_g, const MatRec* __restrict__ mat_g, UnitArgs ua,
    unsigned long long* __restrict__ stats) {
    RTK_BVH_BODY(true)
}
#undef RTK_BVH_BODY

// Direct mode's second pass (rt_kernel.h "Work units"): thread q adds pixel q's stored colors in
// sample order — pixelColor += rayColor(ray), camera.zig:133-136, from pixelColor = 0 — then
// scales (:137) and writes linear f64 or the fused Color.toRgb bytes.  A wave's loads of one sample
// are one contiguous 1536-B run; unrolled 8x to keep loads in flight (the order of the additions
// is unchanged).
template <int kOut>
__global__ __launch_bounds__(256) void reduce_kernel(UnitArgs ua) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= ua.P) return;
    reduce_pixel(ua.samples, ua.P, ua.spp, q, ua.out, kOut, ua.scale);
}

__global__ __launch_bounds__(256) void fold_rest_kernel(FoldArgs f) { fold_chunks(f, lane_id()); }

}  // namespace rtk

// ------------------------------------------------------------------------------------------------
// launch wrappers (called from rt_runtime.cpp)
// ------------------------------------------------------------------------------------------------
// A persistent grid: as many blocks as can be resident (CUs x blocks per CU).  If the occupancy
// query over-reports, the surplus blocks start late and simply find less work.  The device queries
// (and the dynamic-LDS attribute above 64 KiB) are cached per (device, kernel, block, LDS bytes):
// they cost host time between the launch's start event and the kernel, which at 8 GPUs (~9 ms
// frames) is not negligible.
extern "C" hipError_t rtk_resident_blocks(const void* kernel, int block, size_t shmem, uint32_t* blocks) {
    struct Entry {
        int dev;
        const void* kernel;
        int block;
        size_t shmem;
        uint32_t blocks;
    };
    static std::mutex mu;
    static std::vector<Entry> cache;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(mu);
    for (const Entry& c : cache)
        if (c.dev == dev && c.kernel == kernel && c.block == block && c.shmem == shmem) {
            *blocks = c.blocks;
            return hipSuccess;
        }
    if (shmem > 64 * 1024) {
        e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shmem);
        if (e != hipSuccess) return e;
    }
    int cus = 0, per_cu = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, shmem) != hipSuccess || per_cu <= 0)
        per_cu = 1;
    cache.push_back(Entry{dev, kernel, block, shmem, (uint32_t)(cus * per_cu)});
    *blocks = (uint32_t)(cus * per_cu);
    return hipSuccess;
}

namespace {

template <typename K>
uint32_t persistent_blocks(K kernel, size_t shmem) {
    uint32_t b = 0;
    if (rtk_resident_blocks((const void*)kernel, rtk::kBlock, shmem, &b) != hipSuccess) return 1024;
    return b;
}

// blocks of a persistent launch: resident capacity, the work, and (ring mode) the ring's wave capacity
uint32_t grid_blocks(uint64_t need, uint64_t cap, const rtk::UnitArgs* ua, uint32_t block) {
    const uint64_t ring_blocks = ua->ring ? ua->ring_waves / (block / 64) : UINT64_MAX;
    uint64_t b = need < cap ? need : cap;
    return (uint32_t)(b < ring_blocks ? b : ring_blocks);
}

// waves of the persistent grid a launch of `need` blocks would have before the ring's bound: the
// runtime sizes the ring to it (rtk_launch_* with plan_waves != nullptr)
uint32_t plan_of(uint64_t need, uint64_t cap, uint32_t block) {
    return (uint32_t)((need < cap ? need : cap) * (block / 64));
}

template <bool kLds, int U, int kWaves>
void launch_samples(const rtk::KernelParams* p, const rtk::GeoRec* geo, const rtk::MatRec* mat,
                    const rtk::UnitArgs* ua, unsigned long long* st, hipStream_t stream, size_t shmem, uint64_t need,
                    bool direct, uint32_t* plan_waves) {
    auto kernel = p->prof ? (direct ? rtk::sample_kernel<kLds, U, kWaves, true, true> : rtk::sample_kernel<kLds, U, kWaves, true, false>)
                          : (direct ? rtk::sample_kernel<kLds, U, kWaves, false, true> : rtk::sample_kernel<kLds, U, kWaves, false, false>);
    if (plan_waves) {
        *plan_waves = plan_of(need, persistent_blocks(kernel, shmem), rtk::kBlock);
        return;
    }
    const uint32_t blocks = grid_blocks(need, persistent_blocks(kernel, shmem), ua, rtk::kBlock);
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(rtk::kBlock), shmem, stream, *p, geo, mat, *ua, st);
}

// Kernel variant: RTZIG_KERNEL=<geom>_u<U>[_w<waves>], geom in {lds, smem}; default kDefaultVariant.
//   lds  — sphere geometry staged in LDS, read by ds_read_b128 broadcasts
//   smem — geometry read from global memory by scalar loads (s_load_dwordx16), SGPR operands
struct Variant {
    const char* name;
    bool lds;
    int unroll;
    int waves;
};
constexpr Variant kVariants[] = {{"lds_u4", true, 4, 1}, {"smem_u4", false, 4, 1}};

const Variant& variant_choice(bool fits_lds, uint32_t n_pad) {
    const char* e = std::getenv("RTZIG_KERNEL");
    // tiny scenes (the runtime's list-walk case, rt_runtime.cpp use_bvh): LDS broadcasts beat scalar
    // loads there (chapter 13: 9.50 against 9.80 ms at 100 spp)
    const char* want = e ? e : (n_pad <= 8 ? "lds_u4" : rtk::kDefaultVariant);
    for (const Variant& v : kVariants)
        if (std::strcmp(v.name, want) == 0 && (fits_lds || !v.lds)) return v;
    for (const Variant& v : kVariants)
        if (std::strcmp(v.name, rtk::kDefaultVariant) == 0 && (fits_lds || !v.lds)) return v;
    return kVariants[1];  // smem_u4: works for any sphere count
}

}  // namespace

extern "C" hipError_t rtk_launch_samples(const rtk::KernelParams* p, const rtk::GeoRec* geo,
                                         const rtk::MatRec* mat, const rtk::UnitArgs* ua,
                                         void* stats, hipStream_t stream, const char** name, bool direct,
                                         uint32_t* plan_waves) {
    using namespace rtk;
    const uint64_t total = (uint64_t)p->n_rows * p->width * p->s_count;
    if (total == 0) return hipSuccess;
    const Variant& v = variant_choice(p->n_pad <= kMaxLdsSpheres, p->n_pad);
    const size_t shmem = (v.lds ? (size_t)p->n_pad * sizeof(GeoRec) : 0) + (kSeedWin ? (kBlock / 64) * kSeedWinBytes : 0);
    const uint64_t need = (total + kBlock - 1) / kBlock;
    auto* st = (unsigned long long*)stats;
    if (name) *name = v.name;
#define RTK_CASE(L, U, W)                                                                 \
    if (v.lds == L && v.unroll == U && v.waves == W) {                                   \
        launch_samples<L, U, W>(p, geo, mat, ua, st, stream, shmem, need, direct, plan_waves); \
        return hipGetLastError();                                                        \
    }
    RTK_CASE(true, 4, 1) RTK_CASE(false, 4, 1)
#undef RTK_CASE
    return hipErrorInvalidValue;
}

namespace {
template <bool kF32>
hipError_t launch_bvh(const rtk::KernelParams* p, const rtk::BvhArgs* b, const rtk::GeoRec* geo, const rtk::MatRec* mat,
                      const rtk::UnitArgs* ua, void* stats, hipStream_t stream, const char** name, bool direct,
                      uint32_t* plan_waves) {
    using namespace rtk;
    const uint64_t total = (uint64_t)p->n_rows * p->width * p->s_count;
    if (total == 0) return hipSuccess;
    if (b->stack_depth < 2 || b->stack_depth > (uint32_t)kMaxDepthBvh) return hipErrorInvalidValue;
    const bool prof = p->prof != 0;
    const uint32_t block = (uint32_t)bvh_block(prof);
    const size_t scene_bytes = (size_t)bvh_leaves_offset(b->n_nodes) + (size_t)b->n_leaves * sizeof(BvhLeaf);
    // int16 stack entries (RTZIG_STACK16) hold node and leaf byte offsets below 2^15
    const bool refs16 = bvh_leaves_offset(b->n_nodes) < 32768u && (size_t)b->n_leaves * sizeof(BvhLeaf) < 32768u;
    const size_t lds_entry = refs16 ? sizeof(StackEntry) : sizeof(int32_t);
    // scene in LDS when the block's share of a CU holds tree + stacks + seed windows (kLdsSceneBudget)
    const bool lds_scene = (size_t)b->stack_depth * block * lds_entry + scene_bytes <=
                               (prof ? kLdsSceneBudgetProf : kLdsSceneBudget) &&
                           (sizeof(StackEntry) == sizeof(int32_t) || refs16);
    const size_t stack_bytes = (size_t)b->stack_depth * block * (lds_scene ? sizeof(StackEntry) : sizeof(int32_t));
    // + the waves' seed windows (kSeedWin, the f64 kernel with the tree in LDS), 16-B aligned after the stacks
    const size_t shmem = (((lds_scene ? scene_bytes : 0) + stack_bytes + 15) & ~(size_t)15) +
                         (!lds_scene ? 0 : (prof ? kSeedWinProfBytes : kSeedWinBlockBytes));
    const uint64_t need = (total + block - 1) / block;
    auto* st = (unsigned long long*)stats;
    auto launch = [&](auto kernel, const char* nm) -> hipError_t {
        uint32_t cap32 = 0;
        const hipError_t ea = rtk_resident_blocks((const void*)kernel, (int)block, shmem, &cap32);
        if (ea != hipSuccess) return ea;
        if (plan_waves) {
            *plan_waves = plan_of(need, cap32, block);
            return hipSuccess;
        }
        const uint32_t blocks = grid_blocks(need, cap32, ua, block);
        if (name) *name = nm;
        hipLaunchKernelGGL(kernel, dim3(blocks), dim3(block), shmem, stream, *p, *b, geo, mat, *ua, st);
        return hipGetLastError();
    };
#define RTK_BVH(L, PR, D, NM)                                                                          \
    if (lds_scene == L && prof == PR && direct == D) {                                                 \
        if constexpr (kF32) return launch(sample_kernel_fast<L, PR, D>, NM);                           \
        else return launch(sample_kernel_bvh<L, PR, D>, NM);                                           \
    }
    if constexpr (kF32) {
        RTK_BVH(true, true, true, "fast_f32_lds(prof,direct)") RTK_BVH(false, true, true, "fast_f32_global(prof,direct)")
        RTK_BVH(true, false, true, "fast_f32_lds(direct)") RTK_BVH(false, false, true, "fast_f32_global(direct)")
        RTK_BVH(true, true, false, "fast_f32_lds(prof)") RTK_BVH(false, true, false, "fast_f32_global(prof)")
        RTK_BVH(true, false, false, "fast_f32_lds") RTK_BVH(false, false, false, "fast_f32_global")
    } else {
        RTK_BVH(true, true, true, "bvh_lds(prof,direct)") RTK_BVH(false, true, true, "bvh_global(prof,direct)")
        RTK_BVH(true, false, true, "bvh_lds(direct)") RTK_BVH(false, false, true, "bvh_global(direct)")
        RTK_BVH(true, true, false, "bvh_lds(prof)") RTK_BVH(false, true, false, "bvh_global(prof)")
        RTK_BVH(true, false, false, "bvh_lds") RTK_BVH(false, false, false, "bvh_global")
    }
#undef RTK_BVH
    return hipErrorInvalidValue;
}
}  // namespace

extern "C" hipError_t rtk_launch_samples_bvh(const rtk::KernelParams* p, const rtk::BvhArgs* b,
                                             const rtk::GeoRec* geo, const rtk::MatRec* mat, const rtk::UnitArgs* ua,
                                             void* stats, hipStream_t stream, const char** name, bool direct,
                                             uint32_t* plan_waves) {
    return launch_bvh<false>(p, b, geo, mat, ua, stats, stream, name, direct, plan_waves);
}

// Fast mode (RT_PRECISION_F32): the same kernel instantiated with kF32 = true.
extern "C" hipError_t rtk_launch_samples_fast(const rtk::KernelParams* p, const rtk::BvhArgs* b, const rtk::GeoRec* geo,
                                              const rtk::MatRec* mat, const rtk::UnitArgs* ua, void* stats,
                                              hipStream_t stream, const char** name, bool direct,
                                              uint32_t* plan_waves) {
    return launch_bvh<true>(p, b, geo, mat, ua, stats, stream, name, direct, plan_waves);
}

extern "C" hipError_t rtk_launch_fold_rest(const rtk::FoldArgs* f, hipStream_t stream) {
    using namespace rtk;
    if (f->samples == nullptr || f->n_chunks == 0) return hipErrorInvalidValue;
    const uint32_t blocks = (f->n_chunks + 3) / 4;  // at most one wave per chunk; the rest exit at once
    hipLaunchKernelGGL(fold_rest_kernel, dim3(blocks), dim3(256), 0, stream, *f);
    return hipGetLastError();
}

extern "C" hipError_t rtk_launch_reduce(const rtk::UnitArgs* ua, hipStream_t stream) {
    using namespace rtk;
    if (ua->P == 0 || ua->samples == nullptr) return hipErrorInvalidValue;
    const uint32_t blocks = (ua->P + 255) / 256;
    if (ua->out_format == 0)
        hipLaunchKernelGGL(reduce_kernel<0>, dim3(blocks), dim3(256), 0, stream, *ua);
    else
        hipLaunchKernelGGL(reduce_kernel<1>, dim3(blocks), dim3(256), 0, stream, *ua);
    return hipGetLastError();
}

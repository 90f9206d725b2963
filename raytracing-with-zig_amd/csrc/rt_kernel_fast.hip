// rt_kernel_fast.hip — RT_PRECISION_F32: the hot path of Camera.render (reference
// src/camera.zig:123-145) in f32 arithmetic on gfx950.
//
// The parity kernel (rt_kernel.hip) restates the reference's f64 arithmetic bit for bit.  This one
// keeps its structure — persistent waves pulling (sample, pixel) items from one queue, the BVH in
// LDS walked while-while, the capped rejection-trip loop, per-sample color stores reduced by the same
// ordered reduce kernel — but shades, samples and intersects in f32, where gfx950 has
// single-instruction reciprocal / rsqrt / sqrt and FMA is allowed.  Parity is statistical
// (tests/test_fast_mode.py, DESIGN.md "Fast mode").
//
// Precision guard: huge spheres on the BVH's always-list (radius >= 100 or far out, e.g. the final
// scene's r = 1000 ground, rt_bvh.cpp) are tested in f64; the big ones (its r = 1 spheres) in f32.  In f32 a point on a radius-1000 sphere is only
// known to ~6e-5 along the normal, so secondary rays leaving it would re-hit it ("acne") at grazing
// angles; every other sphere's quadratic is well conditioned in f32 at t_min = 1e-3.
//
// The RNG stream of a (pixel, sample) is the parity kernel's (rt_sample_key + DefaultPrng.init); a
// uniform is 24 bits of a Xoshiro256++ word, paired draws take both halves of one word.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstddef>

#include "rt_device.h"
#include "rt_kernel.h"
#include "rt_units.h"

#pragma clang fp contract(fast)

namespace rtf {

using rtk::BvhArgs;
using rtk::BvhLeaf;
using rtk::BvhNode;
using rtk::GeoRec;
using rtk::KernelParams;
using rtk::kBlockBvh;
using rtk::UnitArgs;
using rtk::UnitSched;
using rtk::kLeafBvh;
using rtk::MatRec;
using rtk::Rng;

struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
__device__ __forceinline__ f3 muls(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float len_sq(f3 a) { return dot(a, a); }
__device__ __forceinline__ f3 unit(f3 a) { return muls(a, __builtin_amdgcn_rsqf(len_sq(a))); }
__device__ __forceinline__ f3 reflect(f3 v, f3 n) { return v - muls(n, 2.0f * dot(v, n)); }
__device__ __forceinline__ f3 refract(f3 v, f3 n, float eta) {
    const float cos_t = __builtin_fminf(-dot(v, n), 1.0f);
    const f3 r_perp = muls(v + muls(n, cos_t), eta);
    return r_perp - muls(n, __builtin_sqrtf(__builtin_fabsf(1.0f - len_sq(r_perp))));
}
__device__ __forceinline__ bool near_zero(f3 v) { return v.x < 1e-8f && v.y < 1e-8f && v.z < 1e-8f; }  // vec.zig:26-29

// U[0, 1) from the top 24 bits of one Xoshiro256++ word (exact in f32); uniform2 takes two from one
// word (the top 24 bits of each 32-bit half), halving the generator work of paired draws
__device__ __forceinline__ float uniform(Rng& g) { return (float)(uint32_t)(g.next() >> 40) * 0x1p-24f; }
__device__ __forceinline__ void uniform2(Rng& g, float& a, float& b) {
    const uint64_t w = g.next();
    a = (float)(uint32_t)(w >> 40) * 0x1p-24f;
    b = (float)((uint32_t)w >> 8) * 0x1p-24f;
}
__device__ __forceinline__ float pm1(float u) { return __builtin_fmaf(2.0f, u, -1.0f); }
__device__ __forceinline__ float range_pm1(Rng& g) { return pm1(uniform(g)); }

struct Ray {
    f3 orig, dir;
};

typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kFcam = (int)offsetof(KernelParams, fcam);
static_assert(kFcam % 4 == 0, "fcam kernarg offset");
__device__ __forceinline__ float f(uint32_t w) { return __builtin_bit_cast(float, w); }

// getRay (camera.zig:187-215) in f32; like the parity kernel, the defocus disk sample is drawn by
// the trip loop (camera_start returns true while it is pending; r.dir holds the pixel sample point)
__device__ __forceinline__ bool camera_start(uint32_t i, uint32_t j, Rng& g, Ray& r) {
    u32x16 A;  // fcam[0..15]
    u32x4 B;   // fcam[16..19]
    const uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile(
        "s_load_dwordx16 %0, %2, %3\n\t"
        "s_load_dwordx4 %1, %2, %4\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=s"(A), "=s"(B)
        : "s"(kp), "i"(kFcam), "i"(kFcam + 64));
    const f3 center = mk(f(A[0]), f(A[1]), f(A[2]));
    const f3 p0 = mk(f(A[3]), f(A[4]), f(A[5]));
    const f3 du = mk(f(A[6]), f(A[7]), f(A[8]));
    const f3 dv = mk(f(A[9]), f(A[10]), f(A[11]));
    const float defocus_angle = f(B[2]);
    float ox, oy;
    uniform2(g, ox, oy);
    ox -= 0.5f;
    oy -= 0.5f;
    const f3 ps = (p0 + muls(du, (float)i + ox)) + muls(dv, (float)j + oy);
    r.orig = center;
    if (defocus_angle <= 0) {
        r.dir = ps - center;
        return false;
    }
    r.dir = ps;
    return true;
}
__device__ __forceinline__ void camera_finish(float px, float py, Ray& r) {
    u32x16 A;
    u32x4 B;
    const uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile(
        "s_load_dwordx16 %0, %2, %3\n\t"
        "s_load_dwordx4 %1, %2, %4\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=s"(A), "=s"(B)
        : "s"(kp), "i"(kFcam), "i"(kFcam + 64));
    const f3 center = mk(f(A[0]), f(A[1]), f(A[2]));
    const f3 ddu = mk(f(A[12]), f(A[13]), f(A[14]));
    const f3 ddv = mk(f(A[15]), f(B[0]), f(B[1]));
    const f3 origin = (center + muls(ddu, px)) + muls(ddv, py);
    r.dir = r.dir - origin;
    r.orig = origin;
}

__device__ __forceinline__ uint32_t lane_id() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint32_t rank_in(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

constexpr int32_t kDone = INT32_MIN;
typedef float f2 __attribute__((ext_vector_type(2)));
typedef int32_t i2 __attribute__((ext_vector_type(2)));
template <class T>
__device__ __forceinline__ void lds_b64(T& v, uint32_t addr, int off) {
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
}
__device__ __forceinline__ void lds_b32(int32_t& v, uint32_t addr, int off) {
    asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
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

// Closest hit: always-list spheres in f64, then the BVH (same nodes and traversal as the parity
// kernel's BvhWalker) with f32 leaf tests.  Returns the original sphere index or -1.
template <bool kLdsNodes>
struct Walker {
    const BvhNode* __restrict__ nodes;
    const BvhLeaf* __restrict__ leaves;
    const GeoRec* __restrict__ ageo;
    const uint32_t* __restrict__ asid;
    uint32_t n_always;
    int32_t* stack;
    float origin_bound;

    __device__ __forceinline__ int operator()(const Ray& r, float t_min, float t_max, float* t_hit) const {
        int best = -1;
        float closest = t_max;
        if (n_always) {  // f64: see the header comment
            const double ox = r.orig.x, oy = r.orig.y, oz = r.orig.z;
            const double dx = r.dir.x, dy = r.dir.y, dz = r.dir.z;
            const double a = (dx * dx + dy * dy) + dz * dz;
            double cl = (double)t_max;
            for (uint32_t q = 0; q < n_always; ++q) {
                const GeoRec s = ageo[q];
                if (s.r2 < 1e4 && __builtin_fabs(s.cx) + __builtin_fabs(s.cy) + __builtin_fabs(s.cz) < 1e4) {
                    // a big but not huge sphere (radius < 100): well conditioned in f32
                    const float fx = (float)s.cx - r.orig.x, fy = (float)s.cy - r.orig.y, fz = (float)s.cz - r.orig.z;
                    const float fa = len_sq(r.dir);
                    const float h = r.dir.x * fx + r.dir.y * fy + r.dir.z * fz;
                    const float c = (fx * fx + fy * fy + fz * fz) - (float)s.r2;
                    const float disc = h * h - fa * c;
                    if (disc >= 0) {
                        const float sq = __builtin_sqrtf(disc), ia = __builtin_amdgcn_rcpf(fa);
                        float ts = (h - sq) * ia;
                        if (!(t_min < ts)) ts = (h + sq) * ia;
                        if (t_min < ts && (double)ts < cl) {
                            cl = ts;
                            best = (int)asid[q];
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
                        best = (int)asid[q];
                    }
                }
            }
            closest = best >= 0 ? (float)cl : t_max;
        }

        const float a = len_sq(r.dir);
        const float inv_a = __builtin_amdgcn_rcpf(a);
        float dx = r.dir.x, dy = r.dir.y, dz = r.dir.z;
        if (__builtin_fabsf(dx) < 1e-30f) dx = __builtin_copysignf(1e-30f, dx);
        if (__builtin_fabsf(dy) < 1e-30f) dy = __builtin_copysignf(1e-30f, dy);
        if (__builtin_fabsf(dz) < 1e-30f) dz = __builtin_copysignf(1e-30f, dz);
        const float ix = __builtin_amdgcn_rcpf(dx), iy = __builtin_amdgcn_rcpf(dy), iz = __builtin_amdgcn_rcpf(dz);
        const uint32_t ax = ix < 0 ? 8u : 0u, ay = 16u + (iy < 0 ? 8u : 0u), az = 32u + (iz < 0 ? 8u : 0u);
        // origins outside the boxes' origin bound cull nothing (see rtk::BvhArgs::origin_bound)
        const bool far = __builtin_fmaxf(__builtin_fmaxf(__builtin_fabsf(r.orig.x), __builtin_fabsf(r.orig.y)),
                                         __builtin_fabsf(r.orig.z)) > origin_bound;
        const f2 inv_x = {ix, ix}, inv_y = {iy, iy}, inv_z = {iz, iz};
        const f2 noi_x = {-(r.orig.x * ix), -(r.orig.x * ix)}, noi_y = {-(r.orig.y * iy), -(r.orig.y * iy)},
                 noi_z = {-(r.orig.z * iz), -(r.orig.z * iz)};
        const float lower = t_min;
        float upper = closest;

        int32_t* top = stack;
        int32_t cur = 0;
        while (cur != kDone) {
            while (cur >= 0) {
                f2 bx0, by0, bz0, bx1, by1, bz1;
                int32_t ref0, ref1, popped;
                if constexpr (kLdsNodes) {
                    const uint32_t ad = (uint32_t)cur;
                    i2 refs;
                    lds_b64(bx0, ad + ax, 0); lds_b64(bx1, ad + ax, 48);
                    lds_b64(by0, ad + ay, 0); lds_b64(by1, ad + ay, 48);
                    lds_b64(bz0, ad + az, 0); lds_b64(bz1, ad + az, 48);
                    lds_b64(refs, ad, 96);
                    lds_b32(popped, lds_addr(top), 0);
                    asm volatile("s_waitcnt lgkmcnt(0)"
                                 : "+v"(bx0), "+v"(bx1), "+v"(by0), "+v"(by1), "+v"(bz0), "+v"(bz1), "+v"(refs),
                                   "+v"(popped));
                    ref0 = refs.x;
                    ref1 = refs.y;
                } else {
                    const char* nb = (const char*)nodes + cur;
                    bx0 = *(const f2*)(nb + ax); by0 = *(const f2*)(nb + ay); bz0 = *(const f2*)(nb + az);
                    bx1 = *(const f2*)(nb + 48 + ax); by1 = *(const f2*)(nb + 48 + ay); bz1 = *(const f2*)(nb + 48 + az);
                    ref0 = *(const int32_t*)(nb + 96);
                    ref1 = *(const int32_t*)(nb + 100);
                    popped = *top;
                }
                const f2 tx0 = __builtin_elementwise_fma(bx0, inv_x, noi_x);
                const f2 ty0 = __builtin_elementwise_fma(by0, inv_y, noi_y);
                const f2 tz0 = __builtin_elementwise_fma(bz0, inv_z, noi_z);
                const f2 tx1 = __builtin_elementwise_fma(bx1, inv_x, noi_x);
                const f2 ty1 = __builtin_elementwise_fma(by1, inv_y, noi_y);
                const f2 tz1 = __builtin_elementwise_fma(bz1, inv_z, noi_z);
                const float n0 = slab_near(tx0.x, ty0.x, tz0.x, lower), f0 = slab_far(tx0.y, ty0.y, tz0.y, upper);
                const float n1 = slab_near(tx1.x, ty1.x, tz1.x, lower), f1 = slab_far(tx1.y, ty1.y, tz1.y, upper);
                const bool h0 = n0 <= f0 || far;
                const bool h1 = n1 <= f1 || far;
                const bool first0 = n0 <= n1;
                top[kBlockBvh] = first0 ? ref1 : ref0;
                const bool pick0 = h0 && (!h1 || first0);
                cur = (h0 || h1) ? (pick0 ? ref0 : ref1) : popped;
                top += (h0 && h1) ? kBlockBvh : ((h0 || h1) ? 0 : -kBlockBvh);
            }
            if (cur != kDone) {
                const BvhLeaf* lf = (const BvhLeaf*)((const char*)leaves + (uint32_t)(~cur));
#pragma unroll
                for (int u = 0; u < kLeafBvh; ++u) {
                    const rtk::LeafGeo s = lf->g[u];
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
                            best = (int)lf->sid[u];
                        }
                    }
                }
                upper = closest;
                cur = *top;
                top -= kBlockBvh;
            }
        }
        *t_hit = closest;
        return best;
    }
};

template <bool kDirect, class Walker>
__device__ __forceinline__ void path_loop(const KernelParams& p, const Walker& walk, const GeoRec* __restrict__ geo_orig,
                                          const MatRec* __restrict__ mat_g, const UnitArgs& ua,
                                          unsigned long long* __restrict__ stats) {
    const uint32_t W = p.width;
    const uint32_t lane = lane_id();
    const float t_min = (float)p.t_min, t_max = (float)p.t_max;

    UnitSched<kDirect> us(ua, blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64);  // as the parity kernel
    bool active = false, pending = false, sc_metal = false, dpend = false;
    uint32_t myslot = 0, mi = 0;
    Rng g;
    Ray r;
    f3 att = mk(1, 1, 1), sc_nrm = mk(0, 0, 0), sc_refl = mk(0, 0, 0);
    float sc_fuzz = 0;
    uint32_t bounce = 0;
    uint64_t rays = 0, nsamples = 0;

    while (true) {
        // ---- finalise one unit whose samples have all ended (rt_units.h) --------------------------
        __builtin_amdgcn_s_setprio(2);
        const bool progressed = us.finalize_one(us.ready_mask(active, myslot), lane);
        __builtin_amdgcn_s_setprio(0);
        // ---- refill (as the parity kernel's path_loop) -----------------------------------------
        bool fresh = false;
        uint32_t fq = 0, fs = 0;
        us.refill(active, fresh, myslot, mi, fq, fs, lane);
        // the lanes handed an item above start their path: seeding and getRay run once, outside
        // the claim loop, so the generator state and ray are not loop-carried through it
        if (fresh) {
            const uint32_t row_local = rtk::fastdiv(fq, p.div_width);
            const uint32_t i = fq - row_local * W;
            const uint32_t j = p.row0 + row_local * p.row_step;
            g.seed(rtk::sample_key(p.seed_mix, (uint64_t)j * W + i, fs));
            dpend = camera_start(i, j, g, r);
            att = mk(1, 1, 1);
            bounce = 0;
        }
        const bool idle = __ballot(active) == 0;
        if (idle) {
            if (us.busy == 0 && us.drained) break;
            // a wave that can neither finalise nor claim waits for the previous chunk of a tile
            // another wave holds
            if (!progressed && !us.can_claim() && !us.wait(lane)) break;
            // else: the rest of the iteration runs with every lane idle (no back edge of its own:
            // one measured 17 extra VGPRs)
        }

        // ---- one capped loop for randomUnitVec and randomInUnitDisk trips ----------------------
        bool done = false;
        f3 col = mk(0, 0, 0);
        float ux = 0, uy = 0, uz = 0, uls = 1;
        bool got = false, dgot = false;
        for (int trip = 0; trip < rtk::kRuvTrips; ++trip) {
            const bool wr = pending && !got, wd = dpend && !dgot;
            if (__ballot(wr || wd) == 0) break;
            if (wr || wd) {
                uniform2(g, ux, uy);
                ux = pm1(ux);
                uy = pm1(uy);
                const float xy = ux * ux + uy * uy;
                if (wr) {
                    uz = range_pm1(g);
                    uls = xy + uz * uz;
                    got = 1e-30f < uls && uls <= 1.0f;
                } else {
                    dgot = xy < 1.0f;
                }
            }
        }
        if (dgot) {
            camera_finish(ux, uy, r);
            dpend = false;
        }
        if (got) {
            const f3 ruv = muls(mk(ux, uy, uz), __builtin_amdgcn_rsqf(uls));
            f3 dir;
            bool absorbed = false;
            if (!sc_metal) {
                dir = sc_nrm + ruv;
                if (near_zero(dir)) dir = sc_nrm;
            } else {
                dir = sc_refl + muls(ruv, sc_fuzz);
                absorbed = !(dot(dir, sc_nrm) > 0);
            }
            pending = false;
            if (absorbed) {
                done = true;
            } else {
                r.dir = dir;
                ++bounce;
            }
        }

        // ---- one ray segment per ready lane (rayColor's loop body, camera.zig:153-177) ---------
        if (active && !done && !pending && !dpend) {
            if (bounce >= p.bounce_max) {
                done = true;
            } else {
                float t;
                ++rays;
                __builtin_amdgcn_s_setprio(2);  // as the parity kernel (rt_kernel.hip, path_loop)
                const int k = walk(r, t_min, t_max, &t);
                __builtin_amdgcn_s_setprio(0);
                MatRec m{};
                f3 pt = mk(0, 0, 0), nrm = mk(0, 0, 0);
                bool front = false;
                f3 x = r.dir;
                uint32_t kind = 0;
                if (k >= 0) {
                    const GeoRec sg = geo_orig[k];
                    m = mat_g[k];
                    kind = m.kind;
                    pt = r.orig + muls(r.dir, t);
                    const f3 outward = muls(pt - mk((float)sg.cx, (float)sg.cy, (float)sg.cz), (float)m.inv_r);
                    front = dot(r.dir, outward) < 0;
                    nrm = front ? outward : -outward;
                    if (kind == 1) x = reflect(r.dir, nrm);
                }
                const f3 u = unit(x);
                if (k < 0) {
                    const float a = 0.5f * (u.y + 1.0f);
                    col = att * (muls(mk(1, 1, 1), 1.0f - a) + muls(mk(0.5f, 0.7f, 1.0f), a));
                    done = true;
                } else if (kind <= 1) {
                    att = att * mk((float)m.albedo[0], (float)m.albedo[1], (float)m.albedo[2]);
                    pending = true;
                    sc_metal = kind == 1;
                    sc_fuzz = (float)m.fuzz;
                    sc_nrm = nrm;
                    sc_refl = u;
                    r.orig = pt;
                } else {
                    const float ri = front ? (float)m.inv_ior : (float)m.ior;
                    const float cos_t = __builtin_fminf(-dot(u, nrm), 1.0f);
                    const float sin_t = __builtin_sqrtf(__builtin_fmaxf(1.0f - cos_t * cos_t, 0.0f));
                    const bool cannot = ri * sin_t > 1.0f;
                    const float r0 = front ? (float)m.r0_front : (float)m.r0_back;
                    const float x1 = 1.0f - cos_t, x2 = x1 * x1;
                    const float approx = r0 + (1.0f - r0) * (x1 * (x2 * x2));
                    r.dir = (cannot || approx > uniform(g)) ? reflect(u, nrm) : refract(u, nrm, ri);
                    r.orig = pt;
                    ++bounce;
                }
            }
        }
        if (done) {
            us.store(myslot, mi, col.x, col.y, col.z);
            ++nsamples;
            active = false;
        }
    }
    if (stats) {
        for (int off = 32; off > 0; off >>= 1) {
            rays += __shfl_xor(rays, off, 64);
            nsamples += __shfl_xor(nsamples, off, 64);
        }
        if (lane == 0) {
            atomicAdd(&stats[0], (unsigned long long)rays);
            atomicAdd(&stats[1], (unsigned long long)nsamples);
        }
    }
}

template <bool kLdsScene, bool kDirect>
__global__ __launch_bounds__(kBlockBvh) void sample_kernel_fast(KernelParams p, BvhArgs b,
                                                                const GeoRec* __restrict__ geo_g,
                                                                const MatRec* __restrict__ mat_g, UnitArgs ua,
                                                                unsigned long long* __restrict__ stats) {
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const size_t scene_bytes =
        kLdsScene ? (size_t)rtk::bvh_leaves_offset(b.n_nodes) + (size_t)b.n_leaves * sizeof(BvhLeaf) : 0;
    int32_t* stack = (int32_t*)(lds_raw + scene_bytes);
    stack[threadIdx.x] = kDone;
    const BvhNode* nodes = b.nodes;
    const BvhLeaf* leaves = b.leaves;
    if constexpr (kLdsScene) {
        BvhNode* ln = (BvhNode*)lds_raw;
        BvhLeaf* ll = (BvhLeaf*)(lds_raw + rtk::bvh_leaves_offset(b.n_nodes));
        for (uint32_t k = threadIdx.x; k < b.n_nodes; k += blockDim.x) ln[k] = b.nodes[k];
        for (uint32_t k = threadIdx.x; k < b.n_leaves; k += blockDim.x) ll[k] = b.leaves[k];
        __syncthreads();
        nodes = ln;
        leaves = ll;
    }
    path_loop<kDirect>(p, Walker<kLdsScene>{nodes, leaves, b.always_geo, b.always_sid, b.n_always, stack + threadIdx.x, b.origin_bound},
              geo_g, mat_g, ua, stats);
}

}  // namespace rtf

extern "C" hipError_t rtk_launch_samples_fast(const rtk::KernelParams* p, const rtk::BvhArgs* b,
                                              const rtk::GeoRec* geo, const rtk::MatRec* mat, const rtk::UnitArgs* ua,
                                              void* stats, hipStream_t stream, const char** name) {
    using namespace rtk;
    const uint64_t total = (uint64_t)p->n_rows * p->width * p->s_count;
    if (total == 0) return hipSuccess;
    if (b->stack_depth < 2 || b->stack_depth > (uint32_t)kMaxDepthBvh) return hipErrorInvalidValue;
    const size_t stack_bytes = (size_t)b->stack_depth * kBlockBvh * sizeof(int32_t);
    const size_t scene_bytes = (size_t)bvh_leaves_offset(b->n_nodes) + (size_t)b->n_leaves * sizeof(BvhLeaf);
    const bool lds_scene = stack_bytes + scene_bytes <= kLdsSceneBudget;
    const size_t shmem = stack_bytes + (lds_scene ? scene_bytes : 0);
    const uint64_t need = (total + kBlockBvh - 1) / kBlockBvh;
    auto launch = [&](auto kernel, const char* nm) -> hipError_t {
        uint32_t cap32 = 0;
        const hipError_t ea = rtk_resident_blocks((const void*)kernel, kBlockBvh, shmem, &cap32);
        if (ea != hipSuccess) return ea;
        uint64_t blocks = need < cap32 ? need : cap32;
        const uint64_t ring_blocks = ua->ring_waves / (kBlockBvh / 64);
        if (blocks > ring_blocks) blocks = ring_blocks;
        if (name) *name = nm;
        hipLaunchKernelGGL(kernel, dim3((uint32_t)blocks), dim3(kBlockBvh), shmem, stream, *p, *b, geo, mat, *ua,
                           (unsigned long long*)stats);
        return hipGetLastError();
    };
    if (ua->samples != nullptr)  // direct mode
        return lds_scene ? launch(rtf::sample_kernel_fast<true, true>, "fast_f32_lds(direct)")
                         : launch(rtf::sample_kernel_fast<false, true>, "fast_f32_global(direct)");
    return lds_scene ? launch(rtf::sample_kernel_fast<true, false>, "fast_f32_lds")
                     : launch(rtf::sample_kernel_fast<false, false>, "fast_f32_global");
}

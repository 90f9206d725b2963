// rt_kernel.hip — the per-pixel x per-sample megakernel (gfx950 / CDNA4).
//
// Replaces the loop nest of Camera.render (reference src/camera.zig:123-145):
//   for j, for i, for s: getRay (camera.zig:187-215) -> rayColor (camera.zig:148-183)
//     -> HittableList.hit (hittable.zig:64-77) -> Sphere.hit (sphere.zig:26-54)
//     -> Material.scatter (material.zig:145-151)
//
// Mapping (DESIGN.md "Kernel"):
//   * one lane = one pixel; the lane sums its samples s = 0..spp-1 in order, exactly like
//     camera.zig:133-138, so the f64 sum rounds identically;
//   * the bounce loop and the sample loop are FLATTENED into one loop of ray segments: a lane whose
//     path ends (miss / absorb / bounceMax) immediately starts its next sample, so a wave pays
//     max-over-lanes of total rays, not sum-over-samples of max bounces;
//   * sphere geometry {cx, cy, cz, r^2} is staged once per workgroup into LDS (32 B per sphere);
//     every lane walks the list in order and all lanes of a wave read the same sphere (LDS
//     broadcast, conflict-free); materials are read from global memory only for the hit sphere;
//   * the closest-hit scan keeps the reference's exact acceptance rule (strict surrounds on the
//     shrinking (t_min, closest) interval) and computes the hit record only for the winner — the
//     same bits as recomputing it per accepted sphere;
//   * output is written once per pixel (coalesced: consecutive lanes, consecutive pixels).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_kernel.h"

#pragma clang fp contract(off)

namespace rtk {

struct Ray {
    v3 orig, dir;
};

// getRay (camera.zig:187-200) + sampleSquare (:203-209) + defocusDiskSample (:212-215)
__device__ __forceinline__ Ray get_ray(const KernelParams& p, uint32_t i, uint32_t j, Rng& g) {
    const double ox = g.uniform() - 0.5;
    const double oy = g.uniform() - 0.5;
    const v3 p0 = mk(p.pixel0[0], p.pixel0[1], p.pixel0[2]);
    const v3 du = mk(p.du[0], p.du[1], p.du[2]);
    const v3 dv = mk(p.dv[0], p.dv[1], p.dv[2]);
    const v3 center = mk(p.center[0], p.center[1], p.center[2]);
    const v3 ps = (p0 + muls(du, (double)i + ox)) + muls(dv, (double)j + oy);
    v3 origin = center;
    if (!(p.defocus_angle <= 0)) {
        const v3 d = random_in_unit_disk(g);
        const v3 ddu = mk(p.ddu[0], p.ddu[1], p.ddu[2]);
        const v3 ddv = mk(p.ddv[0], p.ddv[1], p.ddv[2]);
        origin = (center + muls(ddu, d.x)) + muls(ddv, d.y);
    }
    return Ray{origin, ps - origin};
}

// HittableList.hit over Sphere.hit with the exact arithmetic of sphere.zig:27-41.
// Returns the winning sphere index (or -1); *t_hit = its root.
template <bool kLds>
__device__ __forceinline__ int world_hit(const GeoRec* __restrict__ geo, uint32_t n, const Ray& r,
                                         double t_min, double t_max, double* t_hit) {
    const double a = len_sq(r.dir);  // loop-invariant Vec.lenSquared(ray.dir)
    double closest = t_max;
    int best = -1;
    for (uint32_t k = 0; k < n; ++k) {
        const GeoRec s = geo[k];
        const double ocx = s.cx - r.orig.x;
        const double ocy = s.cy - r.orig.y;
        const double ocz = s.cz - r.orig.z;
        const double h = (r.dir.x * ocx + r.dir.y * ocy) + r.dir.z * ocz;
        const double c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - s.r2;
        const double disc = h * h - a * c;
        if (disc >= 0) {  // !(disc < 0); a NaN disc rejects either way
            const double sq = __builtin_sqrt(disc);
            double root = (h - sq) / a;
            bool ok = t_min < root && root < closest;
            if (!ok) {
                root = (h + sq) / a;
                ok = t_min < root && root < closest;
            }
            if (ok) {
                closest = root;
                best = (int)k;
            }
        }
    }
    *t_hit = closest;
    return best;
}

template <bool kLds, int kOut>
__global__ __launch_bounds__(kBlock) void render_kernel(KernelParams p,
                                                        const GeoRec* __restrict__ geo_g,
                                                        const MatRec* __restrict__ mat_g,
                                                        void* __restrict__ out,
                                                        unsigned long long* __restrict__ stats) {
    extern __shared__ GeoRec lds_geo[];
    const GeoRec* geo = geo_g;
    if constexpr (kLds) {
        for (uint32_t k = threadIdx.x; k < p.n_spheres; k += blockDim.x) lds_geo[k] = geo_g[k];
        __syncthreads();
        geo = lds_geo;
    }

    const uint32_t W = p.width;
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = q < (uint64_t)p.n_rows * W;
    uint64_t rays = 0;
    uint64_t samples = 0;

    if (valid) {
        const uint32_t row_local = (uint32_t)(q / W);
        const uint32_t i = (uint32_t)(q - (uint64_t)row_local * W);
        const uint32_t j = p.row0 + row_local * p.row_step;
        const uint64_t pixel = (uint64_t)j * W + i;

        v3 sum = mk(0, 0, 0);
        uint32_t s = 0;
        Rng g;
        g.seed(sample_key(p.seed_mix, pixel, s));
        Ray r = get_ray(p, i, j, g);
        v3 att = mk(1, 1, 1);
        uint32_t bounce = 0;

        while (true) {
            bool done;
            v3 col = mk(0, 0, 0);
            if (bounce >= p.bounce_max) {
                done = true;  // rayColor fall-through: too many bounces -> black (camera.zig:181)
            } else {
                double t;
                ++rays;
                const int k = world_hit<kLds>(geo, p.n_spheres, r, p.t_min, p.t_max, &t);
                if (k < 0) {
                    // sky gradient (camera.zig:171-177)
                    const double a = 0.5 * (unit(r.dir).y + 1.0);
                    const v3 sky = muls(mk(1, 1, 1), 1.0 - a) + muls(mk(0.5, 0.7, 1), a);
                    col = att * sky;
                    done = true;
                } else {
                    const GeoRec sg = geo[k];
                    const MatRec m = mat_g[k];
                    // hit record (sphere.zig:44-53)
                    const v3 pt = r.orig + muls(r.dir, t);
                    const v3 outward = muls(pt - mk(sg.cx, sg.cy, sg.cz), m.inv_r);
                    const bool front = dot(r.dir, outward) < 0;
                    const v3 nrm = front ? outward : -outward;
                    const v3 albedo = mk(m.albedo[0], m.albedo[1], m.albedo[2]);
                    v3 dir;
                    done = false;
                    if (m.kind == 0) {  // Lambertian.scatter (material.zig:27-39)
                        dir = nrm + random_unit_vec(g);
                        if (near_zero(dir)) dir = nrm;
                        att = att * albedo;
                    } else if (m.kind == 1) {  // Metal.scatter (material.zig:55-68)
                        dir = unit(reflect(r.dir, nrm)) + muls(random_unit_vec(g), m.fuzz);
                        if (!(dot(dir, nrm) > 0)) {
                            done = true;  // absorbed -> black
                        } else {
                            att = att * albedo;
                        }
                    } else {  // Dielectric.scatter (material.zig:82-110)
                        const double ri = front ? 1.0 / m.ior : m.ior;
                        const v3 ud = unit(r.dir);
                        const double cos_t = __builtin_fmin(dot(-ud, nrm), 1.0);
                        const double sin_t = __builtin_sqrt(1.0 - cos_t * cos_t);
                        const bool cannot = ri * sin_t > 1.0;
                        double r0 = (1 - ri) / (1 + ri);
                        r0 = r0 * r0;
                        const double approx = r0 + (1 - r0) * zig_pow5(1 - cos_t);
                        // short-circuit `or` (material.zig:94): draw only if refraction is possible
                        if (cannot || approx > g.uniform()) {
                            dir = reflect(ud, nrm);
                        } else {
                            dir = refract(ud, nrm, ri);
                        }
                    }
                    if (!done) {
                        r.orig = pt;
                        r.dir = dir;
                        ++bounce;
                    }
                }
            }
            if (done) {
                sum = sum + col;  // pixelColor += rayColor(ray) (camera.zig:135)
                ++samples;
                if (++s >= p.spp) break;
                g.seed(sample_key(p.seed_mix, pixel, s));
                r = get_ray(p, i, j, g);
                att = mk(1, 1, 1);
                bounce = 0;
            }
        }

        const v3 avg = muls(sum, p.scale);  // camera.zig:137
        const uint64_t o = (uint64_t)row_local * W + i;
        if constexpr (kOut == 0) {
            double* dst = (double*)out + 3 * o;
            dst[0] = avg.x;
            dst[1] = avg.y;
            dst[2] = avg.z;
        } else {
            uint8_t* dst = (uint8_t*)out + 3 * o;
            dst[0] = to_byte(avg.x);
            dst[1] = to_byte(avg.y);
            dst[2] = to_byte(avg.z);
        }
    }

    if (stats) {
        // wave-level reduction, one atomic pair per wave
        for (int off = 32; off > 0; off >>= 1) {
            rays += __shfl_xor(rays, off, 64);
            samples += __shfl_xor(samples, off, 64);
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(&stats[0], (unsigned long long)rays);
            atomicAdd(&stats[1], (unsigned long long)samples);
        }
    }
}

}  // namespace rtk

// ------------------------------------------------------------------------------------------------
// launch wrapper (called from rt_runtime.cpp)
// ------------------------------------------------------------------------------------------------
extern "C" hipError_t rtk_launch_render(const rtk::KernelParams* p, const rtk::GeoRec* geo,
                                        const rtk::MatRec* mat, void* out, void* stats,
                                        hipStream_t stream, const char** name) {
    using namespace rtk;
    const uint64_t total = (uint64_t)p->n_rows * p->width;
    if (total == 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)((total + kBlock - 1) / kBlock);
    const bool lds = p->n_spheres <= kMaxLdsSpheres;
    const size_t shmem = lds ? (size_t)p->n_spheres * sizeof(GeoRec) : 0;
    auto* st = (unsigned long long*)stats;
    if (lds) {
        if (p->out_format == 0) {
            if (name) *name = "render_kernel<lds,f64>";
            hipLaunchKernelGGL((render_kernel<true, 0>), dim3(blocks), dim3(kBlock), shmem, stream,
                               *p, geo, mat, out, st);
        } else {
            if (name) *name = "render_kernel<lds,rgb8>";
            hipLaunchKernelGGL((render_kernel<true, 1>), dim3(blocks), dim3(kBlock), shmem, stream,
                               *p, geo, mat, out, st);
        }
    } else {
        if (p->out_format == 0) {
            if (name) *name = "render_kernel<global,f64>";
            hipLaunchKernelGGL((render_kernel<false, 0>), dim3(blocks), dim3(kBlock), 0, stream,
                               *p, geo, mat, out, st);
        } else {
            if (name) *name = "render_kernel<global,rgb8>";
            hipLaunchKernelGGL((render_kernel<false, 1>), dim3(blocks), dim3(kBlock), 0, stream,
                               *p, geo, mat, out, st);
        }
    }
    return hipGetLastError();
}

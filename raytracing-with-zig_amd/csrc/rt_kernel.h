// rt_kernel.h — device data layout shared by the kernel (rt_kernel.hip) and the host runtime.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtk {

constexpr int kBlock = 256;               // 4 waves of 64 lanes
constexpr uint32_t kMaxLdsSpheres = 2048; // 64 KiB of LDS geometry; above this, read from global

// Geometry walked by every lane for every ray: 32 B, one LDS broadcast pair per sphere.
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
    uint32_t kind;  // 0 lambertian, 1 metal, 2 dielectric
    uint32_t pad;
};

// Kernel arguments (by value).  Mirrors rt_camera + the row partition.
struct KernelParams {
    uint32_t width, height, spp, bounce_max;
    double scale;  // pixelSamplesScale
    double center[3], pixel0[3], du[3], dv[3], ddu[3], ddv[3];
    double defocus_angle, t_min, t_max;
    uint64_t seed_mix;  // sm_mix(seed), hoisted from sample_key
    uint32_t row0, row_step, n_rows, n_spheres;
    uint32_t out_format;  // 0 linear f64, 1 rgb8
    uint32_t pad;
};

}  // namespace rtk

extern "C" hipError_t rtk_launch_render(const rtk::KernelParams* p, const rtk::GeoRec* geo,
                                        const rtk::MatRec* mat, void* out, void* stats,
                                        hipStream_t stream, const char** name);

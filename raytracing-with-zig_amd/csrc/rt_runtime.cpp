// rt_runtime.cpp — device runtime behind the C ABI: contexts, scene upload, launches, and the
// blocking multi-GPU rt_render() that replaces Camera.render (camera.zig:123-145).
//
// Multi-GPU inside one call: one host thread drives every device asynchronously (one stream per
// GPU).  Rows are interleaved (row j on device j mod G) so sky-heavy and ground-heavy rows spread
// evenly; each device renders its rows into its own buffer, copies them back, and the host
// un-interleaves them into the caller's framebuffer.  Because the RNG is keyed by the GLOBAL pixel
// index, the image is bit-identical for any device count.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "../../include/rt.h"
#include "rt_bvh.hpp"
#include "rt_device.h"
#include "rt_kernel.h"

void rt_set_last_error(const std::string& msg);

struct rt_context {
    int device = 0;
    hipStream_t stream = nullptr;
    rtk::GeoRec* d_geo = nullptr;
    rtk::MatRec* d_mat = nullptr;
    uint32_t n_spheres = 0;
    uint32_t capacity = 0;
    // workspace: per-sample colors [s][pixel][3] (HBM is 288 GB: a whole 1200x800x500 frame of
    // samples is 11.5 GB), running per-pixel sums for multi-chunk renders, the work-queue counter
    double* d_samples = nullptr;
    size_t samples_bytes = 0;
    double* d_sums = nullptr;
    size_t sums_bytes = 0;
    unsigned long long* d_queue = nullptr;
    const char* last_kernel = "sample_kernel";
    // BVH over the sphere list (rt_bvh.hpp); empty/!ok => the linear walk
    std::vector<rt_sphere> spheres;  // host copy (rebuilds for far-away cameras)
    bool bvh_ok = false;
    double bvh_origin_bound = 0;
    rtk::BvhNode* d_nodes = nullptr;
    rtk::BvhLeaf* d_leaves = nullptr;
    rtk::GeoRec* d_always_geo = nullptr;
    uint32_t* d_always_sid = nullptr;
    size_t nodes_bytes = 0, leaves_bytes = 0, always_geo_bytes = 0, always_sid_bytes = 0;
    rtk::BvhArgs bvh{};
    // optional per-kernel timing: event pairs around every sample / reduce launch of the last call
    bool timing = false;
    bool profile = false;  // instrumented kernels: d_stats must hold 24 uint64 (rt.h)
    int precision = RT_PRECISION_F64;
    // event pool: every timed chunk of every call takes the next 4 events (sample start/stop,
    // reduce start/stop); `call_first` / `timed_chunks` locate the last call's, `log_used` counts
    // the chunks recorded since timing was (re)enabled (rt_context_kernel_times_total)
    std::vector<hipEvent_t> events;
    uint32_t call_first = 0;
    uint32_t timed_chunks = 0;
    uint32_t log_used = 0;
};

namespace {

constexpr uint32_t kMaxTimedChunks = 1024;  // event-pool bound of rt_context_kernel_times_total

int hip_fail(hipError_t e, const char* what) {
    rt_set_last_error(std::string(what) + ": " + hipGetErrorString(e));
    return e == hipErrorNoDevice || e == hipErrorInvalidDevice ? RT_ERR_NO_DEVICE : RT_ERR_HIP;
}

#define HIP_CHECK(expr)                                  \
    do {                                                 \
        hipError_t _e = (expr);                          \
        if (_e != hipSuccess) return hip_fail(_e, #expr); \
    } while (0)

int validate_camera(const rt_camera* c) {
    if (!c) { rt_set_last_error("null camera"); return RT_ERR_INVALID; }
    if (c->image_width == 0 || c->image_height == 0) {
        rt_set_last_error("image_width and image_height must be > 0");
        return RT_ERR_INVALID;
    }
    if (c->samples_per_pixel == 0) {
        rt_set_last_error("samples_per_pixel must be > 0");
        return RT_ERR_INVALID;
    }
    if ((uint64_t)c->image_width * c->image_height >= (1ULL << 32)) {
        rt_set_last_error("image must have fewer than 2^32 pixels");
        return RT_ERR_INVALID;
    }
    return RT_OK;
}

int validate_spheres(const rt_sphere* s, size_t n) {
    if (n == 0 || !s) { rt_set_last_error("empty sphere list"); return RT_ERR_INVALID; }
    if (n > (1u << 24)) { rt_set_last_error("too many spheres"); return RT_ERR_CAPACITY; }
    for (size_t k = 0; k < n; k++) {
        if (s[k].material > RT_DIELECTRIC) {
            rt_set_last_error("sphere " + std::to_string(k) + ": unknown material kind");
            return RT_ERR_INVALID;
        }
        if (std::isnan(s[k].radius)) {
            rt_set_last_error("sphere " + std::to_string(k) + ": radius is NaN");
            return RT_ERR_INVALID;
        }
    }
    return RT_OK;
}

// Workspace budget for per-sample colors: RTZIG_WORKSPACE_MB, default 64 GiB (MI355X has 288 GB
// of HBM; a whole config-4 frame needs 11.5 GB), never more than 60% of the free memory.
uint64_t workspace_budget() {
    uint64_t budget = 64ULL << 30;
    if (const char* e = std::getenv("RTZIG_WORKSPACE_MB")) budget = std::strtoull(e, nullptr, 10) << 20;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0) {
        const uint64_t cap = (uint64_t)(0.6 * (double)free_b);
        if (budget > cap) budget = cap;
    }
    return budget;
}

int ensure_buffer(void** ptr, size_t* bytes, size_t need) {
    if (*ptr && *bytes >= need) return RT_OK;
    (void)hipFree(*ptr);
    *ptr = nullptr;
    *bytes = 0;
    hipError_t e = hipMalloc(ptr, need ? need : 1);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(workspace)");
    *bytes = need;
    return RT_OK;
}

// Builder ref (node index >= 0, ~leaf index < 0) -> device ref (byte offsets, see upload_bvh).
int32_t device_ref(int32_t ref) {
    if (ref >= 0) return (int32_t)((int64_t)ref * (int64_t)sizeof(rtk::BvhNode));
    return ~(int32_t)((int64_t)(~ref) * (int64_t)sizeof(rtk::BvhLeaf));
}

// Builds and uploads the BVH for the context's scene, valid for ray origins with |o_i| <= bound.
int upload_bvh(rt_context* ctx, double bound) {
    const rtbvh::Bvh bvh = rtbvh::build(ctx->spheres.data(), ctx->spheres.size(), bound);
    // byte-offset refs must fit int32 (and stay clear of the walk's INT32_MIN "done" marker)
    const bool fits = bvh.nodes.size() * sizeof(rtk::BvhNode) < (1ull << 30) &&
                      bvh.slot_to_sphere.size() / rtk::kLeafBvh * sizeof(rtk::BvhLeaf) < (1ull << 30);
    ctx->bvh_ok = bvh.ok && fits;
    ctx->bvh_origin_bound = bound;
    if (!ctx->bvh_ok) return RT_OK;
    static_assert(rtbvh::kLeafMax == rtk::kLeafBvh && rtbvh::kMaxDepth == rtk::kMaxDepthBvh, "BVH constants differ");
    const size_t nn = bvh.nodes.size();
    const size_t na = bvh.n_always;
    const size_t nl = (bvh.slot_to_sphere.size() - na) / rtk::kLeafBvh;
    auto geo_of = [&](uint32_t k) {
        rtk::GeoRec g;
        if (k == rtbvh::kSentinel) {  // never-hit padding slot
            g.cx = g.cy = g.cz = 0.0;
            g.r2 = -std::numeric_limits<double>::infinity();
            return g;
        }
        const rt_sphere& sp = ctx->spheres[k];
        const double r = sp.radius > 0 ? sp.radius : 0.0;
        g.cx = sp.center[0];
        g.cy = sp.center[1];
        g.cz = sp.center[2];
        g.r2 = r * r;
        return g;
    };
    std::vector<rtk::BvhNode> nodes(nn);
    for (size_t i = 0; i < nn; i++) {
        const rtbvh::Node& src = bvh.nodes[i];
        rtk::BvhNode& d = nodes[i];
        std::memset(&d, 0, sizeof d);
        for (int a = 0; a < 3; a++) {  // {lo, hi, hi, lo}: see rtk::BvhNode
            d.c0[a][0] = d.c0[a][3] = src.lo0[a];
            d.c0[a][1] = d.c0[a][2] = src.hi0[a];
            d.c1[a][0] = d.c1[a][3] = src.lo1[a];
            d.c1[a][1] = d.c1[a][2] = src.hi1[a];
        }
        // device refs are BYTE offsets (node: ref * 104 >= 0, leaf: ~(leaf * sizeof(BvhLeaf))) so the
        // walk forms LDS/global addresses with an add instead of a quarter-rate v_mul_lo_u32
        d.ref0 = device_ref(src.ref0);
        d.ref1 = device_ref(src.ref1);
    }
    std::vector<rtk::BvhLeaf> leaves(nl ? nl : 1);
    for (size_t l = 0; l < nl; l++)
        for (int u = 0; u < rtk::kLeafBvh; u++) {
            const uint32_t k = bvh.slot_to_sphere[na + l * rtk::kLeafBvh + u];
            const rtk::GeoRec g = geo_of(k);
            leaves[l].g[u] = rtk::LeafGeo{g.cx, g.cy, g.cz, g.r2};
            leaves[l].sid[u] = k;
        }
    std::vector<rtk::GeoRec> ageo(na ? na : 1);
    std::vector<uint32_t> asid(na ? na : 1, 0);
    for (size_t q = 0; q < na; q++) {
        ageo[q] = geo_of(bvh.slot_to_sphere[q]);
        asid[q] = bvh.slot_to_sphere[q];
    }
    int rc = ensure_buffer((void**)&ctx->d_nodes, &ctx->nodes_bytes, nn * sizeof(rtk::BvhNode));
    if (!rc) rc = ensure_buffer((void**)&ctx->d_leaves, &ctx->leaves_bytes, leaves.size() * sizeof(rtk::BvhLeaf));
    if (!rc) rc = ensure_buffer((void**)&ctx->d_always_geo, &ctx->always_geo_bytes, ageo.size() * sizeof(rtk::GeoRec));
    if (!rc) rc = ensure_buffer((void**)&ctx->d_always_sid, &ctx->always_sid_bytes, asid.size() * sizeof(uint32_t));
    if (rc) return rc;
    HIP_CHECK(hipMemcpyAsync(ctx->d_nodes, nodes.data(), nn * sizeof(rtk::BvhNode), hipMemcpyHostToDevice, ctx->stream));
    HIP_CHECK(hipMemcpyAsync(ctx->d_leaves, leaves.data(), leaves.size() * sizeof(rtk::BvhLeaf), hipMemcpyHostToDevice,
                             ctx->stream));
    HIP_CHECK(hipMemcpyAsync(ctx->d_always_geo, ageo.data(), ageo.size() * sizeof(rtk::GeoRec), hipMemcpyHostToDevice,
                             ctx->stream));
    HIP_CHECK(hipMemcpyAsync(ctx->d_always_sid, asid.data(), asid.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                             ctx->stream));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    ctx->bvh.nodes = ctx->d_nodes;
    ctx->bvh.leaves = ctx->d_leaves;
    ctx->bvh.always_geo = ctx->d_always_geo;
    ctx->bvh.always_sid = ctx->d_always_sid;
    ctx->bvh.n_nodes = (uint32_t)nn;
    ctx->bvh.n_leaves = (uint32_t)nl;
    ctx->bvh.n_always = (uint32_t)na;
    ctx->bvh.stack_depth = (uint32_t)std::max(2, std::min(bvh.depth, rtk::kMaxDepthBvh));
    return RT_OK;
}

// Walk selection: RTZIG_KERNEL names a linear variant (lds_u*, smem_u*) or "bvh"; default: the
// BVH walk when it built, else the linear default variant.
bool use_bvh(const rt_context* ctx) {
    const char* e = std::getenv("RTZIG_KERNEL");
    if (e && std::strncmp(e, "bvh", 3) != 0) return false;
    return ctx->bvh_ok;
}

rtk::KernelParams make_params(const rt_camera* c, uint32_t fmt, uint32_t row0, uint32_t row_step,
                              uint32_t n_rows, uint32_t n_spheres) {
    rtk::KernelParams p;
    std::memset(&p, 0, sizeof p);
    p.width = c->image_width;
    p.height = c->image_height;
    p.spp = c->samples_per_pixel;
    p.bounce_max = c->bounce_max;
    p.scale = c->pixel_samples_scale;
    for (int k = 0; k < 3; k++) {
        p.center[k] = c->center[k];
        p.pixel0[k] = c->pixel0[k];
        p.du[k] = c->du[k];
        p.dv[k] = c->dv[k];
        p.ddu[k] = c->defocus_disk_u[k];
        p.ddv[k] = c->defocus_disk_v[k];
    }
    p.defocus_angle = c->defocus_angle;
    for (int k = 0; k < 3; k++) {  // f32 copies for the fast kernel
        p.fcam[0 + k] = (float)c->center[k];
        p.fcam[3 + k] = (float)c->pixel0[k];
        p.fcam[6 + k] = (float)c->du[k];
        p.fcam[9 + k] = (float)c->dv[k];
        p.fcam[12 + k] = (float)c->defocus_disk_u[k];
        p.fcam[15 + k] = (float)c->defocus_disk_v[k];
    }
    p.fcam[18] = (float)c->defocus_angle;
    p.t_min = c->t_min;
    p.t_max = c->t_max;
    p.seed_mix = rtk::sm_mix_hd(c->seed);
    p.row0 = row0;
    p.row_step = row_step;
    p.n_rows = n_rows;
    p.n_spheres = n_spheres;
    p.n_pad = (n_spheres + rtk::kPad - 1) / rtk::kPad * rtk::kPad;
    p.div_layer = rtk::fastdiv_make(n_rows * c->image_width);  // < 2^32 pixels (checked by callers)
    p.div_width = rtk::fastdiv_make(c->image_width);
    (void)fmt;
    return p;
}

}  // namespace

extern "C" {

int rt_context_create(int device, rt_context** out_ctx) {
    if (!out_ctx) { rt_set_last_error("null out_ctx"); return RT_ERR_INVALID; }
    int count = 0;
    HIP_CHECK(hipGetDeviceCount(&count));
    if (device < 0 || device >= count) {
        rt_set_last_error("device ordinal " + std::to_string(device) + " out of range (" +
                          std::to_string(count) + " visible)");
        return RT_ERR_NO_DEVICE;
    }
    HIP_CHECK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        rt_set_last_error(std::string("device is ") + prop.gcnArchName + ", library built for gfx950");
        return RT_ERR_NO_DEVICE;
    }
    auto* ctx = new rt_context;
    ctx->device = device;
    hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete ctx;
        return hip_fail(e, "hipStreamCreate");
    }
    *out_ctx = ctx;
    return RT_OK;
}

int rt_context_destroy(rt_context* ctx) {
    if (!ctx) return RT_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->d_geo);
    (void)hipFree(ctx->d_mat);
    (void)hipFree(ctx->d_samples);
    (void)hipFree(ctx->d_sums);
    (void)hipFree(ctx->d_queue);
    (void)hipFree(ctx->d_nodes);
    (void)hipFree(ctx->d_leaves);
    (void)hipFree(ctx->d_always_geo);
    (void)hipFree(ctx->d_always_sid);
    for (hipEvent_t e : ctx->events) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return RT_OK;
}

int rt_context_set_scene(rt_context* ctx, const rt_sphere* spheres, size_t n) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    int rc = validate_spheres(spheres, n);
    if (rc) return rc;
    HIP_CHECK(hipSetDevice(ctx->device));
    const size_t n_pad = (n + rtk::kPad - 1) / rtk::kPad * rtk::kPad;
    std::vector<rtk::GeoRec> geo(n_pad);
    std::vector<rtk::MatRec> mat(n);
    for (size_t k = n; k < n_pad; k++) {  // never-hit sentinels (rt_kernel.h)
        geo[k].cx = geo[k].cy = geo[k].cz = 0.0;
        geo[k].r2 = -std::numeric_limits<double>::infinity();
    }
    for (size_t k = 0; k < n; k++) {
        const double r = spheres[k].radius > 0 ? spheres[k].radius : 0.0;  // sphere.zig:21
        geo[k].cx = spheres[k].center[0];
        geo[k].cy = spheres[k].center[1];
        geo[k].cz = spheres[k].center[2];
        geo[k].r2 = r * r;
        std::memset(&mat[k], 0, sizeof mat[k]);
        for (int c = 0; c < 3; c++) mat[k].albedo[c] = spheres[k].albedo[c];
        mat[k].fuzz = spheres[k].fuzz;
        mat[k].ior = spheres[k].refraction_index;
        mat[k].inv_r = 1.0 / r;
        const double ior = spheres[k].refraction_index;
        mat[k].inv_ior = 1.0 / ior;
        for (int face = 0; face < 2; face++) {  // reflectance()'s r0 (material.zig:106-108) per face
            const double ri = face == 0 ? mat[k].inv_ior : ior;
            double r0 = (1 - ri) / (1 + ri);
            r0 = r0 * r0;
            (face == 0 ? mat[k].r0_front : mat[k].r0_back) = r0;
        }
        mat[k].kind = spheres[k].material;
    }
    if (n_pad > ctx->capacity) {
        (void)hipFree(ctx->d_geo);
        (void)hipFree(ctx->d_mat);
        ctx->d_geo = nullptr;
        ctx->d_mat = nullptr;
        ctx->capacity = 0;
        HIP_CHECK(hipMalloc(&ctx->d_geo, n_pad * sizeof(rtk::GeoRec)));
        HIP_CHECK(hipMalloc(&ctx->d_mat, n_pad * sizeof(rtk::MatRec)));
        ctx->capacity = (uint32_t)n_pad;
    }
    HIP_CHECK(hipMemcpyAsync(ctx->d_geo, geo.data(), n_pad * sizeof(rtk::GeoRec), hipMemcpyHostToDevice, ctx->stream));
    HIP_CHECK(hipMemcpyAsync(ctx->d_mat, mat.data(), n * sizeof(rtk::MatRec), hipMemcpyHostToDevice, ctx->stream));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    ctx->n_spheres = (uint32_t)n;
    ctx->spheres.assign(spheres, spheres + n);
    const double extent = rtbvh::scene_extent(spheres, n);
    return upload_bvh(ctx, extent * (1.0 + 0x1p-20) + 1e-300);
}

int rt_render_rows_async(rt_context* ctx, const rt_camera* cam, uint32_t output_format, uint32_t row0,
                         uint32_t row_step, uint32_t n_rows, void* d_out, void* d_stats, void* stream) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    int rc = validate_camera(cam);
    if (rc) return rc;
    if (ctx->n_spheres == 0) { rt_set_last_error("no scene uploaded"); return RT_ERR_INVALID; }
    if (output_format > RT_OUT_RGB8) { rt_set_last_error("bad output_format"); return RT_ERR_INVALID; }
    if (n_rows == 0) return RT_OK;
    if (!d_out) { rt_set_last_error("null output"); return RT_ERR_INVALID; }
    if (row_step == 0) row_step = 1;
    const uint64_t last_row = (uint64_t)row0 + (uint64_t)(n_rows - 1) * row_step;
    if (last_row >= cam->image_height) {
        rt_set_last_error("row range exceeds image_height");
        return RT_ERR_INVALID;
    }
    HIP_CHECK(hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;  // NULL = the HIP null stream, like torch's default stream

    // Chunk the samples so that [s_count][P][3] doubles fit the workspace budget.
    const uint64_t P = (uint64_t)n_rows * cam->image_width;
    const uint64_t layer = P * 3 * sizeof(double);
    // (the free-memory query is skipped when the whole frame fits the workspace already allocated)
    const bool fits = ctx->d_samples && ctx->samples_bytes / layer >= cam->samples_per_pixel;
    uint64_t s_chunk = fits ? cam->samples_per_pixel : workspace_budget() / layer;
    if (s_chunk < 1) s_chunk = 1;
    if (s_chunk > cam->samples_per_pixel) s_chunk = cam->samples_per_pixel;
    if (s_chunk * P > 0xffffffffULL) s_chunk = 0xffffffffULL / P;  // kernel item index is 32-bit
    const uint32_t n_chunks = (uint32_t)((cam->samples_per_pixel + s_chunk - 1) / s_chunk);
    rc = ensure_buffer((void**)&ctx->d_samples, &ctx->samples_bytes, s_chunk * layer);
    if (!rc && n_chunks > 1) rc = ensure_buffer((void**)&ctx->d_sums, &ctx->sums_bytes, layer);
    if (!rc && !ctx->d_queue) {
        size_t qb = 0;
        rc = ensure_buffer((void**)&ctx->d_queue, &qb, rtk::kQueueBufferBytes);
    }
    if (rc) return rc;

    if (ctx->timing) {
        if (ctx->log_used + n_chunks > kMaxTimedChunks) ctx->log_used = 0;  // wrap: totals restart
        ctx->call_first = ctx->log_used;
        ctx->log_used += n_chunks;
        while (ctx->events.size() < 4 * (size_t)ctx->log_used) {
            hipEvent_t e;
            HIP_CHECK(hipEventCreate(&e));
            ctx->events.push_back(e);
        }
        ctx->timed_chunks = n_chunks;
    }
    // camera-ray origins (center + defocus disk) must lie inside the BVH padding's origin bound
    double cam_bound = 0;
    for (int a = 0; a < 3; a++)
        cam_bound = std::max(cam_bound, std::fabs(cam->center[a]) + std::fabs(cam->defocus_disk_u[a]) +
                                            std::fabs(cam->defocus_disk_v[a]));
    if (ctx->bvh_ok && !(cam_bound <= ctx->bvh_origin_bound)) {
        rc = upload_bvh(ctx, std::max(cam_bound, ctx->bvh_origin_bound) * 1.01);
        if (rc) return rc;
    }
    const bool bvh = use_bvh(ctx);
    rtk::KernelParams p = make_params(cam, output_format, row0, row_step, n_rows, ctx->n_spheres);
    p.prof = ctx->profile && d_stats ? 1u : 0u;
    if (const char* e = std::getenv("RTZIG_ORDER"))
        p.order = std::strcmp(e, "pixel") == 0 ? 1u : (std::strcmp(e, "tile") == 0 ? 2u : 0u);
    for (uint32_t c = 0; c < n_chunks; c++) {
        p.s_begin = (uint32_t)(c * s_chunk);
        p.s_count = (uint32_t)std::min<uint64_t>(s_chunk, cam->samples_per_pixel - p.s_begin);
        if (ctx->timing) HIP_CHECK(hipEventRecord(ctx->events[4 * (ctx->call_first + c) + 0], s));
        if (bvh && ctx->precision == RT_PRECISION_F32)
            HIP_CHECK(rtk_launch_samples_fast(&p, &ctx->bvh, ctx->d_geo, ctx->d_mat, ctx->d_samples, ctx->d_queue,
                                              d_stats, s, &ctx->last_kernel));
        else if (bvh)
            HIP_CHECK(rtk_launch_samples_bvh(&p, &ctx->bvh, ctx->d_geo, ctx->d_mat, ctx->d_samples, ctx->d_queue,
                                             d_stats, s, &ctx->last_kernel));
        else
            HIP_CHECK(rtk_launch_samples(&p, ctx->d_geo, ctx->d_mat, ctx->d_samples, ctx->d_queue, d_stats, s,
                                         &ctx->last_kernel));
        if (ctx->timing) HIP_CHECK(hipEventRecord(ctx->events[4 * (ctx->call_first + c) + 1], s));
        rtk::ReduceParams rp;
        std::memset(&rp, 0, sizeof rp);
        rp.n_pixels = (uint32_t)P;
        rp.s_count = p.s_count;
        rp.first = c == 0;
        rp.last = c + 1 == n_chunks;
        rp.out_format = output_format;
        rp.scale = cam->pixel_samples_scale;
        if (ctx->timing) HIP_CHECK(hipEventRecord(ctx->events[4 * (ctx->call_first + c) + 2], s));
        HIP_CHECK(rtk_launch_reduce(&rp, ctx->d_samples, ctx->d_sums, d_out, s));
        if (ctx->timing) HIP_CHECK(hipEventRecord(ctx->events[4 * (ctx->call_first + c) + 3], s));
    }
    return RT_OK;
}

int rt_context_enable_timing(rt_context* ctx, int enable) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    ctx->timing = enable != 0;
    ctx->timed_chunks = 0;
    ctx->call_first = 0;
    ctx->log_used = 0;
    return RT_OK;
}

int rt_context_set_precision(rt_context* ctx, int precision) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    if (precision != RT_PRECISION_F64 && precision != RT_PRECISION_F32) {
        rt_set_last_error("unknown precision");
        return RT_ERR_INVALID;
    }
    ctx->precision = precision;
    return RT_OK;
}

int rt_context_enable_profile(rt_context* ctx, int enable) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    ctx->profile = enable != 0;
    return RT_OK;
}

int rt_context_kernel_times(rt_context* ctx, double* sample_ms, double* reduce_ms) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    if (!ctx->timing || ctx->timed_chunks == 0) { rt_set_last_error("timing not enabled or nothing rendered"); return RT_ERR_INVALID; }
    HIP_CHECK(hipSetDevice(ctx->device));
    double sm = 0, rm = 0;
    for (uint32_t c = ctx->call_first; c < ctx->call_first + ctx->timed_chunks; c++) {
        float a = 0, b = 0;
        HIP_CHECK(hipEventSynchronize(ctx->events[4 * c + 3]));
        HIP_CHECK(hipEventElapsedTime(&a, ctx->events[4 * c + 0], ctx->events[4 * c + 1]));
        HIP_CHECK(hipEventElapsedTime(&b, ctx->events[4 * c + 2], ctx->events[4 * c + 3]));
        sm += a;
        rm += b;
    }
    if (sample_ms) *sample_ms = sm;
    if (reduce_ms) *reduce_ms = rm;
    return RT_OK;
}

int rt_context_kernel_times_total(rt_context* ctx, double* sample_ms, double* reduce_ms, uint32_t* n_chunks) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    if (!ctx->timing) { rt_set_last_error("timing not enabled"); return RT_ERR_INVALID; }
    HIP_CHECK(hipSetDevice(ctx->device));
    double sm = 0, rm = 0;
    for (uint32_t c = 0; c < ctx->log_used; c++) {
        float a = 0, b = 0;
        HIP_CHECK(hipEventSynchronize(ctx->events[4 * c + 3]));
        HIP_CHECK(hipEventElapsedTime(&a, ctx->events[4 * c + 0], ctx->events[4 * c + 1]));
        HIP_CHECK(hipEventElapsedTime(&b, ctx->events[4 * c + 2], ctx->events[4 * c + 3]));
        sm += a;
        rm += b;
    }
    if (sample_ms) *sample_ms = sm;
    if (reduce_ms) *reduce_ms = rm;
    if (n_chunks) *n_chunks = ctx->log_used;
    return RT_OK;
}

const char* rt_kernel_name(rt_context* ctx) { return ctx ? ctx->last_kernel : "render_kernel"; }

int rt_render(const rt_camera* cam, const rt_sphere* spheres, size_t n, const rt_options* opts, void* out) {
    int rc = validate_camera(cam);
    if (rc) return rc;
    rc = validate_spheres(spheres, n);
    if (rc) return rc;
    if (!out) { rt_set_last_error("null output"); return RT_ERR_INVALID; }
    rt_options o{};
    if (opts) o = *opts;
    if (o.output_format > RT_OUT_RGB8) { rt_set_last_error("bad output_format"); return RT_ERR_INVALID; }
    if (o.precision > RT_PRECISION_F32 || o.reserved != 0) {
        rt_set_last_error("bad precision / reserved field");
        return RT_ERR_INVALID;
    }
    const uint32_t stride = o.pixel_stride ? o.pixel_stride : 3;
    if (o.output_format == RT_OUT_LINEAR_F64 && stride < 3) {
        rt_set_last_error("pixel_stride must be >= 3");
        return RT_ERR_INVALID;
    }
    int count = 0;
    HIP_CHECK(hipGetDeviceCount(&count));
    if (count <= 0) { rt_set_last_error("no HIP device"); return RT_ERR_NO_DEVICE; }
    const int first = o.device;
    int G = o.n_gpus > 0 ? o.n_gpus : count - first;
    if (first < 0 || first + G > count || G <= 0) {
        rt_set_last_error("requested devices not available");
        return RT_ERR_NO_DEVICE;
    }
    const uint32_t W = cam->image_width, H = cam->image_height;
    G = std::min<int>(G, (int)H);
    const size_t px_bytes = o.output_format == RT_OUT_LINEAR_F64 ? 3 * sizeof(double) : 3;

    struct Dev {
        rt_context* ctx = nullptr;
        void* d_out = nullptr;
        uint64_t* d_stats = nullptr;
        std::vector<uint8_t> host;
        uint32_t n_rows = 0;
    };
    std::vector<Dev> devs(G);
    auto cleanup = [&]() {
        for (auto& d : devs) {
            if (!d.ctx) continue;
            (void)hipSetDevice(d.ctx->device);
            (void)hipFree(d.d_out);
            (void)hipFree(d.d_stats);
            rt_context_destroy(d.ctx);
        }
    };
    for (int g = 0; g < G; g++) {
        Dev& d = devs[g];
        rc = rt_context_create(first + g, &d.ctx);
        if (!rc) rc = rt_context_set_scene(d.ctx, spheres, n);
        if (!rc) rc = rt_context_set_precision(d.ctx, (int)o.precision);
        if (rc) { cleanup(); return rc; }
        d.n_rows = (H - (uint32_t)g + (uint32_t)G - 1) / (uint32_t)G;
        const size_t bytes = (size_t)d.n_rows * W * px_bytes;
        hipError_t e = hipMalloc(&d.d_out, bytes ? bytes : 1);
        if (e == hipSuccess) e = hipMalloc((void**)&d.d_stats, 2 * sizeof(uint64_t));
        if (e == hipSuccess) e = hipMemsetAsync(d.d_stats, 0, 2 * sizeof(uint64_t), d.ctx->stream);
        if (e != hipSuccess) { cleanup(); return hip_fail(e, "hipMalloc"); }
        rc = rt_render_rows_async(d.ctx, cam, o.output_format, (uint32_t)g, (uint32_t)G, d.n_rows,
                                  d.d_out, d.d_stats, d.ctx->stream);
        if (rc) { cleanup(); return rc; }
    }
    uint64_t stats[2] = {0, 0};
    for (int g = 0; g < G; g++) {
        Dev& d = devs[g];
        (void)hipSetDevice(d.ctx->device);
        d.host.resize((size_t)d.n_rows * W * px_bytes);
        uint64_t st[2] = {0, 0};
        hipError_t e = hipMemcpyAsync(d.host.data(), d.d_out, d.host.size(), hipMemcpyDeviceToHost, d.ctx->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(st, d.d_stats, sizeof st, hipMemcpyDeviceToHost, d.ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(d.ctx->stream);
        if (e != hipSuccess) { cleanup(); return hip_fail(e, "render/copy-back"); }
        stats[0] += st[0];
        stats[1] += st[1];
        // un-interleave rows j = g + k*G into the caller's framebuffer
        for (uint32_t k = 0; k < d.n_rows; k++) {
            const uint32_t j = (uint32_t)g + k * (uint32_t)G;
            if (o.output_format == RT_OUT_RGB8) {
                std::memcpy((uint8_t*)out + (size_t)j * W * 3, d.host.data() + (size_t)k * W * 3, (size_t)W * 3);
            } else {
                const double* src = (const double*)d.host.data() + (size_t)k * W * 3;
                double* dst = (double*)out + (size_t)j * W * stride;
                if (stride == 3) {
                    std::memcpy(dst, src, (size_t)W * 3 * sizeof(double));
                } else {
                    for (uint32_t i = 0; i < W; i++)
                        for (int c = 0; c < 3; c++) dst[(size_t)i * stride + c] = src[3 * (size_t)i + c];
                }
            }
        }
    }
    cleanup();
    if (o.stats_out) {
        o.stats_out[0] = stats[0];
        o.stats_out[1] = stats[1];
    }
    return RT_OK;
}

}  // extern "C"

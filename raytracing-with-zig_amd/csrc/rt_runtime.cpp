// rt_runtime.cpp — device runtime behind the C ABI: contexts, scene upload, launches, and the
// blocking multi-GPU rt_render() that replaces Camera.render (camera.zig:123-145).
//
// One render of rows = ONE persistent launch of the sample kernel.  It accumulates every pixel's
// samples in sample order itself (rt_kernel.h "Work units", rt_units.h): work units of 64 pixels x
// a chunk of samples, wave-private rings for the colors of unfinished units, and per-pixel running
// sums handed from wave to wave behind a per-tile flag.  The workspace is independent of spp: one
// 144-KiB ring per resident wave of the kernel actually launched (the BVH kernels: 16 waves per CU,
// 576 MiB on 256 CUs) plus 24 B of running sum per pixel and 4 B of flag per 64 pixels.  Small
// launches (direct mode) instead store every sample (at most 2 GiB) for a reduce pass; a context
// holds the buffers of one mode at a time (rt.h "Workspace").
//
// rt_render() keeps one cached context per device for the life of the process (SURVEY §8(b):
// "an optional rt_context handle caches device init"): the first call creates them on parallel
// host threads; a later call on the same sphere list uploads nothing and rebuilds nothing.
// Multi-GPU inside one call: rows are interleaved (row j on device j mod G), each device renders its
// rows into its own buffer, copies them to pinned host memory, and the host un-interleaves them into
// the caller's framebuffer.  The RNG is keyed by the GLOBAL pixel index, so the image is
// bit-identical for any device count.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <exception>
#include <functional>
#include <future>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt.h"
#include "rt_bvh.hpp"
#include "rt_device.h"
#include "rt_kernel.h"
#include "rt_schedule.hpp"

void rt_set_last_error(const std::string& msg);

namespace {

constexpr uint32_t kMaxTimed = 1024;  // event-pool bound of rt_context_kernel_times_total
constexpr size_t kEventsPerCall = 4;   // timed call: start, sample kernel done, reduce start, reduce done

// Host-side scene: device records of the Hittable list plus its BVH, built once per sphere list and
// uploaded to every device that renders it.
struct SceneData {
    std::vector<rt_sphere> spheres;
    std::vector<rtk::GeoRec> geo;  // padded to kPad with never-hit sentinels
    std::vector<rtk::MatRec> mat;
    bool bvh_ok = false;
    double origin_bound = 0;
    std::vector<rtk::BvhNode> nodes;
    std::vector<rtk::BvhLeaf> leaves;
    std::vector<rtk::GeoRec> ageo;
    std::vector<uint32_t> asid;
    uint32_t n_nodes = 0, n_leaves = 0, n_always = 0, depth = 0;
    bool trained = false;      // the tree was built from sample rays of camera `view` (train_bvh)
    bool train_tried = false;  // train_bvh ran for `view` (trained or not: a failure is not retried)
    rt_camera view{};
};

// Ray-driven tree (rtbvh::build with sample rays): trained for launches of at least
// kTrainMinSamples samples on scenes of at least kTrainMinSpheres spheres, from the paths of
// kTrainSamples camera samples.  Config 4: node visits per ray 6.97 -> 6.2.
constexpr uint64_t kTrainMinSamples = 1ull << 25;
constexpr size_t kTrainMinSpheres = 32;
#ifndef RTZIG_TRAIN_SAMPLES
#define RTZIG_TRAIN_SAMPLES 6000
#endif
constexpr size_t kTrainSamples = RTZIG_TRAIN_SAMPLES;  // build knob
constexpr uint64_t kTrainSeed = 0x7261792d74726565ull;
constexpr uint32_t kLinearMaxSpheres = 8;    // scenes this small walk the list (use_bvh)
constexpr const char* kStallMsg =
    "render kernel: a wave gave up waiting for a running-sum hand-off (one wait exceeded its bound: 40 s, "
    "scaled with the sphere count for list walks)";

// Phase trace of one rt_render call (diagnostics: RTZIG_TRACE=1 prints one JSON line to stderr).
// The drop-in's cost in the reference's own usage is one call per process (main.zig:14-36), so its
// fixed costs — HIP runtime init, context, scene upload, tree training, workspace, code-object load
// at the first launch — matter as much as the frame; each mark adds the wall time since the
// previous mark to its phase.  Marks are taken only on the thread that called rt_render (the
// per-device threads of a multi-GPU call are covered by the mark after they join).
struct PhaseTrace {
    std::chrono::steady_clock::time_point t0, last;
    std::vector<std::pair<std::string, double>> ms;
};
PhaseTrace g_trace;  // touched only by the tracing thread (g_trace_tid), under g_cache_mu
// the thread of the rt_render call being traced (default id: none); every mark reads it, on any
// thread (context calls of other threads too), so it is the one shared word
std::atomic<std::thread::id> g_trace_tid{};

bool tracing() { return g_trace_tid.load(std::memory_order_relaxed) == std::this_thread::get_id(); }

void trace_mark(const char* phase) {
    if (!tracing()) return;
    const auto now = std::chrono::steady_clock::now();
    const double d = std::chrono::duration<double, std::milli>(now - g_trace.last).count();
    g_trace.last = now;
    for (auto& p : g_trace.ms)
        if (p.first == phase) {
            p.second += d;
            return;
        }
    g_trace.ms.emplace_back(phase, d);
}

// a duration measured elsewhere (a host thread), reported under its own name
void trace_note(const char* name, double ms) {
    if (!tracing()) return;
    g_trace.ms.emplace_back(std::string("[") + name + "]", ms);
}

}  // namespace

struct rt_context {
    int device = 0;
    hipStream_t stream = nullptr;   // uploads, and the stream rt_render renders on
    rtk::GeoRec* d_geo = nullptr;
    rtk::MatRec* d_mat = nullptr;
    uint32_t n_spheres = 0;
    uint32_t capacity = 0;
    // workspace (rt_kernel.h "Work units"): wave rings, running sums, per-tile flags, counters
    double* d_ring = nullptr;
    size_t ring_bytes = 0;
    uint32_t ring_waves = 0;        // waves the ring holds (sized to the launched kernel's grid)
    double* d_sums = nullptr;
    size_t sums_bytes = 0;
    uint32_t* d_flags = nullptr;
    size_t flags_bytes = 0;
    double* d_samples = nullptr;    // direct mode: [spp][P][3] (at most rtk::kDirectBytes)
    size_t samples_bytes = 0;
    double* d_samples2 = nullptr;   // the second per-sample buffer of split calls (rt_render_rows_async_split)
    size_t samples2_bytes = 0;
    uint32_t samples_flip = 0;      // the buffer the next split call's samples go to
    hipEvent_t reduced[2] = {nullptr, nullptr};  // the last reduce pass that read buffer 0 / 1 has ended
    bool reduced_valid[2] = {false, false};
    // a deferred call's reduce pass not yet run (rt_render_rows_async_deferred): its samples sit in
    // buffer fold_buf, its output is promised on fold_stream; the next deferred call's drained waves
    // fold it, or flush_fold runs it whole
    bool fold_pending = false;
    uint32_t fold_buf = 0;
    rtk::FoldArgs fold{};
    hipStream_t fold_stream = nullptr;
    unsigned long long* d_fold_ctr = nullptr;  // 2 chunk counters, 128 B apart
    std::vector<uint32_t> sched;    // chunk table of the last launch (rt_schedule.hpp), and its copy
    uint32_t* d_sched = nullptr;
    size_t sched_bytes = 0;
    uint64_t sched_lanes = 0;       // resident lanes the schedule is sized for (CUs x 16 waves x 64)
    unsigned long long* d_ctr = nullptr;  // rtk::kCtrBytes, zeroed per launch ([kErrWord]: error word)
    const char* last_kernel = "sample_kernel";
    SceneData scene;                // host copy (BVH rebuilds for far-away cameras, scene comparisons)
    rtk::BvhArgs bvh{};
    rtk::BvhNode* d_nodes = nullptr;
    rtk::BvhLeaf* d_leaves = nullptr;
    rtk::GeoRec* d_always_geo = nullptr;
    uint32_t* d_always_sid = nullptr;
    size_t nodes_bytes = 0, leaves_bytes = 0, always_geo_bytes = 0, always_sid_bytes = 0;
    // ordering: `done` is recorded after the last operation of a render call (the reduce pass of a
    // split call: on its out stream, which waited for the sample kernel); device buffers are only
    // rewritten after it (quiesce).  `launched` is recorded on the launch stream after the sample
    // kernel: a render on another stream first waits for it, and a render that writes a per-sample
    // buffer waits for the reduce pass that last read it (`reduced`).
    hipEvent_t done = nullptr;
    bool done_valid = false;
    hipEvent_t launched = nullptr;
    bool launched_valid = false;
    hipStream_t launched_stream = nullptr;
    // optional kernel timing: an event pair around every launch
    bool timing = false;
    bool profile = false;  // instrumented kernels: d_stats must hold RT_PROFILE_STATS_WORDS uint64 (rt.h)
    int precision = RT_PRECISION_F64;
    std::vector<hipEvent_t> events;  // 3 per timed call: start, sample kernel done, reduce done
    uint32_t call_first = 0;
    uint32_t timed_calls = 0;
    uint32_t log_used = 0;
    // rt_render's cached output staging (device rows + pinned host copy + stats)
    void* d_out = nullptr;
    size_t d_out_bytes = 0;
    void* h_out = nullptr;
    size_t h_out_bytes = 0;
    uint64_t* d_stats = nullptr;
    uint64_t* h_stats = nullptr;
};

namespace {

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
    // the camera vectors must be finite (the reference would render NaN pixels; here a NaN center
    // would also defeat the BVH's origin bound); t_max may be +inf, never NaN
    const double* v[6] = {c->center, c->pixel0, c->du, c->dv, c->defocus_disk_u, c->defocus_disk_v};
    bool finite = std::isfinite(c->defocus_angle) && std::isfinite(c->t_min) && !std::isnan(c->t_max);
    for (const double* x : v)
        for (int a = 0; a < 3; a++) finite = finite && std::isfinite(x[a]);
    if (!finite) {
        rt_set_last_error("camera vectors, defocus_angle and t_min must be finite (t_max may be +inf)");
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

// Builder ref (node index >= 0, ~leaf index < 0) -> device ref (byte offsets, see build_bvh).
int32_t device_ref(int32_t ref) {
    if (ref >= 0) return (int32_t)((int64_t)ref * (int64_t)sizeof(rtk::BvhNode));
    return ~(int32_t)((int64_t)(~ref) * (int64_t)sizeof(rtk::BvhLeaf));
}

rtk::GeoRec geo_of(const rt_sphere* s) {
    rtk::GeoRec g;
    if (!s) {  // never-hit sentinel (rt_kernel.h)
        g.cx = g.cy = g.cz = 0.0;
        g.r2 = -std::numeric_limits<double>::infinity();
        return g;
    }
    const double r = s->radius > 0 ? s->radius : 0.0;  // Sphere.init clamps (sphere.zig:21)
    g.cx = s->center[0];
    g.cy = s->center[1];
    g.cz = s->center[2];
    g.r2 = r * r;
    return g;
}

// Sets sd's device tree from `bvh` (built for ray origins with |o_i| <= bound; rt_kernel.h layout).
void set_tree(SceneData& sd, const rtbvh::Bvh& bvh, double bound) {
    sd.trained = false;
    sd.train_tried = false;
    // byte-offset refs must fit int32 (and stay clear of the walk's INT32_MIN "done" marker)
    const bool fits = bvh.nodes.size() * sizeof(rtk::BvhNode) < (1ull << 30) &&
                      bvh.slot_to_sphere.size() / rtk::kLeafBvh * sizeof(rtk::BvhLeaf) < (1ull << 30);
    sd.bvh_ok = bvh.ok && fits;
    sd.origin_bound = bound;
    if (!sd.bvh_ok) return;
    static_assert(rtbvh::kLeafMax == rtk::kLeafBvh && rtbvh::kMaxDepth == rtk::kMaxDepthBvh, "BVH constants differ");
    const size_t nn = bvh.nodes.size();
    const size_t na = bvh.n_always;
    const size_t nl = (bvh.slot_to_sphere.size() - na) / rtk::kLeafBvh;
    auto sphere = [&](uint32_t k) { return k == rtbvh::kSentinel ? nullptr : &sd.spheres[k]; };
    sd.nodes.assign(nn, rtk::BvhNode{});
    for (size_t i = 0; i < nn; i++) {
        const rtbvh::Node& src = bvh.nodes[i];
        rtk::BvhNode& d = sd.nodes[i];
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
    sd.leaves.assign(nl ? nl : 1, rtk::BvhLeaf{});
    for (size_t l = 0; l < nl; l++)
        for (int u = 0; u < rtk::kLeafBvh; u++) {
            const uint32_t k = bvh.slot_to_sphere[na + l * rtk::kLeafBvh + u];
            const rtk::GeoRec g = geo_of(sphere(k));
            sd.leaves[l].g[u] = rtk::LeafGeo{g.cx, g.cy, g.cz, g.r2};
            sd.leaves[l].sid[u] = k;
        }
    sd.ageo.assign(na ? na : 1, geo_of(nullptr));
    sd.asid.assign(na ? na : 1, 0);
    for (size_t q = 0; q < na; q++) {
        sd.ageo[q] = geo_of(sphere(bvh.slot_to_sphere[q]));
        sd.asid[q] = bvh.slot_to_sphere[q];
    }
    sd.n_nodes = (uint32_t)nn;
    sd.n_leaves = (uint32_t)nl;
    sd.n_always = (uint32_t)na;
    sd.depth = (uint32_t)std::max(2, std::min(bvh.depth, rtk::kMaxDepthBvh));
}

// The SAH BVH of sd.spheres, valid for ray origins with |o_i| <= bound.
void build_bvh(SceneData& sd, double bound) {
    rtbvh::Bvh bvh;  // ok = false: the linear walk
    try {            // the builder uses host threads for the top of the tree
        bvh = rtbvh::build(sd.spheres.data(), sd.spheres.size(), bound);
    } catch (const std::exception&) {
        bvh = rtbvh::Bvh{};
    }
    set_tree(sd, bvh, bound);
}

// Do two cameras shoot the same rays (every field getRay / rayColor read except spp and seed)?
bool same_view(const rt_camera& a, const rt_camera& b) {
    rt_camera x = a, y = b;
    x.samples_per_pixel = y.samples_per_pixel = 0;
    x.pixel_samples_scale = y.pixel_samples_scale = 0;
    x.seed = y.seed = 0;
    return std::memcmp(&x, &y, sizeof x) == 0;
}

// Should a launch of `samples` samples train the tree for its camera?  RTZIG_BVH_TRAIN=0|1 forces
// it off / on (test hook: trained trees on small launches).
bool want_train(const SceneData& sd, uint64_t samples) {
    if (const char* e = std::getenv("RTZIG_BVH_TRAIN")) {
        if (std::strcmp(e, "0") == 0) return false;
        if (std::strcmp(e, "1") == 0) return sd.bvh_ok;
    }
    return sd.bvh_ok && samples >= kTrainMinSamples && sd.spheres.size() >= kTrainMinSpheres;
}

// Rebuilds sd's tree from sample rays of `cam` (rtbvh::sample_rays over the SAH tree, then the
// ray-driven build).  The result depends only on (spheres, origin bound, view), so it is memoised
// process-wide: rt_render's devices and later calls reuse it.  Any valid tree returns the same
// bits (rt_bvh.hpp); this one only visits fewer nodes for this camera's rays.  A training that
// fails or is rejected (builder exception, no tree, LDS budget) keeps the current tree and is
// memoised too (train_tried), so later launches of the same view do not quiesce and retry it.
bool try_train(SceneData& sd, const rt_camera& cam) {
    const double bound = sd.origin_bound;
    rtbvh::Bvh sah, tree;
    try {  // the trained build runs on host threads; if they cannot be had, keep the current tree
        sah = rtbvh::build(sd.spheres.data(), sd.spheres.size(), bound);
        if (!sah.ok) return false;
        const std::vector<rtbvh::TrainRay> rays =
            rtbvh::sample_rays(sd.spheres.data(), sd.spheres.size(), cam, sah, kTrainSamples, kTrainSeed);
        tree = rtbvh::build(sd.spheres.data(), sd.spheres.size(), bound, &rays);
    } catch (const std::exception&) {
        return false;
    }
    if (!tree.ok) return false;
    // the kernel stages the tree in LDS when tree + stacks fit a block's 80 KiB (rt_kernel.hip); a
    // trained tree that would not fit where the SAH tree does (or does not build) is not used
    auto lds_bytes = [](const SceneData& t) {
        return (size_t)rtk::bvh_leaves_offset(t.n_nodes) + (size_t)t.n_leaves * sizeof(rtk::BvhLeaf) +
               (size_t)t.depth * rtk::kBlockBvh * sizeof(rtk::StackEntry);
    };
    SceneData sah_sd = sd;
    set_tree(sah_sd, sah, bound);
    SceneData tr = sd;
    set_tree(tr, tree, bound);
    if (!tr.bvh_ok || (lds_bytes(tr) > rtk::kLdsSceneBudget && lds_bytes(sah_sd) <= rtk::kLdsSceneBudget)) {
        if (sah_sd.bvh_ok) sd = sah_sd;
        return false;
    }
    sd = tr;
    return true;
}

// The tree preparation a launch of `samples` samples with camera `cam` does before it runs
// (render_rows): a rebuild with a larger origin bound when the camera's ray origins lie beyond it,
// then the ray-driven training.  Host work only; rt_render runs it on a host thread while the HIP
// runtime and the contexts initialise, so render_rows finds nothing left to do.
double cam_origin_bound(const rt_camera& cam) {
    double b = 0;
    for (int a = 0; a < 3; a++)
        b = std::max(b, std::fabs(cam.center[a]) + std::fabs(cam.defocus_disk_u[a]) + std::fabs(cam.defocus_disk_v[a]));
    return b;
}
bool needs_far_rebuild(const SceneData& sd, const rt_camera& cam) {
    return sd.bvh_ok && !(cam_origin_bound(cam) <= sd.origin_bound);
}
double far_bound(const SceneData& sd, const rt_camera& cam) {
    return std::max(cam_origin_bound(cam), sd.origin_bound) * 1.01;
}
bool needs_training(const SceneData& sd, const rt_camera& cam, uint64_t samples) {
    return want_train(sd, samples) && !(sd.train_tried && same_view(sd.view, cam));
}
void train_bvh(SceneData& sd, const rt_camera& cam);

void train_bvh(SceneData& sd, const rt_camera& cam) {
    static std::mutex mu;
    static SceneData memo;
    static bool memo_valid = false;
    std::lock_guard<std::mutex> lock(mu);
    if (memo_valid && same_view(memo.view, cam) && memo.origin_bound == sd.origin_bound &&
        memo.spheres.size() == sd.spheres.size() &&
        std::memcmp(memo.spheres.data(), sd.spheres.data(), sd.spheres.size() * sizeof(rt_sphere)) == 0) {
        sd = memo;
        return;
    }
    const bool ok = try_train(sd, cam);
    sd.trained = ok;
    sd.train_tried = true;
    sd.view = cam;
    memo = sd;
    memo_valid = true;
}

// Device records + BVH of a sphere list (validated by the caller).
void build_scene(const rt_sphere* spheres, size_t n, SceneData& sd) {
    sd = SceneData{};
    sd.spheres.assign(spheres, spheres + n);
    const size_t n_pad = (n + rtk::kPad - 1) / rtk::kPad * rtk::kPad;
    sd.geo.assign(n_pad, geo_of(nullptr));
    sd.mat.assign(n, rtk::MatRec{});
    for (size_t k = 0; k < n; k++) {
        sd.geo[k] = geo_of(&spheres[k]);
        rtk::MatRec& m = sd.mat[k];
        const double r = spheres[k].radius > 0 ? spheres[k].radius : 0.0;
        for (int c = 0; c < 3; c++) m.albedo[c] = spheres[k].albedo[c];
        m.fuzz = spheres[k].fuzz;
        m.ior = spheres[k].refraction_index;
        m.inv_r = 1.0 / r;
        const double ior = spheres[k].refraction_index;
        m.inv_ior = 1.0 / ior;
        for (int face = 0; face < 2; face++) {  // reflectance()'s r0 (material.zig:106-108) per face
            const double ri = face == 0 ? m.inv_ior : ior;
            double r0 = (1 - ri) / (1 + ri);
            r0 = r0 * r0;
            (face == 0 ? m.r0_front : m.r0_back) = r0;
        }
        m.kind = spheres[k].material;
    }
    const double extent = rtbvh::scene_extent(spheres, n);
    build_bvh(sd, extent * (1.0 + 0x1p-20) + 1e-300);
}

bool same_spheres(const SceneData& sd, const rt_sphere* s, size_t n) {
    return sd.spheres.size() == n && n && std::memcmp(sd.spheres.data(), s, n * sizeof(rt_sphere)) == 0;
}

// Runs a deferred call's pending reduce pass whole, on the stream its output was promised on, after
// the last launch (which wrote or folded nothing of it since it is still pending).  own_stream: on
// the context's own stream instead (rt_context_destroy, which waits for the pass before returning,
// so the caller's stream — possibly destroyed already — is never touched there).
int flush_fold(rt_context* ctx, bool own_stream = false) {
    if (!ctx->fold_pending) return RT_OK;
    ctx->fold_pending = false;
    hipStream_t fs = own_stream ? ctx->stream : ctx->fold_stream;
    if (ctx->launched_valid) HIP_CHECK(hipStreamWaitEvent(fs, ctx->launched, 0));
    HIP_CHECK(hipMemsetAsync(ctx->fold.ctr, 0, sizeof(unsigned long long), fs));
    HIP_CHECK(rtk_launch_fold_rest(&ctx->fold, fs));
    HIP_CHECK(hipEventRecord(ctx->reduced[ctx->fold_buf], fs));
    ctx->reduced_valid[ctx->fold_buf] = true;
    HIP_CHECK(hipEventRecord(ctx->done, fs));
    ctx->done_valid = true;
    return RT_OK;
}

// Waits until the device has finished the context's last render (before rewriting its buffers); a
// pending deferred reduce pass is run first.  `done` marks the end of the LAST call only: a reduce
// pass of an earlier split / deferred call runs on that call's out stream and may still read its
// per-sample buffer, so the passes' own events are waited for too.
int quiesce(rt_context* ctx, bool own_stream = false) {
    int rc = flush_fold(ctx, own_stream);
    if (rc) return rc;
    if (ctx->done_valid) HIP_CHECK(hipEventSynchronize(ctx->done));
    for (int b = 0; b < 2; b++)
        if (ctx->reduced_valid[b]) HIP_CHECK(hipEventSynchronize(ctx->reduced[b]));
    if (ctx->launched_valid) HIP_CHECK(hipEventSynchronize(ctx->launched));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

int ensure_buffer(rt_context* ctx, void** ptr, size_t* bytes, size_t need) {
    if (*ptr && *bytes >= need) return RT_OK;
    int rc = quiesce(ctx);
    if (rc) return rc;
    (void)hipFree(*ptr);
    *ptr = nullptr;
    *bytes = 0;
    hipError_t e = hipMalloc(ptr, need ? need : 1);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(workspace)");
    *bytes = need;
    return RT_OK;
}

// ensure_buffer that also gives memory back: a buffer more than 25% larger than `need` (held for
// an earlier, larger launch or a kernel with more resident waves) is reallocated at `need`
int fit_buffer(rt_context* ctx, void** ptr, size_t* bytes, size_t need) {
    if (*ptr && *bytes > need + need / 4) {
        int rc = quiesce(ctx);
        if (rc) return rc;
        (void)hipFree(*ptr);
        *ptr = nullptr;
        *bytes = 0;
    }
    return ensure_buffer(ctx, ptr, bytes, need);
}

// Frees a workspace buffer the current launch's mode does not use (after the last render).
int release_buffer(rt_context* ctx, void** ptr, size_t* bytes) {
    if (!*ptr) return RT_OK;
    int rc = quiesce(ctx);
    if (rc) return rc;
    (void)hipFree(*ptr);
    *ptr = nullptr;
    *bytes = 0;
    return RT_OK;
}

template <class T>
int upload(rt_context* ctx, T** dptr, size_t* bytes, const std::vector<T>& v) {
    int rc = ensure_buffer(ctx, (void**)dptr, bytes, v.size() * sizeof(T));
    if (rc) return rc;
    HIP_CHECK(hipMemcpyAsync(*dptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
    return RT_OK;
}

// After a failed upload the context holds no scene: its device buffers may have been freed or
// half-written, so the host copy must not vouch for them (a cached rt_render context would compare
// same_spheres() as true and launch on freed memory).  The next set_scene / rt_render re-uploads.
void invalidate_scene(rt_context* ctx) {
    ctx->scene = SceneData{};
    ctx->n_spheres = 0;
    ctx->bvh = rtk::BvhArgs{};
}

int upload_bvh_buffers(rt_context* ctx) {
    const SceneData& sd = ctx->scene;
    ctx->bvh = rtk::BvhArgs{};  // the buffers below may be reallocated
    int rc = quiesce(ctx);
    if (!rc) rc = upload(ctx, &ctx->d_nodes, &ctx->nodes_bytes, sd.nodes);
    if (!rc) rc = upload(ctx, &ctx->d_leaves, &ctx->leaves_bytes, sd.leaves);
    if (!rc) rc = upload(ctx, &ctx->d_always_geo, &ctx->always_geo_bytes, sd.ageo);
    if (!rc) rc = upload(ctx, &ctx->d_always_sid, &ctx->always_sid_bytes, sd.asid);
    if (rc) return rc;
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

// Uploads ctx->scene's tree (any failure leaves the context without a scene: invalidate_scene).
int upload_bvh(rt_context* ctx) {
    if (!ctx->scene.bvh_ok) return RT_OK;
    const int rc = upload_bvh_buffers(ctx);
    if (rc) {
        invalidate_scene(ctx);
        return rc;
    }
    const SceneData& sd = ctx->scene;
    rtk::BvhArgs& b = ctx->bvh;
    b = rtk::BvhArgs{};
    b.nodes = ctx->d_nodes;
    b.leaves = ctx->d_leaves;
    b.always_geo = ctx->d_always_geo;
    b.always_sid = ctx->d_always_sid;
    b.n_nodes = sd.n_nodes;
    b.n_leaves = sd.n_leaves;
    b.n_always = sd.n_always;
    b.stack_depth = sd.depth;
    float ob = (float)sd.origin_bound;  // rounded down: a lane counts as "far" no later than the padding allows
    if ((double)ob > sd.origin_bound) ob = std::nextafterf(ob, 0.0f);
    // test hook: RTZIG_BVH_ORIGIN_SCALE=<s> < 1 marks lanes "far" early, so the tests can check the
    // no-culling walk of far-origin lanes against the oracle on rays that do hit spheres
    if (const char* e = std::getenv("RTZIG_BVH_ORIGIN_SCALE")) ob = (float)(ob * std::min(1.0, std::atof(e)));
    b.origin_bound = ob;
    return RT_OK;
}

// Uploads a host scene to the context's device (a copy stays on the host side of the context).
// The host copy is committed only once every device buffer holds it.
int upload_scene_buffers(rt_context* ctx, const SceneData& sd) {
    HIP_CHECK(hipSetDevice(ctx->device));
    int rc = quiesce(ctx);
    if (rc) return rc;
    const size_t n_pad = sd.geo.size(), n = sd.mat.size();
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
    HIP_CHECK(hipMemcpyAsync(ctx->d_geo, sd.geo.data(), n_pad * sizeof(rtk::GeoRec), hipMemcpyHostToDevice, ctx->stream));
    HIP_CHECK(hipMemcpyAsync(ctx->d_mat, sd.mat.data(), n * sizeof(rtk::MatRec), hipMemcpyHostToDevice, ctx->stream));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return RT_OK;
}

int upload_scene(rt_context* ctx, const SceneData& sd) {
    invalidate_scene(ctx);  // nothing on the device vouches for the old scene any more
    const int rc = upload_scene_buffers(ctx, sd);
    if (rc) return rc;
    ctx->scene = sd;
    ctx->n_spheres = (uint32_t)sd.mat.size();
    return upload_bvh(ctx);  // invalidates again on failure
}

// Walk selection: RTZIG_KERNEL names a linear variant (lds_u4, smem_u4) or "bvh"; default: the
// BVH walk when it built, except for tiny scenes in f64, where the list walk in LDS is faster
// (chapter 9's 2 spheres -11.5%, chapter 13's 5 spheres -2%: profiles/r02_walk_ab/).  Fast mode
// (f32) always walks the tree.
bool use_bvh(const rt_context* ctx) {
    const char* e = std::getenv("RTZIG_KERNEL");
    if (e) return std::strncmp(e, "bvh", 3) == 0 && ctx->scene.bvh_ok;
    if (ctx->precision == RT_PRECISION_F64 && ctx->n_spheres <= kLinearMaxSpheres) return false;
    return ctx->scene.bvh_ok;
}

// Uploads the chunk table of rt_schedule.hpp for `spp` samples over `pixels` (unchanged tables are
// not re-sent; a changed one waits for the last render, which may still read the old one).
int upload_schedule(rt_context* ctx, uint32_t spp, uint64_t pixels) {
    std::vector<uint32_t> t = rtk::chunk_schedule(spp, pixels, ctx->sched_lanes, rtk::kUnitS);
    if (ctx->d_sched && t == ctx->sched) return RT_OK;
    int rc = quiesce(ctx);
    if (!rc) rc = ensure_buffer(ctx, (void**)&ctx->d_sched, &ctx->sched_bytes, t.size() * sizeof(uint32_t));
    if (rc) return rc;
    HIP_CHECK(hipMemcpyAsync(ctx->d_sched, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice, ctx->stream));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    ctx->sched = std::move(t);
    return RT_OK;
}

rtk::KernelParams make_params(const rt_camera* c, uint32_t row0, uint32_t row_step, uint32_t n_rows,
                              uint32_t n_spheres) {
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
    return p;
}

// The sticky error word's message (rt_units.h: bit 0 a hand-off wait gave up; bit 1, debug builds
// only, an index out of range)
std::string err_message(unsigned long long err) {
    std::string m;
    if (err & rtk::kErrBounds) m = "render kernel: an index out of range (RTZIG_BOUNDS debug build)";
    if (err & rtk::kErrStall) m += (m.empty() ? "" : "; ") + std::string(kStallMsg);
    return m;
}

// Bound on one continuous hand-off wait of ring mode (rt_units.h), in wait_clock units.  A wave
// waits for the unit holding the previous sample chunk of the same 64 pixels, traced meanwhile by
// another wave; that unit's time is bounded by its 3072 samples' paths.  Through the BVH it is
// milliseconds on any scene (the final scene: ~1 ms), and 40 s is the bound.  Scenes without a tree
// (list walk: > 2^15 leaves, or RTZIG_KERNEL) cost ~n per ray segment: 70 000 spheres measured
// ~100x the final scene's per-segment cost; the bound grows by 40 s per 2^16 spheres, up to
// kStallMaxSec (2^24 spheres, the ABI's maximum: 10 000 s).
uint32_t stall_bound(bool bvh, uint32_t n_spheres) {
    uint64_t sec = rtk::kStallBaseSec;
    if (!bvh) sec *= std::max<uint64_t>(1, ((uint64_t)n_spheres + 65535) / 65536);
    sec = std::min<uint64_t>(sec, rtk::kStallMaxSec);
    return (uint32_t)(sec * rtk::kStallUnitsPerSec);
}

hipError_t make_event(hipEvent_t* e, bool timed) {
    return timed ? hipEventCreate(e) : hipEventCreateWithFlags(e, hipEventDisableTiming);
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
    trace_mark("ctx_set_device");
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device));
    trace_mark("ctx_device_props");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        rt_set_last_error(std::string("device is ") + prop.gcnArchName + ", library built for gfx950");
        return RT_ERR_NO_DEVICE;
    }
    auto* ctx = new rt_context;
    ctx->device = device;
    hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = make_event(&ctx->done, false);
    if (e == hipSuccess) e = make_event(&ctx->launched, false);
    if (e == hipSuccess) e = make_event(&ctx->reduced[0], false);
    if (e == hipSuccess) e = make_event(&ctx->reduced[1], false);
    int cus = 0;
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    ctx->sched_lanes = (uint64_t)std::max(cus, 1) * 16 * 64;
    trace_mark("ctx_streams_events");
    if (e != hipSuccess) {
        const int rc = hip_fail(e, "rt_context_create: stream / event");
        rt_context_destroy(ctx);
        return rc;
    }
    *out_ctx = ctx;
    return RT_OK;
}

int rt_context_destroy(rt_context* ctx) {
    if (!ctx) return RT_OK;
    (void)hipSetDevice(ctx->device);
    // a deferred call's pending reduce pass is run, not dropped: its output was promised to the
    // caller (the reference's render always fills ppm.pixels, camera.zig:125,138); then every
    // launch and pass that may still use a buffer is waited for before anything is freed.  The
    // pass runs on the context's own stream (after the launch it depends on): destroy blocks until
    // it is complete, so the caller's out stream gives no ordering the caller would not have anyway,
    // and a caller may already have destroyed that stream.  A context whose stream was never
    // created (a failed rt_context_create) has launched nothing and is not waited for.
    const int rc = ctx->stream ? quiesce(ctx, true) : RT_OK;
    if (rc) {  // still free what can be freed after a device-wide wait
        (void)hipDeviceSynchronize();
    }
    for (void* p : {(void*)ctx->d_geo, (void*)ctx->d_mat, (void*)ctx->d_ring, (void*)ctx->d_sums, (void*)ctx->d_flags,
                    (void*)ctx->d_samples, (void*)ctx->d_samples2, (void*)ctx->d_fold_ctr, (void*)ctx->d_sched, (void*)ctx->d_ctr, (void*)ctx->d_nodes, (void*)ctx->d_leaves, (void*)ctx->d_always_geo,
                    (void*)ctx->d_always_sid, ctx->d_out, (void*)ctx->d_stats})
        (void)hipFree(p);
    if (ctx->h_out) (void)hipHostFree(ctx->h_out);
    if (ctx->h_stats) (void)hipHostFree(ctx->h_stats);
    for (hipEvent_t e : ctx->events) (void)hipEventDestroy(e);
    for (hipEvent_t e : {ctx->done, ctx->launched, ctx->reduced[0], ctx->reduced[1]})
        if (e) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
    return rc;  // a failed flush: the context is gone, the pending output may be incomplete
}

int rt_context_set_scene(rt_context* ctx, const rt_sphere* spheres, size_t n) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    int rc = validate_spheres(spheres, n);
    if (rc) return rc;
    SceneData sd;
    build_scene(spheres, n, sd);
    return upload_scene(ctx, sd);
}

int rt_context_sync(rt_context* ctx) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    HIP_CHECK(hipSetDevice(ctx->device));
    int rc = quiesce(ctx);
    if (rc || !ctx->d_ctr) return rc;
    // the error word is sticky across launches: it reports a failure of ANY render since the last
    // report, and is cleared once reported
    // (on the context's stream and waited for: hipMemcpy / hipMemset on the null stream are not
    // ordered with the context's non-blocking streams)
    unsigned long long err = 0;
    HIP_CHECK(hipMemcpyAsync(&err, ctx->d_ctr + rtk::kErrWord, sizeof err, hipMemcpyDeviceToHost, ctx->stream));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (err) {
        HIP_CHECK(hipMemsetAsync(ctx->d_ctr + rtk::kErrWord, 0, sizeof err, ctx->stream));
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
        rt_set_last_error(err_message(err));
        return RT_ERR_HIP;
    }
    return RT_OK;
}

}  // extern "C"

namespace {

// One render call.  !split: everything on s (rt_render_rows_async).  Otherwise the output is
// completed in os's order (os may be the null stream): direct mode's reduce pass runs on os after the sample kernel on s, over
// one of two per-sample buffers taken in turn, so the next call's sample kernel on s need not wait
// for this call's reduce pass (rt_render_rows_async_split).
int render_rows(rt_context* ctx, const rt_camera* cam, uint32_t output_format, uint32_t row0, uint32_t row_step,
                uint32_t n_rows, void* d_out, void* d_stats, hipStream_t s, hipStream_t os, bool split,
                bool defer) {
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
    if (os == s) split = defer = false;  // one stream: the plain call (os may be the null stream)

    // camera-ray origins (center + defocus disk) must lie inside the BVH padding's origin bound
    // (lanes outside it would walk without culling: correct, but every camera ray would pay)
    if (needs_far_rebuild(ctx->scene, *cam)) {
        rc = quiesce(ctx);  // the previous render may still walk the old tree
        if (rc) return rc;
        build_bvh(ctx->scene, far_bound(ctx->scene, *cam));
        rc = upload_bvh(ctx);
        if (rc) return rc;
        trace_mark("bvh_rebuild_far_camera");
    }
    // large launches walk a tree trained on this camera's rays (same bits, fewer node visits)
    if (needs_training(ctx->scene, *cam, (uint64_t)n_rows * cam->image_width * cam->samples_per_pixel)) {
        rc = quiesce(ctx);  // the previous render may still walk the old tree
        if (rc) return rc;
        trace_mark("wait_previous_render");
        train_bvh(ctx->scene, *cam);
        trace_mark("bvh_train_host");
        rc = upload_bvh(ctx);
        if (rc) return rc;
        trace_mark("bvh_upload");
    }

    const uint64_t P = (uint64_t)n_rows * cam->image_width;
    rtk::UnitArgs ua;
    std::memset(&ua, 0, sizeof ua);
    const uint64_t n_tiles = (P + 63) / 64;
    rc = upload_schedule(ctx, cam->samples_per_pixel, P);
    if (rc) return rc;
    trace_mark("schedule_upload");
    ua.chunk_s0 = ctx->d_sched;
    ua.n_chunks = (uint32_t)(ctx->sched.size() - 1);
    if (n_tiles * ua.n_chunks >= (1ull << 32)) {
        rt_set_last_error("too many work units (rows x samples): render fewer rows per call");
        return RT_ERR_CAPACITY;
    }
    // direct mode for small launches (rt_kernel.h "Work units"); RTZIG_UNIT_MODE=ring|direct forces
    // one (test hook: both paths on the same inputs)
    const uint64_t direct_bytes = P * (uint64_t)cam->samples_per_pixel * 3 * sizeof(double);
    bool direct = direct_bytes <= rtk::kDirectBytes;
    if (const char* e = std::getenv("RTZIG_UNIT_MODE")) {
        if (std::strcmp(e, "ring") == 0) direct = false;
        if (std::strcmp(e, "direct") == 0) {
            if (direct_bytes > (16ull << 30)) {
                rt_set_last_error("RTZIG_UNIT_MODE=direct: launch needs more than 16 GiB of sample storage");
                return RT_ERR_CAPACITY;
            }
            direct = true;
        }
    }
    const bool bvh = use_bvh(ctx);
    rtk::KernelParams p = make_params(cam, row0, row_step, n_rows, ctx->n_spheres);
    p.prof = ctx->profile && d_stats ? 1u : 0u;
    p.s_begin = 0;
    p.s_count = cam->samples_per_pixel;
    // the launch for this call's kernel (plan_waves != nullptr: size the grid, launch nothing)
    auto launch = [&](const rtk::UnitArgs* u, uint32_t* plan_waves) -> hipError_t {
        if (bvh && ctx->precision == RT_PRECISION_F32)
            return rtk_launch_samples_fast(&p, &ctx->bvh, ctx->d_geo, ctx->d_mat, u, d_stats, s, &ctx->last_kernel,
                                           direct, plan_waves);
        if (bvh)
            return rtk_launch_samples_bvh(&p, &ctx->bvh, ctx->d_geo, ctx->d_mat, u, d_stats, s, &ctx->last_kernel,
                                          direct, plan_waves);
        return rtk_launch_samples(&p, ctx->d_geo, ctx->d_mat, u, d_stats, s, &ctx->last_kernel, direct, plan_waves);
    };
    // deferred calls (direct mode, an output stream): this call's reduce pass is left pending for the
    // next deferred call's drained waves; a pending pass this call will not fold (a plain or ring-mode
    // call, another launch size) runs whole first
    // The pending pass's follow-up fold runs on this call's out stream, so it is folded only when
    // that is the stream the pending output was promised on (a consumer that queued work there after
    // this call is then ordered after the fold); otherwise it runs whole on its own stream first.
    const bool defer_fold = defer && direct && split;
    if (ctx->fold_pending && !(defer_fold && ctx->fold.P == (uint32_t)P && ctx->fold.spp == cam->samples_per_pixel &&
                               ctx->fold_buf == (ctx->samples_flip ^ 1u) && ctx->fold_stream == os)) {
        rc = flush_fold(ctx);
        if (rc) return rc;
    }
    // a context holds the workspace of one mode at a time (rt.h "Workspace"); split calls in direct
    // mode alternate two per-sample buffers
    const bool split_reduce = direct && split;
    uint32_t sbuf = 0;
    if (direct) {
        rc = release_buffer(ctx, (void**)&ctx->d_ring, &ctx->ring_bytes);
        if (!rc) rc = release_buffer(ctx, (void**)&ctx->d_sums, &ctx->sums_bytes);
        ctx->ring_waves = 0;
        if (!rc) rc = fit_buffer(ctx, (void**)&ctx->d_samples, &ctx->samples_bytes, direct_bytes);
        if (split_reduce) {
            if (!rc) rc = fit_buffer(ctx, (void**)&ctx->d_samples2, &ctx->samples2_bytes, direct_bytes);
            sbuf = ctx->samples_flip;
            ctx->samples_flip ^= 1u;
        } else {
            if (!rc) rc = release_buffer(ctx, (void**)&ctx->d_samples2, &ctx->samples2_bytes);
            ctx->samples_flip = 0;
        }
    } else {
        // the ring holds the persistent grid of the kernel this call launches (its resident waves)
        uint32_t waves = 0;
        HIP_CHECK(launch(&ua, &waves));
        waves = std::max(waves, 1u);
        constexpr size_t kWaveBytes = rtk::kRingWaveDoubles * sizeof(double);
        rc = release_buffer(ctx, (void**)&ctx->d_samples, &ctx->samples_bytes);
        if (!rc) rc = release_buffer(ctx, (void**)&ctx->d_samples2, &ctx->samples2_bytes);
        ctx->samples_flip = 0;
        if (!rc) rc = fit_buffer(ctx, (void**)&ctx->d_ring, &ctx->ring_bytes, (size_t)waves * kWaveBytes);
        ctx->ring_waves = rc ? 0u : (uint32_t)(ctx->ring_bytes / kWaveBytes);
        if (!rc && ua.n_chunks > 1) rc = fit_buffer(ctx, (void**)&ctx->d_sums, &ctx->sums_bytes, P * 3 * sizeof(double));
    }
    const size_t flag_bytes = (n_tiles * sizeof(uint32_t) + 15) & ~(size_t)15;  // memset in 16-B multiples
    if (!rc) rc = ensure_buffer(ctx, (void**)&ctx->d_flags, &ctx->flags_bytes, flag_bytes);
    if (!rc && defer_fold && !ctx->d_fold_ctr) {
        size_t fb = 0;
        rc = ensure_buffer(ctx, (void**)&ctx->d_fold_ctr, &fb, 2 * 16 * sizeof(unsigned long long));
    }
    if (!rc && !ctx->d_ctr) {
        size_t cb = 0;
        rc = ensure_buffer(ctx, (void**)&ctx->d_ctr, &cb, rtk::kCtrBytes);
        // the sticky error word starts clear; launches zero only the counters before it.  On the
        // launch stream: a null-stream hipMemset is asynchronous and NOT ordered with this
        // non-blocking stream, so it could land mid-kernel and reset the claim counters.
        if (!rc) HIP_CHECK(hipMemsetAsync(ctx->d_ctr, 0, rtk::kCtrBytes, s));
    }
    if (rc) return rc;
    trace_mark("workspace_alloc");
    ua.ring = direct ? nullptr : ctx->d_ring;
    ua.sums = direct ? nullptr : ctx->d_sums;
    ua.samples = direct ? (sbuf ? ctx->d_samples2 : ctx->d_samples) : nullptr;
    ua.spp = cam->samples_per_pixel;
    ua.flags = ctx->d_flags;
    ua.out = d_out;
    ua.ctr = ctx->d_ctr;
    ua.n_tiles = (uint32_t)n_tiles;
    ua.n_units = direct ? (uint32_t)(P * cam->samples_per_pixel) : (uint32_t)(n_tiles * ua.n_chunks);
    ua.div_p = rtk::fastdiv_make((uint32_t)P);
    ua.div_tiles = rtk::fastdiv_make((uint32_t)n_tiles);
    ua.P = (uint32_t)P;
    ua.out_format = output_format;
    ua.ring_waves = ctx->ring_waves;
    ua.stall_ticks = stall_bound(bvh, ctx->n_spheres);
    // test hook RTZIG_STALL_US=<µs>: a shorter bound, so the tests can drive the give-up path (the
    // sticky error word, RT_ERR_HIP, and the next render succeeding)
    if (const char* e = std::getenv("RTZIG_STALL_US")) {
        const double us = std::atof(e);
        if (us >= 0 && us / rtk::kStallUnitUs < (double)ua.stall_ticks) ua.stall_ticks = (uint32_t)(us / rtk::kStallUnitUs);
    }
    ua.scale = cam->pixel_samples_scale;

    if (ctx->timing) {
        if (ctx->log_used + 1 > kMaxTimed) ctx->log_used = 0;  // wrap: totals restart
        ctx->call_first = ctx->log_used;
        ctx->log_used += 1;
        while (ctx->events.size() < kEventsPerCall * (size_t)ctx->log_used) {
            hipEvent_t e;
            HIP_CHECK(make_event(&e, true));
            ctx->events.push_back(e);
        }
        ctx->timed_calls = 1;
    }
    // a previous render of this context's on another stream may still run its sample kernel (the
    // counters, flags, ring and sums are the sample kernel's own); the per-sample buffer this call
    // writes may still be read by the reduce pass of an earlier call (on any stream)
    if (ctx->launched_valid && ctx->launched_stream != s) HIP_CHECK(hipStreamWaitEvent(s, ctx->launched, 0));
    if (direct && ctx->reduced_valid[sbuf]) HIP_CHECK(hipStreamWaitEvent(s, ctx->reduced[sbuf], 0));
    // the pending pass this launch folds in its tail (the flush above left only a foldable one)
    const bool folding = defer_fold && ctx->fold_pending;
    if (folding) {
        ua.fold = ctx->fold;
        HIP_CHECK(hipMemsetAsync(ctx->fold.ctr, 0, sizeof(unsigned long long), s));
    }
    HIP_CHECK(hipMemsetAsync(ctx->d_ctr, 0, rtk::kCtrLaunchBytes, s));  // not the sticky error word
    if (!direct) HIP_CHECK(hipMemsetAsync(ctx->d_flags, 0, flag_bytes, s));
    hipEvent_t* ev = ctx->timing ? &ctx->events[kEventsPerCall * ctx->call_first] : nullptr;
    if (ev) HIP_CHECK(hipEventRecord(ev[0], s));
    trace_mark("launch_setup");
    HIP_CHECK(launch(&ua, nullptr));
    trace_mark("launch_issue");
    if (ev) HIP_CHECK(hipEventRecord(ev[1], s));
    HIP_CHECK(hipEventRecord(ctx->launched, s));
    ctx->launched_valid = true;
    ctx->launched_stream = s;
    // the stream on which the output is complete: split calls continue on os, after the sample kernel
    hipStream_t rs = s;
    if (split) {
        HIP_CHECK(hipStreamWaitEvent(os, ctx->launched, 0));
        rs = os;
    }
    if (ev) HIP_CHECK(hipEventRecord(ev[2], rs));
    if (folding) {
        if (p.prof) {
            // the instrumented kernels do not fold: the pass runs whole after them
            HIP_CHECK(rtk_launch_fold_rest(&ctx->fold, rs));
            HIP_CHECK(hipEventRecord(ctx->reduced[ctx->fold_buf], rs));
        } else {
            // every wave of the launch claims fold chunks until none is left before it exits
            // (path_loop), so the pass is complete with the kernel: no follow-up pass, and the next
            // launch on this stream finds the buffer free without waiting on the output stream
            HIP_CHECK(hipEventRecord(ctx->reduced[ctx->fold_buf], s));
        }
        ctx->reduced_valid[ctx->fold_buf] = true;
        ctx->fold_pending = false;
    }
    if (defer_fold) {
        rtk::FoldArgs f{};
        f.samples = ua.samples;
        f.out = d_out;
        f.ctr = ctx->d_fold_ctr + 16 * sbuf;
        f.P = (uint32_t)P;
        f.spp = cam->samples_per_pixel;
        f.format = output_format;
        f.n_chunks = (uint32_t)((P + 63) / 64);
        f.scale = ua.scale;
        ctx->fold = f;
        ctx->fold_buf = sbuf;
        ctx->fold_stream = rs;
        ctx->fold_pending = true;
    } else if (direct) {
        HIP_CHECK(rtk_launch_reduce(&ua, rs));
        HIP_CHECK(hipEventRecord(ctx->reduced[sbuf], rs));
        ctx->reduced_valid[sbuf] = true;
    }
    if (ev) HIP_CHECK(hipEventRecord(ev[3], rs));
    HIP_CHECK(hipEventRecord(ctx->done, rs));
    ctx->done_valid = true;
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_render_rows_async(rt_context* ctx, const rt_camera* cam, uint32_t output_format, uint32_t row0,
                         uint32_t row_step, uint32_t n_rows, void* d_out, void* d_stats, void* stream) {
    // NULL = the HIP null stream, like torch's default stream
    return render_rows(ctx, cam, output_format, row0, row_step, n_rows, d_out, d_stats, (hipStream_t)stream, nullptr,
                       false, false);
}

int rt_render_rows_async_split(rt_context* ctx, const rt_camera* cam, uint32_t output_format, uint32_t row0,
                               uint32_t row_step, uint32_t n_rows, void* d_out, void* d_stats, void* stream,
                               void* out_stream) {
    return render_rows(ctx, cam, output_format, row0, row_step, n_rows, d_out, d_stats, (hipStream_t)stream,
                       (hipStream_t)out_stream, true, false);
}

int rt_render_rows_async_deferred(rt_context* ctx, const rt_camera* cam, uint32_t output_format, uint32_t row0,
                                  uint32_t row_step, uint32_t n_rows, void* d_out, void* d_stats, void* stream,
                                  void* out_stream) {
    if (out_stream == stream) {
        rt_set_last_error("rt_render_rows_async_deferred needs an out_stream other than stream");
        return RT_ERR_INVALID;
    }
    return render_rows(ctx, cam, output_format, row0, row_step, n_rows, d_out, d_stats, (hipStream_t)stream,
                       (hipStream_t)out_stream, true, true);
}

int rt_context_fold_pending(rt_context* ctx, int* pending) {
    if (!ctx || !pending) { rt_set_last_error("null context / output"); return RT_ERR_INVALID; }
    *pending = ctx->fold_pending ? 1 : 0;
    return RT_OK;
}

int rt_context_flush(rt_context* ctx) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    HIP_CHECK(hipSetDevice(ctx->device));
    return flush_fold(ctx);
}

int rt_context_enable_timing(rt_context* ctx, int enable) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    ctx->timing = enable != 0;
    ctx->timed_calls = 0;
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

static int sum_times(rt_context* ctx, uint32_t first, uint32_t count, double* sample_ms, double* reduce_ms) {
    HIP_CHECK(hipSetDevice(ctx->device));
    double sm = 0, rm = 0;
    for (uint32_t c = first; c < first + count; c++) {
        float a = 0, b = 0;
        const hipEvent_t* e = &ctx->events[kEventsPerCall * c];  // start, sample kernel done, reduce start, end
        HIP_CHECK(hipEventSynchronize(e[3]));
        HIP_CHECK(hipEventElapsedTime(&a, e[0], e[1]));
        HIP_CHECK(hipEventElapsedTime(&b, e[2], e[3]));
        sm += a;
        rm += b;
    }
    if (sample_ms) *sample_ms = sm;
    if (reduce_ms) *reduce_ms = rm;  // direct mode's reduce pass (ring mode: an empty interval)
    return RT_OK;
}

int rt_context_kernel_times(rt_context* ctx, double* sample_ms, double* reduce_ms) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    if (!ctx->timing || ctx->timed_calls == 0) { rt_set_last_error("timing not enabled or nothing rendered"); return RT_ERR_INVALID; }
    return sum_times(ctx, ctx->call_first, ctx->timed_calls, sample_ms, reduce_ms);
}

int rt_context_kernel_times_total(rt_context* ctx, double* sample_ms, double* reduce_ms, uint32_t* n_launches) {
    if (!ctx) { rt_set_last_error("null context"); return RT_ERR_INVALID; }
    if (!ctx->timing) { rt_set_last_error("timing not enabled"); return RT_ERR_INVALID; }
    const int rc = sum_times(ctx, 0, ctx->log_used, sample_ms, reduce_ms);
    if (rc) return rc;
    if (n_launches) *n_launches = ctx->log_used;
    return RT_OK;
}

const char* rt_kernel_name(rt_context* ctx) { return ctx ? ctx->last_kernel : "render_kernel"; }

int rt_context_tree_info(rt_context* ctx, uint32_t* info) {
    if (!ctx || !info) { rt_set_last_error("null context / output"); return RT_ERR_INVALID; }
    const SceneData& sd = ctx->scene;
    info[0] = ctx->n_spheres && use_bvh(ctx) ? 1u : 0u;
    info[1] = sd.bvh_ok ? sd.n_nodes : 0u;
    info[2] = sd.bvh_ok ? sd.n_leaves : 0u;
    info[3] = sd.bvh_ok ? sd.depth : 0u;
    info[4] = sd.bvh_ok ? sd.n_always : 0u;
    info[5] = sd.bvh_ok && sd.trained ? 1u : 0u;
    return RT_OK;
}

int rt_context_workspace_bytes(rt_context* ctx, uint64_t* bytes) {
    if (!ctx || !bytes) { rt_set_last_error("null context / output"); return RT_ERR_INVALID; }
    *bytes = (uint64_t)ctx->ring_bytes + ctx->sums_bytes + ctx->flags_bytes + ctx->samples_bytes + ctx->samples2_bytes +
             ctx->sched_bytes + (ctx->d_fold_ctr ? 2 * 16 * sizeof(unsigned long long) : 0) +
             (ctx->d_ctr ? rtk::kCtrBytes : 0);
    return RT_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// rt_render: the blocking drop-in for Camera.render, over process-wide cached contexts
// ------------------------------------------------------------------------------------------------
namespace {

std::mutex g_cache_mu;             // guards g_cache and serialises rt_render calls
std::vector<rt_context*> g_cache;  // one context per logical device ordinal (created on first use)

// rt_render's logical devices: ordinal g runs on physical device map[g].  Normally the identity
// over the visible devices.  Test hook RTZIG_DEVICE_MAP=p0,p1,... (physical ordinals, repeats
// allowed) gives rt_render that many logical devices, so the multi-device branch (contexts created
// on host threads, one stream each, row interleave, un-interleave, stats sum) runs on a 1-GPU host
// exactly as on an 8-GPU one: RTZIG_DEVICE_MAP=0,0,0 is three contexts on GPU 0.
int device_map(std::vector<int>& map) {
    int count = 0;
    HIP_CHECK(hipGetDeviceCount(&count));
    if (count <= 0) { rt_set_last_error("no HIP device"); return RT_ERR_NO_DEVICE; }
    map.clear();
    const char* e = std::getenv("RTZIG_DEVICE_MAP");
    if (!e || !*e) {
        for (int d = 0; d < count; d++) map.push_back(d);
        return RT_OK;
    }
    const char* p = e;
    while (*p) {
        char* endp = nullptr;
        const long d = std::strtol(p, &endp, 10);
        if (endp == p || d < 0 || d >= count) {
            rt_set_last_error(std::string("RTZIG_DEVICE_MAP: bad entry in \"") + e + "\" (" + std::to_string(count) +
                              " visible devices)");
            return RT_ERR_NO_DEVICE;
        }
        map.push_back((int)d);
        p = endp;
        if (*p == ',') ++p;
    }
    return RT_OK;
}

// RTZIG_TRACE=1: starts g_trace for one rt_render call and prints it when the call returns
struct TraceScope {
    std::vector<double> kernel_ms;  // HIP-event sample-kernel time per device
    TraceScope() {
        const char* e = std::getenv("RTZIG_TRACE");
        if (!(e && *e && std::strcmp(e, "0") != 0)) return;
        g_trace = PhaseTrace{};
        g_trace.t0 = g_trace.last = std::chrono::steady_clock::now();
        g_trace_tid.store(std::this_thread::get_id(), std::memory_order_relaxed);
    }
    ~TraceScope() {
        if (!tracing()) return;
        trace_mark("return");
        const double total = std::chrono::duration<double, std::milli>(g_trace.last - g_trace.t0).count();
        std::string j = "{\"rt_render_trace\": {\"total_ms\": " + std::to_string(total) + ", \"phases_ms\": {";
        for (size_t i = 0; i < g_trace.ms.size(); i++)
            j += (i ? ", \"" : "\"") + g_trace.ms[i].first + "\": " + std::to_string(g_trace.ms[i].second);
        j += "}, \"kernel_ms\": [";
        for (size_t i = 0; i < kernel_ms.size(); i++) j += (i ? ", " : "") + std::to_string(kernel_ms[i]);
        j += "]}}\n";
        std::fputs(j.c_str(), stderr);
        g_trace_tid.store(std::thread::id{}, std::memory_order_relaxed);
    }
};

// Gets (creating if needed) the cached contexts of devices [first, first + G) and makes each hold
// `spheres`: contexts are created on parallel host threads; the scene is built on the host once
// per call at most and uploaded only where it differs.
// `scene()` returns the host scene (built on first use; rt_render hands in one built and
// tree-prepared on a host thread meanwhile), called only if some context needs it, before any
// upload and on the calling thread.
int cached_contexts(const std::vector<int>& map, int first, int G, const rt_sphere* spheres, size_t n,
                    const std::function<const SceneData&()>& scene, std::vector<rt_context*>& out) {
    if ((int)g_cache.size() < first + G) g_cache.resize(first + G, nullptr);
    for (int g = 0; g < G; g++) {
        rt_context*& c = g_cache[first + g];
        if (c && c->device != map[first + g]) {  // the logical -> physical map changed
            rt_context_destroy(c);
            c = nullptr;
        }
    }
    std::vector<int> rcs(G, RT_OK);
    std::vector<std::string> msgs(G);
    const SceneData* sd = nullptr;
    auto create = [&](int g) {
        rt_context*& c = g_cache[first + g];
        int rc = RT_OK;
        if (!c) rc = rt_context_create(map[first + g], &c);
        rcs[g] = rc;
        if (rc) msgs[g] = rt_last_error();  // thread-local: carried back to the caller's thread
    };
    auto work = [&](int g) {
        rt_context* c = g_cache[first + g];
        int rc = RT_OK;
        if (!same_spheres(c->scene, spheres, n)) rc = upload_scene(c, *sd);
        trace_mark("scene_upload");
        rcs[g] = rc;
        if (rc) msgs[g] = rt_last_error();
    };
    // 1. contexts (the first stream of a process costs ~20 ms: HIP queue creation)
    if (G == 1) {
        create(0);
    } else {
        std::vector<std::thread> th;
        for (int g = 0; g < G; g++) th.emplace_back(create, g);
        for (auto& t : th) t.join();
        trace_mark("contexts_on_device_threads");
    }
    for (int g = 0; g < G; g++)
        if (rcs[g]) {
            rt_set_last_error(msgs[g]);
            return rcs[g];
        }
    // 2. the scene, where a context does not hold it yet
    bool need_scene = false;
    for (int g = 0; g < G; g++) need_scene = need_scene || !same_spheres(g_cache[first + g]->scene, spheres, n);
    if (need_scene) sd = &scene();
    trace_mark("host_scene_ready");
    if (!need_scene) {
        // nothing to upload
    } else if (G == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (int g = 0; g < G; g++) th.emplace_back(work, g);
        for (auto& t : th) t.join();
        trace_mark("scene_upload_on_device_threads");
    }
    for (int g = 0; g < G; g++)
        if (rcs[g]) {
            rt_set_last_error(msgs[g]);
            return rcs[g];
        }
    out.assign(g_cache.begin() + first, g_cache.begin() + first + G);
    return RT_OK;
}

}  // namespace

extern "C" {

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
    std::lock_guard<std::mutex> lock(g_cache_mu);  // also guards g_trace
    TraceScope trace;
    // The host side of a new scene — device records, the SAH tree, and the tree trained on this
    // camera's rays (≈11 ms for the final scene) — runs on a host thread while this one initialises
    // the HIP runtime and the contexts (60-200 ms on a fresh process: the reference renders one
    // image per process, main.zig:14-36).  Skipped when a cached context already holds the scene.
    bool scene_cached = false;
    for (rt_context* c : g_cache) scene_cached = scene_cached || (c && same_spheres(c->scene, spheres, n));
    SceneData pre;
    double prep_ms = 0;
    bool prep_ok = false;  // the host thread finished (an exception there leaves it false)
    std::thread prep;
    bool pre_ready = false;
    // The training rule is per device launch (render_rows): the first device's rows.  With n_gpus = 0
    // (every visible device) the device count is known only once the HIP runtime is up, so the
    // thread builds the records and the SAH tree first and then waits for it (device_gpus below; 0:
    // the call failed before, no training).
    std::promise<int> gpus_promise;
    std::shared_future<int> gpus = gpus_promise.get_future().share();
    bool gpus_set = false;
    auto device_gpus = [&](int g) {
        if (!gpus_set) {
            gpus_set = true;
            gpus_promise.set_value(g);
        }
    };
    {
        const uint32_t H0 = cam->image_height;
        const int G_opt = opts && opts->n_gpus > 0 ? std::min<int>(opts->n_gpus, (int)H0) : 0;
        auto job = [&pre, &prep_ms, &prep_ok, spheres, n, cam, H0, G_opt, gpus]() {
            try {  // an exception must not leave the thread (std::terminate): the scene is rebuilt inline
                const auto t0 = std::chrono::steady_clock::now();
                build_scene(spheres, n, pre);
                if (needs_far_rebuild(pre, *cam)) build_bvh(pre, far_bound(pre, *cam));
                const int G0 = G_opt > 0 ? G_opt : std::min<int>(gpus.get(), (int)H0);
                if (G0 > 0) {
                    const uint64_t samples =
                        (uint64_t)((H0 + (uint32_t)G0 - 1) / (uint32_t)G0) * cam->image_width * cam->samples_per_pixel;
                    if (needs_training(pre, *cam, samples)) train_bvh(pre, *cam);
                }
                prep_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                prep_ok = true;
            } catch (...) {
            }
        };
        if (!scene_cached) {
            try {
                prep = std::thread(job);
            } catch (const std::exception&) {  // no thread to be had: the scene is built inline below
            }
        }
    }
    // joins the host thread (or builds the scene inline) the first time the scene is needed
    auto scene = [&]() -> const SceneData& {
        if (!pre_ready) {
            if (prep.joinable()) {
                prep.join();
                trace_note("host_scene_and_tree_thread", prep_ms);
            }
            if (!prep_ok) {  // no thread, or it failed: the records here, the tree in render_rows
                pre = SceneData{};
                build_scene(spheres, n, pre);
            }
            pre_ready = true;
        }
        return pre;
    };
    struct Joiner {  // every return path releases (no device count: no training) and joins the host thread
        std::thread& t;
        std::function<void(int)> release;
        ~Joiner() {
            release(0);
            if (t.joinable()) t.join();
        }
    } joiner{prep, device_gpus};
    std::vector<int> map;
    rc = device_map(map);  // the process's first HIP call initialises the runtime
    if (rc) return rc;
    trace_mark("hip_init_device_map");
    const int count = (int)map.size();
    const int first = o.device;
    int G = o.n_gpus > 0 ? o.n_gpus : count - first;
    if (first < 0 || first + G > count || G <= 0) {
        rt_set_last_error("requested devices not available");
        return RT_ERR_NO_DEVICE;
    }
    const uint32_t W = cam->image_width, H = cam->image_height;
    G = std::min<int>(G, (int)H);
    device_gpus(G);  // the host thread's training rule: the first device's ceil(H / G) rows
    const size_t px_bytes = o.output_format == RT_OUT_LINEAR_F64 ? 3 * sizeof(double) : 3;

    std::vector<rt_context*> ctxs;
    rc = cached_contexts(map, first, G, spheres, n, scene, ctxs);
    if (rc) return rc;
    if (tracing())
        for (rt_context* c : ctxs) (void)rt_context_enable_timing(c, 1);
    std::vector<uint32_t> rows(G);
    for (int g = 0; g < G; g++) {
        rt_context* c = ctxs[g];
        HIP_CHECK(hipSetDevice(c->device));
        rc = rt_context_set_precision(c, (int)o.precision);
        rows[g] = (H - (uint32_t)g + (uint32_t)G - 1) / (uint32_t)G;
        const size_t bytes = (size_t)rows[g] * W * px_bytes;
        if (!rc) rc = ensure_buffer(c, &c->d_out, &c->d_out_bytes, bytes);
        if (!rc && !c->d_stats) {
            size_t sb = 0;
            rc = ensure_buffer(c, (void**)&c->d_stats, &sb, 2 * sizeof(uint64_t));
        }
        if (rc) return rc;
        if (c->h_out_bytes < bytes) {
            if (c->h_out) (void)hipHostFree(c->h_out);
            c->h_out = nullptr;
            c->h_out_bytes = 0;
            HIP_CHECK(hipHostMalloc(&c->h_out, bytes, hipHostMallocDefault));
            c->h_out_bytes = bytes;
        }
        if (!c->h_stats) HIP_CHECK(hipHostMalloc((void**)&c->h_stats, 3 * sizeof(uint64_t), hipHostMallocDefault));
        trace_mark("output_staging_alloc");
        HIP_CHECK(hipMemsetAsync(c->d_stats, 0, 2 * sizeof(uint64_t), c->stream));
        rc = rt_render_rows_async(c, cam, o.output_format, (uint32_t)g, (uint32_t)G, rows[g], c->d_out, c->d_stats,
                                  c->stream);
        if (rc) return rc;
        HIP_CHECK(hipMemcpyAsync(c->h_out, c->d_out, bytes, hipMemcpyDeviceToHost, c->stream));
        HIP_CHECK(hipMemcpyAsync(c->h_stats, c->d_stats, 2 * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
        HIP_CHECK(hipMemcpyAsync(c->h_stats + 2, c->d_ctr + rtk::kErrWord, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
        trace_mark("copies_issue");
    }
    // Wait for each device and un-interleave its rows j = g + k*G into the caller's framebuffer, one
    // host thread per device (at 8 GPUs the 23 MB host copy would otherwise rival the render).
    std::vector<int> rcs(G, RT_OK);
    std::vector<std::string> msgs(G);
    std::vector<uint64_t> st_rays(G, 0), st_samples(G, 0);
    auto collect = [&](int g) {
        rt_context* c = ctxs[g];
        hipError_t e = hipSetDevice(c->device);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        trace_mark("device_wait_kernel_and_d2h");
        if (e != hipSuccess) {
            rcs[g] = hip_fail(e, "rt_render: device work");
            msgs[g] = rt_last_error();  // thread-local: carried back to the caller's thread
            return;
        }
        if (c->h_stats[2]) {
            // reported: clear the sticky word (on the context's stream, see rt_context_sync)
            e = hipMemsetAsync(c->d_ctr + rtk::kErrWord, 0, sizeof(uint64_t), c->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
            rcs[g] = RT_ERR_HIP;
            msgs[g] = err_message(c->h_stats[2]);
            return;
        }
        st_rays[g] = c->h_stats[0];
        st_samples[g] = c->h_stats[1];
        const uint8_t* src8 = (const uint8_t*)c->h_out;
        for (uint32_t k = 0; k < rows[g]; k++) {
            const uint32_t j = (uint32_t)g + k * (uint32_t)G;
            if (o.output_format == RT_OUT_RGB8) {
                std::memcpy((uint8_t*)out + (size_t)j * W * 3, src8 + (size_t)k * W * 3, (size_t)W * 3);
            } else {
                const double* src = (const double*)c->h_out + (size_t)k * W * 3;
                double* dst = (double*)out + (size_t)j * W * stride;
                if (stride == 3) {
                    std::memcpy(dst, src, (size_t)W * 3 * sizeof(double));
                } else {
                    for (uint32_t i = 0; i < W; i++)
                        for (int ch = 0; ch < 3; ch++) dst[(size_t)i * stride + ch] = src[3 * (size_t)i + ch];
                }
            }
        }
    };
    if (G == 1) {
        collect(0);
        trace_mark("uninterleave_to_caller");
    } else {
        std::vector<std::thread> th;
        for (int g = 0; g < G; g++) th.emplace_back(collect, g);
        for (auto& t : th) t.join();
        trace_mark("device_wait_and_uninterleave_threads");
    }
    if (tracing())
        for (rt_context* c : ctxs) {
            double k = 0;
            if (rt_context_kernel_times(c, &k, nullptr) == RT_OK) trace.kernel_ms.push_back(k);
            (void)rt_context_enable_timing(c, 0);
        }
    uint64_t stats[2] = {0, 0};
    for (int g = 0; g < G; g++) {
        if (rcs[g]) {
            rt_set_last_error(msgs[g]);
            return rcs[g];
        }
        stats[0] += st_rays[g];
        stats[1] += st_samples[g];
    }
    if (o.stats_out) {
        o.stats_out[0] = stats[0];
        o.stats_out[1] = stats[1];
    }
    return RT_OK;
}

int rt_release_cached_contexts(void) {
    std::lock_guard<std::mutex> lock(g_cache_mu);
    for (rt_context*& c : g_cache) {
        rt_context_destroy(c);
        c = nullptr;
    }
    g_cache.clear();
    return RT_OK;
}

}  // extern "C"

/*
 * rt.h — C ABI of the MI355X path tracer (drop-in for the reference's Camera.render()).
 *
 * The reference (AndrewJarrett/raytracing-with-zig, Zig 0.14) has no FFI of its own.  The cut is
 * `Camera.render(self: Camera) !void` (src/camera.zig:123-145), called from src/main.zig:35.  A Zig
 * shim marshals the Camera fields (camera.zig:82-103), the Hittable list
 * (hittable.zig:43-44, Sphere sphere.zig:13-16, Material material.zig:126-143) and the scene
 * interval/seed (Scene.zig:19-21) into the plain structs below and calls rt_render(), then keeps
 * its own PPM.saveBinary (ppm.zig:42-60, camera.zig:144).
 *
 * Everything is plain C: pointers + sizes, no torch / HIP types in the signatures (device pointers
 * and streams are passed as void*).  All functions return 0 on success and a negative rt_status on
 * failure; rt_last_error() returns a thread-local message for the last failure.
 *
 * Arithmetic contract: IEEE f64, no FMA contraction, correctly-rounded sqrt/div, in the exact
 * operation order of the reference.  The only deviation from the reference is the
 * RNG stream layout: the reference draws every random number from ONE sequential Xoshiro256++
 * stream (Scene.zig:29-38), which cannot be parallelised; here every (pixel, sample) owns its own
 * Xoshiro256++ stream (same generator, same Random.float(f64) conversion) keyed by
 * rt_sample_key(seed, pixel, sample).  See DESIGN.md "RNG".
 */
#ifndef RT_MI355X_H
#define RT_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 3
/* uint64 words of the d_stats buffer of an instrumented render (rt_context_enable_profile) */
#define RT_PROFILE_STATS_WORDS 72

/* ---- status codes ---------------------------------------------------------------------------- */
typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID = -1,   /* bad argument (n==0, W/H/spp==0, bad material, non-finite camera...) */
    RT_ERR_HIP = -2,       /* HIP runtime error (message in rt_last_error) */
    RT_ERR_NO_DEVICE = -3, /* no gfx950 device visible / extension not built for it */
    RT_ERR_CAPACITY = -4,  /* too large: > 2^24 spheres, or a launch with >= 2^32 work units */
    RT_ERR_IO = -5         /* file I/O (PPM writer) */
} rt_status;

/* ---- materials: tag of the reference's `Material` union (material.zig:113-117) ---------------- */
typedef enum rt_material_kind {
    RT_LAMBERTIAN = 0, /* Lambertian.scatter  material.zig:27-39 */
    RT_METAL = 1,      /* Metal.scatter       material.zig:55-68 */
    RT_DIELECTRIC = 2  /* Dielectric.scatter  material.zig:82-103 */
} rt_material_kind;

/* One Hittable (only `.sphere` exists, hittable.zig:22-27).  Replaces Sphere{center, radius, mat}
 * (sphere.zig:13-16).  The Material's `*DefaultPrng` pointer does not cross the boundary.
 * `radius` is stored as given; like Sphere.init (sphere.zig:21) the library clamps it to >= 0. */
typedef struct rt_sphere {
    double center[3];
    double radius;
    uint32_t material;        /* rt_material_kind */
    uint32_t reserved;        /* must be 0 */
    double albedo[3];         /* Lambertian/Metal albedo (material.zig:17,43) */
    double fuzz;              /* Metal.fuzz (material.zig:45) */
    double refraction_index;  /* Dielectric.refractionIndex (material.zig:72) */
} rt_sphere;                  /* 80 bytes */

/* The built Camera (camera.zig:82-103 after CameraBuilder.build camera.zig:300-345) plus the scene
 * fields render() reads (Scene.interval Scene.zig:21, Scene.seed Scene.zig:19). */
typedef struct rt_camera {
    uint32_t image_width;        /* Image.width  (camera.zig:27) */
    uint32_t image_height;       /* Image.height (camera.zig:28), already trunc(W/ratio), >= 1 */
    uint32_t samples_per_pixel;  /* Camera.samplesPerPixel (camera.zig:88) */
    uint32_t bounce_max;         /* Camera.bounceMax (camera.zig:90) */
    double pixel_samples_scale;  /* Camera.pixelSamplesScale = 1.0/spp (camera.zig:89,284) */
    double center[3];            /* Camera.center */
    double pixel0[3];            /* Camera.pixel0 */
    double du[3];                /* Camera.du */
    double dv[3];                /* Camera.dv */
    double defocus_disk_u[3];    /* Camera.defocusDiskU */
    double defocus_disk_v[3];    /* Camera.defocusDiskV */
    double defocus_angle;        /* Camera.defocusAngle (degrees; <= 0 disables the disk) */
    double t_min;                /* Scene.interval.min (1e-3) */
    double t_max;                /* Scene.interval.max (+inf) */
    uint64_t seed;               /* Scene.seed (the shim draws one from scene.prng when null) */
} rt_camera;

/* Options for one render call. */
typedef enum rt_output_format {
    RT_OUT_LINEAR_F64 = 0, /* ppm.pixels: linear Color per pixel (camera.zig:137-138) */
    RT_OUT_RGB8 = 1        /* fused Color.toRgb (color.zig:63-80): 3 bytes per pixel */
} rt_output_format;

/* Arithmetic of the sampling kernel. */
typedef enum rt_precision {
    RT_PRECISION_F64 = 0,  /* parity: the reference's f64 arithmetic bit for bit (default) */
    RT_PRECISION_F32 = 1   /* fast: f32 shading / sampling / intersection (huge spheres in f64);
                              statistical parity only (DESIGN.md "Fast mode") */
} rt_precision;

typedef struct rt_options {
    int32_t n_gpus;        /* 0 => all visible devices; rows are interleaved j mod n_gpus */
    int32_t device;        /* first device ordinal used */
    uint32_t pixel_stride; /* LINEAR_F64 only: doubles between pixels; 0 => 3. Zig's
                              @Vector(3,f64) has stride 4 (32 bytes), so the shim passes 4 */
    uint32_t output_format;/* rt_output_format */
    uint32_t precision;    /* rt_precision (0 = parity) */
    uint32_t reserved;     /* must be 0 */
    uint64_t* stats_out;   /* optional: [0] = rays traced (world.hit calls), [1] = samples */
} rt_options;

/* ---- the drop-in: Camera.render() ------------------------------------------------------------ */
/* Renders the whole image into host memory `out` (row-major, j*W+i).  LINEAR_F64: W*H pixels of
 * `pixel_stride` doubles (first 3 are r,g,b); RGB8: W*H*3 bytes.  Blocks the calling thread.
 * The library keeps one device context per GPU for the life of the process (created on first use,
 * on parallel host threads): a later call on the same sphere list re-uploads and rebuilds nothing.
 * Calls are serialised by an internal lock.
 *
 * Workspace (per device, held by the cached context; rt_context_workspace_bytes reports it).  A
 * context holds the buffers of ONE of two modes at a time (switching frees the other's):
 *   ring mode (launches whose samples need more than 2 GiB, e.g. config 4's full 1200x800x500
 *   frame on one GPU): one 144-KiB ring per resident wave of the launched kernel (the BVH kernels
 *   run 16 waves per CU: 576 MiB on a 256-CU MI355X) + 24 B of running sum per pixel + 4 B of flag
 *   per 64 pixels — config 4: 576 MiB + 22 MiB;
 *   direct mode (smaller launches: a rank's rows of a multi-GPU job, the 400x225 book scenes): every
 *   sample's colour, P x spp x 24 B (at most 2 GiB; a rank's 100 rows of config 4 at N = 8:
 *   1.34 GiB), summed in order by a second pass.
 * A buffer more than 25% larger than the current launch needs is given back and reallocated.
 * Plus the framebuffer rows (W x rows x 24 B) and the scene (≈ 100 KB for 485 spheres). */
int rt_render(const rt_camera* cam, const rt_sphere* spheres, size_t n_spheres,
              const rt_options* opts, void* out);
/* Frees rt_render's cached device contexts (optional; the next rt_render creates them again). */
int rt_release_cached_contexts(void);

/* ---- device-resident path (bench / multi-process drivers) ------------------------------------ */
typedef struct rt_context rt_context;

int rt_context_create(int device, rt_context** out_ctx);
/* Runs a pending deferred reduce pass, waits for every launch and pass of the context, then frees
 * it.  Returns the flush's status (the context is freed either way). */
int rt_context_destroy(rt_context* ctx);
/* Uploads the Hittable list to the context's device (once per scene). */
int rt_context_set_scene(rt_context* ctx, const rt_sphere* spheres, size_t n_spheres);
/* Renders rows j = row0 + k*row_step, k in [0, n_rows), into DEVICE memory `d_out`
 * (n_rows*W pixels; LINEAR_F64 stride 3 doubles, or RGB8) on HIP stream `stream` (NULL = default).
 * Asynchronous: returns after the launches; the output is complete when `stream` reaches the point
 * of the call.  `d_stats` (device, 2 x uint64, may be NULL) is atomically incremented with
 * {rays, samples}.  One kernel launch per call.  A context is not re-entrant: calls on one context
 * must come from one host thread at a time; a call on a different stream than the previous one
 * waits for the previous call's work, and scene changes / buffer growth wait for it on the host.
 * A call of at least 2^25 samples on a scene of at least 32 spheres with a camera the context's
 * tree was not built for first rebuilds the BVH from sample rays of that camera (host work,
 * ≈16 ms for the final scene, memoised per process; it waits for the previous call on the host).
 * Any tree gives the same bits; this one only walks faster for that camera. */
int rt_render_rows_async(rt_context* ctx, const rt_camera* cam, uint32_t output_format,
                         uint32_t row0, uint32_t row_step, uint32_t n_rows,
                         void* d_out, void* d_stats, void* stream);
/* The same render with the output completed on a second stream `out_stream` instead of `stream`
 * (frame pipelining for multi-frame drivers, e.g. bench.py's N > 1 path, which gathers each frame
 * on its collective stream): the sample kernel runs on `stream`; `out_stream` waits for it, and a
 * direct-mode call (small launches: a rank's rows of a multi-GPU job) runs its reduce pass there.
 * The context then alternates two per-sample buffers, so the next call's sample kernel on `stream`
 * does not wait for this call's reduce pass — the pass (HBM-bound, ≈0.25 ms at rank 0 of 8 on
 * config 4) overlaps the next sample kernel.  The output, and `d_stats`, are complete when
 * `out_stream` reaches the point of the call.  Either stream may be NULL (the HIP null stream);
 * out_stream == stream: rt_render_rows_async.
 * Workspace: twice direct mode's per-sample buffer. */
int rt_render_rows_async_split(rt_context* ctx, const rt_camera* cam, uint32_t output_format,
                               uint32_t row0, uint32_t row_step, uint32_t n_rows,
                               void* d_out, void* d_stats, void* stream, void* out_stream);
/* Deferred variant for frame pipelines (bench.py's N > 1 loop): like the split call, but a
 * direct-mode call's reduce pass is left PENDING — the next deferred call's sample kernel folds it
 * (one wave per block starts on it before tracing; the waves that run out of items while a few long
 * paths finish take the rest) and completes it before the kernel ends; with profiling enabled the
 * instrumented kernel does not fold, and a pass on that call's out_stream runs it after the kernel.
 * So the output of call k is complete on ITS out_stream once call k+1 has been issued and its
 * out_stream reaches that point, or after rt_context_flush(ctx) / rt_context_sync(ctx), which run a
 * pending pass whole.  A call that cannot fold the pending pass (a plain or ring-mode call, another
 * launch size, or another out_stream than the pending call's) runs it first.  Ring-mode calls behave
 * as rt_render_rows_async_split.  out_stream (NULL: the HIP null stream) must differ from stream.
 * rt_context_destroy runs a pending pass and waits for it before freeing anything: the output of
 * the last deferred call is complete when destroy returns (RT_OK), never dropped. */
int rt_render_rows_async_deferred(rt_context* ctx, const rt_camera* cam, uint32_t output_format,
                                  uint32_t row0, uint32_t row_step, uint32_t n_rows,
                                  void* d_out, void* d_stats, void* stream, void* out_stream);
/* Runs a pending deferred reduce pass (on the out_stream of the call that deferred it); no-op otherwise. */
int rt_context_flush(rt_context* ctx);
/* *pending = 1 if the last deferred call left its output pending (direct mode), else 0. */
int rt_context_fold_pending(rt_context* ctx, int* pending);
/* Waits for the context's last render (running a pending deferred reduce pass first) and reports a
 * failure the kernel recorded (RT_ERR_HIP: a wave gave up waiting for a running-sum hand-off — a bug
 * guard, never expected). */
int rt_context_sync(rt_context* ctx);
/* Arithmetic of the context's later renders: rt_precision (default RT_PRECISION_F64).  F32 needs
 * the BVH walk (any scene whose BVH builds); otherwise the parity kernel runs. */
int rt_context_set_precision(rt_context* ctx, int precision);
/* Name of the kernel variant the context launches (for profiling / logs). */
const char* rt_kernel_name(rt_context* ctx);
/* The closest-hit structure the context's next render walks (diagnostics / tests), info[6]:
 * {1 if the BVH walk runs (else the reference's list walk), tree nodes, leaves, depth, always-list
 * spheres, 1 if the tree was trained on the rays of the last large launch's camera (DESIGN.md §5.4:
 * same bits as any tree, fewer node visits)}. */
int rt_context_tree_info(rt_context* ctx, uint32_t* info);
/* Device bytes the context's render workspace holds now (rings, sums, flags, direct-mode samples,
 * schedule, counters; not the scene or caller buffers): see rt_render "Workspace". */
int rt_context_workspace_bytes(rt_context* ctx, uint64_t* bytes);
/* Optional kernel timing with HIP events recorded on the launch stream around the kernels of every
 * render call.  rt_context_kernel_times waits for the last event and returns the durations (ms) of
 * the most recent rt_render_rows_async call: the sample kernel, and the reduce pass of direct mode
 * (small launches, see rt_render; ~0 when the sample kernel accumulated in order itself; for a split
 * call, from the point `out_stream` reaches the pass to its end). */
int rt_context_enable_timing(rt_context* ctx, int enable);
int rt_context_kernel_times(rt_context* ctx, double* sample_ms, double* reduce_ms);
/* The same summed over every call since timing was (re)enabled (at most 1024 calls; beyond that the
 * totals restart), so a caller can time many frames without a host sync per frame.
 * *n_launches = the number of sample-kernel launches summed. */
int rt_context_kernel_times_total(rt_context* ctx, double* sample_ms, double* reduce_ms, uint32_t* n_launches);
/* Instrumented kernels (diagnostics): when enabled, `d_stats` of rt_render_rows_async must hold
 * RT_PROFILE_STATS_WORDS (72) uint64: {rays, samples, sphere tests executed, BVH node visits, wave-cycles in queue refill,
 * wave-cycles in the closest-hit walk, wave-cycles in shading, wave-iterations of the BVH inner
 * (internal-node) loop, wave-iterations of BVH leaf rounds, wave-level candidate blocks (sqrt +
 * root division), wave-level second-root divisions, node visits of camera rays, sphere tests of
 * camera rays, [13..15] kernel timeline stamps, [16] wave-cycles in the rejection-trip loop,
 * [17] idle sleeps of waves waiting on a hand-off, [18] deferred unit finalisations (previous chunk
 * of the tile not yet finalised), [19] refills that found no free ring slot, [20] / [21] sum / max over
 * waves of (wave end - the wave's first empty claim), [22] the last wave's first empty claim, [23..25]
 * the parts of [4]: wave-cycles finalising units, handing out items (claims), seeding + getRay;
 * [26..31] wave-level executions: loop iterations, rejection trips, seeding blocks, walks started
 * (always-list tests), shading blocks, unit finalisations; then lane-level executions (the active
 * lanes summed over every wave-level execution of a block) and the wave-level executions they pair
 * with: [32] seeding lanes, [33] rejection-trip lanes, [34] / [35] scatter-finish waves / lanes,
 * [36] / [37] defocus camera-finish waves / lanes, [38] / [39] walk waves / lanes (resumed walks
 * included), [40] walk-start lanes, [41] shading lanes, [42..47] waves / lanes of the sky, Lambertian
 * + metal and dielectric shading branches, [48] / [49] store waves / lanes, [50] lanes holding a path
 * after the hand-out (per iteration), [51] leaf-round lanes, [52] candidate-block lanes, [53]
 * second-root lanes, [54..57] / [58..61] always-list candidate blocks per always-list slot 0..3, waves
 * / lanes, [62] / [63] always-list second-root waves / lanes, [64] / [65] seed-window fills / take
 * passes (RTZIG_SEED_WIN builds), [66..71] unused}.  Counts 0-3 are exact and
 * deterministic; the cycles, wave-level and lane-level counts are diagnostics. */
int rt_context_enable_profile(rt_context* ctx, int enable);

/* ---- host mirror of the reference's Scene / CameraBuilder / Color / PPM ---------------------- */
/* Scene.generateWorld (Scene.zig:48-134) driven by DefaultPrng.init(seed) (Scene.zig:30).
 * Writes up to `cap` spheres, stores the count in *n (485 for seed 0xdeadbeef).  If `prng_state`
 * is non-NULL it receives the 4 Xoshiro256++ words after generation (the reference's render()
 * continues that stream). */
int rt_scene_final(uint64_t seed, rt_sphere* out, size_t cap, size_t* n, uint64_t* prng_state);
/* Scene.generateChapter13 (Scene.zig:136-182): 5 spheres, no RNG. */
int rt_scene_chapter13(rt_sphere* out, size_t cap, size_t* n);

/* CameraBuilder inputs (camera.zig:233-251).  rt_camera_build applies them in the order main.zig
 * uses (setDefocusAngle, setFocusDist, setViewport, setSamplesPerPixel, setBounceMax): the viewport
 * is computed from focus_dist (camera.zig:277) and everything else as in build() (:300-345). */
typedef struct rt_camera_params {
    uint32_t image_width;
    uint32_t samples_per_pixel;
    uint32_t bounce_max;
    uint32_t reserved;
    double aspect_ratio;
    double look_from[3];
    double look_at[3];
    double v_up[3];
    double vfov;           /* degrees */
    double defocus_angle;  /* degrees */
    double focus_dist;
    double t_min, t_max;
    uint64_t seed;
} rt_camera_params;

int rt_camera_build(const rt_camera_params* params, rt_camera* out);
/* Color.toRgb (color.zig:63-76) for n linear pixels with the given stride (doubles). */
int rt_color_to_rgb8(const double* linear, size_t n_pixels, uint32_t pixel_stride, uint8_t* rgb);
/* PPM.saveBinary byte stream (ppm.zig:42-60): "P6\nW H\n255\n" + W*H*3 bytes + "\n".
 * rt_ppm_p6_size gives the byte count; rt_ppm_encode_p6 writes it into `buf`. */
size_t rt_ppm_p6_size(uint32_t width, uint32_t height);
int rt_ppm_encode_p6(const uint8_t* rgb, uint32_t width, uint32_t height, uint8_t* buf, size_t cap);
int rt_ppm_save_p6(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height);
/* PPM.save ASCII byte stream (ppm.zig:25-39, Color.format color.zig:82-87 -> RGB.format :13-18):
 * "P3\nW H\n255\n" then one "r g b\n" line per pixel, decimal, no padding.
 * rt_ppm_p3_size gives the exact byte count for these pixels; rt_ppm_encode_p3 writes the stream
 * into `buf` (cap >= that size). */
size_t rt_ppm_p3_size(const uint8_t* rgb, uint32_t width, uint32_t height);
int rt_ppm_encode_p3(const uint8_t* rgb, uint32_t width, uint32_t height, uint8_t* buf, size_t cap);
int rt_ppm_save_p3(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height);

/* Per-(pixel, sample) stream key (DESIGN.md "RNG"); exposed so host tools can reproduce it. */
uint64_t rt_sample_key(uint64_t seed, uint64_t pixel, uint64_t sample);

const char* rt_last_error(void);
int rt_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* RT_MI355X_H */

/*
 * rt_render_c.c — plain-C driver of the rt.h ABI, mirroring what the Zig shim in INTEGRATION.md
 * marshals from Camera.render (reference src/camera.zig:123-145) and what main() sets up
 * (src/main.zig:14-36): Scene.init(seed) + generateWorld, the main.zig camera preset, render, and
 * PPM.saveBinary.  One image per process, as the reference renders.
 *
 *   rt_render_c <out.ppm> [width=400] [spp=10] [seed=0xdeadbeef] [aspect=1.7777777777777777]
 *               [scene=final|ch13|ch9]
 *
 * scene: final = generateWorld + main.zig:24-31 (configs 4/5); ch13 = generateChapter13
 * (Scene.zig:136-182) with the book's chapter-13 camera (config 3); ch9 = the two Lambertian
 * spheres of config 2.
 *
 * With RTZIG_TRACE=1 it prints one JSON line of CLOCK_MONOTONIC stamps (seconds) at main entry and
 * after each step, so a driver that records the same clock around the process (tools/dropin_cold.py)
 * can split the one-shot wall time into exec + library load, scene, camera, rt_render (whose own
 * phases the library prints to stderr), the P6 write and the exit.
 */
#define _POSIX_C_SOURCE 199309L
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "rt.h"

static double mono(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char** argv) {
    const double t_main = mono();
    if (argc < 2) {
        fprintf(stderr, "usage: %s out.ppm [width] [spp] [seed] [aspect] [final|ch13|ch9]\n", argv[0]);
        return 2;
    }
    const uint32_t width = argc > 2 ? (uint32_t)strtoul(argv[2], NULL, 0) : 400;
    const uint32_t spp = argc > 3 ? (uint32_t)strtoul(argv[3], NULL, 0) : 10;
    const uint64_t seed = argc > 4 ? strtoull(argv[4], NULL, 0) : 0xdeadbeefULL;
    const double aspect = argc > 5 ? strtod(argv[5], NULL) : 16.0 / 9.0;
    const char* scene = argc > 6 ? argv[6] : "final";

    rt_camera_params p;
    memset(&p, 0, sizeof p);
    p.image_width = width;
    p.samples_per_pixel = spp;
    p.bounce_max = 50;
    p.aspect_ratio = aspect;
    p.v_up[1] = 1;
    p.t_min = 1e-3;
    p.t_max = INFINITY;
    p.seed = seed;

    size_t n = 0;
    rt_sphere* spheres = NULL;
    if (strcmp(scene, "final") == 0) {
        /* Scene.init(seed) + generateWorld() (Scene.zig:23-134) */
        if (rt_scene_final(seed, NULL, 0, &n, NULL) != 0) return 1;
        spheres = calloc(n, sizeof *spheres);
        if (rt_scene_final(seed, spheres, n, &n, NULL) != 0) {
            fprintf(stderr, "rt_scene_final: %s\n", rt_last_error());
            return 1;
        }
        /* main.zig:24-31 camera preset */
        p.look_from[0] = 13; p.look_from[1] = 2; p.look_from[2] = 3;
        p.vfov = 20;
        p.defocus_angle = 0.6;
        p.focus_dist = 10;
    } else if (strcmp(scene, "ch13") == 0) {
        /* Scene.generateChapter13 (Scene.zig:136-182) + the book's chapter-13 camera */
        spheres = calloc(8, sizeof *spheres);
        if (rt_scene_chapter13(spheres, 8, &n) != 0) {
            fprintf(stderr, "rt_scene_chapter13: %s\n", rt_last_error());
            return 1;
        }
        p.look_from[0] = -2; p.look_from[1] = 2; p.look_from[2] = 1;
        p.look_at[2] = -1;
        p.vfov = 20;
        p.defocus_angle = 10;
        p.focus_dist = 3.4;
    } else if (strcmp(scene, "ch9") == 0) {
        /* two Lambertian spheres, albedo 0.5 (config 2) */
        n = 2;
        spheres = calloc(n, sizeof *spheres);
        const double cy[2] = {0, -100.5}, r[2] = {0.5, 100};
        for (int k = 0; k < 2; k++) {
            spheres[k].center[1] = cy[k];
            spheres[k].center[2] = -1;
            spheres[k].radius = r[k];
            spheres[k].material = RT_LAMBERTIAN;
            spheres[k].albedo[0] = spheres[k].albedo[1] = spheres[k].albedo[2] = 0.5;
        }
        p.look_at[2] = -1;
        p.vfov = 90;
        p.defocus_angle = 0;
        p.focus_dist = 1;
    } else {
        fprintf(stderr, "unknown scene %s\n", scene);
        return 2;
    }
    const double t_scene = mono();

    /* CameraBuilder.build (camera.zig:300-345) */
    rt_camera cam;
    if (rt_camera_build(&p, &cam) != 0) {
        fprintf(stderr, "rt_camera_build: %s\n", rt_last_error());
        return 1;
    }
    const double t_camera = mono();

    /* Camera.render(): fused toRgb output, then PPM.saveBinary (ppm.zig:42-60) */
    const size_t npx = (size_t)cam.image_width * cam.image_height;
    uint8_t* rgb = malloc(npx * 3);
    uint64_t stats[2] = {0, 0};
    rt_options opts;
    memset(&opts, 0, sizeof opts);
    opts.n_gpus = 0;
    opts.output_format = RT_OUT_RGB8;
    opts.stats_out = stats;
    if (rt_render(&cam, spheres, n, &opts, rgb) != 0) {
        fprintf(stderr, "rt_render: %s\n", rt_last_error());
        return 1;
    }
    const double t_render = mono();
    if (rt_ppm_save_p6(argv[1], rgb, cam.image_width, cam.image_height) != 0) {
        fprintf(stderr, "rt_ppm_save_p6: %s\n", rt_last_error());
        return 1;
    }
    const double t_saved = mono();
    printf("%ux%u %u spp, %zu spheres, %llu rays -> %s\n", cam.image_width, cam.image_height, spp, n,
           (unsigned long long)stats[0], argv[1]);
    const char* tr = getenv("RTZIG_TRACE");
    if (tr && *tr && strcmp(tr, "0") != 0)
        printf("{\"harness_stamps\": {\"main\": %.6f, \"scene\": %.6f, \"camera\": %.6f, \"render\": %.6f, "
               "\"saved\": %.6f}, \"rays\": %llu}\n",
               t_main, t_scene, t_camera, t_render, t_saved, (unsigned long long)stats[0]);
    fflush(stdout);
    free(rgb);
    free(spheres);
    return 0;
}

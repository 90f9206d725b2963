/*
 * rt_render_c.c — plain-C driver of the rt.h ABI, mirroring what the Zig shim in INTEGRATION.md
 * marshals from Camera.render (reference src/camera.zig:123-145) and what main() sets up
 * (src/main.zig:14-36): Scene.init(seed) + generateWorld, the main.zig camera preset, render, and
 * PPM.saveBinary.
 *
 *   rt_render_c <out.ppm> [width=400] [spp=10] [seed=0xdeadbeef] [aspect=1.7777777777777777]
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rt.h"

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s out.ppm [width] [spp] [seed] [aspect]\n", argv[0]);
        return 2;
    }
    const uint32_t width = argc > 2 ? (uint32_t)strtoul(argv[2], NULL, 0) : 400;
    const uint32_t spp = argc > 3 ? (uint32_t)strtoul(argv[3], NULL, 0) : 10;
    const uint64_t seed = argc > 4 ? strtoull(argv[4], NULL, 0) : 0xdeadbeefULL;
    const double aspect = argc > 5 ? strtod(argv[5], NULL) : 16.0 / 9.0;

    /* Scene.init(seed) + generateWorld() (Scene.zig:23-134) */
    size_t n = 0;
    if (rt_scene_final(seed, NULL, 0, &n, NULL) != 0) return 1;
    rt_sphere* spheres = calloc(n, sizeof *spheres);
    if (rt_scene_final(seed, spheres, n, &n, NULL) != 0) {
        fprintf(stderr, "rt_scene_final: %s\n", rt_last_error());
        return 1;
    }

    /* main.zig:24-31 camera preset -> CameraBuilder.build (camera.zig:300-345) */
    rt_camera_params p;
    memset(&p, 0, sizeof p);
    p.image_width = width;
    p.samples_per_pixel = spp;
    p.bounce_max = 50;
    p.aspect_ratio = aspect;
    p.look_from[0] = 13; p.look_from[1] = 2; p.look_from[2] = 3;
    p.v_up[1] = 1;
    p.vfov = 20;
    p.defocus_angle = 0.6;
    p.focus_dist = 10;
    p.t_min = 1e-3;
    p.t_max = INFINITY;
    p.seed = seed;
    rt_camera cam;
    if (rt_camera_build(&p, &cam) != 0) {
        fprintf(stderr, "rt_camera_build: %s\n", rt_last_error());
        return 1;
    }

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
    if (rt_ppm_save_p6(argv[1], rgb, cam.image_width, cam.image_height) != 0) {
        fprintf(stderr, "rt_ppm_save_p6: %s\n", rt_last_error());
        return 1;
    }
    printf("%ux%u %u spp, %zu spheres, %llu rays -> %s\n", cam.image_width, cam.image_height, spp, n,
           (unsigned long long)stats[0], argv[1]);
    free(rgb);
    free(spheres);
    return 0;
}

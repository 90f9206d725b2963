/*
 * rt_oracle.c — CPU ORACLE. TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity checker for the MI355X path tracer.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it (as liboracle.so); the product library
 * (raytracing-with-zig_amd/csrc) never links or calls it.
 *
 * It is a plain-C restatement of the reference's hot path (AndrewJarrett/raytracing-with-zig,
 * /root/reference, Zig 0.14 — the Zig toolchain is absent here, so the reference itself cannot be
 * built: see DESIGN.md "Oracle").  Every function cites the reference file:line it follows.
 * Compiled with -ffp-contract=off so every f64 operation rounds exactly where the Zig code does
 * (Zig's default float mode is strict: no contraction, ordered @reduce(.Add)).
 *
 * Two render modes:
 *   A  (oracle_render_a)  the reference's single sequential Xoshiro256++ stream shared by the
 *      scene generator and the camera (Scene.zig:29-38).  PINNED: reproduces
 *      test-files/chapter14.ppm byte-for-byte (tests/test_oracle.py).
 *   B  (oracle_render_b)  identical arithmetic, but every (pixel, sample) draws from its own
 *      Xoshiro256++ stream keyed by rt_sample_key() — the GPU's RNG layout.  The GPU must match
 *      B bit-for-bit.
 *
 * Third-party algorithm restated (not under /root/reference): Zig 0.14 std.Random —
 * DefaultPrng = Xoshiro256++ (std/Random/Xoshiro256.zig), seeded by SplitMix64
 * (std/Random/SplitMix64.zig), Random.float(f64) (std/Random.zig), std.math.pow(f64,x,5)
 * (std/math/pow.zig, frexp/repeated squaring), std.math.degreesToRadians (std/math.zig).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rt.h"

#define EXPORT __attribute__((visibility("default")))

/* ------------------------------------------------------------------------------------------------
 * Zig std RNG
 * ---------------------------------------------------------------------------------------------- */
typedef struct { uint64_t s[4]; } xoshiro;

static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

/* SplitMix64.next (zig std/Random/SplitMix64.zig) */
static inline uint64_t splitmix_next(uint64_t* s) {
    *s += 0x9e3779b97f4a7c15ULL;
    uint64_t z = *s;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

/* Xoshiro256.init/seed: 4 words from SplitMix64(seed) (zig std/Random/Xoshiro256.zig) */
static inline void xoshiro_seed(xoshiro* g, uint64_t seed) {
    uint64_t sm = seed;
    g->s[0] = splitmix_next(&sm);
    g->s[1] = splitmix_next(&sm);
    g->s[2] = splitmix_next(&sm);
    g->s[3] = splitmix_next(&sm);
}

/* Xoshiro256.next (++ scrambler) */
static inline uint64_t xoshiro_next(xoshiro* g) {
    uint64_t* s = g->s;
    const uint64_t r = rotl64(s[0] + s[3], 23) + s[0];
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl64(s[3], 45);
    return r;
}

static inline uint64_t clz64(uint64_t x) { return x ? (uint64_t)__builtin_clzll(x) : 64; }

/* Random.float(f64) (zig std/Random.zig): 52 mantissa bits from one draw, exponent from its
 * leading zeros; if >= 12 leading zeros, more draws extend the exponent (capped at 1022). */
static inline double zig_float64(xoshiro* g) {
    const uint64_t rnd = xoshiro_next(g);
    uint64_t lz = clz64(rnd);
    if (lz >= 12) {
        lz = 12;
        for (;;) {
            const uint64_t add = clz64(xoshiro_next(g));
            lz += add;
            if (add != 64) break;
            if (lz >= 1022) { lz = 1022; break; }
        }
    }
    const uint64_t bits = ((1022 - lz) << 52) | (rnd & ((1ULL << 52) - 1));
    double d;
    memcpy(&d, &bits, 8);
    return d;
}

/* util.randomDouble (util.zig:15-17) / randomDoubleRange (util.zig:20-22) */
static inline double rd(xoshiro* g) { return zig_float64(g); }
static inline double rdr(double mn, double mx, xoshiro* g) { return mn + (mx - mn) * rd(g); }

/* Per-(pixel, sample) stream key — the GPU's RNG layout (DESIGN.md "RNG").  Same definition as
 * rt_sample_key in the product; restated here independently. */
static inline uint64_t sm_mix(uint64_t x) { return splitmix_next(&x); }
EXPORT uint64_t oracle_sample_key(uint64_t seed, uint64_t pixel, uint64_t sample) {
    return sm_mix(sm_mix(seed) ^ ((pixel << 32) | (sample & 0xffffffffULL)));
}

/* ------------------------------------------------------------------------------------------------
 * Vec (vec.zig:9-136).  Vec3 = @Vector(3, f64); @reduce(.Add) is the ordered (x+y)+z.
 * ---------------------------------------------------------------------------------------------- */
typedef struct { double x, y, z; } v3;
static inline v3 V(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 neg(v3 a) { return V(-a.x, -a.y, -a.z); }
static inline v3 muls(v3 a, double s) { return V(a.x * s, a.y * s, a.z * s); }       /* vec.zig:35 */
static inline v3 divs(v3 a, double s) { return muls(a, 1.0 / s); }                 /* vec.zig:39-45 */
static inline double dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; } /* vec.zig:114 */
static inline double len_sq(v3 a) { return (a.x * a.x + a.y * a.y) + a.z * a.z; }   /* vec.zig:51 */
static inline double len(v3 a) { return sqrt(len_sq(a)); }                          /* vec.zig:47 */
static inline v3 unit(v3 a) { return divs(a, len(a)); }                             /* vec.zig:126 */
static inline v3 cross(v3 a, v3 b) {                                                /* vec.zig:118 */
    return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline int near_zero(v3 v) { return v.x < 1e-8 && v.y < 1e-8 && v.z < 1e-8; } /* vec.zig:26 (no abs) */
static inline v3 reflect(v3 v, v3 n) { return sub(v, muls(muls(n, dot(v, n)), 2)); } /* vec.zig:103 */
static inline v3 refract(v3 v, v3 n, double eta) {                                 /* vec.zig:107-112 */
    const double cos_t = fmin(dot(neg(v), n), 1.0);
    const v3 r_perp = muls(add(v, muls(n, cos_t)), eta);
    const v3 r_par = muls(n, -sqrt(fabs(1.0 - len_sq(r_perp))));
    return add(r_perp, r_par);
}
static inline v3 random_unit_vec(xoshiro* g) {                                     /* vec.zig:71-80 */
    for (;;) {
        const double x = rdr(-1, 1, g), y = rdr(-1, 1, g), z = rdr(-1, 1, g);
        const v3 p = V(x, y, z);
        const double ls = len_sq(p);
        if (1e-160 < ls && ls <= 1) {
            const double l = sqrt(ls);
            return V(p.x / l, p.y / l, p.z / l); /* true division, vec.zig:77 */
        }
    }
}
static inline v3 random_in_unit_disk(xoshiro* g) {                                 /* vec.zig:82-92 */
    for (;;) {
        const double x = rdr(-1, 1, g), y = rdr(-1, 1, g);
        const v3 p = V(x, y, 0);
        if (len_sq(p) < 1) return p;
    }
}

/* std.math.pow(f64, x, 5) for x in [0, 2]: frexp + repeated squaring == x*((x*x)*(x*x)) with the
 * same roundings (all intermediates normal); pow(+-0, odd) = x, pow(1, y) = 1. */
static inline double zig_pow5(double x) {
    if (x == 1.0) return 1.0;
    if (x == 0.0) return x;
    const double x2 = x * x;
    const double x4 = x2 * x2;
    return x * x4;
}

/* ------------------------------------------------------------------------------------------------
 * Scene (Scene.zig:48-182) — sphere list in rt_sphere layout
 * ---------------------------------------------------------------------------------------------- */
static void put_sphere(rt_sphere* out, size_t cap, size_t* n, v3 c, double r, uint32_t kind,
                       v3 albedo, double fuzz, double ior) {
    if (*n < cap) {
        rt_sphere* s = &out[*n];
        memset(s, 0, sizeof *s);
        s->center[0] = c.x; s->center[1] = c.y; s->center[2] = c.z;
        s->radius = r;
        s->material = kind;
        s->albedo[0] = albedo.x; s->albedo[1] = albedo.y; s->albedo[2] = albedo.z;
        s->fuzz = fuzz;
        s->refraction_index = ior;
    }
    (*n)++;
}

/* Scene.init(seed) + generateWorld (Scene.zig:23-46, 48-134) */
EXPORT int oracle_scene_final(uint64_t seed, rt_sphere* out, size_t cap, size_t* n_out,
                              uint64_t* state_out) {
    xoshiro g;
    xoshiro_seed(&g, seed);
    size_t n = 0;
    const v3 one = V(1, 1, 1);
    put_sphere(out, cap, &n, V(0, -1000, 0), 1000, RT_LAMBERTIAN, V(0.5, 0.5, 0.5), 0, 1.0);
    for (int a = 0; a < 22; a++) {
        const double xo = (double)a - 11;
        for (int b = 0; b < 22; b++) {
            const double zo = (double)b - 11;
            const double choose = rd(&g);
            const double cx = xo + 0.9 * rd(&g);
            const double cz = zo + 0.9 * rd(&g);
            const v3 center = V(cx, 0.2, cz);
            if (len(sub(center, V(4, 0.2, 0))) > 0.9) {
                if (choose < 0.8) {
                    /* Vec.random * Vec.random (Scene.zig:83): left operand drawn first */
                    const double a0 = rd(&g), a1 = rd(&g), a2 = rd(&g);
                    const double b0 = rd(&g), b1 = rd(&g), b2 = rd(&g);
                    put_sphere(out, cap, &n, center, 0.2, RT_LAMBERTIAN,
                               mul(V(a0, a1, a2), V(b0, b1, b2)), 0, 1.0);
                } else if (choose < 0.95) {
                    const double a0 = rdr(0.5, 1, &g), a1 = rdr(0.5, 1, &g), a2 = rdr(0.5, 1, &g);
                    const double fuzz = rdr(0, 0.5, &g);
                    put_sphere(out, cap, &n, center, 0.2, RT_METAL, V(a0, a1, a2), fuzz, 1.0);
                } else {
                    put_sphere(out, cap, &n, center, 0.2, RT_DIELECTRIC, one, 0, 1.5);
                }
            }
        }
    }
    put_sphere(out, cap, &n, V(0, 1, 0), 1, RT_DIELECTRIC, one, 0, 1.5);
    put_sphere(out, cap, &n, V(-4, 1, 0), 1, RT_LAMBERTIAN, V(0.4, 0.2, 0.1), 0, 1.0);
    put_sphere(out, cap, &n, V(4, 1, 0), 1, RT_METAL, V(0.7, 0.6, 0.5), 0, 1.0);
    *n_out = n;
    if (state_out) memcpy(state_out, g.s, sizeof g.s);
    return n <= cap ? 0 : RT_ERR_CAPACITY;
}

/* generateChapter13 (Scene.zig:136-182) */
EXPORT int oracle_scene_chapter13(rt_sphere* out, size_t cap, size_t* n_out) {
    size_t n = 0;
    const v3 one = V(1, 1, 1);
    put_sphere(out, cap, &n, V(0, -100.5, -1), 100, RT_LAMBERTIAN, V(0.8, 0.8, 0.0), 0, 1.0);
    put_sphere(out, cap, &n, V(0, 0, -1.2), 0.5, RT_LAMBERTIAN, V(0.1, 0.2, 0.5), 0, 1.0);
    put_sphere(out, cap, &n, V(-1, 0, -1), 0.5, RT_DIELECTRIC, one, 0, 1.5);
    put_sphere(out, cap, &n, V(-1, 0, -1), 0.4, RT_DIELECTRIC, one, 0, 1.0 / 1.5);
    put_sphere(out, cap, &n, V(1, 0, -1), 0.5, RT_METAL, V(0.8, 0.6, 0.2), 1, 1.0);
    *n_out = n;
    return n <= cap ? 0 : RT_ERR_CAPACITY;
}

/* ------------------------------------------------------------------------------------------------
 * Camera (camera.zig:33-72 Image/Viewport, :300-345 CameraBuilder.build)
 * ---------------------------------------------------------------------------------------------- */
static const double RAD_PER_DEG = 0.017453292519943295; /* std.math.rad_per_deg as f64 */

EXPORT int oracle_camera_build(const rt_camera_params* p, rt_camera* c) {
    memset(c, 0, sizeof *c);
    /* Image.init (camera.zig:33-40) */
    size_t h = (size_t)((double)p->image_width / p->aspect_ratio);
    if (h < 1) h = 1;
    const double W = (double)p->image_width, H = (double)h;
    /* Viewport.init (camera.zig:61-72), evaluated at setViewport time with focusDist */
    const double theta = p->vfov * RAD_PER_DEG;
    const double hh = tan(theta / 2.0);
    const double vp_h = 2 * hh * p->focus_dist;
    const double vp_w = vp_h * (W / H);
    /* build() (camera.zig:300-345) */
    const v3 look_from = V(p->look_from[0], p->look_from[1], p->look_from[2]);
    const v3 look_at = V(p->look_at[0], p->look_at[1], p->look_at[2]);
    const v3 vup = V(p->v_up[0], p->v_up[1], p->v_up[2]);
    const v3 center = look_from; /* setViewport: center = lookFrom (camera.zig:274) */
    const v3 w = unit(sub(look_from, look_at));
    const v3 u = unit(cross(vup, w));
    const v3 v = cross(w, u);
    const v3 vu = muls(u, vp_w);
    const v3 vv = muls(neg(v), vp_h);
    const v3 du = divs(vu, W);
    const v3 dv = divs(vv, H);
    const v3 ul = sub(sub(sub(center, muls(w, p->focus_dist)), divs(vu, 2)), divs(vv, 2));
    const v3 pixel0 = add(ul, muls(add(du, dv), 0.5));
    const double defocus_r = p->focus_dist * tan((p->defocus_angle / 2.0) * RAD_PER_DEG);
    const v3 ddu = muls(u, defocus_r), ddv = muls(v, defocus_r);

    c->image_width = p->image_width;
    c->image_height = (uint32_t)h;
    c->samples_per_pixel = p->samples_per_pixel;
    c->bounce_max = p->bounce_max;
    c->pixel_samples_scale = 1.0 / (double)p->samples_per_pixel; /* camera.zig:284 */
#define PUT3(dst, src) do { (dst)[0] = (src).x; (dst)[1] = (src).y; (dst)[2] = (src).z; } while (0)
    PUT3(c->center, center);
    PUT3(c->pixel0, pixel0);
    PUT3(c->du, du);
    PUT3(c->dv, dv);
    PUT3(c->defocus_disk_u, ddu);
    PUT3(c->defocus_disk_v, ddv);
#undef PUT3
    c->defocus_angle = p->defocus_angle;
    c->t_min = p->t_min;
    c->t_max = p->t_max;
    c->seed = p->seed;
    return 0;
}

/* ------------------------------------------------------------------------------------------------
 * Render (camera.zig:123-215, hittable.zig:64-77, sphere.zig:26-54, material.zig:27-110)
 * ---------------------------------------------------------------------------------------------- */
typedef struct { v3 orig, dir; } ray_t;
typedef struct {
    v3 c;
    double r, r2, inv_r;
    uint32_t kind;
    v3 albedo;
    double fuzz, ior;
} osphere;

static osphere* load_spheres(const rt_sphere* s, size_t n) {
    osphere* o = (osphere*)malloc(sizeof(osphere) * (n ? n : 1));
    for (size_t k = 0; k < n; k++) {
        const double r = s[k].radius > 0 ? s[k].radius : 0; /* Sphere.init @max(0, r) sphere.zig:21 */
        o[k].c = V(s[k].center[0], s[k].center[1], s[k].center[2]);
        o[k].r = r;
        o[k].r2 = r * r;
        o[k].inv_r = 1.0 / r;
        o[k].kind = s[k].material;
        o[k].albedo = V(s[k].albedo[0], s[k].albedo[1], s[k].albedo[2]);
        o[k].fuzz = s[k].fuzz;
        o[k].ior = s[k].refraction_index;
    }
    return o;
}

/* HittableList.hit (hittable.zig:64-77) over Sphere.hit (sphere.zig:26-42): returns the index of
 * the accepted sphere (or -1) and its root in *t_out. */
static inline long world_hit(const osphere* sp, size_t n, ray_t r, double t_min, double t_max,
                             double* t_out) {
    long best = -1;
    double closest = t_max;
    const double a = len_sq(r.dir);
    for (size_t k = 0; k < n; k++) {
        const v3 oc = sub(sp[k].c, r.orig);
        const double h = dot(r.dir, oc);
        const double c = len_sq(oc) - sp[k].r2;
        const double disc = h * h - a * c;
        if (disc < 0) continue;
        const double sq = sqrt(disc);
        double root = (h - sq) / a;
        if (!(t_min < root && root < closest)) {
            root = (h + sq) / a;
            if (!(t_min < root && root < closest)) continue;
        }
        closest = root;
        best = (long)k;
    }
    *t_out = closest;
    return best;
}

/* rayColor (camera.zig:148-183) with Material.scatter (material.zig:145-151) */
static v3 ray_color(const osphere* sp, size_t n, ray_t r, const rt_camera* cam, xoshiro* g,
                    uint64_t* rays) {
    v3 att = V(1, 1, 1);
    for (uint32_t b = 0; b < cam->bounce_max; b++) {
        double t;
        (*rays)++;
        const long k = world_hit(sp, n, r, cam->t_min, cam->t_max, &t);
        if (k >= 0) {
            const osphere* s = &sp[k];
            /* hit record (sphere.zig:44-53) */
            const v3 p = add(r.orig, muls(r.dir, t));
            const v3 outward = muls(sub(p, s->c), s->inv_r);
            const int front = dot(r.dir, outward) < 0;
            const v3 nrm = front ? outward : neg(outward);
            v3 dir;
            if (s->kind == RT_LAMBERTIAN) { /* material.zig:27-39 */
                dir = add(nrm, random_unit_vec(g));
                if (near_zero(dir)) dir = nrm;
                att = mul(att, s->albedo);
            } else if (s->kind == RT_METAL) { /* material.zig:55-68 */
                const v3 refl = unit(reflect(r.dir, nrm));
                dir = add(refl, muls(random_unit_vec(g), s->fuzz));
                if (!(dot(dir, nrm) > 0)) return V(0, 0, 0);
                att = mul(att, s->albedo);
            } else { /* dielectric, material.zig:82-103 */
                const double ri = front ? 1.0 / s->ior : s->ior;
                const v3 ud = unit(r.dir);
                const double cos_t = fmin(dot(neg(ud), nrm), 1.0);
                const double sin_t = sqrt(1.0 - cos_t * cos_t);
                const int cannot = ri * sin_t > 1.0;
                /* reflectance (material.zig:106-110), always evaluated */
                double r0 = (1 - ri) / (1 + ri);
                r0 *= r0;
                const double approx = r0 + (1 - r0) * zig_pow5(1 - cos_t);
                /* short-circuit `or`: the RNG is drawn only when refraction is possible */
                if (cannot || approx > rd(g)) dir = reflect(ud, nrm);
                else dir = refract(ud, nrm, ri);
                /* attenuation (1,1,1): att unchanged bit-for-bit */
            }
            r.orig = p;
            r.dir = dir;
            continue;
        }
        /* sky (camera.zig:171-177) */
        const double a = 0.5 * (unit(r.dir).y + 1.0);
        const v3 sky = add(muls(V(1, 1, 1), 1.0 - a), muls(V(0.5, 0.7, 1), a));
        return mul(att, sky);
    }
    return V(0, 0, 0);
}

/* getRay (camera.zig:187-215) */
static inline ray_t get_ray(const rt_camera* c, uint32_t i, uint32_t j, xoshiro* g) {
    const double ox = rd(g) - 0.5; /* sampleSquare camera.zig:203-209 */
    const double oy = rd(g) - 0.5;
    const v3 p0 = V(c->pixel0[0], c->pixel0[1], c->pixel0[2]);
    const v3 du = V(c->du[0], c->du[1], c->du[2]);
    const v3 dv = V(c->dv[0], c->dv[1], c->dv[2]);
    const v3 center = V(c->center[0], c->center[1], c->center[2]);
    const v3 ps = add(add(p0, muls(du, (double)i + ox)), muls(dv, (double)j + oy));
    v3 origin;
    if (c->defocus_angle <= 0) {
        origin = center;
    } else { /* defocusDiskSample camera.zig:212-215 */
        const v3 p = random_in_unit_disk(g);
        const v3 ddu = V(c->defocus_disk_u[0], c->defocus_disk_u[1], c->defocus_disk_u[2]);
        const v3 ddv = V(c->defocus_disk_v[0], c->defocus_disk_v[1], c->defocus_disk_v[2]);
        origin = add(add(center, muls(ddu, p.x)), muls(ddv, p.y));
    }
    ray_t r = {origin, sub(ps, origin)};
    return r;
}

/* Mode A: Camera.render (camera.zig:123-145) with the ONE sequential stream.  `prng_state` is the
 * Xoshiro state after Scene generation (NULL => DefaultPrng.init(cam->seed), i.e. a scene whose
 * generation drew nothing, like generateChapter13).  out: W*H*3 doubles. */
EXPORT int oracle_render_a(const rt_camera* cam, const rt_sphere* spheres, size_t n,
                           const uint64_t* prng_state, double* out, uint64_t* rays_out) {
    xoshiro g;
    if (prng_state) memcpy(g.s, prng_state, sizeof g.s);
    else xoshiro_seed(&g, cam->seed);
    osphere* sp = load_spheres(spheres, n);
    uint64_t rays = 0;
    for (uint32_t j = 0; j < cam->image_height; j++) {
        for (uint32_t i = 0; i < cam->image_width; i++) {
            v3 sum = V(0, 0, 0);
            for (uint32_t s = 0; s < cam->samples_per_pixel; s++) {
                const ray_t r = get_ray(cam, i, j, &g);
                sum = add(sum, ray_color(sp, n, r, cam, &g, &rays));
            }
            const v3 avg = muls(sum, cam->pixel_samples_scale);
            double* o = out + 3 * ((size_t)j * cam->image_width + i);
            o[0] = avg.x; o[1] = avg.y; o[2] = avg.z;
        }
    }
    free(sp);
    if (rays_out) *rays_out = rays;
    return 0;
}

/* Mode B: same arithmetic, stream per (pixel, sample) = Xoshiro256++ seeded by
 * SplitMix64(oracle_sample_key(seed, j*W+i, s)).  Renders rows row0 + k*row_step, k < n_rows into
 * out[k*W + i].  n_threads > 1 splits rows over OpenMP threads (results are independent of it). */
EXPORT int oracle_render_b(const rt_camera* cam, const rt_sphere* spheres, size_t n, uint32_t row0,
                           uint32_t row_step, uint32_t n_rows, double* out, uint64_t* rays_out,
                           int n_threads) {
    osphere* sp = load_spheres(spheres, n);
    const uint32_t W = cam->image_width;
    uint64_t rays = 0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : rays) num_threads(n_threads > 0 ? n_threads : 1)
    for (uint32_t k = 0; k < n_rows; k++) {
        const uint32_t j = row0 + k * row_step;
        for (uint32_t i = 0; i < W; i++) {
            const uint64_t pixel = (uint64_t)j * W + i;
            v3 sum = V(0, 0, 0);
            for (uint32_t s = 0; s < cam->samples_per_pixel; s++) {
                xoshiro g;
                xoshiro_seed(&g, oracle_sample_key(cam->seed, pixel, s));
                const ray_t r = get_ray(cam, i, j, &g);
                sum = add(sum, ray_color(sp, n, r, cam, &g, &rays));
            }
            const v3 avg = muls(sum, cam->pixel_samples_scale);
            double* o = out + 3 * ((size_t)k * W + i);
            o[0] = avg.x; o[1] = avg.y; o[2] = avg.z;
        }
    }
    free(sp);
    if (rays_out) *rays_out = rays;
    return 0;
}

/* ------------------------------------------------------------------------------------------------
 * Color.toRgb (color.zig:63-80) and PPM.saveBinary (ppm.zig:42-60)
 * ---------------------------------------------------------------------------------------------- */
static inline uint8_t to_byte(double lin) {
    double g = lin > 0 ? sqrt(lin) : 0;          /* linearToGamma */
    g = g < 0.0 ? 0.0 : (g > 0.999 ? 0.999 : g); /* Interval(0, 0.999).clamp (interval.zig:40-47) */
    return (uint8_t)(int)(256 * g);              /* @intFromFloat truncates */
}

EXPORT void oracle_to_rgb8(const double* lin, size_t n_pixels, uint8_t* rgb) {
    for (size_t p = 0; p < 3 * n_pixels; p++) rgb[p] = to_byte(lin[p]);
}

EXPORT size_t oracle_ppm_p6(const uint8_t* rgb, uint32_t w, uint32_t h, uint8_t* buf, size_t cap) {
    char hdr[64];
    const int hl = __builtin_snprintf(hdr, sizeof hdr, "P6\n%u %u\n255\n", w, h);
    const size_t total = (size_t)hl + (size_t)w * h * 3 + 1;
    if (buf && cap >= total) {
        memcpy(buf, hdr, (size_t)hl);
        memcpy(buf + hl, rgb, (size_t)w * h * 3);
        buf[total - 1] = '\n';
    }
    return total;
}

/* ------------------------------------------------------------------------------------------------
 * Known-answer helpers for tests (reference unit tests)
 * ---------------------------------------------------------------------------------------------- */
/* Sphere.hit for one sphere (sphere.zig:26-54): returns 1 on hit and fills t, point, normal, front */
EXPORT int oracle_sphere_hit(const rt_sphere* s, const double* orig, const double* dir, double t_min,
                             double t_max, double* t, double* point, double* normal, int* front) {
    osphere* sp = load_spheres(s, 1);
    ray_t r = {V(orig[0], orig[1], orig[2]), V(dir[0], dir[1], dir[2])};
    double tt;
    const long k = world_hit(sp, 1, r, t_min, t_max, &tt);
    if (k >= 0) {
        const v3 p = add(r.orig, muls(r.dir, tt));
        const v3 outward = muls(sub(p, sp->c), sp->inv_r);
        const int fr = dot(r.dir, outward) < 0;
        const v3 nn = fr ? outward : neg(outward);
        *t = tt;
        point[0] = p.x; point[1] = p.y; point[2] = p.z;
        normal[0] = nn.x; normal[1] = nn.y; normal[2] = nn.z;
        *front = fr;
    }
    free(sp);
    return k >= 0;
}

/* HittableList.hit over n spheres: index of the accepted sphere or -1 */
EXPORT long oracle_world_hit(const rt_sphere* s, size_t n, const double* orig, const double* dir,
                             double t_min, double t_max, double* t) {
    osphere* sp = load_spheres(s, n);
    ray_t r = {V(orig[0], orig[1], orig[2]), V(dir[0], dir[1], dir[2])};
    const long k = world_hit(sp, n, r, t_min, t_max, t);
    free(sp);
    return k;
}

/* First `count` Random.float(f64) draws of DefaultPrng.init(seed) */
EXPORT void oracle_random_doubles(uint64_t seed, size_t count, double* out) {
    xoshiro g;
    xoshiro_seed(&g, seed);
    for (size_t k = 0; k < count; k++) out[k] = rd(&g);
}

/* Raw Xoshiro256++ words of DefaultPrng.init(seed) */
EXPORT void oracle_random_u64(uint64_t seed, size_t count, uint64_t* out) {
    xoshiro g;
    xoshiro_seed(&g, seed);
    for (size_t k = 0; k < count; k++) out[k] = xoshiro_next(&g);
}

/* Vec.refract / Vec.reflect KATs (vec.zig:103-112) */
EXPORT void oracle_reflect(const double* v, const double* n, double* out) {
    const v3 r = reflect(V(v[0], v[1], v[2]), V(n[0], n[1], n[2]));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
EXPORT void oracle_refract(const double* v, const double* n, double eta, double* out) {
    const v3 r = refract(V(v[0], v[1], v[2]), V(n[0], n[1], n[2]), eta);
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* ------------------------------------------------------------------------------------------------
 * BASELINE config 1: "chapter5 single-sphere, 400x225, 1 spp" — the book's chapter 4/5 renderer
 * that produced test-files/chapter4.ppm / chapter5.ppm (earlier book-chapter code, no longer in
 * src/; restated from the fixtures' own pixels): focal length 1, viewport height 2, camera at the
 * origin, one centered ray per pixel (no RNG), sky lerp (camera.zig:171-177); chapter 5 adds a
 * red sphere (0,0,-1) r 0.5 hit when disc >= 0 (sphere.zig:27-33 without the root test); colors
 * quantised as trunc(255.999 * c) with no gamma.  Byte-exact vs both fixtures (tests/test_oracle.py).
 * ---------------------------------------------------------------------------------------------- */
/* Chapters 6/7 (test-files/chapter6.ppm, chapter7.ppm — BASELINE config 1's "normals" variant):
 * the same camera, world = sphere (0,0,-1) r 0.5 + ground (0,-100.5,-1) r 100 walked like
 * HittableList.hit (hittable.zig:64-77) over Sphere.hit (sphere.zig:26-54) on the interval
 * (0, inf); a hit shades 0.5 * (normal + (1,1,1)) with the face-forward normal (sphere.zig:45-53).
 * Chapter 6 quantises trunc(255.999 * c); chapter 7 trunc(256 * clamp(c, 0, 0.999))
 * (Interval.clamp interval.zig:40-47, as Color.toRgb color.zig:63-76 without the gamma). */
static int book_hit(v3 o, v3 d, double t_min, v3* nrm) {
    static const double cs[2][4] = {{0, 0, -1, 0.5}, {0, -100.5, -1, 100}};
    double closest = INFINITY;
    int found = 0;
    for (int k = 0; k < 2; k++) {
        const v3 c = V(cs[k][0], cs[k][1], cs[k][2]);
        const double r = cs[k][3];
        const v3 oc = sub(c, o);
        const double a = len_sq(d), h = dot(d, oc), cc = len_sq(oc) - r * r;
        const double disc = h * h - a * cc;
        if (disc < 0) continue;
        const double sq = sqrt(disc);
        double root = (h - sq) / a;
        if (!(t_min < root && root < closest)) {
            root = (h + sq) / a;
            if (!(t_min < root && root < closest)) continue;
        }
        closest = root;
        const v3 p = add(o, muls(d, root));
        const v3 out = divs(sub(p, c), r);
        *nrm = dot(d, out) < 0 ? out : neg(out);
        found = 1;
    }
    return found;
}

static v3 book_color(int chapter, v3 center, v3 d) {
    if (chapter == 5) {
        const v3 oc = sub(V(0, 0, -1), center);
        const double a = len_sq(d), hh = dot(d, oc), c = len_sq(oc) - 0.5 * 0.5;
        if (hh * hh - a * c >= 0) return V(1, 0, 0);
    }
    v3 nrm;
    if ((chapter == 6 || chapter == 7) && book_hit(center, d, 0.0, &nrm)) return muls(add(nrm, V(1, 1, 1)), 0.5);
    const double a = 0.5 * (unit(d).y + 1.0);
    return add(muls(V(1, 1, 1), 1.0 - a), muls(V(0.5, 0.7, 1), a));
}

/* Chapter 7 is the chapter-6 scene antialiased (the book's camera class): `spp` jittered samples
 * per pixel (sampleSquare camera.zig:203-209), averaged, quantised trunc(256 * clamp(c, 0, 0.999)).
 * Its RNG stream is unknown (the fixture predates src/), so it is compared statistically; the
 * jitter here draws from DefaultPrng.init(1). */
EXPORT int oracle_render_book(int chapter, uint32_t width, double ratio, uint8_t* rgb, uint32_t* height_out) {
    size_t h = (size_t)((double)width / ratio);
    if (h < 1) h = 1;
    const double W = (double)width, H = (double)h;
    const double vp_h = 2.0, vp_w = vp_h * (W / H);
    const v3 center = V(0, 0, 0);
    const v3 vu = V(vp_w, 0, 0), vv = V(0, -vp_h, 0);
    const v3 du = divs(vu, W), dv = divs(vv, H);
    const v3 ul = sub(sub(sub(center, V(0, 0, 1.0)), divs(vu, 2)), divs(vv, 2));
    const v3 p00 = add(ul, muls(add(du, dv), 0.5));
    const int spp = chapter == 7 ? 100 : 1;
    xoshiro g;
    xoshiro_seed(&g, 1);
    for (size_t j = 0; j < h; j++) {
        for (uint32_t i = 0; i < width; i++) {
            v3 col;
            if (spp == 1) {
                const v3 pc = add(add(p00, muls(du, (double)i)), muls(dv, (double)j));
                col = book_color(chapter, center, sub(pc, center));
            } else {
                col = V(0, 0, 0);
                for (int s = 0; s < spp; s++) {
                    const double ox = rd(&g) - 0.5, oy = rd(&g) - 0.5;
                    const v3 pc = add(add(p00, muls(du, (double)i + ox)), muls(dv, (double)j + oy));
                    col = add(col, book_color(chapter, center, sub(pc, center)));
                }
                col = muls(col, 1.0 / spp);
            }
            uint8_t* o = rgb + 3 * (j * width + i);
            if (chapter == 7) {
                const double cl[3] = {col.x, col.y, col.z};
                for (int k = 0; k < 3; k++) {
                    const double x = cl[k] < 0.0 ? 0.0 : (cl[k] > 0.999 ? 0.999 : cl[k]);
                    o[k] = (uint8_t)(int)(256.0 * x);
                }
            } else {
                o[0] = (uint8_t)(int)(255.999 * col.x);
                o[1] = (uint8_t)(int)(255.999 * col.y);
                o[2] = (uint8_t)(int)(255.999 * col.z);
            }
        }
    }
    if (height_out) *height_out = (uint32_t)h;
    return 0;
}

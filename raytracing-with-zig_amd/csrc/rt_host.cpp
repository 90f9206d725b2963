// rt_host.cpp — host mirror of Scene / CameraBuilder / Color / PPM (see rt_host.hpp) and the
// host-only C ABI entry points of include/rt.h.  Compiled with -ffp-contract=off: the camera
// constants and the scene's sphere list must carry exactly the reference's bits.
#include "rt_host.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <random>

#pragma STDC FP_CONTRACT OFF

namespace rtzig {

namespace {

inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

inline uint64_t splitmix_next(uint64_t& s) {  // SplitMix64.next (zig std)
    s += 0x9e3779b97f4a7c15ULL;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

inline uint64_t clz64(uint64_t x) { return x ? (uint64_t)__builtin_clzll(x) : 64; }

// Vec helpers with the reference's rounding order (vec.zig)
inline Vec3 add(Vec3 a, Vec3 b) { return {a[0] + b[0], a[1] + b[1], a[2] + b[2]}; }
inline Vec3 sub(Vec3 a, Vec3 b) { return {a[0] - b[0], a[1] - b[1], a[2] - b[2]}; }
inline Vec3 mul(Vec3 a, Vec3 b) { return {a[0] * b[0], a[1] * b[1], a[2] * b[2]}; }
inline Vec3 neg(Vec3 a) { return {-a[0], -a[1], -a[2]}; }
inline Vec3 muls(Vec3 a, double s) { return {a[0] * s, a[1] * s, a[2] * s}; }
inline Vec3 divs(Vec3 a, double s) { return muls(a, 1.0 / s); }
inline double lenSq(Vec3 a) { return (a[0] * a[0] + a[1] * a[1]) + a[2] * a[2]; }
inline double len(Vec3 a) { return std::sqrt(lenSq(a)); }
inline Vec3 unit(Vec3 a) { return divs(a, len(a)); }
inline Vec3 cross(Vec3 a, Vec3 b) {
    return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
}

constexpr double kRadPerDeg = 0.017453292519943295;  // std.math.rad_per_deg as f64

rt_sphere make_sphere(Vec3 c, double r, uint32_t kind, Vec3 albedo, double fuzz, double ior) {
    rt_sphere s;
    std::memset(&s, 0, sizeof s);
    for (int k = 0; k < 3; k++) s.center[k] = c[k];
    s.radius = r > 0 ? r : 0;  // Sphere.init: @max(0, radius) (sphere.zig:21)
    s.material = kind;
    for (int k = 0; k < 3; k++) s.albedo[k] = albedo[k];
    s.fuzz = fuzz;
    s.refraction_index = ior;
    return s;
}

}  // namespace

// ---- DefaultPrng --------------------------------------------------------------------------------
DefaultPrng::DefaultPrng(uint64_t seed) {
    uint64_t sm = seed;
    for (auto& w : s_) w = splitmix_next(sm);
}

uint64_t DefaultPrng::next() {
    const uint64_t r = rotl64(s_[0] + s_[3], 23) + s_[0];
    const uint64_t t = s_[1] << 17;
    s_[2] ^= s_[0];
    s_[3] ^= s_[1];
    s_[1] ^= s_[2];
    s_[0] ^= s_[3];
    s_[2] ^= t;
    s_[3] = rotl64(s_[3], 45);
    return r;
}

double DefaultPrng::randomDouble() {  // Random.float(f64)
    const uint64_t rnd = next();
    uint64_t lz = clz64(rnd);
    if (lz >= 12) {
        lz = 12;
        for (;;) {
            const uint64_t more = clz64(next());
            lz += more;
            if (more != 64) break;
            if (lz >= 1022) { lz = 1022; break; }
        }
    }
    const uint64_t bits = ((1022 - lz) << 52) | (rnd & ((1ULL << 52) - 1));
    double d;
    std::memcpy(&d, &bits, 8);
    return d;
}

double DefaultPrng::randomDoubleRange(double mn, double mx) { return mn + (mx - mn) * randomDouble(); }

// ---- Scene --------------------------------------------------------------------------------------
Scene Scene::init(std::optional<uint64_t> seed) {
    Scene s;
    s.seed = seed;
    if (seed) {
        s.effective_seed = *seed;
    } else {
        std::random_device rd;  // std.posix.getrandom stand-in
        s.effective_seed = ((uint64_t)rd() << 32) ^ rd();
    }
    s.prng = DefaultPrng(s.effective_seed);
    return s;
}

rt_sphere make_lambertian(Vec3 c, double r, Vec3 albedo) { return make_sphere(c, r, RT_LAMBERTIAN, albedo, 0, 1.0); }
rt_sphere make_metal(Vec3 c, double r, Vec3 albedo, double fuzz) { return make_sphere(c, r, RT_METAL, albedo, fuzz, 1.0); }
rt_sphere make_dielectric(Vec3 c, double r, double ior) { return make_sphere(c, r, RT_DIELECTRIC, {1, 1, 1}, 0, ior); }

void Scene::generateWorld() {
    add(make_lambertian({0, -1000, 0}, 1000, {0.5, 0.5, 0.5}));
    for (int a = 0; a < 22; a++) {
        const double xOffset = (double)a - 11;
        for (int b = 0; b < 22; b++) {
            const double zOffset = (double)b - 11;
            const double chooseMat = prng.randomDouble();
            const double cx = xOffset + 0.9 * prng.randomDouble();
            const double cz = zOffset + 0.9 * prng.randomDouble();
            const Vec3 center{cx, 0.2, cz};
            if (len(sub(center, Vec3{4, 0.2, 0})) > 0.9) {
                if (chooseMat < 0.8) {
                    Vec3 r1, r2;  // Vec.random(prng) * Vec.random(prng): left operand first
                    for (auto& x : r1) x = prng.randomDouble();
                    for (auto& x : r2) x = prng.randomDouble();
                    add(make_lambertian(center, 0.2, mul(r1, r2)));
                } else if (chooseMat < 0.95) {
                    Vec3 albedo;
                    for (auto& x : albedo) x = prng.randomDoubleRange(0.5, 1);
                    const double fuzz = prng.randomDoubleRange(0, 0.5);
                    add(make_metal(center, 0.2, albedo, fuzz));
                } else {
                    add(make_dielectric(center, 0.2, 1.5));
                }
            }
        }
    }
    add(make_dielectric({0, 1, 0}, 1, 1.5));
    add(make_lambertian({-4, 1, 0}, 1, {0.4, 0.2, 0.1}));
    add(make_metal({4, 1, 0}, 1, {0.7, 0.6, 0.5}, 0));
}

void Scene::generateChapter13() {
    add(make_lambertian({0, -100.5, -1}, 100, {0.8, 0.8, 0.0}));
    add(make_lambertian({0, 0, -1.2}, 0.5, {0.1, 0.2, 0.5}));
    add(make_dielectric({-1, 0, -1}, 0.5, 1.5));
    add(make_dielectric({-1, 0, -1}, 0.4, 1.0 / 1.5));
    add(make_metal({1, 0, -1}, 0.5, {0.8, 0.6, 0.2}, 1));
}

// ---- Image / Viewport / CameraBuilder -------------------------------------------------------------
Image Image::init(uint32_t width, double ratio) {
    Image img;
    img.width = width;
    const double h = (double)width / ratio;
    uint64_t hi = h >= 1 ? (uint64_t)h : 0;  // @intFromFloat truncates
    img.height = hi < 1 ? 1 : (uint32_t)hi;
    return img;
}

Viewport Viewport::init(const Image& img, double vFov, double focusDist) {
    Viewport vp;
    const double theta = vFov * kRadPerDeg;  // std.math.degreesToRadians
    const double h = std::tan(theta / 2.0);
    vp.height = 2 * h * focusDist;
    vp.width = vp.height * ((double)img.width / (double)img.height);
    vp.vFov = vFov;
    return vp;
}

CameraBuilder::CameraBuilder(uint32_t width, double aspectRatio) : image_(Image::init(width, aspectRatio)) {}
CameraBuilder& CameraBuilder::setScene(const Scene& scene) { scene_ = scene; return *this; }
CameraBuilder& CameraBuilder::setFocusDist(double f) { focusDist_ = f; return *this; }
CameraBuilder& CameraBuilder::setDefocusAngle(double a) { defocusAngle_ = a; return *this; }
CameraBuilder& CameraBuilder::setViewport(Vec3 lookFrom, Vec3 lookAt, double vFov) {
    center_ = lookFrom;
    lookFrom_ = lookFrom;
    lookAt_ = lookAt;
    viewport_ = Viewport::init(image_, vFov, focusDist_);  // uses focusDist at this point (camera.zig:277)
    return *this;
}
CameraBuilder& CameraBuilder::setSamplesPerPixel(uint32_t spp) {
    spp_ = spp;
    pixelSamplesScale_ = 1.0 / (double)spp;
    return *this;
}
CameraBuilder& CameraBuilder::setBounceMax(uint32_t b) { bounceMax_ = b; return *this; }
CameraBuilder& CameraBuilder::setVUp(Vec3 v) { vUp_ = v; return *this; }

Camera CameraBuilder::build() {  // camera.zig:300-345
    Camera c;
    c.scene = scene_ ? *scene_ : Scene::init(std::nullopt);
    if (!viewport_) viewport_ = Viewport::init(image_, 90, focusDist_);  // reference would panic on .?
    const Vec3 w = unit(sub(lookFrom_, lookAt_));
    const Vec3 u = unit(cross(vUp_, w));
    const Vec3 v = cross(w, u);
    const Vec3 vu = muls(u, viewport_->width);
    const Vec3 vv = muls(neg(v), viewport_->height);
    const Vec3 du = divs(vu, (double)image_.width);
    const Vec3 dv = divs(vv, (double)image_.height);
    const Vec3 ul = sub(sub(sub(center_, muls(w, focusDist_)), divs(vu, 2)), divs(vv, 2));
    const Vec3 pixel0 = add(ul, muls(add(du, dv), 0.5));
    const double defocusRadius = focusDist_ * std::tan((defocusAngle_ / 2.0) * kRadPerDeg);
    const Vec3 ddu = muls(u, defocusRadius), ddv = muls(v, defocusRadius);

    c.image = image_;
    c.viewport = *viewport_;
    c.u = u;
    c.v = v;
    c.w = w;
    rt_camera& k = c.cam;
    std::memset(&k, 0, sizeof k);
    k.image_width = image_.width;
    k.image_height = image_.height;
    k.samples_per_pixel = spp_;
    k.bounce_max = bounceMax_;
    k.pixel_samples_scale = pixelSamplesScale_;
    for (int i = 0; i < 3; i++) {
        k.center[i] = center_[i];
        k.pixel0[i] = pixel0[i];
        k.du[i] = du[i];
        k.dv[i] = dv[i];
        k.defocus_disk_u[i] = ddu[i];
        k.defocus_disk_v[i] = ddv[i];
    }
    k.defocus_angle = defocusAngle_;
    k.t_min = c.scene.interval.min;
    k.t_max = c.scene.interval.max;
    k.seed = c.scene.effective_seed;
    return c;
}

int Camera::render(PPM* out, const rt_options* opts) const {
    out->width = cam.image_width;
    out->height = cam.image_height;
    out->pixels.assign((size_t)cam.image_width * cam.image_height * 3, 0.0);
    rt_options o{};
    if (opts) o = *opts;
    o.output_format = RT_OUT_LINEAR_F64;
    o.pixel_stride = 3;
    return rt_render(&cam, scene.world.data(), scene.world.size(), &o, out->pixels.data());
}

// ---- Color / PPM ----------------------------------------------------------------------------------
static inline uint8_t to_byte(double lin) {  // Color.toRgb channel (color.zig:63-80)
    double g = lin > 0 ? std::sqrt(lin) : 0.0;
    g = g < 0.0 ? 0.0 : (g > 0.999 ? 0.999 : g);
    return (uint8_t)(int)(256.0 * g);
}

std::vector<uint8_t> PPM::toRgb() const {
    std::vector<uint8_t> rgb(pixels.size());
    for (size_t k = 0; k < pixels.size(); k++) rgb[k] = to_byte(pixels[k]);
    return rgb;
}

std::vector<uint8_t> PPM::encodeBinary() const {
    const auto rgb = toRgb();
    std::vector<uint8_t> buf(rt_ppm_p6_size(width, height));
    rt_ppm_encode_p6(rgb.data(), width, height, buf.data(), buf.size());
    return buf;
}

int PPM::saveBinary(const std::string& path) const {
    const auto rgb = toRgb();
    return rt_ppm_save_p6(path.c_str(), rgb.data(), width, height);
}

int PPM::save(const std::string& path) const {
    const auto rgb = toRgb();
    return rt_ppm_save_p3(path.c_str(), rgb.data(), width, height);
}

}  // namespace rtzig

// =================================================================================================
// C ABI: host-only entry points
// =================================================================================================
namespace {
thread_local std::string g_last_error;
}

void rt_set_last_error(const std::string& msg) { g_last_error = msg; }

extern "C" {

const char* rt_last_error(void) { return g_last_error.c_str(); }
int rt_abi_version(void) { return RT_ABI_VERSION; }

uint64_t rt_sample_key(uint64_t seed, uint64_t pixel, uint64_t sample) {
    uint64_t a = seed;
    const uint64_t m = rtzig::splitmix_next(a);
    uint64_t b = m ^ ((pixel << 32) | (sample & 0xffffffffULL));
    return rtzig::splitmix_next(b);
}

int rt_scene_final(uint64_t seed, rt_sphere* out, size_t cap, size_t* n, uint64_t* prng_state) {
    auto scene = rtzig::Scene::init(seed);
    scene.generateWorld();
    if (n) *n = scene.world.size();
    if (prng_state) {
        const auto st = scene.prng.state();
        for (int k = 0; k < 4; k++) prng_state[k] = st[k];
    }
    if (out) {
        const size_t m = scene.world.size() < cap ? scene.world.size() : cap;
        std::memcpy(out, scene.world.data(), m * sizeof(rt_sphere));
    }
    if (out && cap < scene.world.size()) {
        rt_set_last_error("rt_scene_final: capacity too small");
        return RT_ERR_CAPACITY;
    }
    return RT_OK;
}

int rt_scene_chapter13(rt_sphere* out, size_t cap, size_t* n) {
    auto scene = rtzig::Scene::init(0);
    scene.generateChapter13();
    if (n) *n = scene.world.size();
    if (out) {
        const size_t m = scene.world.size() < cap ? scene.world.size() : cap;
        std::memcpy(out, scene.world.data(), m * sizeof(rt_sphere));
    }
    if (out && cap < scene.world.size()) {
        rt_set_last_error("rt_scene_chapter13: capacity too small");
        return RT_ERR_CAPACITY;
    }
    return RT_OK;
}

int rt_camera_build(const rt_camera_params* p, rt_camera* out) {
    if (!p || !out) { rt_set_last_error("rt_camera_build: null argument"); return RT_ERR_INVALID; }
    if (p->image_width == 0 || p->samples_per_pixel == 0 || !(p->aspect_ratio > 0)) {
        rt_set_last_error("rt_camera_build: image_width, samples_per_pixel and aspect_ratio must be > 0");
        return RT_ERR_INVALID;
    }
    // main.zig:25-31 call order: setDefocusAngle, setFocusDist, setViewport, setSamplesPerPixel
    auto scene = rtzig::Scene::init(p->seed);
    scene.interval = {p->t_min, p->t_max};
    auto cam = rtzig::Camera::builder(p->image_width, p->aspect_ratio)
                   .setScene(scene)
                   .setDefocusAngle(p->defocus_angle)
                   .setFocusDist(p->focus_dist)
                   .setVUp({p->v_up[0], p->v_up[1], p->v_up[2]})
                   .setViewport({p->look_from[0], p->look_from[1], p->look_from[2]},
                                {p->look_at[0], p->look_at[1], p->look_at[2]}, p->vfov)
                   .setSamplesPerPixel(p->samples_per_pixel)
                   .setBounceMax(p->bounce_max)
                   .build();
    *out = cam.cam;
    return RT_OK;
}

int rt_color_to_rgb8(const double* linear, size_t n_pixels, uint32_t pixel_stride, uint8_t* rgb) {
    if (!linear || !rgb) { rt_set_last_error("rt_color_to_rgb8: null argument"); return RT_ERR_INVALID; }
    const uint32_t st = pixel_stride ? pixel_stride : 3;
    if (st < 3) { rt_set_last_error("rt_color_to_rgb8: pixel_stride < 3"); return RT_ERR_INVALID; }
    for (size_t p = 0; p < n_pixels; p++)
        for (int c = 0; c < 3; c++) rgb[3 * p + c] = rtzig::to_byte(linear[st * p + c]);
    return RT_OK;
}

size_t rt_ppm_p6_size(uint32_t width, uint32_t height) {
    char hdr[64];
    const int hl = std::snprintf(hdr, sizeof hdr, "P6\n%u %u\n255\n", width, height);
    return (size_t)hl + (size_t)width * height * 3 + 1;
}

int rt_ppm_encode_p6(const uint8_t* rgb, uint32_t width, uint32_t height, uint8_t* buf, size_t cap) {
    char hdr[64];
    const int hl = std::snprintf(hdr, sizeof hdr, "P6\n%u %u\n255\n", width, height);
    const size_t body = (size_t)width * height * 3;
    const size_t total = (size_t)hl + body + 1;
    if (!buf || cap < total || (!rgb && body)) {
        rt_set_last_error("rt_ppm_encode_p6: buffer too small or null");
        return RT_ERR_INVALID;
    }
    std::memcpy(buf, hdr, (size_t)hl);
    if (body) std::memcpy(buf + hl, rgb, body);
    buf[total - 1] = '\n';
    return RT_OK;
}

int rt_ppm_save_p6(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height) {
    std::vector<uint8_t> buf(rt_ppm_p6_size(width, height));
    int rc = rt_ppm_encode_p6(rgb, width, height, buf.data(), buf.size());
    if (rc) return rc;
    std::ofstream f(path, std::ios::binary);
    if (!f) { rt_set_last_error(std::string("rt_ppm_save_p6: cannot open ") + path); return RT_ERR_IO; }
    f.write((const char*)buf.data(), (std::streamsize)buf.size());
    if (!f) { rt_set_last_error(std::string("rt_ppm_save_p6: write failed ") + path); return RT_ERR_IO; }
    return RT_OK;
}

namespace {
// decimal digits of a byte value (RGB.format prints "{d}")
inline size_t dec_len(uint8_t v) { return v >= 100 ? 3 : (v >= 10 ? 2 : 1); }
inline uint8_t* put_dec(uint8_t* o, uint8_t v) {
    if (v >= 100) *o++ = (uint8_t)('0' + v / 100);
    if (v >= 10) *o++ = (uint8_t)('0' + v / 10 % 10);
    *o++ = (uint8_t)('0' + v % 10);
    return o;
}
}  // namespace

size_t rt_ppm_p3_size(const uint8_t* rgb, uint32_t width, uint32_t height) {
    char hdr[64];
    const int hl = std::snprintf(hdr, sizeof hdr, "P3\n%u %u\n255\n", width, height);
    const size_t n = (size_t)width * height;
    size_t total = (size_t)hl;
    if (!rgb) return n ? 0 : total;
    for (size_t k = 0; k < n; k++)  // "r g b\n"
        total += dec_len(rgb[3 * k]) + dec_len(rgb[3 * k + 1]) + dec_len(rgb[3 * k + 2]) + 3;
    return total;
}

int rt_ppm_encode_p3(const uint8_t* rgb, uint32_t width, uint32_t height, uint8_t* buf, size_t cap) {
    const size_t n = (size_t)width * height;
    if (!buf || (!rgb && n)) {
        rt_set_last_error("rt_ppm_encode_p3: null argument");
        return RT_ERR_INVALID;
    }
    const size_t total = rt_ppm_p3_size(rgb, width, height);
    if (cap < total) {
        rt_set_last_error("rt_ppm_encode_p3: buffer too small");
        return RT_ERR_INVALID;
    }
    char hdr[64];
    const int hl = std::snprintf(hdr, sizeof hdr, "P3\n%u %u\n255\n", width, height);
    std::memcpy(buf, hdr, (size_t)hl);
    uint8_t* o = buf + hl;
    for (size_t k = 0; k < n; k++) {
        o = put_dec(o, rgb[3 * k]);
        *o++ = ' ';
        o = put_dec(o, rgb[3 * k + 1]);
        *o++ = ' ';
        o = put_dec(o, rgb[3 * k + 2]);
        *o++ = '\n';
    }
    return RT_OK;
}

int rt_ppm_save_p3(const char* path, const uint8_t* rgb, uint32_t width, uint32_t height) {
    if (!path) { rt_set_last_error("rt_ppm_save_p3: null path"); return RT_ERR_INVALID; }
    if (!rgb && (size_t)width * height) { rt_set_last_error("rt_ppm_save_p3: null pixels"); return RT_ERR_INVALID; }
    std::vector<uint8_t> buf(rt_ppm_p3_size(rgb, width, height));
    int rc = rt_ppm_encode_p3(rgb, width, height, buf.data(), buf.size());
    if (rc) return rc;
    std::ofstream f(path, std::ios::binary);
    if (!f) { rt_set_last_error(std::string("rt_ppm_save_p3: cannot open ") + path); return RT_ERR_IO; }
    f.write((const char*)buf.data(), (std::streamsize)buf.size());
    if (!f) { rt_set_last_error(std::string("rt_ppm_save_p3: write failed ") + path); return RT_ERR_IO; }
    return RT_OK;
}

}  // extern "C"

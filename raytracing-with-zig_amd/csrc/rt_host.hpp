// rt_host.hpp — C++ host-side mirror of the reference's Scene / Camera / Material / PPM API.
//
// The reference's host API is Zig (Zig is not in this image), so the host side above the C ABI is
// C++ with the same names and the same argument meaning:
//   Scene::init(seed) / generateWorld() / generateChapter13()      Scene.zig:23-182
//   Camera::builder(width, aspect).setScene(..).setDefocusAngle(..).setFocusDist(..)
//         .setViewport(lookFrom, lookAt, vFov).setSamplesPerPixel(..).setBounceMax(..)
//         .setVUp(..).build()                                       camera.zig:109-345
//   Camera::render()  -> rt_render on the GPU, then PPM::saveBinary camera.zig:123-145
//   PPM::saveBinary(path)                                           ppm.zig:42-60
//   PPM::save(path)                                                 ppm.zig:25-39
// Only host code lives here: the hot path is the HIP kernel behind rt_render().
#pragma once

#include <array>
#include <cstdint>
#include <limits>
#include <optional>
#include <string>
#include <vector>

#include "../../include/rt.h"

namespace rtzig {

using Vec3 = std::array<double, 3>;

// std.Random.DefaultPrng (Xoshiro256++ seeded by SplitMix64) + Random.float(f64)
class DefaultPrng {
public:
    explicit DefaultPrng(uint64_t seed);
    uint64_t next();
    double randomDouble();                         // util.randomDouble (util.zig:15)
    double randomDoubleRange(double mn, double mx);  // util.zig:20
    std::array<uint64_t, 4> state() const { return {s_[0], s_[1], s_[2], s_[3]}; }

private:
    uint64_t s_[4];
};

struct Interval {  // interval.zig:6-48
    double min = std::numeric_limits<double>::infinity();
    double max = -std::numeric_limits<double>::infinity();
};

class Scene {  // Scene.zig:16-187
public:
    // seed == nullopt draws a seed from the OS like std.posix.getrandom (Scene.zig:33-37)
    static Scene init(std::optional<uint64_t> seed);
    void generateWorld();      // Scene.zig:48-134
    void generateChapter13();  // Scene.zig:136-182
    void add(const rt_sphere& s) { world.push_back(s); }

    std::vector<rt_sphere> world;
    std::optional<uint64_t> seed;
    uint64_t effective_seed = 0;  // the seed DefaultPrng was initialised with
    DefaultPrng prng{0};
    Interval interval{1e-3, std::numeric_limits<double>::infinity()};  // Scene.zig:21
};

rt_sphere make_lambertian(Vec3 center, double radius, Vec3 albedo);
rt_sphere make_metal(Vec3 center, double radius, Vec3 albedo, double fuzz);
rt_sphere make_dielectric(Vec3 center, double radius, double refraction_index);

struct Image {  // camera.zig:26-54
    uint32_t width = 100, height = 100;
    static Image init(uint32_t width, double ratio);
};

struct Viewport {  // camera.zig:56-80
    double width = 0, height = 0, vFov = 0;
    static Viewport init(const Image& img, double vFov, double focusDist);
};

class Camera;

class CameraBuilder {  // camera.zig:233-346
public:
    CameraBuilder(uint32_t width, double aspectRatio);
    CameraBuilder& setScene(const Scene& scene);
    CameraBuilder& setFocusDist(double focusDist);
    CameraBuilder& setDefocusAngle(double defocusAngle);
    CameraBuilder& setViewport(Vec3 lookFrom, Vec3 lookAt, double vFov);
    CameraBuilder& setSamplesPerPixel(uint32_t spp);
    CameraBuilder& setBounceMax(uint32_t bounceMax);
    CameraBuilder& setVUp(Vec3 vUp);
    Camera build();

private:
    Image image_;
    std::optional<Scene> scene_;
    uint32_t spp_ = 100, bounceMax_ = 50;
    Vec3 center_{0, 0, 0}, lookFrom_{0, 0, 0}, lookAt_{0, 0, -1}, vUp_{0, 1, 0};
    double defocusAngle_ = 0, focusDist_ = 10;
    std::optional<Viewport> viewport_;
    double pixelSamplesScale_ = 1.0 / 100.0;
};

struct PPM {  // ppm.zig:5-61
    uint32_t width = 0, height = 0;
    std::vector<double> pixels;  // linear colors, 3 doubles per pixel, j*W+i
    std::vector<uint8_t> toRgb() const;              // Color.toRgb per pixel (color.zig:63)
    std::vector<uint8_t> encodeBinary() const;       // saveBinary byte stream
    int saveBinary(const std::string& path) const;   // ppm.zig:42-60
    int save(const std::string& path) const;         // ppm.zig:25-39 (P3 ASCII)
};

class Camera {  // camera.zig:82-216
public:
    static CameraBuilder builder(uint32_t width, double aspectRatio) { return CameraBuilder(width, aspectRatio); }
    // Camera.render(): renders on the GPU(s) through rt_render and returns the framebuffer
    // (the reference writes it to images/<fileName>; use PPM::saveBinary for that).
    int render(PPM* out, const rt_options* opts = nullptr) const;

    Image image;
    Viewport viewport;
    Scene scene;
    rt_camera cam{};  // the flattened fields that cross the ABI
    Vec3 u{}, v{}, w{};
};

}  // namespace rtzig

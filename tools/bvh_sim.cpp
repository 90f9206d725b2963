// bvh_sim.cpp — CPU model of the BVH walk's cost for tree-build experiments (no GPU).
//
// Traces a sample of the final scene's paths (the reference's camera and scatter rules, any RNG:
// only the ray distribution matters here), records every ray segment, then replays the kernel's
// walk (always-list first, near-child-first traversal of the f32 boxes against [t_min, closest],
// kLeafMax-slot leaves) over the tree rtbvh::build produces, and reports
//   visits/ray   internal-node visits per ray (the kernel's instrumented `node_visits_per_ray`)
//   leaves/ray   leaf rounds per ray
//   wave steps   while-while inner steps per 64-ray wave: sum over segments k of the max over the
//                wave's lanes of the inner steps before the lane's k-th leaf (rays shuffled into
//                waves, as the persistent kernel mixes paths)
// Wave models (environment): SIM_LOCKSTEP (+ SIM_STEAL*: walk splitting across lanes),
// SIM_REFETCH=K (+ SIM_REFETCH_P): lanes that finish their walk take a new segment after each leaf
// round once K of them are done.
//
//   g++ -O2 -std=c++17 -pthread tools/bvh_sim.cpp raytracing-with-zig_amd/csrc/rt_bvh.cpp \
//       raytracing-with-zig_amd/csrc/rt_host.cpp -o /tmp/bvh_sim && /tmp/bvh_sim [stride] [spp] [train_stride (<0: surface rays)] [n_samples: rtbvh::sample_rays]
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../include/rt.h"
#include "../raytracing-with-zig_amd/csrc/rt_bvh.hpp"

// rt_host.cpp's Camera::render calls the GPU entry point; the simulator never does
extern "C" int rt_render(const rt_camera*, const rt_sphere*, size_t, const rt_options*, void*) { return -1; }

struct V {
    double x, y, z;
};
static V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V operator-(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V operator*(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
static double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V unit(V a) { return a * (1.0 / std::sqrt(dot(a, a))); }
static V mkv(const double* p) { return {p[0], p[1], p[2]}; }

static double hit_sphere(const rt_sphere& s, V o, V d, double tmin, double closest) {
    const V oc = mkv(s.center) - o;
    const double a = dot(d, d), h = dot(d, oc), c = dot(oc, oc) - s.radius * s.radius;
    const double disc = h * h - a * c;
    if (disc < 0) return INFINITY;
    const double sq = std::sqrt(disc);
    double r = (h - sq) / a;
    if (!(tmin < r && r < closest)) {
        r = (h + sq) / a;
        if (!(tmin < r && r < closest)) return INFINITY;
    }
    return r;
}

// candidate classes of a sphere test at the time the walk runs it (SIM_FAR): 0 no candidate block
// for this lane (miss, or both roots <= t_min: LeafFilter::behind), 1 a block whose root1 provably
// lies beyond the running closest (a far filter could drop it), 2 a live candidate
static int cand_class(const rt_sphere& s, V o, V d, double tmin, double closest) {
    const V oc = mkv(s.center) - o;
    const double a = dot(d, d), h = dot(d, oc), c = dot(oc, oc) - s.radius * s.radius;
    const double disc = h * h - a * c;
    if (disc < 0) return 0;
    const double sq = std::sqrt(disc);
    if ((h + sq) / a <= tmin) return 0;
    if ((h - sq) / a > closest) return 1;
    return 2;
}

struct Ray {
    V o, d;
    double t;  // closest hit (+inf: miss)
    bool camera = false;
};

int main(int argc, char** argv) {
    const int stride = argc > 1 ? std::atoi(argv[1]) : 4;
    const int spp = argc > 2 ? std::atoi(argv[2]) : 1;
    std::vector<rt_sphere> sp(600);
    size_t n = 0;
    rt_scene_final(0xDEADBEEF, sp.data(), sp.size(), &n, nullptr);
    sp.resize(n);
    for (auto& s : sp) s.radius = s.radius > 0 ? s.radius : 0;
    rt_camera_params p{};
    p.image_width = 1200; p.samples_per_pixel = spp; p.bounce_max = 50; p.aspect_ratio = 1.5;
    p.look_from[0] = 13; p.look_from[1] = 2; p.look_from[2] = 3;
    p.v_up[1] = 1; p.vfov = 20; p.defocus_angle = 0.6; p.focus_dist = 10; p.t_min = 1e-3; p.t_max = INFINITY;
    rt_camera cam;
    rt_camera_build(&p, &cam);

    // ---- trace a sample of paths, record every ray segment ----
    std::mt19937_64 rng(12345);
    auto trace = [&](uint64_t seed, int stride, int spp, std::vector<Ray>& rays) {
    rng.seed(seed);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    auto ruv = [&]() {
        while (true) {
            V q{2 * U(rng) - 1, 2 * U(rng) - 1, 2 * U(rng) - 1};
            const double l = dot(q, q);
            if (1e-160 < l && l <= 1) return q * (1.0 / std::sqrt(l));
        }
    };
    for (uint32_t j = 0; j < cam.image_height; j += stride)
        for (uint32_t i = 0; i < cam.image_width; i += stride)
            for (int s = 0; s < spp; s++) {
                const V ps = mkv(cam.pixel0) + mkv(cam.du) * (i + U(rng) - 0.5) + mkv(cam.dv) * (j + U(rng) - 0.5);
                double px, py;
                do { px = 2 * U(rng) - 1; py = 2 * U(rng) - 1; } while (px * px + py * py >= 1);
                V o = mkv(cam.center) + mkv(cam.defocus_disk_u) * px + mkv(cam.defocus_disk_v) * py;
                V d = ps - o;
                for (uint32_t b = 0; b < cam.bounce_max; b++) {
                    double best = INFINITY;
                    int k = -1;
                    for (size_t q = 0; q < n; q++) {
                        const double t = hit_sphere(sp[q], o, d, 1e-3, best);
                        if (t < best) { best = t; k = (int)q; }
                    }
                    rays.push_back({o, d, best, b == 0});
                    if (k < 0) break;
                    const rt_sphere& S = sp[k];
                    const V pt = o + d * best;
                    const V out = (pt - mkv(S.center)) * (1.0 / S.radius);
                    const bool front = dot(d, out) < 0;
                    const V nrm = front ? out : out * -1.0;
                    if (S.material == RT_LAMBERTIAN) {
                        V nd = nrm + ruv();
                        if (std::fabs(nd.x) < 1e-8 && std::fabs(nd.y) < 1e-8 && std::fabs(nd.z) < 1e-8) nd = nrm;
                        d = nd;
                    } else if (S.material == RT_METAL) {
                        const V r = unit(d - nrm * (2 * dot(d, nrm)));
                        d = r + ruv() * S.fuzz;
                        if (!(dot(d, nrm) > 0)) break;
                    } else {
                        const double ri = front ? 1.0 / S.refraction_index : S.refraction_index;
                        const V u = unit(d);
                        const double ct = std::fmin(dot(u * -1.0, nrm), 1.0), st = std::sqrt(1 - ct * ct);
                        double r0 = (1 - ri) / (1 + ri); r0 *= r0;
                        const double sch = r0 + (1 - r0) * std::pow(1 - ct, 5);
                        if (ri * st > 1 || sch > U(rng)) {
                            d = u - nrm * (2 * dot(u, nrm));
                        } else {
                            const V perp = (u + nrm * ct) * ri;
                            const V par = nrm * -std::sqrt(std::fabs(1 - dot(perp, perp)));
                            d = perp + par;
                        }
                    }
                    o = pt;
                }
            }
    std::shuffle(rays.begin(), rays.end(), rng);
    };
    std::vector<Ray> rays, train_rays;
    trace(12345, stride, spp, rays);
    std::fprintf(stderr, "%zu test rays\n", rays.size());
    const int tstride = argc > 3 ? std::atoi(argv[3]) : 0;  // 0: plain SAH build
    std::vector<rtbvh::TrainRay> train;
    if (tstride < 0) {
        // camera-independent training set: diffuse rays leaving random surface points of the
        // boundable spheres (uniform over spheres and over each sphere's surface) and of the ground
        // within the other spheres' xz extent
        rng.seed(777);
        std::uniform_real_distribution<double> U(0.0, 1.0);
        const size_t want = (size_t)(-tstride) * 1000;
        double xlo = 1e300, xhi = -1e300, zlo = 1e300, zhi = -1e300;
        for (auto& s : sp) if (s.radius < 100) {
            xlo = std::min(xlo, s.center[0] - s.radius); xhi = std::max(xhi, s.center[0] + s.radius);
            zlo = std::min(zlo, s.center[2] - s.radius); zhi = std::max(zhi, s.center[2] + s.radius);
        }
        while (train_rays.size() < want) {
            const size_t k = (size_t)(U(rng) * n);
            const rt_sphere& S = sp[k];
            V nrm, o;
            if (S.radius >= 100) {
                const double x = xlo + U(rng) * (xhi - xlo), z = zlo + U(rng) * (zhi - zlo);
                const V c = mkv(S.center);
                nrm = unit(V{x, 0, z} - c);
                o = c + nrm * S.radius;
            } else {
                V q;
                do { q = {2 * U(rng) - 1, 2 * U(rng) - 1, 2 * U(rng) - 1}; } while (dot(q, q) > 1 || dot(q, q) < 1e-6);
                nrm = unit(q);
                o = mkv(S.center) + nrm * S.radius;
            }
            V q;
            do { q = {2 * U(rng) - 1, 2 * U(rng) - 1, 2 * U(rng) - 1}; } while (dot(q, q) > 1 || dot(q, q) < 1e-6);
            const V d = nrm + unit(q);
            double best = INFINITY;
            for (size_t j = 0; j < n; j++) best = std::min(best, hit_sphere(sp[j], o, d, 1e-3, best));
            train_rays.push_back({o, d, best});
        }
        for (const Ray& r : train_rays) train.push_back({{r.o.x, r.o.y, r.o.z}, {r.d.x, r.d.y, r.d.z}, r.t});
    }
    if (tstride > 0 && argc > 4) {  // the library's own sampler (rtbvh::sample_rays) over the SAH tree
        const auto t0 = std::chrono::steady_clock::now();
        const double ob0 = std::max(rtbvh::scene_extent(sp.data(), n), 13.5);
        const rtbvh::Bvh sah = rtbvh::build(sp.data(), n, ob0);
        train = rtbvh::sample_rays(sp.data(), n, cam, sah, (size_t)std::atoi(argv[4]), 0x5eed);
        const rtbvh::Bvh trained = rtbvh::build(sp.data(), n, ob0, &train);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::fprintf(stderr, "%zu training rays (sample_rays); SAH build + sampling + trained build %.1f ms\n",
                     train.size(), ms);
    } else if (tstride > 0) {
        trace(777, tstride, 1, train_rays);
        for (const Ray& r : train_rays) train.push_back({{r.o.x, r.o.y, r.o.z}, {r.d.x, r.d.y, r.d.z}, r.t});
        std::fprintf(stderr, "%zu training rays\n", train.size());
    }

    // optional: regroup each batch of `group` consecutive rays by a coherence key before forming
    // 64-ray waves (upper bound of what regrouping rays across a block's waves could give)
    if (const char* e = std::getenv("SIM_GROUP")) {
        const size_t group = (size_t)std::atoi(e);
        const int key_mode = std::getenv("SIM_KEY") ? std::atoi(std::getenv("SIM_KEY")) : 0;
        auto key = [&](const Ray& r) -> uint64_t {
            const uint64_t oct = (r.d.x < 0) | (r.d.y < 0) << 1 | (r.d.z < 0) << 2;
            if (key_mode == 0) return oct;
            // octant + coarse origin cell (2-unit cells over [-16, 16)^3)
            auto cell = [](double v) { return (uint64_t)std::min(15.0, std::max(0.0, (v + 16) / 2)); };
            const uint64_t c = cell(r.o.x) | cell(r.o.y) << 4 | cell(r.o.z) << 8;
            if (key_mode == 1) return oct << 12 | c;
            if (key_mode == 2) return c << 3 | oct;
            // scalar keys: the unit direction's y (up-going rays leave the clutter sooner), the
            // origin's height, camera vs secondary
            const double uy = r.d.y / std::sqrt(dot(r.d, r.d));
            const uint64_t ybin = (uint64_t)std::min(15.0, std::max(0.0, (uy + 1) * 8));
            const uint64_t hbin = (uint64_t)std::min(7.0, std::max(0.0, r.o.y * 4 + 1));
            if (key_mode == 3) return ybin;
            if (key_mode == 4) return hbin << 4 | ybin;
            if (key_mode == 5) return (uint64_t)r.camera << 8 | hbin << 4 | ybin;
            return (uint64_t)r.camera << 16 | oct << 8 | hbin << 4 | ybin;
        };
        for (size_t b = 0; b + group <= rays.size(); b += group)
            std::stable_sort(rays.begin() + b, rays.begin() + b + group,
                             [&](const Ray& x, const Ray& y) { return key(x) < key(y); });
    }

    // ---- replay the walk over the built tree ----
    const double ob = std::max(rtbvh::scene_extent(sp.data(), n), 13.5);
    rtbvh::Bvh bvh = rtbvh::build(sp.data(), n, ob, tstride != 0 ? &train : nullptr);
    if (!bvh.ok) { std::fprintf(stderr, "build failed\n"); return 1; }
    const size_t na = bvh.n_always;
    double visits = 0, leaves = 0, wave_steps = 0, wave_leaf = 0, tests = 0;
    std::vector<std::vector<int>> runs(64);
    const bool skip_camera = std::getenv("SIM_SKIP_CAMERA") != nullptr;
    const bool skip_dead = std::getenv("SIM_SKIP_DEAD") != nullptr;  // pop past dead stack entries for free
    const bool skip_leaf_only = std::getenv("SIM_SKIP_DEAD_LEAF_ONLY") != nullptr;  // ... only after a leaf round
    double dead = 0;
    size_t nw = 0;
    std::vector<int> ray_visits(rays.size(), 0);  // inner steps of each ray's walk (SIM_GROUP_ORACLE)
    // SIM_FAR: wave-level candidate blocks now (any lane with class >= 1) and with a far filter (any
    // lane with class 2), for the always-list spheres (in list order) and the leaf rounds (a lane's
    // k-th leaf: one block per round while any lane has a slot left)
    const bool sim_far = std::getenv("SIM_FAR") != nullptr;
    std::vector<std::vector<int>> al_cls(64), lf_now(64), lf_far(64);
    double al_blocks_now = 0, al_blocks_far = 0, lf_blocks_now = 0, lf_blocks_far = 0;
    for (size_t w0 = 0; w0 + 64 <= rays.size(); w0 += 64, ++nw) {
        size_t maxleaf = 0;
        for (int l = 0; l < 64; l++) {
            const Ray& R = rays[w0 + l];
            runs[l].clear();
            if (skip_camera && R.camera) {  // this lane does not walk (its hit comes from elsewhere)
                runs[l].push_back(0);
                continue;
            }
            double closest = INFINITY;
            al_cls[l].assign(na, 0);
            lf_now[l].clear();
            lf_far[l].clear();
            for (size_t q = 0; q < na; q++) {
                if (sim_far) al_cls[l][q] = cand_class(sp[bvh.slot_to_sphere[q]], R.o, R.d, 1e-3, closest);
                closest = std::min(closest, hit_sphere(sp[bvh.slot_to_sphere[q]], R.o, R.d, 1e-3, closest));
            }
            const float inv[3] = {1.0f / (float)R.d.x, 1.0f / (float)R.d.y, 1.0f / (float)R.d.z};
            const float org[3] = {(float)R.o.x, (float)R.o.y, (float)R.o.z};
            auto box = [&](const float* lo, const float* hi, float& tn) {
                float t0 = 1e-3f, t1 = (float)closest * (1 + 1e-6f);
                for (int a = 0; a < 3; a++) {
                    float ta = (lo[a] - org[a]) * inv[a], tb = (hi[a] - org[a]) * inv[a];
                    if (ta > tb) std::swap(ta, tb);
                    t0 = std::max(t0, ta);
                    t1 = std::min(t1, tb);
                }
                tn = t0;
                return t0 <= t1;
            };
            std::vector<std::pair<int32_t, float>> stack;  // (ref, entry distance of its box)
            int32_t cur = 0;
            int run = 0;
            // pop, optionally skipping entries whose box starts beyond the current closest (dead)
            auto pop = [&](int32_t& out, bool after_leaf) {
                while (!stack.empty()) {
                    const auto e = stack.back();
                    stack.pop_back();
                    if (e.second > (float)closest * (1 + 1e-6f)) {
                        dead++;
                        if (skip_dead && (after_leaf || !skip_leaf_only)) continue;
                    }
                    out = e.first;
                    return true;
                }
                return false;
            };
            while (true) {
                if (cur >= 0) {
                    const rtbvh::Node& nd = bvh.nodes[cur];
                    ++run;
                    visits++;
                    float n0, n1;
                    const bool h0 = box(nd.lo0, nd.hi0, n0), h1 = box(nd.lo1, nd.hi1, n1);
                    if (h0 && h1) {
                        const bool f0 = n0 <= n1;
                        stack.push_back({f0 ? nd.ref1 : nd.ref0, f0 ? n1 : n0});
                        cur = f0 ? nd.ref0 : nd.ref1;
                    } else if (h0 || h1) {
                        cur = h0 ? nd.ref0 : nd.ref1;
                    } else {
                        if (!pop(cur, false)) break;
                    }
                } else {
                    runs[l].push_back(run);
                    run = 0;
                    leaves++;
                    const size_t base = na + (size_t)rtbvh::kLeafMax * (size_t)(~cur);
                    int n_now = 0, n_far = 0;
                    if (sim_far) {  // classes against the closest at the round's start (both slots' tests run first)
                        for (int u = 0; u < rtbvh::kLeafMax; u++) {
                            const uint32_t k = bvh.slot_to_sphere[base + u];
                            if (k == rtbvh::kSentinel) continue;
                            const int c = cand_class(sp[k], R.o, R.d, 1e-3, closest);
                            n_now += c >= 1;
                            n_far += c == 2;
                        }
                        lf_now[l].push_back(n_now);
                        lf_far[l].push_back(n_far);
                    }
                    for (int u = 0; u < rtbvh::kLeafMax; u++) {
                        const uint32_t k = bvh.slot_to_sphere[base + u];
                        if (k == rtbvh::kSentinel) continue;
                        tests++;
                        closest = std::min(closest, hit_sphere(sp[k], R.o, R.d, 1e-3, closest));
                    }
                    if (!pop(cur, true)) break;
                }
            }
            runs[l].push_back(run);
            for (int v : runs[l]) ray_visits[w0 + l] += v;
            maxleaf = std::max(maxleaf, runs[l].size() - 1);
        }
        wave_leaf += (double)maxleaf;
        if (sim_far) {
            for (size_t q = 0; q < na; q++) {
                bool any_now = false, any_far = false;
                for (int l = 0; l < 64; l++) {
                    any_now |= al_cls[l].size() > q && al_cls[l][q] >= 1;
                    any_far |= al_cls[l].size() > q && al_cls[l][q] == 2;
                }
                al_blocks_now += any_now;
                al_blocks_far += any_far;
            }
            for (size_t k = 0; k < maxleaf; k++) {  // leaf round k: blocks = max slots left over lanes
                int mn = 0, mf = 0;
                for (int l = 0; l < 64; l++)
                    if (k < lf_now[l].size()) { mn = std::max(mn, lf_now[l][k]); mf = std::max(mf, lf_far[l][k]); }
                lf_blocks_now += mn;
                lf_blocks_far += mf;
            }
        }
        for (size_t k = 0; k <= maxleaf; k++) {
            int m = 0;
            for (int l = 0; l < 64; l++)
                if (k < runs[l].size()) m = std::max(m, runs[l][k]);
            wave_steps += m;
        }
    }
    // optional (upper bound of ANY regrouping key): SIM_GROUP_ORACLE=g sorts each batch of g
    // consecutive rays by their true walk length (inner steps, known only after the walk) before the
    // wave models below, as if a block could group its in-flight segments by the cost they are
    // about to have
    if (const char* e = std::getenv("SIM_GROUP_ORACLE")) {
        const size_t group = (size_t)std::atoi(e);
        std::vector<size_t> idx(rays.size());
        for (size_t i = 0; i < idx.size(); i++) idx[i] = i;
        for (size_t b = 0; b + group <= rays.size(); b += group)
            std::stable_sort(idx.begin() + b, idx.begin() + b + group,
                             [&](size_t x, size_t y) { return ray_visits[x] < ray_visits[y]; });
        std::vector<Ray> sorted(rays.size());
        for (size_t i = 0; i < idx.size(); i++) sorted[i] = rays[idx[i]];
        rays.swap(sorted);
    }

    // ---- lockstep model of one wave (SIM_LOCKSTEP): all lanes advance together; with SIM_STEAL a
    // lane whose walk is over takes the oldest stack entry of the lane with the deepest stack and
    // walks that subtree for the same ray (closest shared instantly: an optimistic bound) ----
    double ls_steps = 0, ls_leaf = 0, ls_steals = 0, ls_batches = 0;
    size_t ls_waves = 0;
    if (std::getenv("SIM_LOCKSTEP")) {
        const bool steal = std::getenv("SIM_STEAL") != nullptr;
        // helpers cull with the owner's closest as it was when they stole (no sharing until the end)
        const bool snap = std::getenv("SIM_STEAL_SNAPSHOT") != nullptr;
        const size_t min_victim = std::getenv("SIM_STEAL_MIN") ? (size_t)std::atoi(std::getenv("SIM_STEAL_MIN")) : 1;
        const bool steal_top = std::getenv("SIM_STEAL_TOP") != nullptr;  // take the newest entry instead of the oldest
        // helpers only traverse: a leaf a helper reaches is pushed onto its owner's stack (the owner
        // tests it later with its own f64 ray); a lane with a helper out does not help others
        const bool trav_only = std::getenv("SIM_STEAL_TRAVERSE_ONLY") != nullptr;
        const int max_batches = std::getenv("SIM_STEAL_MAXB") ? std::atoi(std::getenv("SIM_STEAL_MAXB")) : 1 << 30;  // per wave walk
        const int min_idle = std::getenv("SIM_STEAL_MIN_IDLE") ? std::atoi(std::getenv("SIM_STEAL_MIN_IDLE")) : 1;  // idle lanes to start a batch
        const int max_helpers = std::getenv("SIM_STEAL_MAXH") ? std::atoi(std::getenv("SIM_STEAL_MAXH")) : 64;  // per ray, over the walk
        const int32_t kDoneRef = INT32_MIN;
        const int walkers = std::getenv("SIM_WALKERS") ? std::atoi(std::getenv("SIM_WALKERS")) : 64;  // lanes with a ray
        for (size_t w0 = 0; w0 + 64 <= rays.size(); w0 += walkers, ++ls_waves) {
            double cl[64], lc[64];  // per-ray closest (shared); per-lane copies (snapshot mode)
            float org[64][3], inv[64][3];
            int ray[64];
            int32_t cur[64];
            std::vector<int32_t> st[64];
            for (int l = 0; l < 64; l++) {
                const Ray& R = rays[w0 + l];
                cl[l] = INFINITY;
                for (size_t q = 0; q < na; q++) cl[l] = std::min(cl[l], hit_sphere(sp[bvh.slot_to_sphere[q]], R.o, R.d, 1e-3, cl[l]));
                org[l][0] = (float)R.o.x; org[l][1] = (float)R.o.y; org[l][2] = (float)R.o.z;
                inv[l][0] = 1.0f / (float)R.d.x; inv[l][1] = 1.0f / (float)R.d.y; inv[l][2] = 1.0f / (float)R.d.z;
                ray[l] = l;
                lc[l] = cl[l];
                cur[l] = 0;
                if (skip_camera && R.camera) cur[l] = kDoneRef;
                if (l >= walkers) cur[l] = kDoneRef;  // no path to walk this iteration: a helper from the start
            }
            auto boxt = [&](int l, int r, const float* lo, const float* hi, float& tn) {
                float t0 = 1e-3f, t1 = (float)(snap ? lc[l] : cl[r]) * (1 + 1e-6f);
                for (int a = 0; a < 3; a++) {
                    float ta = (lo[a] - org[r][a]) * inv[r][a], tb = (hi[a] - org[r][a]) * inv[r][a];
                    if (ta > tb) std::swap(ta, tb);
                    t0 = std::max(t0, ta);
                    t1 = std::min(t1, tb);
                }
                tn = t0;
                return t0 <= t1;
            };
            auto pop = [&](int l) {
                if (st[l].empty()) { cur[l] = kDoneRef; return; }
                cur[l] = st[l].back();
                st[l].pop_back();
            };
            int helpers[64] = {0};
            int batches = 0;
            int out[64] = {0};   // helpers currently working for lane l's ray
            int owner[64];
            for (int l = 0; l < 64; l++) owner[l] = l;
            auto try_steal = [&](int l) {  // l is idle: take the oldest entry of the deepest stack
                if (trav_only && out[l] > 0) return;  // keeps its stack free for returned leaves
                int v = -1;
                size_t best = 0;
                for (int m = 0; m < 64; m++)
                    if (m != l && st[m].size() >= min_victim && st[m].size() > best && helpers[ray[m]] < max_helpers) {
                        best = st[m].size();
                        v = m;
                    }
                if (v < 0) return;
                helpers[ray[v]]++;
                if (steal_top) {
                    cur[l] = st[v].back();
                    st[v].pop_back();
                } else {
                    cur[l] = st[v].front();
                    st[v].erase(st[v].begin());
                }
                ray[l] = ray[v];
                lc[l] = lc[v];
                owner[l] = owner[v];
                out[owner[v]]++;
                ls_steals++;
            };
            while (true) {
                // inner phase
                while (true) {
                    bool any = false;
                    for (int l = 0; l < 64; l++) {
                        if (cur[l] < 0) continue;
                        any = true;
                        const rtbvh::Node& nd = bvh.nodes[cur[l]];
                        float n0, n1;
                        const int r = ray[l];
                        const bool h0 = boxt(l, r, nd.lo0, nd.hi0, n0), h1 = boxt(l, r, nd.lo1, nd.hi1, n1);
                        if (h0 && h1) {
                            const bool f0 = n0 <= n1;
                            st[l].push_back(f0 ? nd.ref1 : nd.ref0);
                            cur[l] = f0 ? nd.ref0 : nd.ref1;
                        } else if (h0 || h1) {
                            cur[l] = h0 ? nd.ref0 : nd.ref1;
                        } else {
                            pop(l);
                        }
                    }
                    if (!any) break;
                    ls_steps++;
                    if (trav_only)  // helpers hand their leaves to the owner and keep traversing
                        for (int l = 0; l < 64; l++) {
                            if (owner[l] == l) continue;
                            if (cur[l] < 0 && cur[l] != kDoneRef) {
                                const int o = owner[l];
                                if (cur[o] == kDoneRef) cur[o] = cur[l]; else st[o].push_back(cur[l]);
                                pop(l);
                            }
                            if (cur[l] == kDoneRef && st[l].empty()) {  // subtree finished
                                out[owner[l]]--;
                                owner[l] = l;
                                ray[l] = l;
                            }
                        }
                    int idle = 0;
                    for (int l = 0; l < 64; l++) idle += cur[l] == kDoneRef;
                    if (steal && batches < max_batches && idle >= min_idle) {
                        const double before = ls_steals;
                        for (int l = 0; l < 64; l++)
                            if (cur[l] == kDoneRef) try_steal(l);
                        if (ls_steals > before) { ls_batches++; batches++; }
                    }
                }
                bool leaf = false;
                for (int l = 0; l < 64; l++) leaf = leaf || (cur[l] != kDoneRef);
                if (!leaf) break;
                ls_leaf++;
                for (int l = 0; l < 64; l++) {
                    if (cur[l] == kDoneRef) continue;
                    const Ray& R = rays[w0 + ray[l]];
                    const size_t base = na + (size_t)rtbvh::kLeafMax * (size_t)(~cur[l]);
                    for (int u = 0; u < rtbvh::kLeafMax; u++) {
                        const uint32_t k = bvh.slot_to_sphere[base + u];
                        if (k == rtbvh::kSentinel) continue;
                        const double t = hit_sphere(sp[k], R.o, R.d, 1e-3, snap ? lc[l] : cl[ray[l]]);
                        lc[l] = std::min(lc[l], t);
                        cl[ray[l]] = std::min(cl[ray[l]], t);
                    }
                    pop(l);
                }
                int idle2 = 0;
                for (int l = 0; l < 64; l++) idle2 += cur[l] == kDoneRef;
                if (steal && batches < max_batches && idle2 >= min_idle) {
                    const double before = ls_steals;
                    for (int l = 0; l < 64; l++)
                        if (cur[l] == kDoneRef) try_steal(l);
                    if (ls_steals > before) { ls_batches++; batches++; }
                }
            }
        }
        std::fprintf(stderr, "lockstep%s: wave steps %.3f, leaf rounds %.3f, steals per wave %.2f in %.2f batches\n",
                     steal ? "+steal" : "", ls_steps / ls_waves, ls_leaf / ls_waves, ls_steals / ls_waves,
                     ls_batches / ls_waves);
    }

    // ---- dynamic fetch (SIM_REFETCH=K): one 64-lane wave streams through all the rays; after a
    // leaf round, once at least K lanes have finished their walk, each of them takes the next ray
    // (in the kernel: shade the finished segment and start the next one inside the walk loop, one
    // wave-uniform shading block per refetch batch).  Reported per 64 rays, to compare with the
    // lockstep model's per-wave figures. ----
    if (std::getenv("SIM_REFETCH")) {
        const int min_done = std::atoi(std::getenv("SIM_REFETCH"));
        // SIM_REFETCH_P: chance that a lane leaving a shading batch has a segment to walk (the
        // kernel's other lanes wait on rejection trips or a refill: ~40 of 64 walk per iteration)
        const double p_ready = std::getenv("SIM_REFETCH_P") ? std::atof(std::getenv("SIM_REFETCH_P")) : 1.0;
        std::mt19937_64 prng(7);
        std::uniform_real_distribution<double> PU(0.0, 1.0);
        const int32_t kDoneRef = INT32_MIN;
        double cl[64];
        float org[64][3], inv[64][3];
        int32_t cur[64];
        std::vector<int32_t> st[64];
        size_t next = 0, started = 0;
        double steps = 0, leafr = 0, batches = 0, lane_steps = 0;
        auto start = [&](int l) {
            if (next >= rays.size()) { cur[l] = kDoneRef; return; }
            const Ray& R = rays[next++];
            ++started;
            cl[l] = INFINITY;
            for (size_t q = 0; q < na; q++) cl[l] = std::min(cl[l], hit_sphere(sp[bvh.slot_to_sphere[q]], R.o, R.d, 1e-3, cl[l]));
            org[l][0] = (float)R.o.x; org[l][1] = (float)R.o.y; org[l][2] = (float)R.o.z;
            inv[l][0] = 1.0f / (float)R.d.x; inv[l][1] = 1.0f / (float)R.d.y; inv[l][2] = 1.0f / (float)R.d.z;
            st[l].clear();
            cur[l] = 0;
        };
        std::vector<size_t> rid(64);
        for (int l = 0; l < 64; l++) { rid[l] = next; start(l); }
        auto boxt = [&](int l, const float* lo, const float* hi, float& tn) {
            float t0 = 1e-3f, t1 = (float)cl[l] * (1 + 1e-6f);
            for (int a = 0; a < 3; a++) {
                float ta = (lo[a] - org[l][a]) * inv[l][a], tb = (hi[a] - org[l][a]) * inv[l][a];
                if (ta > tb) std::swap(ta, tb);
                t0 = std::max(t0, ta);
                t1 = std::min(t1, tb);
            }
            tn = t0;
            return t0 <= t1;
        };
        auto pop = [&](int l) {
            if (st[l].empty()) { cur[l] = kDoneRef; return; }
            cur[l] = st[l].back();
            st[l].pop_back();
        };
        while (true) {
            bool live = false;
            for (int l = 0; l < 64; l++) live = live || cur[l] != kDoneRef;
            if (!live && next >= rays.size()) break;
            while (true) {  // inner phase
                int act = 0;
                for (int l = 0; l < 64; l++) {
                    if (cur[l] < 0) continue;
                    ++act;
                    const rtbvh::Node& nd = bvh.nodes[cur[l]];
                    float n0, n1;
                    const bool h0 = boxt(l, nd.lo0, nd.hi0, n0), h1 = boxt(l, nd.lo1, nd.hi1, n1);
                    if (h0 && h1) {
                        const bool f0 = n0 <= n1;
                        st[l].push_back(f0 ? nd.ref1 : nd.ref0);
                        cur[l] = f0 ? nd.ref0 : nd.ref1;
                    } else if (h0 || h1) {
                        cur[l] = h0 ? nd.ref0 : nd.ref1;
                    } else {
                        pop(l);
                    }
                }
                if (!act) break;
                ++steps;
                lane_steps += act;
            }
            bool leaf = false;
            for (int l = 0; l < 64; l++) leaf = leaf || cur[l] != kDoneRef;
            if (leaf) {
                ++leafr;
                for (int l = 0; l < 64; l++) {
                    if (cur[l] == kDoneRef) continue;
                    const Ray& R = rays[rid[l]];
                    const size_t base = na + (size_t)rtbvh::kLeafMax * (size_t)(~cur[l]);
                    for (int u = 0; u < rtbvh::kLeafMax; u++) {
                        const uint32_t k = bvh.slot_to_sphere[base + u];
                        if (k == rtbvh::kSentinel) continue;
                        cl[l] = std::min(cl[l], hit_sphere(sp[k], R.o, R.d, 1e-3, cl[l]));
                    }
                    pop(l);
                }
            }
            int done = 0;
            for (int l = 0; l < 64; l++) done += cur[l] == kDoneRef;
            const bool all_done = done == 64;
            if (next < rays.size() && (done >= min_done || all_done)) {
                ++batches;
                for (int l = 0; l < 64; l++)
                    if (cur[l] == kDoneRef && PU(prng) < p_ready) { rid[l] = next; start(l); }
            } else if (all_done) {
                break;
            }
        }
        const double per = 64.0 / (double)started;
        std::fprintf(stderr, "refetch K=%d: per 64 rays: wave steps %.3f, leaf rounds %.3f, shading batches %.3f; lane util %.3f\n",
                     min_done, steps * per, leafr * per, batches * per, lane_steps / (64.0 * steps));
    }

    const double nr = (double)nw * 64;
    // SIM_ALWAYS: wave-level candidate blocks of the always-list tests under other schedules, from
    // the rays' lockstep waves: "seq" = one block per sphere any lane needs (the kernel's), "pairs" =
    // the leaf rounds' compaction over sphere pairs (0,1),(2,3) of the order, "full" = one block per
    // round over all spheres; "far" drops candidates whose root1 lies beyond the running closest;
    // orders: the list's, and the ground (the largest) last
    if (std::getenv("SIM_ALWAYS") && na == 4) {
        for (size_t q = 0; q < na; q++) std::fprintf(stderr, "always[%zu] = sphere %u, r = %.3f\n", q, bvh.slot_to_sphere[q], sp[bvh.slot_to_sphere[q]].radius);
        const std::vector<std::vector<int>> orders = {{0, 1, 2, 3}, {1, 2, 3, 0}};
        for (const auto& ord : orders)
            for (int far = 0; far < 2; far++) {
                double seq = 0, pairs = 0, full = 0;
                size_t waves = 0;
                for (size_t w0 = 0; w0 + 64 <= rays.size(); w0 += 64, ++waves) {
                    bool any[4] = {}, any01 = false, any23 = false, p01 = false, p23 = false;
                    int mx = 0;
                    for (int l = 0; l < 64; l++) {
                        const Ray& R = rays[w0 + l];
                        double closest = INFINITY;
                        bool v[4];
                        for (int i = 0; i < 4; i++) {
                            const rt_sphere& S = sp[bvh.slot_to_sphere[ord[i]]];
                            const int c = cand_class(S, R.o, R.d, 1e-3, closest);
                            v[i] = far ? c == 2 : c >= 1;
                            closest = std::min(closest, hit_sphere(S, R.o, R.d, 1e-3, closest));
                        }
                        for (int i = 0; i < 4; i++) any[i] |= v[i];
                        any01 |= v[0] || v[1]; p01 |= v[0] && v[1];
                        any23 |= v[2] || v[3]; p23 |= v[2] && v[3];
                        mx = std::max(mx, (int)v[0] + v[1] + v[2] + v[3]);
                    }
                    seq += any[0] + any[1] + any[2] + any[3];
                    pairs += any01 + p01 + any23 + p23;
                    full += mx;
                }
                std::fprintf(stderr, "always-list blocks per wave, order %d%d%d%d%s: seq %.3f, pairs %.3f, full %.3f\n",
                             ord[0], ord[1], ord[2], ord[3], far ? " + far filter" : "", seq / waves, pairs / waves, full / waves);
            }
    }
    if (sim_far)
        std::fprintf(stderr, "far filter (lockstep waves of 64 rays): candidate blocks per wave: always-list %.3f -> %.3f, "
                     "leaf rounds %.3f -> %.3f\n", al_blocks_now / nw, al_blocks_far / nw, lf_blocks_now / nw, lf_blocks_far / nw);
    std::printf("{\"nodes\": %zu, \"depth\": %d, \"n_always\": %zu, \"visits_per_ray\": %.4f, \"leaves_per_ray\": %.4f, "
                "\"leaf_tests_per_ray\": %.4f, \"wave_inner_steps\": %.3f, \"wave_leaf_rounds\": %.3f, \"dead_pops_per_ray\": %.4f}\n",
                bvh.nodes.size(), bvh.depth, na, visits / nr, leaves / nr, tests / nr, wave_steps / nw, wave_leaf / nw, dead / nr);
    return 0;
}

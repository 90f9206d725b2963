// trip_bench.hip — the rejection-trip lever measured instead of argued.
//
// Two rejection samplers draw from a lane's stream in the path loop (rt_kernel.hip): randomUnitVec
// (vec.zig:71-80, 3 draws a trip, accept pi/6) for a pending Lambertian / Metal scatter and
// randomInUnitDisk (vec.zig:82-92, 2 draws a trip, accept pi/4) for a camera ray's defocus sample.
// A wave pays the maximum trip count over its lanes.  This microbenchmark replays the loop's
// request pattern with nothing else in the kernel and compares two generators:
//
//   A  the product: per-(pixel, sample) Xoshiro256++ streams (rtk::Rng, the same seeding and
//      Random.float(f64) conversion), the product's capped loop (kRuvTrips = 3 per iteration; a lane
//      still rejected stays pending into the next iteration);
//   B  a counter-based generator: draw k of a request = Random.float(f64) of mix(key ^ k) (one
//      SplitMix64 finaliser per draw, random access), so ANY lane can evaluate candidate j of ANY
//      pending lane: per pass the 64 lanes evaluate 64 candidate slots spread over the pending
//      lanes (slot -> owner by a compacted list in LDS), the acceptance is a ballot, and each
//      pending lane takes its lowest accepted candidate (its own stream's first accepted one, so the
//      draws consumed are exactly the sequential loop's); up to kPasses passes per iteration.
//
// Request pattern per lane and iteration (the path loop's, in the proportions of one instrumented
// config-4 frame, tools/kprofile.py "wave_level"): a lane with no request starts a randomUnitVec
// request with probability P_RUV and else a disk request with probability P_DISK (command line).
// Work is a fixed number of requests per lane; the kernel time divided by the requests served is
// the cost per request, reported with the wave-level trips / passes.  Both generators' accepted
// points are summed into a checksum (keeps the work live).  Each lane draws from ONE stream for all
// its requests, so the per-sample seeding (A: SplitMix64 x 4 into the Xoshiro state; B: none) is
// not in the timing — B would save it on top.
//
//   hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 tools/trip_bench.hip -o tools/bin/trip_bench
//   ./tools/bin/trip_bench [P_RUV=0.45] [P_DISK=0.2] [requests_per_lane=2000]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../raytracing-with-zig_amd/csrc/rt_device.h"

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

namespace tb {
using namespace rtk;

// request arrival: a per-(lane, iteration) hash against the probabilities
__device__ __forceinline__ uint32_t arrive(uint32_t gl, uint32_t it, float p_ruv, float p_disk) {
    const uint32_t h = (uint32_t)(sm_mix_hd(((uint64_t)gl << 32) | it) >> 40);
    const float u = (float)h * 0x1p-24f;
    return u < p_ruv ? 1u : (u < p_ruv + p_disk ? 2u : 0u);
}

__device__ __forceinline__ double u01(uint64_t rnd) {  // Random.float(f64) of one 64-bit draw
    const uint32_t hi = (uint32_t)(rnd >> 32);
    if (hi >= (1u << 20)) {
        const uint32_t lz = __builtin_clz(hi);
        return __builtin_bit_cast(double, ((uint64_t)((1022u - lz) << 20 | (hi & 0xfffffu)) << 32) | (uint32_t)rnd);
    }
    Rng g;  // rare: the exact slow path (>= 12 leading zeros) of rtk::Rng
    g.s0 = g.s1 = g.s2 = g.s3 = 0;
    return g.uniform_slow(rnd);
}

// A: the product's loop (3 capped trips per iteration, pending carried)
__global__ __launch_bounds__(256) void bench_a(uint32_t reqs, float p_ruv, float p_disk, double* sum,
                                                unsigned long long* ctr) {
    const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
    Rng g;
    g.seed(sample_key(0x1234, gl, 0));  // one stream per lane: the trip loop alone is timed
    uint32_t kind = 0, served = 0, it = 0;
    double acc = 0;
    uint64_t trips = 0, iters = 0;
    while (__ballot(served < reqs) != 0) {
        ++it;
        if (kind == 0 && served < reqs) {
            kind = arrive(gl, it, p_ruv, p_disk);
        }
        bool got = false;
        double x = 0, y = 0, z = 0;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const bool need = kind != 0 && !got;
            if (__ballot(need) == 0) break;
            if (threadIdx.x % 64 == 0) ++trips;
            if (need) {
                x = g.range_pm1();
                y = g.range_pm1();
                const double xy = x * x + y * y;
                if (kind == 1) {
                    z = g.range_pm1();
                    const double l = xy + z * z;
                    got = 1e-160 < l && l <= 1;
                } else {
                    got = xy + 0.0 * 0.0 < 1;
                }
            }
        }
        if (threadIdx.x % 64 == 0) ++iters;
        if (got) {
            acc += x + 2 * y + 3 * z;
            kind = 0;
            ++served;
        }
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (threadIdx.x % 64 == 0) {
        atomicAdd(sum, acc);
        atomicAdd(ctr + 0, (unsigned long long)trips);
        atomicAdd(ctr + 1, (unsigned long long)iters);
    }
}

// B: counter-based draws, candidates of every pending lane evaluated by all 64 lanes
constexpr int kPasses = 2;
__device__ __forceinline__ uint64_t draw(uint64_t key, uint32_t k) { return sm_mix_hd(key ^ ((uint64_t)k << 1 | 1)); }

__global__ __launch_bounds__(256) void bench_b(uint32_t reqs, float p_ruv, float p_disk, double* sum,
                                                unsigned long long* ctr) {
    __shared__ uint64_t s_key[256];
    __shared__ uint32_t s_pos[256], s_kind[256];
    const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x % 64, wbase = threadIdx.x - lane;
    const uint64_t key = sample_key(0x1234, gl, 0);  // one stream per lane, drawn at `pos`
    uint32_t pos = 0, kind = 0, served = 0, it = 0;
    double acc = 0;
    uint64_t passes = 0, iters = 0;
    while (__ballot(served < reqs) != 0) {
        ++it;
        if (kind == 0 && served < reqs) {
            kind = arrive(gl, it, p_ruv, p_disk);
        }
        bool got = false;
        double x = 0, y = 0, z = 0;
        for (int ps = 0; ps < kPasses; ++ps) {
            const uint64_t pend = __ballot(kind != 0 && !got);
            const uint32_t np = (uint32_t)__popcll(pend);
            if (np == 0) break;
            if (lane == 0) ++passes;
            // compact the pending lanes' (key, position, kind) into LDS slots 0..np-1
            const uint32_t rk = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(pend >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)pend, 0u));
            if (kind != 0 && !got) {
                s_key[wbase + rk] = key;
                s_pos[wbase + rk] = pos;
                s_kind[wbase + rk] = kind;
            }
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            // slot t evaluates candidate j = t / np of owner o = t % np (owner-interleaved, so every
            // owner gets its candidates 0, 1, ... in stream order)
            const uint32_t per = 64 / np;
            const uint32_t o = lane % np, j = lane / np;
            const bool live = j < per;
            const uint64_t k_o = s_key[wbase + o];
            const uint32_t kd = s_kind[wbase + o], p0 = s_pos[wbase + o];
            const uint32_t d = kd == 1 ? 3u : 2u;
            double cx = 0, cy = 0, cz = 0;
            bool acc_ok = false;
            if (live) {
                cx = __builtin_fma(2.0, u01(draw(k_o, p0 + j * d + 0)), -1.0);
                cy = __builtin_fma(2.0, u01(draw(k_o, p0 + j * d + 1)), -1.0);
                const double xy = cx * cx + cy * cy;
                if (kd == 1) {
                    cz = __builtin_fma(2.0, u01(draw(k_o, p0 + j * d + 2)), -1.0);
                    const double l = xy + cz * cz;
                    acc_ok = 1e-160 < l && l <= 1;
                } else {
                    acc_ok = xy + 0.0 * 0.0 < 1;
                }
            }
            const uint64_t acm = __ballot(acc_ok);
            // owner rk's slots are rk, rk + np, rk + 2 np, ...: its first accepted one
            const bool mine = kind != 0 && !got;
            uint32_t best = 64;
            if (mine)
                for (uint32_t jj = 0; jj < per; ++jj)
                    if ((acm >> (rk + jj * np)) & 1) {
                        best = rk + jj * np;
                        break;
                    }
            // every lane takes part in the shuffles (a bpermute reads only lanes that execute it)
            const uint32_t src = best < 64 ? best : lane;
            const double sx = __shfl(cx, src, 64), sy = __shfl(cy, src, 64), sz = __shfl(cz, src, 64);
            if (mine) {
                if (best < 64) {
                    x = sx;
                    y = sy;
                    z = sz;
                    got = true;
                    pos += ((best - rk) / np + 1) * (kind == 1 ? 3u : 2u);
                } else {
                    pos += per * (kind == 1 ? 3u : 2u);
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (lane == 0) ++iters;
        if (got) {
            acc += x + 2 * y + 3 * z;
            kind = 0;
            ++served;
        }
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) {
        atomicAdd(sum, acc);
        atomicAdd(ctr + 0, (unsigned long long)passes);
        atomicAdd(ctr + 1, (unsigned long long)iters);
    }
}
}  // namespace tb

int main(int argc, char** argv) {
    const float p_ruv = argc > 1 ? (float)std::atof(argv[1]) : 0.45f;
    const float p_disk = argc > 2 ? (float)std::atof(argv[2]) : 0.2f;
    const uint32_t reqs = argc > 3 ? (uint32_t)std::atoi(argv[3]) : 2000;
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t blocks = (uint32_t)cus * 4;  // 16 waves per CU, as the product's BVH kernel
    double* d_sum = nullptr;
    unsigned long long* d_ctr = nullptr;
    CK(hipMalloc(&d_sum, sizeof(double)));
    CK(hipMalloc(&d_ctr, 2 * sizeof(unsigned long long)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double total = (double)blocks * 256 * reqs;
    std::printf("{\"p_ruv\": %.3f, \"p_disk\": %.3f, \"requests\": %.0f, \"waves\": %u, \"results\": [", p_ruv, p_disk, total,
                blocks * 4);
    for (int v = 0; v < 2; ++v) {
        std::vector<float> ms;
        unsigned long long c[2] = {0, 0};
        double sum = 0;
        for (int rep = 0; rep < 4; ++rep) {
            CK(hipMemset(d_sum, 0, sizeof(double)));
            CK(hipMemset(d_ctr, 0, 2 * sizeof(unsigned long long)));
            CK(hipEventRecord(e0));
            if (v == 0)
                hipLaunchKernelGGL(tb::bench_a, dim3(blocks), dim3(256), 0, 0, reqs, p_ruv, p_disk, d_sum, d_ctr);
            else
                hipLaunchKernelGGL(tb::bench_b, dim3(blocks), dim3(256), 0, 0, reqs, p_ruv, p_disk, d_sum, d_ctr);
            CK(hipGetLastError());
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (rep) ms.push_back(t);
            CK(hipMemcpy(c, d_ctr, sizeof c, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&sum, d_sum, sizeof sum, hipMemcpyDeviceToHost));
        }
        std::sort(ms.begin(), ms.end());
        const double med = ms[ms.size() / 2];
        std::printf("%s{\"generator\": \"%s\", \"ms\": %.4f, \"ns_per_request_per_gpu\": %.5f, \"wave_iterations\": %llu, "
                    "\"wave_%s\": %llu, \"per_iteration\": %.4f, \"checksum\": %.6e}",
                    v ? ", " : "", v ? "B counter-based, cooperative" : "A per-lane Xoshiro256++, 3 trips",
                    med, med * 1e6 / total, c[1], v ? "passes" : "trips", c[0], (double)c[0] / (double)c[1], sum);
    }
    std::printf("]}\n");
    return 0;
}

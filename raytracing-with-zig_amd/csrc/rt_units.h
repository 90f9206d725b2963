// rt_units.h — device side of the unit scheduler and the ordered in-kernel accumulation
// (rt_kernel.h "Work units").  Shared by every sample kernel of rt_kernel.hip (parity
// list / BVH walks and the f32 fast mode, all instantiations of one path_loop).
//
// Hand-off between waves (possibly on different XCDs, whose L2s are not coherent with each other):
// the running sums are stored write-through (sc1: agent-scope relaxed atomic stores), every storing
// wave drains them (s_waitcnt vmcnt(0)) before ONE lane stores the tile's flag (an sc1 store), and
// the consumer polls the flag with an sc1 load and reads the sums with sc1 loads only — the
// MI355X hand-off recipe (cdna_hip_programming.md Guideline 16, R1 with sc1 loads).  A wave's ring
// is private to it and written and read by its own CU: plain stores, plain loads behind the wave's
// own s_waitcnt vmcnt(0) (a workgroup's L1 sees its own CU's stores).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_device.h"
#include "rt_kernel.h"

namespace rtk {

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;

// Debug builds (-DRTZIG_BOUNDS=1, tools/diag_modes.py): every index into a global buffer or a lane's
// LDS stack is checked; one out of range sets kErrBounds in the sticky error word (the host reports
// it: rt_context_sync / rt_render) and the access is skipped or redirected in range, so a bad index
// shows up as a reported error instead of a memory fault.  Shipped builds compile the checks away.
#ifndef RTZIG_BOUNDS
#define RTZIG_BOUNDS 0
#endif
constexpr bool kBounds = RTZIG_BOUNDS != 0;
__device__ __forceinline__ bool bounds_ok(bool ok, unsigned long long* ctr) {
    if constexpr (kBounds) {
        if (!ok) atomicOr(ctr + kErrWord, kErrBounds);
        return ok;
    }
    return true;
}

__device__ __forceinline__ double ld_wt(const double* p) {  // global_load_dwordx2 ... sc1
    return __builtin_bit_cast(double, __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_wt(double* p, double v) {  // global_store_dwordx2 ... sc1
    __hip_atomic_store((gu64*)p, __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A wave that cannot claim and has nothing to trace sleeps between polls.  A bug that broke the
// dependency chain would otherwise hang the GPU, so each continuous wait is bounded — by wall clock
// (s_memrealtime, a constant 100 MHz), not by a count of sleeps: a predecessor unit may legitimately
// take seconds to trace (a scene too large for the tree, walked linearly: ~100x the final scene's
// per-ray cost at 70 000 spheres), and a fixed sleep count scaled with nothing.  The clock restarts
// whenever this wave claims or finalises a unit; past ua.stall_ticks the wave reports it in the
// sticky ctr[kErrWord] and gives up (the host returns RT_ERR_HIP).  The bound is set per launch by
// the host (rt_runtime.cpp stall_bound: 40 s, scaled with the sphere count for list walks).  The
// wait's state is ONE SGPR, as the round-2 sleep counter was: a global-progress bound (every
// finalisation counted, the count and the clock carried by the waiting wave) cost 1.1-1.7% of the
// frame through SGPR spills into the walk's VGPRs.  The clock is kept in units of 256 ticks
// (kStallTickNs = 2.56 µs) as 32 bits: wrapping differences are exact below 2^32 units = 3.05 h.
__device__ __forceinline__ uint32_t wait_clock() { return (uint32_t)(__builtin_amdgcn_s_memrealtime() >> 8); }


// Wave-uniform scheduler state (every member is the same in all 64 lanes).  kDirect: direct mode
// (rt_kernel.h): guided claims of flat items t = s * P + q (also the item's index in ua.samples);
// no slots, no finalisation.
template <bool kDirect>
struct UnitSched {
    const UnitArgs& ua;
    double* ring;                    // this wave's ring: kSlots x [kUnitS * 64][3]
    uint32_t busy = 0;               // slots holding a unit that is not finalised yet
    uint32_t cur_slot = 0, cur = 0, end = 0;  // the slot being handed out: items [cur, end)
    uint32_t cur_tile = 0, cur_s0 = 0;
    uint32_t st_u[kSlots];           // unit id held by each slot
    uint32_t spins = 0;              // sleeps in all (diagnostics)
    uint32_t wait_t0 = 0;            // wait_clock() | 1 when the current wait began (0: not waiting)
    uint32_t seen = 0;               // direct mode: item position after this wave's last claim
    uint32_t waves = 1;              // direct mode: the launch's waves
    uint32_t seg = 0, empty = 0;     // direct mode: segment claimed from; segments found empty
    bool away = false;               // direct mode: claiming outside the home segment
    uint32_t n_dep_wait = 0;   // diagnostics (instrumented build): finalisations deferred on a flag
    uint32_t n_no_slot = 0;    // ... refills stopped for want of a free slot
    bool drained = false;            // the claim counter is exhausted
    bool failed = false;             // stall bound reached (reported in ctr[kErrWord])

    __device__ UnitSched(const UnitArgs& a, uint32_t wave) : ua(a), ring(a.ring + (size_t)wave * kRingWaveDoubles) {
        if constexpr (kBounds && !kDirect) {
            if (!bounds_ok(wave < a.ring_waves, a.ctr)) ring = a.ring;
        }
        if constexpr (kDirect) {
            waves = gridDim.x * (blockDim.x / 64);
            seg = blockIdx.x % kSegs;
            seen = seg_lo(seg);
        }
#pragma unroll
        for (uint32_t j = 0; j < kSlots; ++j) st_u[j] = 0;
    }
    // direct mode: first item of queue segment g (segments split the P * spp items evenly)
    __device__ __forceinline__ uint32_t seg_lo(uint32_t g) const {
        return (uint32_t)((uint64_t)ua.n_units * g / kSegs);
    }
    __device__ __forceinline__ bool can_claim() const { return !drained && (kDirect || (~busy & kSlotMask) != 0); }

    // Claims the next unit into a free slot and makes it the one handed out; false if there is no
    // free slot or no unit left.
    __device__ __forceinline__ bool claim(uint32_t lane) {
        if constexpr (kDirect) {
            while (!drained) {
                const uint32_t lo = seg_lo(seg), hi = seg_lo(seg + 1);
                // guided in the home segment: 1/8 of an even share of what it has left (as this
                // wave last saw it; its kSegs-th of the waves claim there), 64..2048 items in whole
                // multiples of 64; elsewhere 64
                const uint32_t left = hi > seen ? hi - seen : 0u;
                uint32_t k = away ? 64u : left / waves;
                k = k < 64u ? 64u : (k > 2048u ? 2048u : k & ~63u);
                uint32_t t = 0;
                if (lane == 0) t = (uint32_t)atomicAdd(ua.ctr + kCtrStride * seg, (unsigned long long)k);
                t = lo + __builtin_amdgcn_readfirstlane(t);
                if (t < hi) {
                    wait_t0 = 0;
                    seen = t + k;
                    cur = t;
                    end = hi - t < k ? hi : t + k;
                    empty = 0;
                    return true;
                }
                if (++empty >= kSegs) drained = true;
                seg = seg + 1 == kSegs ? 0u : seg + 1;
                away = true;
            }
            return false;
        }
        const uint32_t freem = ~busy & kSlotMask;
        if (drained) return false;
        if (freem == 0) {
            ++n_no_slot;
            return false;
        }
        uint32_t u = 0;
        if (lane == 0) u = (uint32_t)atomicAdd(ua.ctr, 1ull);
        u = __builtin_amdgcn_readfirstlane(u);
        if (u >= ua.n_units) {
            drained = true;
            return false;
        }
        const uint32_t k = fastdiv(u, ua.div_tiles), tile = u - k * ua.n_tiles;
        uint32_t s0, n;
        chunk_range(ua, k, &s0, &n);
        const uint32_t js = (uint32_t)__builtin_ctz(freem);
#pragma unroll
        for (uint32_t j = 0; j < kSlots; ++j) st_u[j] = j == js ? u : st_u[j];
        busy |= 1u << js;
        cur_slot = js;
        wait_t0 = 0;
        cur = 0;
        end = n * 64;
        cur_tile = tile;
        cur_s0 = s0;
        return true;
    }

    // Hands items to the lanes without a path (wave-uniform loop).  A lane handed item m of the
    // current unit gets pixel q = 64 * tile + m % 64 and sample s0 + m / 64; items of pixels past
    // the launch's last (a partial last tile) are skipped.  `fresh` marks lanes that start a path.
    __device__ __forceinline__ void refill(bool& active, bool& fresh, uint32_t& myslot, uint32_t& mi, uint32_t& q,
                                           uint32_t& s, uint32_t lane) {
        uint64_t needy = __ballot(!active);
        while (needy != 0) {
            if (cur >= end && !claim(lane)) break;
            const uint32_t avail = end - cur;
            const uint32_t want = (uint32_t)__popcll(needy);
            const uint32_t take = avail < want ? avail : want;
            if (!active) {
                const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(needy >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)needy, 0u));
                if (rk < take) {
                    const uint32_t m = cur + rk;
                    if constexpr (kDirect) {
                        s = fastdiv(m, ua.div_p);
                        q = m - s * ua.P;
                        mi = m;
                        myslot = 0;
                        active = true;
                        fresh = true;
                    } else {
                        const uint32_t pq = cur_tile * 64 + (m & 63);
                        if (pq < ua.P) {
                            myslot = cur_slot;
                            q = pq;
                            s = cur_s0 + (m >> 6);
                            mi = m;
                            active = true;
                            fresh = true;
                        }
                    }
                }
            }
            cur += take;
            needy = __ballot(!active);
        }
    }

    // The color of a finished item goes to its unit's ring slot: [slot][m][3] (direct mode:
    // samples[m = s * P + q]).
    __device__ __forceinline__ void store(uint32_t slot, uint32_t m, double x, double y, double z) const {
        if constexpr (kBounds) {
            if (!bounds_ok(kDirect ? m < ua.n_units : slot < kSlots && m < kUnitS * 64, ua.ctr)) return;
        }
        double* d = kDirect ? ua.samples + 3 * (size_t)m : ring + (size_t)slot * kRingSlotDoubles + 3 * m;
        d[0] = x;
        d[1] = y;
        d[2] = z;
    }

    // Slots whose unit has been handed out completely and has no item in flight in any lane.
    __device__ __forceinline__ uint32_t ready_mask(bool active, uint32_t myslot) const {
        if constexpr (kDirect) return 0;
        uint32_t ready = 0;
#pragma unroll
        for (uint32_t j = 0; j < kSlots; ++j) {
            const bool issued = j != cur_slot || cur >= end;
            if (((busy >> j) & 1u) && issued && __ballot(active && myslot == j) == 0) ready |= 1u << j;
        }
        return ready;
    }

    __device__ __forceinline__ bool finalize_one(uint32_t ready, uint32_t lane) {
        if (kDirect || ready == 0) return false;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's ring stores have completed
        while (ready) {
            const uint32_t j = (uint32_t)__builtin_ctz(ready);
            ready &= ready - 1;
            uint32_t u = st_u[0];
#pragma unroll
            for (uint32_t jj = 1; jj < kSlots; ++jj) u = jj == j ? st_u[jj] : u;
            const uint32_t k = fastdiv(u, ua.div_tiles), tile = u - k * ua.n_tiles;
            if constexpr (kBounds) {
                if (!bounds_ok(tile < ua.n_tiles && k < ua.n_chunks, ua.ctr)) {
                    busy &= ~(1u << j);
                    return true;
                }
            }
            uint32_t f = k;
            if (k) {  // chunk 0 has no predecessor
                if (lane == 0) f = __hip_atomic_load((gu32*)ua.flags + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                f = __builtin_amdgcn_readfirstlane(f);
            }
            if (f != k) {  // the previous chunk of this tile is not finalised yet
                ++n_dep_wait;
                continue;
            }
            // Ordering of the hand-off, pinned explicitly rather than by agent-scope acquire/release
            // (gfx950: buffer_inv sc1, an invalidate of this CU's L1 (~1.7 us), and buffer_wbl2 sc1,
            // a write-back of the XCD L2's dirty lines, per hand-off; MI355X_MICROARCH.md fence
            // table).  Hardware: the sums loads below are issued
            // only after the flag's value has returned (readfirstlane + the scalar branch above wait
            // for it), and they are sc1 loads; the producer drains its sc1 sum stores
            // (s_waitcnt vmcnt(0)) before its flag store.  Compiler: the fence and the "memory"
            // clobber keep every load below this point.
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            asm volatile("" ::: "memory");
            RTK_MARK("fin_work");
            uint32_t s0, n;
            chunk_range(ua, k, &s0, &n);
            const uint32_t q = tile * 64 + lane;
            if (q < ua.P) {
                double x = 0.0, y = 0.0, z = 0.0;
                if (k) {
                    x = ld_wt(ua.sums + 3 * (size_t)q + 0);
                    y = ld_wt(ua.sums + 3 * (size_t)q + 1);
                    z = ld_wt(ua.sums + 3 * (size_t)q + 2);
                }
                // the ring is this wave's own, written by this CU: plain loads behind the drain
                const double* rs = ring + (size_t)j * kRingSlotDoubles + 3 * lane;
#pragma unroll 8
                for (uint32_t t = 0; t < n; ++t) {
                    x = x + rs[0];
                    y = y + rs[1];
                    z = z + rs[2];
                    rs += 3 * 64;
                }
                if (k + 1 < ua.n_chunks) {
                    st_wt(ua.sums + 3 * (size_t)q + 0, x);
                    st_wt(ua.sums + 3 * (size_t)q + 1, y);
                    st_wt(ua.sums + 3 * (size_t)q + 2, z);
                } else if (ua.out_format == 0) {
                    double* o = (double*)ua.out + 3 * (size_t)q;
                    o[0] = x * ua.scale;  // avgColor = pixelColor * pixelSamplesScale
                    o[1] = y * ua.scale;
                    o[2] = z * ua.scale;
                } else {
                    uint8_t* o = (uint8_t*)ua.out + 3 * (size_t)q;
                    o[0] = to_byte(x * ua.scale);
                    o[1] = to_byte(y * ua.scale);
                    o[2] = to_byte(z * ua.scale);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the flag
            if (lane == 0) {
                if (k + 1 < ua.n_chunks)
                    __hip_atomic_store((gu32*)ua.flags + tile, k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            busy &= ~(1u << j);
            wait_t0 = 0;
            return true;
        }
        return false;
    }

    // Nothing to trace in this wave: wait for a dependency (bounded).  False: give up (reported).
    __device__ __forceinline__ bool wait(uint32_t lane) {
        ++spins;
        const uint32_t now = wait_clock() | 1u;
        if (wait_t0 == 0) {
            wait_t0 = now;
        } else if (now - wait_t0 > ua.stall_ticks) {
            if (lane == 0) atomicOr(ua.ctr + kErrWord, kErrStall);
            failed = true;
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
        return true;
    }
};

}  // namespace rtk

// rt_units.h — device side of the unit scheduler and the ordered in-kernel accumulation
// (rt_kernel.h "Work units").  Shared by the parity kernels (rt_kernel.hip) and the
// fast kernel (rt_kernel_fast.hip).
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

#ifndef RTZIG_CLAIM_MAX
#define RTZIG_CLAIM_MAX 2048
#endif
#ifndef RTZIG_FOLD_UNROLL
#define RTZIG_FOLD_UNROLL 4
#endif

namespace rtk {

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;
constexpr uint32_t kDirectClaimMax = RTZIG_CLAIM_MAX;  // direct mode: largest guided claim (items)
constexpr int kAuxSc1 = 16;  // buffer-op cache policy bits: sc1 (cdna_hip_programming.md Guideline 16 R1)

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
// whenever this wave claims or finalises a unit; past kStallTicks the wave reports it in the
// sticky ctr[kErrWord] and gives up (the host returns RT_ERR_HIP).  The wait's state is ONE SGPR,
// as the round-2 sleep counter was: a global-progress bound (every finalisation counted, the count
// and the clock carried by the waiting wave) cost 1.1-1.7% of the frame through SGPR spills into
// the walk's VGPRs.  The clock is kept as its low 32 bits (wrapping differences are exact below
// 2^32 ticks = 42.9 s).
__device__ __forceinline__ uint64_t realtime() { return __builtin_amdgcn_s_memrealtime(); }

// A field of the kernel's by-value UnitArgs read from the kernarg segment by a scalar load where it
// is used (`off`: the field's byte offset in the segment — UnitArgs's offset there, kUaOff, plus
// the field's).  Direct mode's fold and count code reads ~20 dwords of UnitArgs; left to the
// compiler they are loaded once and held in SGPRs across the persistent loop, which pushed the
// direct BVH kernel past the SGPR file (62 spilled to VGPR lanes, 137 VGPRs: 3 waves per SIMD).
// Volatile, so the loads stay at the use.  (Taking the address of the argument instead copies
// the whole struct to scratch.)
template <typename T>
__device__ __forceinline__ T karg_at(uint32_t off) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "karg: 4- or 8-byte fields");
    const uint64_t kp = (uint64_t)__builtin_amdgcn_kernarg_segment_ptr();
    if constexpr (sizeof(T) == 4) {
        uint32_t v;
        asm volatile("s_load_dword %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(kp), "i"(off));
        return __builtin_bit_cast(T, v);
    } else {
        uint64_t v;
        asm volatile("s_load_dwordx2 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(kp), "i"(off));
        return __builtin_bit_cast(T, v);
    }
}
#define RTK_KA(f) karg_at<decltype(UnitArgs::f)>(kUaOff + (uint32_t)offsetof(UnitArgs, f))

// Wave-uniform scheduler state (every member is the same in all 64 lanes).  kDirect: direct mode
// (rt_kernel.h): guided claims of flat items t = s * P + q, fold group after fold group; per-group
// done counts; the wave's own fold units.  No slots, no ring.  Direct mode keeps its small fields
// packed and recomputes what it can (group bounds, fold unit coordinates, the launch's waves): the
// BVH kernel sits at 127 of the 128 VGPRs that 4 waves per SIMD allow, and every SGPR past the
// file spills into VGPR lanes (unpacked, this state took the direct kernel to 143 VGPRs).
template <bool kDirect, uint32_t kUaOff>
struct UnitSched {
    const UnitArgs& ua;
    double* ring;                    // this wave's ring: kSlots x [kUnitS * 64][3]
    uint32_t busy = 0;               // slots holding a unit that is not finalised yet
    uint32_t cur_slot = 0, cur = 0, end = 0;  // the slot being handed out: items [cur, end)
    uint32_t cur_tile = 0, cur_s0 = 0;
    uint32_t st_u[kSlots];           // unit id held by each slot
    uint32_t spins = 0;              // sleeps in all (diagnostics)
    uint32_t wait_t0 = 0;            // realtime (low word, | 1) when the current wait began (0: not waiting)
    uint32_t seen = 0;               // direct mode: item position after this wave's last claim
    // direct mode, packed claim state: group claimed from (bits 0-4), segment (8-10), segments found
    // empty (12-15), claiming away from home (16), group of the items [cur, end) (20-24)
    uint32_t cs = 0;
    // direct mode: unflushed finished-item counts of groups a_base (a0) and a_base + 1 (a1); the
    // next own fold unit fu = g * n_tiles + tile; fs: a_base (bits 0-4), fold unit seen ready by a
    // poll (8), drained-wave poll cadence (12-13)
    uint32_t a0 = 0, a1 = 0, fu = 0, fs = 0;
    uint32_t n_dep_wait = 0;   // diagnostics (instrumented build): finalisations deferred on a flag
    uint32_t n_no_slot = 0;    // ... refills stopped for want of a free slot
    bool drained = false;            // the claim counter is exhausted
    bool failed = false;             // stall bound reached (reported in ctr[kErrWord])

    __device__ UnitSched(const UnitArgs& a, uint32_t wave) : ua(a), ring(a.ring + (size_t)wave * kRingWaveDoubles) {
        if constexpr (kDirect) {
            cs = home() << 8;
            seen = seg_lo(0, home());
            fu = __builtin_amdgcn_readfirstlane(wave);  // uniform (the compiler cannot tell: threadIdx.x / 64)
        }
#pragma unroll
        for (uint32_t j = 0; j < kSlots; ++j) st_u[j] = 0;
    }
    // ---- direct mode's packed fields and recomputed values ---------------------------------------
    __device__ __forceinline__ uint32_t grp() const { return cs & 31u; }
    __device__ __forceinline__ uint32_t seg() const { return (cs >> 8) & 7u; }
    __device__ __forceinline__ uint32_t empty() const { return (cs >> 12) & 15u; }
    __device__ __forceinline__ bool away() const { return (cs >> 16) & 1u; }
    __device__ __forceinline__ uint32_t cur_grp() const { return (cs >> 20) & 31u; }
    __device__ __forceinline__ uint32_t a_base() const { return fs & 31u; }
    __device__ __forceinline__ bool fready() const { return (fs >> 8) & 1u; }
    __device__ __forceinline__ uint32_t home() const { return blockIdx.x % kSegs; }
    __device__ __forceinline__ uint32_t waves() const { return gridDim.x * (blockDim.x / 64); }
    __device__ __forceinline__ uint32_t n_fold() const { return RTK_KA(n_chunks) * RTK_KA(n_tiles); }  // < 2^32 (host check)
    __device__ __forceinline__ uint32_t fg() const { return fastdiv(fu, RTK_KA(div_tiles)); }
    __device__ __forceinline__ uint32_t s0_of(uint32_t g) const { return RTK_KA(chunk_s0)[g]; }  // fold group table
    // first item of queue segment j of group g: fold group g covers the items t in
    // [chunk_s0[g] * P, chunk_s0[g + 1] * P), its kSegs segments split it evenly
    __device__ __forceinline__ uint32_t seg_lo(uint32_t g, uint32_t j) const {
        const uint32_t P = RTK_KA(P), lo = s0_of(g) * P, n = s0_of(g + 1) * P - lo;
        return lo + (uint32_t)((uint64_t)n * j / kSegs);
    }
    __device__ __forceinline__ bool can_claim() const { return !drained && (kDirect || (~busy & kSlotMask) != 0); }
    // nothing left for this wave: ring mode, every unit claimed and finalised; direct mode, every item
    // claimed, every finished count flushed (count_done, at the end of an iteration: a wave that
    // drains at the top of one still has to run that iteration's flush before it may leave, or its
    // last group's count stays short and that group's folds wait forever) and every fold unit it
    // owns done
    __device__ __forceinline__ bool finished() const {
#ifdef RTZIG_ABL_NOFOLD  // timing ablation only (no output)
        return kDirect ? drained && a_base() >= RTK_KA(n_chunks) : busy == 0 && drained;
#endif
        return kDirect ? drained && a_base() >= RTK_KA(n_chunks) && fu >= n_fold() : busy == 0 && drained;
    }

    // Claims the next unit into a free slot and makes it the one handed out; false if there is no
    // free slot or no unit left.
    __device__ __forceinline__ bool claim(uint32_t lane) {
        if constexpr (kDirect) {
            // the fold unit's poll rides on the claim: its load is in flight with the claim's atomic
#ifdef RTZIG_ABL_NOFOLD
            const bool want = false;
#else
            const bool want = !fready() && fu < n_fold();
#endif
            uint32_t pv = 0;
            if (want) pv = poll_issue(lane);
            const bool got = claim_direct(lane);
            if (want && poll_check(pv)) fs |= 1u << 8;
            return got;
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
    __device__ __forceinline__ bool claim_direct(uint32_t lane) {
        while (!drained) {
            const uint32_t g = grp(), j = seg();
            const uint32_t lo = seg_lo(g, j), hi = seg_lo(g, j + 1);
            // guided in the home segment: 1/8 of an even share of what it has left (as this wave
            // last saw it; its kSegs-th of the waves claim there), 64..2048 items in whole multiples
            // of 64; elsewhere 64
            const uint32_t left = hi > seen ? hi - seen : 0u;
            uint32_t k = away() ? 64u : left / waves();
            k = k < 64u ? 64u : (k > kDirectClaimMax ? kDirectClaimMax : k & ~63u);
            uint32_t t = 0;
            if (lane == 0) t = (uint32_t)atomicAdd(RTK_KA(ctr) + kCtrStride * (g * kSegs + j), (unsigned long long)k);
            t = lo + __builtin_amdgcn_readfirstlane(t);
            if (t < hi) {
                wait_t0 = 0;
                seen = t + k;
                cur = t;
                end = hi - t < k ? hi : t + k;
                cs = (cs & ~((15u << 12) | (31u << 20))) | (g << 20);  // empty = 0, cur_grp = g
                return true;
            }
            if (empty() + 1 >= kSegs) {  // every segment of this group is empty: the next group
                cs = (g + 1) | (home() << 8) | (cs & (31u << 20));
                if (g + 1 >= RTK_KA(n_chunks)) {
                    drained = true;
                    break;
                }
                seen = seg_lo(g + 1, home());
                continue;
            }
            cs = ((cs & ~(7u << 8)) + (1u << 12) + (((j + 1) & 7u) << 8)) | (1u << 16);  // next segment, away
        }
        return false;
    }

    // Hands items to the lanes without a path (wave-uniform loop).  A lane handed item m of the
    // current unit gets pixel q = 64 * tile + m % 64 and sample s0 + m / 64; items of pixels past
    // the launch's last (a partial last tile) are skipped.  `fresh` marks lanes that start a path.
    // Direct mode: item t gives s = t / P, q = t % P, the store index mi = s * Ps + q and, in
    // `myslot` (no slots in direct mode), the lane's fold group.
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
                        mi = s * ua.Ps + q;
                        myslot = cur_grp();
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
    // samples[m = s * Ps + q], written through: another wave, on any XCD, folds it).
    __device__ __forceinline__ void store(uint32_t slot, uint32_t m, double x, double y, double z) const {
        if constexpr (kDirect) {
            double* d = RTK_KA(samples) + 3 * (size_t)m;
#ifdef RTZIG_ABL_PLAINST  // timing ablation only (no hand-off guarantee)
            d[0] = x;
            d[1] = y;
            d[2] = z;
#else
            st_wt(d + 0, x);
            st_wt(d + 1, y);
            st_wt(d + 2, z);
#endif
        } else {
            double* d = ring + (size_t)slot * kRingSlotDoubles + 3 * m;
            d[0] = x;
            d[1] = y;
            d[2] = z;
        }
    }

    // ---- direct mode: group done counts and folds ------------------------------------------------
    __device__ __forceinline__ gu32* done_word(uint32_t g) const {
        return (gu32*)(RTK_KA(ctr) + kCtrStride * (kDoneBase + g));  // the low word of a zeroed u64
    }
    // Adds n finished items of group g to its done counter, after this wave's stores of them have
    // completed (sc1 stores, drained: the ring's hand-off recipe, with a counter for the flag).
    __device__ __forceinline__ void flush(uint32_t g, uint32_t n, uint32_t lane) const {
        if (n == 0) return;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add(done_word(g), n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // Called after this iteration's stores (`done`: lanes that stored; `active`: lanes still on a
    // path; `gi`: a lane's group).  Counts are kept per wave for groups a_base and a_base + 1 (a
    // wave's lanes hold items of at most two groups but in odd cases: those flush at once) and
    // flushed when the wave can hold no more items of a_base: it claims from a later group (claims
    // never go back; drained: past the last group) and no lane is on a path of it.
    __device__ __forceinline__ void count_done(bool done, bool active, uint32_t gi, uint32_t lane) {
        if constexpr (kDirect) {
            uint64_t dm = __ballot(done);
            while (dm != 0) {
                const uint32_t g = __builtin_amdgcn_readlane(gi, (uint32_t)__builtin_ctzll(dm));
                const uint64_t same = __ballot(done && gi == g);
                dm &= ~same;
                const uint32_t n = (uint32_t)__popcll(same);
                if (g == a_base()) a0 += n;
                else if (g == a_base() + 1) a1 += n;
                else flush(g, n, lane);
            }
            const uint32_t claimed = drained ? 31u : grp();  // groups below this one get no more items
            while (a_base() < claimed && a_base() < RTK_KA(n_chunks) && __ballot(active && gi == a_base()) == 0) {
                flush(a_base(), a0, lane);
                ++fs;  // a_base + 1
                a0 = a1;
                a1 = 0;
            }
        }
    }
    // Polls fold unit fu = (g, tile): lane 0 loads group g's done counter, lane 1 the tile's flag
    // (sc1 loads); ready when every item of the group has been counted and the tile's groups
    // 0..g-1 are folded (flag == g).  Both conditions only ever become true.
    __device__ __forceinline__ uint32_t poll_issue(uint32_t lane) const {
        const uint32_t g = fg(), tile = fu - g * RTK_KA(n_tiles);
        uint32_t v = 0;
        if (lane < 2)
            v = __hip_atomic_load(lane == 0 ? done_word(g) : (gu32*)RTK_KA(flags) + tile, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
        return v;
    }
    __device__ __forceinline__ bool poll_check(uint32_t v) const {
        const uint32_t g = fg();
        const uint32_t d = __builtin_amdgcn_readlane(v, 0), f = __builtin_amdgcn_readlane(v, 1);
        return d == (s0_of(g + 1) - s0_of(g)) * RTK_KA(P) && f == g;
    }
    // Top of every iteration: folds this wave's next fold unit if a poll has seen it ready.  Polls
    // ride on the claims (claim()); a drained wave, which claims no more, polls here: every
    // iteration when it has nothing to trace, every 4th while it still traces (a poll waits for its
    // loads).  True if it folded.
    __device__ __forceinline__ bool fold_step(bool active, uint32_t lane) {
        if constexpr (!kDirect) return false;
#ifdef RTZIG_ABL_NOFOLD
        return false;
#endif
        if (fu >= n_fold()) return false;
        if (!fready() && drained) {
            fs += 1u << 12;
            if ((__ballot(active) == 0 || ((fs >> 12) & 3u) == 0) && poll_check(poll_issue(lane))) fs |= 1u << 8;
        }
        if (!fready()) return false;
        fold(lane);
        fs &= ~(1u << 8);
        wait_t0 = 0;
        fu += waves();
        return true;
    }
    // Fold unit fu = (g, tile): lane l adds group g's colors of pixel q = 64 * tile + l, in sample
    // order, to the pixel's running sum (camera.zig:133-136's +=, from pixelColor = 0 at group 0),
    // and stores it for group g + 1 (sc1, drained, then the tile's flag) or, for the last group,
    // scales it (:137) and writes the framebuffer (linear f64 or the fused Color.toRgb bytes).
    // Every line read here holds only bytes of this (group, tile): layers start on 128-B lines
    // (Ps), a tile's 64 pixels are 12 whole lines, and each was written through before its
    // group's count was flushed; the loads are sc1, issued only after the polled values returned
    // (readlane + the scalar branch in fold_step), kept below it by the fence and the clobber.
    __device__ __forceinline__ void fold(uint32_t lane) const {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        asm volatile("" ::: "memory");
        const uint32_t g = fg(), tile = fu - g * RTK_KA(n_tiles);
        // wave-uniform by construction; readfirstlane tells the compiler (the buffer descriptor
        // below must be built from SGPRs, or every load becomes a waterfall loop)
        const uint32_t s0 = __builtin_amdgcn_readfirstlane(s0_of(g)), s1 = __builtin_amdgcn_readfirstlane(s0_of(g + 1));
        const bool last = g + 1 == RTK_KA(n_chunks);
        const uint32_t q = tile * 64 + lane;
        if (q < RTK_KA(P)) {
            double* const sums = RTK_KA(sums);
            double x = 0.0, y = 0.0, z = 0.0;
            if (g) {
                x = ld_wt(sums + 3 * (size_t)q + 0);
                y = ld_wt(sums + 3 * (size_t)q + 1);
                z = ld_wt(sums + 3 * (size_t)q + 2);
            }
            // the group's colors of this tile through a buffer descriptor (wave-uniform base: the
            // tile's first pixel in layer s0; < 2 GiB, host check): sc1 buffer loads, which the
            // compiler keeps in flight together (it serialises atomic sc1 loads, one wait each)
            const uint32_t Ps = RTK_KA(Ps);
            // (readfirstlane returns int: each half goes through uint32_t, or the low half's bit 31
            // would sign-extend into the high half)
            const uint64_t base = (uint64_t)(RTK_KA(samples) + 3 * ((size_t)s0 * Ps + tile * 64));
            const uint32_t base_hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
            const uint32_t base_lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)base);
            // records: from the tile's first pixel in layer s0 to the end of layer s1 - 1
            const uint32_t bytes = (uint32_t)__builtin_amdgcn_readfirstlane(((s1 - s0) * Ps - tile * 64) * 24u);
            const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)base_hi << 32) | base_lo), (short)0,
                                                              (int)bytes, 0x00020000);
            uint32_t off = lane * 24u;
            const uint32_t stride = Ps * 24u;
            // batches of kFoldBatch layers: every load of a batch is issued before the first add
            constexpr uint32_t B = RTZIG_FOLD_UNROLL;
            uint32_t s = s0;
            for (; s + B <= s1; s += B) {
                uint64_t v[B][3];
#pragma unroll
                for (uint32_t b = 0; b < B; ++b) {
#pragma unroll
                    for (uint32_t c = 0; c < 3; ++c)
                        v[b][c] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(rs, off + b * stride + 8 * c, 0, kAuxSc1));
                }
#pragma unroll
                for (uint32_t b = 0; b < B; ++b) {
                    x = x + __builtin_bit_cast(double, v[b][0]);
                    y = y + __builtin_bit_cast(double, v[b][1]);
                    z = z + __builtin_bit_cast(double, v[b][2]);
                }
                off += B * stride;
            }
            for (; s < s1; ++s) {
                x = x + __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, kAuxSc1));
                y = y + __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, off + 8, 0, kAuxSc1));
                z = z + __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, off + 16, 0, kAuxSc1));
                off += stride;
            }
            if (!last) {
                st_wt(sums + 3 * (size_t)q + 0, x);
                st_wt(sums + 3 * (size_t)q + 1, y);
                st_wt(sums + 3 * (size_t)q + 2, z);
            } else {
                const double scale = RTK_KA(scale);
                if (RTK_KA(out_format) == 0) {
                    double* o = (double*)RTK_KA(out) + 3 * (size_t)q;
                    o[0] = x * scale;  // avgColor = pixelColor * pixelSamplesScale
                    o[1] = y * scale;
                    o[2] = z * scale;
                } else {
                    uint8_t* o = (uint8_t*)RTK_KA(out) + 3 * (size_t)q;
                    o[0] = to_byte(x * scale);
                    o[1] = to_byte(y * scale);
                    o[2] = to_byte(z * scale);
                }
            }
        }
        if (!last) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the sums are written through before the flag
            if (lane == 0) __hip_atomic_store((gu32*)RTK_KA(flags) + tile, g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
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
            // (which gfx950 implements as buffer_inv sc1 / buffer_wbl2 sc1: an invalidate or a
            // write-back of the whole L2 per hand-off).  Hardware: the sums loads below are issued
            // only after the flag's value has returned (readfirstlane + the scalar branch above wait
            // for it), and they are sc1 loads; the producer drains its sc1 sum stores
            // (s_waitcnt vmcnt(0)) before its flag store.  Compiler: the fence and the "memory"
            // clobber keep every load below this point.
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            asm volatile("" ::: "memory");
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
        const uint32_t now = (uint32_t)realtime() | 1u;
        if (wait_t0 == 0) {
            wait_t0 = now;
        } else if (now - wait_t0 > ua.stall_ticks) {
            if (lane == 0) atomicOr(ua.ctr + kErrWord, 1ull);
            failed = true;
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
        return true;
    }
};

}  // namespace rtk

// rt_device.h — device-side math, RNG and material scatter for the MI355X path tracer (gfx950).
//
// Arithmetic contract (DESIGN.md "Parity"): every f64 operation rounds where the reference's does.
// The reference is Zig 0.14 in strict float mode: no FMA contraction, @reduce(.Add) evaluated as
// (x+y)+z, correctly rounded @sqrt and division.  hipcc defaults to -ffp-contract=fast for HIP, so
// this header pins contraction off with a pragma in addition to the build flag.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

// Region markers (tools/region_table.py): -DRTZIG_MARKS=1 builds emit an assembly comment ";@R <name>"
// where each region of the path loop starts (and "rare" on the slow paths behind wave-uniform
// tests), so the per-region instruction table can attribute the kernel's basic blocks.  Shipped
// builds emit nothing.
#ifndef RTZIG_MARKS
#define RTZIG_MARKS 0
#endif
#if RTZIG_MARKS
#define RTK_MARK(x) asm volatile(";@R " x)
#else
#define RTK_MARK(x) ((void)0)
#endif

namespace rtk {

// ------------------------------------------------------------------------------------------------
// Vec3 (vec.zig:5-136)
// ------------------------------------------------------------------------------------------------
struct v3 {
    double x, y, z;
};

__device__ __forceinline__ v3 mk(double x, double y, double z) { return v3{x, y, z}; }
__device__ __forceinline__ v3 operator+(v3 a, v3 b) { return v3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ v3 operator-(v3 a, v3 b) { return v3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ v3 operator*(v3 a, v3 b) { return v3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ v3 operator-(v3 a) { return v3{-a.x, -a.y, -a.z}; }
// Vec.mulScalar (vec.zig:35)
__device__ __forceinline__ v3 muls(v3 a, double s) { return v3{a.x * s, a.y * s, a.z * s}; }
// Vec.dot / lenSquared: @reduce(.Add) is the ordered (x+y)+z (vec.zig:51,114)
__device__ __forceinline__ double dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ double len_sq(v3 a) { return (a.x * a.x + a.y * a.y) + a.z * a.z; }
// sqrt(x) bit-identical to the compiler's correctly rounded f64 sqrt for x in [2^-767, 2^1023]:
// that sequence scales x by 2^256 only below 2^-767 and patches only +-0 / +inf / NaN
// (v_cmp_class); in between both are identity, and what remains is this rsq + Newton sequence.
__device__ __forceinline__ double sqrt_normal(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    g = __builtin_fma(__builtin_fma(-g, g, x), h, g);
    return __builtin_fma(__builtin_fma(-g, g, x), h, g);
}

struct SharedRcp {
    double l, y;
    __device__ __forceinline__ explicit SharedRcp(double den) : l(den) {
        const double y0 = __builtin_amdgcn_rcp(den);
        const double y1 = __builtin_fma(y0, __builtin_fma(-den, y0, 1.0), y0);
        y = __builtin_fma(y1, __builtin_fma(-den, y1, 1.0), y1);
    }
    __device__ __forceinline__ double div(double x) const {
        const double q0 = x * y;
        return __builtin_fma(__builtin_fma(-l, q0, x), y, q0);
    }
};

// x / a for the two roots of every sphere test of one ray (sphere.zig:38-40), a = |dir|^2: the
// reciprocal part of the division is computed once per ray (SharedRcp); each quotient then takes
// the division's last three steps, bit-identical to the correctly rounded x / a when no operand
// needs scaling: a in [2^-100, 2^100] (checked per ray) and |x| in [2^-600, 2^600) (biased
// exponent in [423, 1623), checked per division on the high word shifted past the sign).  Then
// the quotient lies in [2^-700, 2^700] and v_div_scale / v_div_fixup are the identity.  Other
// lanes take the compiler's full division.
struct RayDiv {
    double a, y;
    uint64_t bad;  // wave mask of the lanes whose `a` is out of range (a ballot: one SGPR pair)
    __device__ __forceinline__ explicit RayDiv(double den) : a(den) {
        bad = __ballot(!(den >= 0x1p-100 && den <= 0x1p100));
        y = SharedRcp(den).y;
    }
    __device__ __forceinline__ double div(double x) const {
        const uint32_t hi2 = (uint32_t)(__builtin_bit_cast(uint64_t, x) >> 32) << 1;
        const double q0 = x * y;
        double q = __builtin_fma(__builtin_fma(-a, q0, x), y, q0);
        const bool far = !(hi2 - (423u << 21) < (1200u << 21));
        // rare: wave-uniform test, see uniform().  The per-ray part is the mask `bad`, OR-ed on the
        // scalar unit; folding it into the per-lane bool made the compiler materialize that bool
        // with two VALU ops per division.  (Round 4: the range test as two f64 |x| compares into
        // lane masks plus an inverse ballot cut walk_setup's static VALU cycles by 11% and made the
        // frame 1.5% slower: a longer scalar chain ahead of the branch, profiles/r04_range_ab/.)
        if (__builtin_expect((__ballot(far) | bad) != 0, 0)) {
            RTK_MARK("rare");
            if (far || ((bad >> lane()) & 1)) q = x / a;
        }
        return q;
    }
    __device__ __forceinline__ static uint32_t lane() {
        return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
    }
};

// __builtin_sqrt(x) with the unscaled sequence when x is in [2^-767, inf) (the high word minus
// that of 2^-767 is below 0x7ff00000 - 0x10000000 as an unsigned number); other lanes (0, tiny,
// inf, NaN, negative) take the compiler's full sequence.  Every lane computes the short form, and
// the rare lanes are redone behind a wave-uniform test, so the common case has no exec-mask branch.
__device__ __forceinline__ bool sqrt_in_range(double x) {
    return (uint32_t)(__builtin_bit_cast(uint64_t, x) >> 32) - 0x10000000u < 0x6ff00000u;
}
__device__ __forceinline__ double sqrt_g(double x) {
    double r = sqrt_normal(x);
    const bool slow = !sqrt_in_range(x);
    if (__builtin_expect(__ballot(slow) != 0, 0)) {
        RTK_MARK("rare");
        if (slow) r = __builtin_sqrt(x);
    }
    return r;
}

// Vec.unit = divScalar(v, len) = v * (1/len) (vec.zig:39-45,126).  For |v|^2 in [2^-767, inf),
// len is in [2^-384, 2^512]: 1/len needs no scaling, so it is the Newton reciprocal of SharedRcp
// followed by the division's last two steps with numerator 1 (q0 = y, r = fma(-len, y, 1),
// q = fma(r, y, y)) — the same bits as the correctly rounded 1.0 / len.
__device__ __forceinline__ v3 unit(v3 a) {
    const double ls = len_sq(a);
    const double len = sqrt_normal(ls);
    const double y = SharedRcp(len).y;
    double inv = __builtin_fma(__builtin_fma(-len, y, 1.0), y, y);
    const bool slow = !sqrt_in_range(ls);
    if (__builtin_expect(__ballot(slow) != 0, 0)) {  // rare: wave-uniform test, see sqrt_g
        RTK_MARK("rare");
        if (slow) inv = 1.0 / __builtin_sqrt(ls);
    }
    return muls(a, inv);
}
// Vec.nearZero: all(v < 1e-8) with no abs (vec.zig:26-29)
__device__ __forceinline__ bool near_zero(v3 v) { return v.x < 1e-8 && v.y < 1e-8 && v.z < 1e-8; }
// Vec.reflect = v - (n * dot(v,n)) * 2 (vec.zig:103-105)
__device__ __forceinline__ v3 reflect(v3 v, v3 n) { return v - muls(muls(n, dot(v, n)), 2.0); }
// Vec.refract (vec.zig:107-112)
__device__ __forceinline__ v3 refract(v3 v, v3 n, double eta) {
    const double cos_t = __builtin_fmin(dot(-v, n), 1.0);
    const v3 r_perp = muls(v + muls(n, cos_t), eta);
    const v3 r_par = muls(n, -sqrt_g(__builtin_fabs(1.0 - len_sq(r_perp))));
    return r_perp + r_par;
}

// ------------------------------------------------------------------------------------------------
// RNG.  The reference draws from ONE Xoshiro256++ stream (std.Random.DefaultPrng, Scene.zig:30).
// Here every (pixel, sample) owns a Xoshiro256++ stream seeded through SplitMix64 exactly like
// DefaultPrng.init, from the key rt_sample_key(seed, pixel, sample) — counter-based, so any
// partition of the image over lanes/GPUs draws the same numbers.
// ------------------------------------------------------------------------------------------------
// A/B knob for the draw's instruction forms (0: rounds 1-3; 1: the 64-bit shift `s1 << 17` as one
// v_lshlrev_b64 — config 4 -0.74%, rank 0 of 8 -0.77%; 2: also Random.float's bit select as
// v_bitop3_b32 instead of v_bfi_b32 — a further -0.2% on config 4, within noise, fewer issue cycles;
// all bit-identical, profiles/r04_rng_ab/)
#ifndef RTZIG_RNG_FORM
#define RTZIG_RNG_FORM 2
#endif
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
// rotl64 by a constant K as two v_alignbit_b32 (the compiler's form is a 64-bit shift, a 32-bit
// shift and an or): for K < 32 the high word is alignbit(hi, lo, 32 - K), the low word
// alignbit(lo, hi, 32 - K); K >= 32 swaps the words first.
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <int K>
__device__ __forceinline__ uint64_t rotl64c(uint64_t x) {
    static_assert(K > 0 && K < 64 && K != 32, "rotate");
    uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
    if constexpr (K > 32) {
        const uint32_t t = lo;
        lo = hi;
        hi = t;
    }
    constexpr uint32_t s = 32u - (uint32_t)(K & 31);
    const uint32_t nhi = __builtin_amdgcn_alignbit(hi, lo, s);
    const uint32_t nlo = __builtin_amdgcn_alignbit(lo, hi, s);
    // a register pair, not (hi << 32) | lo: the compiler turns that `or` into 64-bit adds
    return __builtin_bit_cast(uint64_t, u32x2{nlo, nhi});
}

// a ^ b ^ c of 64-bit words as two gfx950 v_bitop3_b32 (truth table 0x96 = 3-input parity); the
// compiler emits two v_xor_b32 per 64-bit xor and does not form this on its own.
__device__ __forceinline__ uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
    const uint32_t lo = xor3_32((uint32_t)a, (uint32_t)b, (uint32_t)c);
    const uint32_t hi = xor3_32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32));
    return __builtin_bit_cast(uint64_t, u32x2{lo, hi});
}

// SplitMix64.next (zig std/Random/SplitMix64.zig)
__device__ __forceinline__ uint64_t splitmix_next(uint64_t& s) {
    s += 0x9e3779b97f4a7c15ULL;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t sm_mix_hd(uint64_t x) {
    x += 0x9e3779b97f4a7c15ULL;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

struct Rng {
    uint64_t s0, s1, s2, s3;

    // DefaultPrng.init(key): Xoshiro256.seed via SplitMix64 (zig std/Random/Xoshiro256.zig)
    __device__ __forceinline__ void seed(uint64_t key) {
        uint64_t sm = key;
        s0 = splitmix_next(sm);
        s1 = splitmix_next(sm);
        s2 = splitmix_next(sm);
        s3 = splitmix_next(sm);
    }
    // Xoshiro256.next: s2 ^= s0; s3 ^= s1; s1 ^= s2; s0 ^= s3; s2 ^= t; s3 = rotl(s3, 45), with the
    // chained xors folded into 3-input ones (s1 ^ s2 ^ s0, s0 ^ s3 ^ s1, s2 ^ s0 ^ t): 8 bitwise
    // ops per draw instead of 12
    __device__ __forceinline__ uint64_t next() {
        const uint64_t r = rotl64c<23>(s0 + s3) + s0;
#if RTZIG_RNG_FORM >= 1
        // one v_lshlrev_b64 (2.1 SIMD cycles at 4 waves/SIMD): left alone the compiler splits the
        // shift into v_alignbit_b32 + v_lshlrev_b32 (3.1 + 3.0) for the 32-bit xors that consume it
        uint64_t t;
        asm("v_lshlrev_b64 %0, 17, %1" : "=v"(t) : "v"(s1));
#else
        const uint64_t t = s1 << 17;
#endif
        const uint64_t n1 = xor3_64(s1, s2, s0);
        const uint64_t n0 = xor3_64(s0, s3, s1);
        const uint64_t n2 = xor3_64(s2, s0, t);
        const uint64_t n3 = s3 ^ s1;
        s0 = n0;
        s1 = n1;
        s2 = n2;
        s3 = rotl64c<45>(n3);
        return r;
    }
    // Random.float(f64) (zig std/Random.zig): mantissa = low 52 bits, exponent from leading zeros;
    // >= 12 leading zeros (p = 1/4096) pulls further draws.
    // Fast path on 32-bit halves: fewer than 12 leading zeros <=> hi >= 2^20, and then the leading
    // one lies in hi, so lz = clz(hi) and the high word of the result is (hi & 0xfffff) | e << 20.
    __device__ __forceinline__ double uniform() {
        const uint64_t rnd = next();
        const uint32_t hi = (uint32_t)(rnd >> 32);
        // ohi = (hi & 0xfffff) | (1022 - lz) << 20: the exponent field e = 1022*2^20 - lz*2^20 by one
        // v_mad_i32_i24 (lz <= 11; -2^20 is a valid signed 24-bit factor), then one v_bfi_b32
        // (VOP3 takes no literals and one SGPR: the 1022 << 20 addend lives in a VGPR)
        uint32_t e, ohi;
        asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(e) : "v"((uint32_t)__builtin_clz(hi)), "s"(-(1 << 20)), "v"(1022u << 20));
#if RTZIG_RNG_FORM >= 2
        // the same bit select as v_bitop3_b32 (1.9 SIMD cycles against v_bfi_b32's 3.1): truth table
        // 0xe4 = S2 ? S0 : S1 per bit, the mask in S2 (the form LLVM emits for a variable mask)
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xe4" : "=v"(ohi) : "v"(hi), "v"(e), "s"(0xfffffu));
#else
        asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(ohi) : "s"(0xfffffu), "v"(hi), "v"(e));
#endif
        double res = __builtin_bit_cast(double, u32x2{(uint32_t)rnd, ohi});
        // >= 12 leading zeros (p = 2^-12 per draw): the fast result is computed for every lane and
        // the rare lanes are redone, behind a wave-uniform test so the common case has no
        // exec-mask branch
        if (__builtin_expect(__ballot(hi < (1u << 20)) != 0, 0)) {
            RTK_MARK("rare");
            if (hi < (1u << 20)) res = uniform_slow(rnd);
        }
        return res;
    }
    __device__ __forceinline__ double uniform_slow(uint64_t rnd) {  // p = 2^-12 per draw
        uint64_t lz = rnd ? (uint64_t)__builtin_clzll(rnd) : 64;
        if (lz >= 12) {
            lz = 12;
            for (;;) {
                const uint64_t w = next();
                const uint64_t add = w ? (uint64_t)__builtin_clzll(w) : 64;
                lz += add;
                if (add != 64) break;
                if (lz >= 1022) { lz = 1022; break; }
            }
        }
        const uint64_t bits = ((1022 - lz) << 52) | (rnd & ((1ULL << 52) - 1));
        return __builtin_bit_cast(double, bits);
    }
    // util.randomDoubleRange (util.zig:20-22)
    __device__ __forceinline__ double range(double mn, double mx) { return mn + (mx - mn) * uniform(); }
    // range(-1, 1): (1 - -1) * u = 2u is exact, so -1 + 2u has ONE rounding and fma(2, u, -1) gives
    // the same bits with one f64 op instead of two (u may be subnormal: 2u is still exact).
    __device__ __forceinline__ double range_pm1() { return __builtin_fma(2.0, uniform(), -1.0); }
};

// key(seed, pixel, sample) = mix(mix(seed) ^ (pixel << 32 | sample)); seed_mix = mix(seed) is
// hoisted to the host.  For a fixed seed the map (pixel, sample) -> key is a bijection.
__device__ __forceinline__ uint64_t sample_key(uint64_t seed_mix, uint64_t pixel, uint32_t sample) {
    return sm_mix_hd(seed_mix ^ ((pixel << 32) | (uint64_t)sample));
}

// std.math.pow(f64, x, 5) for x in [0, 2] (frexp + repeated squaring == x*((x*x)*(x*x)))
__device__ __forceinline__ double zig_pow5(double x) {
    if (x == 1.0) return 1.0;
    if (x == 0.0) return x;
    const double x2 = x * x;
    const double x4 = x2 * x2;
    return x * x4;
}

// Color.toRgb for one channel (color.zig:63-80): sqrt gamma, clamp [0, 0.999], trunc(256*x)
__device__ __forceinline__ uint8_t to_byte(double lin) {
    double g = lin > 0 ? __builtin_sqrt(lin) : 0.0;
    g = g < 0.0 ? 0.0 : (g > 0.999 ? 0.999 : g);
    return (uint8_t)(int)(256.0 * g);
}

}  // namespace rtk

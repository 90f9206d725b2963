// peak_rates.hip — event-timed VALU throughput on the MI355X, the peak the roofline divides by.
//
// Round 4 priced every opcode with s_memtime deltas (tools/valu_rates.hip) and found f64 fma at
// 2.12 SIMD cycles per wave64 instruction at 4 waves per SIMD — full rate, ≈146 TF/s — while the
// roofline divided by the 78.6 TF/s FP64 vector spec.  This harness settles it without trusting any
// in-kernel counter: every launch covers every CU with W waves per SIMD (W = 1, 2, 4, 8), each wave
// runs `iters` × 64 copies of one instruction over 8 independent register chains, and the rate is
//
//     ops/s = blocks × 4 waves × iters × 64 instructions × 64 lanes × ops per lane ÷ hipEvent time
//
// with ≥ 100 ms per launch.  Beside it, thread 0 of every block stamps s_memtime and
// s_memrealtime (100 MHz) around its loop: Δmemtime ÷ Δmemrealtime × 100 MHz is the in-kernel clock
// (MI355X_MICROARCH.md, DVFS item 6), and the SIMD cycles per wave-instruction follow from the wall
// time and that clock alone:  1024 SIMDs × clock × t ÷ wave-instructions.
//
// Operands are per-lane non-zero values kept finite (x = x·b + c with |b| < 1, x = x + b, x = x·b with
// b ≈ 1): zero operands raise the clock the chip holds (MI355X_MICROARCH.md, DVFS item 1).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/peak_rates.hip -o tools/bin/peak_rates
//   ./tools/bin/peak_rates > peak.json          (one JSON document)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                         \
        }                                                                                         \
    } while (0)

// 64 instructions per asm statement: 8 rounds over 8 independent chains.  ONE asm statement per
// loop iteration, so the compiler inserts no hazard s_nops inside the run.
#define IND8(INS) ".rept 8\n" INS("%0") INS("%1") INS("%2") INS("%3") INS("%4") INS("%5") INS("%6") INS("%7") ".endr\n"

// %8 = b, %9 = c (64-bit pairs for the f64 / packed forms), %10 = an SGPR-pair mask
#define I_FMA_F64(X) "v_fma_f64 " X ", " X ", %8, %9\n"
#define I_ADD_F64(X) "v_add_f64 " X ", " X ", %8\n"
#define I_MUL_F64(X) "v_mul_f64 " X ", " X ", %8\n"
#define I_FMA_F32(X) "v_fma_f32 " X ", " X ", %8, %9\n"
#define I_PK_FMA_F32(X) "v_pk_fma_f32 " X ", " X ", %8, %9\n"
#define I_ADD_U32(X) "v_add_u32 " X ", " X ", %8\n"
#define I_XOR(X) "v_xor_b32 " X ", " X ", %8\n"
#define I_ALIGNBIT(X) "v_alignbit_b32 " X ", " X ", %8, 9\n"
#define I_MAX3_F32(X) "v_max3_f32 " X ", " X ", %8, %9\n"
#define I_CNDMASK_S(X) "v_cndmask_b32_e64 " X ", " X ", %8, %10\n"
#define I_MAD_U64_U32(X) "v_mad_u64_u32 " X ", vcc, %8, %9, " X "\n"

// The full opcode table of round 4's s_memtime harness (tools/valu_rates.hip), re-measured here with
// the event-timed method: issue cost per wave64 instruction = 1024 SIMDs × in-kernel clock × t ÷
// wave-instructions, at 4 and 8 waves per SIMD (the SIMD is saturated from 2 waves on).
#define T_RSQ_F64(X) "v_rsq_f64 " X ", " X "\n"
#define T_LSHL_ADD_U64(X) "v_lshl_add_u64 " X ", " X ", 0, %8\n"
#define T_LSHR_B64(X) "v_lshrrev_b64 " X ", 7, " X "\n"
#define T_MUL_LO_U32(X) "v_mul_lo_u32 " X ", " X ", %8\n"
#define T_MUL_HI_U32(X) "v_mul_hi_u32 " X ", " X ", %8\n"
#define T_BITOP3(X) "v_bitop3_b32 " X ", " X ", %8, %9 bitop3:0x96\n"
#define T_FFBH(X) "v_ffbh_u32 " X ", " X "\n"
#define T_MAD_I32_I24(X) "v_mad_i32_i24 " X ", " X ", %8, %9\n"
#define T_CNDMASK_VCMP(X) "v_cmp_gt_u32 vcc, " X ", %8\nv_cndmask_b32 " X ", " X ", %9, vcc\n"
#define T_CMP_F32(X) "v_cmp_gt_f32 vcc, " X ", %8\n"
#define T_MOV(X) "v_mov_b32 " X ", %8\n"
#define T_MAX_F32(X) "v_max_f32 " X ", " X ", %8\n"
#define T_MED3_F32(X) "v_med3_f32 " X ", " X ", %8, %9\n"
#define T_LSHL_B32(X) "v_lshlrev_b32 " X ", 7, " X "\n"
#define T_BFI(X) "v_bfi_b32 " X ", %8, " X ", %9\n"
#define T_ADD3(X) "v_add3_u32 " X ", " X ", %8, %9\n"
#define T_LSHL_ADD_U32(X) "v_lshl_add_u32 " X ", " X ", 2, %8\n"
#define T_MBCNT(X) "v_mbcnt_lo_u32_b32 " X ", %8, " X "\n"
#define T_RCP_F32(X) "v_rcp_f32 " X ", " X "\n"
#define T_RCP_F64(X) "v_rcp_f64 " X ", " X "\n"
#define T_LDEXP_F64(X) "v_ldexp_f64 " X ", " X ", 1\n"
#define T_BFREV(X) "v_bfrev_b32 " X ", " X "\n"
#define T_AND_OR(X) "v_and_or_b32 " X ", " X ", %8, %9\n"
#define T_NOT(X) "v_not_b32 " X ", " X "\n"
#define T_ADD_CO(X) "v_add_co_u32 " X ", vcc, " X ", %8\n"
#define T_MOV_B64(X) "v_mov_b64 " X ", %8\n"
#define T_MAX_F64(X) "v_max_f64 " X ", " X ", %8\n"
#define T_CMP_F64(X) "v_cmp_lt_f64 vcc, " X ", %8\n"
#define T_CMP_U64(X) "v_cmp_gt_u64 vcc, " X ", %8\n"
#define T_LSHR_B32(X) "v_lshrrev_b32 " X ", 7, " X "\n"
#define T_AND_B32(X) "v_and_b32 " X ", " X ", %8\n"
#define T_LSHL_B64(X) "v_lshlrev_b64 " X ", 7, " X "\n"
#define T_MUL_F32(X) "v_mul_f32 " X ", " X ", %8\n"
#define T_SUB_U32(X) "v_sub_u32 " X ", " X ", %8\n"
#define T_MAX_I32(X) "v_max_i32 " X ", " X ", %8\n"
#define T_MIN_I32(X) "v_min_i32 " X ", " X ", %8\n"
#define T_MAX3_I32(X) "v_max3_i32 " X ", " X ", %8, %9\n"
#define T_MIN3_I32(X) "v_min3_i32 " X ", " X ", %8, %9\n"
#define T_MAX_U32(X) "v_max_u32 " X ", " X ", %8\n"
#define T_CMP_LE_I32(X) "v_cmp_le_i32 vcc, " X ", %8\n"
#define T_MAXIMUM3_F32(X) "v_maximum3_f32 " X ", " X ", %8, %9\n"
#define T_MIN_F32(X) "v_min_f32 " X ", " X ", %8\n"
#define T_SUB_F32(X) "v_sub_f32 " X ", " X ", %8\n"
#define T_PK_ADD_F32(X) "v_pk_add_f32 " X ", " X ", %8\n"
#define T_PK_MUL_F32(X) "v_pk_mul_f32 " X ", " X ", %8\n"
#define T_ASHR_I32(X) "v_ashrrev_i32 " X ", 31, " X "\n"
#define T_ALIGNBIT_SAME(X) "v_alignbit_b32 " X ", " X ", " X ", 9\n"
#define T_CVT_F32_F64(X) "v_cvt_f32_f64 " X ", %8\n"
#define T_ADD_F32(X) "v_add_f32 " X ", " X ", %8\n"
#define T_FMA_F32_SS(X) "v_fma_f32 " X ", " X ", %8, " X "\n"

// Operand forms (round 5): the event-timed table showed v_fma_f32 at 2.2 cycles with two distinct
// VGPR sources (x, b, x) and 4.2 with three (x, b, c), so an op's cost depends on its operands as
// well as its opcode; %11 is a uniform 32-bit SGPR value.
#define O_FMA_F32_S(X) "v_fma_f32 " X ", " X ", %11, %8\n"           /* 2 VGPR + SGPR */
#define O_FMA_F32_K(X) "v_fma_f32 " X ", " X ", 0.5, %8\n"           /* 2 VGPR + inline constant */
#define O_PK_FMA_2(X) "v_pk_fma_f32 " X ", " X ", %8, " X "\n"       /* 2 distinct VGPR pairs */
#define O_PK_FMA_LO(X) "v_pk_fma_f32 " X ", " X ", %8, %9 op_sel_hi:[1,0,0]\n" /* broadcast lo halves */
#define O_PK_ADD_2(X) "v_pk_add_f32 " X ", " X ", " X "\n"
#define O_PK_MUL_S(X) "v_pk_mul_f32 " X ", " X ", %10\n"
#define O_ADD_F64_S(X) "v_add_f64 " X ", " X ", %10\n"
#define O_ADD_F64_K(X) "v_add_f64 " X ", " X ", 1.0\n"
#define O_FMA_F64_2(X) "v_fma_f64 " X ", " X ", %8, " X "\n"
#define O_MUL_F64_SELF(X) "v_mul_f64 " X ", " X ", " X "\n"
#define O_MAX_F32_K(X) "v_max_f32 " X ", 0.5, " X "\n"
#define O_MAX_F32_S(X) "v_max_f32 " X ", %11, " X "\n"
#define O_MIN3_F32_2(X) "v_min3_f32 " X ", " X ", %8, " X "\n"
#define O_MIN3_F32_S(X) "v_min3_f32 " X ", " X ", %8, %11\n"
#define O_LSHL_S(X) "v_lshlrev_b32 " X ", %11, " X "\n"
#define O_LSHL_V(X) "v_lshlrev_b32 " X ", %8, " X "\n"
#define O_LSHR_V(X) "v_lshrrev_b32 " X ", %8, " X "\n"
#define O_OR(X) "v_or_b32 " X ", " X ", %8\n"
#define O_OR3(X) "v_or3_b32 " X ", " X ", %8, %9\n"
#define O_ADD3_2(X) "v_add3_u32 " X ", " X ", %8, " X "\n"
#define O_ADD3_S(X) "v_add3_u32 " X ", " X ", %8, %11\n"
#define O_BITOP3_2(X) "v_bitop3_b32 " X ", " X ", %8, " X " bitop3:0x96\n"
#define O_BITOP3_S(X) "v_bitop3_b32 " X ", " X ", %8, %11 bitop3:0x96\n"
#define O_XOR_S(X) "v_xor_b32 " X ", %11, " X "\n"
#define O_ADD_U32_K(X) "v_add_u32 " X ", 0x1234, " X "\n"
#define O_CNDMASK_K(X) "v_cndmask_b32_e64 " X ", " X ", 0, %10\n"
#define O_MUL_U24(X) "v_mul_u32_u24 " X ", " X ", %8\n"
#define O_MAD_U24(X) "v_mad_u32_u24 " X ", " X ", %8, %9\n"
#define O_CVT_F32_U32(X) "v_cvt_f32_u32 " X ", %8\n"
#define O_ALIGNBIT_S(X) "v_alignbit_b32 " X ", " X ", %11, 9\n"
#define O_LSHL_ADD_2(X) "v_lshl_add_u32 " X ", " X ", 2, " X "\n"
#define O_ADD_LSHL(X) "v_add_lshl_u32 " X ", " X ", %8, 2\n"
#define O_PERM(X) "v_perm_b32 " X ", " X ", %8, %9\n"
#define O_MOV_DPP(X) "v_mov_b32_dpp " X ", %8 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n"
#define O_SUBREV(X) "v_subrev_u32 " X ", %8, " X "\n"
#define O_MUL_F32_K(X) "v_mul_f32 " X ", 0.5, " X "\n"
#define O_FMAC_F32(X) "v_fmac_f32 " X ", %8, %9\n"                 /* dst is the accumulator */
#define O_FMAC_F64(X) "v_fmac_f64 " X ", %8, %9\n"
#define O_PK_MOV(X) "v_pk_mov_b32 " X ", %8, %9 op_sel:[0,1]\n"
#define O_LSHL_ADD_U64_2(X) "v_lshl_add_u64 " X ", " X ", 0, " X "\n"

struct Stamp {
    unsigned long long t0, t1, r0, r1;  // s_memtime, s_memrealtime at loop start / end
};

template <class T>
__device__ __forceinline__ double fold(T x) { return (double)x; }

#define KERNEL(NAME, T, BT, INS, INIT, BINIT, CINIT)                                                    \
    __global__ __launch_bounds__(256) void k_##NAME(int iters, Stamp* st, double* sink) {               \
        const unsigned lane = threadIdx.x + 256u * blockIdx.x;                                          \
        T a0 = INIT(lane, 0), a1 = INIT(lane, 1), a2 = INIT(lane, 2), a3 = INIT(lane, 3),               \
          a4 = INIT(lane, 4), a5 = INIT(lane, 5), a6 = INIT(lane, 6), a7 = INIT(lane, 7);               \
        const BT b = BINIT(lane), c = CINIT(lane);                                                      \
        const uint64_t m = __builtin_amdgcn_read_exec() ^ (uint64_t)(blockIdx.x & 1u);                  \
        const uint32_t su = 0x3f800001u + (blockIdx.x & 7u); /* a uniform 32-bit value (f32 ~1.0) */    \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                                     \
        const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();                                 \
        for (int i = 0; i < iters; ++i)                                                                 \
            asm volatile(IND8(INS) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5),        \
                         "+v"(a6), "+v"(a7) : "v"(b), "v"(c), "s"(m), "s"(su) : "vcc");                 \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                                     \
        const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();                                 \
        if (threadIdx.x == 0) st[blockIdx.x] = Stamp{t0, t1, r0, r1};                                   \
        sink[lane] = fold(a0) + fold(a1) + fold(a2) + fold(a3) + fold(a4) + fold(a5) + fold(a6) +       \
                     fold(a7);                                                                          \
    }

// per-lane values: f64 in [1, 2), a contraction factor b in (0.5, 0.75) and an addend c for fma
#define F64_INIT(l, k) (1.0 + (double)(((l) * 2654435761u + (k) * 40503u) & 0xffff) / 65536.0)
#define F64_B_FMA(l) (0.5 + (double)((l) & 0xff) / 1024.0)
#define F64_C(l) (0.25 + (double)(((l) >> 8) & 0xff) / 1024.0)
#define F64_B_ADD(l) (1e-9 * (1.0 + (double)((l) & 0xff)))
#define F64_B_MUL(l) (1.0 + 1e-12 * (double)((l) & 0xff))
#define F32_INIT(l, k) (1.0f + (float)(((l) * 2654435761u + (k) * 40503u) & 0xffff) / 65536.0f)
#define F32_B(l) (0.5f + (float)((l) & 0xff) / 1024.0f)
#define F32_C(l) (0.25f + (float)(((l) >> 8) & 0xff) / 1024.0f)
#define U32_INIT(l, k) ((l) * 2654435761u + (k) * 0x9e3779b9u)
#define U32_B(l) ((l) * 0x85ebca6bu + 1u)
#define U32_C(l) ((l) * 0xc2b2ae35u + 7u)
#define U64_INIT(l, k) ((uint64_t)((l) * 2654435761u + (k)) << 7)

typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 pk(float x, float y) { return f32x2{x, y}; }
template <>
__device__ __forceinline__ double fold<f32x2>(f32x2 x) { return (double)x.x + (double)x.y; }
#define PK_INIT(l, k) pk(F32_INIT(l, k), F32_INIT((l) + 77u, k))
#define PK_B(l) pk(F32_B(l), F32_B((l) + 3u))
#define PK_C(l) pk(F32_C(l), F32_C((l) + 5u))

KERNEL(fma_f64, double, double, I_FMA_F64, F64_INIT, F64_B_FMA, F64_C)
KERNEL(add_f64, double, double, I_ADD_F64, F64_INIT, F64_B_ADD, F64_C)
KERNEL(mul_f64, double, double, I_MUL_F64, F64_INIT, F64_B_MUL, F64_C)
KERNEL(fma_f32, float, float, I_FMA_F32, F32_INIT, F32_B, F32_C)
KERNEL(pk_fma_f32, f32x2, f32x2, I_PK_FMA_F32, PK_INIT, PK_B, PK_C)
KERNEL(add_u32, uint32_t, uint32_t, I_ADD_U32, U32_INIT, U32_B, U32_C)
KERNEL(xor_b32, uint32_t, uint32_t, I_XOR, U32_INIT, U32_B, U32_C)
KERNEL(alignbit, uint32_t, uint32_t, I_ALIGNBIT, U32_INIT, U32_B, U32_C)
KERNEL(max3_f32, float, float, I_MAX3_F32, F32_INIT, F32_B, F32_C)
KERNEL(cndmask_s, uint32_t, uint32_t, I_CNDMASK_S, U32_INIT, U32_B, U32_C)
KERNEL(mad_u64_u32, uint64_t, uint32_t, I_MAD_U64_U32, U64_INIT, U32_B, U32_C)

#define KD(NAME, INS) KERNEL(NAME, double, double, INS, F64_INIT, F64_B_MUL, F64_C)
#define KU(NAME, INS) KERNEL(NAME, uint32_t, uint32_t, INS, U32_INIT, U32_B, U32_C)
#define KF(NAME, INS) KERNEL(NAME, float, float, INS, F32_INIT, F32_B, F32_C)
#define KP(NAME, INS) KERNEL(NAME, f32x2, f32x2, INS, PK_INIT, PK_B, PK_C)
#define KL(NAME, INS) KERNEL(NAME, uint64_t, uint64_t, INS, U64_INIT, U64_INIT_B, U64_INIT_B)
#define U64_INIT_B(l) ((uint64_t)(l) * 0x9e3779b97f4a7c15ull + 1)
KD(rsq_f64, T_RSQ_F64) KL(lshl_add_u64, T_LSHL_ADD_U64) KL(lshr_b64, T_LSHR_B64) KU(mul_lo_u32, T_MUL_LO_U32)
KU(mul_hi_u32, T_MUL_HI_U32) KU(bitop3, T_BITOP3) KU(ffbh, T_FFBH) KU(mad_i32_i24, T_MAD_I32_I24)
KU(cndmask_vcmp, T_CNDMASK_VCMP) KF(cmp_f32, T_CMP_F32) KU(mov, T_MOV) KF(max_f32, T_MAX_F32) KF(med3_f32, T_MED3_F32)
KU(lshl_b32, T_LSHL_B32) KU(bfi, T_BFI) KU(add3, T_ADD3) KU(lshl_add_u32, T_LSHL_ADD_U32) KU(mbcnt, T_MBCNT)
KF(rcp_f32, T_RCP_F32) KD(rcp_f64, T_RCP_F64) KD(ldexp_f64, T_LDEXP_F64) KU(bfrev, T_BFREV) KU(and_or, T_AND_OR)
KU(not32, T_NOT) KU(add_co, T_ADD_CO) KD(mov_b64, T_MOV_B64) KD(max_f64, T_MAX_F64) KD(cmp_f64, T_CMP_F64)
KL(cmp_u64, T_CMP_U64) KU(lshr_b32, T_LSHR_B32) KU(and32, T_AND_B32) KL(lshl_b64, T_LSHL_B64) KF(mul_f32, T_MUL_F32)
KU(sub_u32, T_SUB_U32) KU(max_i32, T_MAX_I32) KU(min_i32, T_MIN_I32) KU(max3_i32, T_MAX3_I32) KU(min3_i32, T_MIN3_I32)
KU(max_u32, T_MAX_U32) KU(cmp_le_i32, T_CMP_LE_I32) KF(maximum3_f32, T_MAXIMUM3_F32) KF(min_f32, T_MIN_F32)
KF(sub_f32, T_SUB_F32) KP(pk_add_f32, T_PK_ADD_F32) KP(pk_mul_f32, T_PK_MUL_F32) KU(ashr_i32, T_ASHR_I32)
KF(o_fma_f32_s, O_FMA_F32_S) KF(o_fma_f32_k, O_FMA_F32_K) KP(o_pk_fma_2, O_PK_FMA_2) KP(o_pk_fma_lo, O_PK_FMA_LO)
KP(o_pk_add_2, O_PK_ADD_2) KP(o_pk_mul_s, O_PK_MUL_S) KD(o_add_f64_s, O_ADD_F64_S) KD(o_add_f64_k, O_ADD_F64_K)
KD(o_fma_f64_2, O_FMA_F64_2) KD(o_mul_f64_self, O_MUL_F64_SELF) KF(o_max_f32_k, O_MAX_F32_K) KF(o_max_f32_s, O_MAX_F32_S)
KF(o_min3_f32_2, O_MIN3_F32_2) KF(o_min3_f32_s, O_MIN3_F32_S) KU(o_lshl_s, O_LSHL_S) KU(o_lshl_v, O_LSHL_V)
KU(o_lshr_v, O_LSHR_V) KU(o_or, O_OR) KU(o_or3, O_OR3) KU(o_add3_2, O_ADD3_2) KU(o_add3_s, O_ADD3_S)
KU(o_bitop3_2, O_BITOP3_2) KU(o_bitop3_s, O_BITOP3_S) KU(o_xor_s, O_XOR_S) KU(o_add_u32_k, O_ADD_U32_K)
KU(o_cndmask_k, O_CNDMASK_K) KU(o_mul_u24, O_MUL_U24) KU(o_mad_u24, O_MAD_U24) KU(o_cvt_f32_u32, O_CVT_F32_U32)
KU(o_alignbit_s, O_ALIGNBIT_S) KU(o_lshl_add_2, O_LSHL_ADD_2) KU(o_add_lshl, O_ADD_LSHL) KU(o_perm, O_PERM)
KU(o_mov_dpp, O_MOV_DPP) KU(o_subrev, O_SUBREV) KF(o_mul_f32_k, O_MUL_F32_K) KF(o_fmac_f32, O_FMAC_F32)
KD(o_fmac_f64, O_FMAC_F64) KP(o_pk_mov, O_PK_MOV) KL(o_lshl_add_u64_2, O_LSHL_ADD_U64_2)
KU(alignbit_same, T_ALIGNBIT_SAME) KERNEL(cvt_f32_f64_in, float, double, T_CVT_F32_F64, F32_INIT, F64_B_MUL, F64_C) KF(add_f32, T_ADD_F32) KF(fma_f32_ss, T_FMA_F32_SS)

struct Op {
    const char* name;
    void (*fn)(int, Stamp*, double*);
    double ops_per_lane;  // FLOPs (fma = 2, packed fma = 4) or integer ops per lane-instruction
    const char* unit;
};

int main(int argc, char** argv) {
    const double target_ms = argc > 1 ? std::atof(argv[1]) : 120.0;
    const Op ops[] = {
        {"v_fma_f64", k_fma_f64, 2, "TFLOP/s"},     {"v_add_f64", k_add_f64, 1, "TFLOP/s"},
        {"v_mul_f64", k_mul_f64, 1, "TFLOP/s"},     {"v_fma_f32", k_fma_f32, 2, "TFLOP/s"},
        {"v_pk_fma_f32", k_pk_fma_f32, 4, "TFLOP/s"}, {"v_add_u32", k_add_u32, 1, "Tops/s"},
        {"v_xor_b32", k_xor_b32, 1, "Tops/s"},      {"v_alignbit_b32", k_alignbit, 1, "Tops/s"},
        {"v_max3_f32", k_max3_f32, 1, "Tops/s"},    {"v_cndmask_b32_e64", k_cndmask_s, 1, "Tops/s"},
        {"v_mad_u64_u32", k_mad_u64_u32, 1, "Tops/s"},
    };
    const Op table[] = {
        {"v_rsq_f64", k_rsq_f64, 1, "Tops/s"}, {"v_lshl_add_u64", k_lshl_add_u64, 1, "Tops/s"},
        {"v_lshrrev_b64", k_lshr_b64, 1, "Tops/s"}, {"v_mul_lo_u32", k_mul_lo_u32, 1, "Tops/s"},
        {"v_mul_hi_u32", k_mul_hi_u32, 1, "Tops/s"}, {"v_bitop3_b32", k_bitop3, 1, "Tops/s"},
        {"v_ffbh_u32", k_ffbh, 1, "Tops/s"}, {"v_mad_i32_i24", k_mad_i32_i24, 1, "Tops/s"},
        {"v_cmp_gt_u32 vcc + v_cndmask_b32 (pair)", k_cndmask_vcmp, 1, "Tops/s"},
        {"v_cmp_gt_f32 vcc", k_cmp_f32, 1, "Tops/s"}, {"v_mov_b32", k_mov, 1, "Tops/s"},
        {"v_max_f32", k_max_f32, 1, "Tops/s"}, {"v_med3_f32", k_med3_f32, 1, "Tops/s"},
        {"v_lshlrev_b32", k_lshl_b32, 1, "Tops/s"}, {"v_bfi_b32", k_bfi, 1, "Tops/s"},
        {"v_add3_u32", k_add3, 1, "Tops/s"}, {"v_lshl_add_u32", k_lshl_add_u32, 1, "Tops/s"},
        {"v_mbcnt_lo_u32_b32", k_mbcnt, 1, "Tops/s"}, {"v_rcp_f32", k_rcp_f32, 1, "Tops/s"},
        {"v_rcp_f64", k_rcp_f64, 1, "Tops/s"}, {"v_ldexp_f64", k_ldexp_f64, 1, "Tops/s"},
        {"v_bfrev_b32", k_bfrev, 1, "Tops/s"}, {"v_and_or_b32", k_and_or, 1, "Tops/s"},
        {"v_not_b32", k_not32, 1, "Tops/s"}, {"v_add_co_u32", k_add_co, 1, "Tops/s"},
        {"v_mov_b64", k_mov_b64, 1, "Tops/s"}, {"v_max_f64", k_max_f64, 1, "Tops/s"},
        {"v_cmp_lt_f64 vcc", k_cmp_f64, 1, "Tops/s"}, {"v_cmp_gt_u64 vcc", k_cmp_u64, 1, "Tops/s"},
        {"v_lshrrev_b32", k_lshr_b32, 1, "Tops/s"}, {"v_and_b32", k_and32, 1, "Tops/s"},
        {"v_lshlrev_b64", k_lshl_b64, 1, "Tops/s"}, {"v_mul_f32", k_mul_f32, 1, "Tops/s"},
        {"v_sub_u32", k_sub_u32, 1, "Tops/s"}, {"v_max_i32", k_max_i32, 1, "Tops/s"},
        {"v_min_i32", k_min_i32, 1, "Tops/s"}, {"v_max3_i32", k_max3_i32, 1, "Tops/s"},
        {"v_min3_i32", k_min3_i32, 1, "Tops/s"}, {"v_max_u32", k_max_u32, 1, "Tops/s"},
        {"v_cmp_le_i32 vcc", k_cmp_le_i32, 1, "Tops/s"}, {"v_maximum3_f32", k_maximum3_f32, 1, "Tops/s"},
        {"v_min_f32", k_min_f32, 1, "Tops/s"}, {"v_sub_f32", k_sub_f32, 1, "Tops/s"},
        {"v_pk_add_f32", k_pk_add_f32, 2, "TFLOP/s"}, {"v_pk_mul_f32", k_pk_mul_f32, 2, "TFLOP/s"},
        {"v_ashrrev_i32", k_ashr_i32, 1, "Tops/s"}, {"v_alignbit_b32 (x, x: rotate)", k_alignbit_same, 1, "Tops/s"},
        {"v_cvt_f32_f64", k_cvt_f32_f64_in, 1, "Tops/s"}, {"v_add_f32", k_add_f32, 1, "TFLOP/s"},
        {"v_fma_f32 (x, b, x)", k_fma_f32_ss, 2, "TFLOP/s"},
        {"v_fma_f32 (x, s, b)", k_o_fma_f32_s, 2, "TFLOP/s"}, {"v_fma_f32 (x, 0.5, b)", k_o_fma_f32_k, 2, "TFLOP/s"},
        {"v_pk_fma_f32 (x, b, x)", k_o_pk_fma_2, 4, "TFLOP/s"}, {"v_pk_fma_f32 (x, b, c) op_sel_hi:[1,0,0]", k_o_pk_fma_lo, 4, "TFLOP/s"},
        {"v_pk_add_f32 (x, x)", k_o_pk_add_2, 2, "TFLOP/s"}, {"v_pk_mul_f32 (x, s)", k_o_pk_mul_s, 2, "TFLOP/s"},
        {"v_add_f64 (x, s)", k_o_add_f64_s, 1, "TFLOP/s"}, {"v_add_f64 (x, 1.0)", k_o_add_f64_k, 1, "TFLOP/s"},
        {"v_fma_f64 (x, b, x)", k_o_fma_f64_2, 2, "TFLOP/s"}, {"v_mul_f64 (x, x)", k_o_mul_f64_self, 1, "TFLOP/s"},
        {"v_max_f32 (0.5, x)", k_o_max_f32_k, 1, "Tops/s"}, {"v_max_f32 (s, x)", k_o_max_f32_s, 1, "Tops/s"},
        {"v_min3_f32 (x, b, x)", k_o_min3_f32_2, 1, "Tops/s"}, {"v_min3_f32 (x, b, s)", k_o_min3_f32_s, 1, "Tops/s"},
        {"v_lshlrev_b32 (s, x)", k_o_lshl_s, 1, "Tops/s"}, {"v_lshlrev_b32 (b, x)", k_o_lshl_v, 1, "Tops/s"},
        {"v_lshrrev_b32 (b, x)", k_o_lshr_v, 1, "Tops/s"}, {"v_or_b32", k_o_or, 1, "Tops/s"},
        {"v_or3_b32", k_o_or3, 1, "Tops/s"}, {"v_add3_u32 (x, b, x)", k_o_add3_2, 1, "Tops/s"},
        {"v_add3_u32 (x, b, s)", k_o_add3_s, 1, "Tops/s"}, {"v_bitop3_b32 (x, b, x)", k_o_bitop3_2, 1, "Tops/s"},
        {"v_bitop3_b32 (x, b, s)", k_o_bitop3_s, 1, "Tops/s"}, {"v_xor_b32 (s, x)", k_o_xor_s, 1, "Tops/s"},
        {"v_add_u32 (0x1234, x)", k_o_add_u32_k, 1, "Tops/s"}, {"v_cndmask_b32_e64 (x, 0, s)", k_o_cndmask_k, 1, "Tops/s"},
        {"v_mul_u32_u24", k_o_mul_u24, 1, "Tops/s"}, {"v_mad_u32_u24", k_o_mad_u24, 1, "Tops/s"},
        {"v_cvt_f32_u32", k_o_cvt_f32_u32, 1, "Tops/s"}, {"v_alignbit_b32 (x, s)", k_o_alignbit_s, 1, "Tops/s"},
        {"v_lshl_add_u32 (x, 2, x)", k_o_lshl_add_2, 1, "Tops/s"}, {"v_add_lshl_u32", k_o_add_lshl, 1, "Tops/s"},
        {"v_perm_b32", k_o_perm, 1, "Tops/s"}, {"v_mov_b32_dpp", k_o_mov_dpp, 1, "Tops/s"},
        {"v_subrev_u32", k_o_subrev, 1, "Tops/s"}, {"v_mul_f32 (0.5, x)", k_o_mul_f32_k, 1, "TFLOP/s"},
        {"v_fmac_f32 (b, c)", k_o_fmac_f32, 2, "TFLOP/s"}, {"v_fmac_f64 (b, c)", k_o_fmac_f64, 2, "TFLOP/s"},
        {"v_pk_mov_b32", k_o_pk_mov, 1, "Tops/s"}, {"v_lshl_add_u64 (x, 0, x)", k_o_lshl_add_u64_2, 1, "Tops/s"},
    };
    const bool want_table = argc > 2 && std::atoi(argv[2]) != 0;
    int cus = 0, dev_clock_khz = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipDeviceGetAttribute(&dev_clock_khz, hipDeviceAttributeClockRate, 0));
    const int simds = cus * 4;
    const int max_blocks = cus * 8;
    Stamp* d_st = nullptr;
    double* d_sink = nullptr;
    CK(hipMalloc(&d_st, max_blocks * sizeof(Stamp)));
    CK(hipMalloc(&d_sink, (size_t)max_blocks * 256 * sizeof(double)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    auto run = [&](const Op& op, int wps, int iters, double* ms_out, double* clk_ghz, double* memtime_per_instr) {
        const int blocks = cus * wps;  // 256-thread blocks = one wave per SIMD each
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(op.fn, dim3(blocks), dim3(256), 0, 0, iters, d_st, d_sink);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<Stamp> st(blocks);
        CK(hipMemcpy(st.data(), d_st, blocks * sizeof(Stamp), hipMemcpyDeviceToHost));
        std::vector<double> clk(blocks), per(blocks);
        for (int i = 0; i < blocks; ++i) {
            clk[i] = (double)(st[i].t1 - st[i].t0) / (double)(st[i].r1 - st[i].r0) * 0.1;  // GHz
            per[i] = (double)(st[i].t1 - st[i].t0) / ((double)iters * 64);
        }
        std::sort(clk.begin(), clk.end());
        std::sort(per.begin(), per.end());
        *ms_out = ms;
        *clk_ghz = clk[blocks / 2];
        *memtime_per_instr = per[blocks / 2];
    };

    // ≥ 2 s of back-to-back f64 fma launches first: the clock the chip holds under load
    {
        double ms, clk, per;
        const auto t0 = std::chrono::steady_clock::now();
        int iters = 2000;
        while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 2.0) {
            run(ops[0], 4, iters, &ms, &clk, &per);
            if (ms < 100) iters *= 2;
        }
    }

    std::printf("{\"cus\": %d, \"simds\": %d, \"device_clock_attr_MHz\": %.0f, \"target_ms\": %.0f, \"results\": [\n",
                cus, simds, dev_clock_khz / 1000.0, target_ms);
    bool first = true;
    std::vector<std::pair<const Op*, int>> plan;
    const bool table_only = argc > 2 && std::atoi(argv[2]) == 2;
    if (!table_only)
        for (const Op& op : ops)
            for (int wps : {1, 2, 4, 8}) plan.push_back({&op, wps});
    if (want_table)
        for (const Op& op : table)
            for (int wps : {4, 8}) plan.push_back({&op, wps});
    for (const auto& pw : plan) {
        const Op& op = *pw.first;
        const int wps = pw.second;
        {
            // calibrate iterations to ≈ target_ms, then three timed launches (best kept)
            int iters = 1000;
            double ms = 0, clk = 0, per = 0;
            for (int k = 0; k < 12; ++k) {
                run(op, wps, iters, &ms, &clk, &per);
                if (ms >= 0.5 * target_ms) break;
                iters = (int)std::min<double>(2e9 / 64, iters * std::max(2.0, 0.6 * target_ms / std::max(ms, 1e-3)));
            }
            iters = (int)std::min<double>(2e9 / 64, iters * target_ms / ms);
            double best_ms = 1e30, best_clk = 0, best_per = 0;
            for (int rep = 0; rep < 3; ++rep) {
                run(op, wps, iters, &ms, &clk, &per);
                if (ms < best_ms) best_ms = ms, best_clk = clk, best_per = per;
            }
            const double wave_instr = (double)cus * wps * 4 * (double)iters * 64;
            const double rate = wave_instr * 64 * op.ops_per_lane / (best_ms * 1e-3) / 1e12;
            const double simd_cyc = (double)simds * best_clk * 1e9 * (best_ms * 1e-3) / wave_instr;
            std::printf("%s  {\"op\": \"%s\", \"waves_per_simd\": %d, \"iters\": %d, \"ms\": %.3f, \"%s\": %.2f, "
                        "\"in_kernel_clock_GHz\": %.4f, \"simd_cycles_per_wave_instr_event\": %.3f, "
                        "\"memtime_ticks_per_instr_per_wave\": %.3f, \"simd_cycles_per_wave_instr_memtime\": %.3f}",
                        first ? "" : ",\n", op.name, wps, iters, best_ms, op.unit, rate, best_clk, simd_cyc, best_per,
                        best_per / wps);
            first = false;
        }
    }
    std::printf("\n]}\n");
    return 0;
}

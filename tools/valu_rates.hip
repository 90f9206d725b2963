// valu_rates.hip — issue cost of the VALU instruction classes the sample kernel spends its cycles on,
// measured on the MI355X (gfx950), so the per-region instruction table (tools/region_table.py) can be
// priced in cycles instead of the 2/4/8-cycle model.  MI355X_MICROARCH.md lists f32 / transcendental /
// MFMA costs; the f64 and 64-bit integer forms the path tracer uses (v_lshl_add_u64, v_mad_u64_u32,
// v_mul_lo_u32, the f64 quadratic, v_bitop3, v_alignbit) are not in it.
//
// Each kernel runs one wave per SIMD (grid = 4 x CUs waves of 64) and executes, in a loop of
// kIters iterations, 8 independent chains of one instruction (8 x kUnroll instructions per
// iteration), so throughput rather than latency is timed; `dep` variants run ONE chain (latency).
// Cycles per wave-instruction = s_memtime delta / instructions (median over waves).  A second run at
// 4 waves per SIMD (the product's occupancy) gives the SIMD's throughput when several waves issue.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/valu_rates.hip -o tools/bin/valu_rates
//   ./tools/bin/valu_rates            (one JSON line)
#include <hip/hip_runtime.h>

#include <algorithm>
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

constexpr int kIters = 256;  // asm runs of 64 instructions each

// One instruction class = one template string with %X (the updated operand), %B and %C (read
// operands).  The whole unrolled run is ONE asm statement (".rept"): the compiler inserts hazard
// s_nops between separate inline-asm statements (it cannot see what they hold), never inside one.
#define IND8(INS) ".rept 8\n" INS("%0") INS("%1") INS("%2") INS("%3") INS("%4") INS("%5") INS("%6") INS("%7") ".endr\n"
#define DEP64(INS) ".rept 64\n" INS("%0") ".endr\n"

#define KERNEL(NAME, T, INS)                                                                       \
    __global__ void k_##NAME(unsigned long long* cyc, double* sink, int dep) {                     \
        T a0 = seedv<T>(0), a1 = seedv<T>(1), a2 = seedv<T>(2), a3 = seedv<T>(3), a4 = seedv<T>(4), \
          a5 = seedv<T>(5), a6 = seedv<T>(6), a7 = seedv<T>(7);                                    \
        const T b = seedv<T>(11), c = seedv<T>(13);                                                \
        const uint64_t m = __builtin_amdgcn_read_exec() ^ (uint64_t)dep;                           \
        const uint64_t t0 = __builtin_amdgcn_s_memtime();                                          \
        if (dep) {                                                                                 \
            for (int i = 0; i < kIters; ++i)                                                       \
                asm volatile(DEP64(INS) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), \
                             "+v"(a6), "+v"(a7) : "v"(b), "v"(c), "s"(m) : "vcc");                 \
        } else {                                                                                   \
            for (int i = 0; i < kIters; ++i)                                                       \
                asm volatile(IND8(INS) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), \
                             "+v"(a6), "+v"(a7) : "v"(b), "v"(c), "s"(m) : "vcc");                 \
        }                                                                                          \
        const uint64_t t1 = __builtin_amdgcn_s_memtime();                                          \
        if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;                                           \
        sink[blockIdx.x * blockDim.x + threadIdx.x] =                                              \
            fold(a0) + fold(a1) + fold(a2) + fold(a3) + fold(a4) + fold(a5) + fold(a6) + fold(a7);  \
    }

template <class T>
__device__ __forceinline__ T seedv(int k) {
    if constexpr (sizeof(T) == 8) return (T)(threadIdx.x + k) * 1.0000001;
    else return (T)(threadIdx.x * 2654435761u + k);
}
template <class T>
__device__ __forceinline__ double fold(T x) { return (double)x; }

// operands: X updated, %8 = b, %9 = c (pairs for the 64-bit kernels, 32-bit values otherwise)
#define I_ADD_F64(X) "v_add_f64 " X ", " X ", %8\n"
#define I_MUL_F64(X) "v_mul_f64 " X ", " X ", %8\n"
#define I_FMA_F64(X) "v_fma_f64 " X ", " X ", %8, " X "\n"
#define I_RSQ_F64(X) "v_rsq_f64 " X ", " X "\n"
#define I_LSHL_ADD_U64(X) "v_lshl_add_u64 " X ", " X ", 0, %8\n"
#define I_LSHR_B64(X) "v_lshrrev_b64 " X ", 7, " X "\n"
#define I_PK_FMA_F32(X) "v_pk_fma_f32 " X ", " X ", %8, " X "\n"
#define I_ADD_U32(X) "v_add_u32 " X ", " X ", %8\n"
#define I_MUL_LO_U32(X) "v_mul_lo_u32 " X ", " X ", %8\n"
#define I_MUL_HI_U32(X) "v_mul_hi_u32 " X ", " X ", %8\n"
#define I_BITOP3(X) "v_bitop3_b32 " X ", " X ", %8, %9 bitop3:0x96\n"
#define I_ALIGNBIT(X) "v_alignbit_b32 " X ", " X ", %8, 9\n"
#define I_CNDMASK(X) "v_cndmask_b32 " X ", " X ", %8, vcc\n"
#define I_FMA_F32(X) "v_fma_f32 " X ", " X ", %8, " X "\n"
#define I_MAX3_F32(X) "v_max3_f32 " X ", " X ", %8, %9\n"
#define I_FFBH(X) "v_ffbh_u32 " X ", " X "\n"
#define I_MAD_I32_I24(X) "v_mad_i32_i24 " X ", " X ", %8, %9\n"
#define I_MAD_U64_U32(X) "v_mad_u64_u32 " X ", vcc, %8, %9, " X "\n"
#define I_CNDMASK_S(X) "v_cndmask_b32_e64 " X ", " X ", %8, %10\n"
#define I_CNDMASK_VCMP(X) "v_cmp_gt_u32 vcc, " X ", %8\nv_cndmask_b32 " X ", " X ", %9, vcc\n"
#define I_CMP_F32(X) "v_cmp_gt_f32 vcc, " X ", %8\n"
#define I_MOV(X) "v_mov_b32 " X ", %8\n"
#define I_XOR(X) "v_xor_b32 " X ", " X ", %8\n"
#define I_MAX_F32(X) "v_max_f32 " X ", " X ", %8\n"
#define I_MED3_F32(X) "v_med3_f32 " X ", " X ", %8, %9\n"
#define I_LSHL_B32(X) "v_lshlrev_b32 " X ", 7, " X "\n"
#define I_BFI(X) "v_bfi_b32 " X ", %8, " X ", %9\n"
#define I_CVT_F32_F64(X) "v_cvt_f32_f64 " X ", %8\n"
#define I_ADD3(X) "v_add3_u32 " X ", " X ", %8, %9\n"
#define I_LSHL_ADD_U32(X) "v_lshl_add_u32 " X ", " X ", 2, %8\n"
#define I_MBCNT(X) "v_mbcnt_lo_u32_b32 " X ", %8, " X "\n"
#define I_RCP_F32(X) "v_rcp_f32 " X ", " X "\n"
#define I_RCP_F64(X) "v_rcp_f64 " X ", " X "\n"
#define I_LDEXP_F64(X) "v_ldexp_f64 " X ", " X ", 1\n"
#define I_BFREV(X) "v_bfrev_b32 " X ", " X "\n"
#define I_AND_OR(X) "v_and_or_b32 " X ", " X ", %8, %9\n"
#define I_NOT(X) "v_not_b32 " X ", " X "\n"
#define I_ADD_CO(X) "v_add_co_u32 " X ", vcc, " X ", %8\n"
#define I_MOV_B64(X) "v_mov_b64 " X ", %8\n"
#define I_MAX_F64(X) "v_max_f64 " X ", " X ", %8\n"
#define I_CMP_F64(X) "v_cmp_lt_f64 vcc, " X ", %8\n"
#define I_CMP_U64(X) "v_cmp_gt_u64 vcc, " X ", %8\n"
#define I_LSHR_B32(X) "v_lshrrev_b32 " X ", 7, " X "\n"
#define I_AND_B32(X) "v_and_b32 " X ", " X ", %8\n"
#define I_LSHL_B64(X) "v_lshlrev_b64 " X ", 7, " X "\n"
#define I_MUL_F32(X) "v_mul_f32 " X ", " X ", %8\n"
#define I_SUB_U32(X) "v_sub_u32 " X ", " X ", %8\n"
#define I_MAX_I32(X) "v_max_i32 " X ", " X ", %8\n"
#define I_MIN_I32(X) "v_min_i32 " X ", " X ", %8\n"
#define I_MAX3_I32(X) "v_max3_i32 " X ", " X ", %8, %9\n"
#define I_MIN3_I32(X) "v_min3_i32 " X ", " X ", %8, %9\n"
#define I_MAX_U32(X) "v_max_u32 " X ", " X ", %8\n"
#define I_CMP_LE_I32(X) "v_cmp_le_i32 vcc, " X ", %8\n"
#define I_CMP_LE_I32_S(X) "v_cmp_le_i32_e64 %10, " X ", %8\n"
#define I_MAXIMUM3_F32(X) "v_maximum3_f32 " X ", " X ", %8, %9\n"
#define I_MIN_F32(X) "v_min_f32 " X ", " X ", %8\n"
#define I_SUB_F32(X) "v_sub_f32 " X ", " X ", %8\n"
#define I_PK_ADD_F32(X) "v_pk_add_f32 " X ", " X ", %8\n"
#define I_ASHR_I32(X) "v_ashrrev_i32 " X ", 31, " X "\n"

KERNEL(add_f64, double, I_ADD_F64) KERNEL(mul_f64, double, I_MUL_F64) KERNEL(fma_f64, double, I_FMA_F64)
KERNEL(rsq_f64, double, I_RSQ_F64) KERNEL(lshl_add_u64, double, I_LSHL_ADD_U64) KERNEL(lshr_b64, double, I_LSHR_B64)
KERNEL(pk_fma_f32, double, I_PK_FMA_F32) KERNEL(add_u32, uint32_t, I_ADD_U32) KERNEL(mul_lo_u32, uint32_t, I_MUL_LO_U32)
KERNEL(mul_hi_u32, uint32_t, I_MUL_HI_U32) KERNEL(bitop3, uint32_t, I_BITOP3) KERNEL(alignbit, uint32_t, I_ALIGNBIT)
KERNEL(cndmask, uint32_t, I_CNDMASK) KERNEL(fma_f32, uint32_t, I_FMA_F32) KERNEL(max3_f32, uint32_t, I_MAX3_F32)
KERNEL(ffbh, uint32_t, I_FFBH) KERNEL(mad_i32_i24, uint32_t, I_MAD_I32_I24)
KERNEL(cndmask_s, uint32_t, I_CNDMASK_S) KERNEL(cndmask_vcmp, uint32_t, I_CNDMASK_VCMP) KERNEL(cmp_f32, uint32_t, I_CMP_F32)
KERNEL(mov, uint32_t, I_MOV) KERNEL(xor32, uint32_t, I_XOR) KERNEL(max_f32, uint32_t, I_MAX_F32)
KERNEL(med3_f32, uint32_t, I_MED3_F32) KERNEL(lshl_b32, uint32_t, I_LSHL_B32) KERNEL(bfi, uint32_t, I_BFI)
KERNEL(add3, uint32_t, I_ADD3) KERNEL(lshl_add_u32, uint32_t, I_LSHL_ADD_U32) KERNEL(mbcnt, uint32_t, I_MBCNT)
KERNEL(rcp_f32, uint32_t, I_RCP_F32) KERNEL(rcp_f64, double, I_RCP_F64) KERNEL(ldexp_f64, double, I_LDEXP_F64)
KERNEL(bfrev, uint32_t, I_BFREV) KERNEL(and_or, uint32_t, I_AND_OR) KERNEL(not32, uint32_t, I_NOT)
KERNEL(add_co, uint32_t, I_ADD_CO) KERNEL(mov_b64, double, I_MOV_B64) KERNEL(max_f64, double, I_MAX_F64)
KERNEL(cmp_f64, double, I_CMP_F64) KERNEL(cmp_u64, double, I_CMP_U64) KERNEL(lshr_b32, uint32_t, I_LSHR_B32)
KERNEL(and32, uint32_t, I_AND_B32) KERNEL(lshl_b64, double, I_LSHL_B64) KERNEL(mul_f32, uint32_t, I_MUL_F32)
KERNEL(sub_u32, uint32_t, I_SUB_U32)
KERNEL(max_i32, uint32_t, I_MAX_I32) KERNEL(min_i32, uint32_t, I_MIN_I32) KERNEL(max3_i32, uint32_t, I_MAX3_I32)
KERNEL(min3_i32, uint32_t, I_MIN3_I32) KERNEL(max_u32, uint32_t, I_MAX_U32) KERNEL(cmp_le_i32, uint32_t, I_CMP_LE_I32)
KERNEL(maximum3_f32, uint32_t, I_MAXIMUM3_F32) KERNEL(min_f32, uint32_t, I_MIN_F32)
KERNEL(sub_f32, uint32_t, I_SUB_F32) KERNEL(pk_add_f32, double, I_PK_ADD_F32) KERNEL(ashr_i32, uint32_t, I_ASHR_I32)
// v_mad_u64_u32: 32 x 32 -> 64 plus a 64-bit addend, into a pair
__global__ void k_mad_u64_u32(unsigned long long* cyc, double* sink, int dep) {
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const uint32_t b = threadIdx.x * 3 + 1, c = threadIdx.x * 5 + 7;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    if (dep) {
        for (int i = 0; i < kIters; ++i)
            asm volatile(DEP64(I_MAD_U64_U32) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),
                         "+v"(a7) : "v"(b), "v"(c), "s"(0ull) : "vcc");
    } else {
        for (int i = 0; i < kIters; ++i)
            asm volatile(IND8(I_MAD_U64_U32) : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6),
                         "+v"(a7) : "v"(b), "v"(c), "s"(0ull) : "vcc");
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = (double)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

struct K {
    const char* name;
    void (*fn)(unsigned long long*, double*, int);
};

int main() {
    const K ks[] = {{"v_add_f64", k_add_f64},         {"v_mul_f64", k_mul_f64},
                    {"v_fma_f64", k_fma_f64},         {"v_rsq_f64", k_rsq_f64},
                    {"v_lshl_add_u64", k_lshl_add_u64}, {"v_lshrrev_b64", k_lshr_b64},
                    {"v_mad_u64_u32", k_mad_u64_u32},
                    {"v_add_u32", k_add_u32},         {"v_mul_lo_u32", k_mul_lo_u32},
                    {"v_mul_hi_u32", k_mul_hi_u32},   {"v_bitop3_b32", k_bitop3},
                    {"v_alignbit_b32", k_alignbit},   {"v_cndmask_b32", k_cndmask},
                    {"v_fma_f32", k_fma_f32},         {"v_pk_fma_f32", k_pk_fma_f32},
                    {"v_max3_f32", k_max3_f32},       {"v_ffbh_u32", k_ffbh},
                    {"v_mad_i32_i24", k_mad_i32_i24},  {"v_cndmask_b32_e64 (SGPR mask)", k_cndmask_s},
                    {"v_cmp_gt_u32 vcc + v_cndmask_b32 (pair)", k_cndmask_vcmp}, {"v_cmp_gt_f32 vcc", k_cmp_f32},
                    {"v_mov_b32", k_mov},              {"v_xor_b32", k_xor32},
                    {"v_max_f32", k_max_f32},          {"v_med3_f32", k_med3_f32},
                    {"v_lshlrev_b32", k_lshl_b32},     {"v_bfi_b32", k_bfi},
                    {"v_add3_u32", k_add3},            {"v_lshl_add_u32", k_lshl_add_u32},
                    {"v_mbcnt_lo_u32_b32", k_mbcnt},   {"v_rcp_f32", k_rcp_f32},
                    {"v_rcp_f64", k_rcp_f64},          {"v_ldexp_f64", k_ldexp_f64},
                    {"v_bfrev_b32", k_bfrev},          {"v_and_or_b32", k_and_or},
                    {"v_not_b32", k_not32},            {"v_add_co_u32", k_add_co},
                    {"v_mov_b64", k_mov_b64},          {"v_max_f64", k_max_f64},
                    {"v_cmp_lt_f64 vcc", k_cmp_f64},   {"v_cmp_gt_u64 vcc", k_cmp_u64},
                    {"v_lshrrev_b32", k_lshr_b32},     {"v_and_b32", k_and32},
                    {"v_lshlrev_b64", k_lshl_b64},     {"v_mul_f32", k_mul_f32},
                    {"v_sub_u32", k_sub_u32},
                    {"v_max_i32", k_max_i32},          {"v_min_i32", k_min_i32},
                    {"v_max3_i32", k_max3_i32},        {"v_min3_i32", k_min3_i32},
                    {"v_max_u32", k_max_u32},          {"v_cmp_le_i32 vcc", k_cmp_le_i32},
                    {"v_maximum3_f32", k_maximum3_f32}, {"v_min_f32", k_min_f32},
                    {"v_sub_f32", k_sub_f32},          {"v_pk_add_f32", k_pk_add_f32},
                    {"v_ashrrev_i32", k_ashr_i32}};
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    unsigned long long* d_cyc = nullptr;
    double* d_sink = nullptr;
    const int max_blocks = cus * 16;
    CK(hipMalloc(&d_cyc, max_blocks * sizeof(unsigned long long)));
    CK(hipMalloc(&d_sink, (size_t)max_blocks * 64 * sizeof(double)));
    const double n_ins = (double)kIters * 64;
    std::printf("{\"instructions_per_wave\": %.0f, \"results\": [", n_ins);
    bool first = true;
    for (const K& k : ks) {
        double med[3] = {0, 0, 0};
        // (waves per SIMD, dep): 1 independent, 4 independent, 1 dependent
        const int cfg[3][2] = {{1, 0}, {4, 0}, {1, 1}};
        for (int c = 0; c < 3; ++c) {
            const int blocks = cus * 4 * cfg[c][0];  // 64-thread blocks, spread over the SIMDs
            for (int rep = 0; rep < 2; ++rep)
                hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(64), 0, 0, d_cyc, d_sink, cfg[c][1]);
            CK(hipDeviceSynchronize());
            std::vector<unsigned long long> cyc(blocks);
            CK(hipMemcpy(cyc.data(), d_cyc, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            std::sort(cyc.begin(), cyc.end());
            med[c] = (double)cyc[blocks / 2] / n_ins;
        }
        std::printf("%s{\"op\": \"%s\", \"cycles_1wave\": %.2f, \"cycles_per_wave_4waves\": %.2f, "
                    "\"simd_cycles_per_instr_4waves\": %.2f, \"dependent_latency_1wave\": %.2f}",
                    first ? "" : ", ", k.name, med[0], med[1], med[1] / 4, med[2]);
        first = false;
    }
    std::printf("]}\n");
    return 0;
}

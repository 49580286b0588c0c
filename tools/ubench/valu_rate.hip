// VALU issue-rate microbenchmark (gfx950): cycles per wave64 instruction for the packed 16-bit and
// 3-input max/min forms the FAST network could use.  Each wave runs 8 independent dependency chains
// of one instruction; 2048 workgroups x 256 threads fill every SIMD with 4+ waves.
// build: hipcc --offload-arch=gfx950 -O3 -o valu_rate valu_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(s) s s s s s s s s
#define BODY(INS) \
    asm volatile(REP8(INS " %0, %0, %8, %9\n" INS " %1, %1, %8, %9\n" INS " %2, %2, %8, %9\n" INS " %3, %3, %8, %9\n" \
                      INS " %4, %4, %8, %9\n" INS " %5, %5, %8, %9\n" INS " %6, %6, %8, %9\n" INS " %7, %7, %8, %9\n") \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));
#define BODY2(INS) \
    asm volatile(REP8(INS " %0, %0, %8\n" INS " %1, %1, %8\n" INS " %2, %2, %8\n" INS " %3, %3, %8\n" \
                      INS " %4, %4, %8\n" INS " %5, %5, %8\n" INS " %6, %6, %8\n" INS " %7, %7, %8\n") \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));

#define KERNEL3(name, INS) \
    __global__ __launch_bounds__(256) void name(unsigned* out, int iters, unsigned b, unsigned c) { \
        unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
        for (int i = 0; i < iters; i++) { BODY(INS) } \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; }
#define KERNEL2(name, INS) \
    __global__ __launch_bounds__(256) void name(unsigned* out, int iters, unsigned b, unsigned c) { \
        unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7; \
        for (int i = 0; i < iters; i++) { BODY2(INS) } \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; }

KERNEL2(k_pk_max_u16, "v_pk_max_u16")
KERNEL2(k_pk_max_f16, "v_pk_max_f16")
KERNEL2(k_pk_sub_u16, "v_pk_sub_u16")
KERNEL2(k_max_u32, "v_max_u32")
KERNEL2(k_max_u16, "v_max_u16")
KERNEL2(k_add_f32, "v_add_f32")
KERNEL3(k_pk_maximum3_f16, "v_pk_maximum3_f16")
KERNEL3(k_max3_u32, "v_max3_u32")
KERNEL3(k_max3_f32, "v_max3_f32")
KERNEL3(k_perm_b32, "v_perm_b32")
KERNEL3(k_pk_fma_f16, "v_pk_fma_f16")

KERNEL2(k2_v_max_f32, "v_max_f32")
KERNEL2(k2_v_min_f32, "v_min_f32")
KERNEL2(k2_v_max_f16, "v_max_f16")
KERNEL2(k2_v_sub_f32, "v_sub_f32")
KERNEL2(k2_v_and_b32, "v_and_b32")
KERNEL2(k2_v_add_u32, "v_add_u32")
KERNEL2(k2_v_sub_u16, "v_sub_u16")
KERNEL2(k2_v_max_i16, "v_max_i16")
KERNEL2(k2_v_min_u16, "v_min_u16")

KERNEL2(k2_v_pk_min_f16, "v_pk_min_f16")
KERNEL2(k2_v_lshlrev_b32, "v_lshlrev_b32")
KERNEL2(k2_v_xor_b32, "v_xor_b32")
KERNEL2(k2_v_mul_f32, "v_mul_f32")

KERNEL3(k3_v_max3_f16, "v_max3_f16")
KERNEL3(k3_v_med3_f32, "v_med3_f32")
KERNEL3(k3_v_alignbyte_b32, "v_alignbyte_b32")
KERNEL3(k3_v_dot4_u32_u8, "v_dot4_u32_u8")
KERNEL3(k3_v_pk_minimum3_f16, "v_pk_minimum3_f16")
KERNEL3(k3_v_fma_f32, "v_fma_f32")
KERNEL3(k3_v_max3_i16, "v_max3_i16")

KERNEL2(k2_v_mul_u32_u24, "v_mul_u32_u24")
KERNEL2(k2_v_mul_hi_u32_u24, "v_mul_hi_u32_u24")
KERNEL2(k2_v_lshrrev_b32, "v_lshrrev_b32")
KERNEL2(k2_v_or_b32, "v_or_b32")
KERNEL2(k2_v_sub_u32, "v_sub_u32")
KERNEL2(k2_v_min_i32, "v_min_i32")
KERNEL2(k2_v_max_i32, "v_max_i32")
KERNEL2(k2_v_add_f16, "v_add_f16")
KERNEL2(k2_v_mul_f16, "v_mul_f16")
KERNEL2(k2_v_lshlrev_b16, "v_lshlrev_b16")
KERNEL2(k2_v_add_u16, "v_add_u16")
KERNEL2(k2_v_pk_add_u16, "v_pk_add_u16")
KERNEL2(k2_v_pk_max_i16, "v_pk_max_i16")

KERNEL2(k2_v_pk_add_f16, "v_pk_add_f16")

KERNEL2(k2_v_mul_lo_u32, "v_mul_lo_u32")
KERNEL2(k2_v_mul_hi_u32, "v_mul_hi_u32")
KERNEL3(k3_v_mad_u32_u24, "v_mad_u32_u24")
KERNEL3(k3_v_lshl_or_b32, "v_lshl_or_b32")
KERNEL3(k3_v_lshl_add_u32, "v_lshl_add_u32")
KERNEL3(k3_v_add3_u32, "v_add3_u32")
KERNEL3(k3_v_and_or_b32, "v_and_or_b32")
KERNEL3(k3_v_bfe_u32, "v_bfe_u32")
KERNEL3(k3_v_or3_b32, "v_or3_b32")
KERNEL3(k3_v_add_lshl_u32, "v_add_lshl_u32")
KERNEL3(k3_v_dot2_u32_u16, "v_dot2_u32_u16")
KERNEL3(k3_v_alignbit_b32, "v_alignbit_b32")
KERNEL3(k3_v_sad_u8, "v_sad_u8")
KERNEL3(k3_v_min3_u32, "v_min3_u32")
KERNEL3(k3_v_max3_i32, "v_max3_i32")

int main()
{
    unsigned* d;
    hipMalloc(&d, 2048 * 256 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct K { const char* n; void (*f)(unsigned*, int, unsigned, unsigned); };
    K ks[] = {{"v_pk_max_u16", k_pk_max_u16}, {"v_pk_max_f16", k_pk_max_f16}, {"v_pk_sub_u16", k_pk_sub_u16},
              {"v_max_u32", k_max_u32}, {"v_max_u16", k_max_u16}, {"v_add_f32", k_add_f32},
              {"v_pk_maximum3_f16", k_pk_maximum3_f16}, {"v_max3_u32", k_max3_u32}, {"v_max3_f32", k_max3_f32},
              {"v_perm_b32", k_perm_b32}, {"v_pk_fma_f16", k_pk_fma_f16}, {"v_max_f32", k2_v_max_f32}, {"v_min_f32", k2_v_min_f32}, {"v_max_f16", k2_v_max_f16}, {"v_sub_f32", k2_v_sub_f32}, {"v_and_b32", k2_v_and_b32}, {"v_add_u32", k2_v_add_u32}, {"v_sub_u16", k2_v_sub_u16}, {"v_max_i16", k2_v_max_i16}, {"v_min_u16", k2_v_min_u16}, {"v_pk_min_f16", k2_v_pk_min_f16}, {"v_lshlrev_b32", k2_v_lshlrev_b32}, {"v_xor_b32", k2_v_xor_b32}, {"v_mul_f32", k2_v_mul_f32}, {"v_max3_f16", k3_v_max3_f16}, {"v_med3_f32", k3_v_med3_f32}, {"v_alignbyte_b32", k3_v_alignbyte_b32}, {"v_dot4_u32_u8", k3_v_dot4_u32_u8}, {"v_pk_minimum3_f16", k3_v_pk_minimum3_f16}, {"v_fma_f32", k3_v_fma_f32}, {"v_max3_i16", k3_v_max3_i16}, {"v_mul_u32_u24", k2_v_mul_u32_u24}, {"v_mul_hi_u32_u24", k2_v_mul_hi_u32_u24}, {"v_lshrrev_b32", k2_v_lshrrev_b32}, {"v_or_b32", k2_v_or_b32}, {"v_sub_u32", k2_v_sub_u32}, {"v_min_i32", k2_v_min_i32}, {"v_max_i32", k2_v_max_i32}, {"v_add_f16", k2_v_add_f16}, {"v_mul_f16", k2_v_mul_f16}, {"v_lshlrev_b16", k2_v_lshlrev_b16}, {"v_add_u16", k2_v_add_u16}, {"v_pk_add_u16", k2_v_pk_add_u16}, {"v_pk_max_i16", k2_v_pk_max_i16}, {"v_pk_add_f16", k2_v_pk_add_f16}, {"v_mul_lo_u32", k2_v_mul_lo_u32}, {"v_mul_hi_u32", k2_v_mul_hi_u32}, {"v_mad_u32_u24", k3_v_mad_u32_u24}, {"v_lshl_or_b32", k3_v_lshl_or_b32}, {"v_lshl_add_u32", k3_v_lshl_add_u32}, {"v_add3_u32", k3_v_add3_u32}, {"v_and_or_b32", k3_v_and_or_b32}, {"v_bfe_u32", k3_v_bfe_u32}, {"v_or3_b32", k3_v_or3_b32}, {"v_add_lshl_u32", k3_v_add_lshl_u32}, {"v_dot2_u32_u16", k3_v_dot2_u32_u16}, {"v_alignbit_b32", k3_v_alignbit_b32}, {"v_sad_u8", k3_v_sad_u8}, {"v_min3_u32", k3_v_min3_u32}, {"v_max3_i32", k3_v_max3_i32}, };
    const int iters = 2000, blocks = 2048;
    int clk = 0;
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    for (auto& k : ks) {
        for (int rep = 0; rep < 2; rep++) {
            hipEventRecord(e0);
            k.f<<<blocks, 256>>>(d, iters, 0x3c003c00u, 0x40004000u);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            const double insts = (double)blocks * 4 * iters * 64;   // wave-instructions
            const double simd_cyc = ms * 1e-3 * 2.4e9 * cus * 4;      // SIMD-cycles at 2.4 GHz
            if (rep) printf("%-20s %8.3f ms  %.2f cyc per wave64 instruction per SIMD\n", k.n, ms, simd_cyc / insts);
        }
    }
    printf("CUs %d, clock attr %d kHz\n", cus, clk);
    return 0;
}

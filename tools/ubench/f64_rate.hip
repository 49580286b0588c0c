// Issue-rate and latency microbenchmark for the PnP chain's Jacobi round (gfx950): one wave alone on its
// SIMD (the k_pnp_chain / k_pnp_hyp situation), timed with s_memtime around an unrolled block.
//   lat_*   one dependent chain: cycles from one instruction to the next that reads its result
//   thr_*   eight independent chains: cycles per instruction issued by the lone wave
//   lds_*   ds_read_b128 issue / latency, ds_write -> ds_read round trip, ds_bpermute_b32 latency, with 1 or 4
//           waves of a workgroup (4 waves = one per SIMD, sharing the CU's LDS)
// build: hipcc --offload-arch=gfx950 -O3 -o f64_rate f64_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(s) s s s s s s s s
#define REP64(s) REP8(REP8(s))

__device__ __forceinline__ long long tick() { return (long long)__builtin_amdgcn_s_memtime(); }
__device__ __forceinline__ long long rtick() { return (long long)__builtin_amdgcn_s_memrealtime(); }

#define LAT2(name, INS)                                                                                      \
    __global__ void name(long long* out, double b) {                                                      \
        double a = (double)threadIdx.x * 1e-3 + 1.0;                                                        \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)");                                                      \
        const long long t0 = tick(), r0 = rtick();                                                          \
        asm volatile(REP64(INS " %0, %0, %1\n") : "+v"(a) : "v"(b));                                        \
        const long long t1 = tick(), r1 = rtick();                                                          \
        if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }                                      \
        if (a == 12345.0) out[2] = 1;                                                                       \
    }
#define THR2(name, INS)                                                                                      \
    __global__ void name(long long* out, double b) {                                                      \
        double a0 = threadIdx.x + 1.0, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,       \
               a6 = a0 + 6, a7 = a0 + 7;                                                                    \
        const long long t0 = tick(), r0 = rtick();                                                          \
        asm volatile(REP8(INS " %0, %0, %8\n" INS " %1, %1, %8\n" INS " %2, %2, %8\n" INS " %3, %3, %8\n"    \
                          INS " %4, %4, %8\n" INS " %5, %5, %8\n" INS " %6, %6, %8\n" INS " %7, %7, %8\n")   \
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)         \
                     : "v"(b));                                                                             \
        const long long t1 = tick(), r1 = rtick();                                                          \
        if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }                                      \
        if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 12345.0) out[2] = 1;                                   \
    }
#define LAT1(name, INS)                                                                                      \
    __global__ void name(long long* out, double b) {                                                      \
        double a = (double)threadIdx.x * 1e-3 + 1.5;                                                        \
        const long long t0 = tick(), r0 = rtick();                                                          \
        asm volatile(REP64(INS " %0, %0\n") : "+v"(a));                                                     \
        const long long t1 = tick(), r1 = rtick();                                                          \
        if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }                                      \
        if (a == 12345.0) out[2] = 1;                                                                       \
    }
#define THR1(name, INS)                                                                                      \
    __global__ void name(long long* out, double b) {                                                      \
        double a0 = threadIdx.x + 1.0, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,       \
               a6 = a0 + 6, a7 = a0 + 7;                                                                    \
        const long long t0 = tick(), r0 = rtick();                                                          \
        asm volatile(REP8(INS " %0, %0\n" INS " %1, %1\n" INS " %2, %2\n" INS " %3, %3\n"                    \
                          INS " %4, %4\n" INS " %5, %5\n" INS " %6, %6\n" INS " %7, %7\n")                  \
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));      \
        const long long t1 = tick(), r1 = rtick();                                                          \
        if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }                                      \
        if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 12345.0) out[2] = 1;                                   \
    }

LAT2(lat_add_f64, "v_add_f64")
THR2(thr_add_f64, "v_add_f64")
LAT2(lat_mul_f64, "v_mul_f64")
THR2(thr_mul_f64, "v_mul_f64")
LAT1(lat_rcp_f64, "v_rcp_f64")
THR1(thr_rcp_f64, "v_rcp_f64")
LAT1(lat_rsq_f64, "v_rsq_f64")
THR1(thr_rsq_f64, "v_rsq_f64")

// v_cndmask_b32 (32-bit select, the Jacobi's zeroing / selects): one dependent chain and 8 independent ones
__global__ void lat_cndmask(long long* out, double b)
{
    unsigned a = threadIdx.x, c = 7u;
    const long long t0 = tick(), r0 = rtick();
    asm volatile("v_cmp_gt_u32 vcc, 32, %1\n" REP64("v_cndmask_b32 %0, %0, %1, vcc\n") : "+v"(a) : "v"(c) : "vcc");
    const long long t1 = tick(), r1 = rtick();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }
    if (a == 12345u) out[2] = 1;
}
__global__ void thr_cndmask(long long* out, double b)
{
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, c = 7u;
    const long long t0 = tick(), r0 = rtick();
    asm volatile("v_cmp_gt_u32 vcc, 32, %8\n" REP8("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n"
                 "v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n"
                 "v_cndmask_b32 %5, %5, %8, vcc\n v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(c) : "vcc");
    const long long t1 = tick(), r1 = rtick();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }
    if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 12345u) out[2] = 1;
}
__global__ void lat_fma(long long* out, double b)
{
    double a = (double)threadIdx.x * 1e-3 + 1.0;
    const long long t0 = tick(), r0 = rtick();
    asm volatile(REP64("v_fma_f64 %0, %0, %1, %1\n") : "+v"(a) : "v"(b));
    const long long t1 = tick(), r1 = rtick();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }
    if (a == 12345.0) out[2] = 1;
}
__global__ void thr_fma(long long* out, double b)
{
    double a0 = threadIdx.x + 1.0, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const long long t0 = tick(), r0 = rtick();
    asm volatile(REP8("v_fma_f64 %0, %0, %8, %8\n v_fma_f64 %1, %1, %8, %8\n v_fma_f64 %2, %2, %8, %8\n v_fma_f64 %3, %3, %8, %8\n"
                      "v_fma_f64 %4, %4, %8, %8\n v_fma_f64 %5, %5, %8, %8\n v_fma_f64 %6, %6, %8, %8\n v_fma_f64 %7, %7, %8, %8\n")
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
    const long long t1 = tick(), r1 = rtick();
    if (threadIdx.x == 0) { out[0] = t1 - t0; out[1] = r1 - r0; }
    if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 12345.0) out[2] = 1;
}

// LDS: 64 x ds_read_b128 (independent addresses, one wait at the end) per wave; with blockDim 64 or 256
__global__ void lds_read128(long long* out, double b)
{
    __shared__ __attribute__((aligned(16))) double buf[4][64 * 16];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    for (int i = l; i < 64 * 16; i += 64) buf[w][i] = i;
    __syncthreads();
    const unsigned addr = (unsigned)(uintptr_t)&buf[w][(l * 2) & 1023];
    double v0, v1;
    const long long t0 = tick(), r0 = rtick();
    asm volatile(REP64("ds_read_b128 v[40:43], %2\n") "s_waitcnt lgkmcnt(0)\n v_mov_b64 %0, v[40:41]\n v_mov_b64 %1, v[42:43]\n"
                 : "=v"(v0), "=v"(v1) : "v"(addr) : "v40", "v41", "v42", "v43");
    const long long t1 = tick(), r1 = rtick();
    if (l == 0) { out[4 * w] = t1 - t0; out[4 * w + 1] = r1 - r0; }
    if (v0 + v1 == 12345.0) out[2] = 1;
}
// LDS round trip: ds_write_b64 then a dependent ds_read_b64 of another lane's slot, 16 times in a chain
__global__ void lds_roundtrip(long long* out, double b)
{
    __shared__ double buf[4][64];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    double v = l;
    const unsigned a0 = (unsigned)(uintptr_t)&buf[w][l], a1 = (unsigned)(uintptr_t)&buf[w][(l + 1) & 63];
    const long long t0 = tick(), r0 = rtick();
    asm volatile(REP8("ds_write_b64 %1, %0\n ds_read_b64 %0, %2\n s_waitcnt lgkmcnt(0)\n ds_write_b64 %1, %0\n ds_read_b64 %0, %2\n s_waitcnt lgkmcnt(0)\n")
                 : "+v"(v) : "v"(a0), "v"(a1));
    const long long t1 = tick(), r1 = rtick();
    if (l == 0) { out[4 * w] = t1 - t0; out[4 * w + 1] = r1 - r0; }
    if (v == 12345.0) out[2] = 1;
}
// ds_bpermute_b32 latency: 16 dependent permutes
__global__ void lds_bperm(long long* out, double b)
{
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    int v = l;
    const int addr = ((l + 5) & 63) * 4;
    const long long t0 = tick(), r0 = rtick();
    asm volatile(REP8("ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)\n ds_bpermute_b32 %0, %1, %0\n s_waitcnt lgkmcnt(0)\n")
                 : "+v"(v) : "v"(addr));
    const long long t1 = tick(), r1 = rtick();
    if (l == 0) { out[4 * w] = t1 - t0; out[4 * w + 1] = r1 - r0; }
    if (v == 12345) out[2] = 1;
}

typedef void (*KFn)(long long*, double);
static void run(const char* name, KFn k, int threads, int ninst, long long* d, long long* h)
{
    for (int rep = 0; rep < 3; rep++) {
        hipMemset(d, 0, 64 * sizeof(long long));
        hipLaunchKernelGGL(k, dim3(1), dim3(threads), 0, 0, d, 1.0000001);
        hipDeviceSynchronize();
    }
    hipMemcpy(h, d, 64 * sizeof(long long), hipMemcpyDeviceToHost);
    const double mhz = h[1] > 0 ? (double)h[0] / ((double)h[1] * 0.01) : 0.0;   // memrealtime: 100 MHz
    printf("%-16s threads %4d  cycles %7lld  per instruction %6.2f  (memtime at %.0f MHz)", name, threads, h[0],
           (double)h[0] / ninst, mhz);
    if (threads > 64) printf("  waves 1..3: %lld %lld %lld", h[4], h[8], h[12]);
    printf("\n");
}

int main()
{
    long long *d, h[64];
    hipMalloc(&d, 64 * sizeof(long long));
    run("lat_add_f64", lat_add_f64, 64, 64, d, h);
    run("thr_add_f64", thr_add_f64, 64, 64, d, h);
    run("lat_mul_f64", lat_mul_f64, 64, 64, d, h);
    run("thr_mul_f64", thr_mul_f64, 64, 64, d, h);
    run("lat_fma_f64", lat_fma, 64, 64, d, h);
    run("thr_fma_f64", thr_fma, 64, 64, d, h);
    run("lat_rcp_f64", lat_rcp_f64, 64, 64, d, h);
    run("thr_rcp_f64", thr_rcp_f64, 64, 64, d, h);
    run("lat_rsq_f64", lat_rsq_f64, 64, 64, d, h);
    run("thr_rsq_f64", thr_rsq_f64, 64, 64, d, h);
    run("lat_cndmask", lat_cndmask, 64, 64, d, h);
    run("thr_cndmask", thr_cndmask, 64, 64, d, h);
    run("lds_read128", lds_read128, 64, 64, d, h);
    run("lds_read128x4", lds_read128, 256, 64, d, h);
    run("lds_roundtrip", lds_roundtrip, 64, 16, d, h);
    run("lds_roundtrip4", lds_roundtrip, 256, 16, d, h);
    run("lds_bperm", lds_bperm, 64, 16, d, h);
    run("lds_bperm4", lds_bperm, 256, 16, d, h);
    hipFree(d);
    return 0;
}

// match.hip -- brute-force Hamming knn-2 on gfx950.
//
// Reference: Matcher::match -> BFMatcher(NORM_HAMMING)::knnMatch(ref, cur, k=2)
//   (Features/Matcher.cpp:13-17, :113).  OpenCV's batchDistance(K=2) keeps, per query, the two
//   smallest distances with a strict '<' insertion while scanning train rows in index order, i.e.
//   the two smallest (distance, train index) pairs in lexicographic order.
//
// One thread per query keeps its 256-bit descriptor in 8 VGPRs; train descriptors stream through
// LDS in 256-row tiles (8 KB) that every lane reads as a broadcast; distance = 8 x (xor + popcount).
#include <hip/hip_runtime.h>
#include <climits>

namespace rgbd {

constexpr int kKnnThreads = 256;

// pairs p: query frame qf[p] vs train frame tf[p] of a descriptor array desc[frame][kp_cap][32]
// with counts[frame]; out[p][kp_cap] = {d1, i1, d2, i2}
__global__ __launch_bounds__(kKnnThreads) void k_knn2(const uint8_t* __restrict__ desc, const int* __restrict__ counts,
                                                      const int* __restrict__ qf, const int* __restrict__ tf,
                                                      int kp_cap, int4* __restrict__ out)
{
    __shared__ uint4 tile[kKnnThreads * 2];
    const int p = blockIdx.y;
    const int qframe = qf[p], tframe = tf[p];
    const int nq = counts[qframe], nt = counts[tframe];
    const int q0 = blockIdx.x * kKnnThreads;
    if (q0 >= nq)
        return;   // uniform per block
    const int tid = threadIdx.x;
    const int q = q0 + tid;
    uint4 qa = make_uint4(0, 0, 0, 0), qb = make_uint4(0, 0, 0, 0);
    const uint4* qd = reinterpret_cast<const uint4*>(desc + (size_t)qframe * kp_cap * 32);
    if (q < nq) {
        qa = qd[2 * q];
        qb = qd[2 * q + 1];
    }
    const uint4* td = reinterpret_cast<const uint4*>(desc + (size_t)tframe * kp_cap * 32);
    int d1 = INT_MAX, i1 = -1, d2 = INT_MAX, i2 = -1;
    for (int base = 0; base < nt; base += kKnnThreads) {
        __syncthreads();
        if (base + tid < nt) {
            tile[2 * tid] = td[2 * (base + tid)];
            tile[2 * tid + 1] = td[2 * (base + tid) + 1];
        }
        __syncthreads();
        const int cnt = min(kKnnThreads, nt - base);
        for (int j = 0; j < cnt; j++) {
            const uint4 ta = tile[2 * j], tb = tile[2 * j + 1];
            const int d = __popc(qa.x ^ ta.x) + __popc(qa.y ^ ta.y) + __popc(qa.z ^ ta.z) + __popc(qa.w ^ ta.w)
                          + __popc(qb.x ^ tb.x) + __popc(qb.y ^ tb.y) + __popc(qb.z ^ tb.z) + __popc(qb.w ^ tb.w);
            if (d < d2) {
                if (d < d1) {
                    d2 = d1; i2 = i1;
                    d1 = d; i1 = base + j;
                } else {
                    d2 = d; i2 = base + j;
                }
            }
        }
    }
    if (q < nq)
        out[(size_t)p * kp_cap + q] = make_int4(d1, i1, d2, i2);
}

}  // namespace rgbd

#include "launch.h"
namespace rgbd {
void launch_knn2(const uint8_t* desc, const int* counts, const int* qf, const int* tf, int kp_cap, int max_q,
                 int4* out, int npairs, hipStream_t st)
{
    hipLaunchKernelGGL(k_knn2, dim3((max_q + kKnnThreads - 1) / kKnnThreads, npairs), dim3(kKnnThreads), 0, st,
                       desc, counts, qf, tf, kp_cap, out);
}
}  // namespace rgbd

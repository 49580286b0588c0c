// match.hip -- brute-force Hamming knn-2 on gfx950.
//
// Reference: Matcher::match -> BFMatcher(NORM_HAMMING)::knnMatch(ref, cur, k=2)
//   (Features/Matcher.cpp:13-17, :113).  OpenCV's batchDistance(K=2) keeps, per query, the two
//   smallest distances with a strict '<' insertion while scanning train rows in index order, i.e.
//   the two smallest (distance, train index) pairs in lexicographic order.
//
// One lane per query keeps its 256-bit descriptor in 8 VGPRs; the train rows are split over four
// waves, staged in LDS and read as broadcasts; distance = 8 x (xor + popcount).
#include <hip/hip_runtime.h>
#include <climits>

namespace rgbd {

constexpr int kKnnQ = 64;                 // queries per workgroup (one per lane)
constexpr int kKnnSplit = 4;              // waves per workgroup, each scanning a quarter of the train rows
constexpr int kKnnThreads = kKnnQ * kKnnSplit;

// lexicographic (distance, index) top-2 insert; scanning train rows in increasing index with a
// strict '<' is exactly this order, so per-range top-2 lists merge into the global one
__device__ __forceinline__ void top2_insert(int d, int i, int& d1, int& i1, int& d2, int& i2)
{
    const bool lt1 = d < d1 || (d == d1 && i < i1);
    const bool lt2 = d < d2 || (d == d2 && i < i2);
    if (lt1) {
        d2 = d1; i2 = i1;
        d1 = d; i1 = i;
    } else if (lt2) {
        d2 = d; i2 = i;
    }
}

// pairs p: query frame qf[p] vs train frame tf[p] of a descriptor array desc[frame][kp_cap][32]
// with counts[frame]; out[p][kp_cap] = {d1, i1, d2, i2}.  Lane = query (256 bits in 8 VGPRs);
// wave w scans train rows [w n / 4, (w + 1) n / 4), staged in its own LDS slice and read as
// broadcasts; the four partial top-2 lists merge in LDS.
__global__ __launch_bounds__(kKnnThreads) void k_knn2(const uint8_t* __restrict__ desc, const int* __restrict__ counts,
                                                      const int* __restrict__ qf, const int* __restrict__ tf,
                                                      int kp_cap, int4* __restrict__ out)
{
    __shared__ int4 part[kKnnSplit][kKnnQ];
    const int p = blockIdx.y;
    const int qframe = qf[p], tframe = tf[p];
    const int nq = counts[qframe], nt = counts[tframe];
    const int q0 = blockIdx.x * kKnnQ;
    if (q0 >= nq)
        return;   // uniform per block
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
    const int q = q0 + lane;
    uint4 qa = make_uint4(0, 0, 0, 0), qb = make_uint4(0, 0, 0, 0);
    const uint4* qd = reinterpret_cast<const uint4*>(desc + (size_t)qframe * kp_cap * 32);
    if (q < nq) {
        qa = qd[2 * q];
        qb = qd[2 * q + 1];
    }
    const uint4* td = reinterpret_cast<const uint4*>(desc + (size_t)tframe * kp_cap * 32);
    const int t_lo = (int)(((long)nt * w) / kKnnSplit), t_hi = (int)(((long)nt * (w + 1)) / kKnnSplit);
    // the wave's train rows -> its own LDS slice with coalesced 16-B loads (all in flight at once),
    // then every row is a broadcast ds_read_b128 pair
    extern __shared__ uint4 trow_all[];
    const int rpw = (kp_cap + kKnnSplit - 1) / kKnnSplit;   // rows per wave slice
    uint4* tr = trow_all + (size_t)w * rpw * 2;
    {
        const int n16 = 2 * (t_hi - t_lo);
        const uint4* src = td + 2 * t_lo;
        constexpr int kBatch = 8;
        for (int i0 = 0; i0 < n16; i0 += 64 * kBatch) {
            uint4 v[kBatch];
#pragma unroll
            for (int u = 0; u < kBatch; u++) {
                const int i = i0 + u * 64 + lane;
                if (i < n16) v[u] = src[i];
            }
#pragma unroll
            for (int u = 0; u < kBatch; u++) {
                const int i = i0 + u * 64 + lane;
                if (i < n16) tr[i] = v[u];
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    int d1 = INT_MAX, i1 = INT_MAX, d2 = INT_MAX, i2 = INT_MAX;
    auto dist = [&](const uint4& ta, const uint4& tb) {
        return __popc(qa.x ^ ta.x) + __popc(qa.y ^ ta.y) + __popc(qa.z ^ ta.z) + __popc(qa.w ^ ta.w)
               + __popc(qb.x ^ tb.x) + __popc(qb.y ^ tb.y) + __popc(qb.z ^ tb.z) + __popc(qb.w ^ tb.w);
    };
    auto insert = [&](int d, int j) {   // strict '<' in index order (j increases), branch-free
        const bool lt1 = d < d1, lt2 = d < d2;
        d2 = lt1 ? d1 : (lt2 ? d : d2);
        i2 = lt1 ? i1 : (lt2 ? j : i2);
        d1 = lt1 ? d : d1;
        i1 = lt1 ? j : i1;
    };
#pragma unroll 4
    for (int j = t_lo; j < t_hi; j++) {
        const int r = j - t_lo;
        insert(dist(tr[2 * r], tr[2 * r + 1]), j);
    }
    part[w][lane] = make_int4(d1, i1, d2, i2);
    __syncthreads();
    if (w == 0 && q < nq) {
        int e1 = INT_MAX, j1 = INT_MAX, e2 = INT_MAX, j2 = INT_MAX;
#pragma unroll
        for (int k = 0; k < kKnnSplit; k++) {
            const int4 r = part[k][lane];
            if (r.y != INT_MAX) top2_insert(r.x, r.y, e1, j1, e2, j2);
            if (r.w != INT_MAX) top2_insert(r.z, r.w, e1, j1, e2, j2);
        }
        out[(size_t)p * kp_cap + q] = make_int4(e1, j1 == INT_MAX ? -1 : j1, e2, j2 == INT_MAX ? -1 : j2);
    }
}

}  // namespace rgbd

#include "launch.h"
namespace rgbd {
void launch_knn2(const uint8_t* desc, const int* counts, const int* qf, const int* tf, int kp_cap, int max_q,
                 int4* out, int npairs, hipStream_t st)
{
    const size_t lds = (size_t)kKnnSplit * ((kp_cap + kKnnSplit - 1) / kKnnSplit) * 32;
    hipLaunchKernelGGL(k_knn2, dim3((max_q + kKnnQ - 1) / kKnnQ, npairs), dim3(kKnnThreads), lds, st,
                       desc, counts, qf, tf, kp_cap, out);
}
}  // namespace rgbd

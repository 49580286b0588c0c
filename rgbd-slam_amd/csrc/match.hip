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

// pairs p: query frame qf[p] vs train frame tf[p] of a descriptor array desc[frame][kp_cap][32]
// with counts[frame]; out[p][kp_cap] = {d1, i1, d2, i2}.  Lane = query (256 bits in 8 VGPRs);
// wave w scans train rows [w n / 4, (w + 1) n / 4), staged in its own LDS slice and read as
// broadcasts; the four partial top-2 lists merge in LDS.
__global__ __launch_bounds__(kKnnThreads) void k_knn2(const uint8_t* __restrict__ desc, const int* __restrict__ counts,
                                                      const int* __restrict__ qf, const int* __restrict__ tf,
                                                      int kp_cap, int4* __restrict__ out)
{
    __shared__ uint2 part[kKnnSplit][kKnnQ];
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
    // top-2 as packed keys (distance << 16 | train index): rows arrive in increasing index, so the
    // reference's strict '<' on distance is exactly '<' on the key, and the insert is min / max
    unsigned k1 = UINT_MAX, k2 = UINT_MAX;
    auto dist = [&](const uint4& ta, const uint4& tb) {
        return __popc(qa.x ^ ta.x) + __popc(qa.y ^ ta.y) + __popc(qa.z ^ ta.z) + __popc(qa.w ^ ta.w)
               + __popc(qb.x ^ tb.x) + __popc(qb.y ^ tb.y) + __popc(qb.z ^ tb.z) + __popc(qb.w ^ tb.w);
    };
    auto insert = [&](unsigned k) {
        k2 = min(k2, max(k1, k));
        k1 = min(k1, k);
    };
    constexpr int U = 4;   // rows per step: their LDS reads are issued together
    const int nr = t_hi - t_lo;
    int r = 0;
    for (; r + U <= nr; r += U) {
        uint4 ta[U], tb[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            ta[u] = tr[2 * (r + u)];
            tb[u] = tr[2 * (r + u) + 1];
        }
#pragma unroll
        for (int u = 0; u < U; u++) insert(((unsigned)dist(ta[u], tb[u]) << 16) | (unsigned)(t_lo + r + u));
    }
    for (; r < nr; r++) insert(((unsigned)dist(tr[2 * r], tr[2 * r + 1]) << 16) | (unsigned)(t_lo + r));
    part[w][lane] = make_uint2(k1, k2);
    __syncthreads();
    if (w == 0 && q < nq) {
        unsigned e1 = UINT_MAX, e2 = UINT_MAX;
#pragma unroll
        for (int k = 0; k < kKnnSplit; k++) {
            const uint2 pk = part[k][lane];
            e2 = min(e2, max(e1, pk.x));
            e1 = min(e1, pk.x);
            e2 = min(e2, max(e1, pk.y));
            e1 = min(e1, pk.y);
        }
        auto dd = [](unsigned e) { return e == UINT_MAX ? INT_MAX : (int)(e >> 16); };
        auto ii = [](unsigned e) { return e == UINT_MAX ? -1 : (int)(e & 0xFFFFu); };
        out[(size_t)p * kp_cap + q] = make_int4(dd(e1), ii(e1), dd(e2), ii(e2));
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

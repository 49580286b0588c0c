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

// ---------------------------------------------------------------- knn-2 on the matrix cores
// Hamming(q, t) = |q| + |t| - 2 q.t over the 256 descriptor bits as 0/1 bytes: the q.t of a 32-train x
// 32-query tile is one v_mfma_i32_32x32x32_i8 per 32 bits (8 per tile), with the trains as A (rows) and
// the queries as B (columns), so D's column is the lane's query and its 16 registers are 16 trains of the
// tile: the top-2 stays per lane (4 VALU per candidate instead of xor + popcount).  The two operands use
// the same byte order (bit 16h + e of dword s in element e of lane half h, i.e. expanded byte 32s + 16h + e),
// so the MFMA's internal k permutation cancels out of the dot product.
// The rank key per query is ((|t| - 2 q.t + 256) << 16 | t), the reference's (distance, index) order
// (|q| is the same for every train); the distance adds |q| - 256 back.
typedef int knn_v4i __attribute__((ext_vector_type(4)));
typedef int knn_v16i __attribute__((ext_vector_type(16)));
constexpr int kKmWaves = 4;                 // waves per workgroup, one 32-query tile each
constexpr int kKmQ = 32 * kKmWaves;         // queries per workgroup
constexpr int kKmRow = 272;                 // LDS bytes per staged train row: 256 + 16 (bank spread for b128 reads)

// desc [frame][kp_cap][32] bits -> desc8 [frame][kp_cap][256] 0/1 bytes (byte b = bit b), rows < count
__global__ __launch_bounds__(256) void k_desc_expand(const uint8_t* __restrict__ desc, const int* __restrict__ counts,
                                                     int kp_cap, int nframes, uint8_t* __restrict__ desc8)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;   // (frame, row, dword)
    const size_t n = (size_t)nframes * kp_cap * 8;
    if (i >= n) return;
    const int f = (int)(i / ((size_t)kp_cap * 8)), r = (int)((i / 8) % kp_cap);
    if (r >= counts[f]) return;
    const uint32_t x = reinterpret_cast<const uint32_t*>(desc)[i];
    uint32_t o[8];
#pragma unroll
    for (int k = 0; k < 8; k++) o[k] = (((x >> (4 * k)) & 0xFu) * 0x00204081u) & 0x01010101u;
    uint4* dst = reinterpret_cast<uint4*>(desc8 + i * 32);
    dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
    dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
}

__global__ __launch_bounds__(64 * kKmWaves) void k_knn2m(const uint8_t* __restrict__ desc, const uint8_t* __restrict__ desc8,
                                                         const int* __restrict__ counts, const int* __restrict__ qf,
                                                         const int* __restrict__ tf, int kp_cap, int4* __restrict__ out)
{
    __shared__ __attribute__((aligned(16))) uint8_t tile[2][32 * kKmRow];
    __shared__ unsigned tkey[2][32];
    const int p = blockIdx.y;
    const int qframe = qf[p], tframe = tf[p];
    const int nq = counts[qframe], nt = counts[tframe];
    const int q0 = blockIdx.x * kKmQ;
    if (q0 >= nq) return;   // uniform per block
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 31, h = lane >> 5;
    const int q = q0 + 32 * w + c;
    const int qr = q < nq ? q : nq - 1;   // tail lanes repeat a valid query (results not stored)
    // this lane's query: B fragments of the 8 k-steps and |q|
    knn_v4i bq[8];
    {
        const knn_v4i* row = reinterpret_cast<const knn_v4i*>(desc8 + ((size_t)qframe * kp_cap + qr) * 256);
#pragma unroll
        for (int s = 0; s < 8; s++) bq[s] = row[2 * s + h];
    }
    int pq = 0;
    {
        const uint4* rq = reinterpret_cast<const uint4*>(desc + ((size_t)qframe * kp_cap + qr) * 32);
        const uint4 a = rq[0], b = rq[1];
        pq = __popc(a.x) + __popc(a.y) + __popc(a.z) + __popc(a.w) + __popc(b.x) + __popc(b.y) + __popc(b.z) + __popc(b.w);
    }
    const uint8_t* t8 = desc8 + (size_t)tframe * kp_cap * 256;
    const uint8_t* traw = desc + (size_t)tframe * kp_cap * 32;
    // staging: thread = (train row tid / 8, 32-byte part tid % 8) of a 32-train tile
    const int sr = tid >> 3, sp = tid & 7;
    auto stage = [&](int t0, int buf) {
        const int t = t0 + sr;
        uint4 v0 = make_uint4(0, 0, 0, 0), v1 = v0;
        if (t < nt) {
            const uint4* src = reinterpret_cast<const uint4*>(t8 + (size_t)t * 256 + 32 * sp);
            v0 = src[0];
            v1 = src[1];
        }
        uint4* dst = reinterpret_cast<uint4*>(&tile[buf][sr * kKmRow + 32 * sp]);
        dst[0] = v0;
        dst[1] = v1;
        if (sp == 0) {
            unsigned k = 0xFFFFFFFFu;   // rows past nt: never selected
            if (t < nt) {
                const uint4* rt = reinterpret_cast<const uint4*>(traw + (size_t)t * 32);
                const uint4 a = rt[0], b = rt[1];
                const int pt = __popc(a.x) + __popc(a.y) + __popc(a.z) + __popc(a.w) + __popc(b.x) + __popc(b.y) +
                               __popc(b.z) + __popc(b.w);
                k = ((unsigned)(pt + 256) << 16) | (unsigned)t;
            }
            tkey[buf][sr] = k;
        }
    };
    unsigned k1 = 0xFFFFFFFFu, k2 = 0xFFFFFFFFu;
    const int ntiles = (nt + 31) >> 5;
    if (ntiles > 0) stage(0, 0);
    __syncthreads();
    for (int it = 0; it < ntiles; it++) {
        const int buf = it & 1;
        if (it + 1 < ntiles) stage(32 * (it + 1), buf ^ 1);   // the next tile lands while this one computes
        knn_v16i acc = {};
        const uint8_t* arow = &tile[buf][c * kKmRow + 16 * h];
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const knn_v4i a = *reinterpret_cast<const knn_v4i*>(arow + 32 * s);
            acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, bq[s], acc, 0, 0, 0);
        }
        // register j holds train row (j & 3) + 8 (j >> 2) + 4 h of the tile
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const uint4 tk = *reinterpret_cast<const uint4*>(&tkey[buf][8 * g + 4 * h]);
            const unsigned tks[4] = {tk.x, tk.y, tk.z, tk.w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
                const unsigned key = tks[e] == 0xFFFFFFFFu ? tks[e] : tks[e] - ((unsigned)acc[4 * g + e] << 17);
                k2 = min(k2, max(k1, key));
                k1 = min(k1, key);
            }
        }
        __syncthreads();   // this tile's buffer is free; the next one is staged
    }
    // the two lane halves hold different trains of the same query
    const unsigned o1 = __shfl_xor(k1, 32, 64), o2 = __shfl_xor(k2, 32, 64);
    k2 = min(k2, max(k1, o1));
    k1 = min(k1, o1);
    k2 = min(k2, max(k1, o2));
    k1 = min(k1, o2);
    if (h == 0 && q < nq) {
        auto dd = [&](unsigned e) { return e == 0xFFFFFFFFu ? INT_MAX : (int)(e >> 16) - 256 + pq; };
        auto ii = [](unsigned e) { return e == 0xFFFFFFFFu ? -1 : (int)(e & 0xFFFFu); };
        out[(size_t)p * kp_cap + q] = make_int4(dd(k1), ii(k1), dd(k2), ii(k2));
    }
}

}  // namespace rgbd

#include "launch.h"
namespace rgbd {
#ifndef RGBD_KNN_MFMA
#define RGBD_KNN_MFMA 1
#endif
void launch_knn2(const uint8_t* desc, const int* counts, const int* qf, const int* tf, int kp_cap, int max_q,
                 int4* out, int npairs, hipStream_t st, uint8_t* desc8, int nframes)
{
    if (RGBD_KNN_MFMA && desc8 && nframes >= 0) {   // expand the frames' descriptors, then the matrix-core knn-2
        const size_t n = (size_t)nframes * kp_cap * 8;
        if (n > 0)
            hipLaunchKernelGGL(k_desc_expand, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, desc, counts, kp_cap,
                               nframes, desc8);
        hipLaunchKernelGGL(k_knn2m, dim3((max_q + kKmQ - 1) / kKmQ, npairs), dim3(64 * kKmWaves), 0, st, desc, desc8,
                           counts, qf, tf, kp_cap, out);
        return;
    }
    const size_t lds = (size_t)kKnnSplit * ((kp_cap + kKnnSplit - 1) / kKnnSplit) * 32;
    hipLaunchKernelGGL(k_knn2, dim3((max_q + kKnnQ - 1) / kKnnQ, npairs), dim3(kKnnThreads), lds, st,
                       desc, counts, qf, tf, kp_cap, out);
}
}  // namespace rgbd

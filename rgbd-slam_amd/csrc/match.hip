// match.hip -- brute-force Hamming knn-2 on gfx950.
//
// Reference: Matcher::match -> BFMatcher(NORM_HAMMING)::knnMatch(ref, cur, k=2)
//   (Features/Matcher.cpp:13-17, :113).  OpenCV's batchDistance(K=2) keeps, per query, the two
//   smallest distances with a strict '<' insertion while scanning train rows in index order, i.e.
//   the two smallest (distance, train index) pairs in lexicographic order.
//
// The Hamming distances run on the matrix cores (k_knn2m below).  An xor + popcount form (one lane per
// query, 20 VALU per pair) measured 0.63 ms vs 0.27 ms per 1023 pairs and was removed (round 3).
#include <hip/hip_runtime.h>

#include "dispatch.h"
#include <climits>

namespace rgbd {


// ---------------------------------------------------------------- knn-2 on the matrix cores
// Hamming(q, t) = |q| + |t| - 2 q.t over the 256 descriptor bits: the q.t of a 32-train x 32-query tile is
// one v_mfma_i32_32x32x32_i8 per 32 bits (8 per tile) with the trains as A (rows, 0/1 bytes) and the
// queries as B (columns, 0/-1 bytes, so the accumulator is -q.t).  D's column is the lane's query and its
// 16 registers are 16 trains of the tile, so the top-2 stays per lane.  Both operands put bit 16h + e of
// descriptor dword s in element e of lane half h, so the MFMA's internal k order cancels out of the dot
// product.  The rank key per query is ((|t| + 256 - 2 q.t) << 16 | t) = tkey + (acc << 17) (one
// v_lshl_add), the reference's (distance, index) order since |q| is the same for every train; the
// distance adds |q| - 256 back.  Trains are staged per 32-row tile as raw bits (1 KB, one dword per
// thread, loaded three tiles ahead) and expanded into the LDS tile as bytes (256 B rows padded to 272
// for conflict-free b128 fragment reads); rows past the train count are zero, so their key stays
// 0xFFFFFFFF (never selected).
typedef int knn_v4i __attribute__((ext_vector_type(4)));
typedef int knn_v16i __attribute__((ext_vector_type(16)));
#define RGBD_KNN_QT 2
#define RGBD_KNN_WAVES 4
constexpr int kKmWaves = RGBD_KNN_WAVES;    // waves per workgroup (the first four stage the train tiles; 8 waves x 2 / 1 query tiles: 180.5k / 181.4k vs 182.8k)
static_assert(kKmWaves >= 4, "k_knn2m stages a 32-row train tile with 256 threads");
constexpr int kKmQT = RGBD_KNN_QT;          // 32-query tiles per wave (each staged train tile serves all)
constexpr int kKmQ = 32 * kKmQT * kKmWaves; // queries per workgroup
constexpr int kKmRow = 272;                 // LDS bytes per staged train row: 256 + 16 (bank spread for b128 reads)
constexpr int kKmAhead = 3;                 // tiles of raw train bits in flight per thread

__device__ __forceinline__ unsigned med3_u32(unsigned a, unsigned b, unsigned c)
{
    unsigned d;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

__device__ __forceinline__ uint32_t nibble_bytes(uint32_t x, int k)   // bits 4k..4k+3 -> bytes 0/1
{
    return (((x >> (4 * k)) & 0xFu) * 0x00204081u) & 0x01010101u;
}

__global__ __launch_bounds__(64 * kKmWaves) void k_knn2m(const uint8_t* __restrict__ desc, const int* __restrict__ counts,
                                                         const int* __restrict__ qf, const int* __restrict__ tf,
                                                         int kp_cap, int4* __restrict__ out)
{
    __shared__ __attribute__((aligned(16))) uint8_t tile[2][32 * kKmRow];
    __shared__ unsigned tkey[2][32];
    const int p = blockIdx.y;
    const int qframe = qf[p], tframe = tf[p];
    if (qframe < 0) return;   // pair not requested (second-reference rows of the lane chain)
    const int nq = counts[qframe], nt = counts[tframe];
    const int q0 = blockIdx.x * kKmQ;
    if (q0 >= nq) return;   // uniform per block
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int c = lane & 31, h = lane >> 5;
    const int qw = q0 + 32 * kKmQT * w;   // the wave's first query
    // this lane's queries (one per tile): B fragments (bit 16h + e of dword s -> byte e, 0 / -1) and |q|;
    // tail lanes repeat a valid query (results not stored)
    knn_v4i bq[kKmQT][8];
    int pq[kKmQT];
#pragma unroll
    for (int u = 0; u < kKmQT; u++) {
        const int q = qw + 32 * u + c;
        const int qr = q < nq ? q : nq - 1;
        const uint4* rq = reinterpret_cast<const uint4*>(desc + ((size_t)qframe * kp_cap + qr) * 32);
        const uint4 a = rq[0], b = rq[1];
        const uint32_t d[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        pq[u] = 0;
#pragma unroll
        for (int s = 0; s < 8; s++) {
            pq[u] += __popc(d[s]);
            const uint32_t x = d[s] >> (16 * h);
#pragma unroll
            for (int k = 0; k < 4; k++) bq[u][s][k] = (int)(nibble_bytes(x, k) * 0xFFu);
        }
    }
    // staging: thread = (train row tid / 8, descriptor dword tid % 8) of a 32-train tile
    const int sr = tid >> 3, sd = tid & 7;
    const uint32_t* traw = reinterpret_cast<const uint32_t*>(desc + (size_t)tframe * kp_cap * 32);
    auto fetch = [&](int t0) -> uint32_t { const int t = t0 + sr; return t < nt ? traw[(size_t)t * 8 + sd] : 0u; };
    auto stage = [&](uint32_t x, int t0, int buf) {
        uint32_t o[8];
#pragma unroll
        for (int k = 0; k < 8; k++) o[k] = nibble_bytes(x, k);
        uint4* dst = reinterpret_cast<uint4*>(&tile[buf][sr * kKmRow + 32 * sd]);
        dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
        dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
        int pc = __popc(x);   // |t| over the row's 8 threads (consecutive lanes)
        pc += __shfl_xor(pc, 1, 8);
        pc += __shfl_xor(pc, 2, 8);
        pc += __shfl_xor(pc, 4, 8);
        const int t = t0 + sr;
        if (sd == 0) tkey[buf][sr] = t < nt ? ((unsigned)(pc + 256) << 16) | (unsigned)t : 0xFFFFFFFFu;
    };
    unsigned k1[kKmQT], k2[kKmQT];
#pragma unroll
    for (int u = 0; u < kKmQT; u++) k1[u] = k2[u] = 0xFFFFFFFFu;
    const int ntiles = (nt + 31) >> 5;
    uint32_t ring[kKmAhead];
#pragma unroll
    for (int i = 0; i < kKmAhead; i++) ring[i] = fetch(32 * (i + 1));
    const bool stager = tid < 256;   // whole waves
    if (ntiles > 0 && stager) stage(fetch(0), 0, 0);
    __syncthreads();
    for (int it = 0; it < ntiles; it++) {
        const int buf = it & 1;
        if (it + 1 < ntiles && stager) stage(ring[0], 32 * (it + 1), buf ^ 1);   // expand the next tile into the other buffer
#pragma unroll
        for (int i = 0; i + 1 < kKmAhead; i++) ring[i] = ring[i + 1];
        ring[kKmAhead - 1] = fetch(32 * (it + 1 + kKmAhead));
        knn_v16i acc[kKmQT];
#pragma unroll
        for (int u = 0; u < kKmQT; u++) acc[u] = knn_v16i{};
        const uint8_t* arow = &tile[buf][c * kKmRow + 16 * h];
#pragma unroll
        for (int s = 0; s < 8; s++) {
            const knn_v4i av = *reinterpret_cast<const knn_v4i*>(arow + 32 * s);
#pragma unroll
            for (int u = 0; u < kKmQT; u++) acc[u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bq[u][s], acc[u], 0, 0, 0);
        }
        // register j holds train row (j & 3) + 8 (j >> 2) + 4 h of the tile; candidates merged in sorted pairs
#pragma unroll
        for (int g = 0; g < 4; g++) {
            const uint4 tk = *reinterpret_cast<const uint4*>(&tkey[buf][8 * g + 4 * h]);
#pragma unroll
            for (int u = 0; u < kKmQT; u++) {
                const unsigned e[4] = {tk.x + ((unsigned)acc[u][4 * g + 0] << 17), tk.y + ((unsigned)acc[u][4 * g + 1] << 17),
                                       tk.z + ((unsigned)acc[u][4 * g + 2] << 17), tk.w + ((unsigned)acc[u][4 * g + 3] << 17)};
                // insertion of one key into the sorted pair k1 <= k2: the new second is the median of the three
                // (one v_med3_u32), the new first the minimum
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    k2[u] = med3_u32(k1[u], k2[u], e[i]);
                    k1[u] = min(k1[u], e[i]);
                }
            }
        }
        __syncthreads();   // this tile's buffer is free; the next one is staged
    }
    // the two lane halves hold different trains of the same query
#pragma unroll
    for (int u = 0; u < kKmQT; u++) {
        const unsigned o1 = __shfl_xor(k1[u], 32, 64), o2 = __shfl_xor(k2[u], 32, 64);
        const unsigned m2 = min(min(max(k1[u], o1), k2[u]), o2), m1 = min(k1[u], o1);
        const int q = qw + 32 * u + c;
        if (h == 0 && q < nq) {
            auto dd = [&](unsigned e) { return e == 0xFFFFFFFFu ? INT_MAX : (int)(e >> 16) - 256 + pq[u]; };
            auto ii = [](unsigned e) { return e == 0xFFFFFFFFu ? -1 : (int)(e & 0xFFFFu); };
            out[(size_t)p * kp_cap + q] = make_int4(dd(m1), ii(m1), dd(m2), ii(m2));
        }
    }
}

}  // namespace rgbd

#include "launch.h"
namespace rgbd {
hipError_t launch_knn2(const uint8_t* desc, const int* counts, const int* qf, const int* tf, int kp_cap, int max_q,
                 int4* out, int npairs, hipStream_t st)
{
    return dispatch(k_knn2m, dim3((max_q + kKmQ - 1) / kKmQ, npairs), dim3(64 * kKmWaves), 0, st, desc, counts, qf,
                       tf, kp_cap, out);
}
}  // namespace rgbd

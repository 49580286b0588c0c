// lanes.hip -- the per-round lane kernels of the device-resident RansacSE3 tracking chain (lanes_dev.h).
//
// Reference: Tracking::visualOdometry (System/Tracking.cpp:121-163) -> Matcher::match (Features/Matcher.cpp:
// 106-139) -> RansacSE3::compute (Solver/SolverSE3.cpp:23-159) -> second reference -> Gicp (Solver/Gicp.cpp).
// Every step is the oracle's restatement (oracle/orc_solver.cpp) evaluated on the device:
//   * the Matcher filter (ratio in float, first query wins per train index, ref outlier flag, both depths
//     valid) as a parallel first-wins reduction (atomicMin of the query index per train index) and an
//     ordered compaction: a train index is claimed only by a query that passes every test, so the kept
//     set is exactly "the smallest passing query per train index", in query order;
//   * std::sort(vUsedMatches) (DMatch::operator< on the distance, libstdc++ introsort: median-of-3 pivot,
//     unguarded Hoare partition, depth limit 2 lg n with the heap-sort fallback, final insertion sort).
//     The Hoare partition is evaluated in parallel (the k-th left stopper of the ORIGINAL range swaps with
//     the k-th right stopper while it lies before it, see k_svo_select); the segments of one recursion
//     level are partitioned concurrently, one wave each; since every left part is <= and every right part
//     >= its pivot and insertion sort is stable, the final insertion sort equals a stable sort of each
//     leaf segment (<= 16 elements, or a heap-sorted segment, which is already sorted);
//   * sampleMatches: glibc random_r TYPE_3 and Random::randomInt restated, on one lane, for every
//     hypothesis, with the cumulative rand() count after each, so the replay can leave the RNG exactly where
//     the reference's loop leaves it.
#include <hip/hip_runtime.h>

#include "dispatch.h"

#include <climits>

#include "lanes_dev.h"
#include "lane_replay_dev.h"

#include <cstdio>
#include <cstring>

#ifdef RGBD_PNP_PROFILE
// lane 0's k_lane_match block, wall-clock (10 ns) per stage summed over the call (0: calls, 1 filter,
// 2 compaction, 3 outlier marks, 4 sort, 5 gather, 6 sticky + samples)
__device__ long long g_lm_prof[8];
__device__ long long g_sort_prof[20];   // lane 0's sort: wall-clock per recursion level (0-15), 16 = leaves, 17 = levels seen
__device__ long long g_wp_prof[8];   // k_lane_match block 0's wave partitions: [1-4] wave_partition2 stages, [5] calls, [6] elements
__device__ long long g_sort_seg[16][4];   // per level: segments, of them > 64, heap-sort ones (depth 0), max length
#define LM_PROF(k) do { if (lprof) { const long long t_ = wall_clock64(); g_lm_prof[(k)] += t_ - t_prev; t_prev = t_; } } while (0)
#else
#define LM_PROF(k) do { } while (0)
#endif

namespace rgbd {

namespace {

// inclusive wave64 scan on DPP (row_shr 1/2/4/8 within 16-lane rows, then row_bcast 15 / 31)
__device__ __forceinline__ int wave_incl_scan(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
    return v;
}

// the minimum over the wave (wave-uniform): an inclusive min scan on DPP (lanes without a source see INT_MAX),
// read from lane 63 -- six VALU steps instead of six dependent ds_bpermute round trips
__device__ __forceinline__ int wave_min_i(int v)
{
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x142, 0xa, 0xf, false));   // row_bcast:15 into rows 1, 3
    v = min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, 0x143, 0xc, 0xf, false));   // row_bcast:31 into rows 2, 3
    return __builtin_amdgcn_readlane(v, 63);
}

__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- std::sort of the matches by distance
// Elements are u32 keys (distance << 16 | payload), compared by the distance alone (DMatch::operator<).
__device__ __forceinline__ uint32_t kd(uint32_t k) { return k >> 16; }

__device__ __forceinline__ void kswap(uint32_t* a, int i, int j)
{
    const uint32_t t = a[i];
    a[i] = a[j];
    a[j] = t;
}

// std::__move_median_to_first(result, a, b, c) with comp = less (one lane)
__device__ void median_to_first(uint32_t* a, int result, int x, int y, int z)
{
    if (kd(a[x]) < kd(a[y])) {
        if (kd(a[y]) < kd(a[z])) kswap(a, result, y);
        else if (kd(a[x]) < kd(a[z])) kswap(a, result, z);
        else kswap(a, result, x);
    } else if (kd(a[x]) < kd(a[z])) kswap(a, result, x);
    else if (kd(a[y]) < kd(a[z])) kswap(a, result, z);
    else kswap(a, result, y);
}

// libstdc++ __adjust_heap + __push_heap, comp = less (one lane)
__device__ void adjust_heap(uint32_t* a, int first, int hole, int len, uint32_t v)
{
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (kd(a[first + child]) < kd(a[first + child - 1])) child--;
        a[first + hole] = a[first + child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        a[first + hole] = a[first + child - 1];
        hole = child - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && kd(a[first + parent]) < kd(v)) {
        a[first + hole] = a[first + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    a[first + hole] = v;
}

// std::__partial_sort(first, last, last): __make_heap then __sort_heap (one lane)
__device__ void heap_sort(uint32_t* a, int first, int last)
{
    const int len = last - first;
    if (len < 2) return;
    for (int parent = (len - 2) / 2;; parent--) {
        adjust_heap(a, first, parent, len, a[first + parent]);
        if (parent == 0) break;
    }
    for (int l = last; l - first > 1;) {
        --l;   // __pop_heap(first, l, l)
        const uint32_t v = a[l];
        a[l] = a[first];
        adjust_heap(a, first, 0, l - first, v);
    }
}

// The introsort recursion of one segment [f, f + n), 16 < n <= 64, by one wave with the elements in registers
// (lane i holds position f + i): every segment of a recursion level partitioned at once, each exactly as
// wave_partition2 does it, with two dependent cross-lane rounds per recursion step and no bit selects:
// the segment's first element is read beside the three median candidates, so the median's value (the pivot) and
// the swapped array are known without reading them back; the stoppers' rank -> lane tables go through the
// wave's LDS scratch (index first + rank: the segments of a wave are disjoint), so each partner, LK and RK1 is
// one LDS read instead of a 6-step bit select over the ballot masks (the round-5 form, 4 rounds per step).
// Segments that reach <= 16 elements become leaves; a segment whose depth budget runs out with more is handed back
// to the level lists (heap sort).  tl / tr: >= 64 entries of the wave's own scratch.
__device__ void wave_sort_small2(uint32_t* a, int f, int n, int depth, uint32_t* leaf, int4* push, int* npush,
                                 uint16_t* tl, uint16_t* tr)
{
    const int lane = threadIdx.x & 63;
    const bool in = lane < n;
    uint32_t v = in ? a[f + lane] : 0xffffffffu;
    int fs = 0, ls = n, dep = depth;
    const unsigned long long below = (1ull << lane) - 1ull;
    for (;;) {
        const bool act = in && ls - fs > 16 && dep > 0;
        if (__ballot(act) == 0ull) break;
        const int mid = fs + (ls - fs) / 2;
        const uint32_t va = (uint32_t)__shfl((int)v, fs + 1), vb = (uint32_t)__shfl((int)v, mid);
        const uint32_t vc = (uint32_t)__shfl((int)v, ls - 1), v0 = (uint32_t)__shfl((int)v, fs);
        const uint32_t da = kd(va), db = kd(vb), dc = kd(vc);
        int ch;
        if (da < db) ch = db < dc ? mid : (da < dc ? ls - 1 : fs + 1);
        else ch = da < dc ? fs + 1 : (db < dc ? ls - 1 : mid);
        const uint32_t pv = ch == mid ? vb : (ch == ls - 1 ? vc : va);   // the median, moved to fs
        uint32_t vp = v;
        if (act) vp = lane == fs ? pv : (lane == ch ? v0 : v);
        const uint32_t p = kd(pv);
        const bool inr = act && lane > fs && lane < ls;
        const bool A = inr && !(kd(vp) < p), Bq = inr && !(p < kd(vp));
        const unsigned long long seg = (ls - fs >= 64 ? ~0ull : (((1ull << (ls - fs)) - 1ull) << fs));
        const unsigned long long lm = __ballot(A) & seg, rm = __ballot(Bq) & seg;
        const int ka = __popcll(lm & below), kb = __popcll(rm & below);
        const int TA = __popcll(lm), TB = __popcll(rm);
        const bool swapL = A && TB - kb - (Bq ? 1 : 0) >= ka + 1;
        const int K = __popcll(__ballot(swapL) & seg);   // the swapping left stoppers: ranks [0, K)
        const int rr = TB - 1 - kb;                      // this right stopper's rank from the right
        const bool swapR = Bq && rr < K;
        if (A) tl[fs + ka] = (uint16_t)lane;
        if (Bq) tr[fs + kb] = (uint16_t)lane;
        wave_lds_sync();
        int src = lane;
        if (swapL) src = tr[fs + TB - 1 - ka];   // the right stopper of rank ka from the right
        if (swapR) src = tl[fs + rr];            // the left stopper of rank rr
        const int LK = (act && K < TA) ? (int)tl[fs + K] : INT_MAX;
        const int RK1 = (act && K > 0) ? (int)tr[fs + TB - K] : -1;
        const int cut = K == 0 ? LK : min(LK, RK1);
        v = (uint32_t)__shfl((int)vp, src);
        if (act) {
            if (lane < cut) ls = cut;
            else fs = cut;
            dep--;
        }
        wave_lds_sync();   // this step's table reads before the next step's writes
    }
    if (in) {
        a[f + lane] = v;
        const int len = ls - fs;
        if (len <= 16) leaf[f + lane] = (uint32_t)(f + fs) | ((uint32_t)len << 16);
        else if (lane == fs) {   // depth budget spent: heap sort at the next level
            const int slot = atomicAdd(npush, 1);
            push[slot] = make_int4(f + fs, f + ls, 0, 0);
        }
    }
    wave_lds_sync();
}

struct SortLds {
    int4 seg[2][kLaneSegs];   // (first, last, depth, -) per level, double-buffered
    int nseg[2];
    int lmax[2];              // the longest segment pushed to the level (heap-sort segments aside)
    int wred[kLaneThreads / 64][2];   // block_partition: per-wave scan totals, per-wave minima
};

constexpr int kBlockPart = 384;   // segments longer than this are partitioned by the whole workgroup (r06 same-box A/B: 192 / 256 / 384 / 640 gave 118.9 / 118.2 / 117.7 / 118.5 us per se3 pair; 512 / 768 with wave_partition2 slower)
// rank -> position scratch of the sort, entries per posL / posR array: a wave partitions segments of <= kBlockPart
// elements in its own kBlockPart-entry slice, block_partition a longer one in the whole array
constexpr int kSortPos = (kLaneThreads / 64) * kBlockPart > kRansacMaxM ? (kLaneThreads / 64) * kBlockPart : kRansacMaxM;

// __unguarded_partition_pivot(f, l) (std::__move_median_to_first, then __unguarded_partition(f + 1, l, *f)) of one
// segment of 64 < l - f <= kBlockPart elements by one wave.  Left stoppers are the x with !(x < p), right
// stoppers the x with !(p < x); the sequential two-pointer loop swaps the k-th left stopper (from the left) with
// the k-th right stopper (from the right) for as long as the former lies before the latter, and returns the
// position where the pointers cross -- so every swap pair is known from the ranks alone and all swaps run at once.
// Each lane owns a contiguous run of E <= kBlockPart / 64 elements (flags as bit masks, ranks from a wave scan).
// One read round per stage: the four pivot candidates (f, f + 1, mid, l - 1) together, every lane applying the
// median swap to its own elements in registers (lane 0 writes the two swapped positions); the elements; the
// rank -> position tables pl (left, from the left) and pr (right, from the right), with each right stopper's value
// beside its position in vr, so a swapping left stopper reads its partner's position and value together and
// writes both.  Returns the cut (pl / pr / vr: the wave's >= kBlockPart-entry slices).
__device__ int wave_partition2(uint32_t* a, uint16_t* pl, uint16_t* pr, uint32_t* vr, int f, int l, long long* wp = nullptr)
{
    constexpr int kE = kBlockPart / 64;
    const int lane = threadIdx.x & 63;
    long long wt = (wp && lane == 0) ? (long long)wall_clock64() : 0;
    auto wmark = [&](int k) {
        if (wp && lane == 0) {
            const long long t = (long long)wall_clock64();
            wp[k] += t - wt;
            wt = t;
        }
    };
    const int mid = f + (l - f) / 2;
    const uint32_t va = a[f + 1], vb = a[mid], vc = a[l - 1], v0 = a[f];
    const int lo = f + 1, n = l - lo;
    const int E = (n + 63) >> 6;
    const int base = lo + lane * E, cntE = max(0, min(E, l - base));
    uint32_t v[kE];
#pragma unroll
    for (int j = 0; j < kE; j++) v[j] = j < cntE ? a[base + j] : 0u;
    const uint32_t da = kd(va), db = kd(vb), dc = kd(vc);
    int ch;
    if (da < db) ch = db < dc ? mid : (da < dc ? l - 1 : f + 1);
    else ch = da < dc ? f + 1 : (db < dc ? l - 1 : mid);
    const uint32_t pv = ch == mid ? vb : (ch == l - 1 ? vc : va);   // the pivot, moved to f
    if (lane == 0) {
        a[f] = pv;
        a[ch] = v0;
    }
#pragma unroll
    for (int j = 0; j < kE; j++) v[j] = base + j == ch ? v0 : v[j];
    const uint32_t p = kd(pv);
    unsigned fA = 0, fB = 0;
    int ca = 0, cb = 0;
#pragma unroll
    for (int j = 0; j < kE; j++) {
        const bool in = j < cntE;
        const bool A = in && !(kd(v[j]) < p), Bq = in && !(p < kd(v[j]));
        fA |= (unsigned)A << j;
        fB |= (unsigned)Bq << j;
        ca += A;
        cb += Bq;
    }
    wmark(1);
    const int pk = ca | (cb << 16);
    const int inc = wave_incl_scan(pk);
    const int tot = __builtin_amdgcn_readlane(inc, 63);
    const int ex = inc - pk;
    const int TA = tot & 0xffff, TB = tot >> 16;
    int ka = ex & 0xffff, kb = ex >> 16, ff = INT_MAX;
    unsigned sA = 0;
#pragma unroll
    for (int j = 0; j < kE; j++) {
        const int A = (int)((fA >> j) & 1u), Bq = (int)((fB >> j) & 1u);
        if (A) {
            pl[ka] = (uint16_t)(base + j);
            if (TB - kb - Bq >= ka + 1) sA |= 1u << j;   // the right stopper of rank ka from the right lies after it
            else ff = min(ff, ka);
        }
        if (Bq) {
            pr[TB - 1 - kb] = (uint16_t)(base + j);
            vr[TB - 1 - kb] = v[j];
        }
        ka += A;
        kb += Bq;
    }
    wave_lds_sync();
    wmark(2);
    const int K = min(wave_min_i(ff), TA);   // the swapping left stoppers: ranks [0, K)
    const int LK = K < TA ? (int)pl[K] : INT_MAX;
    const int RK1 = K > 0 ? (int)pr[K - 1] : -1;
    // every swap of this lane at once: the partner's position and value in one round, then both stores (the pairs
    // are disjoint: no position is both a swapping left and a swapping right stopper)
    const int ka0 = ex & 0xffff;
    int q[kE];
    uint32_t qv[kE];
#pragma unroll
    for (int j = 0; j < kE; j++) {
        const int r = ka0 + __popc(fA & ((1u << j) - 1u));
        const bool sw = (sA >> j) & 1u;
        q[j] = sw ? (int)pr[r] : 0;
        qv[j] = sw ? vr[r] : 0u;
    }
    wmark(3);
#pragma unroll
    for (int j = 0; j < kE; j++) {
        if ((sA >> j) & 1u) {
            a[base + j] = qv[j];
            a[q[j]] = v[j];
        }
    }
    wave_lds_sync();
    wmark(4);
    return K == 0 ? LK : min(LK, RK1);
}

// __unguarded_partition_pivot(f, l) of one long segment by the whole workgroup (kLaneThreads): the median of
// three moved to f, then wave_partition2's rule over all threads -- thread t owns a contiguous run of <= E
// elements, the stopper ranks come from a workgroup scan, the k-th left stopper swaps with the k-th right
// stopper (from the right) while it lies before it.  Returns the cut (uniform).  posL / posR: >= l - f entries.
__device__ int block_partition(uint32_t* a, uint16_t* posL, uint16_t* posR, int f, int l, SortLds& sh)
{
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int NW = kLaneThreads / 64;
    if (tid == 0) median_to_first(a, f, f + 1, f + (l - f) / 2, l - 1);
    __syncthreads();
    const uint32_t p = kd(a[f]);
    const int lo = f + 1, n = l - lo;
    const int E = (n + kLaneThreads - 1) / kLaneThreads;
    const int base = min(lo + tid * E, l), hi = min(base + E, l);
    unsigned long long fA = 0, fB = 0;
    int ca = 0, cb = 0;
    for (int i = base; i < hi; i++) {
        const uint32_t v = kd(a[i]);
        const bool A = !(v < p), Bq = !(p < v);
        fA |= (unsigned long long)A << (i - base);
        fB |= (unsigned long long)Bq << (i - base);
        ca += A;
        cb += Bq;
    }
    const int pk = ca | (cb << 16);
    const int inc = wave_incl_scan(pk);
    if (lane == 63) sh.wred[w][0] = inc;
    __syncthreads();
    int wpre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < NW; k++) {
        const int v = sh.wred[k][0];
        wpre += k < w ? v : 0;
        tot += v;
    }
    const int ex = wpre + inc - pk;
    const int TA = tot & 0xffff, TB = tot >> 16;
    int ka = ex & 0xffff, kb = ex >> 16, ff = INT_MAX;
    unsigned long long sA = 0;
    for (int i = base; i < hi; i++) {
        const int j = i - base;
        const int A = (int)((fA >> j) & 1ull), Bq = (int)((fB >> j) & 1ull);
        if (A) {
            posL[ka] = (uint16_t)i;
            if (TB - kb - Bq >= ka + 1) sA |= 1ull << j;   // the right stopper of rank ka lies after i
            else ff = min(ff, ka);
        }
        if (Bq) posR[TB - 1 - kb] = (uint16_t)i;
        ka += A;
        kb += Bq;
    }
    const int wm = wave_min_i(ff);
    if (lane == 0) sh.wred[w][1] = wm;
    __syncthreads();   // posL / posR and the wave minima
    int K = TA;
#pragma unroll
    for (int k = 0; k < NW; k++) K = min(K, sh.wred[k][1]);   // the swapping left stoppers: ranks [0, K)
    const int LK = K < TA ? (int)posL[K] : INT_MAX;
    const int RK1 = K > 0 ? (int)posR[K - 1] : -1;
    const int ka0 = ex & 0xffff;
    while (sA) {   // four swaps at a time, every load before the stores (the pairs are disjoint)
        int jl[4], jr[4];
        int nn = 0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            jl[u] = 0;
            jr[u] = 0;
            if (sA) {
                const int j = __builtin_ctzll(sA);
                sA &= sA - 1ull;
                jl[u] = base + j;
                jr[u] = posR[ka0 + __popcll(fA & ((1ull << j) - 1ull))];
                nn = u + 1;
            }
        }
        uint32_t vl[4], vr[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            vl[u] = u < nn ? a[jl[u]] : 0u;
            vr[u] = u < nn ? a[jr[u]] : 0u;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            if (u < nn) {
                a[jl[u]] = vr[u];
                a[jr[u]] = vl[u];
            }
        }
    }
    __syncthreads();
    return K == 0 ? LK : min(LK, RK1);
}

// std::sort(a, a + n) by distance, whole workgroup (kLaneThreads).  leaf[i] = (start of the leaf holding
// i) | (its length << 16), length 0 for a heap-sorted segment; out = the sorted keys.
__device__ void lane_sort(uint32_t* a, uint32_t* out, int n, uint16_t* posL, uint16_t* posR, uint32_t* leaf, SortLds& sh,
                          int depth_limit = -1, bool prof = false)
{
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int NW = kLaneThreads / 64;
    if (tid == 0) {
        sh.nseg[0] = 0;
        sh.nseg[1] = 0;
        sh.lmax[0] = 0;
        if (n > 16) {
            sh.seg[0][0] = make_int4(0, n, depth_limit >= 0 ? depth_limit : 2 * (31 - __clz(n)), 0);
            sh.nseg[0] = 1;
            sh.lmax[0] = n;
        }
    }
    if (n <= 16)
        for (int i = tid; i < n; i += kLaneThreads) leaf[i] = (uint32_t)n << 16;
    __syncthreads();
    uint16_t* pl = posL + (size_t)w * kBlockPart;
    uint16_t* pr = posR + (size_t)w * kBlockPart;
    uint32_t* vrw = reinterpret_cast<uint32_t*>(posR + kSortPos) + (size_t)w * kBlockPart;   // [kSortPos] u32 after posR
#ifdef RGBD_PNP_PROFILE
    const bool sprof = prof && tid == 0;   // k_lane_match's lane 0 (not the parity hook's calls)
    long long st_prev = wall_clock64();
#endif
    for (int lv = 0;; lv++) {
        const int cur = lv & 1, nxt = cur ^ 1;
        const int cnt = sh.nseg[cur];
#ifdef RGBD_PNP_PROFILE
        if (sprof && lv > 0) { const long long t_ = wall_clock64(); g_sort_prof[min(lv - 1, 15)] += t_ - st_prev; st_prev = t_; }
        if (sprof && cnt > 0) g_sort_prof[17] = max(g_sort_prof[17], (long long)lv + 1);
        if (sprof && lv < 16)
            for (int k = 0; k < cnt; k++) {
                const int4 q = sh.seg[cur][k];
                g_sort_seg[lv][0]++;
                g_sort_seg[lv][1] += q.y - q.x > 64 ? 1 : 0;
                g_sort_seg[lv][2] += q.z == 0 ? 1 : 0;
                g_sort_seg[lv][3] = max(g_sort_seg[lv][3], (long long)(q.y - q.x));
            }
#endif
        if (cnt == 0) break;
        const int lmax = sh.lmax[cur];
        if (tid == 0) {
            sh.nseg[nxt] = 0;
            sh.lmax[nxt] = 0;
        }
        __syncthreads();
        // the long segments first, one at a time by the whole workgroup (the level's list is scanned for them
        // only when one was pushed: a scan is a dependent LDS read per segment)
        for (int k = 0; k < (lmax > kBlockPart ? cnt : 0); k++) {
            const int4 s = sh.seg[cur][k];
            const int f = s.x, l = s.y, depth = s.z;
            if (depth == 0 || l - f <= kBlockPart) continue;   // uniform
            const int cut = block_partition(a, posL, posR, f, l, sh);
            const int cf[2] = {f, cut}, cl[2] = {cut, l};
#pragma unroll
            for (int c = 0; c < 2; c++) {
                const int len = cl[c] - cf[c];
                if (len > 16) {
                    if (tid == 0) {
                        const int slot = atomicAdd(&sh.nseg[nxt], 1);
                        sh.seg[nxt][slot] = make_int4(cf[c], cl[c], depth - 1, 0);
                        atomicMax(&sh.lmax[nxt], len);
                    }
                } else if (tid < len) {
                    leaf[cf[c] + tid] = (uint32_t)cf[c] | ((uint32_t)len << 16);
                }
            }
        }
        for (int k = w; k < cnt; k += NW) {
            const int4 s = sh.seg[cur][k];
            const int f = s.x, l = s.y, depth = s.z;
            if (depth > 0 && l - f > kBlockPart) continue;   // done above
            if (depth == 0) {   // introsort's depth limit: __partial_sort of the whole segment
                if (lane == 0) heap_sort(a, f, l);
                wave_lds_sync();
                for (int i = f + lane; i < l; i += 64) leaf[i] = (uint32_t)f;   // length 0: sorted already
                continue;
            }
            if (l - f <= 64) {   // the rest of this subtree in registers
                wave_sort_small2(a, f, l - f, depth, leaf, sh.seg[nxt], &sh.nseg[nxt], pl, pr);
                continue;
            }
#ifdef RGBD_PNP_PROFILE
            long long* wp = prof ? g_wp_prof : nullptr;
            if (wp && lane == 0) {
                wp[5]++;
                wp[6] += l - f;
            }
#else
            long long* wp = nullptr;
#endif
            const int cut = wave_partition2(a, pl, pr, vrw, f, l, wp);
            // children [f, cut) and [cut, l) with depth - 1: longer than 16 -> next level, else a leaf
            const int cf[2] = {f, cut}, cl[2] = {cut, l};
#pragma unroll
            for (int c = 0; c < 2; c++) {
                const int len = cl[c] - cf[c];
                if (len > 16) {
                    if (lane == 0) {
                        const int slot = atomicAdd(&sh.nseg[nxt], 1);
                        sh.seg[nxt][slot] = make_int4(cf[c], cl[c], depth - 1, 0);
                        atomicMax(&sh.lmax[nxt], len);
                    }
                } else if (lane < len) {
                    leaf[cf[c] + lane] = (uint32_t)cf[c] | ((uint32_t)len << 16);
                }
            }
        }
        __syncthreads();
    }
    // the final insertion sort: a stable sort of every leaf (elements move only past strictly greater ones)
    for (int i = tid; i < n; i += kLaneThreads) {
        const uint32_t lf = leaf[i];
        const int s = (int)(lf & 0xffffu), len = (int)(lf >> 16);
        const uint32_t v = a[i];
        if (len == 0) {
            out[i] = v;
            continue;
        }
        int r = 0;
        for (int j = s; j < s + len; j++) {
            const uint32_t u = kd(a[j]);
            r += (u < kd(v) || (u == kd(v) && j < i)) ? 1 : 0;
        }
        out[s + r] = v;
    }
    __syncthreads();
#ifdef RGBD_PNP_PROFILE
    if (sprof) g_sort_prof[16] += wall_clock64() - st_prev;
#endif
}

struct MatchLds {
    SortLds sort;
    int wsum[kLaneThreads / 64];
    int m;
};

}  // namespace


// ---------------------------------------------------------------- Matcher + RansacSE3 set-up, one lane per block
// Dynamic LDS: minq [K] i32 | cand [K] u8 (padded) | keys [Mcap] u32 | sorted [Mcap] u32 | leaf [Mcap] u32 |
// posL / posR [kSortPos] u16 | sort values [kSortPos] u32 | mq / mtr [Mcap] i32
__global__ __launch_bounds__(kLaneThreads) void k_lane_match(LaneBufs lb, LaneCfg lc)
{
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ MatchLds sh;
    const int l = blockIdx.x, tid = threadIdx.x;
    LaneCtl& c = lb.ctl[l];
    const int K = lc.K;
    if (c.b > c.end) return;
#ifdef RGBD_PNP_PROFILE
    const bool lprof = l == 0 && tid == 0;
    long long t_prev = wall_clock64();
    if (lprof) g_lm_prof[0]++;
#endif
    // the lane's attempt: 0 (the previous frame) or, the round after attempt 0 failed, 1 (the second reference)
    const int att = c.retry;
    const int b = c.b;
    const int ref = att == 0 ? b - 1 : max(b - 2, c.start);
    int* minq = reinterpret_cast<int*>(smem);
    uint8_t* cand = reinterpret_cast<uint8_t*>(minq + K);
    uint32_t* keys = reinterpret_cast<uint32_t*>(cand + ((K + 15) & ~15));
    uint32_t* sorted = keys + lc.Mcap;
    uint32_t* leaf = sorted + lc.Mcap;
    uint16_t* posL = reinterpret_cast<uint16_t*>(leaf + lc.Mcap);
    uint16_t* posR = posL + kSortPos;
    int* mq = reinterpret_cast<int*>(posR + kSortPos) + kSortPos;   // after the sort's value table
    int* mtr = mq + lc.Mcap;
    uint32_t* tq = reinterpret_cast<uint32_t*>(mtr + lc.Mcap);   // [K]: query q's (distance << 16 | train index)
    const int nq = lb.counts[ref], nt = lb.counts[b];
    // attempt 1's rows: pair (ref, b), ref = max(b - 2, start): the consecutive pair's rows when ref = b - 1, else
    // the precomputed (b - 2 -> b) rows (skip_rows) or the ones the round's k_knn2m launch wrote
    const int4* knn = (att == 0 || ref == b - 1) ? lb.knn + (size_t)(b - 1) * K
                                                 : (lc.skip_rows ? lb.knn_skip + (size_t)(b - 2) * K : lb.knn_r + (size_t)l * K);
    // a lane's first frame starts with clear outlier flags (an independent chain; the frame is also the
    // previous lane's last, whose flags that lane writes): its own row B + l
    const uint8_t* fref = lb.flags + (size_t)((l > 0 && ref == c.start) ? lc.B + l : ref) * K;
    const float* zr = lb.xyz + (size_t)ref * K * 3;
    const float* zc = lb.xyz + (size_t)b * K * 3;
    for (int t = tid; t < nt; t += kLaneThreads) minq[t] = INT_MAX;
    __syncthreads();
    // Matcher::match (:115-137): candidates pass the ratio, ref-outlier and depth tests; a train index goes
    // to the first query (lowest index) that passes them
    // (a thread's kQB queries at a time: their knn rows and reference depths first, then the dependent train
    // depths, so the global loads' latencies overlap instead of queueing one query after another)
    constexpr int kQB = 4;
    for (int q0 = tid; q0 < nq; q0 += kQB * kLaneThreads) {
        int4 r[kQB];
        bool pre[kQB];
#pragma unroll
        for (int u = 0; u < kQB; u++) {
            const int q = q0 + u * kLaneThreads;
            r[u] = make_int4(0, 0, 0, -1);
            pre[u] = false;
            if (q < nq) {
                r[u] = knn[q];
                pre[u] = !fref[q] && zr[3 * q + 2] > 0.0f;
            }
        }
        float zt[kQB];
#pragma unroll
        for (int u = 0; u < kQB; u++) zt[u] = r[u].w >= 0 ? zc[3 * r[u].y + 2] : 0.0f;   // i2 >= 0: i1 is a train row
#pragma unroll
        for (int u = 0; u < kQB; u++) {
            const int q = q0 + u * kLaneThreads;
            if (q >= nq) continue;
            // i2 < 0: fewer than 2 train rows
            const bool ok = r[u].w >= 0 && (float)r[u].x < lc.nnratio * (float)r[u].z && pre[u] && zt[u] > 0.0f;
            cand[q] = ok ? 1 : 0;
            tq[q] = ((uint32_t)r[u].x << 16) | (uint32_t)r[u].y;
            if (ok) atomicMin(&minq[r[u].y], q);
        }
    }
    __syncthreads();
    LM_PROF(1);
    // ordered compaction: thread t owns queries [t E, t E + E)
    const int E = (nq + kLaneThreads - 1) / kLaneThreads;
    const int q0 = min(tid * E, nq), q1 = min(q0 + E, nq);
    int mine = 0;
    for (int q = q0; q < q1; q++) mine += (cand[q] && minq[tq[q] & 0xffffu] == q) ? 1 : 0;
    const int lane = tid & 63, w = tid >> 6;
    const int inc = wave_incl_scan(mine);
    if (lane == 63) sh.wsum[w] = inc;
    __syncthreads();
    int pre = 0, m = 0;
    for (int i = 0; i < kLaneThreads / 64; i++) {
        pre += i < w ? sh.wsum[i] : 0;
        m += sh.wsum[i];
    }
    int j = pre + inc - mine;
    for (int q = q0; q < q1; q++) {
        const uint32_t v = tq[q];
        if (cand[q] && minq[v & 0xffffu] == q) {
            if (j < lc.Mcap) {
                mq[j] = q;
                mtr[j] = (int)(v & 0xffffu);
                keys[j] = (v & 0xffff0000u) | (uint32_t)j;
            }
            j++;
        }
    }
    __syncthreads();
    LM_PROF(2);
    if (tid == 0) {
        c.ref = ref;
        c.m = m;
        c.need_more = 0;
        c.run = 0;
        c.early = 0;
    }
    // RansacSE3::compute (:29-30, :44-45): fewer than mMinInlierTh matches -> false, nothing else touched
    if ((uint32_t)m < lc.minTh) {
        if (tid == 0) c.early = 1;
        return;
    }
    if (m > lc.Mcap) {   // more matches than the hypothesis kernel keeps in LDS
        if (tid == 0) {
            c.err = 1;
            c.early = 1;
        }
        return;
    }
    // updateF2: every matched train index is an outlier until the inliers are known (:38-42)
    uint8_t* fcur = lb.flags + (size_t)b * K;
    for (int i = tid; i < m; i += kLaneThreads) fcur[mtr[i]] = 1;
    LM_PROF(3);
    // sort(vUsedMatches) (:52)
#ifdef RGBD_PNP_PROFILE
    lane_sort(keys, sorted, m, posL, posR, leaf, sh.sort, -1, lprof);
#else
    lane_sort(keys, sorted, m, posL, posR, leaf, sh.sort);
#endif
    LM_PROF(4);
    int2* mt = lb.mt + (size_t)l * lc.Mcap;
    float* pts = lb.pts + (size_t)l * lc.Mcap * 6;
    const float* x1 = lb.xyz + (size_t)ref * K * 3;
    const float* x2 = lb.xyz + (size_t)b * K * 3;
    for (int i0 = tid; i0 < m; i0 += kQB * kLaneThreads) {   // kQB matches at a time (overlapped gathers)
        float v[kQB][6];
#pragma unroll
        for (int u = 0; u < kQB; u++) {
            const int i = i0 + u * kLaneThreads;
            if (i >= m) continue;
            const int jj = (int)(sorted[i] & 0xffffu);
            const int q = mq[jj], t = mtr[jj];
            mt[i] = make_int2(q, t);
#pragma unroll
            for (int k = 0; k < 3; k++) {
                v[u][k] = x1[3 * q + k];
                v[u][3 + k] = x2[3 * t + k];
            }
        }
#pragma unroll
        for (int u = 0; u < kQB; u++) {
            const int i = i0 + u * kLaneThreads;
            if (i >= m) continue;
#pragma unroll
            for (int k = 0; k < 6; k++) pts[6 * i + k] = v[u][k];
        }
    }
    __syncthreads();
    LM_PROF(5);
    if (tid >= 64) return;   // wave 0 from here
    // the sticky depth covariance: set by the process's first errorFunction2 past the NaN test (:282-287): the
    // first match (in sorted order) with both depths non-zero and no NaN, found 64 at a time by a ballot
    if (!c.cov_set) {
        for (int i0 = 0; i0 < m; i0 += 64) {
            const int i = i0 + tid;
            bool hit = false;
            if (i < m) {
                const float* o = pts + 6 * i;
                hit = !(o[2] == 0.0f || o[3] == 0.0f) && !(isnan(o[2]) || isnan(o[5]));
            }
            const unsigned long long bal = __ballot(hit);
            if (bal) {
                if (tid == (int)__builtin_ctzll(bal)) {
                    const double z = (double)pts[6 * i + 2];
                    const double sd = 0.01 * z * z;
                    c.cov = sd * sd;
                    c.cov_set = 1;
                }
                break;
            }
        }
    }
    // sampleMatches (:135-159) for the first e0 hypotheses the loop may run (k_lane_replay draws the rest for
    // the few chains that get that far); cumulative rand() calls after each
    const int H = (m >= lc.SS) ? lc.iters : 0;
    WaveGlibc g;
    g.load(c.rng);
    sample_hyps(lb, lc, l, g, 0, min(H, lc.e0), m, 0);
    g.store(c.srng);
    if (tid == 0) {
        c.H = H;
        c.run = 1;   // hypotheses [0, H) and the identity slot
    }
    LM_PROF(6);
}

__global__ __launch_bounds__(64) void k_lane_replay(LaneBufs lb, LaneCfg lc, int phase)
{
    lane_replay(lb, lc, blockIdx.x, phase);
}

// ---------------------------------------------------------------- the deferred GICP problems of a call
// k_gicp_list: the pairs whose GICP aligns (>= 20 inlier pairs), and the exclusive prefix of their 2 n
// points (k_gicp_cov_pairs walks (pair, point) items); one 1024-thread block
__global__ __launch_bounds__(1024) void k_gicp_list(LaneBufs lb, LaneCfg lc)
{
    __shared__ int wv[16], wp[16];
    __shared__ int nprob_s, npts_s;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) {
        nprob_s = 0;
        npts_s = 0;
    }
    __syncthreads();
    for (int b0 = 0; b0 < lc.B; b0 += 1024) {
        const int b = b0 + tid;
        const int n = b < lc.B ? lb.gn[b] : 0;
        // < 20 pairs: Gicp::compute returns false; fewer than k_correspondences: PCL's covariances refuse
        const int v = n >= max(20, lc.gp.k) ? 1 : 0, pts = v ? 2 * n : 0;
        const int iv = wave_incl_scan(v), ip = wave_incl_scan(pts);
        if (lane == 63) {
            wv[w] = iv;
            wp[w] = ip;
        }
        __syncthreads();
        int prev = 0, prep = 0, totv = 0, totp = 0;
        for (int i = 0; i < 16; i++) {
            prev += i < w ? wv[i] : 0;
            prep += i < w ? wp[i] : 0;
            totv += wv[i];
            totp += wp[i];
        }
        const int nb = nprob_s, pb = npts_s;
        if (v) {
            const int k = nb + prev + iv - 1;
            lb.plist[k] = b;
            lb.ppre[k] = pb + prep + ip - pts;
        }
        __syncthreads();
        if (tid == 0) {
            nprob_s = nb + totv;
            npts_s = pb + totp;
        }
        __syncthreads();
    }
    if (tid == 0) {
        lb.pcount[0] = nprob_s;
        lb.pcount[1] = npts_s;
    }
}

// k_gicp_post: every GICP pair's result (Gicp::compute, Solver/Gicp.cpp:21-35): fewer than 20 pairs or not
// converged -> identity -> false; T.isIdentity() (Eigen, float precision 1e-5) -> false
__global__ __launch_bounds__(256) void k_gicp_post(LaneBufs lb, LaneCfg lc)
{
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= lc.B) return;
    PairOut& po = lb.out[b];
    if (!po.gicp_run) return;
    int ok = 0;
    const GicpOut& g = lb.gout[b];
    if (lb.gn[b] >= max(20, lc.gp.k) && g.converged) {
        bool ident = true;
        for (int i = 0; i < 4 && ident; i++)
            for (int j = 0; j < 4; j++) {
                const float v = g.T[4 * i + j];
                if (i == j ? !(fabsf(v - 1.0f) <= 1e-5f * fminf(fabsf(v), 1.0f)) : !(fabsf(v) <= 1e-5f)) {
                    ident = false;
                    break;
                }
            }
        ok = ident ? 0 : 1;
    }
    po.ok = ok;
    po.gicp_ok = ok;
    for (int e = 0; e < 16; e++) po.T[e] = ok ? g.T[e] : ((e % 5 == 0) ? 1.0f : 0.0f);
}

// ---------------------------------------------------------------- parity hook for the sort
__global__ __launch_bounds__(kLaneThreads) void k_lane_sort_test(const float* dist, int n, int depth_limit, int* order)
{
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ SortLds sh;
    uint32_t* keys = reinterpret_cast<uint32_t*>(smem);
    uint32_t* sorted = keys + kRansacMaxM;
    uint32_t* leaf = sorted + kRansacMaxM;
    uint16_t* posL = reinterpret_cast<uint16_t*>(leaf + kRansacMaxM);
    uint16_t* posR = posL + kSortPos;
    for (int i = threadIdx.x; i < n; i += kLaneThreads) keys[i] = ((uint32_t)dist[i] << 16) | (uint32_t)i;
    __syncthreads();
    lane_sort(keys, sorted, n, posL, posR, leaf, sh, depth_limit);
    for (int i = threadIdx.x; i < n; i += kLaneThreads) order[i] = (int)(sorted[i] & 0xffffu);
}

static size_t match_lds_bytes(int K, int Mcap)
{
    return (size_t)K * 4 + (size_t)((K + 15) & ~15) + (size_t)Mcap * 12 + (size_t)2 * kSortPos * 2 + (size_t)kSortPos * 4 + (size_t)Mcap * 8 +
           (size_t)K * 4 + 64;
}

hipError_t launch_lane_match(const LaneBufs& lb, const LaneCfg& lc, hipStream_t st)
{
    const size_t lds = match_lds_bytes(lc.K, lc.Mcap);
    return dispatch(k_lane_match, dim3(lc.L), dim3(kLaneThreads), lds, st, lb, lc);
}

hipError_t launch_lane_replay(const LaneBufs& lb, const LaneCfg& lc, int phase, hipStream_t st)
{
    return dispatch(k_lane_replay, dim3(lc.L), dim3(64), 0, st, lb, lc, phase);
}

hipError_t launch_gicp_list(const LaneBufs& lb, const LaneCfg& lc, hipStream_t st)
{
    return dispatch(k_gicp_list, dim3(1), dim3(1024), 0, st, lb, lc);
}

hipError_t launch_gicp_post(const LaneBufs& lb, const LaneCfg& lc, hipStream_t st)
{
    return dispatch(k_gicp_post, dim3((lc.B + 255) / 256), dim3(256), 0, st, lb, lc);
}

hipError_t launch_lane_sort_test(const float* dist, int n, int depth_limit, int* order, hipStream_t st)
{
    const size_t lds = (size_t)kRansacMaxM * 12 + (size_t)2 * kSortPos * 2 + (size_t)kSortPos * 4;
    return dispatch(k_lane_sort_test, dim3(1), dim3(kLaneThreads), lds, st, dist, n, depth_limit, order);
}

#ifdef RGBD_PNP_PROFILE
void lane_prof_dump(hipStream_t st)
{
    long long b[8];
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(b, HIP_SYMBOL(g_lm_prof), sizeof(b));
    fprintf(stderr, "[lm_prof] calls %lld us: filter %.1f compact %.1f marks %.1f sort %.1f gather %.1f samples %.1f\n", b[0],
            b[1] * 0.01, b[2] * 0.01, b[3] * 0.01, b[4] * 0.01, b[5] * 0.01, b[6] * 0.01);
    long long q[20];
    (void)hipMemcpyFromSymbol(q, HIP_SYMBOL(g_sort_prof), sizeof(q));
    fprintf(stderr, "[sort_prof] levels %lld us:", q[17]);
    for (int k = 0; k < 16 && k < q[17]; k++) fprintf(stderr, " %.1f", q[k] * 0.01);
    fprintf(stderr, " | leaves %.1f\n", q[16] * 0.01);
    std::memset(q, 0, sizeof(q));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sort_prof), q, sizeof(q));
    long long sg[16][4];
    (void)hipMemcpyFromSymbol(sg, HIP_SYMBOL(g_sort_seg), sizeof(sg));
    long long wpv[8];
    (void)hipMemcpyFromSymbol(wpv, HIP_SYMBOL(g_wp_prof), sizeof(wpv));
    fprintf(stderr, "[wp_prof] wave partitions %lld (mean %.0f elements) us: pivot+elements+flags %.1f scan+tables %.1f K+partners %.1f swaps %.1f\n",
            wpv[5], wpv[5] ? (double)wpv[6] / wpv[5] : 0.0, wpv[1] * 0.01, wpv[2] * 0.01, wpv[3] * 0.01, wpv[4] * 0.01);
    std::memset(wpv, 0, sizeof(wpv));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wp_prof), wpv, sizeof(wpv));
    fprintf(stderr, "[sort_seg] per level (segments, > 64, heap, max len):");
    for (int k = 0; k < 16 && sg[k][0] > 0; k++) fprintf(stderr, " L%d %lld/%lld/%lld/%lld", k, sg[k][0], sg[k][1], sg[k][2], sg[k][3]);
    fprintf(stderr, "\n");
    std::memset(sg, 0, sizeof(sg));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_sort_seg), sg, sizeof(sg));
    std::memset(b, 0, sizeof(b));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_lm_prof), b, sizeof(b));
}
#endif

}  // namespace rgbd

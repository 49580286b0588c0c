// svo.hip -- the reference's DEFAULT front end on gfx950: Extractor(SVO, BRIEF, NORMAL) (main.cpp:31).
//   Frame::Frame cvtColor            Core/Frame.cpp:47            -> k_svo_pyramid (fused with the levels + box sums)
//   SVOextractor::createImagePyramid Features/SVOextractor.cpp:139-148, halfSample :16-37 -> k_svo_pyramid
//   SVOextractor::detect             :86-137: fast_corner_detect_10 + fast_corner_score_10 + fast_nonmax_3x3
//                                    + ShiTomasiScore (:39-84) + the 5-px grid               -> k_svo_detect
//   Extractor::detectAndCompute      Features/Extractor.cpp:50-61: retainBest(nfeatures)     -> k_svo_select
//   BriefDescriptorExtractor::compute (xfeatures2d, 32 B): runByImageBorder(28) -> k_svo_select,
//                                    integral-image 9x9 box sums -> k_svo_pyramid (fused), 256 tests -> k_svo_brief
// then Frame::undistortKeyPoints + uprojectCamera reuse k_undistort (extract.hip).
//
// Layout in HBM (per batch of B frames):
//   pyr   [B][frame_bytes]       halfSample levels 0..L-1, tight rows (level 0 = the gray image)
//   cells [B][ncells] u64        per grid cell: (Shi-Tomasi score bits << 32) | ~(level, y, x) -- the
//                                reference's "first strictly greater score wins" as one atomicMax
//   box   [B][H][W] u16          9x9 box sums of the gray image (the integral-image differences)
//   cand  [B][ncells] uint2      the grid keypoints with response > 20 in cell order (before retainBest)
//   out   counts[B], kps [B][kp_cap] (cv::KeyPoint), desc [B][kp_cap][32]
// Every stage is bit-exact with oracle/orc_svo.cpp; the float Shi-Tomasi expression keeps the
// reference's operation order with -ffp-contract=off and IEEE sqrt.
#include <hip/hip_runtime.h>

#include "dispatch.h"

#include <climits>
#include <cstdio>
#include <cstdint>

#include "svo_dev.h"

namespace rgbd {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------ pyramid (gray + halfSample) + box sums
// One 256-thread workgroup per 128 x 128 level-0 tile:
//   1. BGR -> gray (cvtColor 8U fixed point) of the tile plus a 4-pixel ring into LDS (the tile itself
//      also to HBM as level 0), zero outside the image;
//   2. the 9x9 box sums of the tile (BRIEF's smoothedSum, KERNEL_SIZE 9: the four-corner integral-image
//      difference == the plain window sum) from the ring-extended gray, separably (row sums in LDS);
//   3. each level's 2x2 means from the previous level's tile in LDS.  A level-L pixel inside the level
//      only reads level-(L-1) pixels inside that level, so tiles never exchange data.
constexpr int kPyrT = 128;
constexpr int kPyrR = 4;                    // box half-width
constexpr int kPyrG = kPyrT + 2 * kPyrR;    // 136: staged gray side

__device__ __forceinline__ uint8_t gray_px(const uint8_t* p)
{
    return (uint8_t)((p[0] * 1868 + p[1] * 9617 + p[2] * 4899 + (1 << 13)) >> 14);
}

__global__ __launch_bounds__(256) void k_svo_pyramid(const uint8_t* __restrict__ bgr, uint8_t* __restrict__ pyr,
                                                     uint16_t* __restrict__ box, SvoCfg cfg)
{
    __shared__ __attribute__((aligned(16))) uint8_t G0[kPyrG * kPyrG];
    __shared__ __attribute__((aligned(16))) uint8_t A[(kPyrT / 2) * (kPyrT / 2)];
    __shared__ __attribute__((aligned(16))) uint8_t Bt[(kPyrT / 4) * (kPyrT / 4)];
    __shared__ __attribute__((aligned(16))) uint16_t hs[kPyrG * kPyrT];
    const int tid = threadIdx.x, b = blockIdx.z;
    const int tx0 = blockIdx.x * kPyrT, ty0 = blockIdx.y * kPyrT;
    const int W = cfg.W, H = cfg.H;
    uint8_t* P = pyr + (size_t)b * cfg.frame_bytes;
    const uint8_t* src0 = bgr ? bgr + (size_t)b * W * H * 3 : nullptr;
    // 1a. the tile's columns, 16-pixel groups, all 136 staged rows
    for (int g = tid; g < kPyrG * 8; g += 256) {
        const int r = g >> 3, c16 = (g & 7) << 4;
        const int y = ty0 - kPyrR + r, x = tx0 + c16;
        uint8_t out[16];
        const bool inner = r >= kPyrR && r < kPyrR + kPyrT;   // rows of the tile itself (level 0 output)
        if (y >= 0 && y < H && x < W) {
            if (src0) {
                const uint8_t* src = src0 + ((size_t)y * W + x) * 3;
                if (x + 16 <= W && (W & 15) == 0 && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
                    uint8_t in[48];
                    const uint4* s4 = reinterpret_cast<const uint4*>(src);
                    *reinterpret_cast<uint4*>(in) = s4[0];
                    *reinterpret_cast<uint4*>(in + 16) = s4[1];
                    *reinterpret_cast<uint4*>(in + 32) = s4[2];
#pragma unroll
                    for (int i = 0; i < 16; i++) out[i] = gray_px(in + 3 * i);
                    if (inner) *reinterpret_cast<uint4*>(P + (size_t)y * W + x) = *reinterpret_cast<uint4*>(out);
                } else {
                    for (int i = 0; i < 16; i++) {
                        out[i] = x + i < W ? gray_px(src + 3 * i) : (uint8_t)0;
                        if (inner && x + i < W) P[(size_t)y * W + x + i] = out[i];
                    }
                }
            } else {   // level 0 already holds the gray image (rgbd_detect_and_compute)
                for (int i = 0; i < 16; i++) out[i] = x + i < W ? P[(size_t)y * W + x + i] : (uint8_t)0;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; i++) out[i] = 0;
        }
#pragma unroll
        for (int i = 0; i < 16; i++) G0[r * kPyrG + kPyrR + c16 + i] = out[i];
    }
    // 1b. the ring's 4 + 4 columns of every staged row
    for (int t = tid; t < kPyrG * 2 * kPyrR; t += 256) {
        const int r = t >> 3, k = t & 7;
        const int c = k < kPyrR ? k : kPyrR + kPyrT + (k - kPyrR);
        const int y = ty0 - kPyrR + r, x = tx0 - kPyrR + c;
        uint8_t v = 0;
        if (y >= 0 && y < H && x >= 0 && x < W) v = src0 ? gray_px(src0 + ((size_t)y * W + x) * 3) : P[(size_t)y * W + x];
        G0[r * kPyrG + c] = v;
    }
    __syncthreads();
    // 2. box sums, separably with sliding windows: a task sums 9 columns for 16 consecutive outputs of one
    //    staged row (24 reads), then 9 rows for 16 consecutive outputs of one column
    for (int t = tid; t < kPyrG * (kPyrT / 16); t += 256) {
        const int r = t >> 3, c0 = (t & 7) << 4;
        const uint8_t* q = G0 + r * kPyrG + c0;
        uint16_t* o = hs + r * kPyrT + c0;
        int v = 0;
#pragma unroll
        for (int k = 0; k < 9; k++) v += q[k];
        o[0] = (uint16_t)v;
#pragma unroll
        for (int k = 1; k < 16; k++) {
            v += (int)q[k + 8] - (int)q[k - 1];
            o[k] = (uint16_t)v;
        }
    }
    __syncthreads();
    uint16_t* bx = box + (size_t)b * W * H;
    for (int t = tid; t < (kPyrT / 16) * kPyrT; t += 256) {
        const int c = t & (kPyrT - 1), r0 = (t >> 7) << 4;
        const int x = tx0 + c;
        const uint16_t* q = hs + r0 * kPyrT + c;
        int v = 0;
#pragma unroll
        for (int k = 0; k < 9; k++) v += q[k * kPyrT];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            if (k) v += (int)q[(k + 8) * kPyrT] - (int)q[(k - 1) * kPyrT];
            const int y = ty0 + r0 + k;
            if (y < H && x < W)
                bx[(size_t)y * W + x] = (x >= kPyrR && x < W - kPyrR && y >= kPyrR && y < H - kPyrR) ? (uint16_t)v : (uint16_t)0;
        }
    }
    // 3. halfSample levels (level 1 from the tile inside G0)
    const uint8_t* src = G0 + kPyrR * kPyrG + kPyrR;
    int sstride = kPyrG;
    uint8_t* dst = A;
    int sd = kPyrT;
    for (int L = 1; L < cfg.nlevels; L++) {
        const int d = sd >> 1;
        const int lx0 = tx0 >> L, ly0 = ty0 >> L, lw = cfg.lw[L], lh = cfg.lh[L];
        uint8_t* PL = P + cfg.loff[L];
        for (int i = tid; i < d * d; i += 256) {
            const int r = i / d, c = i - r * d;
            const uint8_t* q = src + (2 * r) * sstride + 2 * c;
            const int v = ((int)q[0] + q[1] + q[sstride] + q[sstride + 1]) >> 2;
            dst[r * d + c] = (uint8_t)v;
            if (lx0 + c < lw && ly0 + r < lh) PL[(size_t)(ly0 + r) * lw + lx0 + c] = (uint8_t)v;
        }
        __syncthreads();
        src = dst;
        sstride = d;
        dst = (dst == A) ? Bt : A;
        sd = d;
    }
}

// ------------------------------------------------------------------ FAST-10 + NMS + Shi-Tomasi + grid
constexpr int kDetTW = 64, kDetTH = 32;
constexpr int kDetHy = 5, kDetHx = 8;               // staged halo: 5 rows, 8 columns (dword-aligned)
constexpr int kDetGW = kDetTW + 2 * kDetHx;         // 80 staged columns: x0-8 .. x0+71
constexpr int kDetGH = kDetTH + 2 * kDetHy;         // 42 staged rows: y0-5 .. y0+36
constexpr int kDetSW = kDetTW + 4, kDetSH = kDetTH + 2;   // score map: the tile + 1-pixel ring, rows
                                                         // padded to a dword multiple (66 used of 68)

// m for two horizontally adjacent pixels at once (packed u16 lanes): max over the 16 ten-pixel arcs of
// the ring of min(v - x) (darker) or min(x - v) (brighter), clamped to [0, 255] by saturation.  The
// darker side of arc A is v (-) max_A x, the brighter min_A x (-) v, so only the smallest arc maximum MM
// and the largest arc minimum mm are needed.  Arcs k and k+1 (k even) share the core k+1 .. k+9, so the
// pair contributes max(core max, min(x_k, x_k+10)) to MM (and dually to mm).
__device__ __forceinline__ u16x2 fast10_m2(const uint32_t* P, int S, int r, int c)
{
    const uint32_t* p = P + r * S + c;
    uint32_t raw[16];
    raw[0] = p[3 * S];       raw[1] = p[3 * S + 1];   raw[2] = p[2 * S + 2];   raw[3] = p[1 * S + 3];
    raw[4] = p[3];           raw[5] = p[-1 * S + 3];  raw[6] = p[-2 * S + 2];  raw[7] = p[-3 * S + 1];
    raw[8] = p[-3 * S];      raw[9] = p[-3 * S - 1];  raw[10] = p[-2 * S - 2]; raw[11] = p[-1 * S - 3];
    raw[12] = p[-3];         raw[13] = p[1 * S - 3];  raw[14] = p[2 * S - 2];  raw[15] = p[3 * S - 1];
    const u16x2 v = __builtin_bit_cast(u16x2, p[0]);
    u16x2 x[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = __builtin_bit_cast(u16x2, raw[k]);
    u16x2 mx2[16], mn2[16], mx4[16], mn4[16];
#pragma unroll
    for (int j = 1; j < 16; j += 2) {
        mx2[j] = __builtin_elementwise_max(x[j], x[(j + 1) & 15]);
        mn2[j] = __builtin_elementwise_min(x[j], x[(j + 1) & 15]);
    }
#pragma unroll
    for (int j = 1; j < 16; j += 2) {
        mx4[j] = __builtin_elementwise_max(mx2[j], mx2[(j + 2) & 15]);
        mn4[j] = __builtin_elementwise_min(mn2[j], mn2[(j + 2) & 15]);
    }
    u16x2 MM = {0xffff, 0xffff}, mm = {0, 0};
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        const int j = k + 1;   // core j .. j+8 = max over j..j+7 and x[j+8]
        const u16x2 cmax = __builtin_elementwise_max(__builtin_elementwise_max(mx4[j], mx4[(j + 4) & 15]), x[(j + 8) & 15]);
        const u16x2 cmin = __builtin_elementwise_min(__builtin_elementwise_min(mn4[j], mn4[(j + 4) & 15]), x[(j + 8) & 15]);
        const u16x2 lo = __builtin_elementwise_min(x[k], x[(k + 10) & 15]);
        const u16x2 hi = __builtin_elementwise_max(x[k], x[(k + 10) & 15]);
        MM = __builtin_elementwise_min(MM, __builtin_elementwise_max(cmax, lo));
        mm = __builtin_elementwise_max(mm, __builtin_elementwise_min(cmin, hi));
    }
    return __builtin_elementwise_max(__builtin_elementwise_sub_sat(v, MM), __builtin_elementwise_sub_sat(mm, v));
}

// ShiTomasiScore's tail (Features/SVOextractor.cpp:79-83) from the three box sums: they are integers below
// 2^24, so integer accumulation equals the reference's float accumulation, and / (2.0 * 64) is exact; the
// rest keeps the reference's float operation order (no contraction, IEEE sqrt)
__device__ __forceinline__ float shi_tomasi_from_sums(int sxx, int syy, int sxy)
{
    const float dXX = (float)sxx * 0.0078125f, dYY = (float)syy * 0.0078125f, dXY = (float)sxy * 0.0078125f;
    const float s = dXX + dYY;
    const float q = dXX * dYY - dXY * dXY;
    const float disc = s * s - 4.0f * q;
    return (float)(0.5 * (double)(s - __builtin_sqrtf(disc)));
}

__global__ __launch_bounds__(256) void k_svo_detect(const uint8_t* __restrict__ pyr, const SvoTile* __restrict__ tiles,
                                                    SvoCfg cfg, unsigned long long* __restrict__ cell_keys)
{
    __shared__ __attribute__((aligned(16))) uint8_t G[kDetGH * kDetGW];
    __shared__ __attribute__((aligned(16))) uint32_t PI[kDetGH * kDetGW];
    __shared__ __attribute__((aligned(16))) uint8_t S[kDetSH * kDetSW];
    // strict 3x3 maxima are never 8-adjacent: at most (64 / 2) x (32 / 2) of them per tile
    __shared__ uint16_t list[(kDetTW / 2) * (kDetTH / 2)];
    __shared__ int nlist;
    const int tid = threadIdx.x, b = blockIdx.y;
    const SvoTile t = tiles[blockIdx.x];
    const int L = t.level, w = cfg.lw[L], h = cfg.lh[L];
    const int x0 = t.x0, y0 = t.y0;
    const uint8_t* img = pyr + (size_t)b * cfg.frame_bytes + cfg.loff[L];
    // rows start dword-aligned when the level's width and offset are multiples of 4 (frame_bytes is)
    const bool al4 = ((w | cfg.loff[L]) & 3) == 0;
    if (tid == 0) nlist = 0;
    // 1. stage rows y0-5 .. y0+36, columns x0-8 .. x0+71 as dwords (zero outside the level)
    for (int i = tid; i < kDetGH * (kDetGW / 4); i += 256) {
        const int r = i / (kDetGW / 4), q = i - r * (kDetGW / 4);
        const int y = y0 - kDetHy + r, x = x0 - kDetHx + 4 * q;
        uint32_t v = 0;
        if (y >= 0 && y < h) {
            const uint8_t* row = img + (size_t)y * w;
            if (al4 && x >= 0 && x + 4 <= w) {
                v = *reinterpret_cast<const uint32_t*>(row + x);
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (x + k >= 0 && x + k < w) v |= (uint32_t)row[x + k] << (8 * k);
            }
        }
        reinterpret_cast<uint32_t*>(G)[i] = v;
    }
    __syncthreads();
    // pair image PI[r][c] = G[r][c] | G[r][c+1] << 16, four entries per task
    for (int i = tid; i < kDetGH * (kDetGW / 4); i += 256) {
        const int q = i % (kDetGW / 4);
        const uint32_t v = reinterpret_cast<const uint32_t*>(G)[i];
        const uint32_t nb = q + 1 < kDetGW / 4 ? (uint32_t)G[4 * i + 4] : 0u;
        uint4 o;
        o.x = (v & 0xffu) | ((v & 0xff00u) << 8);
        o.y = ((v >> 8) & 0xffu) | ((v & 0xff0000u));
        o.z = ((v >> 16) & 0xffu) | ((v >> 24) << 16);
        o.w = (v >> 24) | (nb << 16);
        reinterpret_cast<uint4*>(PI)[i] = o;
    }
    __syncthreads();
    // 2. score map over the tile + 1-pixel ring: S = m - 1 where m > barrier (a FAST-10 corner), else 0;
    //    pixels outside the detector's domain [3, w-3) x [3, h-3) are never corners
    for (int task = tid; task < kDetSH * ((kDetTW + 2) / 2); task += 256) {
        const int sr = task / ((kDetTW + 2) / 2), cp = task - sr * ((kDetTW + 2) / 2);
        const int ty = sr - 1, tx = 2 * cp - 1;   // tile coordinates of the pair's first pixel
        const u16x2 m = fast10_m2(PI, kDetGW, ty + kDetHy, tx + kDetHx);
        const int Y = y0 + ty;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int X = x0 + tx + k;
            const int mv = m[k];
            const bool dom = X >= 3 && X < w - 3 && Y >= 3 && Y < h - 3;
            S[sr * kDetSW + 2 * cp + k] = (uint8_t)((dom && mv > cfg.barrier) ? mv - 1 : 0);
        }
    }
    __syncthreads();
    // 3. fast_nonmax_3x3: a corner survives iff no 8-neighbour corner scores >= it.  Four pixels of a row
    //    per task: the three score rows' 6 bytes are one dword + one u16 load each, the vertical maxima
    //    of the six columns are shared by the four pixels.
    for (int task = tid; task < kDetTH * (kDetTW / 4); task += 256) {
        const int ty = task / (kDetTW / 4), tx0 = 4 * (task - ty * (kDetTW / 4));
        int v[3][6];
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const uint8_t* r = S + (ty + k) * kDetSW + tx0;   // S column tx0 = tile column tx0 - 1
            const uint32_t d = *reinterpret_cast<const uint32_t*>(r);
            const uint32_t e = *reinterpret_cast<const uint16_t*>(r + 4);
#pragma unroll
            for (int j = 0; j < 4; j++) v[k][j] = (int)((d >> (8 * j)) & 255u);
            v[k][4] = (int)(e & 255u);
            v[k][5] = (int)(e >> 8);
        }
        int cm[6];
#pragma unroll
        for (int j = 0; j < 6; j++) cm[j] = max(v[0][j], v[2][j]);
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const int c = v[1][p + 1];
            const int nb = max(max(max(cm[p], cm[p + 1]), cm[p + 2]), max(v[1][p], v[1][p + 2]));
            const int tx = tx0 + p;
            if (c > nb && x0 + tx < w && y0 + ty < h) list[atomicAdd(&nlist, 1)] = (uint16_t)(ty * kDetTW + tx);
        }
    }
    __syncthreads();
    // 4. Shi-Tomasi of each survivor, then the grid: the reference keeps the first strictly greater
    //    score of a cell over levels 0.. and raster order, i.e. the max of (score, ~(level, y, x)).
    //    Eight lanes per survivor, one box row each; the integer sums are exact in any order.
    const int n = nlist;
    const int sc = 1 << L;
    const int l8 = tid & 7;
    for (int j = tid >> 3; j < n; j += 256 / 8) {
        const int i = list[j];
        const int ty = i / kDetTW, tx = i - ty * kDetTW;
        const int X = x0 + tx, Y = y0 + ty;
        if (X < 5 || X > w - 6 || Y < 5 || Y > h - 6) continue;   // patch too close to the boundary: 0
        const int gr = ty + kDetHy - 4 + l8, gc = tx + kDetHx;
        const uint8_t* row = G + gr * kDetGW;
        int sxx = 0, syy = 0, sxy = 0;
#pragma unroll
        for (int c = gc - 4; c < gc + 4; c++) {
            const int dx = (int)row[c + 1] - (int)row[c - 1];
            const int dy = (int)row[c + kDetGW] - (int)row[c - kDetGW];
            sxx += dx * dx;
            syy += dy * dy;
            sxy += dx * dy;
        }
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) {
            sxx += __shfl_xor(sxx, o, 8);
            syy += __shfl_xor(syy, o, 8);
            sxy += __shfl_xor(sxy, o, 8);
        }
        if (l8 != 0) continue;
        const float score = shi_tomasi_from_sums(sxx, syy, sxy);
        if (!(score > 0.0f)) continue;
        const int k = ((Y * sc) / cfg.cell) * cfg.gcols + (X * sc) / cfg.cell;
        const uint32_t ord = ((uint32_t)L << 22) | ((uint32_t)Y << 11) | (uint32_t)X;
        const unsigned long long key = ((unsigned long long)__float_as_uint(score) << 32) | (unsigned long long)(~ord);
        atomicMax(cell_keys + (size_t)b * cfg.ncells + k, key);
    }
}

#ifdef RGBD_PNP_PROFILE
__device__ long long g_sel_prof[64];   // k_svo_select of frame 0: wall-clock stamps of thread 0
#define SEL_PROF(k) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_sel_prof[(k)] = wall_clock64(); } while (0)
#define SEL_PROF_V(k, v) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_sel_prof[(k)] = (v); } while (0)
#else
#define SEL_PROF(k) do { } while (0)
#define SEL_PROF_V(k, v) do { } while (0)
#endif

// ------------------------------------------------------------------ retainBest on one workgroup
// cv::KeyPointsFilter::retainBest (OpenCV 3.4) = libstdc++ std::nth_element(begin, begin + n - 1, end,
// response >) + std::partition(begin + n, end, response >= boundary).  Both are Hoare-style: the k-th
// "left stopper" and the k-th "right stopper" (counted from the right) swap while the left one lies
// before the right one; since the scans only meet untouched elements or the previous pair's swapped
// ones, the k-th swap pairs the k-th stoppers of the ORIGINAL range.  That is computed here with block
// ranks: every pair swaps at once, and libstdc++'s element order is reproduced exactly.  The rest of
// introselect (median-of-3, depth limit 2 lg n with the heap-select fallback, final insertion sort)
// runs on one lane.  R = responses, I = payload (u16), posL / posR = rank -> position scratch.
struct SelLds {
    int wa[32];      // wave totals of block_scan2, two buffers
    int phase;       // block_scan2 buffer parity
    int first_false; // pair_swap: rank of the first left stopper that does not swap
};

// inclusive wave64 scan on DPP: row_shr 1/2/4/8 inside 16-lane rows, then row_bcast:15 / row_bcast:31
// carry the row totals (out-of-row sources and masked rows contribute 0)
__device__ __forceinline__ int wave_incl_scan(int v)
{
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// exclusive block scan of (a, b) (each < 2^16 in total) in thread order: one packed DPP scan per wave,
// the wave totals through LDS (double-buffered by the caller's phase bit, so one barrier per call)
__device__ __forceinline__ void block_scan2(int a, int b, int& ea, int& eb, int& ta, int& tb, SelLds& sh)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int v = a | (b << 16);
    const int iv = wave_incl_scan(v);
    int* buf = sh.wa + (sh.phase & 1) * 16;
    if (lane == 63) buf[w] = iv;
    __syncthreads();
    int pre = 0, tot = 0;
    for (int i = 0; i < nw; i++) {
        const int x = buf[i];
        pre += i < w ? x : 0;
        tot += x;
    }
    if (threadIdx.x == 0) sh.phase++;   // read by no one before the next barrier
    const int ex = pre + iv - v;
    ea = ex & 0xffff;
    eb = ex >> 16;
    ta = tot & 0xffff;
    tb = tot >> 16;
}

// Pair the left stoppers (mode 0: !(x > p); mode 1: !(x >= p)) with the right stoppers (mode 0: !(p > x);
// mode 1: x >= p) of [a, e) and swap every pair whose left stopper lies before its right one.  Returns K
// (swaps), L_K (the K-th left stopper, INT_MAX if none) and R_{K-1} (-1 if K == 0); TB = right stoppers.
// Each thread owns a contiguous run of <= 32 elements (flags as bit masks, nothing else kept in
// registers); a swap is done by the owner of its left stopper, and pairs are disjoint, so it needs no
// staging: read both, write both.
__device__ int pair_swap(float* R, uint16_t* I, uint16_t* posL, uint16_t* posR, int a, int e, float p, int mode,
                         int& LK, int& RK1, int& TB, SelLds& sh)
{
    const int T = blockDim.x, tid = threadIdx.x;
    const int E = (e - a + T - 1) / T;
    const int base = a + tid * E, hi = min(base + E, e);
    if (tid == 0) sh.first_false = INT_MAX;   // ordered before the atomics by block_scan2's barrier
    unsigned fA = 0, fB = 0;
    int ca = 0, cb = 0;
    for (int i = base; i < hi; i++) {
        const float v = R[i];
        const bool A = mode == 0 ? !(v > p) : !(v >= p);
        const bool Bq = mode == 0 ? !(p > v) : (v >= p);
        fA |= (unsigned)A << (i - base);
        fB |= (unsigned)Bq << (i - base);
        ca += A;
        cb += Bq;
    }
    int ea, eb, TA;
    block_scan2(ca, cb, ea, eb, TA, TB, sh);
    int ka = ea, kb = eb, ff = INT_MAX;
    unsigned sA = 0;
    for (int i = base; i < hi; i++) {
        const int j = i - base;
        const int A = (fA >> j) & 1, Bq = (fB >> j) & 1;
        if (A) {
            posL[ka] = (uint16_t)i;
            if (TB - kb - Bq >= ka + 1) sA |= 1u << j;   // the right stopper of rank ka lies after i
            else ff = min(ff, ka);
        }
        if (Bq) posR[TB - 1 - kb] = (uint16_t)i;
        ka += A;
        kb += Bq;
    }
    // swapping is a prefix of the left-stopper ranks: K = the first rank that does not swap (else TA)
    if (ff != INT_MAX) atomicMin(&sh.first_false, ff);
    __syncthreads();
    const int K = min(sh.first_false, TA);
    LK = K < TA ? (int)posL[K] : INT_MAX;
    RK1 = K > 0 ? (int)posR[K - 1] : -1;
    ka = ea;
    for (int i = base; i < hi; i++) {
        const int j = i - base;
        if ((sA >> j) & 1) {
            const int q = posR[ka];
            const float r = R[i];
            R[i] = R[q];
            R[q] = r;
            const uint16_t t = I[i];
            I[i] = I[q];
            I[q] = t;
        }
        ka += (fA >> j) & 1;
    }
    __syncthreads();
    return K;
}

__device__ __forceinline__ void el_swap(float* R, uint16_t* I, int a, int b)
{
    const float r = R[a];
    R[a] = R[b];
    R[b] = r;
    const uint16_t t = I[a];
    I[a] = I[b];
    I[b] = t;
}

// libstdc++ __adjust_heap / __push_heap with comp(a, b) = a > b (one lane)
__device__ void adjust_heap(float* R, uint16_t* I, int first, int hole, int len, float vr, uint16_t vi)
{
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (R[first + child] > R[first + child - 1]) child--;
        R[first + hole] = R[first + child];
        I[first + hole] = I[first + child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        R[first + hole] = R[first + child - 1];
        I[first + hole] = I[first + child - 1];
        hole = child - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && R[first + parent] > vr) {
        R[first + hole] = R[first + parent];
        I[first + hole] = I[first + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    R[first + hole] = vr;
    I[first + hole] = vi;
}

// std::__heap_select(first, middle, last) + iter_swap(first, nth): introselect's depth-limit fallback
__device__ void heap_select_one_lane(float* R, uint16_t* I, int first, int middle, int last, int nth)
{
    const int len = middle - first;
    if (len >= 2) {
        int parent = (len - 2) / 2;
        for (;;) {
            adjust_heap(R, I, first, parent, len, R[first + parent], I[first + parent]);
            if (parent == 0) break;
            parent--;
        }
    }
    for (int i = middle; i < last; i++)
        if (R[i] > R[first]) {   // __pop_heap(first, middle, i)
            const float vr = R[i];
            const uint16_t vi = I[i];
            R[i] = R[first];
            I[i] = I[first];
            adjust_heap(R, I, first, 0, len, vr, vi);
        }
    el_swap(R, I, first, nth);
}

// std::__insertion_sort(first, last) with comp = greater (one lane)
__device__ void insertion_sort_one_lane(float* R, uint16_t* I, int f, int l)
{
    if (f == l) return;
    for (int i = f + 1; i < l; i++) {
        const float vr = R[i];
        const uint16_t vi = I[i];
        int j = i;
        if (vr > R[f]) {
            for (; j > f; j--) { R[j] = R[j - 1]; I[j] = I[j - 1]; }
        } else {
            while (vr > R[j - 1]) { R[j] = R[j - 1]; I[j] = I[j - 1]; j--; }
        }
        R[j] = vr;
        I[j] = vi;
    }
}

// std::__move_median_to_first(result, a, b, c) with comp = greater (one lane)
__device__ void median_to_first(float* R, uint16_t* I, int result, int a, int b, int c)
{
    if (R[a] > R[b]) {
        if (R[b] > R[c]) el_swap(R, I, result, b);
        else if (R[a] > R[c]) el_swap(R, I, result, c);
        else el_swap(R, I, result, a);
    } else if (R[a] > R[c]) el_swap(R, I, result, a);
    else if (R[b] > R[c]) el_swap(R, I, result, c);
    else el_swap(R, I, result, b);
}

// retainBest(n_points = nkeep) over R[0..n) (n > nkeep >= 1): returns the kept count (block-uniform)
// depth_limit < 0: libstdc++'s 2 * lg(n); an explicit value pins the heap-select fallback in the tests
__device__ int retain_best_block(float* R, uint16_t* I, uint16_t* posL, uint16_t* posR, int n, int nkeep, SelLds& sh,
                                 int depth_limit = -1)
{
    const int nth = nkeep - 1;
    int f = 0, l = n;
    int depth = depth_limit >= 0 ? depth_limit : 2 * (31 - __clz(n));
    bool heap = false;
    int it = 0;
    while (l - f > 3) {
        if (depth == 0) {
            if (threadIdx.x == 0) heap_select_one_lane(R, I, f, nth + 1, l, nth);
            __syncthreads();
            heap = true;
            break;
        }
        --depth;
        if (threadIdx.x == 0) median_to_first(R, I, f, f + 1, f + (l - f) / 2, l - 1);
        __syncthreads();
        const float p = R[f];
        int LK, RK1, TB;
        const int K = pair_swap(R, I, posL, posR, f + 1, l, p, 0, LK, RK1, TB, sh);
        const int cut = min(K == 0 ? LK : min(LK, RK1), l);   // (the min with l never binds: median-of-3 sentinels)
        if (cut <= nth) f = cut;
        else l = cut;
        SEL_PROF(2 + min(it, 40));
        it++;
    }
    SEL_PROF_V(60, it);
    (void)it;
    if (!heap) {
        if (threadIdx.x == 0) insertion_sort_one_lane(R, I, f, l);
        __syncthreads();
    }
    // std::partition(begin + nkeep, end, response >= R[nkeep - 1]): the kept prefix grows by the preds
    const float amb = R[nth];
    int LK, RK1, TB;
    SEL_PROF(45);
    pair_swap(R, I, posL, posR, nkeep, n, amb, 1, LK, RK1, TB, sh);
    SEL_PROF(46);
    return nkeep + TB;
}

// ------------------------------------------------------------------ grid -> keypoints (one frame per block)
// 1. the grid keypoints with response > 20 in cell order (SVOextractor::detect :131-134) -> R / I
// 2. retainBest(nfeatures) when more than nfeatures (Extractor::detectAndCompute :56-57)
// 3. runByImageBorder(28) (stable remove_if), keypoints written as cv::KeyPoint (size 0, angle -1,
//    response = Shi-Tomasi score, octave = level, class_id -1); cells reset to 0 for the next batch
__global__ __launch_bounds__(kSvoSelThreads) void k_svo_select(unsigned long long* __restrict__ cell_keys, SvoCfg cfg,
                                                               uint2* __restrict__ cand, int* __restrict__ ncand,
                                                               int* __restrict__ counts, float* __restrict__ kps,
                                                               int* __restrict__ err)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ SelLds sh;
    const int b = blockIdx.x, tid = threadIdx.x, T = blockDim.x;
    const int NC = cfg.ncells;
    float* R = reinterpret_cast<float*>(smem);
    uint16_t* I = reinterpret_cast<uint16_t*>(R + NC);
    uint16_t* posL = I + NC;
    uint16_t* posR = posL + NC;
    unsigned long long* cells = cell_keys + (size_t)b * NC;
    const int E = (NC + T - 1) / T, base = tid * E;
    if (tid == 0) sh.phase = 0;
    __syncthreads();
    // 1. (all of a thread's cell loads issued together)
    SEL_PROF(0);
    unsigned long long key[kSvoSelMaxE];
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < kSvoSelMaxE; j++) {
        key[j] = (j < E && base + j < NC) ? cells[base + j] : 0ull;
        cnt += __uint_as_float((uint32_t)(key[j] >> 32)) > 20.0f;
    }
    int off, d0, n, d1;
    block_scan2(cnt, 0, off, d0, n, d1, sh);
#pragma unroll
    for (int j = 0; j < kSvoSelMaxE; j++) {
        const float s = __uint_as_float((uint32_t)(key[j] >> 32));
        if (s > 20.0f) {
            R[off] = s;
            I[off] = (uint16_t)(base + j);
            cand[(size_t)b * NC + off] = make_uint2((uint32_t)(key[j] >> 32), (uint32_t)key[j]);
            off++;
        }
    }
    SEL_PROF_V(61, n);
    if (tid == 0) ncand[b] = n;
    __syncthreads();
    // 2.
    int m = n;
    if (n > cfg.nfeatures) m = cfg.nfeatures > 0 ? retain_best_block(R, I, posL, posR, n, cfg.nfeatures, sh) : 0;
    SEL_PROF(1);
    // 3.
    const int E2 = (m + T - 1) / T, base2 = tid * E2;
    int keep = 0;
    for (int j = 0; j < E2; j++) {
        const int i = base2 + j;
        if (i >= m) break;
        const uint32_t ord = ~(uint32_t)cells[I[i]];
        const int L = ord >> 22, x = (int)(ord & 2047u) << L, y = (int)((ord >> 11) & 2047u) << L;
        keep += x >= cfg.border && x < cfg.W - cfg.border && y >= cfg.border && y < cfg.H - cfg.border;
    }
    int o, d2, total, d3;
    block_scan2(keep, 0, o, d2, total, d3, sh);
    for (int j = 0; j < E2; j++) {
        const int i = base2 + j;
        if (i >= m) break;
        const unsigned long long kv = cells[I[i]];
        const uint32_t ord = ~(uint32_t)kv;
        const int L = ord >> 22, x = (int)(ord & 2047u) << L, y = (int)((ord >> 11) & 2047u) << L;
        if (!(x >= cfg.border && x < cfg.W - cfg.border && y >= cfg.border && y < cfg.H - cfg.border)) continue;
        if (o < cfg.kp_cap) {
            float* K = kps + ((size_t)b * cfg.kp_cap + o) * 7;
            K[0] = (float)x;
            K[1] = (float)y;
            K[2] = 0.0f;
            K[3] = -1.0f;
            K[4] = __uint_as_float((uint32_t)(kv >> 32));
            reinterpret_cast<int*>(K)[5] = L;
            reinterpret_cast<int*>(K)[6] = -1;
        }
        o++;
    }
    if (tid == 0) {
        counts[b] = min(total, cfg.kp_cap);
        if (total > cfg.kp_cap) err[b] |= 2;   // one block per frame
    }
    SEL_PROF(47);
    __syncthreads();
    for (int i = tid; i < NC; i += T) cells[i] = 0ull;
    SEL_PROF(48);
}

__global__ __launch_bounds__(kSvoSelThreads) void k_svo_retain_test(const float* __restrict__ resp, int n, int nkeep,
                                                                    int depth_limit, int* __restrict__ order,
                                                                    int* __restrict__ mout)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ SelLds sh;
    float* R = reinterpret_cast<float*>(smem);
    uint16_t* I = reinterpret_cast<uint16_t*>(R + n);
    uint16_t* posL = I + n;
    uint16_t* posR = posL + n;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        R[i] = resp[i];
        I[i] = (uint16_t)i;
    }
    if (threadIdx.x == 0) sh.phase = 0;
    __syncthreads();
    int m = n;
    if (n > nkeep) m = nkeep > 0 ? retain_best_block(R, I, posL, posR, n, nkeep, sh, depth_limit) : 0;
    for (int i = threadIdx.x; i < m; i += blockDim.x) order[i] = I[i];
    if (threadIdx.x == 0) *mout = m;
}

// ------------------------------------------------------------------ BRIEF-32 tests (one wave per keypoint)
// pixelTests32 with use_orientation false: bit t = SMOOTHED(y1, x1) < SMOOTHED(y2, x2) at the keypoint
// rounded by (int)(pt + 0.5); lane l runs tests l, l+64, l+128, l+192, a ballot gives 64 bits and a
// per-byte bit reversal puts test 8i+k at bit 7-k of byte i (the generated code's << (7 - k)).
constexpr int kBriefWaves = 4;
__global__ __launch_bounds__(64 * kBriefWaves) void k_svo_brief(const uint16_t* __restrict__ box,
                                                                const int* __restrict__ counts,
                                                                const float* __restrict__ kps,
                                                                const uint32_t* __restrict__ pattern, SvoCfg cfg,
                                                                uint8_t* __restrict__ desc)
{
    const int b = blockIdx.y, lane = threadIdx.x & 63;
    const int i = blockIdx.x * kBriefWaves + (threadIdx.x >> 6);
    if (i >= counts[b]) return;
    const size_t o = (size_t)b * cfg.kp_cap + i;
    const float* K = kps + o * 7;
    const int x = (int)(K[0] + 0.5f), y = (int)(K[1] + 0.5f);
    const uint16_t* bx = box + (size_t)b * cfg.W * cfg.H + (size_t)y * cfg.W + x;
    unsigned long long word[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t pt = pattern[lane + 64 * q];
        const int y1 = (int8_t)(pt & 255u), x1 = (int8_t)((pt >> 8) & 255u);
        const int y2 = (int8_t)((pt >> 16) & 255u), x2 = (int8_t)(pt >> 24);
        const bool bit = bx[y1 * cfg.W + x1] < bx[y2 * cfg.W + x2];
        word[q] = __builtin_bswap64(__builtin_bitreverse64(__ballot(bit)));
    }
    if (lane < 4) {
        const unsigned long long w = lane == 0 ? word[0] : lane == 1 ? word[1] : lane == 2 ? word[2] : word[3];
        reinterpret_cast<unsigned long long*>(desc + o * 32)[lane] = w;
    }
}

#ifdef RGBD_PNP_PROFILE
void svo_prof_dump(hipStream_t st)
{
    static long long p[64];
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(p, HIP_SYMBOL(g_sel_prof), sizeof(p));
    const int it = (int)p[60];
    fprintf(stderr, "[sel_prof] n=%lld iters=%d load %.2f us | iters:", p[61], it, 0.0);
    long long prev = p[1];
    (void)prev;
    fprintf(stderr, " (stamps in us from start)");
    for (int k = 0; k < it && k < 40; k++) fprintf(stderr, " %.1f", (p[2 + k] - p[0]) * 0.01);
    fprintf(stderr, " | loop end %.1f partition %.1f step2 end %.1f counts %.1f end %.1f\n", (p[45] - p[0]) * 0.01,
            (p[46] - p[0]) * 0.01, (p[1] - p[0]) * 0.01, (p[47] - p[0]) * 0.01, (p[48] - p[0]) * 0.01);
}
#endif

// ------------------------------------------------------------------ launchers
hipError_t launch_svo_pyramid(const uint8_t* bgr, uint8_t* pyr, uint16_t* box, const SvoCfg& cfg, int B, hipStream_t st)
{
    return dispatch(k_svo_pyramid, dim3((cfg.W + kPyrT - 1) / kPyrT, (cfg.H + kPyrT - 1) / kPyrT, B), dim3(256), 0, st,
                       bgr, pyr, box, cfg);
}

hipError_t launch_svo_detect(const uint8_t* pyr, const SvoTile* tiles, int ntiles, const SvoCfg& cfg,
                       unsigned long long* cell_keys, int B, hipStream_t st)
{
    return dispatch(k_svo_detect, dim3(ntiles, B), dim3(256), 0, st, pyr, tiles, cfg, cell_keys);   // ntiles 0: nothing queued
}

size_t svo_select_lds_bytes(const SvoCfg& cfg) { return (size_t)cfg.ncells * 10 + 16; }

hipError_t launch_svo_select(unsigned long long* cell_keys, const SvoCfg& cfg, uint2* cand, int* ncand, int* counts,
                       float* kps, int* err, int B, hipStream_t st)
{
    return dispatch(k_svo_select, dim3(B), dim3(kSvoSelThreads), svo_select_lds_bytes(cfg), st, cell_keys, cfg,
                       cand, ncand, counts, kps, err);
}

hipError_t launch_svo_brief(const uint16_t* box, const int* counts, const float* kps, const uint32_t* pattern,
                      const SvoCfg& cfg, uint8_t* desc, int B, hipStream_t st)
{
    return dispatch(k_svo_brief, dim3((cfg.kp_cap + kBriefWaves - 1) / kBriefWaves, B), dim3(64 * kBriefWaves), 0,
                       st, box, counts, kps, pattern, cfg, desc);
}

hipError_t launch_svo_retain_test(const float* resp, int n, int nkeep, int depth_limit, int* order, int* m, hipStream_t st)
{
    return dispatch(k_svo_retain_test, dim3(1), dim3(kSvoSelThreads), (size_t)n * 10 + 16, st, resp, n, nkeep,
                       depth_limit, order, m);
}

}  // namespace rgbd

// svo.hip -- the reference's DEFAULT front end on gfx950: Extractor(SVO, BRIEF, NORMAL) (main.cpp:31).
//   Frame::Frame cvtColor            Core/Frame.cpp:47            -> k_svo_pyramid (fused)
//   SVOextractor::createImagePyramid Features/SVOextractor.cpp:139-148, halfSample :16-37 -> k_svo_pyramid
//   SVOextractor::detect             :86-137: fast_corner_detect_10 + fast_corner_score_10 + fast_nonmax_3x3
//                                    + ShiTomasiScore (:39-84) + the 5-px grid               -> k_svo_detect
//   Extractor::detectAndCompute      Features/Extractor.cpp:50-61: retainBest(nfeatures)     -> k_svo_select
//   BriefDescriptorExtractor::compute (xfeatures2d, 32 B): runByImageBorder(28) -> k_svo_select,
//                                    integral-image 9x9 box sums -> k_svo_box, 256 tests -> k_svo_brief
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

#include <climits>
#include <cstdint>

#include "svo_dev.h"

namespace rgbd {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// ------------------------------------------------------------------ pyramid (gray + halfSample)
// One 256-thread workgroup per 128 x 128 level-0 tile: BGR -> gray (cvtColor 8U fixed point) into LDS
// and HBM, then each level's 2x2 means from the previous level's tile in LDS.  A level-L pixel inside
// the level only reads level-(L-1) pixels inside that level, so tiles never exchange data.
constexpr int kPyrT = 128;

__global__ __launch_bounds__(256) void k_svo_pyramid(const uint8_t* __restrict__ bgr, uint8_t* __restrict__ pyr,
                                                     SvoCfg cfg)
{
    __shared__ __attribute__((aligned(16))) uint8_t A[kPyrT * kPyrT];
    __shared__ __attribute__((aligned(16))) uint8_t Bt[(kPyrT / 2) * (kPyrT / 2)];
    const int tid = threadIdx.x, b = blockIdx.z;
    const int tx0 = blockIdx.x * kPyrT, ty0 = blockIdx.y * kPyrT;
    const int W = cfg.W, H = cfg.H;
    uint8_t* P = pyr + (size_t)b * cfg.frame_bytes;
    // level 0: 128 rows x 8 groups of 16 pixels
    for (int g = tid; g < kPyrT * 8; g += 256) {
        const int r = g >> 3, c16 = (g & 7) << 4;
        const int y = ty0 + r, x = tx0 + c16;
        uint8_t out[16];
        if (y < H && x < W) {
            if (bgr) {
                const uint8_t* src = bgr + ((size_t)b * W * H + (size_t)y * W + x) * 3;
                if (x + 16 <= W && (W & 15) == 0 && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
                    uint8_t in[48];
                    const uint4* s4 = reinterpret_cast<const uint4*>(src);
                    *reinterpret_cast<uint4*>(in) = s4[0];
                    *reinterpret_cast<uint4*>(in + 16) = s4[1];
                    *reinterpret_cast<uint4*>(in + 32) = s4[2];
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        out[i] = (uint8_t)((in[3 * i] * 1868 + in[3 * i + 1] * 9617 + in[3 * i + 2] * 4899 + (1 << 13)) >> 14);
                    *reinterpret_cast<uint4*>(P + (size_t)y * W + x) = *reinterpret_cast<uint4*>(out);
                } else {
                    for (int i = 0; i < 16; i++) {
                        out[i] = 0;
                        if (x + i < W) {
                            out[i] = (uint8_t)((src[3 * i] * 1868 + src[3 * i + 1] * 9617 + src[3 * i + 2] * 4899 + (1 << 13)) >> 14);
                            P[(size_t)y * W + x + i] = out[i];
                        }
                    }
                }
            } else {   // level 0 already holds the gray image (rgbd_detect_and_compute)
                for (int i = 0; i < 16; i++) out[i] = x + i < W ? P[(size_t)y * W + x + i] : 0;
            }
#pragma unroll
            for (int i = 0; i < 16; i++) A[r * kPyrT + c16 + i] = out[i];
        }
    }
    __syncthreads();
    uint8_t* src = A;
    uint8_t* dst = Bt;
    int sd = kPyrT;
    for (int L = 1; L < cfg.nlevels; L++) {
        const int d = sd >> 1;
        const int lx0 = tx0 >> L, ly0 = ty0 >> L, lw = cfg.lw[L], lh = cfg.lh[L];
        uint8_t* PL = P + cfg.loff[L];
        for (int i = tid; i < d * d; i += 256) {
            const int r = i / d, c = i - r * d;
            const uint8_t* s = src + (2 * r) * sd + 2 * c;
            const int v = ((int)s[0] + s[1] + s[sd] + s[sd + 1]) >> 2;
            dst[r * d + c] = (uint8_t)v;
            if (lx0 + c < lw && ly0 + r < lh) PL[(size_t)(ly0 + r) * lw + lx0 + c] = (uint8_t)v;
        }
        __syncthreads();
        uint8_t* t = src;
        src = dst;
        dst = t;
        sd = d;
    }
}

// ------------------------------------------------------------------ FAST-10 + NMS + Shi-Tomasi + grid
constexpr int kDetTW = 64, kDetTH = 16, kDetHalo = 5;
constexpr int kDetGW = kDetTW + 2 * kDetHalo + 2;   // staged columns (74 used, 2 zero pad)
constexpr int kDetGH = kDetTH + 2 * kDetHalo;       // 26 staged rows
constexpr int kDetSW = kDetTW + 2, kDetSH = kDetTH + 2;   // score map: the tile + 1-pixel ring

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

// ShiTomasiScore (Features/SVOextractor.cpp:39-84) at staged (gr, gc): the three sums are integers below
// 2^24, so integer accumulation equals the reference's float accumulation; the rest keeps its order.
__device__ __forceinline__ float shi_tomasi_lds(const uint8_t* G, int gr, int gc)
{
    int sxx = 0, syy = 0, sxy = 0;
    for (int r = gr - 4; r < gr + 4; r++) {
        const uint8_t* row = G + r * kDetGW;
#pragma unroll
        for (int c = gc - 4; c < gc + 4; c++) {
            const int dx = (int)row[c + 1] - (int)row[c - 1];
            const int dy = (int)row[c + kDetGW] - (int)row[c - kDetGW];
            sxx += dx * dx;
            syy += dy * dy;
            sxy += dx * dy;
        }
    }
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
    __shared__ uint8_t S[kDetSH * kDetSW];
    __shared__ uint16_t list[kDetTW * kDetTH];
    __shared__ int nlist;
    const int tid = threadIdx.x, b = blockIdx.y;
    const SvoTile t = tiles[blockIdx.x];
    const int L = t.level, w = cfg.lw[L], h = cfg.lh[L];
    const int x0 = t.x0, y0 = t.y0;
    const uint8_t* img = pyr + (size_t)b * cfg.frame_bytes + cfg.loff[L];
    if (tid == 0) nlist = 0;
    // 1. stage rows y0-5 .. y0+20, columns x0-5 .. x0+70 (zero outside the level)
    for (int i = tid; i < kDetGH * kDetGW; i += 256) {
        const int r = i / kDetGW, c = i - r * kDetGW;
        const int y = y0 - kDetHalo + r, x = x0 - kDetHalo + c;
        G[i] = (y >= 0 && y < h && x >= 0 && x < w && c < kDetGW - 2) ? img[(size_t)y * w + x] : (uint8_t)0;
    }
    __syncthreads();
    for (int i = tid; i < kDetGH * kDetGW; i += 256) {
        const int c = i % kDetGW;
        PI[i] = (uint32_t)G[i] | ((c + 1 < kDetGW ? (uint32_t)G[i + 1] : 0u) << 16);
    }
    __syncthreads();
    // 2. score map over the tile + 1-pixel ring: S = m - 1 where m > barrier (a FAST-10 corner), else 0;
    //    pixels outside the detector's domain [3, w-3) x [3, h-3) are never corners
    for (int task = tid; task < kDetSH * (kDetSW / 2); task += 256) {
        const int sr = task / (kDetSW / 2), cp = task - sr * (kDetSW / 2);
        const int ty = sr - 1, tx = 2 * cp - 1;   // tile coordinates of the pair's first pixel
        const u16x2 m = fast10_m2(PI, kDetGW, ty + kDetHalo, tx + kDetHalo);
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
    // 3. fast_nonmax_3x3: a corner survives iff no 8-neighbour corner scores >= it
    for (int i = tid; i < kDetTW * kDetTH; i += 256) {
        const int ty = i / kDetTW, tx = i - ty * kDetTW;
        const uint8_t* s = S + (ty + 1) * kDetSW + tx + 1;
        const int v = s[0];
        if (v == 0) continue;
        const int nb = max(max(max(s[-kDetSW - 1], s[-kDetSW]), max(s[-kDetSW + 1], s[-1])),
                           max(max(s[1], s[kDetSW - 1]), max(s[kDetSW], s[kDetSW + 1])));
        if (nb >= v) continue;
        if (x0 + tx >= w || y0 + ty >= h) continue;
        list[atomicAdd(&nlist, 1)] = (uint16_t)i;
    }
    __syncthreads();
    // 4. Shi-Tomasi of each survivor, then the grid: the reference keeps the first strictly greater
    //    score of a cell over levels 0.. and raster order, i.e. the max of (score, ~(level, y, x))
    const int n = nlist;
    const int sc = 1 << L;
    for (int j = tid; j < n; j += 256) {
        const int i = list[j];
        const int ty = i / kDetTW, tx = i - ty * kDetTW;
        const int X = x0 + tx, Y = y0 + ty;
        if (X < 5 || X > w - 6 || Y < 5 || Y > h - 6) continue;   // patch too close to the boundary: 0
        const float score = shi_tomasi_lds(G, ty + kDetHalo, tx + kDetHalo);
        if (!(score > 0.0f)) continue;
        const int k = ((Y * sc) / cfg.cell) * cfg.gcols + (X * sc) / cfg.cell;
        const uint32_t ord = ((uint32_t)L << 22) | ((uint32_t)Y << 11) | (uint32_t)X;
        const unsigned long long key = ((unsigned long long)__float_as_uint(score) << 32) | (unsigned long long)(~ord);
        atomicMax(cell_keys + (size_t)b * cfg.ncells + k, key);
    }
}

// ------------------------------------------------------------------ 9x9 box sums (BRIEF smoothing)
// box[y][x] = sum of gray over [y-4, y+4] x [x-4, x+4] == the four-corner integral-image difference of
// smoothedSum (KERNEL_SIZE 9).  Defined for 4 <= x < W-4, 4 <= y < H-4 (0 elsewhere, never sampled).
constexpr int kBoxTW = 64, kBoxTH = 16;
__global__ __launch_bounds__(256) void k_svo_box(const uint8_t* __restrict__ pyr, uint16_t* __restrict__ box, SvoCfg cfg)
{
    __shared__ uint8_t g[(kBoxTH + 8) * (kBoxTW + 8)];
    __shared__ uint16_t hs[(kBoxTH + 8) * kBoxTW];
    const int tid = threadIdx.x, b = blockIdx.z;
    const int x0 = blockIdx.x * kBoxTW, y0 = blockIdx.y * kBoxTH;
    const int W = cfg.W, H = cfg.H;
    const uint8_t* img = pyr + (size_t)b * cfg.frame_bytes;
    for (int i = tid; i < (kBoxTH + 8) * (kBoxTW + 8); i += 256) {
        const int r = i / (kBoxTW + 8), c = i - r * (kBoxTW + 8);
        const int y = y0 - 4 + r, x = x0 - 4 + c;
        g[i] = (y >= 0 && y < H && x >= 0 && x < W) ? img[(size_t)y * W + x] : (uint8_t)0;
    }
    __syncthreads();
    for (int i = tid; i < (kBoxTH + 8) * kBoxTW; i += 256) {
        const int r = i / kBoxTW, c = i - r * kBoxTW;
        const uint8_t* s = g + r * (kBoxTW + 8) + c;
        int v = 0;
#pragma unroll
        for (int k = 0; k < 9; k++) v += s[k];
        hs[i] = (uint16_t)v;
    }
    __syncthreads();
    uint16_t* out = box + (size_t)b * W * H;
    for (int i = tid; i < kBoxTH * kBoxTW; i += 256) {
        const int r = i / kBoxTW, c = i - r * kBoxTW;
        const int y = y0 + r, x = x0 + c;
        if (y >= H || x >= W) continue;
        int v = 0;
#pragma unroll
        for (int k = 0; k < 9; k++) v += hs[(r + k) * kBoxTW + c];
        out[(size_t)y * W + x] = (x >= 4 && x < W - 4 && y >= 4 && y < H - 4) ? (uint16_t)v : (uint16_t)0;
    }
}

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
    int wa[16], wb[16];
};

__device__ __forceinline__ int wave_incl_scan(int v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

// exclusive block scan of (a, b) in thread order (all threads of the block call it)
__device__ __forceinline__ void block_scan2(int a, int b, int& ea, int& eb, int& ta, int& tb, SelLds& sh)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int ia = wave_incl_scan(a), ib = wave_incl_scan(b);
    if (lane == 63) { sh.wa[w] = ia; sh.wb[w] = ib; }
    __syncthreads();
    int pa = 0, pb = 0;
    ta = 0;
    tb = 0;
    for (int i = 0; i < nw; i++) {
        const int x = sh.wa[i], y = sh.wb[i];
        if (i < w) { pa += x; pb += y; }
        ta += x;
        tb += y;
    }
    __syncthreads();
    ea = pa + ia - a;
    eb = pb + ib - b;
}

// Pair the left stoppers (mode 0: !(x > p); mode 1: !(x >= p)) with the right stoppers (mode 0: !(p > x);
// mode 1: x >= p) of [a, e) and swap every pair whose left stopper lies before its right one.  Returns K
// (swaps), L_K (the K-th left stopper, INT_MAX if none) and R_{K-1} (-1 if K == 0); TB = right stoppers.
__device__ int pair_swap(float* R, uint16_t* I, uint16_t* posL, uint16_t* posR, int a, int e, float p, int mode,
                         int& LK, int& RK1, int& TB, SelLds& sh)
{
    const int T = blockDim.x, tid = threadIdx.x;
    const int len = e - a;
    const int E = (len + T - 1) / T;
    const int base = a + tid * E;
    float v[kSvoSelMaxE];
    uint16_t id[kSvoSelMaxE];
    unsigned fA = 0, fB = 0;
    int ca = 0, cb = 0;
#pragma unroll
    for (int j = 0; j < kSvoSelMaxE; j++) {
        const int i = base + j;
        v[j] = 0.f;
        id[j] = 0;
        if (j < E && i < e) {
            v[j] = R[i];
            id[j] = I[i];
            const bool A = mode == 0 ? !(v[j] > p) : !(v[j] >= p);
            const bool Bq = mode == 0 ? !(p > v[j]) : (v[j] >= p);
            fA |= (unsigned)A << j;
            fB |= (unsigned)Bq << j;
            ca += A;
            cb += Bq;
        }
    }
    int ea, eb, TA;
    block_scan2(ca, cb, ea, eb, TA, TB, sh);
    int ka = ea, kb = eb, nsw = 0;
    unsigned sA = 0, sB = 0;
#pragma unroll
    for (int j = 0; j < kSvoSelMaxE; j++) {
        const int i = base + j;
        if (j < E && i < e) {
            const int A = (fA >> j) & 1, Bq = (fB >> j) & 1;
            if (A) {
                posL[ka] = (uint16_t)i;
                if (TB - kb - Bq >= ka + 1) { sA |= 1u << j; nsw++; }   // a right stopper of rank ka lies after i
            }
            if (Bq) {
                const int kr = TB - 1 - kb;
                posR[kr] = (uint16_t)i;
                if (ka >= kr + 1) sB |= 1u << j;                        // a left stopper of rank kr lies before i
            }
            ka += A;
            kb += Bq;
        }
    }
    int K, dummy0, dummy1, dummy2;
    block_scan2(nsw, 0, dummy0, dummy1, K, dummy2, sh);   // also orders the pos writes before the reads
    LK = K < TA ? (int)posL[K] : INT_MAX;
    RK1 = K > 0 ? (int)posR[K - 1] : -1;
    int dest[kSvoSelMaxE];
    ka = ea;
    kb = eb;
#pragma unroll
    for (int j = 0; j < kSvoSelMaxE; j++) {
        dest[j] = -1;
        const int i = base + j;
        if (j < E && i < e) {
            const int A = (fA >> j) & 1, Bq = (fB >> j) & 1;
            if ((sA >> j) & 1) dest[j] = posR[ka];
            else if ((sB >> j) & 1) dest[j] = posL[TB - 1 - kb];
            ka += A;
            kb += Bq;
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kSvoSelMaxE; j++)
        if (dest[j] >= 0) {
            R[dest[j]] = v[j];
            I[dest[j]] = id[j];
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
    }
    if (!heap) {
        if (threadIdx.x == 0) insertion_sort_one_lane(R, I, f, l);
        __syncthreads();
    }
    // std::partition(begin + nkeep, end, response >= R[nkeep - 1]): the kept prefix grows by the preds
    const float amb = R[nth];
    int LK, RK1, TB;
    pair_swap(R, I, posL, posR, nkeep, n, amb, 1, LK, RK1, TB, sh);
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
    // 1.
    unsigned long long key[kSvoSelMaxE];
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < kSvoSelMaxE; j++) {
        key[j] = 0;
        if (j < E && base + j < NC) {
            key[j] = cells[base + j];
            cnt += __uint_as_float((uint32_t)(key[j] >> 32)) > 20.0f;
        }
    }
    int off, d0, n, d1;
    block_scan2(cnt, 0, off, d0, n, d1, sh);
#pragma unroll
    for (int j = 0; j < kSvoSelMaxE; j++) {
        const float s = __uint_as_float((uint32_t)(key[j] >> 32));
        if (j < E && base + j < NC && s > 20.0f) {
            R[off] = s;
            I[off] = (uint16_t)(base + j);
            cand[(size_t)b * NC + off] = make_uint2((uint32_t)(key[j] >> 32), (uint32_t)key[j]);
            off++;
        }
    }
    if (tid == 0) ncand[b] = n;
    __syncthreads();
    // 2.
    int m = n;
    if (n > cfg.nfeatures) m = cfg.nfeatures > 0 ? retain_best_block(R, I, posL, posR, n, cfg.nfeatures, sh) : 0;
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
        if (total > cfg.kp_cap) atomicOr(err, 2);
    }
    __syncthreads();
    for (int i = tid; i < NC; i += T) cells[i] = 0ull;
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

// ------------------------------------------------------------------ launchers
void launch_svo_pyramid(const uint8_t* bgr, uint8_t* pyr, const SvoCfg& cfg, int B, hipStream_t st)
{
    hipLaunchKernelGGL(k_svo_pyramid, dim3((cfg.W + kPyrT - 1) / kPyrT, (cfg.H + kPyrT - 1) / kPyrT, B), dim3(256), 0, st,
                       bgr, pyr, cfg);
}

void launch_svo_detect(const uint8_t* pyr, const SvoTile* tiles, int ntiles, const SvoCfg& cfg,
                       unsigned long long* cell_keys, int B, hipStream_t st)
{
    if (ntiles > 0)
        hipLaunchKernelGGL(k_svo_detect, dim3(ntiles, B), dim3(256), 0, st, pyr, tiles, cfg, cell_keys);
}

void launch_svo_box(const uint8_t* pyr, uint16_t* box, const SvoCfg& cfg, int B, hipStream_t st)
{
    hipLaunchKernelGGL(k_svo_box, dim3((cfg.W + kBoxTW - 1) / kBoxTW, (cfg.H + kBoxTH - 1) / kBoxTH, B), dim3(256), 0,
                       st, pyr, box, cfg);
}

size_t svo_select_lds_bytes(const SvoCfg& cfg) { return (size_t)cfg.ncells * 10 + 16; }

void launch_svo_select(unsigned long long* cell_keys, const SvoCfg& cfg, uint2* cand, int* ncand, int* counts,
                       float* kps, int* err, int B, hipStream_t st)
{
    hipLaunchKernelGGL(k_svo_select, dim3(B), dim3(kSvoSelThreads), svo_select_lds_bytes(cfg), st, cell_keys, cfg,
                       cand, ncand, counts, kps, err);
}

void launch_svo_brief(const uint16_t* box, const int* counts, const float* kps, const uint32_t* pattern,
                      const SvoCfg& cfg, uint8_t* desc, int B, hipStream_t st)
{
    hipLaunchKernelGGL(k_svo_brief, dim3((cfg.kp_cap + kBriefWaves - 1) / kBriefWaves, B), dim3(64 * kBriefWaves), 0,
                       st, box, counts, kps, pattern, cfg, desc);
}

void launch_svo_retain_test(const float* resp, int n, int nkeep, int depth_limit, int* order, int* m, hipStream_t st)
{
    hipLaunchKernelGGL(k_svo_retain_test, dim3(1), dim3(kSvoSelThreads), (size_t)n * 10 + 16, st, resp, n, nkeep,
                       depth_limit, order, m);
}

}  // namespace rgbd

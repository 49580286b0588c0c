// extract.hip -- gfx950 kernels of the ORB2 extractor + Frame glue (batched over frames).
//
// Reference path (toniortiz/rgbd-slam):
//   Frame::Frame            Core/Frame.cpp:34-73   (cvtColor, convertTo, undistort, unproject)
//   ORBextractor::operator() Features/ORBextractor.cpp:706-766
//     cvtColor + ComputePyramid  Core/Frame.cpp:47, :773-797 -> k_pyramid (k_gray for 1-level pyramids)
//     ComputeKeyPointsOctTree :613-695 -> k_fast (per-cell FAST + 20->7 fallback), k_distribute
//     DistributeOctTree      :414-611  -> k_distribute (quadtree, parallel restatement)
//     IC_Angle / blur / computeOrbDescriptor :16-87, :745-750 -> k_describe
//
// Layout in HBM (per batch of B frames):
//   pyr   [B][frame_pyr_bytes]          levels 0..L-1, rows padded to 64 B
//   cellc [B][n_cells] i32, cells [B][n_cells][cell_cap] u32 (packed x|y|score, raster order)
//   keys  [B][keys_per_frame] u32 + node [B][keys_per_frame] u16 (quadtree scratch)
//   selc  [B][L] i32, sel [B][sel_per_frame] u32 (quadtree output, list order)
//   out   counts[B], kps/kps_un [B][kp_cap] (cv::KeyPoint), desc [B][kp_cap][32], xyz [B][kp_cap][3]
//
// Every integer stage is bit-exact with the oracle; float/double stages use the same
// operation order with -ffp-contract=off (no FMA), IEEE division/sqrt.
#include <hip/hip_runtime.h>
#include <type_traits>

#include "dispatch.h"

#include "rgbd_internal.h"

namespace rgbd {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

constexpr int kPatternRaw[256 * 4] = {
#include "orb_pattern.inc"
};
// the same table with each test packed into one dword (x0, y0, x1, y1 as int8, coordinates in [-13, 12])
struct Pattern8 { uint32_t v[256]; };
constexpr Pattern8 make_pattern8()
{
    Pattern8 p{};
    for (int t = 0; t < 256; t++) {
        uint32_t w = 0;
        for (int i = 0; i < 4; i++) w |= (uint32_t)(uint8_t)(int8_t)kPatternRaw[4 * t + i] << (8 * i);
        p.v[t] = w;
    }
    return p;
}
__constant__ Pattern8 c_pattern8 = make_pattern8();

// ------------------------------------------------------------------ gray (Core/Frame.cpp:47)
// cvtColor BGR2GRAY 8U fixed point: (B*1868 + G*9617 + R*4899 + 8192) >> 14.  16 px per thread,
// three 16-B loads and one 16-B store.
__global__ __launch_bounds__(256) void k_gray(const uint8_t* __restrict__ bgr, uint8_t* __restrict__ pyr,
                                               int W, int H, int frame_pyr_bytes, int B)
{
    const int groups_per_frame = (W * H) >> 4;
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= groups_per_frame * B)
        return;
    const int b = gid / groups_per_frame;
    const int g = gid - b * groups_per_frame;
    const size_t pix = (size_t)g << 4;
    const uint4* src = reinterpret_cast<const uint4*>(bgr + ((size_t)b * W * H + pix) * 3);
    const uint4 v0 = src[0], v1 = src[1], v2 = src[2];
    uint8_t in[48];
    *reinterpret_cast<uint4*>(in) = v0;
    *reinterpret_cast<uint4*>(in + 16) = v1;
    *reinterpret_cast<uint4*>(in + 32) = v2;
    uint8_t out[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const int B_ = in[3 * i], G_ = in[3 * i + 1], R_ = in[3 * i + 2];
        out[i] = (uint8_t)((B_ * 1868 + G_ * 9617 + R_ * 4899 + (1 << 13)) >> 14);
    }
    const int y = (int)(pix / W), x = (int)(pix - (size_t)y * W);
    // level 0 stride == W when W % 64 == 0 (host enforces W % 16 == 0 and stride == align64(W))
    uint8_t* dst = pyr + (size_t)b * frame_pyr_bytes;
    const int stride0 = (W + 63) & ~63;
    *reinterpret_cast<uint4*>(dst + (size_t)y * stride0 + x) = *reinterpret_cast<const uint4*>(out);
}

// ------------------------------------------------------------------ resize (:786-790)
// OpenCV 3.4 INTER_LINEAR 8U: horizontal int taps (11-bit weights); vertical pass = SSE2
// VResizeLinearVec_32s8u arithmetic on [0, rs_simd), FixedPtCast<int,uchar,22> on the tail.
// cv::resize INTER_LINEAR tables (api.cpp resize_tables, the same float / double operations)
__device__ __forceinline__ ResizeX resize_xt(int dx, double scale_x, int sw)
{
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = (int)floorf(fx);
    fx -= sx;
    if (sx < 0) { fx = 0; sx = 0; }
    if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
    const float c0 = 1.f - fx, c1 = fx;
    ResizeX r;
    r.sx = (int16_t)sx;
    r.a0 = (int16_t)min(max((int)rintf(c0 * 2048), -32768), 32767);
    r.a1 = (int16_t)min(max((int)rintf(c1 * 2048), -32768), 32767);
    r.pad = (int16_t)(sx + 1 < sw ? sx + 1 : sx);
    return r;
}

__device__ __forceinline__ ResizeY resize_yt(int y, double scale_y, int sh)
{
    float fy = (float)((y + 0.5) * scale_y - 0.5);
    const int sy = (int)floorf(fy);
    fy -= sy;
    const float c0 = 1.f - fy, c1 = fy;
    ResizeY r;
    r.sy0 = (int16_t)(sy >= 0 ? (sy < sh ? sy : sh - 1) : 0);
    r.sy1 = (int16_t)(sy + 1 >= 0 ? (sy + 1 < sh ? sy + 1 : sh - 1) : 0);
    r.b0 = (int16_t)min(max((int)rintf(c0 * 2048), -32768), 32767);
    r.b1 = (int16_t)min(max((int)rintf(c1 * 2048), -32768), 32767);
    return r;
}

// The vertical pass of one output byte from the two horizontal sums r0, r1 (rows sy0, sy1).  All
// weights are non-negative and sum to ~2048, so the int16 saturations of VResizeLinearVec_32s8u never
// engage (|r >> 4| <= 32655, m0 + m1 + 2 <= 2042): they are omitted.  Every product has operands
// below 2^23 (r >> 4 15 bits, r 20, weights 12): the full-rate 24-bit multiplies are exact.
// resize_vs = the SSE2 form on [0, rs_simd), resize_vt = the scalar FixedPtCast<int, uchar, 22> tail.
__device__ __forceinline__ int resize_vs(int r0, int r1, const ResizeY ry)
{
    return min(((__mul24(r0 >> 4, ry.b0) >> 16) + (__mul24(r1 >> 4, ry.b1) >> 16) + 2) >> 2, 255);
}
__device__ __forceinline__ int resize_vt(int r0, int r1, const ResizeY ry)
{
    return min((__mul24(r0, ry.b0) + __mul24(r1, ry.b1) + (1 << 21)) >> 22, 255);
}

// cvtColor BGR2GRAY of 4 pixels (12 bytes in dwords d0..d2): (B, G) of each pixel as a zero-extended u16
// pair by v_perm, 4 (1868 B + 9617 G + 4899 R) + 2^15 by two v_dot2, and the result (X + 8192) >> 14 is
// byte 2 of that sum (< 2^24), gathered by two v_perm
__device__ __forceinline__ uint32_t gray4(uint32_t d0, uint32_t d1, uint32_t d2)
{
    const u16x2 kbg = {7472, 38468}, kr = {19596, 0};
    const uint32_t bg[4] = {__builtin_amdgcn_perm(d1, d0, 0x0c010c00u), __builtin_amdgcn_perm(d1, d0, 0x0c040c03u),
                            __builtin_amdgcn_perm(d2, d1, 0x0c030c02u), __builtin_amdgcn_perm(d2, d1, 0x0c060c05u)};
    const uint32_t rr[4] = {__builtin_amdgcn_perm(d1, d0, 0x0c0c0c02u), __builtin_amdgcn_perm(d1, d0, 0x0c0c0c05u),
                            __builtin_amdgcn_perm(d2, d1, 0x0c0c0c04u), __builtin_amdgcn_perm(d2, d1, 0x0c0c0c07u)};
    uint32_t a[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
        a[i] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, rr[i]), kr,
                                      __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, bg[i]), kbg, 1u << 15, false), false);
    return __builtin_amdgcn_perm(a[1], a[0], 0x0c0c0602u) | __builtin_amdgcn_perm(a[3], a[2], 0x06020c0cu);
}

__device__ __forceinline__ uint4 gray16(uint4 v0, uint4 v1, uint4 v2)
{
    return make_uint4(gray4(v0.x, v0.y, v0.z), gray4(v0.w, v1.x, v1.y), gray4(v1.z, v1.w, v2.x), gray4(v2.y, v2.z, v2.w));
}

__device__ __forceinline__ int reflect101(int p, int n)
{
    if (n == 1) return 0;
    while (p < 0 || p >= n) {
        if (p < 0) p = -p;
        if (p >= n) p = 2 * n - 2 - p;
    }
    return p;
}

// Horizontal 7-tap sums (x 256) of the column quad px 4q .. 4q + 3: bytes 4q + j - 3 .. 4q + j + 3 of
// (d0 = 4q - 4 .. 4q - 1, d1, d2).  The 7 taps split over the three dwords as shifted weight quads
// (10 v_dot4, no byte alignment); every sum <= 255 * 256 = 65280 fits a u16.
__device__ __forceinline__ void blur_h4(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t* h)
{
    constexpr uint32_t k0a = (18u << 8) | (34u << 16) | (49u << 24), k0b = 54u | (49u << 8) | (34u << 16) | (18u << 24);
    constexpr uint32_t k1a = (18u << 16) | (34u << 24), k1b = 49u | (54u << 8) | (49u << 16) | (34u << 24), k1c = 18u;
    constexpr uint32_t k2a = 18u << 24, k2b = 34u | (49u << 8) | (54u << 16) | (49u << 24), k2c = 34u | (18u << 8);
    constexpr uint32_t k3b = 18u | (34u << 8) | (49u << 16) | (54u << 24), k3c = 49u | (34u << 8) | (18u << 16);
    h[0] = __builtin_amdgcn_udot4(d1, k0b, __builtin_amdgcn_udot4(d0, k0a, 0u, false), false);
    h[1] = __builtin_amdgcn_udot4(d2, k1c, __builtin_amdgcn_udot4(d1, k1b, __builtin_amdgcn_udot4(d0, k1a, 0u, false), false), false);
    h[2] = __builtin_amdgcn_udot4(d2, k2c, __builtin_amdgcn_udot4(d1, k2b, __builtin_amdgcn_udot4(d0, k2a, 0u, false), false), false);
    h[3] = __builtin_amdgcn_udot4(d2, k3c, __builtin_amdgcn_udot4(d1, k3b, 0u, false), false);
}

// The vertical half of the 7x7 blur over one column quad, as a window of ROW PAIRS: P[k][j] packs pixel
// j's horizontal sums of input rows (r - 1, r) as u16 (lo, hi), for the last six rows r (the loops around
// it are fully unrolled, so the shifts are renames).  An output row y (newest input row y + 3) is then
// three v_dot2 with two useful taps each, (k0, k1) . P(y - 2) + (k2, k3) . P(y) + (k4, k5) . P(y + 2),
// and one (0, k6) . P(y + 3): 16 v_dot2 per quad instead of 28 single-tap ones, for 4 v_lshl_or per
// input row.  Bit-exact ufixedpoint16 rounding: out = (acc + 2^15) >> 16, which never exceeds 255
// (acc <= 256 * 65280), so it is byte 2 of acc + 2^15 and the four bytes are gathered by two v_perm.
struct BlurCol {
    uint32_t hp[4] = {0u, 0u, 0u, 0u};   // the newest row's sums
    uint32_t P[6][4];                    // P[5]: the pair ending at the newest row
    __device__ __forceinline__ void push(uint32_t d0, uint32_t d1, uint32_t d2)
    {
        uint32_t h[4];
        blur_h4(d0, d1, d2, h);
#pragma unroll
        for (int k = 0; k < 5; k++)
#pragma unroll
            for (int j = 0; j < 4; j++) P[k][j] = P[k + 1][j];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            P[5][j] = hp[j] | (h[j] << 16);
            hp[j] = h[j];
        }
    }
    __device__ __forceinline__ uint32_t out() const   // the output row three rows above the newest
    {
        const u16x2 k01 = __builtin_bit_cast(u16x2, 18u | (34u << 16)), k23 = __builtin_bit_cast(u16x2, 49u | (54u << 16));
        const u16x2 k45 = __builtin_bit_cast(u16x2, 49u | (34u << 16)), k6 = __builtin_bit_cast(u16x2, 18u << 16);
        uint32_t acc[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t a = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, P[0][j]), k01, 1u << 15, false);
            a = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, P[2][j]), k23, a, false);
            a = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, P[4][j]), k45, a, false);
            acc[j] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, P[5][j]), k6, a, false);
        }
        return __builtin_amdgcn_perm(acc[1], acc[0], 0x0c0c0602u) | __builtin_amdgcn_perm(acc[3], acc[2], 0x06020c0cu);
    }
};


// Edge-quad window: the aligned 16-byte window A .. A + 15 of a row that holds the 12 bytes columns
// x - 4 .. x + 7 (REFLECT_101) of quad x need: A = 0 at the left edge, (w - 12) & ~3 at the right edge;
// source dword j is one v_perm of window dwords (p[j], p[j] + 1) with selector sel[j].
__device__ __forceinline__ int blur_edge_window(int x, int w, int* p, uint32_t* sel)
{
    const int A = x == 0 ? 0 : ((w - 12) & ~3);
#pragma unroll
    for (int j = 0; j < 3; j++) {
        int o[4], mn = 16;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            o[i] = reflect101(x - 4 + 4 * j + i, w) - A;
            mn = min(mn, o[i]);
        }
        p[j] = min(mn >> 2, 2);   // the (<= 4-byte) span lies in window dwords p, p + 1
        sel[j] = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) sel[j] |= (uint32_t)(o[i] - 4 * p[j]) << (8 * i);
    }
    return A;
}

// ------------------------------------------------------------------ fused level blur (k_pyramid)
// GaussianBlur 7x7 (:745-746) of one level's strip while it is LDS-resident in k_pyramid (rows
// [r0, r1) of the level, the strip's own rows +- 3 and every REFLECT_101 row they reach): item =
// (segment of kPbRows own rows, column quad); the item walks its rows + 6 with a 7-row register window
// of horizontal sums as row pairs (three LDS dwords and BlurCol::push per input row, BlurCol::out per output row).  Items
// are dealt from the last thread down, so the threads the level's resize leaves idle take them first;
// inner quads first, edge quads (REFLECT_101 columns) after them, so only one wave runs the v_perm path.
template <bool kEdge, bool kLin>
__device__ __forceinline__ void pb_walk(const uint8_t* lv, int r0, int r1, uint8_t* __restrict__ out, const LevelCfg& L,
                                        int x, int ya, int yb)
{
    int p[3] = {0, 1, 2};
    uint32_t sel[3] = {0x03020100u, 0x03020100u, 0x03020100u};
    const int A = kEdge ? blur_edge_window(x, L.w, p, sel) : x - 4;
    const uint8_t* base = lv + A;
    const int h = L.h, nr = r1 - r0;
    BlurCol col;
#pragma unroll
    for (int i = 0; i < kPbRows + 6; i++) {
        int ro;
        if (kLin) {   // every input row inside the strip and the level: consecutive LDS rows
            ro = (ya - 3 - r0) * L.stride + i * L.stride;
        } else {
            int yi = ya - 3 + i;
            yi = yi < 0 ? -yi : (yi >= h ? 2 * h - 2 - yi : yi);
            yi = min(max(yi - r0, 0), nr - 1);   // rows past the segment's end feed outputs never stored
            ro = __mul24(yi, L.stride);
        }
        const uint32_t* rp = reinterpret_cast<const uint32_t*>(base + ro);
        uint32_t d[3];
        if (kEdge) {
            const uint32_t r[4] = {rp[0], rp[1], rp[2], rp[3]};
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const uint32_t lo = p[j] == 0 ? r[0] : (p[j] == 1 ? r[1] : r[2]);
                const uint32_t hi = p[j] == 0 ? r[1] : (p[j] == 1 ? r[2] : r[3]);
                d[j] = __builtin_amdgcn_perm(hi, lo, sel[j]);
            }
        } else {
            d[0] = rp[0];
            d[1] = rp[1];
            d[2] = rp[2];
        }
        col.push(d[0], d[1], d[2]);
        const int y = ya + i - 6;
        if (i >= 6 && y < yb)   // bytes of a last quad past w land in the row padding
            *reinterpret_cast<uint32_t*>(out + ((uint32_t)y * (uint32_t)L.stride + (uint32_t)x)) = col.out();
    }
}

__device__ __forceinline__ void pyr_blur(const uint8_t* lv, const LevelCfg& L, int r0, int r1, uint8_t* __restrict__ out,
                                         int o0, int o1, int nseg, int qin, int qex, int tid)
{
    const int nin = nseg * qin, ntot = nin + nseg * qex;
    for (int i = kPyrThreads - 1 - tid; i < ntot; i += kPyrThreads) {
        const bool edge = i >= nin;
        const int j = edge ? i - nin : i, Q = edge ? qex : qin;
        const int seg = (int)((unsigned)j / (unsigned)Q), qi = j - seg * Q;
        const int ya = o0 + seg * kPbRows;
        if (ya >= o1) continue;
        const int yb = min(ya + kPbRows, o1);
        const bool lin = ya - 3 >= max(r0, 0) && ya + kPbRows + 3 <= min(r1, L.h);
        if (!edge) {
            if (lin) pb_walk<false, true>(lv, r0, r1, out, L, 4 * (qi + 1), ya, yb);
            else pb_walk<false, false>(lv, r0, r1, out, L, 4 * (qi + 1), ya, yb);
        } else {   // x = 0, then the quads from the first with x + 8 > w
            pb_walk<true, false>(lv, r0, r1, out, L, qi == 0 ? 0 : 4 * (qin + qi), ya, yb);
        }
    }
}

// One 4-px column quad of a resized row (cv::resize INTER_LINEAR, level l from l - 1) from the 12-byte
// tap windows a (source row sy0) and c (sy1) at the quad's window base wb: the quad's host table QuadX
// holds the window's byte shift, per-pixel v_perm selectors into it and packed x16 weights.
struct QuadTaps {
    int wb;
    uint32_t wsh, sel[4], wt[4], simd;
    __device__ __forceinline__ explicit QuadTaps(const QuadX* qp_)
    {
        const uint4* qp = reinterpret_cast<const uint4*>(qp_);
        const uint4 qa = qp[0], qb = qp[1], qc = qp[2];
        wb = (int)(qa.x & 0xFFFFu);
        wsh = qa.x >> 16;   // byte shift of the quad's 8-byte tap window
        sel[0] = qa.y; sel[1] = qa.z; sel[2] = qa.w; sel[3] = qb.x;
        wt[0] = qb.y; wt[1] = qb.z; wt[2] = qb.w; wt[3] = qc.x;
        simd = qc.y;
    }
    // kAll: every pixel of the quad in the SSE2 vertical range (the quads before the row's last rs_simd / 4),
    // no branch; else the per-pixel choice (only the few quads at a row's end take it)
    template <bool kAll = false>
    __device__ __forceinline__ uint32_t resize(const uint32_t a[3], const uint32_t c[3], const ResizeY& ry) const
    {
        uint32_t rr0[4], rr1[4];   // 16 x the horizontal sums
        const uint32_t wa0 = __builtin_amdgcn_alignbyte(a[1], a[0], wsh), wa1 = __builtin_amdgcn_alignbyte(a[2], a[1], wsh);
        const uint32_t wc0 = __builtin_amdgcn_alignbyte(c[1], c[0], wsh), wc1 = __builtin_amdgcn_alignbyte(c[2], c[1], wsh);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t t0 = __builtin_amdgcn_perm(wa1, wa0, sel[i]);
            const uint32_t t1 = __builtin_amdgcn_perm(wc1, wc0, sel[i]);
            rr0[i] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, t0), __builtin_bit_cast(u16x2, wt[i]), 0u, false);
            rr1[i] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, t1), __builtin_bit_cast(u16x2, wt[i]), 0u, false);
        }
        // SSE2 VResizeLinearVec_32s8u: ((r >> 4) b >> 16) per row as one 24-bit mul-hi of (r >> 4) << 8
        // (= 16 r with the low byte cleared) and b << 8; the uchar saturation never engages
        const uint32_t b0s = (uint32_t)(uint16_t)ry.b0 << 8, b1s = (uint32_t)(uint16_t)ry.b1 << 8;
        auto vs = [&](int i) -> uint32_t {
            const uint32_t m0 = (uint32_t)(((unsigned long long)(rr0[i] & 0xFFFF00u) * b0s) >> 32);
            const uint32_t m1 = (uint32_t)(((unsigned long long)(rr1[i] & 0xFFFF00u) * b1s) >> 32);
            return (m0 + m1 + 2u) >> 2;
        };
        if (kAll || simd == 0xFu)   // every pixel of the quad in the SSE2 vertical range
            return vs(0) | (vs(1) << 8) | (vs(2) << 16) | (vs(3) << 24);
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < 4; i++)
            v |= ((simd >> i) & 1u ? vs(i) : (uint32_t)resize_vt((int)(rr0[i] >> 4), (int)(rr1[i] >> 4), ry)) << (8 * i);
        return v;
    }
};

// The pyramid's large levels (1 .. pyr_top-1; k_pyr_tail the rest) in one launch: one workgroup per (strip, frame).  The strip's
// level-0 rows are staged in LDS with 16-B loads; each level is computed from the previous level's
// LDS strip into LDS (for the next level) and HBM (for FAST / describe).  Strips overlap by the
// halo rows the next level reads; overlapping rows are computed identically by both strips.
#ifdef RGBD_PNP_PROFILE
extern __device__ long long g_pyr_prof[8][16];
extern __device__ long long g_pyr_span[2048][2];
#define PYR_PROF(k) do { if (threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < 8) g_pyr_prof[blockIdx.x][(k)] = wall_clock64(); } while (0)
#else
#define PYR_PROF(k) do { } while (0)
#endif
__global__ __launch_bounds__(kPyrThreads) void k_pyramid(uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                                         const uint8_t* __restrict__ bgr, const ResizeY* __restrict__ rsy,
                                                         const QuadX* __restrict__ qxt, const ExtractCfg* __restrict__ cfgp)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t lbuf[];
    const ExtractCfg& cfg = *cfgp;
    const int st = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    uint8_t* frame = pyr + (size_t)b * cfg.frame_pyr_bytes;
    PYR_PROF(0);
#ifdef RGBD_PNP_PROFILE
    const int span_id = b * gridDim.x + st;
    if (tid == 0 && span_id < 2048) g_pyr_span[span_id][0] = wall_clock64();
#endif
    // stage level-0 rows: cvtColor BGR2GRAY (Core/Frame.cpp:47) fused here, 16 px per task, the
    // strip's own rows also written to HBM; or a gray level 0 already in HBM (bgr == nullptr)
    {
        const LevelCfg& L0 = cfg.lv[0];
        const int r0 = cfg.strip_r0[st][0], r1 = cfg.strip_r1[st][0];
        if (bgr) {
            const int own0 = (int)((long)L0.h * st / kPyrStrips), own1 = (int)((long)L0.h * (st + 1) / kPyrStrips);
            // task (row rr, 16-px group g): thread tid takes group tg of rows tr, tr + RPS, ... (one division
            // per thread, not per task; 32-bit offsets from the frame's base: a frame is < 4 GiB)
            const int G = cfg.W >> 4;
            const int RPS = kPyrThreads / G;   // rows per pass
            const int tr = tid / G, tg = tid - tr * G;
            const uint8_t* fb = bgr + (size_t)b * cfg.W * cfg.H * 3;
            const int nrows = r1 - r0;
            const uint32_t srow = (uint32_t)cfg.W * 3u;
            auto put = [&](int rr, uint4 o) {
                const int y = r0 + rr;
                *reinterpret_cast<uint4*>(lbuf + (uint32_t)rr * (uint32_t)L0.stride + 16u * (uint32_t)tg) = o;
                if (y >= own0 && y < own1)
                    *reinterpret_cast<uint4*>(frame + ((uint32_t)L0.off + (uint32_t)y * (uint32_t)L0.stride + 16u * (uint32_t)tg)) = o;
            };
            if (tr < RPS) {
                // every task's loads first (one HBM round trip), then the conversions
                constexpr int kStage = 4;
                uint4 v[kStage][3];
#pragma unroll
                for (int u = 0; u < kStage; u++) {
                    const int rr = tr + u * RPS;
                    if (rr < nrows) {
                        const uint4* src = reinterpret_cast<const uint4*>(fb + ((uint32_t)(r0 + rr) * srow + 48u * (uint32_t)tg));
                        v[u][0] = src[0];
                        v[u][1] = src[1];
                        v[u][2] = src[2];
                    }
                }
#pragma unroll
                for (int u = 0; u < kStage; u++) {
                    const int rr = tr + u * RPS;
                    if (rr < nrows) put(rr, gray16(v[u][0], v[u][1], v[u][2]));
                }
                for (int rr = tr + kStage * RPS; rr < nrows; rr += RPS) {   // taller strips
                    const uint4* src = reinterpret_cast<const uint4*>(fb + ((uint32_t)(r0 + rr) * srow + 48u * (uint32_t)tg));
                    put(rr, gray16(src[0], src[1], src[2]));
                }
            }
        } else {
            const uint4* src = reinterpret_cast<const uint4*>(frame + L0.off + (size_t)r0 * L0.stride);
            uint4* dst = reinterpret_cast<uint4*>(lbuf);
            const int n16 = (r1 - r0) * L0.stride / 16;
            for (int i = tid; i < n16; i += kPyrThreads) dst[i] = src[i];
        }
    }
    // the strip's resize row entries (cv::resize yofs / ibeta of every computed row of levels 1..L-1) in LDS
    // after the level buffers: one ds_read_b64 per output row instead of the float row arithmetic
    ResizeY* rsl = reinterpret_cast<ResizeY*>(lbuf + cfg.pyr_lds);
    {
        int cum = 0;
        for (int l = 1; l < cfg.pyr_top; l++) {
            const int r0 = cfg.strip_r0[st][l], n = cfg.strip_r1[st][l] - r0;
            for (int i = tid; i < n; i += kPyrThreads) rsl[cum + i] = rsy[cfg.lv[l].rsy_off + r0 + i];
            cum += n;
        }
    }
    __syncthreads();
    PYR_PROF(1);
    uint8_t* prev = lbuf;
    int rs_cum = 0;   // level l's first entry in rsl
    for (int l = 1; l < cfg.pyr_top; l++) {
        const LevelCfg& S = cfg.lv[l - 1];
        const LevelCfg& D = cfg.lv[l];
        const int pr0 = cfg.strip_r0[st][l - 1];
        const int r0 = cfg.strip_r0[st][l], r1 = cfg.strip_r1[st][l];
        uint8_t* cur = (l & 1) ? lbuf + cfg.pyr_lds_b : lbuf;
        // all-SSE2 quads q < Qi (no per-pixel branch): thread = (quad q, row phase ph), the quad's taps loaded
        // once and reused down the strip's rows ph, ph + RP, ... (quads q0 + k * kPyrThreads when a row has
        // more quads than threads); then the row-end quads (at most 2 per row: the SSE2 loop leaves at most 4 px,
        // LevelCfg::rs_simd) as items (quad, row), so no wave of the main pass runs both paths
        const int own0 = (int)((long)D.h * st / kPyrStrips), own1 = (int)((long)D.h * (st + 1) / kPyrStrips);
        const int Q = (D.w + 3) >> 2, Qi = min(max(D.rs_simd, 0) >> 2, Q);
        auto quad_row = [&](const QuadTaps& tq, int q, int y, auto kall) {
            const ResizeY ry = rsl[rs_cum + y - r0];
            const uint32_t* s0 = reinterpret_cast<const uint32_t*>(prev + __mul24(ry.sy0 - pr0, S.stride) + tq.wb);
            const uint32_t* s1 = reinterpret_cast<const uint32_t*>(prev + __mul24(ry.sy1 - pr0, S.stride) + tq.wb);
            const uint32_t a[3] = {s0[0], s0[1], s0[2]};
            const uint32_t c[3] = {s1[0], s1[1], s1[2]};
            const uint32_t v = tq.template resize<decltype(kall)::value>(a, c, ry);
            if (y >= own0 && y < own1)   // halo rows are another strip's own rows (24-bit products: y, stride < 2^14)
                *reinterpret_cast<uint32_t*>(frame + (uint32_t)(D.off + __mul24(y, D.stride) + 4 * q)) = v;
            *reinterpret_cast<uint32_t*>(cur + __mul24(y - r0, D.stride) + 4 * q) = v;
        };
        if (Qi > 0) {
            const int RP = kPyrThreads / Qi > 0 ? kPyrThreads / Qi : 1;
            const int ph = tid / Qi, q0 = tid - ph * Qi;
            for (int q = ph < RP ? q0 : Qi; q < Qi; q += kPyrThreads) {
                const QuadTaps tq(qxt + D.qx_off + q);
                for (int y = r0 + ph; y < r1; y += RP) quad_row(tq, q, y, std::true_type{});
            }
        }
        {
            const int Qe = Q - Qi, n = Qe * (r1 - r0);
            for (int e = tid; e < n; e += kPyrThreads) {
                const int yy = e / Qe, q = Qi + (e - yy * Qe);
                quad_row(QuadTaps(qxt + D.qx_off + q), q, r0 + yy, std::false_type{});
            }
        }
        // the level blur of level l - 1 from its LDS strip (read-only in this phase)
        if (cfg.pb_seg[l - 1] > 0)
            pyr_blur(prev, S, cfg.strip_r0[st][l - 1], cfg.strip_r1[st][l - 1], blur + (size_t)b * cfg.frame_pyr_bytes + S.off,
                     cfg.pb_r0[st][l - 1], cfg.pb_r1[st][l - 1], cfg.pb_seg[l - 1], cfg.blur_tx[l - 1], cfg.blur_ex[l - 1], tid);
        __syncthreads();
        PYR_PROF(1 + l);
        prev = cur;
        rs_cum += r1 - r0;
    }
    {
        const int l = cfg.pyr_top - 1;
        if (cfg.pb_seg[l] > 0)
            pyr_blur(prev, cfg.lv[l], cfg.strip_r0[st][l], cfg.strip_r1[st][l], blur + (size_t)b * cfg.frame_pyr_bytes + cfg.lv[l].off,
                     cfg.pb_r0[st][l], cfg.pb_r1[st][l], cfg.pb_seg[l], cfg.blur_tx[l], cfg.blur_ex[l], tid);
    }
#ifdef RGBD_PNP_PROFILE
    if (tid == 0 && span_id < 2048) g_pyr_span[span_id][1] = wall_clock64();
#endif
}

// k_pyr_tail: rows per batch of a thread's tap-window loads
#ifndef RGBD_PYR_LEVEL_ROWS
#define RGBD_PYR_LEVEL_ROWS 8
#endif
constexpr int kPyrLevelRows = RGBD_PYR_LEVEL_ROWS;

// The levels after the strips (pyr_top .. L-1), one frame per workgroup: each level from the previous
// one as this workgroup wrote it to HBM (only the strips' last level, pyr_top - 1, was written by other
// workgroups, in the previous launch), a barrier between levels (the waves of a workgroup share one CU's
// write-through L1, so its workgroup-scope release / acquire makes the stores visible).  Inside the strips
// these levels were latency-bound passes of a few rows each, and the halo rows they read cascaded down
// every lower level's strip (k_pyramid 1.14 -> 0.84 ms, this launch ~0.2 ms; profiles/r06_ab/ab27).
// Thread = (column quad q, row phase ph), the quad's taps (QuadTaps, the strips' arithmetic) loaded once
// per level and kPyrLevelRows rows' tap windows loaded before their stores (the stores may alias the
// loads for the compiler, which would otherwise serialize one memory round trip per row).  The 12-byte
// tap window of a row's last quad may run past the row into the next one (or the next level's first
// row): bytes never selected.  An LDS ping-pong version (levels kept in LDS, 1024 threads) measured the
// same (profiles/r06_ab/ab24, ab27).
__global__ __launch_bounds__(kPyrTailThreads) void k_pyr_tail(uint8_t* __restrict__ pyr, const ResizeY* __restrict__ rsy,
                                                              const QuadX* __restrict__ qxt, const ExtractCfg* __restrict__ cfgp)
{
    const ExtractCfg& cfg = *cfgp;
    const int tid = threadIdx.x;
    uint8_t* frame = pyr + (size_t)blockIdx.x * cfg.frame_pyr_bytes;
    for (int l = cfg.pyr_top; l < cfg.nlevels; l++) {
        // the level constants in registers (the stores below may alias cfg for the compiler, which would
        // reload them after every store); 32-bit offsets from the frame's uniform base with 24-bit products
        // (rows and strides < 2^14), so loads and stores take the scalar-base + vector-offset form
        const int sstride = cfg.lv[l - 1].stride, soff = cfg.lv[l - 1].off;
        const int dstride = cfg.lv[l].stride, doff = cfg.lv[l].off, dh = cfg.lv[l].h, rsy0 = cfg.lv[l].rsy_off;
        const int qxo = cfg.lv[l].qx_off;
        const int Q = (cfg.lv[l].w + 3) >> 2, Qi = min(max(cfg.lv[l].rs_simd, 0) >> 2, Q);   // all-SSE2 quads first, as in k_pyramid
        if (Qi > 0) {
            const int RP = kPyrTailThreads / Qi > 0 ? kPyrTailThreads / Qi : 1;
            const int ph = tid / Qi, q0 = tid - ph * Qi;
            // thread = quad q0 + k * kPyrTailThreads of row phase 0 when a row has more quads than threads
            for (int q = ph < RP ? q0 : Qi; q < Qi; q += kPyrTailThreads) {
                const QuadTaps tq(qxt + qxo + q);
                const int sb = soff + tq.wb, db = doff + 4 * q;
                for (int y0 = ph; y0 < dh; y0 += kPyrLevelRows * RP) {
                    ResizeY ry[kPyrLevelRows];
                    uint32_t a[kPyrLevelRows][3], c[kPyrLevelRows][3];
#pragma unroll
                    for (int k = 0; k < kPyrLevelRows; k++) {
                        ry[k] = rsy[rsy0 + min(y0 + k * RP, dh - 1)];
                        const uint32_t* s0 = reinterpret_cast<const uint32_t*>(frame + (uint32_t)(sb + __mul24(ry[k].sy0, sstride)));
                        const uint32_t* s1 = reinterpret_cast<const uint32_t*>(frame + (uint32_t)(sb + __mul24(ry[k].sy1, sstride)));
#pragma unroll
                        for (int j = 0; j < 3; j++) {
                            a[k][j] = s0[j];
                            c[k][j] = s1[j];
                        }
                    }
#pragma unroll
                    for (int k = 0; k < kPyrLevelRows; k++) {
                        const int y = y0 + k * RP;
                        if (y < dh)
                            *reinterpret_cast<uint32_t*>(frame + (uint32_t)(db + __mul24(y, dstride))) = tq.resize<true>(a[k], c[k], ry[k]);
                    }
                }
            }
        }
        const int Qe = Q - Qi, n = Qe * dh;   // the row-end quads: items (quad, row)
        for (int e = tid; e < n; e += kPyrTailThreads) {
            const int y = e / Qe, q = Qi + (e - y * Qe);
            const QuadTaps tq(qxt + qxo + q);
            const ResizeY ry = rsy[rsy0 + y];
            const uint32_t* s0 = reinterpret_cast<const uint32_t*>(frame + (uint32_t)(soff + tq.wb + __mul24(ry.sy0, sstride)));
            const uint32_t* s1 = reinterpret_cast<const uint32_t*>(frame + (uint32_t)(soff + tq.wb + __mul24(ry.sy1, sstride)));
            const uint32_t a[3] = {s0[0], s0[1], s0[2]};
            const uint32_t c[3] = {s1[0], s1[1], s1[2]};
            *reinterpret_cast<uint32_t*>(frame + (uint32_t)(doff + __mul24(y, dstride) + 4 * q)) = tq.resize(a, c, ry);
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ FAST (:613-672)
// m(p) = max over the 16 contiguous 9-arcs of the ring of min(v - x) (darker) or min(x - v)
// (brighter).  FAST_t<16> marks p a corner at threshold t iff m > t, and cornerScore<16>
// returns m - 1 for every such corner, so one m map serves both thresholds (20 and 7).
//
// m for two horizontally adjacent pixels at once, the ring as packed f16 whose bits are the pixel bytes x
// (the subnormals x * 2^-24: equally spaced, so ordered like x, and differences of two are exact; the
// f16 subnormals are kept by the kernel's default FP mode), so the network can use gfx950's 3-input
// v_pk_maximum3_f16 / v_pk_minimum3_f16:
// measured on MI355X (tools/ubench/valu_rate.hip) they issue at the rate of the 2-input
// v_pk_max_u16 (~4.3 vs 4.5 cycles per wave64 instruction per SIMD) while doing two operations, so
// the arc network takes 75 instructions per pixel pair (a packed-u16 form takes 99).
// Only the smallest arc maximum MM and the largest arc minimum mm are needed (v - max_A x is the
// darker side of arc A, min_A x - v the brighter); arcs k..k+8 and k+1..k+9 (k even) share the core
// k+1..k+8, so the pair contributes max(core max, min(x_k, x_k+9)) to MM (and dually to mm).  Returns the scores m as
// packed u16 integers 0 .. 255 (the bits of the non-negative subnormal results; the NMS below
// compares them as u16 or as f16, which order alike).  No input is NaN, so IEEE maximum / minimum = max / min.
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h16x2 hmax(h16x2 a, h16x2 b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ h16x2 hmin(h16x2 a, h16x2 b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ h16x2 hmax3(h16x2 a, h16x2 b, h16x2 c) { return hmax(hmax(a, b), c); }
__device__ __forceinline__ h16x2 hmin3(h16x2 a, h16x2 b, h16x2 c) { return hmin(hmin(a, b), c); }
__device__ __forceinline__ uint32_t fast_m2h(const uint32_t (&raw)[16], uint32_t vr)
{
    const h16x2 v = __builtin_bit_cast(h16x2, vr);
    h16x2 x[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = __builtin_bit_cast(h16x2, raw[k]);
    h16x2 mx2[16], mn2[16], mx4[16], mn4[16];
#pragma unroll
    for (int j = 1; j < 16; j += 2) {
        mx2[j] = hmax(x[j], x[(j + 1) & 15]);
        mn2[j] = hmin(x[j], x[(j + 1) & 15]);
    }
#pragma unroll
    for (int j = 1; j < 16; j += 2) {
        mx4[j] = hmax(mx2[j], mx2[(j + 2) & 15]);
        mn4[j] = hmin(mn2[j], mn2[(j + 2) & 15]);
    }
    // arcs k..k+8 and k+1..k+9 (k even): max(core max, min(x_k, x_k+9)) in one 3-input op
    h16x2 cM[8], cm[8];
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
        cM[k >> 1] = hmax3(mx4[k + 1], mx4[(k + 5) & 15], hmin(x[k], x[(k + 9) & 15]));
        cm[k >> 1] = hmin3(mn4[k + 1], mn4[(k + 5) & 15], hmax(x[k], x[(k + 9) & 15]));
    }
    const h16x2 MM = hmin(hmin3(cM[0], cM[1], cM[2]), hmin3(cM[3], cM[4], hmin3(cM[5], cM[6], cM[7])));
    const h16x2 mm = hmax(hmax3(cm[0], cm[1], cm[2]), hmax3(cm[3], cm[4], hmax3(cm[5], cm[6], cm[7])));
    const h16x2 zero = {(_Float16)0.0f, (_Float16)0.0f};
    return __builtin_bit_cast(uint32_t, hmax3(v - MM, mm - v, zero));
}

struct FastLg4 { static constexpr bool v = true; };
struct FastLgN { static constexpr bool v = false; };
#define FAST_IS4(L4) (decltype(L4)::v)

#ifdef RGBD_PNP_PROFILE
__device__ long long g_fast_prof[1024][4];   // frame 0, segments 0..1023: stage timestamps of lane 0
#define FAST_PROF(k) do { if (threadIdx.x == 0 && b == 0 && si < 1024) g_fast_prof[si][(k)] = clock64(); } while (0)
#else
#define FAST_PROF(k) do { } while (0)
#endif

// The 7 pixel pairs (x[sh + k], x[sh + k + 1]), k = 0..6, of the 12 bytes d0 | d1 << 32 | d2 << 64 as
// packed u16 (= the f16 subnormal ring of fast_m2h): one v_perm each, with the lane's byte shift sh in
// its selectors (sel[k] = sh + k | 0x0c << 8 | sh + k + 1 << 16 | 0x0c << 24; selector byte 0x0c reads
// 0x00).  Pairs 0..3 lie in d0 | d1 (bytes <= 3 + 3 + 1), pairs 4..6 in d1 | d2 with the same selectors.
__device__ __forceinline__ void row_pairs(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t sh, uint32_t* w)
{
    const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sh), hi = __builtin_amdgcn_alignbyte(d2, d1, sh);
    w[0] = __builtin_amdgcn_perm(hi, lo, 0x0c010c00u);
    w[1] = __builtin_amdgcn_perm(hi, lo, 0x0c020c01u);
    w[2] = __builtin_amdgcn_perm(hi, lo, 0x0c030c02u);
    w[3] = __builtin_amdgcn_perm(hi, lo, 0x0c040c03u);
    w[4] = __builtin_amdgcn_perm(hi, lo, 0x0c050c04u);
    w[5] = __builtin_amdgcn_perm(hi, lo, 0x0c060c05u);
    w[6] = __builtin_amdgcn_perm(hi, lo, 0x0c070c06u);
}

// One wave per segment: up to 64 / lpc consecutive cells of one cell row of one level (FastSeg).  The
// segment's ROI rows are staged in LDS with 16-B loads (all in flight at once), then lane (cell k,
// pair p) owns the pixel pair at ROI columns 3 + 2p, 4 + 2p of cell k and walks the cell's interior
// rows top to bottom with the 7 rows x 7 pairs its ring needs in registers (the next row read one step
// ahead).  Per row: m of both pixels (fast_m2), the row's horizontal maxima from the neighbour lanes
// (DPP row shifts: a 16-lane cell is one DPP row), and the NMS of the previous row: keep iff
// m > max(t, 1, every neighbour's M) (OpenCV's NMS with the neighbour score n > t ? n - 1 : 0; cells
// never see each other: pixels outside the cell interior score 0).  Survivors are appended to the
// cell's list in raster order by ballot ranks (one running count per cell, no barrier).  A cell with no
// survivor at iniThFAST walks again at minThFAST (:655-661).  Corners are emitted with pt relative to
// the level's (minBorderX, minBorderY), i.e. vToDistributeKeys order.
#define RGBD_FAST_WPE 4   // waves per SIMD: 126 VGPRs for the exit-free 7-row walk blocks (at 5 waves, 96 VGPRs, they spill 48; r05 same-box A/B against 5 waves with per-row exits: +0.6 %, k_fast 1.67 -> 1.65 ms)
constexpr int kFastRowBytes = 160;   // staged segment row: <= 4 x 32 + 6 ROI bytes + 16-B alignment + over-read
__device__ __forceinline__ void blur_thread(const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                            const ExtractCfg& cfg, int b, int t);
// k_fast's emission rank for 16-lane cells (one cell = one DPP row): corners below the lane over the whole
// wave (pre), less those below the row (its lane 0's pre, row_newbcast:0) = the rank in the cell; the cell
// total from its lane 15's inclusive count (row_newbcast:15).  cnt = the cell's next free slot (the same in
// every lane of the row); returns this lane's slot.  The row_newbcast moves stay v_mov_b32_dpp: folded into a
// v_subrev_u32_dpp / v_add_u32_dpp by the compiler they gave wrong ranks on the MI355X, so the empty asm keeps
// the combine from happening.  Pinned on its own by k_debug_rank16 (tests/test_gpu_extract.py).
__device__ __forceinline__ uint32_t fast_rank16(bool f, uint32_t& cnt)
{
    const unsigned long long bf = __ballot(f);
    const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bf >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bf, 0u));
    int base = __builtin_amdgcn_update_dpp(0, pre, 0x150, 0xf, 0xf, true);
    int tot = __builtin_amdgcn_update_dpp(0, pre + (f ? 1 : 0), 0x15f, 0xf, 0xf, true);
    asm volatile("" : "+v"(base), "+v"(tot));
    const uint32_t c2 = cnt - (uint32_t)base;
    const uint32_t slot = c2 + (uint32_t)pre;
    cnt = c2 + (uint32_t)tot;
    return slot;
}

// one wave: rows x 64 lane flags -> every lane's slot per row (0xffffffff where its flag is clear) and each
// lane's final count, each 16-lane row starting from slot 1000 * row (a cell's base, as k_fast's slot0)
__global__ __launch_bounds__(64) void k_debug_rank16(const uint8_t* __restrict__ flags, int rows,
                                                     uint32_t* __restrict__ slots, uint32_t* __restrict__ counts)
{
    const int lane = (int)threadIdx.x;
    uint32_t cnt = 1000u * (uint32_t)(lane >> 4);
    for (int r = 0; r < rows; r++) {
        const bool f = flags[r * 64 + lane] != 0;
        const uint32_t slot = fast_rank16(f, cnt);
        slots[r * 64 + lane] = f ? slot : 0xffffffffu;
    }
    counts[lane] = cnt;
}

hipError_t launch_debug_rank16(const uint8_t* flags, int rows, uint32_t* slots, uint32_t* counts, hipStream_t st)
{
    return dispatch(k_debug_rank16, dim3(1), dim3(64), 0, st, flags, rows, slots, counts);
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RGBD_FAST_WPE, 8))) void k_fast(const uint8_t* __restrict__ pyr, const Cell* __restrict__ cells,
                                             const FastSeg* __restrict__ segs, const ExtractCfg* __restrict__ cfgp,
                                             int nseg, int* __restrict__ cell_count, uint32_t* __restrict__ cell_slots,
                                             int xcd_map, uint8_t* __restrict__ blur, int nbb)
{
    const ExtractCfg& cfg = *cfgp;
    __shared__ __attribute__((aligned(16))) uint32_t roi[(kCellStride + 1) * kFastRowBytes / 4];   // + the walk's read-ahead row
    // xcd_map (1-D grid, B a multiple of 8): all blocks of frame b run on XCD b % 8, in order, so the rows
    // shared by neighbouring segments are fetched once into that XCD's L2.
    // nbb > 0: each frame's block sequence also holds the level blur's nbb 64-lane blocks (blur_thread,
    // levels RGBD_PB_LEVELS.. = 1-7) ahead of its segments, so blur and FAST waves share the CUs inside one launch instead
    // of the blur competing from another stream with the quadtree
    const int n = nseg + nbb;
    int i = blockIdx.x, b = blockIdx.y;
    if (xcd_map) {
        const int j = blockIdx.x >> 3;
        b = (j / n) * 8 + (blockIdx.x & 7);
        i = j % n;
    }
    int si = i;
    if (nbb > 0) {
        if (i < nbb) {
            blur_thread(pyr, blur, cfg, b, i * 64 + (int)threadIdx.x);
            return;
        }
        si = i - nbb;
    }
    const int lane = threadIdx.x;
    FAST_PROF(0);
    const FastSeg S = segs[si];
    const int LPC = S.lpc;   // wave-uniform
    const int k = (lane >= LPC ? 1 : 0) + (lane >= 2 * LPC ? 1 : 0) + (lane >= 3 * LPC ? 1 : 0), p = lane - k * LPC;
    const bool cell_on = k < S.ncell;
    const int ci = S.cell0 + (cell_on ? k : 0);
    const Cell c = cells[ci];
    const Cell c0 = cells[S.cell0], cl = cells[S.cell0 + S.ncell - 1];
    const LevelCfg& L = cfg.lv[c.level];
    // ch is the same for every cell of the segment: wave-uniform, so the row loop's bound tests are scalar
    const int cw = c.x1 - c.x0, ch = __builtin_amdgcn_readfirstlane(c.y1 - c.y0);
    const int a = cw - 6;
    const int np = (a + 1) >> 1;
    const bool act = cell_on && p < np;              // pixel A evaluated
    const bool actB = act && 2 * p + 1 < a;          // pixel B evaluated (the second pixel of an odd end is not)
    // ---- stage ROI rows [0, ch), columns [xs, xs + 16 q) of the segment (xs 16-B aligned: rows are 64-B
    //      padded and level bases 256-B aligned)
    {
        const int xs = c0.x0 & ~15;
        const int q = (cl.x1 + 6 - xs + 15) >> 4;    // 16-B chunks per row (the walk reads up to x1 + 6)
        const uint8_t* src = pyr + (size_t)b * cfg.frame_pyr_bytes + L.off + (size_t)c0.y0 * L.stride + xs;
        // chunk (row r, 16-B column j) of lane, lane + 64, ...: one division per lane, then (r, j) stepped by
        // the wave-uniform (64 / q, 64 % q)
        const int dr = 64 / q, dj = 64 - dr * q;
        int r = lane / q, j = lane - r * q;
        for (; r < ch; r += dr, j += dj) {
            if (j >= q) {
                j -= q;
                r++;
                if (r >= ch) break;
            }
            const uint4 v = *reinterpret_cast<const uint4*>(src + (uint32_t)(r * L.stride + 16 * j));
            *reinterpret_cast<uint4*>(&roi[r * (kFastRowBytes / 4) + 4 * j]) = v;
        }
    }
    __syncthreads();
    FAST_PROF(1);
    const int off = c.x0 + (act ? 2 * p : 0) - (c0.x0 & ~15);   // byte column of this lane's 8 bytes
    const uint32_t sh = (uint32_t)off & 3u;
    const uint32_t* rp = roi + (off >> 2);
    auto rd3 = [&](int y, uint32_t& d0, uint32_t& d1, uint32_t& d2) {
        const uint32_t* q = rp + y * (kFastRowBytes / 4);
        d0 = q[0];
        d1 = q[1];
        d2 = q[2];
    };
    auto build = [&](uint32_t d0, uint32_t d1, uint32_t d2, uint32_t* w) { row_pairs(d0, d1, d2, sh, w); };
    const size_t slot0 = ((size_t)b * cfg.n_cells + ci) * cfg.cell_cap;
    const int x_base = c.x0 + 3 + 2 * p - L.minBX, y_base = c.y0 - L.minBY;
    const bool mask_l = p == 0, mask_r = p == LPC - 1;
    // lanes of the cell (32-lane cells): rebuilt at each use from the lane id, so no 64-bit mask stays live
    // through the walk (the 16-lane walk, which sets the kernel's VGPR budget, does not use it)
    auto cell_mask = [&]() -> unsigned long long {
        int kk = k;
        asm volatile("" : "+v"(kk));
        return (LPC == 64 ? ~0ull : ((1ull << LPC) - 1ull)) << (kk * LPC & 63);
    };
    const uint32_t maskM = (act ? 0xffffu : 0u) | (actB ? 0xffff0000u : 0u);
    const int rend = ch - 3;
    // the lane's cell list as 32-bit slot indices into cell_slots (the host keeps the slot buffer below
    // 4 GiB), so the stores take the SGPR-base form with a 32-bit byte offset and no 64-bit address stays
    // live.  cnt: the cell's next free slot (the same in every lane of the cell); corners emitted so far =
    // cnt - slot0
    uint8_t* const slots_b = reinterpret_cast<uint8_t*>(cell_slots);
    const uint32_t slot_first = (uint32_t)slot0;
    uint32_t cnt = slot_first;
    // x + 1 | y << 11 of pixel B (pixel A's is one less); the key's -1 << 22 joins the row term (scalar)
    const uint32_t xy0B = (uint32_t)(x_base + 1) | ((uint32_t)y_base << 11);

    // NMS of row r (ROI coordinates) with M = its M row, NB = the max of its 8 neighbours and t' = max(t, 1)
    // (packed): keep iff m > NB.  Pixels A and B of a lane are neighbours, so at most one of them survives
    // (a survivor is a strict maximum over its 8 neighbours): one ballot, one rank and one store per lane.
    // Ballot ranks append to the cell list in raster order.
    auto emit = [&](auto L4, int r, uint32_t Mr, uint32_t NB, bool on) __attribute__((always_inline)) {
        const uint32_t D = __builtin_bit_cast(uint32_t, __builtin_elementwise_sub_sat(__builtin_bit_cast(u16x2, Mr),
                                                                                      __builtin_bit_cast(u16x2, NB)));
        const bool f = on && D != 0u;
        const bool fA = (D & 0xffffu) != 0u;   // the survivor is pixel A (else B)
        uint32_t slot;
        if (FAST_IS4(L4)) {
            // the cell is this lane's 16-lane DPP row: corners below the lane over the whole wave (pre), less
            // those below the row (its lane 0's pre, row_newbcast:0) = the rank in the cell; the cell total
            // from its lane 15's inclusive count (row_newbcast:15)
            slot = fast_rank16(f, cnt);
        } else {
            const unsigned long long bf = __ballot(f) & cell_mask();   // this lane's cell
            slot = cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(bf >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bf, 0u));
            cnt += (uint32_t)__popcll(bf);
        }
        // pack_key(x, y, m - 1) = ((m - 1) << 22) + (x | y << 11): the survivor's m is the low (A) or high (B)
        // half of Mr, shifted left by 22 (m < 256).  No capacity test: NMS survivors are strict maxima over
        // their 8 neighbours, so no two are adjacent, and an independent set of the king graph on an a x b
        // interior holds at most ceil(a/2) ceil(b/2) corners, which is how the host sizes cell_cap (api.cpp)
        const uint32_t ms = fA ? Mr : (Mr >> 16);
        const uint32_t key = (ms << 22) + (xy0B - (fA ? 1u : 0u)) + (((uint32_t)r << 11) - (1u << 22));
        if (f) *reinterpret_cast<uint32_t*>(slots_b + 4u * slot) = key;
    };
    // horizontal neighbour maxima of a packed M row: Hn (neighbours only) and Hf (with the centre and the
    // threshold t', so that the NMS of a row is one 3-input maximum of Hf above, Hn, Hf below).
    // 16 lanes per cell: the neighbour lanes by DPP row shifts (no source at a row end = 0); else bpermute
    auto hrow = [&](auto L4, uint32_t M, uint32_t thr, uint32_t& Hn, uint32_t& Hf) __attribute__((always_inline)) {
        uint32_t Lm, Rm;
        if (FAST_IS4(L4)) {
            Lm = (uint32_t)__builtin_amdgcn_mov_dpp((int)M, 0x111, 0xf, 0xf, true);   // row_shr:1 (row end: 0)
            Rm = (uint32_t)__builtin_amdgcn_mov_dpp((int)M, 0x101, 0xf, 0xf, true);   // row_shl:1
        } else {
            Lm = __shfl_up(M, 1);
            Rm = __shfl_down(M, 1);
            Lm = mask_l ? 0u : Lm;
            Rm = mask_r ? 0u : Rm;
        }
        const u16x2 V1 = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(M, Lm, 0x05040302u));   // (L.B, A)
        const u16x2 V2 = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(Rm, M, 0x05040302u));   // (B, R.A)
        const u16x2 hn = __builtin_elementwise_max(V1, V2);
        Hn = __builtin_bit_cast(uint32_t, hn);
        // non-negative f16 (subnormal) bits order like u16: one v_pk_maximum3_f16
        Hf = __builtin_bit_cast(uint32_t, hmax3(__builtin_bit_cast(h16x2, hn), __builtin_bit_cast(h16x2, M),
                                                __builtin_bit_cast(h16x2, thr)));
    };
    // The first walk leaves each interior row's scores in the staged ROI, in place of the pixels: M of row r
    // (its two bytes, m <= 255) over ROI row r at the lane's pixel columns (off + 3, off + 4), stored at step r,
    // when no lane reads row r's pixels any more (row r was read at step r - 4 and lives in registers until
    // r + 3).  The minThFAST walk then reads the scores instead of re-running the ring network: m does not
    // depend on the threshold, only the NMS does.  A lane without pixel A or B stores that byte to ROI column
    // 0 or 1 (never a pixel of the walk: those start at column 3), so no two lanes store to one score byte (the
    // odd end's B column is the next cell's first pixel).
    uint8_t* const roi8 = reinterpret_cast<uint8_t*>(roi);
    const uint32_t m_at = act ? (uint32_t)(off + 3) : 0u, m_bt = actB ? (uint32_t)(off + 4) : 1u;
    // one walk over the interior rows at threshold tt, emitting for lanes with `on`
    auto walk = [&](auto L4, uint32_t tt, bool on) __attribute__((always_inline)) {
        const uint32_t thr = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tt | (tt << 16)));   // t' in both halves (SGPR)
        uint32_t win[7][7];   // pair rows, row y in slot y % 7; pair j = ROI columns 2p + j, 2p + j + 1
#pragma unroll
        for (int y = 0; y < 6; y++) {
            uint32_t d0, d1, d2;
            rd3(y, d0, d1, d2);
            build(d0, d1, d2, win[y]);
        }
        uint32_t n0, n1, n2;   // bytes of the next row (read one step ahead)
        rd3(6, n0, n1, n2);
        // rows r-1 (M, Hn, Hf) and r-2 (Hf); above the interior M = 0, so Hf = t'
        uint32_t Mp = 0, Hnp = 0, Hfp = thr, Hfpp = thr;
        // whole blocks of 7 rows with no exit test inside (an exit per unrolled row costs copies of the
        // loop-carried values on every row), then the last partial block with its per-row exits
        const int nfull = (rend - 3) / 7;   // wave-uniform
        int r0 = 3;
        auto row = [&](int u, int r) __attribute__((always_inline)) {
            build(n0, n1, n2, win[(6 + u) % 7]);   // row r + 3
            rd3(r + 4, n0, n1, n2);   // row ch (after the last interior row) is read but never used
            const uint32_t(&wm3)[7] = win[(u) % 7];       // row r - 3
            const uint32_t(&wm2)[7] = win[(1 + u) % 7];
            const uint32_t(&wm1)[7] = win[(2 + u) % 7];
            const uint32_t(&w0)[7] = win[(3 + u) % 7];    // row r
            const uint32_t(&wp1)[7] = win[(4 + u) % 7];
            const uint32_t(&wp2)[7] = win[(5 + u) % 7];
            const uint32_t(&wp3)[7] = win[(6 + u) % 7];   // row r + 3
            // ring k at (dx, dy) -> w_dy[3 + dx]
            const uint32_t ring[16] = {wp3[3], wp3[4], wp2[5], wp1[6], w0[6], wm1[6], wm2[5], wm3[4],
                                       wm3[3], wm3[2], wm2[1], wm1[0], w0[0], wp1[0], wp2[1], wp3[2]};
            const uint32_t M = fast_m2h(ring, w0[3]) & maskM;
            roi8[m_at + (uint32_t)r * kFastRowBytes] = (uint8_t)M;
            roi8[m_bt + (uint32_t)r * kFastRowBytes] = (uint8_t)(M >> 16);
            uint32_t Hn, Hf;
            hrow(L4, M, thr, Hn, Hf);
            if (r > 3) {   // NMS of row r - 1
                const h16x2 nb = hmax3(__builtin_bit_cast(h16x2, Hfpp), __builtin_bit_cast(h16x2, Hnp),
                                       __builtin_bit_cast(h16x2, Hf));
                emit(L4, r - 1, Mp, __builtin_bit_cast(uint32_t, nb), on);
            }
            Hfpp = Hfp;
            Hfp = Hf;
            Hnp = Hn;
            Mp = M;
        };
        for (int blk = 0; blk < nfull; blk++, r0 += 7) {
#pragma unroll
            for (int u = 0; u < 7; u++) row(u, r0 + u);
        }
#pragma unroll
        for (int u = 0; u < 6; u++) {
            if (r0 + u >= rend) break;
            row(u, r0 + u);
        }
        if (rend > 3) {   // the last interior row (row rend is outside: M = 0)
            const u16x2 nb = __builtin_elementwise_max(__builtin_bit_cast(u16x2, Hfpp), __builtin_bit_cast(u16x2, Hnp));
            emit(L4, rend - 1, Mp, __builtin_bit_cast(uint32_t, nb), on);
        }
    };
    // the NMS + emission of the walk above at threshold tt over the scores the first walk stored (no ring
    // network); the same row sequence, so the same survivors in the same order as a full walk at tt
    auto rewalk = [&](auto L4, uint32_t tt, bool on) __attribute__((always_inline)) {
        const uint32_t thr = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tt | (tt << 16)));
        const uint8_t* ma = roi8 + m_at;
        const uint8_t* mb = roi8 + m_bt;
        uint32_t a0 = ma[3 * kFastRowBytes], b0 = mb[3 * kFastRowBytes];   // row r's scores, read a row ahead
        uint32_t Mp = 0, Hnp = 0, Hfp = thr, Hfpp = thr;
        for (int r = 3; r < rend; r++) {
            const uint32_t M = (a0 | (b0 << 16)) & maskM;
            a0 = ma[(r + 1) * kFastRowBytes];   // row rend (< ch) is read but never used
            b0 = mb[(r + 1) * kFastRowBytes];
            uint32_t Hn, Hf;
            hrow(L4, M, thr, Hn, Hf);
            if (r > 3) {
                const h16x2 nb = hmax3(__builtin_bit_cast(h16x2, Hfpp), __builtin_bit_cast(h16x2, Hnp),
                                       __builtin_bit_cast(h16x2, Hf));
                emit(L4, r - 1, Mp, __builtin_bit_cast(uint32_t, nb), on);
            }
            Hfpp = Hfp;
            Hfp = Hf;
            Hnp = Hn;
            Mp = M;
        }
        if (rend > 3) {
            const u16x2 nb = __builtin_elementwise_max(__builtin_bit_cast(u16x2, Hfpp), __builtin_bit_cast(u16x2, Hnp));
            emit(L4, rend - 1, Mp, __builtin_bit_cast(uint32_t, nb), on);
        }
    };
    // thresholds t' = max(t, 1) as integers (compared as u16 with the scores; m <= 255, so t' is capped at 256)
    const uint32_t th_ini = (uint32_t)min(max(cfg.ini_th, 1), 256);
    const uint32_t th_min = (uint32_t)min(max(cfg.min_th, 1), 256);
    auto run = [&](auto L4) __attribute__((always_inline)) {
        walk(L4, th_ini, true);
        FAST_PROF(2);
        // cells without a corner at iniThFAST: the NMS again at minThFAST over the stored scores, emitting for
        // those cells only
        const bool redo = cell_on && cnt == slot_first && cfg.min_th < cfg.ini_th;
        if (__ballot(redo) != 0ull)
            rewalk(L4, th_min, redo);
    };
    if (LPC == 16)   // 16-lane cells (a DPP row each): the walk compiled for them, no per-row layout branches
        run(FastLg4{});
    else
        run(FastLgN{});
    if (cell_on && p == 0)
        cell_count[(size_t)b * cfg.n_cells + ci] = (int)(cnt - slot_first);
    FAST_PROF(3);
}

// ------------------------------------------------------------------ quadtree (:414-611)
// Parallel restatement of DistributeOctTree.  The std::list is an array in list order;
// a division round pushes all children to the front (newest first) and keeps the other
// nodes in order, so after a round: [children in reverse creation order] ++ [survivors].
// Phase 1 divides every node with >1 keys in list order; phase 2 divides them in
// (size, creation id) descending order until the list reaches N (creation id stands in
// for the reference's ExtractorNode* tie-break).
#define RGBD_DIST_THREADS 512   // 1024 / 512 / 256 measured 153.7k / 156.0k / 148.0k frames/s (LDS 76 / 38 / 38 KB)
constexpr int kDistThreads = RGBD_DIST_THREADS;

#ifdef RGBD_PNP_PROFILE
__device__ long long g_pyr_prof[8][16];   // k_pyramid strips 0..7 of frame 0: stage timestamps of thread 0
__device__ long long g_pyr_span[2048][2];  // k_pyramid: wall-clock start / end of every workgroup
__device__ long long g_dist_prof[4][64];   // per level 0..3 of frame 0: stage timestamps of thread 0
#define DIST_PROF(k) do { if (threadIdx.x == 0 && b == 0 && level < 4 && (k) < 64) g_dist_prof[level][(k)] = clock64(); } while (0)
#else
#define DIST_PROF(k) do { } while (0)
#endif
#ifdef RGBD_PNP_PROFILE
__device__ long long g_desc_prof[256][10];   // frame 0, slots 0..255: stage timestamps of lane 0
#define DESC_PROF(k) do { if (lane == 0 && b == 0 && s0 < 256) g_desc_prof[s0][(k)] = clock64(); } while (0)
#else
#define DESC_PROF(k) do { } while (0)
#endif

struct NodeBuf {
    int16_t* x0; int16_t* y0; int16_t* x1; int16_t* y1;
    int* size; int* cid;
};

__device__ __forceinline__ int quad_of(int kx, int ky, int x0, int y0, int x1, int y1)
{
    const int halfX = (x1 - x0 + 1) >> 1;   // ceil((float)(UR.x-UL.x)/2) for non-negative widths
    const int halfY = (y1 - y0 + 1) >> 1;
    const int mx = x0 + halfX, my = y0 + halfY;
    return (kx < mx) ? ((ky < my) ? 0 : 2) : ((ky < my) ? 1 : 3);
}

// quadrant of (kx, ky) in node nd of a packed {x0, y0, x1, y1} int16 box array (one 8-byte LDS read)
__device__ __forceinline__ int quad_in(int kx, int ky, const int16_t* bx, int nd)
{
    const uint64_t bb = *reinterpret_cast<const uint64_t*>(bx + 4 * nd);
    return quad_of(kx, ky, (int16_t)(bb & 0xFFFFu), (int16_t)((bb >> 16) & 0xFFFFu), (int16_t)((bb >> 32) & 0xFFFFu),
                   (int16_t)(bb >> 48));
}

// ordering of LDS traffic among the lanes of one wave
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave scans by DPP (GFX9 row_shr / row_bcast moves, every lane of the wave active): one VALU per step
// instead of a ds_bpermute round trip.  The moves stay v_mov_b32_dpp (the empty asm, as in fast_rank16).
__device__ __forceinline__ int dpp_add(int x, int t)
{
    asm volatile("" : "+v"(t));
    return x + t;
}
__device__ __forceinline__ int dpp_row_scan(int x)   // inclusive scan inside each row of 16 lanes
{
    x = dpp_add(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false));   // row_shr:1
    x = dpp_add(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false));   // row_shr:2
    x = dpp_add(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false));   // row_shr:4
    return dpp_add(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false));   // row_shr:8
}
__device__ __forceinline__ int wave_scan_incl(int x)   // inclusive scan over the 64 lanes
{
    x = dpp_row_scan(x);
    x = dpp_add(x, __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false));   // row_bcast:15 into rows 1, 3
    return dpp_add(x, __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false));   // row_bcast:31 into rows 2, 3
}
__device__ __forceinline__ int wave_sum(int x) { return __builtin_amdgcn_readlane(wave_scan_incl(x), 63); }

// base[idx] += 1 for every active lane, by runs: keys arrive in list (raster) order, so a wave's consecutive
// lanes mostly share idx.  A lane whose idx differs from the previous lane's (DPP wave_shr:1) starts a run; the
// run's first lane adds the run length (up to the next start or inactive lane): one ds_add of the run heads,
// which hit distinct addresses unless two runs share an idx.  (Round 4 combined the first distinct idx and left
// every other lane its own atomic in one ds_add, serialised by bank conflicts: 0.52 -> 0.46 ms per 1024 frames.)
__device__ __forceinline__ void lds_count(int* base, int idx, bool active)
{
    const int lane = (int)(threadIdx.x & 63);
    const int key = active ? idx : -1;
    int prev = __builtin_amdgcn_update_dpp(-2, key, 0x138, 0xf, 0xf, false);   // wave_shr:1, lane 0 keeps -2
    asm volatile("" : "+v"(prev));
    const bool start = active && key != prev;
    const unsigned long long bnd = __ballot(start) | ~__ballot(active);
    if (start) {
        const unsigned long long above = bnd & ~((2ull << lane) - 1ull);   // boundaries after this lane (lane 63: none)
        const int end = above ? __ffsll((long long)above) - 1 : 64;
        atomicAdd(&base[idx], end - lane);
    }
}

// atomicMax(&base[idx], v) for every active lane
__device__ __forceinline__ void lds_max(unsigned int* base, int idx, unsigned int v, bool active)
{
    if (active) atomicMax(&base[idx], v);
}

__device__ int block_scan_excl(int* a, int n, int* wsum)
{
    const int tid = threadIdx.x;
    const int per = (n + kDistThreads - 1) / kDistThreads;
    const int beg = min(tid * per, n), end = min(beg + per, n);
    int s = 0;
    for (int i = beg; i < end; i++) s += a[i];
    const int lane = tid & 63, w = tid >> 6;
    const int x = wave_scan_incl(s);
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int wpre = 0, total = 0;
#pragma unroll
    for (int i = 0; i < kDistThreads / 64; i++) {
        if (i < w) wpre += wsum[i];
        total += wsum[i];
    }
    int run = wpre + x - s;
    for (int i = beg; i < end; i++) {
        const int v = a[i];
        a[i] = run;
        run += v;
    }
    __syncthreads();
    return total;
}

#define RGBD_DIST_WPE 8
// NodeT: the per-key node id in LDS (uint8_t while node_cap <= 256, i.e. nfeatures <= ~1700; else uint16_t).
// Levels [l0, l0 + nlv) of every frame, one workgroup each; kc = the keys per level whose round state (the
// u32 key as FAST wrote it + the node id) fits in this launch's LDS.  A level with more candidates keeps it
// in the HBM scratch (keys_g / node_g) instead -- correct for any count, but every round then goes to memory.
template <typename NodeT>
__global__ __launch_bounds__(kDistThreads) __attribute__((amdgpu_waves_per_eu(RGBD_DIST_WPE, 8))) void k_distribute(const int* __restrict__ cell_count,
                                                             const uint32_t* __restrict__ cell_slots,
                                                             const ExtractCfg* __restrict__ cfgp,
                                                             uint32_t* __restrict__ keys_g,
                                                             uint16_t* __restrict__ node_g,
                                                             int* __restrict__ sel_count, uint32_t* __restrict__ sel,
                                                             int* __restrict__ err, int l0, int nlv, int kc, int xcd)
{
    extern __shared__ __align__(16) unsigned char smem[];
    const ExtractCfg& cfg = *cfgp;
    // Level-major dispatch: every frame's level-0 tree is dispatched before any level-1 tree, and so on (the
    // longest trees first, so the launch does not end on a tail of level-0 trees: 0.76 -> 0.53 ms at
    // B = 1024).  xcd (1-D grid, B a multiple of 8): frame b runs on XCD b % 8, the XCD k_fast wrote its
    // cell lists from and k_describe reads its selection on.
    int b, level;
    if (xcd) {
        const int j = (int)blockIdx.x >> 3, G = (int)gridDim.x / (8 * nlv);
        b = (j % G) * 8 + ((int)blockIdx.x & 7);
        level = l0 + j / G;
    } else {
        const int B = (int)gridDim.x / nlv;
        b = (int)blockIdx.x % B;
        level = l0 + (int)blockIdx.x / B;
    }
    const int tid = threadIdx.x;
    const LevelCfg& LV = cfg.lv[level];
    const int NC = cfg.node_cap;
    // ---- LDS carve
    unsigned long long* sortkey = reinterpret_cast<unsigned long long*>(smem);          // NC
    int* childcnt = reinterpret_cast<int*>(sortkey + NC);                                // 4 NC
    int* childcnt2 = childcnt + 4 * NC;                                                  // 4 NC
    const int SC = cfg.scan_cap;                                                         // max(NC, cells/level)+1
    int* tmp = childcnt2 + 4 * NC;                                                        // SC
    int* tmp2 = tmp + SC;                                                                // SC
    int* sizeA = tmp2 + SC;
    int* cidA = sizeA + NC;
    int* sizeB = cidA + NC;
    int* cidB = sizeB + NC;
    int* best = cidB + NC;                                                               // NC
    int16_t* childIdx = reinterpret_cast<int16_t*>(best + NC);                           // 4 NC
    int16_t* newIdx = childIdx + 4 * NC;                                                 // NC
    int16_t* ord = newIdx + NC;                                                          // NC
    int16_t* bxA = ord + NC;                                                             // 4 NC (x0,y0,x1,y1)
    int16_t* bxB = bxA + 4 * NC;                                                         // 4 NC
    uint32_t* kk32 = reinterpret_cast<uint32_t*>(bxB + 4 * NC);                          // kc keys: x | y << 11 | score << 22
    NodeT* kno = reinterpret_cast<NodeT*>(kk32 + kc);                                    // kc node ids
    __shared__ int wsum[kDistThreads / 64];
    __shared__ int s_J;

    uint32_t* keys = keys_g + (size_t)b * cfg.keys_per_frame + LV.key_off;
    uint16_t* nodeOf = node_g + (size_t)b * cfg.keys_per_frame + LV.key_off;
    const int N = LV.N;
    DIST_PROF(0);
#ifdef RGBD_PNP_PROFILE
    if (threadIdx.x == 0 && b == 0 && level < 4) g_dist_prof[level][46] = wall_clock64();
#endif

    // ---- gather this level's cell lists in cell order (vToDistributeKeys order), fused with the
    //      root assignment (:420-446): 16 lanes per cell, four cells per wave in flight
    const int nCells = LV.cell_count;
    const int nIni = LV.nIni;
    const float hX = LV.hX;
    for (int i = tid; i < nCells; i += kDistThreads)
        tmp[i] = cell_count[(size_t)b * cfg.n_cells + LV.cell_begin + i];
    for (int i = tid; i < nIni; i += kDistThreads) sizeA[i] = 0;
    __syncthreads();
    for (int i = tid; i < nCells; i += kDistThreads) tmp2[i] = tmp[i];
    __syncthreads();
    const int n = block_scan_excl(tmp2, nCells, wsum);   // tmp2 = offsets, tmp = counts
    // the per-round key state (the key as FAST wrote it + its node id) lives in LDS when it fits, else in HBM
    // Per-round key state: the key as FAST wrote it + its node id.  Both in LDS when they fit (inL); else the node
    // ids alone in the same LDS region (ndL: the level's keys are written to the HBM scratch once by the gather
    // and only read after it, so no division round writes to HBM); else both in the HBM scratch
    const bool inL = n <= kc;
    const bool ndL = !inL && n * (int)sizeof(NodeT) <= kc * (4 + (int)sizeof(NodeT));
    NodeT* kndL = reinterpret_cast<NodeT*>(kk32);   // ndL: node ids from the region's start
    auto key_at = [&](int kk) -> uint32_t { return inL ? kk32[kk] : keys[kk]; };
    auto nd_get = [&](int kk) -> int { return inL ? (int)kno[kk] : (ndL ? (int)kndL[kk] : (int)nodeOf[kk]); };
    auto nd_set = [&](int kk, int v) {
        if (inL)
            kno[kk] = (NodeT)v;
        else if (ndL)
            kndL[kk] = (NodeT)v;
        else
            nodeOf[kk] = (uint16_t)v;
    };
    {
        const int w = tid >> 6, sub = (tid >> 4) & 3, l16 = tid & 15;
        constexpr int kCStep = 4 * (kDistThreads / 64);   // cells per workgroup step
        // two cell groups per step, the first 16 keys of each loaded before either is processed
        for (int c00 = 4 * w; c00 < nCells; c00 += 2 * kCStep) {
            int cntg[2], og[2], tripsg[2];
            const uint32_t* srcg[2];
            uint32_t v0g[2];
            // every key of the first kPre trips of both groups loaded before any is processed (one global
            // round trip per step instead of one per trip: level-0 cells hold ~34 keys, three trips)
            constexpr int kPre = 4;
            uint32_t vpre[2][kPre];
#pragma unroll
            for (int g = 0; g < 2; g++) {
                const int ci = c00 + g * kCStep + sub;
                // wave-uniform trip count so the counting below sees the whole wave
                int trips = (ci < nCells) ? (tmp[ci] + 15) >> 4 : 0;
#pragma unroll
                for (int o = 16; o < 64; o <<= 1) trips = max(trips, __shfl_xor(trips, o, 64));
                tripsg[g] = trips;
                cntg[g] = (ci < nCells) ? tmp[ci] : 0;
                og[g] = (ci < nCells) ? tmp2[ci] : 0;
                srcg[g] = cell_slots + ((size_t)b * cfg.n_cells + LV.cell_begin + (ci < nCells ? ci : 0)) * cfg.cell_cap;
#pragma unroll
                for (int t = 0; t < kPre; t++) vpre[g][t] = l16 + 16 * t < cntg[g] ? srcg[g][l16 + 16 * t] : 0u;
            }
            (void)v0g;
#pragma unroll
            for (int g = 0; g < 2; g++) {
            const int trips = tripsg[g], cnt = cntg[g], o = og[g];
            const uint32_t* src = srcg[g];
            for (int tr = 0; tr < trips; tr++) {
                const int j = l16 + 16 * tr;
                const bool on = j < cnt;
                int idx = 0;
                if (on) {
                    uint32_t v;
                    if (tr < kPre) {
                        v = vpre[g][0];
#pragma unroll
                        for (int t = 1; t < kPre; t++) v = tr == t ? vpre[g][t] : v;
                    } else {
                        v = src[j];
                    }
                    // one root (nIni == 1: any image wider than tall and < 1.5x as wide, every 640 x 480
                    // level): no division, no root count (the root holds all n keys, set below) and no node
                    // id (the root pass writes every key's)
                    if (nIni > 1) {
                        idx = (int)((float)(int)(v & 2047u) / hX);
                        idx = min(max(idx, 0), nIni - 1);
                    }
                    if (inL) {
                        kk32[o + j] = v;
                        if (nIni > 1) kno[o + j] = (NodeT)idx;
                    } else {
                        keys[o + j] = v;
                        if (nIni > 1) nd_set(o + j, idx);
                    }
                }
                if (nIni > 1) lds_count(sizeA, idx, on);
            }
            }
        }
    }
    if (nIni == 1 && tid == 0) sizeA[0] = n;
    __threadfence_block();
    __syncthreads();
    DIST_PROF(1);

    // ---- compaction of the non-empty roots (:448-459) on wave 0; current node arrays start as B
    const int lane = tid & 63;
    const unsigned long long lanes_below = (1ull << lane) - 1ull;
    int* sz = sizeB; int* cd = cidB; int16_t* bx = bxB;
    int* szN = sizeA; int* cdN = cidA; int16_t* bxN = bxA;
    int* cc = childcnt; int* ccN = childcnt2;
    if (tid < 64) {
        int carry = 0;
        for (int base = 0; base < nIni; base += 64) {
            const int i = base + lane;
            const bool f = i < nIni && sizeA[i] > 0;
            const unsigned long long bal = __ballot(f);
            if (f) {
                const int j = carry + __popcll(bal & lanes_below);
                tmp[i] = j;
                sz[j] = sizeA[i];
                cd[j] = i;
                bx[4 * j + 0] = (int16_t)(int)(hX * (float)i);
                bx[4 * j + 1] = 0;
                bx[4 * j + 2] = (int16_t)(int)(hX * (float)(i + 1));
                bx[4 * j + 3] = (int16_t)(LV.maxBY - LV.minBY);
            }
            carry += __popcll(bal);
        }
        for (int i = lane; i < 4 * carry; i += 64) cc[i] = 0;
        if (lane == 0) s_J = carry;
    }
    __syncthreads();
    int L = s_J;
    // root ids -> compacted ids, fused with the first round's child counts: two keys per thread per step, the
    // next step's keys loaded ahead (as in the division rounds below)
    {
        constexpr int kStep = 2 * kDistThreads;
        uint32_t kpa = n > 0 ? key_at(tid < n ? tid : n - 1) : 0u;
        uint32_t kpb = n > 0 ? key_at(tid + kDistThreads < n ? tid + kDistThreads : n - 1) : 0u;
        for (int k0 = 0; k0 < n; k0 += kStep) {
            const int ka = k0 + tid, kb = ka + kDistThreads;
            const int ca = ka < n ? ka : n - 1, cb = kb < n ? kb : n - 1;   // clamped loads; stores / counts masked
            const uint32_t va = kpa, vb = kpb;
            if (k0 + kStep < n) {
                kpa = key_at(ka + kStep < n ? ka + kStep : n - 1);
                kpb = key_at(kb + kStep < n ? kb + kStep : n - 1);
            }
            const int nda = nIni == 1 ? 0 : tmp[nd_get(ca)], ndb = nIni == 1 ? 0 : tmp[nd_get(cb)];
            const int xa = (int)(va & 2047u), ya = (int)((va >> 11) & 2047u);
            const int xb = (int)(vb & 2047u), yb = (int)((vb >> 11) & 2047u);
            const bool ona = ka < n && sz[nda] > 1, onb = kb < n && sz[ndb] > 1;
            const int ta = ona ? 4 * nda + quad_in(xa, ya, bx, nda) : 0;
            const int tb = onb ? 4 * ndb + quad_in(xb, yb, bx, ndb) : 0;
            if (ka < n) nd_set(ka, nda);
            if (kb < n) nd_set(kb, ndb);
            lds_count(cc, ta, ona);
            lds_count(cc, tb, onb);
        }
    }
    __threadfence_block();
    __syncthreads();

    DIST_PROF(2);
    // ---- division rounds.  Node bookkeeping (order, child offsets, survivors) runs on wave 0 with
    //      wave-level scans; the one pass over the keys per round moves every key to its new node
    //      and counts it into the new node's quadrant for the next round (or, in the last round,
    //      into the best-key slot of its final node)
    unsigned int* ubest = reinterpret_cast<unsigned int*>(best);
    int nextCid = nIni;
    int phase = 1;
    int rounds = 0;
    bool best_done = false;
    __shared__ int s_round[4];   // T, Lnew, nToExpand, last
    while (L > 0 && rounds < 4096) {
        rounds++;
        const int prevSize = L;
        if (phase == 2 && L <= kDistThreads) {
            // (size, creation id) descending order by rank: every divisible node counts the larger keys
            unsigned long long key = 0ull;
            if (tid < L && sz[tid] > 1)
                key = ((unsigned long long)sz[tid] << 44) | ((unsigned long long)cd[tid] << 16) | (unsigned long long)tid;
            if (tid < L) sortkey[tid] = key;
            __syncthreads();
            if (key != 0ull) {
                int rank = 0;
                for (int j = 0; j < L; j++) rank += sortkey[j] > key ? 1 : 0;
                ord[rank] = (int16_t)tid;
            }
            __syncthreads();
        }
        if (tid < 64) {
            // division order: phase 1 list order, phase 2 (size, creation id) descending
            int nS = 0;
            if (phase == 1) {
                for (int base = 0; base < L; base += 64) {
                    const int i = base + lane;
                    const bool f = i < L && sz[i] > 1;
                    const unsigned long long bal = __ballot(f);
                    if (f) ord[nS + __popcll(bal & lanes_below)] = (int16_t)i;
                    nS += __popcll(bal);
                }
            } else {
                int P = 2;
                while (P < L) P <<= 1;
                if (L <= kDistThreads) {   // ord was ranked by the whole block
                    for (int i = lane; i < L; i += 64) nS += sz[i] > 1 ? 1 : 0;
                    nS = wave_sum(nS);
                } else {
                for (int i = lane; i < P; i += 64) {
                    unsigned long long key = 0ull;
                    if (i < L && sz[i] > 1)
                        key = ((unsigned long long)sz[i] << 44) | ((unsigned long long)cd[i] << 16) | (unsigned long long)i;
                    sortkey[i] = key;
                    nS += (i < L && sz[i] > 1) ? 1 : 0;
                }
                nS = wave_sum(nS);
                wave_lds_sync();
                for (int k2 = 2; k2 <= P; k2 <<= 1) {
                    for (int j = k2 >> 1; j > 0; j >>= 1) {
                        for (int i = lane; i < P; i += 64) {
                            const int ixj = i ^ j;
                            if (ixj > i) {
                                const unsigned long long x = sortkey[i], y = sortkey[ixj];
                                const bool descBlock = (i & k2) == 0;
                                if (descBlock ? (x < y) : (x > y)) {
                                    sortkey[i] = y;
                                    sortkey[ixj] = x;
                                }
                            }
                        }
                        wave_lds_sync();
                    }
                }
                for (int j = lane; j < nS; j += 64) ord[j] = (int16_t)(sortkey[j] & 0xFFFFull);
                }
            }
            wave_lds_sync();
            // children per division c_j, creation offsets C_j, and (phase 2) the first division J
            // after which the list reaches N
            int carry = 0, J = nS;
            for (int base = 0; base < nS; base += 64) {
                const int j = base + lane;
                int cj = 0;
                if (j < nS) {
                    const int nd = ord[j];
                    cj = (cc[4 * nd] > 0) + (cc[4 * nd + 1] > 0) + (cc[4 * nd + 2] > 0) + (cc[4 * nd + 3] > 0);
                }
                const int incl = wave_scan_incl(cj);
                const int Cj = carry + incl - cj;
                if (j < nS) { tmp[j] = Cj; tmp2[j] = cj; }
                if (phase == 2 && J == nS) {
                    const unsigned long long hb = __ballot(j < nS && L + (Cj + cj) - (j + 1) >= N);
                    if (hb) J = base + __ffsll((long long)hb) - 1;
                }
                carry += __builtin_amdgcn_readlane(incl, 63);
            }
            const int nApply = (phase == 2 && J < nS) ? J + 1 : nS;
            wave_lds_sync();
            const int T = (nApply > 0) ? tmp[nApply - 1] + tmp2[nApply - 1] : 0;
            for (int i = lane; i < L; i += 64) newIdx[i] = 0;
            wave_lds_sync();
            for (int j = lane; j < nApply; j += 64) newIdx[ord[j]] = -1;
            wave_lds_sync();
            // survivors keep their order behind the new children
            int sv = 0;
            for (int base = 0; base < L; base += 64) {
                const int i = base + lane;
                const bool f = i < L && newIdx[i] == 0;
                const unsigned long long bal = __ballot(f);
                if (f) {
                    const int ni = T + sv + __popcll(bal & lanes_below);
                    newIdx[i] = (int16_t)ni;
                    szN[ni] = sz[i];
                    cdN[ni] = cd[i];
#pragma unroll
                    for (int q = 0; q < 4; q++) bxN[4 * ni + q] = bx[4 * i + q];
                }
                sv += __popcll(bal);
            }
            // children, newest first
            for (int j = lane; j < nApply; j += 64) {
                const int nd = ord[j];
                int o = tmp[j];
                const int x0 = bx[4 * nd], y0 = bx[4 * nd + 1], x1 = bx[4 * nd + 2], y1 = bx[4 * nd + 3];
                const int mx = x0 + ((x1 - x0 + 1) >> 1), my = y0 + ((y1 - y0 + 1) >> 1);
                for (int q = 0; q < 4; q++) {
                    const int cnt = cc[4 * nd + q];
                    if (cnt > 0) {
                        const int ni = T - 1 - o;
                        szN[ni] = cnt;
                        cdN[ni] = nextCid + o;
                        const int cx0 = (q & 1) ? mx : x0, cx1 = (q & 1) ? x1 : mx;
                        const int cy0 = (q & 2) ? my : y0, cy1 = (q & 2) ? y1 : my;
                        bxN[4 * ni + 0] = (int16_t)cx0;
                        bxN[4 * ni + 1] = (int16_t)cy0;
                        bxN[4 * ni + 2] = (int16_t)cx1;
                        bxN[4 * ni + 3] = (int16_t)cy1;
                        childIdx[4 * nd + q] = (int16_t)ni;
                        o++;
                    }
                }
            }
            wave_lds_sync();
            const int Lnew = T + (L - nApply);
            int expand = 0;
            for (int i = lane; i < T; i += 64) expand += szN[i] > 1 ? 1 : 0;
            expand = wave_sum(expand);
            const bool last = Lnew >= N || Lnew == prevSize || Lnew > NC - 4 || rounds >= 4096;
            if (last)
                for (int i = lane; i < Lnew; i += 64) ubest[i] = 0u;
            else
                for (int i = lane; i < 4 * Lnew; i += 64) ccN[i] = 0;
            if (lane == 0) { s_round[0] = T; s_round[1] = Lnew; s_round[2] = expand; s_round[3] = last ? 1 : 0; }
        }
        __syncthreads();
        DIST_PROF(20 + rounds);
        const int T = s_round[0], Lnew = s_round[1], nToExpand = s_round[2];
        const bool last = s_round[3] != 0;
        // two keys per thread per step (their dependent LDS chains -- node id -> new index -> child slot ->
        // size -> box -- interleaved), the next step's two keys loaded before them, so the keys' L2 round
        // trips (levels whose keys live in the HBM scratch) and the chains overlap
        constexpr int kStep = 2 * kDistThreads;
        uint32_t kpa = n > 0 ? key_at(tid < n ? tid : n - 1) : 0u;
        uint32_t kpb = n > 0 ? key_at(tid + kDistThreads < n ? tid + kDistThreads : n - 1) : 0u;
        for (int k0 = 0; k0 < n; k0 += kStep) {
            const int ka = k0 + tid, kb = ka + kDistThreads;
            const int ca = ka < n ? ka : n - 1, cb = kb < n ? kb : n - 1;   // clamped loads; stores / counts masked
            const uint32_t va = kpa, vb = kpb;
            if (k0 + kStep < n) {
                kpa = key_at(ka + kStep < n ? ka + kStep : n - 1);
                kpb = key_at(kb + kStep < n ? kb + kStep : n - 1);
            }
            const int nda = nd_get(ca), ndb = nd_get(cb);
            const int xa = (int)(va & 2047u), ya = (int)((va >> 11) & 2047u);
            const int xb = (int)(vb & 2047u), yb = (int)((vb >> 11) & 2047u);
            int nia = newIdx[nda], nib = newIdx[ndb];
            const int cia = childIdx[4 * nda + quad_in(xa, ya, bx, nda)], cib = childIdx[4 * ndb + quad_in(xb, yb, bx, ndb)];
            nia = nia < 0 ? cia : nia;
            nib = nib < 0 ? cib : nib;
            if (last) {
                lds_max(ubest, nia, ((unsigned int)key_s(va) << 24) | (unsigned int)(0xFFFFFF - ka), ka < n);
                lds_max(ubest, nib, ((unsigned int)key_s(vb) << 24) | (unsigned int)(0xFFFFFF - kb), kb < n);
            } else {
                const int sna = szN[nia], snb = szN[nib];
                const bool ona = ka < n && sna > 1, onb = kb < n && snb > 1;
                const int ta = ona ? 4 * nia + quad_in(xa, ya, bxN, nia) : 0;
                const int tb = onb ? 4 * nib + quad_in(xb, yb, bxN, nib) : 0;
                if (ka < n) nd_set(ka, nia);
                if (kb < n) nd_set(kb, nib);
                lds_count(ccN, ta, ona);
                lds_count(ccN, tb, onb);
            }
        }
        __threadfence_block();
        __syncthreads();
        // swap buffers
        { int* t1 = sz; sz = szN; szN = t1; }
        { int* t2 = cd; cd = cdN; cdN = t2; }
        { int16_t* t3 = bx; bx = bxN; bxN = t3; }
        { int* t4 = cc; cc = ccN; ccN = t4; }
        L = Lnew;
        nextCid += T;
        DIST_PROF(2 + rounds);
        best_done = last;
        if (L >= N || L == prevSize)
            break;
        if (phase == 1 && L + nToExpand * 3 > N)
            phase = 2;
        if (L > NC - 4) {   // capacity guard (cannot trigger for budgets the host accepted)
            if (tid == 0) atomicOr(err + b, 1);   // per frame
            break;
        }
    }
    DIST_PROF(40);
    if (threadIdx.x == 0 && b == 0 && level < 4) { DIST_PROF(41); }
    // ---- retain the best key per node (:594-608): max response, first in key order
    if (!best_done) {   // no division round ran
        for (int i = tid; i < L; i += kDistThreads) ubest[i] = 0u;
        __syncthreads();
        for (int k = tid; k < n; k += kDistThreads)
            atomicMax(&ubest[nd_get(k)], ((unsigned int)key_s(key_at(k)) << 24) | (unsigned int)(0xFFFFFF - k));
    }
    __syncthreads();
    uint32_t* out = sel + (size_t)b * cfg.sel_per_frame + LV.sel_off;
    for (int i = tid; i < L; i += kDistThreads) {
        const int k = 0xFFFFFF - (int)(ubest[i] & 0xFFFFFFu);
        out[i] = key_at(k);
    }
    if (tid == 0) sel_count[b * cfg.nlevels + level] = L;
#ifdef RGBD_PNP_PROFILE
    if (threadIdx.x == 0 && b == 0 && level < 4) { g_dist_prof[level][42] = clock64(); g_dist_prof[level][43] = rounds; g_dist_prof[level][44] = n; g_dist_prof[level][45] = phase; g_dist_prof[level][47] = wall_clock64(); }
#endif
}

// ------------------------------------------------------------------ describe (:16-87, :697-766)
__device__ __forceinline__ float fast_atan2_deg(float y, float x)
{
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = fabsf(x), ay = fabsf(y);
    // both branches of the reference as one division of selected operands (no divergent paths when the
    // two keypoints of a wave fall on different sides)
    const bool ge = ax >= ay;
    const float c = (ge ? ay : ax) / ((ge ? ax : ay) + (float)2.220446049250313080847e-16);
    const float c2 = c * c;
    const float t = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    float a = ge ? t : 90.f - t;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// float cos/sin as the rounding of a double evaluation built from + - * only (same
// operation sequence as the oracle's definition; see DESIGN.md "Oracle definitions").
__device__ __forceinline__ void cos_sin_f(float xf, float* co, float* si)
{
    const double PIO2_1 = 1.57079632673412561417e+00;
    const double PIO2_1T = 6.07710050650619224932e-11;
    const double INV_PIO2 = 6.36619772367581382433e-01;
    const double x = (double)xf;
    const double kd = floor(x * INV_PIO2 + 0.5);
    const int k = (int)kd;
    const double r = (x - kd * PIO2_1) - kd * PIO2_1T;
    const double r2 = r * r;
    double s = -1.0 / 121645100408832000.0;
    s = s * r2 + 1.0 / 355687428096000.0;
    s = s * r2 - 1.0 / 1307674368000.0;
    s = s * r2 + 1.0 / 6227020800.0;
    s = s * r2 - 1.0 / 39916800.0;
    s = s * r2 + 1.0 / 362880.0;
    s = s * r2 - 1.0 / 5040.0;
    s = s * r2 + 1.0 / 120.0;
    s = s * r2 - 1.0 / 6.0;
    s = s * r2 + 1.0;
    const double sr = s * r;
    double c = -1.0 / 6402373705728000.0;
    c = c * r2 + 1.0 / 20922789888000.0;
    c = c * r2 - 1.0 / 87178291200.0;
    c = c * r2 + 1.0 / 479001600.0;
    c = c * r2 - 1.0 / 3628800.0;
    c = c * r2 + 1.0 / 40320.0;
    c = c * r2 - 1.0 / 720.0;
    c = c * r2 + 1.0 / 24.0;
    c = c * r2 - 0.5;
    c = c * r2 + 1.0;
    double cc, ss;
    switch (k & 3) {
    case 0: cc = c; ss = sr; break;
    case 1: cc = -sr; ss = c; break;
    case 2: cc = -c; ss = -sr; break;
    default: cc = sr; ss = -c; break;
    }
    *co = (float)cc;
    *si = (float)ss;
}

// ------------------------------------------------------------------ level blur (:745-746)
// GaussianBlur(level.clone(), 7x7, sigma 2, BORDER_REFLECT_101) of every pyramid level, bit-exact
// ufixedpoint16 (kernel {18,34,49,54,49,34,18}/256): the reference blurs whole levels
// once and samples the 256 rBRIEF tests from them, so the blurred pyramid is built once per frame
// here (same layout as the pyramid) and k_describe only gathers from it.
// One thread = one column quad (4 px) of one 32-row strip of a level; it walks the strip's 38 input
// rows (REFLECT_101 row index) top to bottom: three dword loads per row, the horizontal 7-tap sums of
// its 4 px as 2-3 v_dot4 each, kept as u16 row pairs in a BlurCol window (the loop is fully
// unrolled, so the window shifts are renames), and one vertical 7-tap output dword per row.  No LDS,
// no barriers; neighbouring lanes read neighbouring dwords (coalesced) and write a coalesced row.
// Level l owns threads [blur_t0[l], blur_t0[l + 1]) = strips x blur_tx[l] (quads per row).
#define RGBD_BLUR_PF 8

// One strip column walk.  Inner quads (bytes x - 4 .. x + 11 inside the row) use the window
// A = x - 4 as is.  Edge quads (x = 0, x + 8 > w) load the aligned 16-byte window A .. A + 15 of each
// row that holds the 12 bytes they need (columns x - 4 .. x + 7, REFLECT_101: A = 0 at the left edge,
// (w - 12) & ~3 at the right edge); each of their three source dwords is one v_perm of a dword pair
// of the window with a per-thread selector computed once.
// REFLECT_101 of a walk row p in [-3, h + 2] for h >= 4: one reflection, min(|p|, 2h - 2 - |p|)
__device__ __forceinline__ int reflect_row1(int p, int n)
{
    const int q = p < 0 ? -p : p;
    return min(q, 2 * n - 2 - q);
}
template <bool kEdge, bool kOne>
__device__ __forceinline__ void blur_walk(const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur, uint32_t fo,
                                          const LevelCfg& L, int x, int y0)
{
    // (kOne: level height >= 4, every walk row one reflection from the level; else the general REFLECT_101)
    auto rrow = [&](int p) { return kOne ? reflect_row1(p, L.h) : reflect101(p, L.h); };
    // addresses as 32-bit byte offsets fo + ... from the kernel-argument bases (frame pyramids < 4 GiB,
    // api.cpp): SGPR-base loads and stores, no 64-bit pointer live through the walk
    int p[3] = {0, 1, 2};
    uint32_t sel[3] = {0x03020100u, 0x03020100u, 0x03020100u};
    const int A = kEdge ? blur_edge_window(x, L.w, p, sel) : x - 4;
    const uint32_t base = fo + (uint32_t)A;
    BlurCol col;   // horizontal sums of the last input rows (row pairs)
    // software pipeline: the loads of row i + kPf are issued before row i is consumed
    constexpr int kPf = RGBD_BLUR_PF, kRows = kBlurTH + 6;
    typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));   // a dword-aligned window
    u32x4_a4 ring[kPf + 1];
#pragma unroll
    for (int i = 0; i < kPf; i++)
        ring[i] = *reinterpret_cast<const u32x4_a4*>(pyr + (base + (uint32_t)(rrow(y0 - 3 + i) * L.stride)));
#pragma unroll
    for (int i = 0; i < kRows; i++) {
        if (i + kPf < kRows)
            ring[(i + kPf) % (kPf + 1)] = *reinterpret_cast<const u32x4_a4*>(pyr + (base + (uint32_t)(rrow(y0 - 3 + i + kPf) * L.stride)));
        const u32x4_a4 r = ring[i % (kPf + 1)];
        uint32_t d[3];
        if (kEdge) {
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const uint32_t lo = p[j] == 0 ? r.x : (p[j] == 1 ? r.y : r.z);
                const uint32_t hi = p[j] == 0 ? r.y : (p[j] == 1 ? r.z : r.w);
                d[j] = __builtin_amdgcn_perm(hi, lo, sel[j]);
            }
        } else {
            d[0] = r.x;
            d[1] = r.y;
            d[2] = r.z;
        }
        col.push(d[0], d[1], d[2]);
        const int y = y0 + i - 6;
        if (i >= 6 && y < L.h)   // bytes of a last quad past w land in the row padding
            *reinterpret_cast<uint32_t*>(blur + (fo + (uint32_t)(y * L.stride + x))) = col.out();
    }
}

// The edge quads' walk as a function of its own: inlined beside the inner walk, the compiler merged the two
// (they differ only in p / sel) into one walk that ran the edge selects (12 v_cndmask + 3 v_perm per row) and
// the REFLECT_101 loop on every inner quad too.
__attribute__((noinline)) __device__ void blur_walk_edge(const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                                         uint32_t fo, const LevelCfg& L, int x, int y0)
{
    blur_walk<true, false>(pyr, blur, fo, L, x, y0);
}

// Threads [0, blur_t0[kMaxLevels]) walk the inner quads of every level strip, the threads after them
// the edge quads, so all but one wave run the select-free inner walk.
__device__ __forceinline__ void blur_thread(const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                            const ExtractCfg& cfg, int b, int t)
{
    const bool edge = t >= cfg.blur_t0[kMaxLevels];
    if (edge) {
        t -= cfg.blur_t0[kMaxLevels];
        if (t >= cfg.blur_e0[kMaxLevels]) return;
    }
    const int* t0 = edge ? cfg.blur_e0 : cfg.blur_t0;
    int l = 0;
#pragma unroll
    for (int i = 1; i < kMaxLevels; i++) l += (i < cfg.nlevels && t >= t0[i]) ? 1 : 0;
    const LevelCfg& L = cfg.lv[l];
    const int Q = edge ? cfg.blur_ex[l] : cfg.blur_tx[l];
    const int tl = t - t0[l];
    const int strip = tl / Q, qi = tl - strip * Q;
    const uint32_t fo = (uint32_t)b * (uint32_t)cfg.frame_pyr_bytes + (uint32_t)L.off;
    if (!edge) {
        if (L.h >= 4)
            blur_walk<false, true>(pyr, blur, fo, L, 4 * (qi + 1), strip * kBlurTH);
        else
            blur_walk<false, false>(pyr, blur, fo, L, 4 * (qi + 1), strip * kBlurTH);
    } else {   // x = 0, then the quads from the first with x + 8 > w
        blur_walk_edge(pyr, blur, fo, L, qi == 0 ? 0 : 4 * (cfg.blur_tx[l] + qi), strip * kBlurTH);
    }
}

#define RGBD_DESC_WAVES 2   // waves per k_describe workgroup: 1 / 2 / 4 / 8 measured 134.1k / 134.2k / 132.1k / 126.1k frames/s at B = 512
#define RGBD_DESC_EU 8   // min waves per SIMD: 64 VGPRs, so the 8 waves the LDS now allows fit (r04: 80 VGPRs held 6)
constexpr int kDescWaves = RGBD_DESC_WAVES;
constexpr int kBlurR = 18;    // max |rotated pattern offset|: the blurred square every test point lies in
constexpr int kBlurW = 2 * kBlurR + 1;                     // 37

// the dword at byte column x (a multiple of 4) of row gy, as the level's bytes with REFLECT_101
// column and row indices (the slow path of k_describe; see there)
__device__ __forceinline__ uint32_t dword_reflect(const uint8_t* img, int stride, int w, int h, int gy, int x)
{
    const uint8_t* row = img + (size_t)reflect101(gy, h) * stride;
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) v |= (uint32_t)row[reflect101(x + i, w)] << (8 * i);
    return v;
}

constexpr int kSqDw = 12;                    // staged dwords per square row (11 used: columns from (x - 18) & ~3)
constexpr int kSqN = kBlurW * kSqDw;         // 444
// each lane loads its IC disk row (9 dwords) into VGPRs in round trip 2 instead of staging the disk in LDS,
// so a keypoint holds 1,776 B of LDS (the blurred square) instead of 3,264 B (r04: 0.74 -> 0.706 ms,
// profiles/r04_ab_desc_disk; the LDS-staged disk was removed)
constexpr int kDescLds = 4 * kSqN;   // LDS bytes per keypoint

// Two selection slots (level l, index i) per wave, one per 32-lane half: the per-keypoint scalar work
// (level, addresses, fastAtan2, the f64 cos/sin) is evaluated once per half, so every VALU
// instruction of it serves two keypoints.  Slots are laid out as k_distribute's per-level selection
// (sel_off).  Every load whose address does not depend on the keypoint (the selection counts, the
// slots' keys, this lane's IC disk row weight and test pairs) is issued in the first round trip;
// the keypoint's rows (IC disk of the unblurred level; the 37 x 37 square of the blurred level,
// k_blur) in the second, lanes along rows, staged raw in LDS.  A keypoint's output position is its
// level-major rank (the sum of the lower levels' counts + i, :739-765).
// FAST keeps keypoints >= 19 px inside the level (minBorder 16 + the 3-px ring, :619-622), so the
// 18-px test square is always inside; the reflecting slow path only guards other geometries.
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int kDescKpw = 2;                   // keypoints per wave
constexpr int kDescG = 64 / kDescKpw;         // lanes per keypoint
static_assert(kDescG == 32, "k_describe assumes 32 lanes (one per IC disk row / descriptor byte) per keypoint");
__global__ __launch_bounds__(64 * kDescWaves, RGBD_DESC_EU) void k_describe(const uint8_t* __restrict__ pyr,
                                                               const uint8_t* __restrict__ blur,
                                                               const int* __restrict__ sel_count,
                                                               const uint32_t* __restrict__ sel,
                                                               const ExtractCfg* __restrict__ cfgp,
                                                               int* __restrict__ out_count,
                                                               float* __restrict__ out_kps,
                                                               uint8_t* __restrict__ out_desc, int xcd_nblk)
{
    __shared__ __attribute__((aligned(16))) uint8_t sq_all[kDescWaves][kDescKpw][kDescLds];
    const ExtractCfg& cfg = *cfgp;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int h = lane / kDescG, hl = lane % kDescG;   // half, lane in the half
    // xcd_nblk > 0 (1-D grid, B a multiple of 8): every keypoint of frame b runs on XCD b % 8, so a
    // frame's pyramid and blurred pyramid rows are fetched into one L2 (as k_fast)
    int b = blockIdx.y, blk = blockIdx.x;
    if (xcd_nblk > 0) {
        const int j = blockIdx.x >> 3;
        b = (j / xcd_nblk) * 8 + (blockIdx.x & 7);
        blk = j % xcd_nblk;
    }
    // the wave's first slot: wave-uniform (an SGPR), so the slot and level arithmetic below is scalar
    const int s0 = (blk * kDescWaves + __builtin_amdgcn_readfirstlane(w)) * kDescKpw;
    const int spf = cfg.sel_per_frame, nl = cfg.nlevels;
    if (s0 >= spf) return;
    uint8_t* Bl = sq_all[w][h];
    DESC_PROF(0);
    // round trip 1: slot levels, keys and counts (scalar), this lane's disk half-width and tests.  Every
    // load is unconditional (the counts row has kMaxLevels of slack after the last frame, api.cpp; the slot
    // offsets table is INT32_MAX above nlevels), so they all issue before the first wait, and no per-level
    // nlevels test is needed: a slot's level lq < nlevels, so only counts below nlevels are ever summed
    const int* cnt_p = sel_count + b * nl;
    int so[kMaxLevels], cnt[kMaxLevels];
#pragma unroll
    for (int l = 0; l < kMaxLevels; l++) {
        so[l] = cfg.sel_off_tab[l];
        cnt[l] = cnt_p[l];
    }
    uint32_t kvh[kDescKpw];
#pragma unroll
    for (int q = 0; q < kDescKpw; q++) kvh[q] = sel[(size_t)b * spf + (s0 + q < spf ? s0 + q : s0)];
    int lvh[kDescKpw];
#pragma unroll
    for (int q = 0; q < kDescKpw; q++) {
        int l0 = 0;
#pragma unroll
        for (int l = 1; l < kMaxLevels; l++) l0 += s0 + q >= so[l] ? 1 : 0;
        lvh[q] = l0;
        if (s0 + q >= spf) kvh[q] = 0u;
    }
    // this lane's disk row weights (row hl; lane 31 has none and reads row 30), loaded beside the pattern
    const uint4* icu = reinterpret_cast<const uint4*>(cfg.ic_wu[hl < 31 ? hl : 30]);
    const uint4* ic1 = reinterpret_cast<const uint4*>(cfg.ic_w1[hl < 31 ? hl : 30]);
    const uint4 wu0 = icu[0], wu1 = icu[1], w10 = ic1[0], w11 = ic1[1];
    const uint4 pat0 = reinterpret_cast<const uint4*>(c_pattern8.v)[2 * hl];
    const uint4 pat1 = reinterpret_cast<const uint4*>(c_pattern8.v)[2 * hl + 1];
    if (s0 == 0 && lane == 0) {
        int total = 0;
#pragma unroll
        for (int l = 0; l < kMaxLevels; l++) total += l < nl ? cnt[l] : 0;
        out_count[b] = total;
    }
    // per-slot values, wave-uniform (SGPRs: readfirstlane keeps a lane select from turning a level-field
    // read into a per-lane load of cfg.lv[h ? l1 : l0]); the lanes of half h only select between them
    auto sg = [](int v) { return __builtin_amdgcn_readfirstlane(v); };
    auto sgf = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
    int q_on[kDescKpw], q_rank[kDescKpw], q_x[kDescKpw], q_y[kDescKpw];
    float q_scale[kDescKpw], q_size[kDescKpw];
    // every slot's level-dependent loads first (the level offset and count at lq, the LevelCfg fields), so
    // both slots share one dependent scalar round trip; no select chains over the levels
    int soq[kDescKpw], clq[kDescKpw], mbx[kDescKpw], mby[kDescKpw];
    float scq[kDescKpw], szq[kDescKpw];
#pragma unroll
    for (int q = 0; q < kDescKpw; q++) {
        const int lq = lvh[q];   // < nlevels
        const LevelCfg& Lq = cfg.lv[lq];
        soq[q] = cfg.sel_off_tab[lq];
        clq[q] = cnt_p[lq];
        mbx[q] = Lq.minBX;
        mby[q] = Lq.minBY;
        scq[q] = Lq.scale;
        szq[q] = Lq.size;
    }
#pragma unroll
    for (int q = 0; q < kDescKpw; q++) {
        int rb = 0;
#pragma unroll
        for (int l = 0; l < kMaxLevels; l++) rb += l < lvh[q] ? cnt[l] : 0;
        const int iq = s0 + q - soq[q];   // index in the level's selection
        q_on[q] = (s0 + q < spf && iq < clq[q]) ? 1 : 0;
        q_rank[q] = rb + iq;              // level-major output position
        q_x[q] = sg(key_x(kvh[q]) + mbx[q]);
        q_y[q] = sg(key_y(kvh[q]) + mby[q]);
        q_scale[q] = sgf(scq[q]);
        q_size[q] = sgf(szq[q]);
    }
    const int level = h ? lvh[1] : lvh[0];
    const uint32_t kv = h ? kvh[1] : kvh[0];
    const int rank = h ? q_rank[1] : q_rank[0];
    const bool on = (h ? q_on[1] : q_on[0]) != 0;
    DESC_PROF(1);
    if ((q_on[0] | q_on[1]) == 0)
        return;
    // round trip 2: the two slots' rows, staged by whole-wave LDS-DMA loads (global_load_lds_dwordx4,
    // no VGPR staging): per slot q the blurred 37 x 37 square as 37 rows x 48 B (columns from
    // (x - 18) & ~3) and the unblurred IC disk as 31 rows x 48 B (columns from (x - 15) & ~3); lane t of
    // a load takes 16 B (row t / 3, quarter t % 3) to LDS dword 4 t, so each staging is row-major with a
    // 12-dword row stride.  Offsets are 32-bit from the kernel-argument bases (frame pyramids < 4 GiB,
    // api.cpp).  Row windows run <= 30 B past x: into the row padding / next row (64 B buffer slack).
    const int x = h ? q_x[1] : q_x[0], y = h ? q_y[1] : q_y[0];
    const int score = key_s(kv);
    const int xi = x - 15, xb = x - kBlurR;   // first disk column, first square column
    // this lane's (row, 16-B quarter) in the two loads of a staging (the same for every slot)
    int ldR[2], ldC[2];
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int t = 64 * j + lane;
        ldR[j] = t / 3;
        ldC[j] = 16 * (t - 3 * ldR[j]);
    }
#pragma unroll
    for (int q = 0; q < kDescKpw; q++) {
        if (!q_on[q]) continue;
        const LevelCfg& Lq = cfg.lv[lvh[q]];
        const int xq = q_x[q], yq = q_y[q];
        const int lw = sg(Lq.w), lh = sg(Lq.h);
        const uint32_t st = (uint32_t)sg(Lq.stride);
        const uint32_t base = (uint32_t)b * (uint32_t)cfg.frame_pyr_bytes + (uint32_t)sg(Lq.off);
        uint32_t* Sq = reinterpret_cast<uint32_t*>(sq_all[w][q]);
        if (xq >= kBlurR && yq >= kBlurR && xq + kBlurR < lw && yq + kBlurR < lh) {
            const uint32_t sq0 = base + (uint32_t)((xq - kBlurR) & ~3) + (uint32_t)(yq - kBlurR) * st;
#pragma unroll
            for (int j = 0; j < 2; j++) {
                const int t = 64 * j + lane;
                const uint32_t o = __umul24((uint32_t)ldR[j], st) + (uint32_t)ldC[j];
                if (t < 3 * kBlurW)
                    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(blur + (sq0 + o)),
                                                     (void __attribute__((address_space(3)))*)(Sq + 256 * j), 16, 0, 0);
            }
        } else {
            // slow path (other geometries): REFLECT_101 dwords by VGPR stores into the same layout
            const uint8_t* bimg = blur + base;
            for (int t = lane; t < kSqN; t += 64) {
                const int R = t / kSqDw, c = t - R * kSqDw;
                Sq[t] = dword_reflect(bimg, (int)st, lw, lh, yq - kBlurR + R, ((xq - kBlurR) & ~3) + 4 * c);
            }
        }
    }
    // this lane's disk row (row hl of its half's keypoint; lane 31 reads row 30), 9 dwords from column
    // (x - 15) & ~3, loaded beside the LDS-DMA (REFLECT_101 dwords on the slow path)
    uint32_t dreg[9];
    {
        const int rw = hl < 31 ? hl : 30;
        const LevelCfg& L0 = cfg.lv[lvh[0]];
        const LevelCfg& L1 = cfg.lv[lvh[1]];
        const int st0 = sg(L0.stride), st1 = sg(L1.stride), lw0 = sg(L0.w), lw1 = sg(L1.w), lh0 = sg(L0.h), lh1 = sg(L1.h);
        const uint32_t of0 = (uint32_t)sg(L0.off), of1 = (uint32_t)sg(L1.off);
        const int st = h ? st1 : st0, lw = h ? lw1 : lw0, lh = h ? lh1 : lh0;
        const uint32_t base = (uint32_t)b * (uint32_t)cfg.frame_pyr_bytes + (h ? of1 : of0);
        if (on) {
            if (x >= kBlurR && y >= kBlurR && x + kBlurR < lw && y + kBlurR < lh) {
                typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
                const uint32_t off = base + (uint32_t)(y - 15 + rw) * (uint32_t)st + (uint32_t)((x - 15) & ~3);
                const u32x4_a4 a0 = *reinterpret_cast<const u32x4_a4*>(pyr + off);
                const u32x4_a4 a1 = *reinterpret_cast<const u32x4_a4*>(pyr + off + 16);
                dreg[0] = a0.x; dreg[1] = a0.y; dreg[2] = a0.z; dreg[3] = a0.w;
                dreg[4] = a1.x; dreg[5] = a1.y; dreg[6] = a1.z; dreg[7] = a1.w;
                dreg[8] = *reinterpret_cast<const uint32_t*>(pyr + off + 32);
            } else {
#pragma unroll
                for (int k = 0; k < 9; k++) dreg[k] = dword_reflect(pyr + base, st, lw, lh, y - 15 + rw, ((x - 15) & ~3) + 4 * k);
            }
        }
    }
    // output assembly (:753-764)
    const float scale = h ? q_scale[1] : q_scale[0];
    float kx = (float)x, ky = (float)y;
    if (level != 0) {
        kx = kx * scale;
        ky = ky * scale;
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the LDS-DMA writes have landed
    // each wave owns its staging: a wave-level fence orders its LDS writes before the reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    DESC_PROF(2);
    // IC_Angle on the unblurred level (:16-41): integer moments over the radius-15 disk
    // (integer sums: any order).  Per row: sum u * val = sum (u + 16) * val - 16 * sum val, both as
    // v_dot4 over byte windows with the disk's weights.
    int m10 = 0, m01 = 0;
    if (on && hl < 31) {
        const int v = hl - 15;
        uint32_t dr[12];
#pragma unroll
        for (int k = 0; k < 9; k++) dr[k] = dreg[k];
        // dword k's weights (host table from umax): byte i = 1 (w1) or u + 16 = 4k + i + 1 (wu) inside the
        // disk, 0 outside
        const uint32_t WU[8] = {wu0.x, wu0.y, wu0.z, wu0.w, wu1.x, wu1.y, wu1.z, wu1.w};
        const uint32_t W1[8] = {w10.x, w10.y, w10.z, w10.w, w11.x, w11.y, w11.z, w11.w};
        uint32_t su = 0, s1 = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t wv = __builtin_amdgcn_alignbyte(dr[k + 1], dr[k], xi & 3);
            const uint32_t w1 = W1[k], wu = WU[k];
            su = __builtin_amdgcn_udot4(wv, wu, su, false);
            s1 = __builtin_amdgcn_udot4(wv, w1, s1, false);
        }
        m10 = (int)su - 16 * (int)s1;
        m01 = v * (int)s1;
    }
    {   // the sums over each 32-lane half: row scans, rows 0 + 1 into lane 31 and rows 2 + 3 into lane 63
        int r10 = dpp_row_scan(m10), r01 = dpp_row_scan(m01);
        r10 = dpp_add(r10, __builtin_amdgcn_update_dpp(0, r10, 0x142, 0xa, 0xf, false));
        r01 = dpp_add(r01, __builtin_amdgcn_update_dpp(0, r01, 0x142, 0xa, 0xf, false));
        m10 = h ? __builtin_amdgcn_readlane(r10, 63) : __builtin_amdgcn_readlane(r10, 31);
        m01 = h ? __builtin_amdgcn_readlane(r01, 63) : __builtin_amdgcn_readlane(r01, 31);
    }
    DESC_PROF(3);
    const float angle = fast_atan2_deg((float)m01, (float)m10);
    const float rad = angle * (float)(M_PI / 180.f);
    float a, bsin;
    cos_sin_f(rad, &a, &bsin);
    DESC_PROF(4);
    DESC_PROF(5);
    // computeOrbDescriptor (:45-87): lane hl evaluates tests 8 hl .. 8 hl + 7 = descriptor byte hl
    // cvRound (round to nearest even) by the 1.5 * 2^23 magic: the float sum's bits are 0x4B400000 + r for
    // |r| < 2^22, so the square offset (18 + r) * 48 + 18 + c + (xb & 3) is one 24-bit multiply-add of the
    // raw bits (low 24 bits 2^22 + r) with the constant parts folded into kOff (mod 2^32)
    const float kMagic = 12582912.0f;
    const uint32_t kOff = (uint32_t)(kBlurR * 4 * kSqDw + kBlurR + (xb & 3)) - (uint32_t)(4 * kSqDw) * 0x400000u - 0x4B400000u;
    int byte = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        const uint32_t pw = i < 4 ? (i == 0 ? pat0.x : i == 1 ? pat0.y : i == 2 ? pat0.z : pat0.w)
                                  : (i == 4 ? pat1.x : i == 5 ? pat1.y : i == 6 ? pat1.z : pat1.w);
        const float x0 = (float)(int8_t)(pw & 0xFFu), y0 = (float)(int8_t)((pw >> 8) & 0xFFu);
        const float x1 = (float)(int8_t)((pw >> 16) & 0xFFu), y1 = (float)(int8_t)(pw >> 24);
        // the test's two points side by side as packed f32 (v_pk_mul_f32 / v_pk_add_f32: the same IEEE
        // operations, in the same order, as the scalar (x * sin + y * cos) + magic and (x * cos - y * sin) + magic)
        const f32x2 X = {x0, x1}, Y = {y0, y1}, A2 = {a, a}, S2 = {bsin, bsin}, M2 = {kMagic, kMagic};
        const f32x2 R = (X * S2 + Y * A2) + M2, Cc = (X * A2 - Y * S2) + M2;
        const uint32_t r0 = __float_as_uint(R.x), c0 = __float_as_uint(Cc.x);
        const uint32_t r1 = __float_as_uint(R.y), c1 = __float_as_uint(Cc.y);
        const int t0 = Bl[__umul24(r0, 4 * kSqDw) + c0 + kOff];
        const int t1 = Bl[__umul24(r1, 4 * kSqDw) + c1 + kOff];
        byte |= (t0 < t1) << i;
    }
    DESC_PROF(6);
    if (!on) return;
    const size_t o = (size_t)b * cfg.kp_cap + rank;
    out_desc[o * 32 + hl] = (uint8_t)byte;
    if (hl == 0) {
        float* K = out_kps + o * 7;
        K[0] = kx; K[1] = ky; K[2] = h ? q_size[1] : q_size[0]; K[3] = angle; K[4] = (float)score;
        reinterpret_cast<int*>(K)[5] = level;
        reinterpret_cast<int*>(K)[6] = -1;
    }
    DESC_PROF(7);
}

// Frame::undistortKeyPoints + uprojectCamera (Core/Frame.cpp:91-117, 251-281) for every keypoint of
// the batch, one lane per keypoint (the f64 iteration is per-keypoint scalar work: one lane each, not
// one wave each).  kps_un = the keypoint with the undistorted pt; depth is read at the truncated
// DISTORTED pt (:103), the 3D point uses the undistorted one (:110-113), z <= 0 -> (0, 0, 0).
constexpr int kUndThreads = 256;
__global__ __launch_bounds__(kUndThreads) void k_undistort(const uint16_t* __restrict__ depth,
                                                          const int* __restrict__ counts,
                                                          const ExtractCfg* __restrict__ cfgp,
                                                          const float* __restrict__ kps, float* __restrict__ out_kun,
                                                          float* __restrict__ out_xyz)
{
    const ExtractCfg& cfg = *cfgp;
    const int b = blockIdx.y;
    const int i = blockIdx.x * kUndThreads + threadIdx.x;
    if (i >= counts[b]) return;
    const size_t o = (size_t)b * cfg.kp_cap + i;
    const float* K = kps + o * 7;
    const float kx = K[0], ky = K[1];
    const int vi = (int)ky, ui = (int)kx;
    const uint16_t draw = depth ? depth[((size_t)b * cfg.H + vi) * cfg.W + ui] : (uint16_t)0;
    float ux = kx, uy = ky;
    if (cfg.undistort) {
        // cv::undistortPoints(..., P=K): 5 iterations in double (Core/Frame.cpp:270)
        const double fx = cfg.fx, fy = cfg.fy, cx = cfg.cx, cy = cfg.cy;
        const double k0 = cfg.k1, k1 = cfg.k2, k2 = cfg.p1, k3 = cfg.p2, k4 = cfg.k3;
        const double ifx = 1. / fx, ify = 1. / fy;
        double xx = kx, yy = ky;
        xx = (xx - cx) * ifx;
        yy = (yy - cy) * ify;
        const double x0 = xx, y0 = yy;
        for (int j = 0; j < 5; j++) {
            const double r2 = xx * xx + yy * yy;
            const double icdist = 1 / (1 + ((k4 * r2 + k1) * r2 + k0) * r2);
            const double deltaX = 2 * k2 * xx * yy + k3 * (r2 + 2 * xx * xx);
            const double deltaY = k2 * (r2 + 2 * yy * yy) + 2 * k3 * xx * yy;
            xx = (x0 - deltaX) * icdist;
            yy = (y0 - deltaY) * icdist;
        }
        ux = (float)(fx * xx + cx);
        uy = (float)(fy * yy + cy);
    }
    float* KU = out_kun + o * 7;
    KU[0] = ux; KU[1] = uy;
#pragma unroll
    for (int k = 2; k < 7; k++) KU[k] = K[k];
    const float z = depth ? (float)draw * cfg.depth_factor + 0.0f : 0.0f;
    float X = 0.f, Y = 0.f, Z = 0.f;
    if (z > 0) {
        X = (ux - cfg.cx) * z * cfg.invfx;
        Y = (uy - cfg.cy) * z * cfg.invfy;
        Z = z;
    }
    out_xyz[o * 3 + 0] = X;
    out_xyz[o * 3 + 1] = Y;
    out_xyz[o * 3 + 2] = Z;
}

}  // namespace rgbd

// ------------------------------------------------------------------ launchers
#include "launch.h"
namespace rgbd {

hipError_t launch_gray(const uint8_t* bgr, uint8_t* pyr, int W, int H, int frame_pyr_bytes, int B, hipStream_t st)
{
    const long groups = (long)B * ((W * H) >> 4);
    const int blocks = (int)((groups + 255) / 256);
    return dispatch(k_gray, dim3(blocks), dim3(256), 0, st, bgr, pyr, W, H, frame_pyr_bytes, B);
}

hipError_t launch_pyramid(uint8_t* pyr, uint8_t* blur, const uint8_t* bgr, const ResizeY* rsy, const QuadX* qx, const ExtractCfg* d_cfg,
                    int lds_bytes, int B, hipStream_t st)
{
    return dispatch(k_pyramid, dim3(kPyrStrips, B), dim3(kPyrThreads), lds_bytes, st, pyr, blur, bgr, rsy, qx, d_cfg);
}

hipError_t launch_pyr_tail(uint8_t* pyr, const ResizeY* rsy, const QuadX* qx, const ExtractCfg* d_cfg, int B, hipStream_t st)
{
    return dispatch(k_pyr_tail, dim3(B), dim3(kPyrTailThreads), 0, st, pyr, rsy, qx, d_cfg);
}

hipError_t launch_fast(const uint8_t* pyr, const Cell* cells, const FastSeg* segs, int nseg, const ExtractCfg* d_cfg,
                 int* cell_count, uint32_t* cell_slots, int B, hipStream_t st, uint8_t* blur, int blur_threads)
{
    // blur_threads > 0: the level blur's threads (per frame) as 64-lane blocks of the same grid (see k_fast)
    const int nbb = blur_threads > 0 ? (blur_threads + 63) / 64 : 0;
    // B a multiple of 8: 1-D grid of (nbb + nseg) * B single-wave blocks, frame b on XCD b % 8
    if (B % 8 == 0)
        return dispatch(k_fast, dim3((nbb + nseg) * B), dim3(64), 0, st, pyr, cells, segs, d_cfg, nseg, cell_count,
                           cell_slots, 1, blur, nbb);
    else
        return dispatch(k_fast, dim3(nbb + nseg, B), dim3(64), 0, st, pyr, cells, segs, d_cfg, nseg, cell_count,
                           cell_slots, 0, blur, nbb);
}

size_t distribute_lds_bytes(int NC, int SC)
{
    // sortkey 8NC + childcnt x2 32NC + tmp/tmp2 8SC + size/cid A,B 16NC + best 4NC
    // + childIdx 8NC + newIdx 2NC + ord 2NC + bbox A,B 16NC
    return (size_t)NC * 8 + (size_t)NC * 32 + (size_t)SC * 8 + (size_t)NC * 16 + (size_t)NC * 4
           + (size_t)NC * 8 + (size_t)NC * 2 + (size_t)NC * 2 + (size_t)NC * 16 + 64;
}

hipError_t launch_distribute(const int* cell_count, const uint32_t* cell_slots, const ExtractCfg* d_cfg, int node_cap,
                       int scan_cap, int l0, int nlv, int kc, uint32_t* keys, uint16_t* node, int* sel_count,
                       uint32_t* sel, int* err, int B, hipStream_t st)
{
    const bool u8 = node_cap <= 256;
    const size_t lds = distribute_lds_bytes(node_cap, scan_cap) + (size_t)kc * (4 + (u8 ? 1 : 2));
    const int xcd = B % 8 == 0 ? 1 : 0;
    if (u8)
        return dispatch(k_distribute<uint8_t>, dim3(nlv * B), dim3(kDistThreads), lds, st, cell_count, cell_slots,
                           d_cfg, keys, node, sel_count, sel, err, l0, nlv, kc, xcd);
    else
        return dispatch(k_distribute<uint16_t>, dim3(nlv * B), dim3(kDistThreads), lds, st, cell_count, cell_slots,
                           d_cfg, keys, node, sel_count, sel, err, l0, nlv, kc, xcd);
}

#ifdef RGBD_PNP_PROFILE
}  // namespace rgbd
#include <algorithm>
#include <cstdio>
namespace rgbd {
void desc_prof_dump(hipStream_t st)
{
    static long long buf[256][10];
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(buf, HIP_SYMBOL(g_desc_prof), sizeof(buf));
    double acc[8] = {0};
    int n = 0;
    for (int i = 0; i < 256; i++) {
        if (buf[i][7] == 0) continue;
        n++;
        for (int k = 1; k < 8; k++) acc[k] += (double)(buf[i][k] - buf[i][k - 1]);
    }
    if (n)
        fprintf(stderr, "[desc_prof] waves %d mean cycles: scan %.0f loads %.0f angle %.0f trig %.0f fence %.0f tests %.0f tail %.0f\n", n,
                acc[1] / n, acc[2] / n, acc[3] / n, acc[4] / n, acc[5] / n, acc[6] / n, acc[7] / n);
}

void fast_prof_dump(hipStream_t st, int n_seg)
{
    static long long buf[1024][4];
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(buf, HIP_SYMBOL(g_fast_prof), sizeof(buf));
    double a[3] = {0, 0, 0};
    const int n = n_seg < 1024 ? n_seg : 1024;
    for (int i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) a[k] += (double)(buf[i][k + 1] - buf[i][k]);
    fprintf(stderr, "[fast_prof] %d segments, mean cycles: ROI staging %.0f  walk %.0f  minTh rerun + count %.0f\n", n,
            a[0] / n, a[1] / n, a[2] / n);
}

void pyr_prof_dump(hipStream_t st)
{
    static long long buf[8][16];
    static long long sp[2048][2];
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(sp, HIP_SYMBOL(g_pyr_span), sizeof(sp));
    {
        long long t0 = sp[0][0], t1 = sp[0][1];
        double dur = 0;
        int n = 0;
        for (int i = 0; i < 1024; i++) {
            if (sp[i][1] <= sp[i][0]) continue;
            t0 = std::min(t0, sp[i][0]);
            t1 = std::max(t1, sp[i][1]);
            dur += (double)(sp[i][1] - sp[i][0]);
            n++;
        }
        long long late = 0;
        for (int i = 0; i < 1024; i++) late = std::max(late, sp[i][0] - t0);
        fprintf(stderr, "[pyr_span] %d workgroups: span %.1f us, mean duration %.1f us, last start %.1f us, mean concurrency %.0f\n",
                n, (t1 - t0) * 0.01, n ? dur / n * 0.01 : 0.0, late * 0.01, dur / (double)(t1 - t0));
    }
    (void)hipMemcpyFromSymbol(buf, HIP_SYMBOL(g_pyr_prof), sizeof(buf));
    for (int s = 0; s < 8; s++) {
        fprintf(stderr, "[pyr_prof] strip %d (us): stage %.1f levels:", s, (buf[s][1] - buf[s][0]) * 0.01);
        for (int l = 1; l < 8; l++) fprintf(stderr, " %.1f", (buf[s][1 + l] - buf[s][l]) * 0.01);
        fprintf(stderr, " | total %.1f\n", (buf[s][8] - buf[s][0]) * 0.01);
    }
}

void dist_prof_dump(hipStream_t st)
{
    static long long buf[4][64];
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(buf, HIP_SYMBOL(g_dist_prof), sizeof(buf));
    for (int l = 0; l < 4; l++) {
        const long long* p = buf[l];
        const int rounds = (int)p[43];
        fprintf(stderr, "[dist_prof] level %d n=%lld rounds=%d phase=%lld gather %lld roots %lld rounds:", l, p[44], rounds,
                p[45], p[1] - p[0], p[2] - p[1]);
        for (int r = 1; r <= rounds && r < 18; r++) fprintf(stderr, " %lld+%lld", p[20 + r] - p[1 + r], p[2 + r] - p[20 + r]);
        fprintf(stderr, " | best %lld total %lld wall %.1f us\n", p[42] - p[40], p[42] - p[0], (p[47] - p[46]) * 0.01);
    }
}
#endif

hipError_t launch_describe(const uint8_t* pyr, const uint8_t* blur, const int* sel_count, size_t selc_elems, int nlevels, const uint32_t* sel,
                     const ExtractCfg* d_cfg, int kp_cap, int* out_count, float* kps, uint8_t* desc, int B,
                     hipStream_t st)
{
    if (nlevels < 1 || nlevels > kMaxLevels || selc_elems < sel_count_elems(B, nlevels)) return hipErrorInvalidValue;
    // kDescKpw selection slots per wave (sel_per_frame <= kp_cap slots per frame)
    const int nblk = (kp_cap + kDescWaves * kDescKpw - 1) / (kDescWaves * kDescKpw);
    if (B % 8 == 0)
        return dispatch(k_describe, dim3(nblk * B), dim3(64 * kDescWaves), 0, st, pyr, blur, sel_count, sel, d_cfg,
                           out_count, kps, desc, nblk);
    else
        return dispatch(k_describe, dim3(nblk, B), dim3(64 * kDescWaves), 0, st, pyr, blur, sel_count, sel, d_cfg,
                           out_count, kps, desc, 0);
}

hipError_t launch_undistort(const uint16_t* depth, const int* counts, const ExtractCfg* d_cfg, int kp_cap, const float* kps,
                      float* kun, float* xyz, int B, hipStream_t st)
{
    return dispatch(k_undistort, dim3((kp_cap + kUndThreads - 1) / kUndThreads, B), dim3(kUndThreads), 0, st,
                       depth, counts, d_cfg, kps, kun, xyz);
}

}  // namespace rgbd

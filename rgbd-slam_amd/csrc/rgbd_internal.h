// rgbd_internal.h -- configuration blocks shared by the host runtime and the gfx950 kernels.
//
// All geometry is computed once on the host (geometry.cpp) with the reference's own
// float/double semantics and passed to kernels by value (kernel-argument SGPRs), so
// the kernels never re-derive a float-rounded size or budget.
#pragma once
#include <stdint.h>

namespace rgbd {

constexpr int kMaxLevels = 12;
// k_describe reads kMaxLevels selection counts from each frame's row of nlevels unconditionally (and relies on
// ExtractCfg::sel_off_tab being INT32_MAX above nlevels, so no count above nlevels is ever summed): the counts
// buffer carries kMaxLevels entries of slack after the last frame's row.  launch_describe checks the size.
inline size_t sel_count_elems(int max_batch, int nlevels) { return (size_t)max_batch * nlevels + kMaxLevels; }
constexpr int kCellStride = 48;
#define RGBD_PYR_THREADS 512
constexpr int kPyrThreads = RGBD_PYR_THREADS;  // k_pyramid: threads per strip workgroup
#ifndef RGBD_PYR_STRIPS
#define RGBD_PYR_STRIPS 16
#endif
constexpr int kPyrStrips = RGBD_PYR_STRIPS;  // k_pyramid: horizontal strips per frame (one workgroup each)
#define RGBD_BLUR_TH 48   // r04 (level blur of levels 1-7 in the k_fast grid): 16 / 32 / 48 rows -> 230.5k / 232.6k / 233.3k frames/s (profiles/r04_ab_blur_rows)
constexpr int kBlurTH = RGBD_BLUR_TH;        // level blur: rows per strip (one thread per 4-px column quad)
#define RGBD_PB_ROWS 7   // (sweep r03: 5 1.34 ms, 6 1.29, 7 1.21, 8 1.24, 10 1.32, 13 1.39, 16 1.38 k_pyramid)
constexpr int kPbRows = RGBD_PB_ROWS;        // k_pyramid's fused level blur: output rows per (quad, segment) item
#define RGBD_PB_LEVELS 1   // (r03 with kPbRows 7: 2 -> 202-203k frames/s, k_pyramid 1.07 ms; 3 -> 200k, 1.20 ms; 4 -> 182k;
                           //  r04: 0 / 1 / 2 -> 232.2k / 232.7k / 230.8k, k_pyramid 0.82 / 0.95 / 1.07 ms, k_fast 1.83 / 1.69 / 1.60 ms)
constexpr int kPbLevels = RGBD_PB_LEVELS;    // levels 0 .. kPbLevels-1 blurred inside k_pyramid, the rest inside k_fast's grid
#ifndef RGBD_PYR_STRIP_LEVELS
#define RGBD_PYR_STRIP_LEVELS 4
#endif
// levels 0 .. kPyrStripLevels-1 are computed by k_pyramid's strips, the smaller ones after them by
// k_pyr_tail (one workgroup per frame; r06 A/B: 3 / 4 / 5 / all strip levels -> 228.4k / 229.6k / 226k / 225.7k
// frames/s, profiles/r06_ab/ab25-ab26)
constexpr int kPyrStripLevels = RGBD_PYR_STRIP_LEVELS;
#ifndef RGBD_PYR_TAIL_THREADS
#define RGBD_PYR_TAIL_THREADS 256
#endif
constexpr int kPyrTailThreads = RGBD_PYR_TAIL_THREADS;   // k_pyr_tail: threads per frame workgroup (256 / 512 alike, ab25)
static_assert(kPyrStripLevels > kPbLevels, "the strips must hold every level blurred inside k_pyramid");

struct LevelCfg {
    int32_t w, h, stride;      // level image, row stride in the pyramid buffer
    int32_t off;               // byte offset of the level inside one frame's pyramid
    int32_t minBX, maxBX, minBY, maxBY;   // ComputeKeyPointsOctTree borders (:619-622)
    int32_t cell_begin, cell_count;       // this level's FAST cells in the cell table
    int32_t N;                 // mnFeaturesPerLevel[level]
    int32_t nIni;              // DistributeOctTree root count (:420)
    float hX;                  // root width (:422)
    float scale;               // mvScaleFactor[level]
    float size;                // (float)(int)(PATCH_SIZE * scale) (:680)
    int32_t key_off;           // offset of this level's candidate region in a frame's key scratch
    int32_t key_cap;           // capacity of that region (sum of its cells' slot capacity)
    int32_t sel_off;           // offset of this level's selected-keypoint slots (per frame)
    int32_t rsx_off, rsy_off;  // resize tables (level l from l-1): x entries / y entries
    int32_t rs_xmax;           // first dx whose tap sx+1 falls outside the source row
    int32_t rs_simd;           // VResizeLinearVec_32s8u coverage [0, rs_simd)
    int32_t qx_off;            // this level's QuadX entries (k_pyramid's per-quad horizontal taps)
    double rs_scale_x, rs_scale_y;   // 1 / ((double)dst / src) of cv::resize (level l from l-1)
};

struct ExtractCfg {
    int32_t W, H, nlevels;
    int32_t frame_pyr_bytes;   // one frame's pyramid (all levels, padded rows)
    int32_t n_cells;           // FAST cells over all levels
    int32_t cell_cap;          // max NMS survivors of any cell (king-graph bound)
    int32_t dist_kc;           // quadtree: candidates per level whose round state fits in LDS (else HBM)
    int32_t keys_per_frame;    // key scratch entries per frame
    int32_t sel_per_frame;     // selected-keypoint slots per frame (sum of N+3)
    int32_t node_cap;          // quadtree node capacity (power of two)
    int32_t scan_cap;          // LDS scan scratch: max(node_cap, cells of any level) + 1
    int32_t kp_cap;            // output keypoints per frame
    int32_t ini_th, min_th;
    int32_t umax[16];
    // IC_Angle row weights for v_dot4 (row v + 15, dword k covers columns u = 4k - 15 .. 4k - 12):
    // ic_wu byte = u + 16 inside the disk (|u| <= umax[|v|]) else 0; ic_w1 byte = 1 inside else 0
    alignas(16) uint32_t ic_wu[31][8];
    alignas(16) uint32_t ic_w1[31][8];
    // camera
    float fx, fy, cx, cy, invfx, invfy;
    float k1, k2, p1, p2, k3;
    float depth_factor;
    int32_t undistort;
    // k_pyramid: rows [strip_r0, strip_r1) of each level computed (level > 0) or staged (level 0) by
    // strip s; a strip's rows include the halo its next level reads, so strips never exchange data
    int16_t strip_r0[kPyrStrips][kMaxLevels], strip_r1[kPyrStrips][kMaxLevels];
    int32_t pyr_top;           // levels [0, pyr_top) in the strips (min(nlevels, kPyrStripLevels)), the rest by k_pyr_tail
    int32_t pyr_lds;           // bytes of LDS per strip workgroup: even levels at 0, odd levels at pyr_lds_b
    int32_t pyr_lds_b;
    int32_t pyr_rsy_lds;       // bytes of the strip's resize row entries, staged after the level buffers
    // level blur (blur_thread): inner quads (x = 4 .. 4 * blur_tx[l]) of level l are threads [blur_t0[l], blur_t0[l + 1]),
    // strip-major; its edge quads (x = 0, then blur_ex[l] - 1 quads from 4 * (blur_tx[l] + 1)) are
    // threads blur_t0[kMaxLevels] + [blur_e0[l], blur_e0[l + 1])
    int32_t blur_t0[kMaxLevels + 1];
    int32_t blur_tx[kMaxLevels];
    int32_t blur_e0[kMaxLevels + 1];
    int32_t blur_ex[kMaxLevels];
    // k_pyramid's fused blur of the lowest levels (l < kPbLevels, multi-level pyramids): strip s blurs rows
    // [pb_r0, pb_r1) of level l (a partition of the level chosen inside the strips' overlaps, so the rows
    // +- 3 it reads are mostly computed for the next level anyway) in pb_seg[l] segments of kPbRows rows;
    // items = (segment, inner quad) then (segment, edge quad) with the quad sets of blur_tx / blur_ex.
    // blur_thread (k_fast's leading blocks) covers the other levels (its ranges are empty for the fused ones).
    int16_t pb_r0[kPyrStrips][kMaxLevels], pb_r1[kPyrStrips][kMaxLevels];
    int32_t pb_seg[kMaxLevels];
    // k_describe: lv[l].sel_off for l < nlevels, INT32_MAX above (one contiguous scalar load; a slot's level is
    // the count of levels >= 1 whose first slot it has reached, with no nlevels test)
    int32_t sel_off_tab[kMaxLevels];
    LevelCfg lv[kMaxLevels];
};

struct Cell {                  // one FAST ROI (rowRange/colRange of :655-660), level coordinates
    int16_t level, x0, y0, x1, y1, pad;
};

struct FastSeg {               // k_fast: up to 64 / lpc consecutive cells of one cell row of one level
    int32_t cell0;             // first cell (index into the cell table)
    int16_t ncell;             // cells in the segment
    int16_t lpc;               // lanes per cell: 16 (interior <= 32 px wide, one DPP row) or the level's widest
                               // cell's pixel pairs, 17 .. 32 (so 3 cells of 17-21 pairs share a wave)
};

struct ResizeX { int16_t sx, a0, a1, pad; };   // xofs + ialpha
// k_pyramid's horizontal resize taps of one output quad (4 px): the quad's taps lie in the 12-byte source
// window wb .. wb + 11; pixel i's two taps are v_perm(sel[i]) of window dwords (pi_i, pi_i + 1) into a
// zero-extended u16 pair, dotted with wt[i] = (16 a0 | 16 a1 << 16) (weights x 16: the vertical pass
// then takes (r >> 4) << 8 as one mask); wbpi = wb | pi_bits << 16; simd bit i: pixel i in the SSE2
// vertical range [0, rs_simd)
struct QuadX { uint32_t wbpi; uint32_t sel[4]; uint32_t wt[4]; uint32_t simd; uint32_t pad[2]; };
struct ResizeY { int16_t sy0, sy1, b0, b1; };  // clipped source rows + ibeta

// packed candidate / selected keypoint: x (11 bits) | y (11 bits) | score (8 bits), coords
// relative to (minBorderX, minBorderY) of the level
__host__ __device__ inline uint32_t pack_key(int x, int y, int s) { return (uint32_t)x | ((uint32_t)y << 11) | ((uint32_t)s << 22); }
__host__ __device__ inline int key_x(uint32_t k) { return (int)(k & 2047u); }
__host__ __device__ inline int key_y(uint32_t k) { return (int)((k >> 11) & 2047u); }
__host__ __device__ inline int key_s(uint32_t k) { return (int)(k >> 22); }

}  // namespace rgbd

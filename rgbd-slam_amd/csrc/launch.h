// launch.h -- host-side launchers of the gfx950 kernels (defined next to each kernel).
#pragma once
#include <hip/hip_runtime.h>

#include "rgbd_internal.h"

namespace rgbd {

hipError_t launch_gray(const uint8_t* bgr, uint8_t* pyr, int W, int H, int frame_pyr_bytes, int B, hipStream_t st);
hipError_t launch_pyramid(uint8_t* pyr, uint8_t* blur, const uint8_t* bgr, const ResizeY* rsy, const QuadX* qx, const ExtractCfg* d_cfg,
                    int lds_bytes, int B, hipStream_t st);
hipError_t launch_pyr_tail(uint8_t* pyr, const ResizeY* rsy, const QuadX* qx, const ExtractCfg* d_cfg, int B, hipStream_t st);
hipError_t launch_fast(const uint8_t* pyr, const Cell* cells, const FastSeg* segs, int nseg, const ExtractCfg* d_cfg,
                 int* cell_count, uint32_t* cell_slots, int B, hipStream_t st, uint8_t* blur = nullptr,
                 int blur_threads = 0);
// the quadtrees of levels [l0, l0 + nlv) of every frame; kc = LDS-resident keys per level
hipError_t launch_distribute(const int* cell_count, const uint32_t* cell_slots, const ExtractCfg* d_cfg, int node_cap,
                       int scan_cap, int l0, int nlv, int kc, uint32_t* keys, uint16_t* node, int* sel_count,
                       uint32_t* sel, int* err, int B, hipStream_t st);
size_t distribute_lds_bytes(int node_cap, int scan_cap);
hipError_t launch_undistort(const uint16_t* depth, const int* counts, const ExtractCfg* d_cfg, int kp_cap, const float* kps,
                      float* kun, float* xyz, int B, hipStream_t st);
// sel_count holds selc_elems counts: at least sel_count_elems(B, nlevels) (rgbd_internal.h), else hipErrorInvalidValue
hipError_t launch_describe(const uint8_t* pyr, const uint8_t* blur, const int* sel_count, size_t selc_elems, int nlevels, const uint32_t* sel,
                     const ExtractCfg* d_cfg, int kp_cap, int* out_count, float* kps, uint8_t* desc, int B,
                     hipStream_t st);
// k_fast's 16-lane emission rank on its own (rgbd_debug_fast_rank16)
hipError_t launch_debug_rank16(const uint8_t* flags, int rows, uint32_t* slots, uint32_t* counts, hipStream_t st);
// knn-2 of pairs (qf[p], tf[p]) on the matrix cores (k_knn2m)
hipError_t launch_knn2(const uint8_t* desc, const int* counts, const int* qf, const int* tf, int kp_cap, int max_q,
                 int4* out, int npairs, hipStream_t st);

#ifdef RGBD_PNP_PROFILE
void fast_prof_dump(hipStream_t st, int n_cells);   // profiling builds: k_fast stage cycles (frame 0)
void pyr_prof_dump(hipStream_t st);    // profiling builds: k_pyramid stage wall times (frame 0, strips 0..7)
void dist_prof_dump(hipStream_t st);   // profiling builds: k_distribute stage cycles (levels 0..3, frame 0)
void desc_prof_dump(hipStream_t st);   // profiling builds: k_describe stage cycles (frame 0, 256 keypoints)
#endif

}  // namespace rgbd

// ransac_dev.h -- RansacSE3 hypothesis-kernel interface (host <-> device).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rgbd {

constexpr int kRansacMaxM = 2304;   // LDS-resident matches per RansacSE3 call (<= 147 KB)

struct RansacDev {
    int32_t M;          // used matches (sorted by distance)
    int32_t H;          // hypotheses (the identity slot is block H)
    int32_t SS;         // sample size (stride of the sample table)
    int32_t MWcap;      // mask words per hypothesis in masks_out
    uint32_t minTh;     // mMinInlierTh
    float maxMahal;     // mMaxMahalanobisDistance
    double C;           // depthCovariance sticky value
    double rcx, rcy;    // raster_cov_x / raster_cov_y (Solver/SolverSE3.cpp:218-225)
};

struct HypOut {
    float T[16];
    double err;
    int32_t n;
    int32_t pad;
};

size_t ransac_lds_bytes(int M);
hipError_t launch_ransac_hyp(const float* pts, const int* samples, const int* scount, const RansacDev& prm, HypOut* out,
                       uint32_t* masks, hipStream_t st);

}  // namespace rgbd

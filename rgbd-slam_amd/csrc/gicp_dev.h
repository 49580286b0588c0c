// gicp_dev.h -- GICP kernels interface (host <-> device).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rgbd {

constexpr int kGicpMaxM = 2048;   // points per cloud (LDS-resident target / transformed source)

struct GicpDevPrm {
    int32_t max_iterations, k, gn_iterations, pad;
    double thr;          // max_corr_dist^2 (double)
    double trans_eps, rot_eps, gicp_eps;
};

struct GicpOut {
    float T[16];         // final_transformation_ (identity unless converged)
    int32_t converged, iters, n_corr, pad;
};

// covariances of both clouds (cov scratch: 2 M x 9 doubles), then the outer iterations; writes *out
hipError_t launch_gicp(const float* src, const float* tgt, int M, const float* guess, const GicpDevPrm& prm, double* cov,
                 GicpOut* out, double* Mi, hipStream_t st);   // Mi: M x 9 doubles of scratch

}  // namespace rgbd

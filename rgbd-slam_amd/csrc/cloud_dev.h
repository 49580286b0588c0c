// cloud_dev.h -- keyframe dense cloud: the point type and the per-launch configuration (cloud.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rgbd {

struct CloudPoint {            // pcl::PointXYZRGB payload: xyz + the packed rgb word (bytes b, g, r, 0)
    float x, y, z;
    uint8_t b, g, r, pad;
};

struct CloudCfg {
    int W, H, res, rows, cols;    // image, sample stride, sample grid
    int cap;                      // points per keyframe (rows * cols)
    int sort_cap;                 // power of two >= cap (LDS keys of k_cloud_voxel)
    float cx, cy, invfx, invfy, depth_factor;
    float zmin, zmax, inv_leaf;
    int sor_k;
    double sor_std;
};

// depth: u16 raw depth (z = d * depth_factor, Frame.cpp:48), or, when depthf is set, Frame::mImDepth itself (f32)
hipError_t launch_cloud(const uint8_t* bgr, const uint16_t* depth, const float* depthf, const int* frames, int nkf,
                  const CloudCfg& cfg, CloudPoint* pts, CloudPoint* vox, int* nvox, float* dist, CloudPoint* out, int* nout, hipStream_t st);

}  // namespace rgbd

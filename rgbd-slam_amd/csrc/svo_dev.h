// svo_dev.h -- the SVO detector + BRIEF descriptor (the reference's default Extractor(SVO, BRIEF, NORMAL),
// main.cpp:31): per-launch configuration and launchers (svo.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace rgbd {

constexpr int kSvoMaxLevels = 8;       // 128 x 128 pyramid tiles: levels 0..7
constexpr int kSvoSelThreads = 1024;   // k_svo_select: one workgroup per frame
constexpr int kSvoSelMaxE = 12;        // candidates per thread in k_svo_select (cells <= 12288)

struct SvoTile { int16_t level, x0, y0, pad; };   // k_svo_detect: a 64 x 32 tile of one level

struct SvoCfg {
    int32_t W, H, nlevels;
    int32_t cell, barrier;          // SVOextractor(nlevels, 5, 20): grid cell size, FAST-10 barrier
    int32_t gcols, grows, ncells;   // ceil(W / cell) x ceil(H / cell)
    int32_t lw[kSvoMaxLevels], lh[kSvoMaxLevels], loff[kSvoMaxLevels];   // halfSample levels, tight
    int32_t frame_bytes;            // one frame's pyramid (all levels)
    int32_t nfeatures;              // retainBest(nfeatures), Features/Extractor.cpp:56-57
    int32_t kp_cap;                 // output keypoints per frame
    int32_t border;                 // BRIEF runByImageBorder: PATCH_SIZE / 2 + KERNEL_SIZE / 2 = 28
};

hipError_t launch_svo_pyramid(const uint8_t* bgr, uint8_t* pyr, uint16_t* box, const SvoCfg& cfg, int B, hipStream_t st);
hipError_t launch_svo_detect(const uint8_t* pyr, const SvoTile* tiles, int ntiles, const SvoCfg& cfg,
                       unsigned long long* cell_keys, int B, hipStream_t st);
size_t svo_select_lds_bytes(const SvoCfg& cfg);
hipError_t launch_svo_select(unsigned long long* cell_keys, const SvoCfg& cfg, uint2* cand, int* ncand, int* counts,
                       float* kps, int* err, int B, hipStream_t st);
hipError_t launch_svo_brief(const uint16_t* box, const int* counts, const float* kps, const uint32_t* pattern,
                      const SvoCfg& cfg, uint8_t* desc, int B, hipStream_t st);
// the device std::nth_element + std::partition of k_svo_select on a given response array (parity tests)
hipError_t launch_svo_retain_test(const float* resp, int n, int nkeep, int depth_limit, int* order, int* m, hipStream_t st);

#ifdef RGBD_PNP_PROFILE
void svo_prof_dump(hipStream_t st);   // profiling builds: k_svo_select stage stamps (frame 0)
#endif

}  // namespace rgbd

// lanes_host.h -- the device-resident RansacSE3 tracking chain (lanes_host.cpp) as the solver sees it.
#pragma once
#include <vector>

#include "context.h"
#include "lanes_dev.h"

namespace rgbd {

struct LaneSpec {
    int start;   // the lane's first frame (its reference; flags clear unless the caller's flags_f0 / f1)
    int end;     // the lane's last frame
    int first;   // the first frame the lane tracks (start + 1, or start + 2 for a continuing chunk)
};

// L lanes of the extracted batch (rgbd_extract_batch before): per-pair results in out[b] for every tracked b;
// rngs / stickies (one per lane) advance as the reference's process globals would over the lane's chain.
// flags_f0 / f1 (optional): outlier flags of frames 0 / 1 (a continuing chunk); flags_out2 / 1 (optional):
// the flags of frames B - 2 / B - 1 after the chain.
rgbd_status lanes_track(rgbd_ctx* c, int B, float nnratio, const rgbd_ransac_params& prm, const LaneSpec* spec, int L,
                        rgbd_rng* rngs, rgbd_sticky* stickies, const uint8_t* flags_f0, const uint8_t* flags_f1,
                        std::vector<PairOut>& out, uint8_t* flags_out2, uint8_t* flags_out1);
rgbd_status lanes_sort_test(rgbd_ctx* c, const float* dist, int n, int depth_limit, int* order);
void lanes_free(rgbd_ctx* c);

}  // namespace rgbd

// solver.cpp -- RansacSE3 / tracking host logic (placeholder until the GPU hypothesis kernel lands).
#include <hip/hip_runtime.h>
#include "context.h"

namespace rgbd { void ransac_free(rgbd_ctx*) {} }

extern "C" {
void rgbd_rng_seed(rgbd_rng* st, uint32_t seed)
{
    if (seed == 0) seed = 1;
    st->state[0] = (int32_t)seed;
    int32_t word = (int32_t)seed;
    for (int i = 1; i < 31; ++i) {
        long hi = word / 127773, lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        st->state[i] = word;
    }
    st->f = 3;
    st->r = 0;
    for (int k = 0; k < 310; k++) {
        uint32_t val = (uint32_t)st->state[st->f] + (uint32_t)st->state[st->r];
        st->state[st->f] = (int32_t)val;
        if (++st->f >= 31) { st->f = 0; ++st->r; }
        else if (++st->r >= 31) st->r = 0;
    }
}
rgbd_status rgbd_ransac_se3(rgbd_ctx* c, const float*, int32_t, const float*, int32_t, const rgbd_dmatch*, int32_t,
                            const rgbd_ransac_params*, rgbd_rng*, rgbd_sticky*, int32_t, uint8_t*, float*, rgbd_dmatch*,
                            int32_t*, float*, int32_t*)
{
    return rgbd::fail(c, RGBD_ERR_UNSUPPORTED, "ransac not built yet");
}
rgbd_status rgbd_track_batch(rgbd_ctx* c, const void*, const void*, int32_t, float, const rgbd_ransac_params*,
                             rgbd_rng*, rgbd_sticky*, float*, int32_t*, int32_t*)
{
    return rgbd::fail(c, RGBD_ERR_UNSUPPORTED, "tracking not built yet");
}
}

// context.h -- the rgbd_ctx behind the C ABI (host runtime, not exported).
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <string>
#include <vector>

#include "../../include/rgbd_hip.h"
#include "rgbd_internal.h"

struct rgbd_ctx {
    int device = 0;
    int W = 0, H = 0, maxB = 0;
    rgbd_orb_params orb{};
    rgbd_camera cam{};
    rgbd::ExtractCfg cfg{};              // host copy
    std::vector<rgbd::Cell> cells;
    std::vector<rgbd::FastSeg> segs;     // k_fast segments (consecutive cells of one cell row)
    std::string err;

    hipStream_t stream = nullptr;        // launch stream (own or external)
    hipStream_t own_stream = nullptr;
    hipStream_t match_stream = nullptr;  // pipelined API: knn-2 + gather of a step beside the next extraction
    hipStream_t solve_stream = nullptr;  // high-priority stream of the pipelined PnPRansac solves: the
                                         // latency-bound solve of step i runs beside step i+1's extraction
    bool serial = false;                 // RGBD_SERIAL=1: match / solve streams are the launch stream
                                         // (kernels never overlap: attributable PMC counters)

    // device workspace
    rgbd::ExtractCfg* d_cfg = nullptr;
    rgbd::Cell* d_cells = nullptr;
    rgbd::FastSeg* d_segs = nullptr;
    rgbd::ResizeX* d_rsx = nullptr;
    rgbd::ResizeY* d_rsy = nullptr;
    rgbd::QuadX* d_qx = nullptr;
    uint8_t* d_pyr = nullptr;
    uint8_t* d_blur = nullptr;           // blurred pyramid, same layout as d_pyr
    int* d_cellc = nullptr;
    uint32_t* d_slots = nullptr;
    uint32_t* d_keys = nullptr;
    uint16_t* d_node = nullptr;
    int* d_selc = nullptr;
    uint32_t* d_sel = nullptr;
    int* d_count = nullptr;
    float* d_kps = nullptr;
    float* d_kun = nullptr;
    uint8_t* d_desc = nullptr;
    float* d_xyz = nullptr;
    int* d_err = nullptr;
    uint8_t* d_in_bgr = nullptr;         // single-frame staging (host-buffer entry points)
    uint16_t* d_in_depth = nullptr;
    int4* d_knn = nullptr;               // [maxB][kp_cap]
    int* d_pairs = nullptr;              // qf[maxB], tf[maxB]
    // host-array knn staging
    uint8_t* d_mdesc = nullptr;
    int* d_mcount = nullptr;
    int4* d_mknn = nullptr;
    int mcap = 0;
    int last_B = 0;
    hipEvent_t extract_done = nullptr;   // recorded after every extraction on the stream it ran on
    hipStream_t extract_stream = nullptr;

    // ransac workspace (solver.cpp), PnPRansac workspace (pnp_host.cpp)
    void* ransac = nullptr;
    void* pnp = nullptr;
    void* pnp_pipe = nullptr;            // two PnPRansac workspaces of the submit / collect tracking API
    int pnp_chunk = 0, pnp_chunk2 = 0;   // PnPRansac device chunks, adapted per solve (pnp_host.cpp)
    void* gicp = nullptr;                // GICP workspace (gicp_host.cpp)
    void* lanes = nullptr;               // device-resident RansacSE3 tracking chain workspace (lanes_host.cpp)
    void* cloud = nullptr;               // keyframe cloud workspace (cloud_host.cpp)
    void* svo = nullptr;                 // SVO + BRIEF extractor (svo_host.cpp); null: ORBextractor
    rgbd_gicp_params track_gicp{10, 20, 0.07, 1e-9, 2e-3, 1e-3, 4, 1};

    // timing
    bool timing = false;
    std::string timing_only;             // non-empty: only launches of this kernel are timed
    struct TEntry { std::string name; double ms = 0; long launches = 0; };
    std::vector<TEntry> tentries;
    struct Pending { int idx; hipEvent_t a, b; hipStream_t st; bool ended; };   // ended: b was recorded
    std::vector<Pending> pending;
    std::vector<hipEvent_t> event_pool;
};

namespace rgbd {
// called by an extraction at its launch points (launch-stream order): 0 before FAST, 1 after FAST,
// 2 after the quadtree (the pipelined PnP solves use point 1; SVO extractions call points 1 and 2)
using ExtractHook = std::function<rgbd_status(int at)>;
rgbd_status extract_batch(rgbd_ctx* c, const void* d_bgr, const void* d_depth, int B, const ExtractHook* after_fast);
// records the elapsed time of the launches between begin and end under `name`
int timer_begin(rgbd_ctx* c, const char* name, hipStream_t st = nullptr);   // nullptr: the context stream
void timer_end(rgbd_ctx* c, int tok);
void timer_flush(rgbd_ctx* c);
rgbd_status fail(rgbd_ctx* c, rgbd_status code, const std::string& msg);
rgbd_status check_hip(rgbd_ctx* c, hipError_t e, const char* what);
// c->stream waits for the last extraction when that ran on another stream (api.cpp)
rgbd_status order_after_extraction(rgbd_ctx* c);
// a launcher's status (dispatch.h: geometry, LDS opt-in and launch checked) as the entry point's result
#define RGBD_TRY(c, call, what)                                                            \
    do {                                                                                   \
        const rgbd_status rgbd_try_s_ = check_hip((c), (call), "launch of k_" what);        \
        if (rgbd_try_s_) return rgbd_try_s_;                                               \
    } while (0)
void ransac_free(rgbd_ctx* c);   // solver.cpp
void pnp_free(rgbd_ctx* c);      // pnp_host.cpp
void gicp_free(rgbd_ctx* c);     // gicp_host.cpp
void cloud_free(rgbd_ctx* c);    // cloud_host.cpp
// svo_host.cpp: the Extractor(SVO, BRIEF, NORMAL) front end of an rgbd_create_svo context
rgbd_status svo_configure(rgbd_ctx* c, const rgbd_svo_params& p);   // before the output allocations
rgbd_status svo_alloc(rgbd_ctx* c);
void svo_free(rgbd_ctx* c);
rgbd_status svo_run_extract(rgbd_ctx* c, const uint8_t* d_bgr, const uint16_t* d_depth, int B, bool from_gray,
                            const ExtractHook* after_fast);
uint8_t* svo_gray_level(rgbd_ctx* c);   // level 0 of the SVO pyramid (frame 0): the gray upload target
}  // namespace rgbd

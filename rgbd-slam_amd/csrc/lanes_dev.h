// lanes_dev.h -- the device-resident Tracking::visualOdometry chain over L independent lanes (host <-> device).
//
// A lane is one contiguous run of frames of a device-resident batch tracked as its own chain
// (System/Tracking.cpp:121-163): pair (b-1 -> b) for b in (start, end].  Round r advances every lane by one
// pair; all of a round's work is on the device, with no host wait inside it:
//   k_lane_match       Matcher::match (Features/Matcher.cpp:106-139) on the knn-2 rows, RansacSE3's outlier
//                      marking (Solver/SolverSE3.cpp:38-42), std::sort by distance (:52, libstdc++'s introsort
//                      order reproduced), the gathered points, the sticky depth covariance (:282-287) and the
//                      glibc-rand samples of every hypothesis (sampleMatches :135-159) with the rand() count after each
//   k_ransac_hyp_lanes every hypothesis' refinement chain (:58-86), (lane, hypothesis) per workgroup
//   k_lane_replay      the sequential accept / n += 10 / break replay (:88-102), identity fallback (:105-117),
//                      inlier flags (:119-122), the RNG advanced by the hypotheses drawn; then the second
//                      reference (Tracking.cpp:134-143, the lane's next round) or the GICP staging (:145-151),
//                      the pair's result and the next frame (three phases: hypotheses [0, e0), [e0, e1), [e1, H));
//                      with few lanes (LaneCfg::fuse) the same replay runs inside k_ransac_hyp_lanes, in the last
//                      of the lane's active workgroups to finish (an agent-scope release / atomic count / acquire;
//                      idle workgroups leave at once), so a round is 3-4 launches instead of 7-8
// then, once per call, Gicp::compute (Solver/Gicp.cpp:21-66) of every pair whose rmse >= 0.8: its problem
// (inlier clouds, guess) was staged in the pair's slot; nothing the chain reads later depends on GICP
// (flags, RNG and sticky covariance are RansacSE3's), so all problems are solved in one batched pass
//   k_gicp_list, k_gicp_cov_pairs, k_gicp_align_pairs, k_gicp_post
// Poses are pure outputs of the chain (no RANSAC / GICP input depends on them), so the host composes them
// from the per-pair results afterwards: T pose(ref) or recover(), and Tracking::track's keyframe bookkeeping.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gicp_dev.h"
#include "ransac_dev.h"

namespace rgbd {

constexpr int kLaneThreads = 512;   // k_lane_match workgroup (its sort: one wave per segment of a level); r06 same-box A/B: 256 / 512 gave se3_chain_one 117.8 / 114.6 us, cfg3 chain 181.2 / 171.6 us per pair
constexpr int kLaneSnap = 33;       // glibc random_r TYPE_3: 31 state words + the two indices
constexpr int kLaneSegs = 256;      // introsort segments per level (n / 17 + 1 <= 136 for n <= 2304)

struct LaneCtl {
    int32_t start, end;        // the lane's frames [start, end]; pairs (b-1, b) for b in (first, end]
    int32_t b;                 // frame tracked in this round (> end: the lane is done)
    int32_t ref;               // reference frame of the running attempt
    int32_t run;               // 1: the running attempt's RansacSE3 evaluates hypotheses for this lane
    int32_t early;             // the running attempt returned before sorting (m < mMinInlierTh)
    int32_t m;                 // matches of the running attempt
    int32_t H;                 // hypotheses of the running attempt
    int32_t need_more;         // the replay needs the hypotheses of chunk need_more (1: [e0, e1), 2: [e1, H))
    int32_t retry;             // attempt 0 failed: the lane's next round runs attempt 1 (the second reference) on the same pair
    int32_t pad3, pad4;
    int32_t err;               // capacity error (host reports RGBD_ERR_UNSUPPORTED)
    int32_t pad;
    int32_t rng[kLaneSnap];    // the lane's glibc RNG: state[31], f, r
    int32_t srng[kLaneSnap];   // the sampler's RNG after the first e1 hypotheses (k_lane_replay phase 1 continues it)
    double cov;                // sticky depth covariance (RansacSE3::depthCovariance's statics)
    int32_t cov_set, pad2;
};

struct PairOut {               // one per tracked frame b
    float T[16];               // the increment applied when ok: pose(b) = T pose(ref)
    float Tsac[16];            // RansacSE3's mT21 (final attempt)
    float rmse;                // RansacSE3's rmse (final attempt)
    int32_t ok;                // visualOdometry's b
    int32_t sac_ok;
    int32_t n_inliers;         // |sac.mvInliers|
    int32_t ref;               // reference frame of the final attempt
    int32_t retried;
    int32_t gicp_run;          // Gicp::compute was called (rmse >= 0.8)
    int32_t gicp_ok;
    int32_t hyps;              // RANSAC hypotheses the final attempt's loop drew (diagnostics)
    int32_t pad;
};

struct LaneBufs {
    LaneCtl* ctl;              // [L]
    PairOut* out;              // [B]
    uint8_t* flags;            // [B + L][K] mvbOutlier of every frame; row B + l: lane l's first frame (l > 0)
    const int* counts;         // [B] keypoints per frame
    const float* xyz;          // [B][K][3] mvKeys3Dc
    const int4* knn;           // [B-1][K] knn-2 rows of the consecutive pairs (p -> p+1)
    int4* knn_r;               // [L][K] knn-2 rows of the second-reference pairs
    const int4* knn_skip;      // [B-2][K] knn-2 rows of the pairs (p -> p+2) (LaneCfg::skip_rows: the second
                               // references of a few-lane call, computed with the consecutive pairs' rows)
    int* rq;                   // [L] second-reference query frame (-1: none) ...
    int* rt;                   // [L] ... and train frame (k_knn2m pairs)
    int2* mt;                  // [L][Mcap] (queryIdx, trainIdx) in sorted order
    float* pts;                // [L][Mcap][6] (F1 xyz, F2 xyz) in sorted order
    int* samples;              // [L][H][SS]
    int* scount;               // [L][H]
    int* snap;                 // [L][H] cumulative rand() calls after hypothesis h
    HypOut* hyp;               // [L][H + 1] (slot H: the identity transform)
    uint32_t* masks;           // [L][H + 1][MWcap]
    // GICP problems, one slot per pair b (solved after the rounds: GICP feeds nothing back into the chain)
    int* gn;                   // [B] RANSAC inliers staged (0: no alignment, < 20 pairs)
    float* gsrc;               // [B][GM][3]
    float* gtgt;               // [B][GM][3]
    float* gguess;             // [B][16]
    double* gcov;              // [B][2 GM][9]
    double* gM;                // [B][GM][9] Mahalanobis matrices of one outer iteration
    GicpOut* gout;             // [B]
    int* plist;                // [B] pairs with an alignment, then
    int* ppre;                 // [B] their points' exclusive prefix (2 n per pair)
    int* pcount;               // [2] problems, points
    int* done;                 // [L] active hypothesis workgroups of the running launch that finished (fused
                               // replay; the last one resets it)
};

struct LaneCfg {
    int32_t L, B, K, H, iters, SS, MWcap, Mcap, gicp;   // H: hypothesis slots (>= iters, >= 1)
    int32_t e0, e1;            // hypothesis chunks [0, e0) [e0, e1) [e1, H): replays after each (most chains stop in the first)
    int32_t GM;                // GICP points per problem slot (min(Mcap, kGicpMaxM))
    int32_t skip_rows;         // 1: second-reference rows from knn_skip (no per-round k_knn2m launch)
    int32_t fuse;              // 1: each phase's replay runs in the last-finishing active hypothesis workgroup of its lane
                               // (k_ransac_hyp_lanes) instead of a k_lane_replay launch
    uint32_t minTh;
    float maxMahal, nnratio;
    double rcx, rcy;
    GicpDevPrm gp;
};

hipError_t launch_lane_match(const LaneBufs& lb, const LaneCfg& lc, hipStream_t st);
hipError_t launch_ransac_hyp_lanes(const LaneBufs& lb, const LaneCfg& lc, int chunk, hipStream_t st);
hipError_t launch_lane_replay(const LaneBufs& lb, const LaneCfg& lc, int phase, hipStream_t st);
hipError_t launch_gicp_list(const LaneBufs& lb, const LaneCfg& lc, hipStream_t st);
hipError_t launch_gicp_cov_pairs(const LaneBufs& lb, const LaneCfg& lc, hipStream_t st);
hipError_t launch_gicp_align_pairs(const LaneBufs& lb, const LaneCfg& lc, hipStream_t st);
hipError_t launch_gicp_post(const LaneBufs& lb, const LaneCfg& lc, hipStream_t st);
// parity hook: the device sort (libstdc++ std::sort order of distances) on one array of n <= kRansacMaxM
#ifdef RGBD_PNP_PROFILE
void lane_prof_dump(hipStream_t st);   // stage profiles of the profiling build (lanes.hip, ransac.hip)
void hyp_prof_dump(hipStream_t st);
#endif
hipError_t launch_lane_sort_test(const float* dist, int n, int depth_limit, int* order, hipStream_t st);

}  // namespace rgbd

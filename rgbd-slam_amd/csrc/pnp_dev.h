// pnp_dev.h -- PnPRansac kernels interface (host <-> device).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rgbd {

constexpr int kPnpMaxM = 4096;     // correspondences per problem (LDS inlier list of the refine kernel)
constexpr int kPnpModel = 5;       // EPnP minimal sample (solvePnPRansac with SOLVEPNP_ITERATIVE)

struct PnpProbDev {                // one solvePnPRansac call: points [off, off + count) of p3 / p2
    int32_t off;
    int32_t count;
};

struct PnpCam {                    // the camera matrix K as double (cv::Mat K is CV_32F in the reference)
    double fu, fv, uc, vc;
};

struct PnpModel {                  // [R | t], x_cam = R X + t, row-major R
    double R[9];
    double t[3];
};

struct PnpRep {                    // RANSAC replay state of one problem after the device chunks
    int32_t best;                  // global hypothesis slot of the best model, -1 if none
    int32_t maxGood, iter, niters;
    int32_t done;                  // 1: the replay reached niters (or the problem is inactive)
    int32_t count, force_all, nh;  // points, count == 5 path, hypotheses drawn (both chunks)
    int32_t nh2, pad_;             // hypotheses of the second chunk
    uint64_t rng;                  // cv::RNG state after the drawn subsets (host continuation)
};

struct PnpChainRes {               // one pair of the outlier-flag chain (k_pnp_chain; the model from k_pnp_refine)
    int32_t count, ok, n_inliers, iters;
};

struct PnpPrm {                    // solvePnPRansac arguments as the device replay uses them
    int32_t iterations, min_matches, chunk, chunk2;   // hypotheses per problem of the first / second device chunk
    double confidence;
};

// one thread per problem: the first `chunk` subsets of the cv::RNG((uint64)-1) stream (one fixed
// subset for count == 5), hyp_prob[p * chunk + i] = p or -1, rep[p].{count, force_all, nh, rng}
hipError_t launch_pnp_sample(const PnpProbDev* probs, int P, const PnpPrm& prm, int* samples, int* hyp_prob, PnpRep* rep,
                       hipStream_t st);
// one thread per problem: solvePnPRansac's sequential loop over the evaluated chunk (the portable
// RANSACUpdateNumIters), rep[p] updated, best[p] / best[P + p] = refine inputs (-1 unless done)
hipError_t launch_pnp_replay(const int* good, int P, const PnpPrm& prm, PnpRep* rep, int* best, hipStream_t st);
// the second device chunk: for every problem still short of its niters, the next min(chunk2, niters - nh)
// subsets from its saved RNG state into samples / hyp_prob [p * chunk2 + i] (-1: no hypothesis), rep[p].nh2
hipError_t launch_pnp_sample2(int P, const PnpPrm& prm, int* samples, int* hyp_prob, PnpRep* rep, hipStream_t st);
// the replay continued over the second chunk (hypothesis slots h01 + p * chunk2 + i of good / the models)
hipError_t launch_pnp_replay2(const int* good, int h01, int P, const PnpPrm& prm, PnpRep* rep, int* best, hipStream_t st);
// one workgroup (64 lanes) per hypothesis h: EPnP on samples[5h..5h+4] of problem hyp_prob[h], then
// the inlier count over the problem's points.  good[h] = count, or -1 when EPnP found no model.
hipError_t launch_pnp_hyp(const float* p3, const float* p2, const PnpProbDev* probs, const int* hyp_prob,
                    const int* samples, const PnpCam& cam, float thr, int H, int* good, PnpModel* models,
                    hipStream_t st);
// one workgroup per problem with best[p] >= 0: inlier mask of models[best[p]] (all ones when
// force_all[p]), then 10 Gauss-Newton steps on the inliers.  mask: u8 at p3/p2 positions.
hipError_t launch_pnp_refine(const float* p3, const float* p2, const PnpProbDev* probs, const int* best,
                       const int* force_all, const PnpModel* models, const PnpCam& cam, float thr, int P,
                       uint8_t* mask, PnpModel* out, hipStream_t st);
// Matcher::match(ref, cur, m, discardOutliers) for every pair p from its knn-2 rows, fused with
// the PnPRansac 3D-2D gather: p3 = ref mvKeys3Dc[q], p2 = cur mvKeysUn[t].pt, packed at p * kp_cap.
// probs[p] = {p * kp_cap, m}; mq / mt = the kept (queryIdx, trainIdx) in query order.
// qflags = nullptr: discardOutliers = false; else the per-frame mvbOutlier rows [frame][kp_cap] u8
// (discardOutliers = true: flagged queries are skipped).  krow = nullptr: pair p reads knn-2 row block
// p; else block krow[p].
hipError_t launch_match_gather(const int4* knn, const int* counts, const int* qf, const int* tf, const float* xyz,
                         const float* kun, int kp_cap, float nnratio, int npairs, float* p3, float* p2,
                         PnpProbDev* probs, int* mq, int* mt, hipStream_t st, const uint8_t* qflags = nullptr,
                         const int* krow = nullptr);
// The outlier-flag chain (Features/Matcher.cpp:125-128 with discardOutliers = true; Solver/PnPRansac.cpp:31,51)
// over S contiguous runs of consecutive pairs, one 256-thread workgroup per run: for each pair p of run s
// (pairs seg[s] .. seg[s + 1] - 1; pair p = query frame p, train frame p + 1, knn-2 row block p) in order,
// the Matcher filter on frame p's flags + the 3D-2D gather, solvePnPRansac (subsets, EPnP hypotheses in
// passes of 20, the sequential replay, the RANSAC inlier mask) and the flag writes on frame p + 1 (except
// after a run's last pair: the next run starts on that frame's fresh flags).  flags = [B][kp_cap], cleared
// by the caller; p3 / p2 / mq / mt / mask = the pairs' points [P][kp_cap]; res[p] = the pair's RANSAC result.
// The refinement's inputs are left for launch_pnp_refine over the P pairs: probs[p], best[p] (= p, or -1),
// best[P + p] (force_all), models[p] (the RANSAC model).  rngtab[j] =
// the (j + 1)-th raw output of cv::RNG((uint64)-1) for j < ntab, rng_end = the generator state after them.
hipError_t launch_pnp_chain(const int4* knn, const int* counts, const float* xyz, const float* kun, int kp_cap,
                      float nnratio, const int* seg, int S, const PnpCam& cam, float thr, const PnpPrm& prm, float* p3,
                      float* p2, int* mq, int* mt, uint8_t* mask, uint8_t* flags, PnpChainRes* res,
                      const uint32_t* rngtab, int ntab, unsigned long long rng_end, PnpProbDev* probs, int* best,
                      PnpModel* models, int P, hipStream_t st);

hipError_t launch_debug_rotation_ops(const double* x, const double* num, const double* den, const double* theta, int n,
                                     double* sq, double* q, double* t, hipStream_t st);
#ifdef RGBD_PNP_PROFILE
void pnp_prof_dump(int H, hipStream_t st);   // profiling builds: per-stage cycle means of k_pnp_hyp
void chain_prof_dump(hipStream_t st);         // profiling builds: per-stage times of k_pnp_chain's first run
#endif

}  // namespace rgbd

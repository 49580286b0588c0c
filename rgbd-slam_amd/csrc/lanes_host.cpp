// lanes_host.cpp -- host driver of the device-resident RansacSE3 tracking chain (lanes_dev.h).
//
// Tracking::visualOdometry (System/Tracking.cpp:121-163) over L independent lanes of an extracted batch:
// the knn-2 rows of every consecutive pair in one launch, then one round per pair of the longest lane, each
// round a fixed sequence of launches on the context stream with no host wait: Matcher + RansacSE3 set-up,
// the first hypothesis chunk (+ identity), replay, the rest of the hypotheses for the lanes that need them,
// replay, the same for the second reference (second-reference knn-2 rows, launches whose lanes all skip
// when none failed), GICP of the lanes whose rmse >= 0.8, and the pair's result.  One read-back at the end.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "context.h"
#include "lanes_dev.h"
#include "lanes_host.h"
#include "launch.h"

namespace rgbd {

// LaneCfg::fuse for calls of at most this many lanes.  r06 same-box A/B of the single chain (se3_chain_one, us per
// pair): separate replay launches 126.0, fused with every workgroup of a launch counted 139.4 (a phase-2 launch is
// ~H workgroups, each paying an agent-scope release), fused with only the active workgroups counted 126.1, and
// that with a first chunk of one hypothesis 119.0 (separate launches with it: 124.7)
constexpr int kLaneFuseMax = 4;   // LaneCfg::fuse for calls of at most this many lanes
constexpr int kLaneChunk0 = 2;   // RansacSE3 hypotheses per lane evaluated before the first replay
constexpr int kLaneChunk0Few = 1;   // the same for calls of <= kLaneFuseMax lanes (r06 same-box A/B (fused replay): 1 vs 2: se3_chain_one 119.0 vs 126.0 us per pair)
constexpr int kLaneChunk1Few = 4 * kLaneChunk0Few;   // end of the second chunk for those calls (2 / 8 measured the same)
// At most 2 x kLaneWindow rounds (8 dispatches each) are enqueued ahead of the device: every kLaneWindow rounds
// the host waits for the marker recorded two windows earlier.  A call otherwise queues all of its ~8 B dispatches
// before its first host wait; under rocprofv3 counter collection (which adds its own packets per dispatch to the
// queue) such runs aborted twice with HSA_STATUS_ERROR_INVALID_PACKET_FORMAT ("Lane chain under
// rocprofv3").  The waits cost < 0.5 % of a 1023-round call.
#ifndef RGBD_LANE_WINDOW
#define RGBD_LANE_WINDOW 32   // 0: no window (only the diagnostic build of tools/lane_window_exp.sh)
#endif
constexpr int kLaneWindow = RGBD_LANE_WINDOW;

struct LaneWS {
    int capL = 0, capB = 0, K = 0, H = 0, SS = 0, Mcap = 0, MWcap = 0, GM = 0;
    bool gicp = false;          // GICP problem slots allocated (only for calls that run GICP)
    LaneBufs d{};
    std::vector<void*> owned;
    LaneCtl* h_ctl = nullptr;   // pinned
    PairOut* h_out = nullptr;   // pinned
    hipEvent_t ev_window[2] = {nullptr, nullptr};   // round markers bounding the rounds in flight
    int* d_pairs = nullptr;     // consecutive pairs (p, p + 1): [capB = maxB] query | [capB] train, then the
                                // pairs (p, p + 2) the same way
    int4* d_knn_skip = nullptr; // [capB][K] knn-2 rows of the pairs (p, p + 2)
};

static void ws_free(LaneWS* w)
{
    for (void* p : w->owned) (void)hipFree(p);
    w->owned.clear();
    if (w->h_ctl) (void)hipHostFree(w->h_ctl);
    if (w->h_out) (void)hipHostFree(w->h_out);
    for (hipEvent_t& e : w->ev_window) {
        if (e) (void)hipEventDestroy(e);
        e = nullptr;
    }
    w->h_ctl = nullptr;
    w->h_out = nullptr;
    w->d = LaneBufs{};
    w->d_pairs = nullptr;
    w->d_knn_skip = nullptr;
}

void lanes_free(rgbd_ctx* c)
{
    LaneWS* w = static_cast<LaneWS*>(c->lanes);
    if (!w) return;
    ws_free(w);
    delete w;
    c->lanes = nullptr;
}

template <typename T>
static rgbd_status dal(rgbd_ctx* c, LaneWS* w, T** p, size_t n, const char* what)
{
    rgbd_status s = check_hip(c, hipMalloc((void**)p, std::max<size_t>(n * sizeof(T), 16)), what);
    if (!s) w->owned.push_back((void*)*p);
    return s;
}

static rgbd_status lanes_ws(rgbd_ctx* c, int L, int H, int SS, bool gicp, LaneWS** out)
{
    LaneWS* w = static_cast<LaneWS*>(c->lanes);
    if (!w) {
        w = new LaneWS();
        c->lanes = w;
    }
    const int K = c->cfg.kp_cap, B = c->maxB;
    if (w->d.ctl && L <= w->capL && H <= w->H && SS <= w->SS && (!gicp || w->gicp)) {
        *out = w;
        return RGBD_OK;
    }
    ws_free(w);
    w->capL = std::max(L, w->capL);
    w->capB = B;
    w->K = K;
    w->H = std::max(H, w->H);
    w->SS = std::max(SS, std::max(w->SS, 1));
    w->Mcap = std::min(K, kRansacMaxM);
    w->MWcap = (w->Mcap + 31) / 32 + 1;
    w->GM = std::min(w->Mcap, kGicpMaxM);
    w->gicp = gicp || w->gicp;
    const size_t Lc = (size_t)w->capL, Hc = (size_t)w->H;
    LaneBufs& d = w->d;
    rgbd_status s = dal(c, w, &d.ctl, Lc, "lane ctl");
    if (!s) s = dal(c, w, &d.out, (size_t)B, "lane pair out");
    if (!s) s = dal(c, w, &d.flags, ((size_t)B + Lc) * K, "lane flags");
    if (!s) s = dal(c, w, &d.knn_r, Lc * K, "lane knn rows");
    if (!s) s = dal(c, w, &d.rq, Lc, "lane rq");
    if (!s) s = dal(c, w, &d.rt, Lc, "lane rt");
    if (!s) s = dal(c, w, &d.mt, Lc * w->Mcap, "lane matches");
    if (!s) s = dal(c, w, &d.pts, Lc * w->Mcap * 6, "lane points");
    if (!s) s = dal(c, w, &d.samples, Lc * Hc * w->SS, "lane samples");
    if (!s) s = dal(c, w, &d.scount, Lc * Hc, "lane sample counts");
    if (!s) s = dal(c, w, &d.snap, Lc * Hc, "lane rand counts");
    if (!s) s = dal(c, w, &d.hyp, Lc * (Hc + 1), "lane hypotheses");
    if (!s) s = dal(c, w, &d.masks, Lc * (Hc + 1) * w->MWcap, "lane masks");
    // GICP problem slots, one per pair (~0.5 GB at max_batch 1024): only when a call runs GICP
    const size_t Bs = (size_t)B, GM = w->gicp ? (size_t)w->GM : 0;
    if (!s) s = dal(c, w, &d.gn, Bs, "gicp n");
    if (!s) s = dal(c, w, &d.gsrc, Bs * GM * 3, "gicp src");
    if (!s) s = dal(c, w, &d.gtgt, Bs * GM * 3, "gicp tgt");
    if (!s) s = dal(c, w, &d.gguess, Bs * 16, "gicp guess");
    if (!s) s = dal(c, w, &d.gcov, Bs * 2 * GM * 9, "gicp cov");
    if (!s) s = dal(c, w, &d.gM, Bs * GM * 9, "gicp M");
    if (!s) s = dal(c, w, &d.gout, Bs, "gicp out");
    if (!s) s = dal(c, w, &d.plist, Bs, "gicp list");
    if (!s) s = dal(c, w, &d.ppre, Bs, "gicp prefix");
    if (!s) s = dal(c, w, &d.pcount, 2, "gicp count");
    if (!s) s = dal(c, w, &d.done, Lc, "lane done counts");
    if (!s) s = check_hip(c, hipMemset(d.done, 0, Lc * sizeof(int)), "lane done clear");
    if (!s) s = dal(c, w, &w->d_pairs, 4 * (size_t)B, "lane pairs");
    if (!s) s = dal(c, w, &w->d_knn_skip, (size_t)B * K, "lane second-reference rows");
    if (!s) s = check_hip(c, hipHostMalloc((void**)&w->h_ctl, Lc * sizeof(LaneCtl), hipHostMallocDefault), "lane ctl pinned");
    if (!s) s = check_hip(c, hipHostMalloc((void**)&w->h_out, (size_t)B * sizeof(PairOut), hipHostMallocDefault), "lane out pinned");
    if (!s) {
        std::vector<int> pairs(4 * (size_t)B, 0);
        for (int p = 0; p + 1 < B; p++) {
            pairs[p] = p;
            pairs[B + p] = p + 1;
        }
        for (int p = 0; p + 2 < B; p++) {
            pairs[2 * (size_t)B + p] = p;
            pairs[3 * (size_t)B + p] = p + 2;
        }
        s = check_hip(c, hipMemcpy(w->d_pairs, pairs.data(), pairs.size() * 4, hipMemcpyHostToDevice), "lane pairs");
    }
    if (s) {
        ws_free(w);
        return s;
    }
    *out = w;
    return RGBD_OK;
}

static void raster_consts(double* rcx, double* rcy)
{
    const double cam_angle_x = 58.0 / 180.0 * M_PI;   // Solver/SolverSE3.cpp:218-225
    const double cam_angle_y = 45.0 / 180.0 * M_PI;
    const double sx = 3 * std::tan(cam_angle_x / 640.0);
    const double sy = 3 * std::tan(cam_angle_y / 480.0);
    *rcx = sx * sx;
    *rcy = sy * sy;
}

rgbd_status lanes_track(rgbd_ctx* c, int B, float nnratio, const rgbd_ransac_params& prm, const LaneSpec* spec, int L,
                        rgbd_rng* rngs, rgbd_sticky* stickies, const uint8_t* flags_f0, const uint8_t* flags_f1,
                        std::vector<PairOut>& out, uint8_t* flags_out2, uint8_t* flags_out1)
{
    if (L < 1 || L > B) return fail(c, RGBD_ERR_ARG, "lanes: 1 <= L <= B");
    if (prm.sample_size < 1 || prm.sample_size > 8) return fail(c, RGBD_ERR_UNSUPPORTED, "sample_size must be in [1, 8]");
    if (prm.iterations < 0) return fail(c, RGBD_ERR_ARG, "iterations < 0");
    const int K = c->cfg.kp_cap;
    const int H = std::max(prm.iterations, 1);
    LaneWS* w = nullptr;
    rgbd_status s = lanes_ws(c, L, H, (int)prm.sample_size, c->track_gicp.enable != 0, &w);
    if (s) return s;
    const hipStream_t st = c->stream;
    // knn-2 rows of every consecutive pair (query = frame p, train = frame p + 1)
    if (B > 1) {
        const int tk = timer_begin(c, "k_knn2");
        RGBD_TRY(c, launch_knn2(c->d_desc, c->d_count, w->d_pairs, w->d_pairs + w->capB, K, K, c->d_knn, B - 1, st), "knn2");
        timer_end(c, tk);
    }
    // few lanes: the second references' rows (p -> p + 2) of every frame in one launch here, instead of a
    // k_knn2m launch in every round (a launch costs ~4.5 us on the single chain's critical path, the batched
    // rows ~0.25 us per pair); many lanes keep the per-round launch, whose cost their rounds share
    const bool skip_rows = L <= kLaneFuseMax;
    if (skip_rows && B > 2) {
        const int tk = timer_begin(c, "k_knn2");
        RGBD_TRY(c, launch_knn2(c->d_desc, c->d_count, w->d_pairs + 2 * (size_t)w->capB, w->d_pairs + 3 * (size_t)w->capB, K, K,
                                w->d_knn_skip, B - 2, st), "knn2 skip");
        timer_end(c, tk);
    }
    LaneBufs lb = w->d;
    lb.counts = c->d_count;
    lb.xyz = c->d_xyz;
    lb.knn = c->d_knn;
    lb.knn_skip = w->d_knn_skip;
    // every frame starts with clear outlier flags; a continuing chunk's first two frames carry theirs
    s = check_hip(c, hipMemsetAsync(lb.flags, 0, ((size_t)B + L) * K, st), "lane flags clear");
    if (!s) s = check_hip(c, hipMemsetAsync(lb.gn, 0, (size_t)B * 4, st), "gicp problems clear");
    if (!s && flags_f0) s = check_hip(c, hipMemcpyAsync(lb.flags, flags_f0, (size_t)K, hipMemcpyHostToDevice, st), "flags f0");
    if (!s && flags_f1 && B > 1)
        s = check_hip(c, hipMemcpyAsync(lb.flags + K, flags_f1, (size_t)K, hipMemcpyHostToDevice, st), "flags f1");
    if (s) return s;
    int rounds = 0;
    for (int l = 0; l < L; l++) {
        LaneCtl& k = w->h_ctl[l];
        std::memset(&k, 0, sizeof(k));
        k.start = spec[l].start;
        k.end = spec[l].end;
        k.b = spec[l].first;
        for (int i = 0; i < 31; i++) k.rng[i] = rngs[l].state[i];
        k.rng[31] = rngs[l].f;
        k.rng[32] = rngs[l].r;
        k.cov = stickies[l].cov;
        k.cov_set = stickies[l].set;
        rounds = std::max(rounds, k.end - k.b + 1);
        if (k.start < 0 || k.end >= B || k.b <= k.start) return fail(c, RGBD_ERR_ARG, "lanes: bad lane range");
    }
    s = check_hip(c, hipMemcpyAsync(lb.ctl, w->h_ctl, (size_t)L * sizeof(LaneCtl), hipMemcpyHostToDevice, st), "lane ctl");
    if (s) return s;
    LaneCfg lc{};
    lc.L = L;
    lc.B = B;
    lc.K = K;
    lc.H = H;
    lc.iters = prm.iterations;
    lc.SS = (int)prm.sample_size;
    lc.MWcap = w->MWcap;
    lc.Mcap = w->Mcap;
    // hypothesis chunks: 95 % of the chains stop at their first hypothesis (> 80 % inliers, :99-100), the rest
    // within the first few (measured round 3); e0 / e1 = kLaneChunk0 / 4 kLaneChunk0
    lc.e0 = std::min(H, L <= kLaneFuseMax ? kLaneChunk0Few : kLaneChunk0);
    lc.e1 = std::min(H, L <= kLaneFuseMax ? kLaneChunk1Few : 4 * lc.e0);
    lc.GM = w->GM;
    // few lanes (the single chains): the replays ride in the hypothesis launches, 3-4 launches a round instead of
    // 7-8.  Many lanes keep the separate replay launches: there a round's launches are few next to its work, and
    // a fused tail would add an L2 writeback per workgroup beside the other contexts' extractions
    lc.fuse = L <= kLaneFuseMax ? 1 : 0;
    lc.skip_rows = skip_rows ? 1 : 0;
    lc.gicp = c->track_gicp.enable ? 1 : 0;
    lc.minTh = prm.min_inlier_th;
    lc.maxMahal = prm.max_mahalanobis;
    lc.nnratio = nnratio;
    raster_consts(&lc.rcx, &lc.rcy);
    const rgbd_gicp_params& g = c->track_gicp;
    if (lc.gicp && (g.k_correspondences < 1 || g.k_correspondences > 32))
        return fail(c, RGBD_ERR_UNSUPPORTED, "GICP k_correspondences must be in [1, 32]");
    lc.gp = GicpDevPrm{g.max_iterations, g.k_correspondences, g.gn_iterations, 0, g.max_corr_dist * g.max_corr_dist,
                       g.transformation_epsilon, g.rotation_epsilon, g.gicp_epsilon};
    // one round = one attempt of every lane's current pair: attempt 0 against the previous frame or, the
    // round after it failed, attempt 1 against the second reference (the pair's knn-2 rows of that round's
    // first launch; lanes without a retry skip it).  A retry costs its lane one more round: after the planned
    // rounds the lanes' progress is read back and the rounds continue until every lane has finished
    s = check_hip(c, hipMemsetAsync(lb.rq, 0xff, (size_t)L * sizeof(int), st), "second references clear");
    if (s) return s;
    bool any_retry = false;   // no second-reference rows are due before the first round
    for (hipEvent_t& e : w->ev_window)
        if (!e && (s = check_hip(c, hipEventCreateWithFlags(&e, hipEventDisableTiming), "lane window event"))) return s;
    bool marked[2] = {false, false};
    int enqueued = 0;   // rounds enqueued by this call
    for (int left = rounds; left > 0;) {
        for (int r = 0; r < left; r++) {
            if (kLaneWindow > 0 && enqueued > 0 && enqueued % kLaneWindow == 0) {   // bound the rounds in flight
                const int k = (enqueued / kLaneWindow) & 1;
                if (marked[k] && (s = check_hip(c, hipEventSynchronize(w->ev_window[k]), "lane window wait"))) return s;
                if ((s = check_hip(c, hipEventRecord(w->ev_window[k], st), "lane window mark"))) return s;
                marked[k] = true;
            }
            enqueued++;
            if (!skip_rows && (any_retry || r > 0)) {
                const int tk = timer_begin(c, "k_knn2");
                RGBD_TRY(c, launch_knn2(c->d_desc, c->d_count, lb.rq, lb.rt, K, K, lb.knn_r, L, st), "knn2");
                timer_end(c, tk);
            }
            int tk = timer_begin(c, "k_lane_match");
            RGBD_TRY(c, launch_lane_match(lb, lc, st), "lane_match");
            timer_end(c, tk);
            for (int ph = 0; ph <= 2; ph++) {   // phases 1, 2: the chains that need more hypotheses
                tk = timer_begin(c, "k_ransac_hyp");
                RGBD_TRY(c, launch_ransac_hyp_lanes(lb, lc, ph, st), "ransac_hyp_lanes");
                timer_end(c, tk);
                if (lc.fuse) continue;   // the replay ran in the phase's last hypothesis workgroup
                tk = timer_begin(c, "k_lane_replay");
                RGBD_TRY(c, launch_lane_replay(lb, lc, ph, st), "lane_replay");
                timer_end(c, tk);
            }
        }
        s = check_hip(c, hipMemcpyAsync(w->h_ctl, lb.ctl, (size_t)L * sizeof(LaneCtl), hipMemcpyDeviceToHost, st), "lane progress");
        if (!s) s = check_hip(c, hipStreamSynchronize(st), "lane progress sync");
        if (s) return s;
        left = 0;
        any_retry = false;
        for (int l = 0; l < L; l++) {
            left = std::max(left, w->h_ctl[l].end - w->h_ctl[l].b + 1);
            any_retry = any_retry || w->h_ctl[l].retry;
        }
    }
#ifdef RGBD_PNP_PROFILE
    lane_prof_dump(st);
    hyp_prof_dump(st);
#endif
    if (lc.gicp && rounds > 0) {   // every pair's GICP problem at once (the chain never reads GICP's results)
        int tk = timer_begin(c, "k_gicp_list");
        RGBD_TRY(c, launch_gicp_list(lb, lc, st), "gicp_list");
        timer_end(c, tk);
        tk = timer_begin(c, "k_gicp_cov");
        RGBD_TRY(c, launch_gicp_cov_pairs(lb, lc, st), "gicp_cov_pairs");
        timer_end(c, tk);
        tk = timer_begin(c, "k_gicp_align");
        RGBD_TRY(c, launch_gicp_align_pairs(lb, lc, st), "gicp_align_pairs");
        timer_end(c, tk);
        tk = timer_begin(c, "k_gicp_post");
        RGBD_TRY(c, launch_gicp_post(lb, lc, st), "gicp_post");
        timer_end(c, tk);
    }
    s = check_hip(c, hipMemcpyAsync(w->h_out, lb.out, (size_t)B * sizeof(PairOut), hipMemcpyDeviceToHost, st), "lane out");
    if (!s) s = check_hip(c, hipMemcpyAsync(w->h_ctl, lb.ctl, (size_t)L * sizeof(LaneCtl), hipMemcpyDeviceToHost, st), "lane ctl back");
    if (!s && flags_out2 && B >= 2)
        s = check_hip(c, hipMemcpyAsync(flags_out2, lb.flags + (size_t)(B - 2) * K, (size_t)K, hipMemcpyDeviceToHost, st), "flags out2");
    if (!s && flags_out1)
        s = check_hip(c, hipMemcpyAsync(flags_out1, lb.flags + (size_t)(B - 1) * K, (size_t)K, hipMemcpyDeviceToHost, st), "flags out1");
    if (!s) s = check_hip(c, hipStreamSynchronize(st), "lane sync");
    if (s) return s;
    for (int l = 0; l < L; l++) {
        const LaneCtl& k = w->h_ctl[l];
        if (k.err == 1) return fail(c, RGBD_ERR_UNSUPPORTED, "more matches than RansacSE3's LDS-resident cap (2304)");
        if (k.err == 2) return fail(c, RGBD_ERR_UNSUPPORTED, "more than 2048 RANSAC inliers for GICP");
        for (int i = 0; i < 31; i++) rngs[l].state[i] = k.rng[i];
        rngs[l].f = k.rng[31];
        rngs[l].r = k.rng[32];
        stickies[l].cov = k.cov;
        stickies[l].set = k.cov_set;
    }
    out.assign(w->h_out, w->h_out + B);
    return RGBD_OK;
}

rgbd_status lanes_sort_test(rgbd_ctx* c, const float* dist, int n, int depth_limit, int* order)
{
    float* d_dist = nullptr;
    int* d_order = nullptr;
    rgbd_status s = check_hip(c, hipMalloc((void**)&d_dist, std::max(n, 1) * 4), "sort dist");
    if (!s) s = check_hip(c, hipMalloc((void**)&d_order, std::max(n, 1) * 4), "sort order");
    if (!s) s = check_hip(c, hipMemcpy(d_dist, dist, (size_t)n * 4, hipMemcpyHostToDevice), "sort in");
    if (!s) {
        s = check_hip(c, launch_lane_sort_test(d_dist, n, depth_limit, d_order, c->stream), "launch of k_lane_sort_test");
    }
    if (!s) s = check_hip(c, hipMemcpyAsync(order, d_order, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream), "sort out");
    if (!s) s = check_hip(c, hipStreamSynchronize(c->stream), "sort sync");
    if (d_dist) (void)hipFree(d_dist);
    if (d_order) (void)hipFree(d_order);
    return s;
}

}  // namespace rgbd

// pnp_host.cpp -- PnPRansac host control (C ABI): sample streams, the sequential RANSAC replay, and
// the extract + match + PnPRansac chain over a device-resident batch.
//
// cv::solvePnPRansac (called at Solver/PnPRansac.cpp:39) is RANSACPointSetRegistrator::run with a
// fresh cv::RNG((uint64)-1): the subset drawn at iteration i depends only on the point count.  So
// the host draws the subsets of a chunk of iterations, k_pnp_hyp evaluates all of them (and all
// problems of a batch) in one launch, and the host replays the loop in order:
//     goodCount > max(maxGood, modelPoints - 1)  ->  best, niters = RANSACUpdateNumIters(...)
// drawing further chunks only while the replay has not reached niters.  k_pnp_refine then refines
// every problem's best model on its inliers.  Semantics: oracle/orc_pnp.cpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "context.h"
#include "launch.h"
#include "pnp_dev.h"

using namespace rgbd;

namespace rgbd {

namespace {

// cv::RNG: multiply-with-carry, state = (uint64)-1 for RANSACPointSetRegistrator
struct CvRng {
    uint64_t state;
    explicit CvRng(uint64_t s = ~0ull) : state(s ? s : 0xffffffffull) {}
    unsigned next()
    {
        state = (uint64_t)(unsigned)state * 4164903690u + (unsigned)(state >> 32);
        return (unsigned)state;
    }
    int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + a); }
};

// oracle log_det (portable log from + - * / and exact frexp; the device replay computes the same)
double log_det(double x)
{
    int e = 0;
    double m = std::frexp(x, &e);
    if (m < 0.70710678118654752440) {
        m = m * 2.0;
        e -= 1;
    }
    const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
    double t = 1.0 / 23.0;
    t = t * s2 + 1.0 / 21.0;
    t = t * s2 + 1.0 / 19.0;
    t = t * s2 + 1.0 / 17.0;
    t = t * s2 + 1.0 / 15.0;
    t = t * s2 + 1.0 / 13.0;
    t = t * s2 + 1.0 / 11.0;
    t = t * s2 + 1.0 / 9.0;
    t = t * s2 + 1.0 / 7.0;
    t = t * s2 + 1.0 / 5.0;
    t = t * s2 + 1.0 / 3.0;
    t = t * s2 + 1.0;
    const double de = (double)e;
    return de * 6.93147180559945286227e-01 + (de * 2.31904681384629955842e-17 + 2.0 * s * t);
}

// RANSACUpdateNumIters (OpenCV 3.4 ptsetreg.cpp), portable log / power (oracle update_num_iters)
int update_num_iters(double p, double ep, int modelPoints, int maxIters)
{
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    const double q = 1. - ep;
    double qm = 1.0;
    for (int i = 0; i < modelPoints; i++) qm = qm * q;
    double denom = 1. - qm;
    if (denom < DBL_MIN) return 0;
    num = log_det(num);
    denom = log_det(denom);
    return denom >= 0 || -num >= maxIters * (-denom) ? maxIters : (int)std::nearbyint(num / denom);
}

// RANSACPointSetRegistrator::getSubset with an always-true checkSubset: 5 distinct indices
void draw_subset(CvRng& rng, int count, int* idx)
{
    for (int i = 0; i < kPnpModel; i++) {
        for (;;) {
            const int v = rng.uniform(0, count);
            int j;
            for (j = 0; j < i; j++)
                if (idx[j] == v) break;
            if (j == i) { idx[i] = v; break; }
        }
    }
}

// iterations per problem evaluated on the device, in two chunks: every problem's first K0 subsets, then
// for the problems whose replay has not reached niters the next K1 (k_pnp_sample2 / k_pnp_replay2, no
// host wait).  Iterations past a problem's niters are wasted work beside the description kernel, and
// problems still running after both chunks cost a host round trip, so the chunks follow the data: after
// every solve K0 = the 90th percentile of that solve's iteration counts + 1 and K0 + K1 = the 99th + 2,
// K1 rounded up to a multiple of 4, both clamped to [kPnpChunkMin, kPnpChunkMax] (the results do not depend
// on them).  Round 4: one adaptive chunk of the 99th percentile (~20 hypotheses per pair at B = 1024)
// evaluated ~4x the ~5 iterations a pair runs on average.
constexpr int kPnpFirstChunk = 8, kPnpFirstChunk2 = 16;   // the first solve's chunks
constexpr int kPnpChunkMin = 4, kPnpChunkMax = 64;
constexpr int kChainRngTab = 8192;   // raw RNG outputs tabulated for k_pnp_chain (~1600 iterations at 400 points)


template <typename T>
rgbd_status grow_dev(rgbd_ctx* c, T** p, size_t* cap, size_t need, const char* what)
{
    if (need <= *cap) return RGBD_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    const size_t n = std::max(need, *cap * 2);
    rgbd_status s = check_hip(c, hipMalloc((void**)p, n * sizeof(T)), what);
    *cap = s ? 0 : n;
    return s;
}

template <typename T>
rgbd_status grow_host(rgbd_ctx* c, T** p, size_t* cap, size_t need, const char* what)
{
    if (need <= *cap) return RGBD_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    const size_t n = std::max(need, *cap * 2);
    rgbd_status s = check_hip(c, hipHostMalloc((void**)p, n * sizeof(T), hipHostMallocDefault), what);
    *cap = s ? 0 : n;
    return s;
}

}  // namespace

struct PnpWS {
    int h01 = 0;   // hypothesis slots of the device chunks of the solve in flight (pnp_launch -> pnp_finish)
    int k0 = 0, k1 = 0;     // subsets per problem of the two device chunks (fixed when the subsets are drawn)
    bool sampled = false;   // the first chunk's subsets are drawn (pnp_sample_launch), the rest not launched yet
    // device
    float* d_p3 = nullptr; size_t c_p3 = 0;
    float* d_p2 = nullptr; size_t c_p2 = 0;
    uint8_t* d_mask = nullptr; size_t c_mask = 0;
    int* d_mq = nullptr; size_t c_mq = 0;
    int* d_mt = nullptr; size_t c_mt = 0;
    PnpProbDev* d_probs = nullptr; size_t c_probs = 0;
    int* d_hprob = nullptr; size_t c_hprob = 0;      // hypothesis -> problem
    int* d_samples = nullptr; size_t c_samples = 0;
    int* d_good = nullptr; size_t c_good = 0;
    PnpModel* d_models = nullptr; size_t c_models = 0;
    int* d_best = nullptr; size_t c_best = 0;        // [best | force_all] per problem
    int* d_cpairs = nullptr;   // consecutive pairs (b-1, b) for b < maxB: [query frames | train frames]
    // per-problem results in one block [rep | out] (device and pinned host), read back by one copy
    unsigned char* d_res = nullptr; unsigned char* h_res = nullptr; size_t c_res = 0;
    PnpRep* d_rep = nullptr; PnpModel* d_out = nullptr;
    // pinned host mirrors
    PnpProbDev* h_probs = nullptr; size_t ch_probs = 0;
    int* h_hprob = nullptr; size_t ch_hprob = 0;
    int* h_samples = nullptr; size_t ch_samples = 0;
    int* h_good = nullptr; size_t ch_good = 0;
    int* h_best = nullptr; size_t ch_best = 0;
    PnpRep* h_rep = nullptr; PnpModel* h_out = nullptr;
    // outlier-flag chain (rgbd_pnp_params.flag_segments > 0): per-frame mvbOutlier rows, the runs' first
    // pairs, the per-pair results (k_pnp_chain) and the per-frame extraction error flags
    uint8_t* d_flags = nullptr; size_t c_flags = 0;
    int* d_seg = nullptr; size_t c_seg = 0;
    int* h_seg = nullptr; size_t ch_seg = 0;
    PnpChainRes* d_cres = nullptr; size_t c_cres = 0;
    PnpChainRes* h_cres = nullptr; size_t ch_cres = 0;
    uint32_t* d_rngtab = nullptr;   // the raw cv::RNG((uint64)-1) stream (kChainRngTab outputs)
    int* h_err = nullptr; size_t ch_err = 0;
    hipEvent_t ev = nullptr;   // recorded after the first-chunk read-back (pnp_launch)
    hipEvent_t ev_in = nullptr;   // recorded on the extraction stream after the 3D-2D gather
    hipStream_t st = nullptr;     // solve stream: nullptr = the context stream
};

static hipStream_t ws_stream(const rgbd_ctx* c, const PnpWS* w) { return w->st ? w->st : c->stream; }

static void ws_free(PnpWS* w)
{
    if (!w) return;
    void* dev[] = {w->d_p3, w->d_p2, w->d_mask, w->d_mq, w->d_mt, w->d_probs, w->d_hprob, w->d_samples,
                   w->d_good, w->d_models, w->d_best, w->d_res, w->d_cpairs, w->d_flags, w->d_seg, w->d_cres, w->d_rngtab};
    for (void* p : dev)
        if (p) (void)hipFree(p);
    void* host[] = {w->h_probs, w->h_hprob, w->h_samples, w->h_good, w->h_best, w->h_res, w->h_seg, w->h_cres,
                    w->h_err};
    for (void* p : host)
        if (p) (void)hipHostFree(p);
    if (w->ev) (void)hipEventDestroy(w->ev);
    if (w->ev_in) (void)hipEventDestroy(w->ev_in);
    delete w;
}

// submit / collect tracking: kPipeDepth workspaces used in turn, submissions collected in order.
// A submission's PnPRansac solve is launched (on the solve stream) by the NEXT submission right after
// that one's k_fast is enqueued, behind an event on it: the latency-bound solve then runs beside the
// quadtree / blur / description kernels, not beside the VALU-bound FAST.  collect launches a solve
// still due itself.
constexpr int kPipeDepth = 3;
// the per-batch extraction outputs a step's knn-2 / gather read: consecutive pipelined submissions
// alternate between the context's own set (0) and a second one (1), so step i's matching (on the
// match stream) overlaps step i+1's extraction
struct OutSet {
    int* count = nullptr;
    float* kps = nullptr;
    float* kun = nullptr;
    uint8_t* desc = nullptr;
    float* xyz = nullptr;
    int4* knn = nullptr;
};
struct PnpPending {
    int B = 0, P = 0;
    rgbd_pnp_params prm{};
    float nnratio = 0.9f;
    bool solve_due = false;   // gathered, solve not launched yet
    OutSet out{};             // the output set this submission's extraction wrote
    int set = 0;
};
struct PnpPipe {
    PnpWS* ws[kPipeDepth] = {};
    PnpPending q[kPipeDepth];
    int head = 0;    // slot of the oldest outstanding submission
    int count = 0;   // outstanding submissions (0..kPipeDepth)
    hipEvent_t ev_fast = nullptr;   // recorded on the launch stream after a submission's k_fast
    OutSet set[2];
    int parity = 0;                 // output set of the next submission
    hipEvent_t ev_free[2] = {};     // recorded on the match stream after the last gather reading a set
    hipEvent_t ev_desc = nullptr;   // recorded on the launch stream after a submission's extraction
};

static OutSet ctx_outputs(const rgbd_ctx* c) { return OutSet{c->d_count, c->d_kps, c->d_kun, c->d_desc, c->d_xyz, c->d_knn}; }
static void set_ctx_outputs(rgbd_ctx* c, const OutSet& o)
{
    c->d_count = o.count;
    c->d_kps = o.kps;
    c->d_kun = o.kun;
    c->d_desc = o.desc;
    c->d_xyz = o.xyz;
    c->d_knn = o.knn;
}

void pnp_free(rgbd_ctx* c)
{
    ws_free(static_cast<PnpWS*>(c->pnp));
    c->pnp = nullptr;
    if (PnpPipe* pp = static_cast<PnpPipe*>(c->pnp_pipe)) {
        for (PnpWS* w : pp->ws) ws_free(w);
        if (pp->ev_fast) (void)hipEventDestroy(pp->ev_fast);
        if (pp->ev_desc) (void)hipEventDestroy(pp->ev_desc);
        for (hipEvent_t e : pp->ev_free)
            if (e) (void)hipEventDestroy(e);
        if (pp->set[0].count) set_ctx_outputs(c, pp->set[0]);   // the context frees its own set
        const OutSet& a = pp->set[1];
        void* ptrs[] = {a.count, a.kps, a.kun, a.desc, a.xyz, a.knn};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
        delete pp;
        c->pnp_pipe = nullptr;
    }
}

static PnpWS* pnp_ws(rgbd_ctx* c)
{
    if (!c->pnp) c->pnp = new PnpWS();
    return static_cast<PnpWS*>(c->pnp);
}

static rgbd_status ws_points(rgbd_ctx* c, PnpWS* w, size_t npts, size_t P)
{
    rgbd_status s = grow_dev(c, &w->d_p3, &w->c_p3, 3 * std::max<size_t>(npts, 1), "pnp p3");
    if (!s) s = grow_dev(c, &w->d_p2, &w->c_p2, 2 * std::max<size_t>(npts, 1), "pnp p2");
    if (!s) s = grow_dev(c, &w->d_mask, &w->c_mask, std::max<size_t>(npts, 1), "pnp mask");
    if (!s) s = grow_dev(c, &w->d_probs, &w->c_probs, std::max<size_t>(P, 1), "pnp probs");
    if (!s) s = grow_dev(c, &w->d_best, &w->c_best, 2 * std::max<size_t>(P, 1), "pnp best");
    if (!s) s = grow_host(c, &w->h_probs, &w->ch_probs, std::max<size_t>(P, 1), "pnp h probs");
    if (!s) s = grow_host(c, &w->h_best, &w->ch_best, 2 * std::max<size_t>(P, 1), "pnp h best");
    if (!s && P > w->c_res) {
        const size_t n = std::max<size_t>(P, 1);
        const size_t bytes = n * (sizeof(PnpRep) + sizeof(PnpModel));
        static_assert(sizeof(PnpRep) % alignof(PnpModel) == 0, "results block alignment");
        if (w->d_res) (void)hipFree(w->d_res);
        if (w->h_res) (void)hipHostFree(w->h_res);
        w->d_res = w->h_res = nullptr;
        w->c_res = 0;
        s = check_hip(c, hipMalloc((void**)&w->d_res, bytes), "pnp results");
        if (!s) s = check_hip(c, hipHostMalloc((void**)&w->h_res, bytes, hipHostMallocDefault), "pnp h results");
        if (s) return s;
        w->c_res = n;
        w->d_rep = reinterpret_cast<PnpRep*>(w->d_res);
        w->d_out = reinterpret_cast<PnpModel*>(w->d_res + n * sizeof(PnpRep));
        w->h_rep = reinterpret_cast<PnpRep*>(w->h_res);
        w->h_out = reinterpret_cast<PnpModel*>(w->h_res + n * sizeof(PnpRep));
    }
    return s;
}

struct PnpResult {
    int count = 0;
    int ok = 0;
    int n_inliers = 0;
    int iters = 0;
    PnpModel model{};
};

// grow the hypothesis arrays (good, models) to `need` slots, keeping the first `keep` models
static rgbd_status grow_hyp(rgbd_ctx* c, PnpWS* w, size_t need, size_t keep)
{
    if (need <= w->c_good) return RGBD_OK;
    const size_t n = std::max(need, w->c_good * 2);
    int* ng = nullptr;
    PnpModel* nm = nullptr;
    rgbd_status s = check_hip(c, hipMalloc((void**)&ng, n * sizeof(int)), "pnp good");
    if (!s) s = check_hip(c, hipMalloc((void**)&nm, n * sizeof(PnpModel)), "pnp models");
    if (!s && keep > 0) {
        s = check_hip(c, hipMemcpyAsync(nm, w->d_models, keep * sizeof(PnpModel), hipMemcpyDeviceToDevice, ws_stream(c, w)), "pnp models copy");
        if (!s) s = check_hip(c, hipStreamSynchronize(ws_stream(c, w)), "sync");
    }
    if (s) {
        if (ng) (void)hipFree(ng);
        if (nm) (void)hipFree(nm);
        return s;
    }
    if (w->d_good) (void)hipFree(w->d_good);
    if (w->d_models) (void)hipFree(w->d_models);
    w->d_good = ng;
    w->d_models = nm;
    w->c_good = w->c_models = n;
    return RGBD_OK;
}

static void adapt_chunk(rgbd_ctx* c, const PnpResult* res, int P)
{
    std::vector<int> it;
    it.reserve(P);
    for (int p = 0; p < P; p++)
        if (res[p].count >= kPnpModel) it.push_back(res[p].iters);
    if (it.empty()) return;
    auto pct = [&](int q) {
        const size_t k = std::min(it.size() - 1, (it.size() * q) / 100);
        std::nth_element(it.begin(), it.begin() + k, it.end());
        return it[k];
    };
    const int k0 = std::min(kPnpChunkMax, std::max(kPnpChunkMin, pct(90) + 1));
    const int k1 = std::min(kPnpChunkMax, std::max(kPnpChunkMin, (pct(99) + 2 - k0 + 3) & ~3));
    c->pnp_chunk = k0;
    c->pnp_chunk2 = k1;
}

// solvePnPRansac over the P problems resident in w->d_p3 / d_p2 / d_probs.  First chunk entirely on
// the device (subsets, hypotheses, replay, refinement) with one synchronisation; problems whose
// replay needs more iterations continue on the host in doubling chunks.  Results in res[P]
// (res[p].count too); masks stay in w->d_mask.
// pnp_launch enqueues the first chunk (subsets, hypotheses, replay, refinement) and the read-back,
// and records w->ev; pnp_finish waits for that event only (not for later work on the stream).
// the first chunk's subsets (k_pnp_sample) on stream st: the chunk sizes are fixed here for the whole solve
static rgbd_status pnp_sample_launch(rgbd_ctx* c, PnpWS* w, int P, const rgbd_pnp_params& prm, hipStream_t st)
{
    if (c->pnp_chunk <= 0) c->pnp_chunk = kPnpFirstChunk;
    if (c->pnp_chunk2 <= 0) c->pnp_chunk2 = kPnpFirstChunk2;
    w->k0 = c->pnp_chunk;
    w->k1 = c->pnp_chunk2;
    const PnpPrm dp{prm.iterations, prm.min_matches, w->k0, w->k1, prm.confidence};
    const int H01 = P * (w->k0 + w->k1);
    w->h01 = H01;   // pnp_finish's host continuation writes its hypotheses after both chunks
    rgbd_status s = grow_hyp(c, w, (size_t)std::max(H01, 1), 0);
    if (!s) s = grow_dev(c, &w->d_hprob, &w->c_hprob, (size_t)std::max(H01, 1), "pnp hprob");
    if (!s) s = grow_dev(c, &w->d_samples, &w->c_samples, (size_t)std::max(H01, 1) * kPnpModel, "pnp samples");
    if (s) return s;
    const int tk = timer_begin(c, "k_pnp_sample", st);
    RGBD_TRY(c, launch_pnp_sample(w->d_probs, P, dp, w->d_samples, w->d_hprob, w->d_rep, st), "pnp_sample");
    timer_end(c, tk);
    w->sampled = true;
    return RGBD_OK;
}

static rgbd_status pnp_launch(rgbd_ctx* c, PnpWS* w, int P, const PnpCam& cam, const rgbd_pnp_params& prm)
{
    const hipStream_t st = ws_stream(c, w);
    const float thr = (float)((double)prm.reprojection_error * (double)prm.reprojection_error);
    rgbd_status s = RGBD_OK;
    if (!w->sampled && (s = pnp_sample_launch(c, w, P, prm, st))) return s;
    w->sampled = false;
    const int K0 = w->k0, K1 = w->k1;
    const PnpPrm dp{prm.iterations, prm.min_matches, K0, K1, prm.confidence};
    const int H0 = P * K0;
    int tk = timer_begin(c, "k_pnp_hyp", st);
    RGBD_TRY(c, launch_pnp_hyp(w->d_p3, w->d_p2, w->d_probs, w->d_hprob, w->d_samples, cam, thr, H0, w->d_good, w->d_models, st), "pnp_hyp");
    timer_end(c, tk);
#ifdef RGBD_PNP_PROFILE
    pnp_prof_dump((H0 + 4) / 5, st);
#endif
    tk = timer_begin(c, "k_pnp_replay", st);
    RGBD_TRY(c, launch_pnp_replay(w->d_good, P, dp, w->d_rep, w->d_best, st), "pnp_replay");
    timer_end(c, tk);
    // the second chunk for the problems still short of niters (the others' workgroups exit at once)
    tk = timer_begin(c, "k_pnp_sample", st);
    RGBD_TRY(c, launch_pnp_sample2(P, dp, w->d_samples + (size_t)H0 * kPnpModel, w->d_hprob + H0, w->d_rep, st), "pnp_sample2");
    timer_end(c, tk);
    tk = timer_begin(c, "k_pnp_hyp", st);
    RGBD_TRY(c, launch_pnp_hyp(w->d_p3, w->d_p2, w->d_probs, w->d_hprob + H0, w->d_samples + (size_t)H0 * kPnpModel, cam, thr,
                   P * K1, w->d_good + H0, w->d_models + H0, st), "pnp_hyp");
    timer_end(c, tk);
    tk = timer_begin(c, "k_pnp_replay", st);
    RGBD_TRY(c, launch_pnp_replay2(w->d_good, H0, P, dp, w->d_rep, w->d_best, st), "pnp_replay2");
    timer_end(c, tk);
    tk = timer_begin(c, "k_pnp_refine", st);
    RGBD_TRY(c, launch_pnp_refine(w->d_p3, w->d_p2, w->d_probs, w->d_best, w->d_best + P, w->d_models, cam, thr, P, w->d_mask,
                      w->d_out, st), "pnp_refine");
    timer_end(c, tk);
    // replay states and refined models in one copy
    s = check_hip(c, hipMemcpyAsync(w->h_res, w->d_res, w->c_res * (sizeof(PnpRep) + sizeof(PnpModel)),
                                        hipMemcpyDeviceToHost, st), "results");
    if (!s && !w->ev) s = check_hip(c, hipEventCreateWithFlags(&w->ev, hipEventDisableTiming), "pnp event");
    if (!s) s = check_hip(c, hipEventRecord(w->ev, st), "pnp event record");
    return s;
}

static rgbd_status pnp_finish(rgbd_ctx* c, PnpWS* w, int P, const PnpCam& cam, const rgbd_pnp_params& prm,
                              PnpResult* res)
{
    const hipStream_t st = ws_stream(c, w);
    const float thr = (float)((double)prm.reprojection_error * (double)prm.reprojection_error);
    const int H0 = w->h01;   // hypothesis slots of the two device chunks
    rgbd_status s = check_hip(c, hipEventSynchronize(w->ev), "pnp wait");
    if (s) return s;
    int tk = 0;
    std::vector<int> todo;
    for (int p = 0; p < P; p++) {
        const PnpRep& r = w->h_rep[p];
        res[p] = PnpResult{};
        res[p].count = r.count;
        if (!r.done) {
            todo.push_back(p);
            continue;
        }
        const bool ok = r.best >= 0 && r.maxGood > 0;
        res[p].ok = ok ? 1 : 0;
        res[p].n_inliers = ok ? r.maxGood : 0;
        res[p].iters = r.iter;
        if (ok) res[p].model = w->h_out[p];
    }
    if (todo.empty()) {
        adapt_chunk(c, res, P);
        return RGBD_OK;
    }

    // ---- host continuation (solvePnPRansac still iterating after the first chunk)
    struct Run {
        int p = 0, count = 0, niters = 0, iter = 0, evaluated = 0, maxGood = 0, best = -1, chunk = 0;
        CvRng rng;
        std::vector<int> slot;   // global hypothesis slot of each evaluated iteration >= K0 ... (by index)
    };
    std::vector<Run> run;
    for (int p : todo) {
        const PnpRep& r = w->h_rep[p];
        Run u;
        u.p = p;
        u.count = r.count;
        u.niters = r.niters;
        u.iter = r.iter;
        u.evaluated = r.nh;
        u.maxGood = r.maxGood;
        u.best = r.best;
        u.chunk = 2 * w->k1;
        u.rng.state = r.rng;
        run.push_back(u);
    }
    int Htot = H0;
    size_t nactive = run.size();
    while (nactive > 0) {
        int H = 0;
        for (const Run& u : run)
            if (u.iter < u.niters) H += std::min(u.chunk, u.niters - u.evaluated);
        s = grow_host(c, &w->h_hprob, &w->ch_hprob, (size_t)H, "pnp h hprob");
        if (!s) s = grow_host(c, &w->h_samples, &w->ch_samples, (size_t)H * kPnpModel, "pnp h samples");
        if (!s) s = grow_host(c, &w->h_good, &w->ch_good, (size_t)H, "pnp h good");
        if (!s) s = grow_dev(c, &w->d_hprob, &w->c_hprob, (size_t)H, "pnp hprob");
        if (!s) s = grow_dev(c, &w->d_samples, &w->c_samples, (size_t)H * kPnpModel, "pnp samples");
        if (!s) s = grow_hyp(c, w, (size_t)Htot + H, (size_t)Htot);
        if (s) return s;
        int h = 0;
        for (Run& u : run) {
            if (u.iter >= u.niters) continue;
            const int k = std::min(u.chunk, u.niters - u.evaluated);
            u.slot.assign(k, 0);
            for (int i = 0; i < k; i++, h++) {
                w->h_hprob[h] = u.p;
                draw_subset(u.rng, u.count, &w->h_samples[(size_t)h * kPnpModel]);
                u.slot[i] = Htot + h;
            }
            u.chunk *= 2;
        }
        s = check_hip(c, hipMemcpyAsync(w->d_hprob, w->h_hprob, (size_t)H * 4, hipMemcpyHostToDevice, st), "hprob");
        if (!s) s = check_hip(c, hipMemcpyAsync(w->d_samples, w->h_samples, (size_t)H * kPnpModel * 4, hipMemcpyHostToDevice, st), "samples");
        if (s) return s;
        tk = timer_begin(c, "k_pnp_hyp", st);
        RGBD_TRY(c, launch_pnp_hyp(w->d_p3, w->d_p2, w->d_probs, w->d_hprob, w->d_samples, cam, thr, H, w->d_good + Htot,
                       w->d_models + Htot, st), "pnp_hyp");
        timer_end(c, tk);
        s = check_hip(c, hipMemcpyAsync(w->h_good, w->d_good + Htot, (size_t)H * 4, hipMemcpyDeviceToHost, st), "good");
        if (!s) s = check_hip(c, hipStreamSynchronize(st), "sync");
        if (s) return s;
        for (Run& u : run) {   // replay (RANSACPointSetRegistrator::run)
            if (u.iter >= u.niters) continue;
            const int first = u.evaluated;
            u.evaluated += (int)u.slot.size();
            while (u.iter < u.niters && u.iter < u.evaluated) {
                const int slot = u.slot[u.iter - first];
                const int g = w->h_good[slot - Htot];
                if (g >= 0 && g > std::max(u.maxGood, kPnpModel - 1)) {
                    u.maxGood = g;
                    u.best = slot;
                    u.niters = update_num_iters(prm.confidence, (double)(u.count - g) / u.count, kPnpModel, u.niters);
                }
                u.iter++;
            }
            if (u.iter >= u.niters) nactive--;
        }
        Htot += H;
    }
    for (int p = 0; p < P; p++) w->h_best[p] = -1, w->h_best[P + p] = 0;
    for (const Run& u : run) {
        const bool ok = u.best >= 0 && u.maxGood > 0;
        w->h_best[u.p] = ok ? u.best : -1;
        res[u.p].ok = ok ? 1 : 0;
        res[u.p].n_inliers = ok ? u.maxGood : 0;
        res[u.p].iters = u.iter;
    }
    s = check_hip(c, hipMemcpyAsync(w->d_best, w->h_best, (size_t)2 * P * 4, hipMemcpyHostToDevice, st), "best");
    if (s) return s;
    tk = timer_begin(c, "k_pnp_refine", st);
    RGBD_TRY(c, launch_pnp_refine(w->d_p3, w->d_p2, w->d_probs, w->d_best, w->d_best + P, w->d_models, cam, thr, P, w->d_mask,
                      w->d_out, st), "pnp_refine");
    timer_end(c, tk);
    s = check_hip(c, hipMemcpyAsync(w->h_out, w->d_out, (size_t)P * sizeof(PnpModel), hipMemcpyDeviceToHost, st), "out");
    if (!s) s = check_hip(c, hipStreamSynchronize(st), "sync");
    if (s) return s;
    for (const Run& u : run)
        if (res[u.p].ok) res[u.p].model = w->h_out[u.p];
    adapt_chunk(c, res, P);
    return RGBD_OK;
}

static rgbd_status pnp_solve(rgbd_ctx* c, PnpWS* w, int P, const PnpCam& cam, const rgbd_pnp_params& prm,
                             PnpResult* res)
{
    rgbd_status s = pnp_launch(c, w, P, cam, prm);
    return s ? s : pnp_finish(c, w, P, cam, prm, res);
}

static void matmul4(const float* A, const float* B, float* C)   // cv::Mat 32F gemm: double accumulation
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0.0;
            for (int k = 0; k < 4; k++) s += (double)A[4 * i + k] * (double)B[4 * k + j];
            C[4 * i + j] = (float)s;
        }
}

}  // namespace rgbd

extern "C" {

rgbd_status rgbd_pnp_ransac_batch(rgbd_ctx* c, int32_t P, const int32_t* counts, const float* p3, const float* p2,
                                  const float* K4, const rgbd_pnp_params* prm, double* R9, double* t3,
                                  uint8_t* masks, int32_t* n_inliers, int32_t* iters_run, int32_t* ok)
{
    if (!c || P < 0 || !counts || !K4 || !prm || !R9 || !t3 || !n_inliers || !ok) return RGBD_ERR_ARG;
    size_t npts = 0;
    for (int p = 0; p < P; p++) {
        if (counts[p] < 0) return fail(c, RGBD_ERR_ARG, "negative point count");
        if (counts[p] > kPnpMaxM) return fail(c, RGBD_ERR_UNSUPPORTED, "more than 4096 correspondences per problem");
        npts += (size_t)counts[p];
    }
    if (npts > 0 && (!p3 || !p2)) return RGBD_ERR_ARG;
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    PnpWS* w = pnp_ws(c);
    if ((s = ws_points(c, w, npts, (size_t)P))) return s;
    size_t off = 0;
    for (int p = 0; p < P; p++) {
        w->h_probs[p] = PnpProbDev{(int)off, counts[p]};
        off += (size_t)counts[p];
    }
    const hipStream_t st = c->stream;
    if (npts > 0) {
        s = check_hip(c, hipMemcpyAsync(w->d_p3, p3, npts * 12, hipMemcpyHostToDevice, st), "p3");
        if (!s) s = check_hip(c, hipMemcpyAsync(w->d_p2, p2, npts * 8, hipMemcpyHostToDevice, st), "p2");
    }
    if (!s && P > 0) s = check_hip(c, hipMemcpyAsync(w->d_probs, w->h_probs, (size_t)P * sizeof(PnpProbDev), hipMemcpyHostToDevice, st), "probs");
    if (s) return s;
    const PnpCam cam{K4[0], K4[1], K4[2], K4[3]};
    std::vector<PnpResult> res(P);
    if ((s = pnp_solve(c, w, P, cam, *prm, res.data()))) return s;
    if (masks && npts > 0) {
        s = check_hip(c, hipMemcpyAsync(masks, w->d_mask, npts, hipMemcpyDeviceToHost, st), "mask");
        if (!s) s = check_hip(c, hipStreamSynchronize(st), "sync");
        if (s) return s;
    }
    off = 0;
    for (int p = 0; p < P; p++) {
        const PnpResult& r = res[p];
        ok[p] = r.ok;
        n_inliers[p] = r.n_inliers;
        if (iters_run) iters_run[p] = r.iters;
        for (int i = 0; i < 9; i++) R9[9 * p + i] = r.ok ? r.model.R[i] : ((i % 4 == 0) ? 1.0 : 0.0);
        for (int i = 0; i < 3; i++) t3[3 * p + i] = r.ok ? r.model.t[i] : 0.0;
        if (masks && !r.ok) std::memset(masks + off, 0, (size_t)counts[p]);
        off += (size_t)counts[p];
    }
    return RGBD_OK;
}

rgbd_status rgbd_pnp_ransac(rgbd_ctx* c, const float* p3, const float* p2, int32_t count, const float* K4,
                            const rgbd_pnp_params* prm, double* R9, double* t3, uint8_t* mask, int32_t* n_inliers,
                            int32_t* iters_run, int32_t* ok)
{
    return rgbd_pnp_ransac_batch(c, 1, &count, p3, p2, K4, prm, R9, t3, mask, n_inliers, iters_run, ok);
}

}  // extern "C"

namespace rgbd {

// extract + match + the device part of PnPRansac for B frames into workspace w (no host wait).
// Outlier-flag chain (prm.flag_segments > 0): extraction and knn-2, then the whole chain (filter, gather,
// solve and flags of every pair) in one k_pnp_chain launch (flag_chain_launch); collect reads the results.
static rgbd_status match_launch(rgbd_ctx* c, PnpWS* w, int B, float nnratio, int segments, PnpPipe* pp, int set);
static rgbd_status flag_chain_launch(rgbd_ctx* c, PnpWS* w, const OutSet& o, int B, float nnratio,
                                     const rgbd_pnp_params& prm);

// A pipelined step's knn-2 + gather runs on the match stream right after the step's own extraction (beside
// the next step's pyramid), the stream at the lowest priority (+0.19 % / +0.22 % in two r04 A/Bs).  Measured
// and removed (r04): the knn-2 + gather at the next submission's pyramid / FAST hook (-1.9 %,
// profiles/r04_ab_match_at) and the first subsets drawn on the match stream (-0.02 %, profiles/r04_ab_sample_early).
// The deferred solves launch at extraction hook 1 (after FAST; after the pyramid / the quadtree -1.2 % / -0.5 %,
// profiles/r04_ab_solve_at2).
constexpr int kSolveAt = 1;

static rgbd_status track_submit(rgbd_ctx* c, PnpWS* w, const void* d_bgr, const void* d_depth, int B, float nnratio,
                                const rgbd_pnp_params& prm, const ExtractHook* after_fast = nullptr,
                                PnpPipe* pp = nullptr, int set = 0)
{
    const int segments = prm.flag_segments;
    const int K = c->cfg.kp_cap;
    if (K > kPnpMaxM) return fail(c, RGBD_ERR_UNSUPPORTED, "keypoint capacity above 4096 for PnPRansac");
    rgbd_status s = extract_batch(c, d_bgr, d_depth, B, after_fast);
    if (s) return s;
    // per-frame capacity flags of this extraction, read by collect (ordered before every later event)
    if ((s = grow_host(c, &w->h_err, &w->ch_err, (size_t)B, "pnp h err"))) return s;
    if ((s = check_hip(c, hipMemcpyAsync(w->h_err, c->d_err, (size_t)B * 4, hipMemcpyDeviceToHost, c->stream), "err")))
        return s;
    // pipelined: knn-2 + gather on the match stream, after this extraction (event)
    if (pp && (s = check_hip(c, hipEventRecord(pp->ev_desc, c->stream), "extraction event"))) return s;
    const OutSet o = pp ? pp->set[set] : ctx_outputs(c);
    if ((s = match_launch(c, w, B, nnratio, segments, pp, set))) return s;
    return segments > 0 ? flag_chain_launch(c, w, o, B, nnratio, prm) : RGBD_OK;
}

// knn-2 (+ the Matcher filter and 3D-2D gather) of a submission's consecutive pairs, reading output set
// `set` (pipelined: on the match stream, after the extraction that wrote the set)
static rgbd_status match_launch(rgbd_ctx* c, PnpWS* w, int B, float nnratio, int segments, PnpPipe* pp, int set)
{
    const int K = c->cfg.kp_cap;
    rgbd_status s = RGBD_OK;
    hipStream_t st = c->stream;
    OutSet cur{};
    if (pp) {
        s = check_hip(c, hipStreamWaitEvent(c->match_stream, pp->ev_desc, 0), "extraction wait");
        if (s) return s;
        st = c->match_stream;
        cur = ctx_outputs(c);
        set_ctx_outputs(c, pp->set[set]);
    }
    struct Restore {
        rgbd_ctx* c; PnpPipe* pp; OutSet o;
        ~Restore() { if (pp) set_ctx_outputs(c, o); }
    } restore{c, pp, cur};
    const int P = B - 1;
    if (P == 0) return RGBD_OK;
    if (!w->d_cpairs) {   // written once: the layout does not depend on B
        std::vector<int> pairs(2 * (size_t)c->maxB, 0);
        for (int p = 0; p + 1 < c->maxB; p++) {
            pairs[p] = p;                 // query = reference frame b-1
            pairs[c->maxB + p] = p + 1;   // train = current frame b
        }
        s = check_hip(c, hipMalloc((void**)&w->d_cpairs, pairs.size() * 4), "pnp pairs");
        if (!s) s = check_hip(c, hipMemcpy(w->d_cpairs, pairs.data(), pairs.size() * 4, hipMemcpyHostToDevice), "pairs");
        if (s) return s;
    }
    int tk = timer_begin(c, "k_knn2", st);
    RGBD_TRY(c, launch_knn2(c->d_desc, c->d_count, w->d_cpairs, w->d_cpairs + c->maxB, K, K, c->d_knn, P, st), "knn2");
    timer_end(c, tk);
    if (segments > 0) {   // the flag chain waits for the knn-2 rows (flag_chain_launch)
        if (!w->ev_in) s = check_hip(c, hipEventCreateWithFlags(&w->ev_in, hipEventDisableTiming), "pnp knn event");
        if (!s) s = check_hip(c, hipEventRecord(w->ev_in, st), "pnp knn record");
        return s;
    }
    if ((s = ws_points(c, w, (size_t)P * K, (size_t)P))) return s;
    if ((s = grow_dev(c, &w->d_mq, &w->c_mq, (size_t)P * K, "pnp mq"))) return s;
    if ((s = grow_dev(c, &w->d_mt, &w->c_mt, (size_t)P * K, "pnp mt"))) return s;
    tk = timer_begin(c, "k_match_gather", st);
    RGBD_TRY(c, launch_match_gather(c->d_knn, c->d_count, w->d_cpairs, w->d_cpairs + c->maxB, c->d_xyz, c->d_kun, K, nnratio, P,
                        w->d_p3, w->d_p2, w->d_probs, w->d_mq, w->d_mt, st), "match_gather");
    timer_end(c, tk);
    // pipelined: the first chunk's subsets right behind the gather on this stream, so the solve stream's
    // chain starts at the hypotheses (a one-workgroup kernel launched beside the quadtree waits for a
    // free wave slot)
    if (w->st && w->st != st) {   // the solve waits for this step's gather (pnp_solve_launch)
        if (!w->ev_in) s = check_hip(c, hipEventCreateWithFlags(&w->ev_in, hipEventDisableTiming), "pnp gather event");
        if (!s) s = check_hip(c, hipEventRecord(w->ev_in, st), "pnp gather record");
    }
    if (!s && pp) s = check_hip(c, hipEventRecord(pp->ev_free[set], st), "output set free record");
    return s;
}

// enqueue the device part of PnPRansac for a gathered step: on the workspace's stream, after its
// gather (and after `also`, an event of the launch stream, when given)
static rgbd_status pnp_solve_launch(rgbd_ctx* c, PnpWS* w, int P, const rgbd_pnp_params& prm, hipEvent_t also = nullptr)
{
    if (P == 0) return RGBD_OK;
    rgbd_status s = RGBD_OK;
    if (w->st && w->st != c->stream) {
        s = check_hip(c, hipStreamWaitEvent(w->st, w->ev_in, 0), "pnp gather wait");
        if (!s && also) s = check_hip(c, hipStreamWaitEvent(w->st, also, 0), "pnp launch-stream wait");
        if (s) return s;
    }
    const PnpCam cam{c->cam.fx, c->cam.fy, c->cam.cx, c->cam.cy};
    return pnp_launch(c, w, P, cam, prm);
}

// The reference's outlier-flag chain around PnPRansac (Features/Matcher.cpp:125-128 with
// discardOutliers = true; Solver/PnPRansac.cpp:31,51): pair b's Matcher filter skips the queries that
// pair b-1's PnPRansac flagged on frame b.  The B-1 pairs are split into `segments` contiguous runs, each
// an exact chain of the reference's; a run's first pair reads the cleared flags of a fresh frame
// (segments = 1: the reference's single chain).  One k_pnp_chain launch (one workgroup per run) after the
// knn-2 rows, then one read-back of every pair's result (w->ev).
static rgbd_status flag_chain_launch(rgbd_ctx* c, PnpWS* w, const OutSet& o, int B, float nnratio,
                                     const rgbd_pnp_params& prm)
{
    const int K = c->cfg.kp_cap;
    const int P = B - 1;
    if (P <= 0) return RGBD_OK;
    const int S = std::max(1, std::min(prm.flag_segments, P));
    const hipStream_t st = ws_stream(c, w);
    rgbd_status s = grow_host(c, &w->h_seg, &w->ch_seg, (size_t)S + 1, "flag runs h");
    if (!s) s = grow_dev(c, &w->d_seg, &w->c_seg, (size_t)S + 1, "flag runs");
    if (!s) s = grow_host(c, &w->h_cres, &w->ch_cres, (size_t)P, "flag results h");
    if (!s) s = grow_dev(c, &w->d_cres, &w->c_cres, (size_t)P, "flag results");
    if (!s) s = grow_dev(c, &w->d_flags, &w->c_flags, (size_t)B * K, "flags");
    if (!s) s = ws_points(c, w, (size_t)P * K, (size_t)P);
    if (!s) s = grow_dev(c, &w->d_mq, &w->c_mq, (size_t)P * K, "pnp mq");
    if (!s) s = grow_dev(c, &w->d_mt, &w->c_mt, (size_t)P * K, "pnp mt");
    if (!s) s = grow_hyp(c, w, (size_t)P, 0);
    if (s) return s;
    // the first kChainRngTab raw outputs of cv::RNG((uint64)-1), shared by every solvePnPRansac call
    CvRng gen;
    if (!w->d_rngtab) {
        std::vector<uint32_t> tab(kChainRngTab);
        for (int j = 0; j < kChainRngTab; j++) tab[j] = gen.next();
        s = check_hip(c, hipMalloc((void**)&w->d_rngtab, tab.size() * 4), "rng table");
        if (!s) s = check_hip(c, hipMemcpy(w->d_rngtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice), "rng table");
        if (s) return s;
    } else {
        for (int j = 0; j < kChainRngTab; j++) (void)gen.next();
    }
    for (int k = 0; k <= S; k++) w->h_seg[k] = (int)(((long long)P * k) / S);
    if (w->st && w->st != c->stream) {   // after this submission's knn-2 (match_launch)
        if ((s = check_hip(c, hipStreamWaitEvent(st, w->ev_in, 0), "flag knn wait"))) return s;
    }
    s = check_hip(c, hipMemcpyAsync(w->d_seg, w->h_seg, (size_t)(S + 1) * 4, hipMemcpyHostToDevice, st), "flag runs");
    if (!s) s = check_hip(c, hipMemsetAsync(w->d_flags, 0, (size_t)B * K, st), "flags clear");   // fresh frames
    if (s) return s;
    const PnpCam cam{c->cam.fx, c->cam.fy, c->cam.cx, c->cam.cy};
    const float thr = (float)((double)prm.reprojection_error * (double)prm.reprojection_error);
    const PnpPrm dp{prm.iterations, prm.min_matches, 0, 0, prm.confidence};
    const int tk = timer_begin(c, "k_pnp_chain", st);
    RGBD_TRY(c, launch_pnp_chain(o.knn, o.count, o.xyz, o.kun, K, nnratio, w->d_seg, S, cam, thr, dp, w->d_p3, w->d_p2, w->d_mq,
                     w->d_mt, w->d_mask, w->d_flags, w->d_cres, w->d_rngtab, kChainRngTab,
                     (unsigned long long)gen.state, w->d_probs, w->d_best, w->d_models, P, st), "pnp_chain");
    timer_end(c, tk);
    // every pair's Gauss-Newton refinement, off the chain's critical path
    const int tr = timer_begin(c, "k_pnp_refine", st);
    RGBD_TRY(c, launch_pnp_refine(w->d_p3, w->d_p2, w->d_probs, w->d_best, w->d_best + P, w->d_models, cam, thr, P, w->d_mask,
                      w->d_out, st), "pnp_refine");
    timer_end(c, tr);
    s = check_hip(c, hipMemcpyAsync(w->h_cres, w->d_cres, (size_t)P * sizeof(PnpChainRes), hipMemcpyDeviceToHost, st),
                  "flag results");
    if (!s)
        s = check_hip(c, hipMemcpyAsync(w->h_out, w->d_out, (size_t)P * sizeof(PnpModel), hipMemcpyDeviceToHost, st),
                      "flag models");
    if (!s && !w->ev) s = check_hip(c, hipEventCreateWithFlags(&w->ev, hipEventDisableTiming), "pnp event");
    if (!s) s = check_hip(c, hipEventRecord(w->ev, st), "pnp event record");
    return s;
}

static rgbd_status flag_chain_finish(rgbd_ctx* c, PnpWS* w, int P, PnpResult* res)
{
    rgbd_status s = check_hip(c, hipEventSynchronize(w->ev), "flag chain wait");
    if (s) return s;
#ifdef RGBD_PNP_PROFILE
    chain_prof_dump(ws_stream(c, w));
    pnp_prof_dump(1, ws_stream(c, w));   // the stages of run 0's last hypothesis and refinement
#endif
    for (int p = 0; p < P; p++) {
        const PnpChainRes& r = w->h_cres[p];
        res[p] = PnpResult{};
        res[p].count = r.count;
        res[p].ok = r.ok;
        res[p].n_inliers = r.n_inliers;
        res[p].iters = r.iters;
        if (r.ok) res[p].model = w->h_out[p];
    }
    return RGBD_OK;
}

// waits for a submission's read-back, finishes its RANSAC (or runs the flag chain), chains the poses
static rgbd_status track_collect(rgbd_ctx* c, PnpWS* w, int B, float nnratio, const rgbd_pnp_params& prm,
                                 const OutSet& o, float* poses, int32_t* status, int32_t* n_inliers,
                                 int32_t* n_matches)
{
    const int P = B - 1;
    status[0] = 1;
    if (n_inliers) n_inliers[0] = 0;
    if (n_matches) n_matches[0] = 0;
    const PnpCam cam{c->cam.fx, c->cam.fy, c->cam.cx, c->cam.cy};
    std::vector<PnpResult> res(std::max(P, 1));
    rgbd_status s = RGBD_OK;
    if (P == 0)
        s = check_hip(c, hipStreamSynchronize(c->stream), "sync");
    else if (prm.flag_segments > 0)
        s = flag_chain_finish(c, w, P, res.data());
    else
        s = pnp_finish(c, w, P, cam, prm, res.data());
    if (s) return s;
    for (int b = 0; b < B; b++)   // the extraction's per-frame flags (copied before the solve's events)
        if (w->h_err[b]) return fail(c, RGBD_ERR_CAPACITY, (w->h_err[b] & 2)
                                     ? "SVO: keypoints kept by retainBest exceed rgbd_max_keypoints"
                                     : "quadtree node capacity exceeded");
    for (int b = 1; b < B; b++) {
        const PnpResult& r = res[b - 1];
        if (r.ok) {
            float T[16];
            for (int i = 0; i < 3; i++) {
                for (int j = 0; j < 3; j++) T[4 * i + j] = (float)r.model.R[3 * i + j];
                T[4 * i + 3] = (float)r.model.t[i];
            }
            T[12] = T[13] = T[14] = 0.0f;
            T[15] = 1.0f;
            matmul4(T, &poses[(size_t)(b - 1) * 16], &poses[(size_t)b * 16]);   // T21 * pose(F1)
        } else {
            std::memcpy(&poses[(size_t)(b - 1) * 16 + 16], &poses[(size_t)(b - 1) * 16], 64);   // recover()
        }
        status[b] = r.ok;
        if (n_inliers) n_inliers[b] = r.n_inliers;
        if (n_matches) n_matches[b] = r.count;
    }
    return RGBD_OK;
}

}  // namespace rgbd

extern "C" {

rgbd_status rgbd_pnp_track_batch(rgbd_ctx* c, const void* d_bgr, const void* d_depth, int32_t B, float nnratio,
                                 const rgbd_pnp_params* prm, float* poses, int32_t* status, int32_t* n_inliers,
                                 int32_t* n_matches)
{
    if (!c || !d_bgr || !d_depth || B < 1 || !prm || !poses || !status || prm->flag_segments < 0) return RGBD_ERR_ARG;
    if (B > c->maxB) return fail(c, RGBD_ERR_CAPACITY, "batch larger than max_batch");
    PnpWS* w = pnp_ws(c);
    rgbd_status s = track_submit(c, w, d_bgr, d_depth, B, nnratio, *prm);
    if (!s && prm->flag_segments == 0) s = pnp_solve_launch(c, w, B - 1, *prm);
    return s ? s : track_collect(c, w, B, nnratio, *prm, ctx_outputs(c), poses, status, n_inliers, n_matches);
}

rgbd_status rgbd_pnp_track_submit(rgbd_ctx* c, const void* d_bgr, const void* d_depth, int32_t B, float nnratio,
                                  const rgbd_pnp_params* prm)
{
    if (!c || !d_bgr || !d_depth || B < 1 || !prm || prm->flag_segments < 0) return RGBD_ERR_ARG;
    if (B > c->maxB) return fail(c, RGBD_ERR_CAPACITY, "batch larger than max_batch");
    if (!c->pnp_pipe) c->pnp_pipe = new PnpPipe();
    PnpPipe* pp = static_cast<PnpPipe*>(c->pnp_pipe);
    if (pp->count >= kPipeDepth) return fail(c, RGBD_ERR_ARG, "three submissions outstanding: collect first");
    // flag chain: an output set is read until its collect's last round, so a set comes back only after
    // that collect (two output sets -> at most two outstanding)
    for (int k = 0; k < pp->count; k++)
        if ((pp->q[(pp->head + k) % kPipeDepth].prm.flag_segments > 0 || prm->flag_segments > 0) && pp->count >= 2)
            return fail(c, RGBD_ERR_ARG, "outlier-flag chain: at most two submissions outstanding");
    const int slot = (pp->head + pp->count) % kPipeDepth;
    rgbd_status s = RGBD_OK;
    if (!c->solve_stream) {   // highest priority: the solve is a short latency-bound chain (normal / low priority
                              // measured the same in round 4: profiles/r04_ab_solve_prio)
        int lo = 0, hi = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo, &hi);   // hi = numerically lowest = most urgent
        s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
        if (!s && c->serial) c->solve_stream = c->own_stream;
        else if (!s) s = check_hip(c, hipStreamCreateWithPriority(&c->solve_stream, hipStreamNonBlocking, hi), "solve stream");
        if (!s) s = check_hip(c, hipEventCreateWithFlags(&pp->ev_fast, hipEventDisableTiming), "pipe event");
        if (s) return s;
    }
    if (!c->match_stream) {   // the second output set, the match stream and its events
        const size_t Bm = (size_t)c->maxB, K = (size_t)c->cfg.kp_cap;
        OutSet& a = pp->set[1];
        pp->set[0] = ctx_outputs(c);
        s = check_hip(c, hipMalloc((void**)&a.count, std::max<size_t>(Bm * 4, 16)), "set count");
        if (!s) s = check_hip(c, hipMalloc((void**)&a.kps, Bm * K * 28), "set kps");
        if (!s) s = check_hip(c, hipMalloc((void**)&a.kun, Bm * K * 28), "set kun");
        if (!s) s = check_hip(c, hipMalloc((void**)&a.desc, Bm * K * 32), "set desc");
        if (!s) s = check_hip(c, hipMalloc((void**)&a.xyz, Bm * K * 12), "set xyz");
        if (!s) s = check_hip(c, hipMalloc((void**)&a.knn, Bm * K * sizeof(int4)), "set knn");
        for (int k = 0; !s && k < 2; k++)
            s = check_hip(c, hipEventCreateWithFlags(&pp->ev_free[k], hipEventDisableTiming), "set event");
        if (!s) s = check_hip(c, hipEventCreateWithFlags(&pp->ev_desc, hipEventDisableTiming), "extraction event");
        if (!s && c->serial) c->match_stream = c->own_stream;
        else if (!s) {   // the match stream at the lowest priority
            int lo = 0, hi = 0;
            s = check_hip(c, hipDeviceGetStreamPriorityRange(&lo, &hi), "stream priorities");
            if (!s) s = check_hip(c, hipStreamCreateWithPriority(&c->match_stream, hipStreamNonBlocking, lo), "match stream");
        }
        if (s) return s;
    }
    // this submission's output set: wait until the gather that last read it has run
    const int set = pp->parity;
    pp->parity ^= 1;
    set_ctx_outputs(c, pp->set[set]);
    if ((s = check_hip(c, hipStreamWaitEvent(c->stream, pp->ev_free[set], 0), "output set wait"))) return s;
    if (!pp->ws[slot]) pp->ws[slot] = new PnpWS();
    pp->ws[slot]->st = c->solve_stream;
    // the solves still due (earlier submissions), in submission order, are launched right after this
    // step's k_fast is enqueued (launch point 1), so the f64 latency chains run beside the quadtree and the
    // description instead of beside the VALU-bound FAST.  Measured at B = 512 (round 1): launch points
    // before FAST / after FAST / after the quadtree 125.6k / 131.6k / 132.8k frames/s; at the end of round 2
    // with the faster FAST, after FAST 190.7k vs after the quadtree 188.5k (B = 1024); round 4 (faster quadtree):
    // after the pyramid / FAST / the quadtree 211.4-212.0k / 218.0-218.7k / 217.6-218.1k (profiles/r04_ab_solve_at)
    const ExtractHook launch_due = [c, pp](int at) -> rgbd_status {
        if (at != kSolveAt) return RGBD_OK;
        bool any = false;
        for (int k = 0; k < pp->count; k++) {
            const PnpPending& q = pp->q[(pp->head + k) % kPipeDepth];
            any = any || q.solve_due;
        }
        if (!any) return RGBD_OK;
        rgbd_status hs = check_hip(c, hipEventRecord(pp->ev_fast, c->stream), "pipe event record");
        for (int k = 0; !hs && k < pp->count; k++) {
            const int j = (pp->head + k) % kPipeDepth;
            if (!pp->q[j].solve_due) continue;
            hs = pnp_solve_launch(c, pp->ws[j], pp->q[j].P, pp->q[j].prm, pp->ev_fast);
            if (!hs) pp->q[j].solve_due = false;
        }
        return hs;
    };
    s = track_submit(c, pp->ws[slot], d_bgr, d_depth, B, nnratio, *prm, &launch_due, pp, set);
    if (s) return s;
    pp->q[slot].B = B;
    pp->q[slot].P = B - 1;
    pp->q[slot].prm = *prm;
    pp->q[slot].nnratio = nnratio;
    pp->q[slot].solve_due = B > 1 && prm->flag_segments == 0;
    pp->q[slot].out = pp->set[set];
    pp->q[slot].set = set;
    pp->count++;
    return RGBD_OK;
}

rgbd_status rgbd_pnp_track_collect(rgbd_ctx* c, float* poses, int32_t* status, int32_t* n_inliers, int32_t* n_matches)
{
    if (!c || !poses || !status) return RGBD_ERR_ARG;
    PnpPipe* pp = static_cast<PnpPipe*>(c->pnp_pipe);
    if (!pp || pp->count == 0) return fail(c, RGBD_ERR_ARG, "nothing submitted");
    const int slot = pp->head;
    PnpPending& q = pp->q[slot];
    if (q.solve_due) {   // no later submission launched it
        const rgbd_status s = pnp_solve_launch(c, pp->ws[slot], q.P, q.prm);
        if (s) return s;
        q.solve_due = false;
    }
    const PnpPending done = q;
    pp->head = (pp->head + 1) % kPipeDepth;
    pp->count--;
    rgbd_status s = track_collect(c, pp->ws[slot], done.B, done.nnratio, done.prm, done.out, poses, status, n_inliers,
                                  n_matches);
    if (done.prm.flag_segments > 0 && done.P > 0) {   // the flag rounds were the set's last readers
        const rgbd_status e = check_hip(c, hipEventRecord(pp->ev_free[done.set], ws_stream(c, pp->ws[slot])), "set free");
        if (!s) s = e;
    }
    return s;
}

}  // extern "C"

// solver.cpp -- RansacSE3 host control + the tracking front-end chain (C ABI).
//
// RansacSE3::compute (Solver/SolverSE3.cpp:23-133) is split in three:
//   host:   outlier marking (:38-42), std::sort by distance (:52, libstdc++ -- same algorithm as the
//           reference, unstable, ties decided by its comparison sequence), glibc-rand sample draws
//           (sampleMatches :135-159) for every iteration that may run, sticky depth covariance (:282)
//   device: k_ransac_hyp -- every iteration's refinement chain (:58-86) in parallel
//   host:   replay of the sequential accept / n += 10 / break logic (:88-102), the identity
//           fallback (:105-117), inlier flags (:119-122), and the RNG advanced by exactly the
//           samples the reference would have drawn.
// Tracking::visualOdometry (System/Tracking.cpp:121-163) over a device-resident batch runs entirely on the
// device (lanes_host.cpp); the host composes the poses and Tracking::track's bookkeeping from its results.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "context.h"
#include "lanes_host.h"
#include "launch.h"
#include "pnp_dev.h"
#include "ransac_dev.h"

using namespace rgbd;

namespace rgbd {

struct RansacWS {
    int capM = 0, capH = 0, MWcap = 0;
    // device: [pts 6*capM f32][samples capH*8 i32][scount capH i32] and [out capH HypOut][masks capH*MWcap u32]
    unsigned char* d_in = nullptr;
    unsigned char* d_res = nullptr;
    unsigned char* h_in = nullptr;    // pinned mirrors
    unsigned char* h_res = nullptr;
    size_t in_bytes = 0, res_bytes = 0;
    float* pts() { return reinterpret_cast<float*>(h_in); }
    int* samples() { return reinterpret_cast<int*>(h_in + (size_t)capM * 24); }
    int* scount() { return samples() + (size_t)capH * 8; }
    HypOut* out() { return reinterpret_cast<HypOut*>(h_res); }
    uint32_t* masks() { return reinterpret_cast<uint32_t*>(h_res + (size_t)capH * sizeof(HypOut)); }
    std::vector<rgbd_dmatch> used;
    std::vector<rgbd_rng> after;
};

static void ws_release(RansacWS* w)
{
    if (w->d_in) (void)hipFree(w->d_in);
    if (w->d_res) (void)hipFree(w->d_res);
    if (w->h_in) (void)hipHostFree(w->h_in);
    if (w->h_res) (void)hipHostFree(w->h_res);
    w->d_in = w->d_res = w->h_in = w->h_res = nullptr;
}

void ransac_free(rgbd_ctx* c)
{
    lanes_free(c);
    RansacWS* w = static_cast<RansacWS*>(c->ransac);
    if (!w) return;
    ws_release(w);
    delete w;
    c->ransac = nullptr;
}

static rgbd_status ransac_ws(rgbd_ctx* c, int M, int H, int SS, RansacWS** out)
{
    RansacWS* w = static_cast<RansacWS*>(c->ransac);
    if (!w) {
        w = new RansacWS();
        c->ransac = w;
    }
    const int needM = std::max(M, 1), needH = std::max(H, 1) + 1;
    if (needM > w->capM || needH > w->capH || SS > 8) {
        ws_release(w);
        w->capM = std::max(needM, std::max(w->capM, 1024));
        w->capH = std::max(needH, std::max(w->capH, 256));
        w->MWcap = (w->capM + 31) / 32 + 1;
        w->in_bytes = (size_t)w->capM * 24 + (size_t)w->capH * 8 * 4 + (size_t)w->capH * 4;
        w->res_bytes = (size_t)w->capH * sizeof(HypOut) + (size_t)w->capH * w->MWcap * 4;
        rgbd_status s = check_hip(c, hipMalloc((void**)&w->d_in, w->in_bytes), "ransac in");
        if (!s) s = check_hip(c, hipMalloc((void**)&w->d_res, w->res_bytes), "ransac res");
        if (!s) s = check_hip(c, hipHostMalloc((void**)&w->h_in, w->in_bytes, hipHostMallocDefault), "ransac pinned in");
        if (!s) s = check_hip(c, hipHostMalloc((void**)&w->h_res, w->res_bytes, hipHostMallocDefault), "ransac pinned res");
        if (s) return s;
    }
    *out = w;
    return RGBD_OK;
}

// glibc random_r TYPE_3 (System/Random.cpp:19 calls rand())
static int32_t rng_next(rgbd_rng* st)
{
    const uint32_t val = (uint32_t)st->state[st->f] + (uint32_t)st->state[st->r];
    st->state[st->f] = (int32_t)val;
    const int32_t result = (int32_t)(val >> 1);
    if (++st->f >= 31) {
        st->f = 0;
        ++st->r;
    } else if (++st->r >= 31) {
        st->r = 0;
    }
    return result;
}

// Random::randomInt, System/Random.cpp:16-20
static int random_int(rgbd_rng* st, int mn, int mx)
{
    const int d = mx - mn + 1;
    return int(((double)rng_next(st) / ((double)2147483647 + 1.0)) * d) + mn;
}

// RansacSE3::sampleMatches (:135-159): ids in std::set order (ascending, distinct)
static int sample_ids(rgbd_rng* st, int M, int SS, int* ids)
{
    int n = 0;
    int safety = 0;
    while (n < SS && M >= SS) {
        int id1 = random_int(st, 0, M - 1);
        const int id2 = random_int(st, 0, M - 1);
        if (id1 > id2) id1 = id2;
        int pos = 0;
        while (pos < n && ids[pos] < id1) pos++;
        if (pos == n || ids[pos] != id1) {
            for (int k = n; k > pos; k--) ids[k] = ids[k - 1];
            ids[pos] = id1;
            n++;
        }
        if (++safety > 10000) break;
    }
    return n;
}

static void raster_consts(double* rcx, double* rcy)
{
    const double cam_angle_x = 58.0 / 180.0 * M_PI;
    const double cam_angle_y = 45.0 / 180.0 * M_PI;
    const double sx = 3 * std::tan(cam_angle_x / 640.0);
    const double sy = 3 * std::tan(cam_angle_y / 480.0);
    *rcx = sx * sx;
    *rcy = sy * sy;
}

static const int kFirstChunk = 24;   // hypotheses evaluated before the first replay

struct RansacResult {
    bool ok = false;
    float T[16];
    float rmse = 1e6f;
    std::vector<rgbd_dmatch> inliers;
};

// RansacSE3::compute on host arrays
rgbd_status ransac_se3(rgbd_ctx* c, const float* xyz1, const float* xyz2, const rgbd_dmatch* m12, int m,
                       const rgbd_ransac_params& prm, rgbd_rng* rng, rgbd_sticky* sticky, bool update_f2,
                       uint8_t* flags2, RansacResult& R)
{
    R.ok = false;
    R.rmse = 1e6f;
    R.inliers.clear();
    for (int i = 0; i < 16; i++) R.T[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    if ((uint32_t)m < prm.min_inlier_th) return RGBD_OK;
    if (prm.sample_size > 8) return fail(c, RGBD_ERR_UNSUPPORTED, "sample_size > 8");
    if (m > kRansacMaxM) return fail(c, RGBD_ERR_UNSUPPORTED, "more than 2304 matches for RansacSE3");
    RansacWS* w = nullptr;
    const int M = m;
    const int SS = (int)prm.sample_size;
    const int H = (M >= SS) ? std::max(prm.iterations, 0) : 0;
    rgbd_status s = ransac_ws(c, M, H, std::max(SS, 1), &w);
    if (s) return s;
    std::vector<rgbd_dmatch>& used = w->used;
    used.assign(m12, m12 + m);
    if (update_f2 && flags2)
        for (int i = 0; i < m; i++) flags2[m12[i].trainIdx] = 1;
    std::sort(used.begin(), used.end(), [](const rgbd_dmatch& a, const rgbd_dmatch& b) { return a.distance < b.distance; });
    // gathered points in sorted order: (x1,y1,z1, x2,y2,z2), straight into pinned staging
    float* pts = w->pts();
    for (int j = 0; j < M; j++) {
        const float* o = xyz1 + 3 * (size_t)used[j].queryIdx;
        const float* t = xyz2 + 3 * (size_t)used[j].trainIdx;
        for (int k = 0; k < 3; k++) {
            pts[6 * j + k] = o[k];
            pts[6 * j + 3 + k] = t[k];
        }
    }
    // sticky depth covariance: first errorFunction2 call in the process (:282-287)
    if (!sticky->set) {
        for (int j = 0; j < M; j++) {
            const float* o = &pts[6 * j];
            const float* t = o + 3;
            if (o[2] == 0.0f || t[0] == 0.0f) continue;
            if (std::isnan(o[2]) || std::isnan(t[2])) continue;
            const double z = (double)o[2];
            const double sd = 0.01 * z * z;
            sticky->cov = sd * sd;
            sticky->set = 1;
            break;
        }
    }
    // samples are drawn lazily, chunk by chunk, on a copy of the RNG; the state after each is kept
    const rgbd_rng snapshot = *rng;
    rgbd_rng r = *rng;
    w->after.resize(std::max(H, 1));
    const int SSd = std::max(SS, 1);
    int drawn = 0;
    auto draw_to = [&](int hend) {
        for (; drawn < hend; drawn++) {
            w->scount()[drawn] = sample_ids(&r, M, SS, &w->samples()[(size_t)drawn * SSd]);
            w->after[drawn] = r;
        }
    };
    RansacDev dv{};
    dv.M = M;
    dv.SS = SSd;
    dv.MWcap = w->MWcap;
    dv.minTh = prm.min_inlier_th;
    dv.maxMahal = prm.max_mahalanobis;
    dv.C = sticky->cov;
    raster_consts(&dv.rcx, &dv.rcy);
    const hipStream_t st = c->stream;
    const int MW = (M + 31) / 32;
    float* d_pts = reinterpret_cast<float*>(w->d_in);
    int* d_samples = reinterpret_cast<int*>(w->d_in + (size_t)w->capM * 24);
    int* d_scount = d_samples + (size_t)w->capH * 8;
    HypOut* d_out = reinterpret_cast<HypOut*>(w->d_res);
    uint32_t* d_masks = reinterpret_cast<uint32_t*>(w->d_res + (size_t)w->capH * sizeof(HypOut));
    int evaluated = 0;   // hypotheses [0, evaluated) done; a chunk's identity slot follows its last one
    bool pts_sent = false;
    auto run_chunk = [&](int h0, int h1) -> rgbd_status {
        draw_to(h1);
        rgbd_status e = RGBD_OK;
        if (!pts_sent) {
            e = check_hip(c, hipMemcpyAsync(d_pts, pts, (size_t)M * 24, hipMemcpyHostToDevice, st), "pts");
            pts_sent = true;
        }
        if (!e && h1 > h0) {
            e = check_hip(c, hipMemcpyAsync(d_samples + (size_t)h0 * SSd, &w->samples()[(size_t)h0 * SSd],
                                            (size_t)(h1 - h0) * SSd * 4, hipMemcpyHostToDevice, st), "samples");
            if (!e) e = check_hip(c, hipMemcpyAsync(d_scount + h0, &w->scount()[h0], (size_t)(h1 - h0) * 4,
                                                    hipMemcpyHostToDevice, st), "scount");
        }
        if (e) return e;
        RansacDev d = dv;
        d.H = h1 - h0;
        const int tk = timer_begin(c, "k_ransac_hyp");
        RGBD_TRY(c, launch_ransac_hyp(d_pts, d_samples + (size_t)h0 * SSd, d_scount + h0, d, d_out + h0,
                          d_masks + (size_t)h0 * w->MWcap, st), "ransac_hyp");
        timer_end(c, tk);
        const int nout = h1 - h0 + 1;
        e = check_hip(c, hipMemcpyAsync(&w->out()[h0], d_out + h0, (size_t)nout * sizeof(HypOut), hipMemcpyDeviceToHost, st), "out");
        if (!e) e = check_hip(c, hipMemcpyAsync(&w->masks()[(size_t)h0 * w->MWcap], d_masks + (size_t)h0 * w->MWcap,
                                                (size_t)nout * w->MWcap * 4, hipMemcpyDeviceToHost, st), "masks");
        if (!e) e = check_hip(c, hipStreamSynchronize(st), "sync");
        return e;
    };
    HypOut ident{};
    std::vector<uint32_t> identMask(MW + 1, 0);
    {
        const int h1 = std::min(H, kFirstChunk);
        if ((s = run_chunk(0, h1))) return s;
        evaluated = h1;
        ident = w->out()[h1];
        std::copy(&w->masks()[(size_t)h1 * w->MWcap], &w->masks()[(size_t)h1 * w->MWcap] + MW, identMask.begin());
    }
    // replay (:56-103)
    int validIters = 0;
    float rmse = 1e6f;
    int bestH = -1;
    size_t bestN = 0;
    int h = 0;
    for (int n = 0; n < prm.iterations && (uint32_t)M >= prm.sample_size; n++) {
        if (h >= evaluated) {
            if ((s = run_chunk(evaluated, H))) return s;
            evaluated = H;
        }
        const HypOut& o = w->out()[h];
        h++;
        if (o.n > 0) {
            validIters++;
            const size_t nr = (size_t)o.n;
            if (o.err <= (double)rmse && nr >= bestN && nr >= prm.min_inlier_th) {
                rmse = (float)o.err;
                bestH = h - 1;
                bestN = nr;
                if (nr > used.size() * 0.5) n += 10;
                if (nr > used.size() * 0.75) n += 10;
                if (nr > used.size() * 0.8) break;
            }
        }
    }
    *rng = (h > 0) ? w->after[h - 1] : snapshot;
    const uint32_t* mask = nullptr;
    if (bestH >= 0) {
        std::memcpy(R.T, w->out()[bestH].T, sizeof(R.T));
        mask = &w->masks()[(size_t)bestH * w->MWcap];
    }
    if (validIters == 0) {   // identity fallback (:105-117)
        if ((uint32_t)ident.n > prm.min_inlier_th && ident.err < (double)prm.max_mahalanobis) {
            for (int i = 0; i < 16; i++) R.T[i] = (i % 5 == 0) ? 1.0f : 0.0f;
            mask = identMask.data();
            rmse = (float)((double)rmse + ident.err);
            bestN = (size_t)ident.n;
        }
    }
    R.rmse = rmse;
    if (mask)
        for (int j = 0; j < M; j++)
            if (mask[j >> 5] & (1u << (j & 31))) R.inliers.push_back(used[j]);
    R.ok = R.inliers.size() >= prm.min_inlier_th;
    if (R.ok && update_f2 && flags2)
        for (const rgbd_dmatch& mm : R.inliers) flags2[mm.trainIdx] = 0;
    return RGBD_OK;
}

// cv::Mat(CV_32F) * cv::Mat: OpenCV gemm for 32F accumulates each dot product in double in k order
// (GEMMSingleMul<float,double>) and rounds once.
static void matmul4(const float* A, const float* B, float* C)
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0.0;
            for (int k = 0; k < 4; k++) s += (double)A[4 * i + k] * (double)B[4 * k + j];
            C[4 * i + j] = (float)s;
        }
}

// Frame::getPoseInverse (Core/Frame.cpp:137-153): Twc = [Rcw^T | Ow] with Ow = -Rcw^T tcw as one cv::gemm
// (GEMM_1_T, alpha = -1: double accumulation in k order, scaled by alpha, one rounding)
static void pose_inverse(const float* T, float* Ti)
{
    for (int i = 0; i < 3; i++) {
        double sacc = 0.0;
        for (int k = 0; k < 3; k++) sacc += (double)T[4 * k + i] * (double)T[4 * k + 3];
        for (int j = 0; j < 3; j++) Ti[4 * i + j] = T[4 * j + i];
        Ti[4 * i + 3] = (float)(sacc * -1.0);
    }
    Ti[12] = Ti[13] = Ti[14] = 0.0f;
    Ti[15] = 1.0f;
}

// Tracking::needKeyFrame (System/Tracking.cpp:201-225): delta = cur.getPoseInverse() * lastKF.getPose();
// tnorm = cv::norm of the float translation (double sums), rnorm = acos(0.5 * (R00 + R11 + R22 - 1.0))
// with the three float entries summed in float first; a NaN angle compares false
static bool need_keyframe(const float* Tcur, const float* Tkf)
{
    float inv[16], d[16];
    pose_inverse(Tcur, inv);
    matmul4(inv, Tkf, d);
    const double tn = std::sqrt((double)d[3] * d[3] + (double)d[7] * d[7] + (double)d[11] * d[11]);
    const float tr = (d[0] + d[5]) + d[10];
    const double rn = std::acos(0.5 * ((double)tr - 1.0));
    return (tn > 0.20) | (rn > 0.1745);
}

}  // namespace rgbd

extern "C" {

void rgbd_rng_seed(rgbd_rng* st, uint32_t seed)
{
    // glibc __srandom_r (TYPE_3): Schrage LCG fill + 310 discarded outputs
    if (seed == 0) seed = 1;
    st->state[0] = (int32_t)seed;
    int32_t word = (int32_t)seed;
    for (int i = 1; i < 31; ++i) {
        const long hi = word / 127773, lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0) word += 2147483647;
        st->state[i] = word;
    }
    st->f = 3;
    st->r = 0;
    for (int k = 0; k < 310; k++) (void)rng_next(st);
}

rgbd_status rgbd_ransac_se3(rgbd_ctx* c, const float* xyz1, int32_t n1, const float* xyz2, int32_t n2,
                            const rgbd_dmatch* m12, int32_t m, const rgbd_ransac_params* prm, rgbd_rng* rng,
                            rgbd_sticky* sticky, int32_t update_f2, uint8_t* flags2, float* T21,
                            rgbd_dmatch* inliers, int32_t* n_inliers, float* rmse, int32_t* ok)
{
    if (!c || !prm || !rng || !sticky || !T21 || !n_inliers || !rmse || !ok || m < 0) return RGBD_ERR_ARG;
    if (m > 0 && (!m12 || !xyz1 || !xyz2)) return RGBD_ERR_ARG;
    for (int i = 0; i < m; i++)
        if (m12[i].queryIdx < 0 || m12[i].queryIdx >= n1 || m12[i].trainIdx < 0 || m12[i].trainIdx >= n2)
            return fail(c, RGBD_ERR_ARG, "match index out of range");
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    RansacResult R;
    if ((s = ransac_se3(c, xyz1, xyz2, m12, m, *prm, rng, sticky, update_f2 != 0, flags2, R))) return s;
    std::memcpy(T21, R.T, sizeof(R.T));
    *n_inliers = (int32_t)R.inliers.size();
    if (inliers) std::copy(R.inliers.begin(), R.inliers.end(), inliers);
    *rmse = R.rmse;
    *ok = R.ok ? 1 : 0;
    return RGBD_OK;
}

static rgbd_status track_chain(rgbd_ctx* c, const void* d_bgr, const void* d_depth, int32_t B, float nnratio,
                               const rgbd_ransac_params* prm, rgbd_rng* rng, rgbd_sticky* sticky, float* poses,
                               int32_t* status, int32_t* n_inliers, rgbd_track_state* ts, float* rel_out,
                               int32_t* kf_out);

rgbd_status rgbd_track_batch(rgbd_ctx* c, const void* d_bgr, const void* d_depth, int32_t B, float nnratio,
                             const rgbd_ransac_params* prm, rgbd_rng* rng, rgbd_sticky* sticky, float* poses,
                             int32_t* status, int32_t* n_inliers)
{
    return track_chain(c, d_bgr, d_depth, B, nnratio, prm, rng, sticky, poses, status, n_inliers, nullptr, nullptr,
                       nullptr);
}

rgbd_status rgbd_track_batch_kf(rgbd_ctx* c, const void* d_bgr, const void* d_depth, int32_t B, float nnratio,
                                const rgbd_ransac_params* prm, rgbd_rng* rng, rgbd_sticky* sticky,
                                rgbd_track_state* state, float* poses, int32_t* status, int32_t* n_inliers,
                                float* rel_poses, int32_t* keyframe)
{
    if (!state) return RGBD_ERR_ARG;
    return track_chain(c, d_bgr, d_depth, B, nnratio, prm, rng, sticky, poses, status, n_inliers, state, rel_poses,
                       keyframe);
}

static rgbd_status track_chain(rgbd_ctx* c, const void* d_bgr, const void* d_depth, int32_t B, float nnratio,
                               const rgbd_ransac_params* prm, rgbd_rng* rng, rgbd_sticky* sticky, float* poses,
                               int32_t* status, int32_t* n_inliers, rgbd_track_state* ts, float* rel_out,
                               int32_t* kf_out)
{
    if (!c || !d_bgr || !d_depth || B < 1 || !prm || !rng || !sticky || !poses || !status) return RGBD_ERR_ARG;
    if (B > c->maxB) return fail(c, RGBD_ERR_CAPACITY, "batch larger than max_batch");
    const int K = c->cfg.kp_cap;
    if (ts && (ts->flags2 || ts->flags1) && ts->flags_cap < K)
        return fail(c, RGBD_ERR_CAPACITY, "rgbd_track_state flag buffers smaller than rgbd_max_keypoints");
    if (ts && ts->valid && B < 2)
        return fail(c, RGBD_ERR_ARG, "a continuing chunk starts with the previous chunk's last two frames");
    rgbd_status s = rgbd_extract_batch(c, d_bgr, d_depth, B);
    if (s) return s;
    std::vector<int> errf(B);   // the extraction's per-frame capacity flags (read with the chain's results)
    if ((s = check_hip(c, hipMemcpyAsync(errf.data(), c->d_err, (size_t)B * 4, hipMemcpyDeviceToHost, c->stream), "err")))
        return s;
    const bool cont = ts && ts->valid;
    const int first = cont ? 2 : 1;   // first frame tracked in this call
    // the whole chain on the device (lanes_host.cpp): one lane over the batch
    const LaneSpec sp{0, B - 1, first};
    std::vector<PairOut> po;
    s = lanes_track(c, B, nnratio, *prm, &sp, 1, rng, sticky, cont ? ts->flags2 : nullptr, cont ? ts->flags1 : nullptr, po,
                    (ts && B >= 2) ? ts->flags2 : nullptr, (ts && B >= 2) ? ts->flags1 : nullptr);
    if (s) return s;
    for (int b = 0; b < B; b++)
        if (errf[b]) return fail(c, RGBD_ERR_CAPACITY, (errf[b] & 2) ? "SVO: keypoints kept by retainBest exceed rgbd_max_keypoints"
                                                                    : "quadtree node capacity exceeded");
    status[0] = 1;
    if (n_inliers) n_inliers[0] = 0;
    // Tracking's bookkeeping (ts != NULL; System/Tracking.cpp:39-73, 227-256): P = every frame's current
    // pose (updateLastFrame rewrites the previous frame's), kfo[b] = its reference keyframe (-1: the
    // state's keyframe from an earlier chunk), rel[b] = mRelativeFramePoses entry
    std::vector<float> P, rel;
    std::vector<int> kfo;
    int kf = 0;
    auto kfpose = [&](int k) -> const float* { return k < 0 ? ts->kf_pose : &P[(size_t)k * 16]; };
    if (ts) {
        P.assign((size_t)B * 16, 0.0f);
        rel.assign((size_t)B * 16, 0.0f);
        kfo.assign(B, 0);
        float inv[16];
        if (cont) {   // frames 0, 1 = the previous chunk's last two (mpRefFrame.second, .first)
            std::memcpy(&P[0], ts->ref2_pose, 64);
            std::memcpy(&P[16], &poses[16], 64);
            std::memcpy(&poses[0], ts->ref2_pose, 64);
            kf = ts->first_is_kf ? 1 : -1;
            kfo[1] = kf;
            std::memcpy(&rel[16], ts->first_rel, 64);
        } else {      // Tracking::initialize (:86-116): keyframe, relative pose to itself
            std::memcpy(&P[0], poses, 64);
            kf = 0;
            pose_inverse(&P[0], inv);
            matmul4(&P[0], inv, &rel[0]);
            kfo[0] = kf;
            if (kf_out) kf_out[0] = 1;
        }
    }
    auto refpose = [&](int r) -> const float* { return ts ? &P[(size_t)r * 16] : &poses[(size_t)r * 16]; };
    for (int b = first; b < B; b++) {
        const PairOut& r = po[b];
        float* Pb = ts ? &P[(size_t)b * 16] : &poses[(size_t)b * 16];
        if (r.ok)
            matmul4(r.T, refpose(r.ref), Pb);       // T * pose(F1) (Solver/SolverSE3.cpp:124-126, Gicp.cpp:31)
        else
            std::memcpy(Pb, refpose(b - 1), 64);   // recover() (System/Tracking.cpp:195-199)
        status[b] = r.ok ? 1 : 0;
        if (n_inliers) n_inliers[b] = r.n_inliers;
        if (ts) {
            // updateLastFrame (:242-247): the previous frame's pose = Tlr * pose(its reference keyframe)
            float tmp[16], inv[16];
            matmul4(&rel[(size_t)(b - 1) * 16], kfpose(kfo[b - 1]), tmp);
            std::memcpy(&P[(size_t)(b - 1) * 16], tmp, 64);
            kfo[b] = kf;   // mpCurFrame->mpReferenceKF = mpLastKeyFrame (:51)
            if (need_keyframe(Pb, kfpose(kf))) kf = kfo[b] = b;   // createKeyFrame (:227-240)
            // updateRelativePose (:249-256): Tcr = pose(cur) * pose(reference keyframe)^-1
            pose_inverse(kfpose(kfo[b]), inv);
            matmul4(Pb, inv, &rel[(size_t)b * 16]);
            std::memcpy(&poses[(size_t)b * 16], Pb, 64);   // track() returns mpCurFrame->getPose()
            if (kf_out) kf_out[b] = (kf == b) ? 1 : 0;
        }
    }
    if (ts) {
        if (rel_out) std::memcpy(&rel_out[(size_t)first * 16], &rel[(size_t)first * 16], (size_t)(B - first) * 64);
        if (!cont && rel_out) std::memcpy(rel_out, rel.data(), 64);
        if (kf >= 0 && kf != B - 1) std::memcpy(ts->kf_pose, kfpose(kf), 64);
        ts->first_is_kf = (kf == B - 1) ? 1 : 0;
        std::memcpy(ts->first_rel, &rel[(size_t)(B - 1) * 16], 64);
        if (B >= 2) std::memcpy(ts->ref2_pose, &P[(size_t)(B - 2) * 16], 64);   // re-anchored at step B - 1
        ts->valid = B >= 2 ? 1 : ts->valid;
    }
    return RGBD_OK;
}

rgbd_status rgbd_track_lanes(rgbd_ctx* c, const void* d_bgr, const void* d_depth, int32_t B, float nnratio,
                             const rgbd_ransac_params* prm, int32_t L, const int32_t* lane_first, rgbd_rng* rngs,
                             rgbd_sticky* stickies, float* poses, int32_t* status, int32_t* n_inliers)
{
    // d_bgr == d_depth == nullptr: the frames of the context's last rgbd_extract_batch (of exactly B frames)
    const bool extracted = !d_bgr && !d_depth;
    if (!c || (!extracted && (!d_bgr || !d_depth)) || B < 2 || !prm || L < 1 || !lane_first || !rngs || !stickies ||
        !poses || !status)
        return RGBD_ERR_ARG;
    if (B > c->maxB) return fail(c, RGBD_ERR_CAPACITY, "batch larger than max_batch");
    if (extracted && c->last_B != B) return fail(c, RGBD_ERR_ARG, "no rgbd_extract_batch of B frames to track");
    if (lane_first[0] != 0 || lane_first[L] != B - 1) return fail(c, RGBD_ERR_ARG, "lane_first[0] = 0, lane_first[L] = B - 1");
    std::vector<LaneSpec> sp(L);
    for (int l = 0; l < L; l++) {
        if (lane_first[l + 1] <= lane_first[l]) return fail(c, RGBD_ERR_ARG, "lane_first must increase strictly");
        sp[l] = LaneSpec{lane_first[l], lane_first[l + 1], lane_first[l] + 1};
    }
    rgbd_status s = extracted ? RGBD_OK : rgbd_extract_batch(c, d_bgr, d_depth, B);
    if (s) return s;
    // the extraction may have run on another stream (rgbd_set_stream in between): order behind it
    if (extracted && (s = order_after_extraction(c))) return s;
    std::vector<int> errf(B);
    if ((s = check_hip(c, hipMemcpyAsync(errf.data(), c->d_err, (size_t)B * 4, hipMemcpyDeviceToHost, c->stream), "err")))
        return s;
    std::vector<PairOut> po;
    if ((s = lanes_track(c, B, nnratio, *prm, sp.data(), L, rngs, stickies, nullptr, nullptr, po, nullptr, nullptr)))
        return s;
    for (int b = 0; b < B; b++)
        if (errf[b]) return fail(c, RGBD_ERR_CAPACITY, (errf[b] & 2) ? "SVO: keypoints kept by retainBest exceed rgbd_max_keypoints"
                                                                    : "quadtree node capacity exceeded");
    for (int l = 0; l < L; l++) {   // lane-major rows: frame f of lane l at row f + l
        const int r0 = sp[l].start + l;
        status[r0] = 1;
        if (n_inliers) n_inliers[r0] = 0;
        for (int b = sp[l].first; b <= sp[l].end; b++) {
            const PairOut& r = po[b];
            float* Pb = &poses[(size_t)(b + l) * 16];
            if (r.ok)
                matmul4(r.T, &poses[(size_t)(r.ref + l) * 16], Pb);
            else
                std::memcpy(Pb, &poses[(size_t)(b - 1 + l) * 16], 64);
            status[b + l] = r.ok ? 1 : 0;
            if (n_inliers) n_inliers[b + l] = r.n_inliers;
        }
    }
    return RGBD_OK;
}

rgbd_status rgbd_debug_rotation_ops(rgbd_ctx* c, const double* x, const double* num, const double* den,
                                    const double* theta, int32_t n, double* sq, double* q, double* t)
{
    if (!c || n < 1 || n > (1 << 24) || !x || !num || !den || !theta || !sq || !q || !t) return RGBD_ERR_ARG;
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    double* d = nullptr;
    const size_t m = (size_t)n, bytes = m * sizeof(double);
    s = check_hip(c, hipMalloc((void**)&d, 7 * bytes), "rotation ops buffers");
    const double* in[4] = {x, num, den, theta};
    for (int k = 0; k < 4 && !s; k++)
        s = check_hip(c, hipMemcpyAsync(d + k * m, in[k], bytes, hipMemcpyHostToDevice, c->stream), "rotation ops in");
    if (!s)
        s = check_hip(c, rgbd::launch_debug_rotation_ops(d, d + m, d + 2 * m, d + 3 * m, n, d + 4 * m, d + 5 * m, d + 6 * m,
                                                         c->stream),
                      "launch of k_debug_rotation_ops");
    double* out[3] = {sq, q, t};
    for (int k = 0; k < 3 && !s; k++)
        s = check_hip(c, hipMemcpyAsync(out[k], d + (4 + k) * m, bytes, hipMemcpyDeviceToHost, c->stream), "rotation ops out");
    if (!s) s = check_hip(c, hipStreamSynchronize(c->stream), "rotation ops sync");
    if (d) (void)hipFree(d);
    return s;
}

rgbd_status rgbd_debug_sort_matches(rgbd_ctx* c, const float* dist, int32_t n, int32_t depth_limit, int32_t* order)
{
    if (!c || n < 0 || n > kRansacMaxM || (n > 0 && (!dist || !order))) return RGBD_ERR_ARG;
    for (int i = 0; i < n; i++)
        if (!(dist[i] >= 0.0f && dist[i] <= 65535.0f) || dist[i] != (float)(int)dist[i])
            return fail(c, RGBD_ERR_ARG, "distances must be integers in [0, 65535]");
    if (n == 0) return RGBD_OK;
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    return s ? s : lanes_sort_test(c, dist, n, depth_limit, order);
}

}  // extern "C"

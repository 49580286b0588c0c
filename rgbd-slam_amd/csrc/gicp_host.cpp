// gicp_host.cpp -- GICP host control (C ABI) and the Gicp::compute decision rule.
//
// Gicp::compute (Solver/Gicp.cpp:21-35) -> align (:54-66): clouds from the RANSAC inlier matches
// (createCloudsFromMatches :37-52), pcl GICP align with mT21 as the guess, hasConverged() ? final
// transformation : identity, and identity (Eigen isIdentity) means failure.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "context.h"
#include "gicp_dev.h"

using namespace rgbd;

namespace rgbd {

struct GicpWS {
    float* d_pts = nullptr;      // src [kGicpMaxM][3] | tgt [kGicpMaxM][3] | guess[16]
    double* d_cov = nullptr;     // [2][kGicpMaxM][9]
    double* d_M = nullptr;       // [kGicpMaxM][9] Mahalanobis matrices of one outer iteration
    GicpOut* d_out = nullptr;
    float* h_pts = nullptr;      // pinned mirror of d_pts
    GicpOut* h_out = nullptr;
};

void gicp_free(rgbd_ctx* c)
{
    GicpWS* w = static_cast<GicpWS*>(c->gicp);
    if (!w) return;
    if (w->d_pts) (void)hipFree(w->d_pts);
    if (w->d_cov) (void)hipFree(w->d_cov);
    if (w->d_M) (void)hipFree(w->d_M);
    if (w->d_out) (void)hipFree(w->d_out);
    if (w->h_pts) (void)hipHostFree(w->h_pts);
    if (w->h_out) (void)hipHostFree(w->h_out);
    delete w;
    c->gicp = nullptr;
}

static rgbd_status gicp_ws(rgbd_ctx* c, GicpWS** out)
{
    GicpWS* w = static_cast<GicpWS*>(c->gicp);
    if (!w) {
        w = new GicpWS();
        c->gicp = w;
        const size_t pts = ((size_t)2 * kGicpMaxM * 3 + 16) * sizeof(float);
        rgbd_status s = check_hip(c, hipMalloc((void**)&w->d_pts, pts), "gicp pts");
        if (!s) s = check_hip(c, hipMalloc((void**)&w->d_cov, (size_t)2 * kGicpMaxM * 9 * sizeof(double)), "gicp cov");
        if (!s) s = check_hip(c, hipMalloc((void**)&w->d_M, (size_t)kGicpMaxM * 9 * sizeof(double)), "gicp M");
        if (!s) s = check_hip(c, hipMalloc((void**)&w->d_out, sizeof(GicpOut)), "gicp out");
        if (!s) s = check_hip(c, hipHostMalloc((void**)&w->h_pts, pts, hipHostMallocDefault), "gicp pinned pts");
        if (!s) s = check_hip(c, hipHostMalloc((void**)&w->h_out, sizeof(GicpOut), hipHostMallocDefault), "gicp pinned out");
        if (s) {
            gicp_free(c);
            return s;
        }
    }
    *out = w;
    return RGBD_OK;
}

// align: src / tgt given as host arrays (or gathered by the caller into the pinned staging)
rgbd_status gicp_align(rgbd_ctx* c, int M, const float* guess, const rgbd_gicp_params& prm, GicpOut* res,
                       const float* src, const float* tgt)
{
    std::memset(res, 0, sizeof(*res));
    for (int i = 0; i < 16; i++) res->T[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    if (M > kGicpMaxM) return fail(c, RGBD_ERR_UNSUPPORTED, "more than 2048 points for GICP");
    if (prm.k_correspondences < 1 || prm.k_correspondences > 32)
        return fail(c, RGBD_ERR_UNSUPPORTED, "GICP k_correspondences must be in [1, 32]");
    if (M < prm.k_correspondences || M < 1) return RGBD_OK;   // PCL computeCovariances refuses: not converged
    GicpWS* w = nullptr;
    rgbd_status s = gicp_ws(c, &w);
    if (s) return s;
    float* hs = w->h_pts;
    float* ht = w->h_pts + (size_t)kGicpMaxM * 3;
    float* hg = w->h_pts + (size_t)2 * kGicpMaxM * 3;
    if (src != hs) std::memcpy(hs, src, (size_t)M * 12);
    if (tgt != ht) std::memcpy(ht, tgt, (size_t)M * 12);
    std::memcpy(hg, guess, 64);
    const hipStream_t st = c->stream;
    s = check_hip(c, hipMemcpyAsync(w->d_pts, hs, (size_t)M * 12, hipMemcpyHostToDevice, st), "gicp src");
    if (!s) s = check_hip(c, hipMemcpyAsync(w->d_pts + (size_t)kGicpMaxM * 3, ht, (size_t)M * 12, hipMemcpyHostToDevice, st), "gicp tgt");
    if (!s) s = check_hip(c, hipMemcpyAsync(w->d_pts + (size_t)2 * kGicpMaxM * 3, hg, 64, hipMemcpyHostToDevice, st), "gicp guess");
    if (s) return s;
    GicpDevPrm dp{prm.max_iterations, prm.k_correspondences, prm.gn_iterations, 0,
                  prm.max_corr_dist * prm.max_corr_dist, prm.transformation_epsilon, prm.rotation_epsilon,
                  prm.gicp_epsilon};
    const int tk = timer_begin(c, "k_gicp");
    RGBD_TRY(c, launch_gicp(w->d_pts, w->d_pts + (size_t)kGicpMaxM * 3, M, w->d_pts + (size_t)2 * kGicpMaxM * 3, dp, w->d_cov,
                w->d_out, w->d_M, st), "gicp");
    timer_end(c, tk);
    s = check_hip(c, hipMemcpyAsync(w->h_out, w->d_out, sizeof(GicpOut), hipMemcpyDeviceToHost, st), "gicp out");
    if (!s) s = check_hip(c, hipStreamSynchronize(st), "sync");
    if (s) return s;
    *res = *w->h_out;
    return RGBD_OK;
}

// Eigen isIdentity() with float dummy precision 1e-5
static bool is_identity(const float* T)
{
    const float prec = 1e-5f;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            const float v = T[4 * i + j];
            if (i == j) {
                if (!(std::fabs(v - 1.0f) <= prec * std::fmin(std::fabs(v), 1.0f))) return false;
            } else if (!(std::fabs(v) <= prec)) {
                return false;
            }
        }
    return true;
}

// Gicp::compute: ok and T (identity when not ok)
rgbd_status gicp_compute(rgbd_ctx* c, int M, const float* guess, const rgbd_gicp_params& prm, const float* src,
                         const float* tgt, float* T, bool* ok)
{
    *ok = false;
    for (int i = 0; i < 16; i++) T[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    if (M < 20) return RGBD_OK;
    GicpOut r;
    rgbd_status s = gicp_align(c, M, guess, prm, &r, src, tgt);
    if (s) return s;
    if (!r.converged) return RGBD_OK;
    std::memcpy(T, r.T, 64);
    *ok = !is_identity(T);
    return RGBD_OK;
}

}  // namespace rgbd

extern "C" {

rgbd_status rgbd_gicp(rgbd_ctx* c, const float* src, const float* tgt, int32_t M, const float* guess,
                      const rgbd_gicp_params* prm, float* T, int32_t* converged, int32_t* iterations)
{
    if (!c || !prm || !guess || !T || !converged || M < 0 || (M > 0 && (!src || !tgt))) return RGBD_ERR_ARG;
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    GicpOut r;
    if ((s = gicp_align(c, M, guess, *prm, &r, src, tgt))) return s;
    std::memcpy(T, r.T, 64);
    *converged = r.converged;
    if (iterations) *iterations = r.iters;
    return RGBD_OK;
}

rgbd_status rgbd_gicp_compute(rgbd_ctx* c, const float* src, const float* tgt, int32_t M, const float* guess,
                              const rgbd_gicp_params* prm, float* T, int32_t* ok)
{
    if (!c || !prm || !guess || !T || !ok || M < 0 || (M > 0 && (!src || !tgt))) return RGBD_ERR_ARG;
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    bool b = false;
    if ((s = gicp_compute(c, M, guess, *prm, src, tgt, T, &b))) return s;
    *ok = b ? 1 : 0;
    return RGBD_OK;
}

rgbd_status rgbd_set_tracking_gicp(rgbd_ctx* c, const rgbd_gicp_params* prm)
{
    if (!c) return RGBD_ERR_ARG;
    c->track_gicp = prm ? *prm : rgbd_gicp_params{10, 20, 0.07, 1e-9, 2e-3, 1e-3, 4, 1};
    return RGBD_OK;
}

}  // extern "C"

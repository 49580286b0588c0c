// cloud_host.cpp -- C ABI of the keyframe dense cloud (cloud.hip): Tracking::createKeyFrame's
// createCloud(6) + passThroughFilter("z", 0.5, 4.0) + downsampleCloud(0.04f) + statisticalFilterCloud(50, 1.0)
// (System/Tracking.cpp:234-237, Core/Frame.cpp:475-549).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "cloud_dev.h"
#include "context.h"

using namespace rgbd;

namespace rgbd {

struct CloudWS {
    int cap = 0, nkf = 0;
    CloudPoint *d_pts = nullptr, *d_vox = nullptr, *d_out = nullptr;
    float* d_dist = nullptr;
    int *d_nvox = nullptr, *d_nout = nullptr, *d_frames = nullptr;
    uint8_t* d_bgr = nullptr;   // single-frame staging (host-buffer entry point)
    uint16_t* d_depth = nullptr;
    float* d_depthf = nullptr;  // ... Frame::mImDepth (f32) for rgbd_keyframe_cloud_f32
};

void cloud_free(rgbd_ctx* c)
{
    CloudWS* w = static_cast<CloudWS*>(c->cloud);
    if (!w) return;
    void* p[] = {w->d_pts, w->d_vox, w->d_out, w->d_dist, w->d_nvox, w->d_nout, w->d_frames, w->d_bgr, w->d_depth, w->d_depthf};
    for (void* q : p)
        if (q) (void)hipFree(q);
    delete w;
    c->cloud = nullptr;
}

}  // namespace rgbd

namespace {

rgbd_status cloud_cfg(rgbd_ctx* c, const rgbd_cloud_params* prm, CloudCfg* g)
{
    if (prm->stride < 1 || !(prm->leaf > 0) || prm->sor_k < 1 || prm->sor_k > 63)
        return fail(c, RGBD_ERR_ARG, "cloud params: stride >= 1, leaf > 0, 1 <= sor_k <= 63");
    g->W = c->W;
    g->H = c->H;
    g->res = prm->stride;
    g->rows = (c->H + prm->stride - 1) / prm->stride;
    g->cols = (c->W + prm->stride - 1) / prm->stride;
    g->cap = g->rows * g->cols;
    if (g->cap > 16384) return fail(c, RGBD_ERR_UNSUPPORTED, "keyframe cloud: more than 16384 samples (stride too small)");
    g->sort_cap = 1;
    while (g->sort_cap < g->cap) g->sort_cap <<= 1;
    g->cx = c->cam.cx;
    g->cy = c->cam.cy;
    g->invfx = 1.0f / c->cam.fx;   // IntrinsicMatrix::mInvfx
    g->invfy = 1.0f / c->cam.fy;
    g->depth_factor = c->cam.depth_map_factor;
    g->zmin = prm->zmin;
    g->zmax = prm->zmax;
    g->inv_leaf = 1.0f / prm->leaf;
    g->sor_k = prm->sor_k;
    g->sor_std = prm->sor_std;
    return RGBD_OK;
}

template <typename T>
rgbd_status dgrow(rgbd_ctx* c, T** p, size_t n, const char* what)
{
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    return check_hip(c, hipMalloc((void**)p, std::max<size_t>(n, 1) * sizeof(T)), what);
}

rgbd_status ws_get(rgbd_ctx* c, int cap, int nkf, CloudWS** out)
{
    CloudWS* w = static_cast<CloudWS*>(c->cloud);
    if (!w) c->cloud = w = new CloudWS();
    if (w->cap < cap || w->nkf < nkf) {
        const int nk = std::max(nkf, w->nkf);
        const size_t np = (size_t)cap * nk;
        rgbd_status s = dgrow(c, &w->d_pts, np, "cloud pts");
        if (!s) s = dgrow(c, &w->d_vox, np, "cloud vox");
        if (!s) s = dgrow(c, &w->d_out, np, "cloud out");
        if (!s) s = dgrow(c, &w->d_dist, np, "cloud dist");
        if (!s) s = dgrow(c, &w->d_nvox, (size_t)nk, "cloud nvox");
        if (!s) s = dgrow(c, &w->d_nout, (size_t)nk, "cloud nout");
        if (!s) s = dgrow(c, &w->d_frames, (size_t)nk, "cloud frames");
        if (s) return s;
        w->cap = cap;
        w->nkf = nk;
    }
    *out = w;
    return RGBD_OK;
}

rgbd_status run_cloud(rgbd_ctx* c, const uint8_t* d_bgr, const uint16_t* d_depth, const float* d_depthf,
                      const int32_t* frames, int nkf, const rgbd_cloud_params* prm, rgbd_point* out, int32_t cap,
                      int32_t* counts)
{
    CloudCfg g{};
    rgbd_status s = cloud_cfg(c, prm, &g);
    if (s) return s;
    CloudWS* w = nullptr;
    if ((s = ws_get(c, g.cap, nkf, &w))) return s;
    const hipStream_t st = c->stream;
    s = check_hip(c, hipMemcpyAsync(w->d_frames, frames, (size_t)nkf * 4, hipMemcpyHostToDevice, st), "cloud frames");
    if (s) return s;
    const int tk = timer_begin(c, "k_cloud");
    RGBD_TRY(c, launch_cloud(d_bgr, d_depth, d_depthf, w->d_frames, nkf, g, w->d_pts, w->d_vox, w->d_nvox, w->d_dist, w->d_out, w->d_nout, st), "cloud");
    timer_end(c, tk);
    std::vector<int> n(nkf);
    s = check_hip(c, hipMemcpyAsync(n.data(), w->d_nout, (size_t)nkf * 4, hipMemcpyDeviceToHost, st), "cloud counts");
    if (!s) s = check_hip(c, hipStreamSynchronize(st), "sync");
    if (s) return s;
    for (int k = 0; k < nkf; k++) {
        counts[k] = n[k];
        const int m = std::min(n[k], cap);
        if (m > 0)
            s = check_hip(c, hipMemcpyAsync(out + (size_t)k * cap, w->d_out + (size_t)k * g.cap, (size_t)m * sizeof(rgbd_point),
                                            hipMemcpyDeviceToHost, st), "cloud read");
        if (s) return s;
    }
    s = check_hip(c, hipStreamSynchronize(st), "sync");
    if (s) return s;
    for (int k = 0; k < nkf; k++)
        if (n[k] > cap) return fail(c, RGBD_ERR_CAPACITY, "keyframe cloud larger than the output capacity");
    return RGBD_OK;
}

// one host frame: the BGR image and either the u16 depth (depth) or Frame::mImDepth as f32 (depthf)
rgbd_status cloud_host_frame(rgbd_ctx* c, const uint8_t* bgr, const uint16_t* depth, const float* depthf,
                             const rgbd_cloud_params* prm, rgbd_point* out, int32_t cap, int32_t* n)
{
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    CloudCfg g{};
    if ((s = cloud_cfg(c, prm, &g))) return s;
    CloudWS* w = nullptr;
    if ((s = ws_get(c, g.cap, 1, &w))) return s;
    const size_t px = (size_t)c->W * c->H;
    if (!w->d_bgr) s = check_hip(c, hipMalloc((void**)&w->d_bgr, px * 3), "cloud bgr");
    if (!s && depth && !w->d_depth) s = check_hip(c, hipMalloc((void**)&w->d_depth, px * 2), "cloud depth");
    if (!s && depthf && !w->d_depthf) s = check_hip(c, hipMalloc((void**)&w->d_depthf, px * 4), "cloud depth f32");
    if (!s) s = check_hip(c, hipMemcpyAsync(w->d_bgr, bgr, px * 3, hipMemcpyHostToDevice, c->stream), "cloud bgr up");
    if (!s && depth)
        s = check_hip(c, hipMemcpyAsync(w->d_depth, depth, px * 2, hipMemcpyHostToDevice, c->stream), "cloud depth up");
    if (!s && depthf)
        s = check_hip(c, hipMemcpyAsync(w->d_depthf, depthf, px * 4, hipMemcpyHostToDevice, c->stream), "cloud depth up");
    if (s) return s;
    const int32_t f0 = 0;
    return run_cloud(c, w->d_bgr, depth ? w->d_depth : nullptr, depthf ? w->d_depthf : nullptr, &f0, 1, prm, out, cap, n);
}

}  // namespace

extern "C" {

rgbd_status rgbd_keyframe_cloud_batch(rgbd_ctx* c, const void* d_bgr, const void* d_depth, int32_t B,
                                      const int32_t* frames, int32_t nkf, const rgbd_cloud_params* prm,
                                      rgbd_point* out, int32_t cap, int32_t* counts)
{
    if (!c || !d_bgr || !d_depth || !frames || nkf < 0 || !prm || !out || !counts || cap < 0) return RGBD_ERR_ARG;
    for (int k = 0; k < nkf; k++)
        if (frames[k] < 0 || frames[k] >= B) return fail(c, RGBD_ERR_ARG, "keyframe index outside the batch");
    if (nkf == 0) return RGBD_OK;
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    return run_cloud(c, (const uint8_t*)d_bgr, (const uint16_t*)d_depth, nullptr, frames, nkf, prm, out, cap, counts);
}

rgbd_status rgbd_keyframe_cloud(rgbd_ctx* c, const uint8_t* bgr, const uint16_t* depth, const rgbd_cloud_params* prm,
                                rgbd_point* out, int32_t cap, int32_t* n)
{
    if (!c || !bgr || !depth || !prm || !out || !n || cap < 0) return RGBD_ERR_ARG;
    return cloud_host_frame(c, bgr, depth, nullptr, prm, out, cap, n);
}

rgbd_status rgbd_keyframe_cloud_f32(rgbd_ctx* c, const uint8_t* bgr, const float* depth, const rgbd_cloud_params* prm,
                                    rgbd_point* out, int32_t cap, int32_t* n)
{
    if (!c || !bgr || !depth || !prm || !out || !n || cap < 0) return RGBD_ERR_ARG;
    return cloud_host_frame(c, bgr, nullptr, depth, prm, out, cap, n);
}

}  // extern "C"

// svo_host.cpp -- host side of the SVO + BRIEF front end (svo.hip): Extractor(SVO, BRIEF, NORMAL), the
// reference's default (main.cpp:31), behind the same extraction entry points as the ORBextractor.
//   Extractor::createDetector SVO   Features/Extractor.cpp:162-165  -> svo_configure (SvoCfg, tile table)
//   Extractor::detectAndCompute     Features/Extractor.cpp:50-61    -> svo_run_extract (one launch chain)
//   Frame::undistortKeyPoints + uprojectCamera (Core/Frame.cpp:91-117, 251-281) -> k_undistort
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "context.h"
#include "launch.h"
#include "svo_dev.h"

namespace rgbd {

namespace {

const int8_t kDefaultBrief[256 * 4] = {
#include "brief_pattern.inc"
};

struct SvoWS {
    SvoCfg cfg{};
    std::vector<SvoTile> tiles;
    SvoTile* d_tiles = nullptr;
    uint8_t* d_pyr = nullptr;
    unsigned long long* d_cells = nullptr;
    uint16_t* d_box = nullptr;
    uint2* d_cand = nullptr;
    int* d_ncand = nullptr;
    uint32_t* d_pat = nullptr;
    float* d_rt_resp = nullptr;   // rgbd_svo_retain_best staging
    int* d_rt_order = nullptr;
    int8_t pattern[256 * 4];
};

SvoWS* ws(rgbd_ctx* c) { return static_cast<SvoWS*>(c->svo); }

rgbd_status upload_pattern(rgbd_ctx* c, SvoWS* w)
{
    uint32_t packed[256];
    for (int t = 0; t < 256; t++) {
        const uint8_t* q = reinterpret_cast<const uint8_t*>(w->pattern + 4 * t);
        packed[t] = (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) | ((uint32_t)q[3] << 24);
    }
    return check_hip(c, hipMemcpyAsync(w->d_pat, packed, sizeof(packed), hipMemcpyHostToDevice, c->stream), "brief pattern");
}

}  // namespace

rgbd_status svo_configure(rgbd_ctx* c, const rgbd_svo_params& p)
{
    if (p.nlevels < 1 || p.nlevels > kSvoMaxLevels)
        return fail(c, RGBD_ERR_UNSUPPORTED, "SVO: nlevels must be 1..8");
    if (p.cell_size < 1 || p.threshold < 0 || p.threshold > 254 || p.nfeatures < 0 || p.max_keypoints < 0)
        return fail(c, RGBD_ERR_ARG, "SVO: cell_size >= 1, 0 <= threshold <= 254, nfeatures >= 0, max_keypoints >= 0");
    if (c->W < 1 || c->H < 1 || c->W > 2047 || c->H > 2047)
        return fail(c, RGBD_ERR_UNSUPPORTED, "SVO: image sides 1..2047");
    SvoWS* w = new SvoWS();
    c->svo = w;
    SvoCfg& g = w->cfg;
    g.W = c->W;
    g.H = c->H;
    g.nlevels = p.nlevels;
    g.cell = p.cell_size;
    g.barrier = p.threshold;
    g.gcols = (int)std::ceil((double)c->W / p.cell_size);   // SVOextractor::detect :93-94
    g.grows = (int)std::ceil((double)c->H / p.cell_size);
    g.ncells = g.gcols * g.grows;
    if (g.ncells > kSvoSelThreads * kSvoSelMaxE)
        return fail(c, RGBD_ERR_UNSUPPORTED, "SVO: more than 12288 grid cells (raise cell_size)");
    int off = 0;
    for (int l = 0; l < p.nlevels; l++) {
        g.lw[l] = l ? g.lw[l - 1] / 2 : c->W;
        g.lh[l] = l ? g.lh[l - 1] / 2 : c->H;
        if (l + 1 < p.nlevels && (g.lw[l] & 1))   // halfSample's row walk (:24-35) assumes even widths
            return fail(c, RGBD_ERR_UNSUPPORTED, "SVO: odd level width above the last level");
        g.loff[l] = off;
        off += g.lw[l] * g.lh[l];
    }
    g.frame_bytes = (off + 63) & ~63;
    g.nfeatures = p.nfeatures;
    // retainBest keeps nfeatures + every tie of the boundary response (more fail loudly, RGBD_ERR_CAPACITY)
    g.kp_cap = std::min(g.ncells, p.max_keypoints > 0 ? p.max_keypoints : p.nfeatures + 64);
    g.border = 48 / 2 + 9 / 2;                            // BriefDescriptorExtractorImpl PATCH_SIZE, KERNEL_SIZE
    for (int l = 0; l < p.nlevels; l++) {   // FAST-10 tiles of 64 x 32 over the detector's domain
        if (g.lw[l] < 7 || g.lh[l] < 7) continue;
        for (int y = 0; y < g.lh[l]; y += 32)
            for (int x = 0; x < g.lw[l]; x += 64) w->tiles.push_back(SvoTile{(int16_t)l, (int16_t)x, (int16_t)y, 0});
    }
    std::memcpy(w->pattern, kDefaultBrief, sizeof(kDefaultBrief));
    c->cfg.kp_cap = g.kp_cap;   // the output arrays (kps, desc, xyz, knn) are sized by it
    return RGBD_OK;
}

rgbd_status svo_alloc(rgbd_ctx* c)
{
    SvoWS* w = ws(c);
    const SvoCfg& g = w->cfg;
    const size_t B = (size_t)c->maxB;
    auto al = [&](auto** p, size_t bytes, const char* what) {
        return check_hip(c, hipMalloc((void**)p, std::max<size_t>(bytes, 16)), what);
    };
    rgbd_status s = al(&w->d_tiles, w->tiles.size() * sizeof(SvoTile), "svo tiles");
    if (!s) s = al(&w->d_pyr, B * g.frame_bytes + 64, "svo pyramid");
    if (!s) s = al(&w->d_cells, B * g.ncells * 8, "svo cells");
    if (!s) s = al(&w->d_box, B * g.W * g.H * 2, "svo box");
    if (!s) s = al(&w->d_cand, B * g.ncells * 8, "svo candidates");
    if (!s) s = al(&w->d_ncand, B * 4, "svo candidate counts");
    if (!s) s = al(&w->d_pat, 256 * 4, "svo pattern");
    if (s) return s;
    if (!w->tiles.empty())
        s = check_hip(c, hipMemcpy(w->d_tiles, w->tiles.data(), w->tiles.size() * sizeof(SvoTile), hipMemcpyHostToDevice),
                      "svo tiles up");
    if (!s) s = check_hip(c, hipMemset(w->d_cells, 0, B * g.ncells * 8), "svo cells zero");
    if (!s) s = check_hip(c, hipMemset(w->d_ncand, 0, B * 4), "svo ncand zero");
    if (!s) s = upload_pattern(c, w);
    if (!s) s = check_hip(c, hipStreamSynchronize(c->stream), "sync");
    return s;
}

void svo_free(rgbd_ctx* c)
{
    SvoWS* w = ws(c);
    if (!w) return;
    void* p[] = {w->d_tiles, w->d_pyr, w->d_cells, w->d_box, w->d_cand, w->d_ncand, w->d_pat, w->d_rt_resp, w->d_rt_order};
    for (void* q : p)
        if (q) (void)hipFree(q);
    delete w;
    c->svo = nullptr;
}

uint8_t* svo_gray_level(rgbd_ctx* c) { return ws(c)->d_pyr; }

rgbd_status svo_run_extract(rgbd_ctx* c, const uint8_t* d_bgr, const uint16_t* d_depth, int B, bool from_gray,
                            const ExtractHook* after_fast)
{
    SvoWS* w = ws(c);
    const SvoCfg& g = w->cfg;
    const hipStream_t st = c->stream;
    int tk = timer_begin(c, "k_svo_pyramid");
    RGBD_TRY(c, launch_svo_pyramid(from_gray ? nullptr : d_bgr, w->d_pyr, w->d_box, g, B, st), "svo_pyramid");
    timer_end(c, tk);
    tk = timer_begin(c, "k_svo_detect");
    RGBD_TRY(c, launch_svo_detect(w->d_pyr, w->d_tiles, (int)w->tiles.size(), g, w->d_cells, B, st), "svo_detect");
    timer_end(c, tk);
    if (after_fast) {   // e.g. the deferred PnPRansac solves of earlier pipelined steps (pnp_host.cpp)
        rgbd_status hs = (*after_fast)(1);
        if (!hs) hs = (*after_fast)(2);
        if (hs) return hs;
    }
    tk = timer_begin(c, "k_svo_select");
    RGBD_TRY(c, launch_svo_select(w->d_cells, g, w->d_cand, w->d_ncand, c->d_count, c->d_kps, c->d_err, B, st), "svo_select");
    timer_end(c, tk);
#ifdef RGBD_PNP_PROFILE
    svo_prof_dump(st);
#endif
    tk = timer_begin(c, "k_svo_brief");
    RGBD_TRY(c, launch_svo_brief(w->d_box, c->d_count, c->d_kps, w->d_pat, g, c->d_desc, B, st), "svo_brief");
    timer_end(c, tk);
    tk = timer_begin(c, "k_undistort");
    RGBD_TRY(c, launch_undistort(d_depth, c->d_count, c->d_cfg, g.kp_cap, c->d_kps, c->d_kun, c->d_xyz, B, st), "undistort");
    timer_end(c, tk);
    c->last_B = B;
    return RGBD_OK;
}

}  // namespace rgbd

using namespace rgbd;

extern "C" {

rgbd_status rgbd_svo_set_brief_pattern(rgbd_ctx* c, const int8_t* pairs)
{
    if (!c || !pairs) return RGBD_ERR_ARG;
    if (!c->svo) return fail(c, RGBD_ERR_ARG, "not an SVO context (rgbd_create_svo)");
    for (int i = 0; i < 1024; i++)
        if (pairs[i] < -24 || pairs[i] > 24) return fail(c, RGBD_ERR_ARG, "BRIEF offsets must lie in [-24, 24]");
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    std::memcpy(ws(c)->pattern, pairs, 1024);
    if ((s = upload_pattern(c, ws(c)))) return s;
    return check_hip(c, hipStreamSynchronize(c->stream), "sync");
}

rgbd_status rgbd_svo_get_brief_pattern(rgbd_ctx* c, int8_t* pairs)
{
    if (!c || !pairs) return RGBD_ERR_ARG;
    if (!c->svo) return fail(c, RGBD_ERR_ARG, "not an SVO context (rgbd_create_svo)");
    std::memcpy(pairs, ws(c)->pattern, 1024);
    return RGBD_OK;
}

rgbd_status rgbd_svo_debug_level(rgbd_ctx* c, int32_t b, int32_t level, uint8_t* out)
{
    if (!c || !out || !c->svo || b < 0 || b >= c->last_B) return RGBD_ERR_ARG;
    SvoWS* w = ws(c);
    const SvoCfg& g = w->cfg;
    if (level < 0 || level >= g.nlevels) return RGBD_ERR_ARG;
    rgbd_status s = check_hip(c, hipMemcpyAsync(out, w->d_pyr + (size_t)b * g.frame_bytes + g.loff[level],
                                                (size_t)g.lw[level] * g.lh[level], hipMemcpyDeviceToHost, c->stream),
                              "read level");
    return s ? s : check_hip(c, hipStreamSynchronize(c->stream), "sync");
}

rgbd_status rgbd_svo_debug_grid(rgbd_ctx* c, int32_t b, int32_t* xyl, float* resp, int32_t cap, int32_t* n)
{
    if (!c || !n || !c->svo || b < 0 || b >= c->last_B) return RGBD_ERR_ARG;
    SvoWS* w = ws(c);
    const SvoCfg& g = w->cfg;
    int cnt = 0;
    rgbd_status s = check_hip(c, hipMemcpyAsync(&cnt, w->d_ncand + b, 4, hipMemcpyDeviceToHost, c->stream), "read ncand");
    if (!s) s = check_hip(c, hipStreamSynchronize(c->stream), "sync");
    if (s) return s;
    *n = cnt;
    if (cnt > cap) return fail(c, RGBD_ERR_CAPACITY, "output capacity smaller than the grid keypoint count");
    std::vector<uint2> v((size_t)cnt);
    if (cnt) {
        s = check_hip(c, hipMemcpyAsync(v.data(), w->d_cand + (size_t)b * g.ncells, (size_t)cnt * 8, hipMemcpyDeviceToHost,
                                        c->stream), "read candidates");
        if (!s) s = check_hip(c, hipStreamSynchronize(c->stream), "sync");
        if (s) return s;
    }
    for (int i = 0; i < cnt; i++) {
        const uint32_t ord = ~v[i].y;
        const int L = (int)(ord >> 22);
        if (xyl) {
            xyl[3 * i] = (int)(ord & 2047u) << L;
            xyl[3 * i + 1] = (int)((ord >> 11) & 2047u) << L;
            xyl[3 * i + 2] = L;
        }
        if (resp) std::memcpy(resp + i, &v[i].x, 4);
    }
    return RGBD_OK;
}

rgbd_status rgbd_svo_retain_best(rgbd_ctx* c, const float* resp, int32_t n, int32_t n_points, int32_t depth_limit,
                                 int32_t* order, int32_t* m)
{
    if (!c || !order || !m || n < 0 || (n > 0 && !resp)) return RGBD_ERR_ARG;
    if (!c->svo) return fail(c, RGBD_ERR_ARG, "not an SVO context (rgbd_create_svo)");
    if (n > kSvoSelThreads * kSvoSelMaxE) return fail(c, RGBD_ERR_UNSUPPORTED, "retainBest: n <= 12288");
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    SvoWS* w = ws(c);
    if (!w->d_rt_resp) {
        s = check_hip(c, hipMalloc((void**)&w->d_rt_resp, (size_t)kSvoSelThreads * kSvoSelMaxE * 4), "retain resp");
        if (!s) s = check_hip(c, hipMalloc((void**)&w->d_rt_order, ((size_t)kSvoSelThreads * kSvoSelMaxE + 1) * 4), "retain order");
        if (s) return s;
    }
    if (n == 0) { *m = 0; return RGBD_OK; }
    s = check_hip(c, hipMemcpyAsync(w->d_rt_resp, resp, (size_t)n * 4, hipMemcpyHostToDevice, c->stream), "retain up");
    if (s) return s;
    int* d_m = w->d_rt_order + kSvoSelThreads * kSvoSelMaxE;
    RGBD_TRY(c, launch_svo_retain_test(w->d_rt_resp, n, n_points < 0 ? n : n_points, depth_limit, w->d_rt_order, d_m, c->stream), "svo_retain_test");
    int mm = 0;
    s = check_hip(c, hipMemcpyAsync(&mm, d_m, 4, hipMemcpyDeviceToHost, c->stream), "retain m");
    if (!s) s = check_hip(c, hipStreamSynchronize(c->stream), "sync");
    if (s) return s;
    *m = mm;
    s = check_hip(c, hipMemcpyAsync(order, w->d_rt_order, (size_t)mm * 4, hipMemcpyDeviceToHost, c->stream), "retain order");
    return s ? s : check_hip(c, hipStreamSynchronize(c->stream), "sync");
}

}  // extern "C"

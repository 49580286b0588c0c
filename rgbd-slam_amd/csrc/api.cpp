// api.cpp -- C ABI (include/rgbd_hip.h): context, geometry, extraction and matching entry points.
//
// Geometry is derived here once per context with the reference's own float/double rules:
//   ORBextractor ctor (Features/ORBextractor.cpp:348-406): scale factors, per-level budgets, umax
//   ComputePyramid (:773-797): level sizes; OpenCV resize tables (xofs/ialpha/yofs/ibeta)
//   ComputeKeyPointsOctTree (:613-672): borders, 30-px cell grid, ROI ranges
//   DistributeOctTree (:420-422): nIni, hX
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <set>
#include <string>
#include <vector>

#include "context.h"
#include "launch.h"

#define RGBD_DIST_LDS_KB 38   // LDS per quadtree workgroup (four 512-thread workgroups per CU)

using namespace rgbd;

namespace rgbd {

rgbd_status fail(rgbd_ctx* c, rgbd_status code, const std::string& msg)
{
    if (c) c->err = msg;
    return code;
}

rgbd_status check_hip(rgbd_ctx* c, hipError_t e, const char* what)
{
    if (e == hipSuccess) return RGBD_OK;
    return fail(c, RGBD_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

rgbd_status order_after_extraction(rgbd_ctx* c)
{
    if (!c->extract_done || c->extract_stream == c->stream) return RGBD_OK;
    const rgbd_status s = check_hip(c, hipStreamWaitEvent(c->stream, c->extract_done, 0), "wait for extraction");
    if (!s) c->extract_stream = c->stream;   // ordered: later calls on this stream need no second wait
    return s;
}

static hipEvent_t ev_get(rgbd_ctx* c)
{
    if (!c->event_pool.empty()) {
        hipEvent_t e = c->event_pool.back();
        c->event_pool.pop_back();
        return e;
    }
    hipEvent_t e;
    (void)hipEventCreate(&e);
    return e;
}

int timer_begin(rgbd_ctx* c, const char* name, hipStream_t st)
{
    if (!c->timing) return -1;
    if (!c->timing_only.empty() && c->timing_only != name) return -1;
    int idx = -1;
    for (size_t i = 0; i < c->tentries.size(); i++)
        if (c->tentries[i].name == name) idx = (int)i;
    if (idx < 0) {
        c->tentries.push_back(rgbd_ctx::TEntry{name, 0.0, 0});
        idx = (int)c->tentries.size() - 1;
    }
    rgbd_ctx::Pending p{idx, ev_get(c), ev_get(c), st ? st : c->stream, false};
    (void)hipEventRecord(p.a, p.st);
    c->pending.push_back(p);
    return (int)c->pending.size() - 1;
}

void timer_end(rgbd_ctx* c, int tok)
{
    if (tok < 0) return;
    (void)hipEventRecord(c->pending[tok].b, c->pending[tok].st);
    c->pending[tok].ended = true;
}

void timer_flush(rgbd_ctx* c)
{
    for (auto& p : c->pending) {
        // a launch whose entry point returned early (RGBD_TRY) never recorded its end: not a timed launch
        float ms = 0;
        if (p.ended && hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            c->tentries[p.idx].ms += ms;
            c->tentries[p.idx].launches++;
        }
        c->event_pool.push_back(p.a);
        c->event_pool.push_back(p.b);
    }
    c->pending.clear();
}

}  // namespace rgbd

namespace {

inline int round_half_even_f(float v) { return (int)std::nearbyintf(v); }
inline int align_up(int v, int a) { return (v + a - 1) / a * a; }

struct HostGeom {
    std::vector<ResizeX> rsx;
    std::vector<ResizeY> rsy;
    std::vector<QuadX> qx;
};

// resize(INTER_LINEAR) tables of OpenCV 3.4 resize() for src (sw,sh) -> dst (dw,dh)
void resize_tables(int sw, int sh, int dw, int dh, HostGeom& g, LevelCfg& D)
{
    const double inv_scale_x = (double)dw / sw, inv_scale_y = (double)dh / sh;
    const double scale_x = 1. / inv_scale_x, scale_y = 1. / inv_scale_y;
    D.rs_scale_x = scale_x;
    D.rs_scale_y = scale_y;
    D.qx_off = 0;
    D.rsx_off = (int)g.rsx.size();
    D.rsy_off = (int)g.rsy.size();
    int xmax = dw;
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)std::floor(fx);
        fx -= sx;
        if (sx < 0) { fx = 0; sx = 0; }
        if (sx + 1 >= sw) {
            xmax = std::min(xmax, dx);
            if (sx >= sw - 1) { fx = 0; sx = sw - 1; }
        }
        const float c0 = 1.f - fx, c1 = fx;
        ResizeX e;
        e.sx = (int16_t)sx;
        e.a0 = (int16_t)std::min(std::max(round_half_even_f(c0 * 2048), -32768), 32767);
        e.a1 = (int16_t)std::min(std::max(round_half_even_f(c1 * 2048), -32768), 32767);
        e.pad = 0;
        g.rsx.push_back(e);
    }
    auto clip = [](int x, int a, int b) { return x >= a ? (x < b ? x : b - 1) : a; };
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        int sy = (int)std::floor(fy);
        fy -= sy;
        const float c0 = 1.f - fy, c1 = fy;
        ResizeY e;
        e.sy0 = (int16_t)clip(sy, 0, sh);
        e.sy1 = (int16_t)clip(sy + 1, 0, sh);
        e.b0 = (int16_t)std::min(std::max(round_half_even_f(c0 * 2048), -32768), 32767);
        e.b1 = (int16_t)std::min(std::max(round_half_even_f(c1 * 2048), -32768), 32767);
        g.rsy.push_back(e);
    }
    D.rs_xmax = xmax;
    int x = 0;
    for (; x <= dw - 16; x += 16) {}
    for (; x < dw - 4; x += 4) {}
    D.rs_simd = x;
}

rgbd_status build_geometry(rgbd_ctx* c, HostGeom& g)
{
    const rgbd_orb_params& o = c->orb;
    ExtractCfg& C = c->cfg;
    std::memset(&C, 0, sizeof(C));
    const int nl = o.nlevels;
    if (nl < 1 || nl > kMaxLevels) return fail(c, RGBD_ERR_UNSUPPORTED, "nlevels must be in [1, 12]");
    if (c->W % 16 != 0 || c->W <= 64 || c->H <= 64) return fail(c, RGBD_ERR_UNSUPPORTED, "width must be a multiple of 16 and > 64");
    if (c->W > 16 * kPyrThreads) return fail(c, RGBD_ERR_UNSUPPORTED, "width above 16 x the pyramid's threads per strip");
    C.W = c->W;
    C.H = c->H;
    C.nlevels = nl;
    C.ini_th = std::min(std::max(o.ini_th_fast, 0), 255);
    C.min_th = std::min(std::max(o.min_th_fast, 0), 255);
    // ORBextractor ctor
    const double scaleFactor = (double)o.scale_factor;
    std::vector<float> sf(nl), inv(nl);
    sf[0] = 1.0f;
    for (int i = 1; i < nl; i++) sf[i] = (float)((double)sf[i - 1] * scaleFactor);
    for (int i = 0; i < nl; i++) inv[i] = 1.0f / sf[i];
    const float factor = (float)(1.0f / scaleFactor);
    float nDesired = o.nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nl));
    std::vector<int> N(nl);
    int sum = 0;
    for (int l = 0; l < nl - 1; l++) {
        N[l] = round_half_even_f(nDesired);
        sum += N[l];
        nDesired *= factor;
    }
    N[nl - 1] = std::max(o.nfeatures - sum, 0);
    {
        int umax[16];
        const int HP = 15;
        const int vmax = (int)std::floor(HP * std::sqrt(2.f) / 2 + 1);
        const int vmin = (int)std::ceil(HP * std::sqrt(2.f) / 2);
        const double hp2 = HP * HP;
        int v, v0;
        for (v = 0; v <= vmax; ++v) umax[v] = (int)std::nearbyint(std::sqrt(hp2 - v * v));
        for (v = HP, v0 = 0; v >= vmin; --v) {
            while (umax[v0] == umax[v0 + 1]) ++v0;
            umax[v] = v0;
            ++v0;
        }
        for (int i = 0; i < 16; i++) C.umax[i] = umax[i];
        for (int r = 0; r < 31; r++) {
            const int um = umax[r < 15 ? 15 - r : r - 15];
            for (int k = 0; k < 8; k++) {
                uint32_t wu = 0, w1 = 0;
                for (int i = 0; i < 4; i++) {
                    const int u = 4 * k + i - 15;
                    if (u >= -um && u <= um) {
                        wu |= (uint32_t)(u + 16) << (8 * i);
                        w1 |= 1u << (8 * i);
                    }
                }
                C.ic_wu[r][k] = wu;
                C.ic_w1[r][k] = w1;
            }
        }
    }
    // levels
    int off = 0, cell_cap = 1, key_off = 0, sel_off = 0, maxNode = 8;
    c->cells.clear();
    c->segs.clear();
    for (int l = 0; l < nl; l++) {
        LevelCfg& L = C.lv[l];
        L.w = round_half_even_f((float)c->W * inv[l]);
        L.h = round_half_even_f((float)c->H * inv[l]);
        if (L.w < 48 || L.h < 48) return fail(c, RGBD_ERR_UNSUPPORTED, "pyramid level smaller than 48 px");
        L.stride = align_up(L.w, 64);
        L.off = off;
        off += align_up(L.stride * L.h, 256);
        L.scale = sf[l];
        L.size = (float)(int)(31 * sf[l]);
        L.N = N[l];
        const int EDGE = 19;
        L.minBX = EDGE - 3;
        L.minBY = EDGE - 3;
        L.maxBX = L.w - EDGE + 3;
        L.maxBY = L.h - EDGE + 3;
        // cells (:627-667)
        const float Wc = 30;
        const float width = (float)(L.maxBX - L.minBX), height = (float)(L.maxBY - L.minBY);
        const int nCols = (int)(width / Wc), nRows = (int)(height / Wc);
        if (nCols <= 0 || nRows <= 0) return fail(c, RGBD_ERR_UNSUPPORTED, "level too small for the 30-px cell grid");
        const int wCell = (int)std::ceil(width / nCols), hCell = (int)std::ceil(height / nRows);
        L.cell_begin = (int)c->cells.size();
        for (int i = 0; i < nRows; i++) {
            const float iniY = (float)(L.minBY + i * hCell);
            float maxY = iniY + hCell + 6;
            if (iniY >= L.maxBY - 3) continue;
            if (maxY > L.maxBY) maxY = (float)L.maxBY;
            for (int j = 0; j < nCols; j++) {
                const float iniX = (float)(L.minBX + j * wCell);
                float maxX = iniX + wCell + 6;
                if (iniX >= L.maxBX - 6) continue;
                if (maxX > L.maxBX) maxX = (float)L.maxBX;
                Cell cc;
                cc.level = (int16_t)l;
                cc.x0 = (int16_t)(int)iniX;
                cc.y0 = (int16_t)(int)iniY;
                cc.x1 = (int16_t)(int)maxX;
                cc.y1 = (int16_t)(int)maxY;
                cc.pad = 0;
                const int cw = cc.x1 - cc.x0, ch = cc.y1 - cc.y0;
                if (cw > kCellStride || ch > kCellStride)
                    return fail(c, RGBD_ERR_UNSUPPORTED, "FAST cell ROI larger than 48 px");
                const int a = std::max(cw - 6, 0), b = std::max(ch - 6, 0);
                cell_cap = std::max(cell_cap, ((a + 1) / 2) * ((b + 1) / 2));
                c->cells.push_back(cc);
            }
        }
        L.cell_count = (int)c->cells.size() - L.cell_begin;
        {   // k_fast segments: consecutive cells of one cell row, 64 / lanes-per-cell of them per wave
            int np_max = 1;
            for (int q = L.cell_begin; q < (int)c->cells.size(); q++)
                np_max = std::max(np_max, (c->cells[q].x1 - c->cells[q].x0 - 6 + 1) / 2);
            // 16 lanes (a DPP row) per cell when the pairs fit, else exactly the widest cell's pairs: a level
            // whose cells hold 17-19 pairs (640 x 480: levels 5 and 7) packs 3 cells per wave, not 2 of 32 lanes
            const int lpc = np_max <= 16 ? 16 : np_max;
            if (lpc > 32) return fail(c, RGBD_ERR_UNSUPPORTED, "FAST cell interior wider than 64 px");
            const int cpw = 64 / lpc;
            // a segment's staged row (16-B aligned start .. x1 + 6) must fit k_fast's kFastRowBytes = 160
            auto row_bytes = [&](int q0, int e0) { return c->cells[e0 - 1].x1 + 6 - (c->cells[q0].x0 & ~15); };
            for (int q = L.cell_begin; q < (int)c->cells.size();) {
                int e = q + 1;
                while (e < (int)c->cells.size() && e - q < cpw && c->cells[e].y0 == c->cells[q].y0 &&
                       row_bytes(q, e + 1) <= 160)
                    e++;
                if (row_bytes(q, e) > 160) return fail(c, RGBD_ERR_UNSUPPORTED, "FAST segment row wider than 160 B");
                c->segs.push_back(FastSeg{q, (int16_t)(e - q), (int16_t)lpc});
                q = e;
            }
        }
        // DistributeOctTree roots (:420-422)
        const int dX = L.maxBX - L.minBX, dY = L.maxBY - L.minBY;
        L.nIni = (int)std::round(static_cast<float>(dX) / dY);
        if (L.nIni < 1) return fail(c, RGBD_ERR_UNSUPPORTED, "image taller than 2x its width (nIni == 0)");
        L.hX = static_cast<float>(dX) / L.nIni;
        const int selCap = std::max(L.N + 3, 4 * L.nIni);
        L.sel_off = sel_off;
        sel_off += align_up(selCap, 4);
        maxNode = std::max(maxNode, std::max(L.N + 8, 4 * L.nIni + 8));
    }
    C.frame_pyr_bytes = off;
    C.n_cells = (int)c->cells.size();
    C.cell_cap = cell_cap;
    for (int l = 0; l < nl; l++) {
        LevelCfg& L = C.lv[l];
        L.key_off = key_off;
        L.key_cap = L.cell_count * cell_cap;
        key_off += L.key_cap;
        if (L.key_cap >= (1 << 24)) return fail(c, RGBD_ERR_UNSUPPORTED, "too many FAST candidates per level");
    }
    C.keys_per_frame = key_off;
    C.sel_per_frame = sel_off;
    for (int l = 0; l < kMaxLevels; l++) C.sel_off_tab[l] = l < nl ? C.lv[l].sel_off : INT32_MAX;
    int NC = 64;
    while (NC < maxNode) NC <<= 1;
    if (NC > 4096) return fail(c, RGBD_ERR_UNSUPPORTED, "nfeatures too large for the quadtree node capacity");
    C.node_cap = NC;
    {
        int mc = 0;
        for (int l = 0; l < nl; l++) mc = std::max(mc, C.lv[l].cell_count);
        C.scan_cap = std::max(NC, mc) + 1;
    }
    // quadtree round state in LDS: per candidate its u32 key + its node id (u8 while node_cap <= 256, else
    // u16), within RGBD_DIST_LDS_KB per workgroup (four 512-thread workgroups per CU); a level with more
    // candidates keeps it in HBM.  Round 4 (level-major dispatch): 32 / 38 / 44 / 52 / 80 KB measured
    // 0.54 / 0.53 / 0.62 / 0.61 / 0.74 ms per 1024 frames -- occupancy beats residency for this latency-bound kernel
    {
        const int per_key = 4 + (NC <= 256 ? 1 : 2);
        const long room = (long)RGBD_DIST_LDS_KB * 1024 - (long)distribute_lds_bytes(NC, C.scan_cap);
        C.dist_kc = room > 0 ? (int)(room / per_key / 64 * 64) : 0;
    }
    C.kp_cap = align_up(sel_off, 4);
    // resize tables (level l from level l-1)
    for (int l = 1; l < nl; l++)
        resize_tables(C.lv[l - 1].w, C.lv[l - 1].h, C.lv[l].w, C.lv[l].h, g, C.lv[l]);
    // k_pyramid strips (levels < pyr_top): each strip owns an equal share of every level's rows (written to HBM); walking
    // down from the top level, level l-1 must also hold the source rows (sy0, sy1) of the rows level l
    // computes.  Levels l < Lf are also blurred in k_pyramid (GaussianBlur 7x7): the level is partitioned
    // into blur rows [pb_r0, pb_r1) per strip with the boundaries in the middle of the neighbouring
    // strips' overlap, and a strip's computed rows are widened to its blur rows +- 3 (REFLECT_101 rows
    // at the image edges fall inside them).  The overlaps of the lowest levels already exceed 6 rows,
    // so fusing them costs almost no extra resize work; the top levels' would cascade down the chain.
    {
        size_t lds_a = 0, lds_b = 0;   // even / odd level strip buffers
        const int Lf = nl > 1 ? std::min(kPbLevels, nl) : 0;
        const int top = std::min(nl, kPyrStripLevels);   // levels top .. nl-1: k_pyr_tail, no strip rows
        C.pyr_top = top;
        int r0[kPyrStrips][kMaxLevels], r1[kPyrStrips][kMaxLevels];
        for (int l = 0; l < kMaxLevels; l++) C.pb_seg[l] = 0;
        for (int s_ = 0; s_ < kPyrStrips; s_++)
            for (int l = 0; l < kMaxLevels; l++) {
                C.strip_r0[s_][l] = C.strip_r1[s_][l] = 0;
                C.pb_r0[s_][l] = C.pb_r1[s_][l] = 0;
            }
        for (int l = top - 1; l >= 0; l--) {
            const int h = C.lv[l].h;
            for (int s_ = 0; s_ < kPyrStrips; s_++) {
                r0[s_][l] = (int)((long)h * s_ / kPyrStrips);
                r1[s_][l] = (int)((long)h * (s_ + 1) / kPyrStrips);
                if (l + 1 < top && r1[s_][l + 1] > r0[s_][l + 1]) {
                    const ResizeY& a = g.rsy[C.lv[l + 1].rsy_off + r0[s_][l + 1]];
                    const ResizeY& z = g.rsy[C.lv[l + 1].rsy_off + r1[s_][l + 1] - 1];
                    r0[s_][l] = std::min(r0[s_][l], (int)a.sy0);
                    r1[s_][l] = std::max(r1[s_][l], (int)z.sy1 + 1);
                }
                C.pb_r0[s_][l] = C.pb_r1[s_][l] = 0;
            }
            if (l >= Lf) continue;
            int beta[kPyrStrips + 1];
            beta[0] = 0;
            beta[kPyrStrips] = h;
            for (int s_ = 1; s_ < kPyrStrips; s_++)
                beta[s_] = std::min(std::max((r0[s_][l] + r1[s_ - 1][l]) / 2, beta[s_ - 1]), h);
            int maxrows = 0;
            for (int s_ = 0; s_ < kPyrStrips; s_++) {
                const int b0 = beta[s_], b1 = std::max(beta[s_ + 1], b0);
                C.pb_r0[s_][l] = (int16_t)b0;
                C.pb_r1[s_][l] = (int16_t)b1;
                if (b1 <= b0) continue;
                r0[s_][l] = std::min(r0[s_][l], std::max(b0 - 3, 0));
                r1[s_][l] = std::max(r1[s_][l], std::min(b1 + 3, h));
                maxrows = std::max(maxrows, b1 - b0);
                // every row the blur reads (REFLECT_101) is computed by this strip
                for (int y = b0 - 3; y < b1 + 3; y++) {
                    const int ry = y < 0 ? -y : (y >= h ? 2 * h - 2 - y : y);
                    if (ry < r0[s_][l] || ry >= r1[s_][l])
                        return fail(c, RGBD_ERR_UNSUPPORTED, "fused blur row outside its pyramid strip");
                }
            }
            C.pb_seg[l] = (maxrows + kPbRows - 1) / kPbRows;
        }
        for (int s_ = 0; s_ < kPyrStrips; s_++) {
            for (int l = 0; l < top; l++) {
                const size_t bytes = (size_t)(r1[s_][l] - r0[s_][l]) * C.lv[l].stride;
                if (l % 2 == 0) lds_a = std::max(lds_a, bytes);
                else lds_b = std::max(lds_b, bytes);
                C.strip_r0[s_][l] = (int16_t)r0[s_][l];
                C.strip_r1[s_][l] = (int16_t)r1[s_][l];
            }
        }
        lds_a = (lds_a + 15) / 16 * 16;

        C.pyr_lds_b = (int)lds_a;
        C.pyr_lds = (int)((lds_a + lds_b + 16 + 15) / 16 * 16);   // + 16: a quad's 12-byte tap window may run past the last row
        // + the strip's resize row entries of levels 1..L-1 (k_pyramid stages them after the level buffers)
        int rows = 0;
        for (int s_ = 0; s_ < kPyrStrips; s_++) {
            int n = 0;
            for (int l = 1; l < top; l++) n += r1[s_][l] - r0[s_][l];
            rows = std::max(rows, n);
        }
        C.pyr_rsy_lds = (int)(rows * sizeof(ResizeY));
    }
    if (C.pyr_lds + C.pyr_rsy_lds > 150 * 1024) return fail(c, RGBD_ERR_UNSUPPORTED, "pyramid strip does not fit in LDS");
    // k_pyramid reads a quad's horizontal taps from the 12-byte window (sx of its first pixel) & ~3 ..
    // + 11 of each source row, aligned to the 8 bytes from that pixel's left tap (two v_alignbyte per
    // row): the right tap of its last pixel must lie within them (scale <= ~2)
    g.qx.clear();
    for (int l = 1; l < nl; l++) {
        LevelCfg& D = C.lv[l];
        const int sw = C.lv[l - 1].w;
        D.qx_off = (int)g.qx.size();
        for (int dx = 0; dx < D.w; dx += 4) {
            const int sx0 = g.rsx[D.rsx_off + dx].sx, wb = sx0 & ~3;
            const int sx3 = g.rsx[D.rsx_off + std::min(dx + 3, D.w - 1)].sx;
            if (std::min(sx3 + 1, sw - 1) - sx0 > 7)
                return fail(c, RGBD_ERR_UNSUPPORTED, "pyramid scale factor too large for the resize tap window");
            QuadX q{};
            for (int i = 0; i < 4; i++) {
                const ResizeX& rx = g.rsx[D.rsx_off + std::min(dx + i, D.w - 1)];
                const int pad = rx.sx + 1 < sw ? rx.sx + 1 : rx.sx;
                const int o0 = rx.sx - sx0, o1 = pad - sx0;   // bytes of the 8-byte window from sx0
                q.sel[i] = (uint32_t)o0 | 0x0c00u | ((uint32_t)o1 << 16) | 0x0c000000u;
                const int a0 = dx + i < D.rs_xmax ? rx.a0 : 2048, a1 = dx + i < D.rs_xmax ? rx.a1 : 0;
                q.wt[i] = (uint32_t)(16 * a0) | ((uint32_t)(16 * a1) << 16);
                q.simd |= (dx + i < D.rs_simd ? 1u : 0u) << i;
            }
            q.wbpi = (uint32_t)wb | ((uint32_t)(sx0 - wb) << 16);   // window base | its byte shift
            g.qx.push_back(q);
        }
    }
    // level blur threads: one per column quad of each 32-row strip of each level; inner quads (bytes
    // x - 4 .. x + 11 inside the row) first, edge quads after them
    {
        int t = 0, e = 0;
        for (int l = 0; l < kMaxLevels; l++) {
            C.blur_t0[l] = t;
            C.blur_e0[l] = e;
            C.blur_tx[l] = C.blur_ex[l] = 0;
            if (l >= nl) continue;
            const int w = C.lv[l].w, Q = (w + 3) / 4, ty = (C.lv[l].h + kBlurTH - 1) / kBlurTH;
            if (w < 16 || C.lv[l].h < 8) return fail(c, RGBD_ERR_UNSUPPORTED, "pyramid level smaller than 16x8");
            const int qe = (w - 8) / 4 + 1;   // first quad with 4q + 8 > w
            C.blur_tx[l] = qe - 1;            // inner quads 1 .. qe - 1
            C.blur_ex[l] = 1 + (Q - qe);      // quad 0 and quads qe .. Q - 1
            if (C.pb_seg[l] > 0) continue;    // blurred inside k_pyramid: no blur threads
            t += C.blur_tx[l] * ty;
            e += C.blur_ex[l] * ty;
        }
        C.blur_t0[kMaxLevels] = t;
        C.blur_e0[kMaxLevels] = e;
    }
    // camera
    const rgbd_camera& k = c->cam;
    C.fx = k.fx; C.fy = k.fy; C.cx = k.cx; C.cy = k.cy;
    C.invfx = 1.0f / k.fx;
    C.invfy = 1.0f / k.fy;
    C.k1 = k.k1; C.k2 = k.k2; C.p1 = k.p1; C.p2 = k.p2; C.k3 = k.k3;
    C.depth_factor = k.depth_map_factor;
    C.undistort = (k.k1 != 0.0f) ? 1 : 0;
    return RGBD_OK;
}

template <typename T>
rgbd_status dalloc(rgbd_ctx* c, T** p, size_t count, const char* what)
{
    const size_t bytes = std::max<size_t>(count * sizeof(T), 16);
    return check_hip(c, hipMalloc((void**)p, bytes), what);
}

// a later call that reads the extraction's outputs on another stream waits on this event
// (order_after_extraction: rgbd_set_stream, and rgbd_track_lanes on the extracted frames)
static rgbd_status mark_extracted(rgbd_ctx* c)
{
    rgbd_status s;
    if (!c->extract_done &&
        (s = check_hip(c, hipEventCreateWithFlags(&c->extract_done, hipEventDisableTiming), "extract event")))
        return s;
    if ((s = check_hip(c, hipEventRecord(c->extract_done, c->stream), "extract event record"))) return s;
    c->extract_stream = c->stream;
    return RGBD_OK;
}

rgbd_status run_extract(rgbd_ctx* c, const uint8_t* d_bgr, const uint16_t* d_depth, int B, bool from_gray,
                        const rgbd::ExtractHook* after_fast = nullptr)
{
    // per-frame capacity flags (k_distribute / k_svo_select), cleared for every extraction
    rgbd_status s0 = check_hip(c, hipMemsetAsync(c->d_err, 0, sizeof(int) * (size_t)B, c->stream), "clear err");
    if (s0) return s0;
    if (c->svo) {
        if ((s0 = svo_run_extract(c, d_bgr, d_depth, B, from_gray, after_fast))) return s0;
        return mark_extracted(c);
    }
    ExtractCfg& C = c->cfg;
    hipStream_t st = c->stream;
    int tk;
    if (C.nlevels > 1) {   // k_pyramid converts BGR -> gray (level 0) itself unless given a gray level 0
        tk = timer_begin(c, "k_pyramid");
        RGBD_TRY(c, launch_pyramid(c->d_pyr, c->d_blur, from_gray ? nullptr : d_bgr, c->d_rsy, c->d_qx, c->d_cfg, C.pyr_lds + C.pyr_rsy_lds, B, st), "pyramid");
        timer_end(c, tk);
        if (C.pyr_top < C.nlevels) {   // the small levels after the strips
            tk = timer_begin(c, "k_pyr_tail");
            RGBD_TRY(c, launch_pyr_tail(c->d_pyr, c->d_rsy, c->d_qx, c->d_cfg, B, st), "pyramid tail");
            timer_end(c, tk);
        }
    } else if (!from_gray) {
        tk = timer_begin(c, "k_gray");
        RGBD_TRY(c, launch_gray(d_bgr, c->d_pyr, C.W, C.H, C.frame_pyr_bytes, B, st), "gray");
        timer_end(c, tk);
    }
    auto hook = [&](int at) -> rgbd_status { return after_fast ? (*after_fast)(at) : RGBD_OK; };
    rgbd_status hs;
    if ((hs = hook(0))) return hs;
    // the lowest levels' blur is fused into k_pyramid (blurred while the strip is in LDS); the others (all
    // of a 1-level pyramid) are blurred by each frame's leading blocks of the k_fast grid (blur_thread), so
    // blur and FAST waves share the CUs inside one launch
    tk = timer_begin(c, "k_fast");
#ifdef RGBD_PNP_PROFILE
    // profiling build: RGBD_PROF_FAST_SPLIT=1 dispatches the grid's blur blocks and its FAST segments as two
    // k_fast launches (blur-only grid first), so per-dispatch counters give the blur's share of the launch
    if (getenv("RGBD_PROF_FAST_SPLIT")) {
        RGBD_TRY(c, launch_fast(c->d_pyr, c->d_cells, c->d_segs, 0, c->d_cfg, c->d_cellc, c->d_slots, B, st, c->d_blur,
                    C.blur_t0[kMaxLevels] + C.blur_e0[kMaxLevels]), "fast (blur blocks)");
        RGBD_TRY(c, launch_fast(c->d_pyr, c->d_cells, c->d_segs, (int)c->segs.size(), c->d_cfg, c->d_cellc, c->d_slots, B, st,
                    c->d_blur, 0), "fast (segments)");
    } else
#endif
    RGBD_TRY(c, launch_fast(c->d_pyr, c->d_cells, c->d_segs, (int)c->segs.size(), c->d_cfg, c->d_cellc, c->d_slots, B, st, c->d_blur,
                C.blur_t0[kMaxLevels] + C.blur_e0[kMaxLevels]), "fast");
    timer_end(c, tk);
    // e.g. the deferred PnPRansac solves of earlier pipelined steps (pnp_host.cpp)
    if ((hs = hook(1))) return hs;
    tk = timer_begin(c, "k_distribute");
    RGBD_TRY(c, launch_distribute(c->d_cellc, c->d_slots, c->d_cfg, C.node_cap, C.scan_cap, 0, C.nlevels, C.dist_kc, c->d_keys,
                      c->d_node, c->d_selc, c->d_sel, c->d_err, B, st), "distribute");
    timer_end(c, tk);
    if ((hs = hook(2))) return hs;
#ifdef RGBD_PNP_PROFILE
    pyr_prof_dump(st);
    fprintf(stderr, "[pyr_lds] %d bytes per workgroup (odd levels at %d)\n", C.pyr_lds, C.pyr_lds_b);
    fast_prof_dump(st, (int)c->segs.size());
    dist_prof_dump(st);
#endif
    tk = timer_begin(c, "k_describe");
    RGBD_TRY(c, launch_describe(c->d_pyr, c->d_blur, c->d_selc, sel_count_elems(c->maxB, C.nlevels), C.nlevels, c->d_sel, c->d_cfg,
                                C.kp_cap, c->d_count, c->d_kps, c->d_desc, B, st), "describe");
    timer_end(c, tk);
    tk = timer_begin(c, "k_undistort");
    RGBD_TRY(c, launch_undistort(d_depth, c->d_count, c->d_cfg, C.kp_cap, c->d_kps, c->d_kun, c->d_xyz, B, st), "undistort");
    timer_end(c, tk);
    c->last_B = B;
#ifdef RGBD_PNP_PROFILE
    desc_prof_dump(st);
#endif
    return mark_extracted(c);
}

rgbd_status read_frame(rgbd_ctx* c, int b, rgbd_keypoint* kps, rgbd_keypoint* kun, uint8_t* desc, float* xyz,
                       int cap, int* n)
{
    const int K = c->cfg.kp_cap;
    int cnt = 0;
    rgbd_status s = check_hip(c, hipMemcpyAsync(&cnt, c->d_count + b, sizeof(int), hipMemcpyDeviceToHost, c->stream),
                              "read count");
    if (s) return s;
    int errflag = 0;
    if ((s = check_hip(c, hipMemcpyAsync(&errflag, c->d_err + b, sizeof(int), hipMemcpyDeviceToHost, c->stream), "read err")))
        return s;
    if ((s = check_hip(c, hipStreamSynchronize(c->stream), "sync"))) return s;
    if (errflag & 2) return fail(c, RGBD_ERR_CAPACITY, "SVO: keypoints kept by retainBest exceed rgbd_max_keypoints");
    if (errflag) return fail(c, RGBD_ERR_CAPACITY, "quadtree node capacity exceeded");
    if (n) *n = cnt;
    if (cnt > cap) return fail(c, RGBD_ERR_CAPACITY, "output capacity smaller than keypoint count");
    if (cnt == 0) return RGBD_OK;
    const size_t o = (size_t)b * K;
    if (kps && (s = check_hip(c, hipMemcpyAsync(kps, c->d_kps + o * 7, (size_t)cnt * 28, hipMemcpyDeviceToHost, c->stream), "read kps"))) return s;
    if (kun && (s = check_hip(c, hipMemcpyAsync(kun, c->d_kun + o * 7, (size_t)cnt * 28, hipMemcpyDeviceToHost, c->stream), "read kun"))) return s;
    if (desc && (s = check_hip(c, hipMemcpyAsync(desc, c->d_desc + o * 32, (size_t)cnt * 32, hipMemcpyDeviceToHost, c->stream), "read desc"))) return s;
    if (xyz && (s = check_hip(c, hipMemcpyAsync(xyz, c->d_xyz + o * 3, (size_t)cnt * 12, hipMemcpyDeviceToHost, c->stream), "read xyz"))) return s;
    return check_hip(c, hipStreamSynchronize(c->stream), "sync");
}

rgbd_status create_ctx(int device, int width, int height, int max_batch, const rgbd_orb_params* orb,
                       const rgbd_svo_params* svo, const rgbd_camera* cam, rgbd_ctx** out)
{
    if (!out || !orb || !cam || max_batch < 1) return RGBD_ERR_ARG;
    *out = nullptr;
    rgbd_ctx* c = new rgbd_ctx();
    c->device = device;
    c->W = width;
    c->H = height;
    c->maxB = max_batch;
    c->orb = *orb;
    c->cam = *cam;
    HostGeom g;
    rgbd_status s = build_geometry(c, g);
    if (s) { *out = c; return s; }
    if (svo && (s = svo_configure(c, *svo))) { *out = c; return s; }   // sets cfg.kp_cap before the allocations
    if ((s = check_hip(c, hipSetDevice(device), "hipSetDevice"))) { *out = c; return s; }
    if ((s = check_hip(c, hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking), "stream"))) { *out = c; return s; }
    c->stream = c->own_stream;
    {
        const char* ser = std::getenv("RGBD_SERIAL");
        c->serial = ser && std::atoi(ser) != 0;
    }
    const ExtractCfg& C = c->cfg;
    const size_t B = (size_t)max_batch;
    // k_describe addresses the pyramids with 32-bit byte offsets from the buffer base
    if (B * C.frame_pyr_bytes + 64 > 0xFFFFFFFFull) {
        *out = c;
        return fail(c, RGBD_ERR_CAPACITY, "max_batch x pyramid bytes exceeds 4 GiB (use more contexts)");
    }
    // k_fast addresses the FAST cell lists with 32-bit byte offsets too
    if (B * C.n_cells * C.cell_cap * 4 > 0xFFFFFFFFull) {
        *out = c;
        return fail(c, RGBD_ERR_CAPACITY, "max_batch x FAST cell lists exceed 4 GiB (use more contexts)");
    }
    s = dalloc(c, &c->d_cfg, 1, "cfg");
    if (!s) s = dalloc(c, &c->d_cells, C.n_cells, "cells");
    if (!s) s = dalloc(c, &c->d_segs, c->segs.size(), "fast segments");
    if (!s) s = dalloc(c, &c->d_rsx, g.rsx.size(), "rsx");
    if (!s) s = dalloc(c, &c->d_qx, g.qx.size(), "resize quads");
    if (!s) s = dalloc(c, &c->d_rsy, g.rsy.size(), "rsy");
    if (!s) s = dalloc(c, &c->d_pyr, B * C.frame_pyr_bytes + 64, "pyramid");
    if (!s) s = dalloc(c, &c->d_blur, B * C.frame_pyr_bytes + 64, "blurred pyramid");
    if (!s) s = dalloc(c, &c->d_cellc, B * C.n_cells, "cell counts");
    if (!s) s = dalloc(c, &c->d_slots, B * C.n_cells * C.cell_cap, "cell slots");
    if (!s) s = dalloc(c, &c->d_keys, B * C.keys_per_frame, "keys");
    if (!s) s = dalloc(c, &c->d_node, B * C.keys_per_frame, "node ids");
    // + kMaxLevels of slack: k_describe reads kMaxLevels counts from any frame's row unconditionally
    if (!s) s = dalloc(c, &c->d_selc, sel_count_elems((int)B, C.nlevels), "sel counts");
    if (!s) s = dalloc(c, &c->d_sel, B * C.sel_per_frame, "sel");
    if (!s) s = dalloc(c, &c->d_count, B, "counts");
    if (!s) s = dalloc(c, &c->d_kps, B * C.kp_cap * 7, "kps");
    if (!s) s = dalloc(c, &c->d_kun, B * C.kp_cap * 7, "kps_un");
    if (!s) s = dalloc(c, &c->d_desc, B * C.kp_cap * 32, "desc");
    if (!s) s = dalloc(c, &c->d_xyz, B * C.kp_cap * 3, "xyz");
    if (!s) s = dalloc(c, &c->d_err, B, "err");   // one flag per frame
    if (!s) s = dalloc(c, &c->d_in_bgr, (size_t)width * height * 3, "bgr staging");
    if (!s) s = dalloc(c, &c->d_in_depth, (size_t)width * height, "depth staging");
    if (!s) s = dalloc(c, &c->d_knn, B * C.kp_cap, "knn");
    if (!s) s = dalloc(c, &c->d_pairs, 2 * B, "pairs");
    if (s) { *out = c; return s; }
    s = check_hip(c, hipMemcpy(c->d_cfg, &c->cfg, sizeof(ExtractCfg), hipMemcpyHostToDevice), "upload cfg");
    if (!s) s = check_hip(c, hipMemcpy(c->d_cells, c->cells.data(), c->cells.size() * sizeof(Cell), hipMemcpyHostToDevice), "upload cells");
    if (!s) s = check_hip(c, hipMemcpy(c->d_segs, c->segs.data(), c->segs.size() * sizeof(FastSeg), hipMemcpyHostToDevice), "upload segments");
    if (!s && !g.rsx.empty()) s = check_hip(c, hipMemcpy(c->d_rsx, g.rsx.data(), g.rsx.size() * sizeof(ResizeX), hipMemcpyHostToDevice), "upload rsx");
    if (!s && !g.qx.empty()) s = check_hip(c, hipMemcpy(c->d_qx, g.qx.data(), g.qx.size() * sizeof(QuadX), hipMemcpyHostToDevice), "upload quads");
    if (!s && !g.rsy.empty()) s = check_hip(c, hipMemcpy(c->d_rsy, g.rsy.data(), g.rsy.size() * sizeof(ResizeY), hipMemcpyHostToDevice), "upload rsy");
    if (!s) s = check_hip(c, hipMemset(c->d_err, 0, sizeof(int) * B), "memset err");
    if (!s) s = check_hip(c, hipMemset(c->d_pyr, 0, B * C.frame_pyr_bytes + 64), "memset pyr");
    if (!s) s = check_hip(c, hipMemset(c->d_blur, 0, B * C.frame_pyr_bytes + 64), "memset blur");
    if (!s && svo) s = svo_alloc(c);
    *out = c;
    return s;
}

}  // namespace

extern "C" {

rgbd_status rgbd_create(int device, int width, int height, int max_batch, const rgbd_orb_params* orb,
                        const rgbd_camera* cam, rgbd_ctx** out)
{
    return create_ctx(device, width, height, max_batch, orb, nullptr, cam, out);
}

rgbd_status rgbd_create_svo(int device, int width, int height, int max_batch, const rgbd_svo_params* svo,
                            const rgbd_camera* cam, rgbd_ctx** out)
{
    if (!svo) return RGBD_ERR_ARG;
    // Extractor::Extractor -> setParameters(1000, 1.2f, 8, 20, 7) (Features/Extractor.cpp:15-22): the ORB
    // fields only shape the scale tables the reference's getters report (the ORB workspace is never run,
    // so its budget is kept small)
    const rgbd_orb_params orb{std::max(1, std::min(svo->nfeatures, 1000)), 1.2f, 8, 20, 7};
    return create_ctx(device, width, height, max_batch, &orb, svo, cam, out);
}

void rgbd_destroy(rgbd_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
    if (c->solve_stream) (void)hipStreamSynchronize(c->solve_stream);
    if (c->match_stream) (void)hipStreamSynchronize(c->match_stream);
    rgbd::pnp_free(c);   // first: restores the context's own output buffers (pipelined double buffering)
    void* ptrs[] = {c->d_cfg, c->d_cells, c->d_segs, c->d_rsx, c->d_rsy, c->d_qx, c->d_pyr, c->d_blur, c->d_cellc, c->d_slots, c->d_keys,
                    c->d_node, c->d_selc, c->d_sel, c->d_count, c->d_kps, c->d_kun, c->d_desc, c->d_xyz,
                    c->d_err, c->d_in_bgr, c->d_in_depth, c->d_knn, c->d_pairs, c->d_mdesc, c->d_mcount,
                    c->d_mknn};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    rgbd::ransac_free(c);
    rgbd::gicp_free(c);
    rgbd::cloud_free(c);
    rgbd::svo_free(c);
    for (auto& p : c->pending) { (void)hipEventDestroy(p.a); (void)hipEventDestroy(p.b); }
    for (auto e : c->event_pool) (void)hipEventDestroy(e);
    if (c->extract_done) (void)hipEventDestroy(c->extract_done);
    for (hipStream_t* sp : {&c->solve_stream, &c->match_stream})   // serial: aliases of own_stream
        if (*sp && *sp != c->own_stream) (void)hipStreamDestroy(*sp);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
}

const char* rgbd_last_error(const rgbd_ctx* c) { return c ? c->err.c_str() : "null context"; }

int32_t rgbd_max_keypoints(const rgbd_ctx* c) { return c ? c->cfg.kp_cap : 0; }

rgbd_status rgbd_debug_fast_rank16(rgbd_ctx* c, const uint8_t* flags, int32_t rows, uint32_t* slots, uint32_t* counts)
{
    if (!c || rows < 1 || rows > 4096 || !flags || !slots || !counts) return RGBD_ERR_ARG;
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    uint8_t* d_f = nullptr;
    uint32_t* d_s = nullptr;
    const size_t n = (size_t)rows * 64;
    s = check_hip(c, hipMalloc((void**)&d_f, n), "rank flags");
    if (!s) s = check_hip(c, hipMalloc((void**)&d_s, n * 4 + 64 * 4), "rank slots");
    if (!s) s = check_hip(c, hipMemcpyAsync(d_f, flags, n, hipMemcpyHostToDevice, c->stream), "rank in");
    if (!s) {
        s = check_hip(c, rgbd::launch_debug_rank16(d_f, rows, d_s, d_s + n, c->stream), "launch of k_debug_rank16");
    }
    if (!s) s = check_hip(c, hipMemcpyAsync(slots, d_s, n * 4, hipMemcpyDeviceToHost, c->stream), "rank out");
    if (!s) s = check_hip(c, hipMemcpyAsync(counts, d_s + n, 64 * 4, hipMemcpyDeviceToHost, c->stream), "rank counts");
    if (!s) s = check_hip(c, hipStreamSynchronize(c->stream), "rank sync");
    if (d_f) (void)hipFree(d_f);
    if (d_s) (void)hipFree(d_s);
    return s;
}

rgbd_status rgbd_set_stream(rgbd_ctx* c, void* stream)
{
    if (!c) return RGBD_ERR_ARG;
    const hipStream_t prev = c->stream;
    c->stream = stream ? (hipStream_t)stream : c->own_stream;
    // every consumer of the last extraction's outputs (rgbd_track_lanes / rgbd_batch_frame / the debug
    // readers, or the caller's own kernels on this stream) is then ordered behind it; if that wait cannot be
    // queued the context keeps its previous stream, so the call can be retried
    const rgbd_status s = order_after_extraction(c);
    if (s) c->stream = prev;
    return s;
}

rgbd_status rgbd_detect_and_compute(rgbd_ctx* c, const uint8_t* gray, int32_t step, rgbd_keypoint* kps,
                                    uint8_t* desc, int32_t cap, int32_t* n)
{
    if (!c) return RGBD_ERR_ARG;
    if (n) *n = 0;
    if (!gray) return RGBD_OK;   // empty image -> no output (:708-709)
    if (step < c->W) return fail(c, RGBD_ERR_ARG, "step < width");
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    if (c->svo)
        s = check_hip(c, hipMemcpy2DAsync(svo_gray_level(c), c->W, gray, step, c->W, c->H, hipMemcpyHostToDevice, c->stream),
                      "upload gray");
    else
        s = check_hip(c, hipMemcpy2DAsync(c->d_pyr, c->cfg.lv[0].stride, gray, step, c->W, c->H, hipMemcpyHostToDevice, c->stream),
                      "upload gray");
    if (s) return s;
    if ((s = run_extract(c, nullptr, nullptr, 1, true))) return s;
    return read_frame(c, 0, kps, nullptr, desc, nullptr, cap, n);
}

rgbd_status rgbd_frame(rgbd_ctx* c, const uint8_t* bgr, const uint16_t* depth, rgbd_keypoint* kps,
                       rgbd_keypoint* kun, uint8_t* desc, float* xyz, int32_t cap, int32_t* n)
{
    if (!c || !bgr || !depth) return RGBD_ERR_ARG;
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    const size_t px = (size_t)c->W * c->H;
    if ((s = check_hip(c, hipMemcpyAsync(c->d_in_bgr, bgr, px * 3, hipMemcpyHostToDevice, c->stream), "upload bgr"))) return s;
    if ((s = check_hip(c, hipMemcpyAsync(c->d_in_depth, depth, px * 2, hipMemcpyHostToDevice, c->stream), "upload depth"))) return s;
    if ((s = run_extract(c, c->d_in_bgr, c->d_in_depth, 1, false))) return s;
    return read_frame(c, 0, kps, kun, desc, xyz, cap, n);
}

rgbd_status rgbd_extract_batch(rgbd_ctx* c, const void* d_bgr, const void* d_depth, int32_t B)
{
    if (!c || !d_bgr || B < 1) return RGBD_ERR_ARG;
    if (B > c->maxB) return fail(c, RGBD_ERR_CAPACITY, "batch larger than max_batch");
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    return run_extract(c, (const uint8_t*)d_bgr, (const uint16_t*)d_depth, B, false);
}

rgbd_status rgbd_batch_frame(rgbd_ctx* c, int32_t b, rgbd_keypoint* kps, rgbd_keypoint* kun, uint8_t* desc,
                             float* xyz, int32_t cap, int32_t* n)
{
    if (!c || b < 0 || b >= c->last_B) return RGBD_ERR_ARG;
    return read_frame(c, b, kps, kun, desc, xyz, cap, n);
}

rgbd_status rgbd_batch_outputs(rgbd_ctx* c, void** counts, void** kps, void** kun, void** desc, void** xyz)
{
    if (!c) return RGBD_ERR_ARG;
    if (counts) *counts = c->d_count;
    if (kps) *kps = c->d_kps;
    if (kun) *kun = c->d_kun;
    if (desc) *desc = c->d_desc;
    if (xyz) *xyz = c->d_xyz;
    return RGBD_OK;
}

rgbd_status rgbd_debug_level(rgbd_ctx* c, int32_t b, int32_t level, uint8_t* out)
{
    if (!c || !out || b < 0 || b >= c->maxB || level < 0 || level >= c->cfg.nlevels) return RGBD_ERR_ARG;
    const LevelCfg& L = c->cfg.lv[level];
    rgbd_status s = check_hip(c, hipMemcpy2DAsync(out, L.w, c->d_pyr + (size_t)b * c->cfg.frame_pyr_bytes + L.off, L.stride,
                                                  L.w, L.h, hipMemcpyDeviceToHost, c->stream), "read level");
    if (s) return s;
    return check_hip(c, hipStreamSynchronize(c->stream), "sync");
}

rgbd_status rgbd_debug_blurred(rgbd_ctx* c, int32_t b, int32_t level, uint8_t* out)
{
    if (!c || !out || b < 0 || b >= c->maxB || level < 0 || level >= c->cfg.nlevels) return RGBD_ERR_ARG;
    const LevelCfg& L = c->cfg.lv[level];
    rgbd_status s = check_hip(c, hipMemcpy2DAsync(out, L.w, c->d_blur + (size_t)b * c->cfg.frame_pyr_bytes + L.off, L.stride,
                                                  L.w, L.h, hipMemcpyDeviceToHost, c->stream), "read blurred level");
    if (s) return s;
    return check_hip(c, hipStreamSynchronize(c->stream), "sync");
}

rgbd_status rgbd_debug_candidates(rgbd_ctx* c, int32_t b, int32_t level, int32_t* xys, int32_t cap, int32_t* n)
{
    if (!c || b < 0 || b >= c->maxB || level < 0 || level >= c->cfg.nlevels) return RGBD_ERR_ARG;
    const ExtractCfg& C = c->cfg;
    const LevelCfg& L = C.lv[level];
    std::vector<int> cnt(L.cell_count);
    std::vector<uint32_t> slots((size_t)L.cell_count * C.cell_cap);
    rgbd_status s = check_hip(c, hipMemcpyAsync(cnt.data(), c->d_cellc + (size_t)b * C.n_cells + L.cell_begin,
                                                cnt.size() * 4, hipMemcpyDeviceToHost, c->stream), "read cell counts");
    if (s) return s;
    s = check_hip(c, hipMemcpyAsync(slots.data(), c->d_slots + ((size_t)b * C.n_cells + L.cell_begin) * C.cell_cap,
                                    slots.size() * 4, hipMemcpyDeviceToHost, c->stream), "read cell slots");
    if (s) return s;
    if ((s = check_hip(c, hipStreamSynchronize(c->stream), "sync"))) return s;
    int k = 0;
    for (int i = 0; i < L.cell_count; i++)
        for (int j = 0; j < cnt[i]; j++) {
            const uint32_t v = slots[(size_t)i * C.cell_cap + j];
            if (k < cap && xys) {
                xys[3 * k] = key_x(v);
                xys[3 * k + 1] = key_y(v);
                xys[3 * k + 2] = key_s(v);
            }
            k++;
        }
    if (n) *n = k;
    return k > cap ? fail(c, RGBD_ERR_CAPACITY, "capacity") : RGBD_OK;
}

rgbd_status rgbd_debug_selected(rgbd_ctx* c, int32_t b, int32_t level, int32_t* xys, int32_t cap, int32_t* n)
{
    if (!c || b < 0 || b >= c->maxB || level < 0 || level >= c->cfg.nlevels) return RGBD_ERR_ARG;
    const ExtractCfg& C = c->cfg;
    const LevelCfg& L = C.lv[level];
    int cnt = 0;
    rgbd_status s = check_hip(c, hipMemcpyAsync(&cnt, c->d_selc + (size_t)b * C.nlevels + level, 4, hipMemcpyDeviceToHost,
                                                c->stream), "read sel count");
    if (s) return s;
    if ((s = check_hip(c, hipStreamSynchronize(c->stream), "sync"))) return s;
    std::vector<uint32_t> v(std::max(cnt, 1));
    s = check_hip(c, hipMemcpy(v.data(), c->d_sel + (size_t)b * C.sel_per_frame + L.sel_off, (size_t)cnt * 4,
                               hipMemcpyDeviceToHost), "read sel");
    if (s) return s;
    for (int i = 0; i < cnt && i < cap; i++) {
        xys[3 * i] = key_x(v[i]);
        xys[3 * i + 1] = key_y(v[i]);
        xys[3 * i + 2] = key_s(v[i]);
    }
    if (n) *n = cnt;
    return cnt > cap ? fail(c, RGBD_ERR_CAPACITY, "capacity") : RGBD_OK;
}

// ------------------------------------------------------------------ matching
static rgbd_status ensure_mcap(rgbd_ctx* c, int need)
{
    if (need <= c->mcap) return RGBD_OK;
    int cap = std::max(need, c->cfg.kp_cap);
    if (c->d_mdesc) (void)hipFree(c->d_mdesc);
    if (c->d_mcount) (void)hipFree(c->d_mcount);
    if (c->d_mknn) (void)hipFree(c->d_mknn);
    c->d_mdesc = nullptr; c->d_mcount = nullptr; c->d_mknn = nullptr;
    rgbd_status s = dalloc(c, &c->d_mdesc, (size_t)2 * cap * 32, "match desc");
    if (!s) s = dalloc(c, &c->d_mcount, 4, "match counts");
    if (!s) s = dalloc(c, &c->d_mknn, (size_t)cap, "match knn");
    if (!s) {
        int pr[2] = {0, 1};
        s = check_hip(c, hipMemcpy(c->d_mcount + 2, pr, 8, hipMemcpyHostToDevice), "pairs");
    }
    if (!s) c->mcap = cap;
    return s;
}

rgbd_status rgbd_knn2(rgbd_ctx* c, const uint8_t* dq, int32_t nq, const uint8_t* dt, int32_t nt, int32_t* out)
{
    if (!c || nq < 0 || nt < 0 || (nq > 0 && (!dq || !out)) || (nt > 0 && !dt)) return RGBD_ERR_ARG;
    if (nq == 0) return RGBD_OK;
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    if ((s = ensure_mcap(c, std::max(nq, nt)))) return s;
    const int cap = c->mcap;
    int counts[2] = {nq, nt};
    if ((s = check_hip(c, hipMemcpyAsync(c->d_mcount, counts, 8, hipMemcpyHostToDevice, c->stream), "counts"))) return s;
    if ((s = check_hip(c, hipMemcpyAsync(c->d_mdesc, dq, (size_t)nq * 32, hipMemcpyHostToDevice, c->stream), "dq"))) return s;
    if (nt > 0 && (s = check_hip(c, hipMemcpyAsync(c->d_mdesc + (size_t)cap * 32, dt, (size_t)nt * 32, hipMemcpyHostToDevice, c->stream), "dt")))
        return s;
    const int tk = timer_begin(c, "k_knn2");
    RGBD_TRY(c, launch_knn2(c->d_mdesc, c->d_mcount, c->d_mcount + 2, c->d_mcount + 3, cap, nq, c->d_mknn, 1, c->stream), "knn2");
    timer_end(c, tk);
    if ((s = check_hip(c, hipMemcpyAsync(out, c->d_mknn, (size_t)nq * 16, hipMemcpyDeviceToHost, c->stream), "knn out"))) return s;
    return check_hip(c, hipStreamSynchronize(c->stream), "sync");
}

}  // extern "C"

namespace rgbd {
// Matcher::match filter stage (Features/Matcher.cpp:115-136) over knn-2 rows, query order.
int match_filter(const int32_t* knn, int nq, const uint8_t* outlier_q, const float* z_q, const float* z_t,
                 float nnratio, int discard, rgbd_dmatch* out, int cap)
{
    std::vector<uint8_t> used;
    int m = 0;
    for (int i = 0; i < nq; i++) {
        const int i2b = knn[4 * i + 3];
        if (i2b < 0) continue;   // fewer than 2 train rows: reference UB (matchesKnn[i][1]); skip
        const float d1 = (float)knn[4 * i], d2 = (float)knn[4 * i + 2];
        if (d1 < nnratio * d2) {
            const int i2 = knn[4 * i + 1];
            if ((int)used.size() <= i2) used.resize(i2 + 1, 0);
            if (used[i2]) continue;
            if (discard && outlier_q && outlier_q[i]) continue;
            if (!(z_q[i] > 0) || !(z_t[i2] > 0)) continue;
            used[i2] = 1;
            if (m < cap) {
                out[m].queryIdx = i;
                out[m].trainIdx = i2;
                out[m].imgIdx = 0;
                out[m].distance = d1;
            }
            m++;
        }
    }
    return m;
}
}  // namespace rgbd

extern "C" {

rgbd_status rgbd_match(rgbd_ctx* c, const uint8_t* dq, int32_t nq, const uint8_t* dt, int32_t nt,
                       const uint8_t* outlier_q, const float* z_q, const float* z_t, float nnratio,
                       int32_t discard, rgbd_dmatch* out, int32_t cap, int32_t* m)
{
    if (!c || !m) return RGBD_ERR_ARG;
    *m = 0;
    if (nq <= 0 || nt <= 0) return RGBD_OK;   // knnMatch on an empty set returns no rows
    if (!z_q || !z_t) return fail(c, RGBD_ERR_ARG, "z arrays required");
    std::vector<int32_t> knn((size_t)nq * 4);
    rgbd_status s = rgbd_knn2(c, dq, nq, dt, nt, knn.data());
    if (s) return s;
    const int cnt = match_filter(knn.data(), nq, outlier_q, z_q, z_t, nnratio, discard, out, cap);
    *m = cnt;
    return cnt > cap ? fail(c, RGBD_ERR_CAPACITY, "match capacity") : RGBD_OK;
}

rgbd_status rgbd_set_timing(rgbd_ctx* c, int32_t enable)
{
    if (!c) return RGBD_ERR_ARG;
    c->timing = enable != 0;
    return RGBD_OK;
}

rgbd_status rgbd_set_timing_filter(rgbd_ctx* c, const char* kernel)
{
    if (!c) return RGBD_ERR_ARG;
    c->timing_only = kernel ? kernel : "";
    return RGBD_OK;
}

rgbd_status rgbd_reset_timing(rgbd_ctx* c)
{
    if (!c) return RGBD_ERR_ARG;
    timer_flush(c);
    c->tentries.clear();
    return RGBD_OK;
}

int32_t rgbd_timing_count(const rgbd_ctx* c) { return c ? (int32_t)c->tentries.size() : 0; }

rgbd_status rgbd_timing_entry(rgbd_ctx* c, int32_t idx, const char** name, double* total_ms, int64_t* launches)
{
    if (!c) return RGBD_ERR_ARG;
    timer_flush(c);
    if (idx < 0 || idx >= (int)c->tentries.size()) return RGBD_ERR_ARG;
    if (name) *name = c->tentries[idx].name.c_str();
    if (total_ms) *total_ms = c->tentries[idx].ms;
    if (launches) *launches = c->tentries[idx].launches;
    return RGBD_OK;
}

rgbd_status rgbd_synchronize(rgbd_ctx* c)
{
    if (!c) return RGBD_ERR_ARG;
    rgbd_status s = check_hip(c, hipStreamSynchronize(c->stream), "sync");
    if (!s && c->match_stream) s = check_hip(c, hipStreamSynchronize(c->match_stream), "sync match stream");
    if (!s && c->solve_stream) s = check_hip(c, hipStreamSynchronize(c->solve_stream), "sync solve stream");
    return s;
}

}  // extern "C"

namespace rgbd {
rgbd_status extract_batch(rgbd_ctx* c, const void* d_bgr, const void* d_depth, int B, const ExtractHook* after_fast)
{
    if (!c || !d_bgr || B < 1) return RGBD_ERR_ARG;
    if (B > c->maxB) return fail(c, RGBD_ERR_CAPACITY, "batch larger than max_batch");
    rgbd_status s = check_hip(c, hipSetDevice(c->device), "hipSetDevice");
    if (s) return s;
    return run_extract(c, (const uint8_t*)d_bgr, (const uint16_t*)d_depth, B, false, after_fast);
}
}  // namespace rgbd

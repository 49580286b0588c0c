// orc_cloud.cpp -- ORACLE (test infrastructure only): the keyframe dense cloud of the reference,
// Tracking::createKeyFrame (System/Tracking.cpp:234-237):
//   createCloud(6)                 Core/Frame.cpp:475-505  (stride-6 samples, z <= 0 skipped, BGR)
//   passThroughFilter("z", .5, 4)  Core/Frame.cpp:537-549  (PCL PassThrough: keep ll <= z <= ul)
//   downsampleCloud(0.04f)         Core/Frame.cpp:516-524  (PCL 1.8 VoxelGrid, downsample_all_data)
//   statisticalFilterCloud(50, 1)  Core/Frame.cpp:526-535  (PCL 1.8 StatisticalOutlierRemoval)
// PCL is absent; its published algorithms are restated (DESIGN.md "Keyframe cloud definition").
// One deviation: VoxelGrid's std::sort of (voxel, point) pairs by voxel only is unstable, so the
// order in which a voxel's points are summed is not defined by PCL; here it is point order.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <vector>

#include "rgbd_oracle.h"

namespace {

void centroid_points(const orc_point* in, const std::vector<std::pair<int64_t, int>>& iv, size_t a, size_t b,
                     orc_point* o)
{
    float s[6] = {0, 0, 0, 0, 0, 0};
    for (size_t li = a; li < b; li++) {
        const orc_point& p = in[iv[li].second];
        s[0] += p.x; s[1] += p.y; s[2] += p.z;
        s[3] += (float)p.r; s[4] += (float)p.g; s[5] += (float)p.b;
    }
    const float n = (float)(b - a);
    for (float& v : s) v /= n;
    o->x = s[0]; o->y = s[1]; o->z = s[2];
    // pack r/g/b (int) into rgb: (r << 16) | (g << 8) | b, i.e. bytes b, g, r
    o->r = (uint8_t)(int)s[3]; o->g = (uint8_t)(int)s[4]; o->b = (uint8_t)(int)s[5];
    o->pad = 0;
}

}  // namespace

extern "C" {

int orc_cloud(const uint8_t* bgr, const uint16_t* depth, int W, int H, const orc_camera* cam, int res, float zmin,
              float zmax, orc_point* out, int cap)
{
    const float invfx = 1.0f / cam->fx, invfy = 1.0f / cam->fy;   // IntrinsicMatrix::mInvfx
    int n = 0;
    for (int m = 0; m < H; m += res) {
        for (int c = 0; c < W; c += res) {
            const float z = (float)depth[(size_t)m * W + c] * cam->depth_map_factor + 0.0f;   // convertTo (Frame.cpp:48)
            if (z <= 0) continue;
            if (z < zmin || z > zmax) continue;                     // PassThrough (z is finite)
            if (n >= cap) return -1;
            orc_point& p = out[n++];
            const uint8_t* px = bgr + ((size_t)m * W + c) * 3;
            p.b = px[0]; p.g = px[1]; p.r = px[2]; p.pad = 0;
            p.x = ((float)c - cam->cx) * z * invfx;                 // RGBDcamera::unproject (:147-161)
            p.y = ((float)m - cam->cy) * z * invfy;
            p.z = z;
        }
    }
    return n;
}

int orc_voxel(const orc_point* in, int n, float leaf, orc_point* out)
{
    if (n <= 0) return 0;
    float mn[3] = {in[0].x, in[0].y, in[0].z}, mx[3] = {in[0].x, in[0].y, in[0].z};
    for (int i = 1; i < n; i++) {
        const float v[3] = {in[i].x, in[i].y, in[i].z};
        for (int d = 0; d < 3; d++) { mn[d] = std::min(mn[d], v[d]); mx[d] = std::max(mx[d], v[d]); }
    }
    const float inv = 1.0f / leaf;                                   // inverse_leaf_size_ (Array4f)
    int64_t dd[3];
    for (int d = 0; d < 3; d++) dd[d] = (int64_t)((mx[d] - mn[d]) * inv) + 1;
    if (dd[0] * dd[1] * dd[2] > (int64_t)std::numeric_limits<int32_t>::max()) {   // leaf too small: input
        std::memcpy(out, in, sizeof(orc_point) * (size_t)n);
        return n;
    }
    int minb[3], maxb[3], divb[3];
    for (int d = 0; d < 3; d++) {
        minb[d] = (int)std::floor(mn[d] * inv);
        maxb[d] = (int)std::floor(mx[d] * inv);
        divb[d] = maxb[d] - minb[d] + 1;
    }
    const int64_t mul1 = divb[0], mul2 = (int64_t)divb[0] * divb[1];
    std::vector<std::pair<int64_t, int>> iv((size_t)n);
    for (int i = 0; i < n; i++) {
        const int i0 = (int)(std::floor(in[i].x * inv) - (float)minb[0]);
        const int i1 = (int)(std::floor(in[i].y * inv) - (float)minb[1]);
        const int i2 = (int)(std::floor(in[i].z * inv) - (float)minb[2]);
        iv[i] = {(int64_t)i0 + (int64_t)i1 * mul1 + (int64_t)i2 * mul2, i};
    }
    std::sort(iv.begin(), iv.end());                                 // (voxel, point): point order inside a voxel
    int nv = 0;
    size_t a = 0;
    while (a < iv.size()) {
        size_t b = a + 1;
        while (b < iv.size() && iv[b].first == iv[a].first) b++;
        centroid_points(in, iv, a, b, &out[nv++]);
        a = b;
    }
    return nv;
}

int orc_sor(const orc_point* in, int n, int k, double std_mul, orc_point* out, float* dist_out)
{
    if (n <= 0) return 0;
    std::vector<float> dist((size_t)n), d2((size_t)n);
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < n; j++) {   // FLANN L2_Simple<float>: ((dx^2 + dy^2) + dz^2) in float
            const float dx = in[i].x - in[j].x, dy = in[i].y - in[j].y, dz = in[i].z - in[j].z;
            float r = 0.0f;
            r += dx * dx;
            r += dy * dy;
            r += dz * dz;
            d2[j] = r;
        }
        const int kk = std::min(k + 1, n);
        std::partial_sort(d2.begin(), d2.begin() + kk, d2.end());
        double s = 0.0;
        for (int q = 1; q < kk; q++) s += std::sqrt((double)d2[q]);   // k = 0 is the query point
        dist[i] = (float)(s / k);
    }
    double sum = 0.0, sq = 0.0;
    for (int i = 0; i < n; i++) {
        sum += dist[i];
        sq += dist[i] * dist[i];                                     // float product
    }
    const double mean = sum / (double)n;
    const double var = (sq - sum * sum / (double)n) / ((double)n - 1);
    const double thr = mean + std_mul * std::sqrt(var);
    int m = 0;
    for (int i = 0; i < n; i++) {
        if (dist_out) dist_out[i] = dist[i];
        if (dist[i] > thr) continue;
        out[m++] = in[i];
    }
    return m;
}

int orc_keyframe_cloud(const uint8_t* bgr, const uint16_t* depth, int W, int H, const orc_camera* cam,
                       orc_point* out, int cap)
{
    std::vector<orc_point> a((size_t)cap), b((size_t)cap);
    const int n = orc_cloud(bgr, depth, W, H, cam, 6, 0.5f, 4.0f, a.data(), cap);
    if (n < 0) return -1;
    const int nv = orc_voxel(a.data(), n, 0.04f, b.data());
    return orc_sor(b.data(), nv, 50, 1.0, out, nullptr);
}

}  // extern "C"

// cloud.hip -- the keyframe dense cloud on gfx950 (Tracking::createKeyFrame, System/Tracking.cpp:234-237):
// createCloud(6) + passThroughFilter("z", 0.5, 4.0) + downsampleCloud(0.04) + statisticalFilterCloud(50, 1)
// (Core/Frame.cpp:475-549; PCL 1.8 PassThrough / VoxelGrid / StatisticalOutlierRemoval restated in
// oracle/orc_cloud.cpp, DESIGN.md "Keyframe cloud definition").  One launch chain for a batch of
// keyframes:
//   k_cloud_voxel  one 1024-thread workgroup per keyframe: stride samples in raster order -> kept points
//                  (block-ranked, z in [zmin, zmax]) -> voxel keys (voxel index << 14 | point index) ->
//                  bitonic sort in LDS -> one thread per voxel sums its run in point order -> centroids
//   k_sor_dist     one wave per voxel point: its squared distances to every point in LDS, the k+1-th
//                  smallest by a bitwise binary search on the float bits, the k+1 smallest sorted across
//                  the lanes, their square roots summed in ascending order (FLANN's result order)
//   k_sor_filter   one workgroup per keyframe: mean / variance in point order (one lane, as PCL), then
//                  the kept points compacted in order
#include <hip/hip_runtime.h>

#include "dispatch.h"

#include <algorithm>
#include <cstdint>

#include "cloud_dev.h"

namespace rgbd {

constexpr int kCloudThreads = 1024;
constexpr int kCloudWaves = kCloudThreads / 64;

__device__ __forceinline__ int block_excl_scan_flag(bool f, int* wsum, int* total)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long bal = __ballot(f);
    if (lane == 0) wsum[w] = __popcll(bal);
    __syncthreads();
    int pre = 0, tot = 0;
    for (int i = 0; i < kCloudWaves; i++) {
        pre += i < w ? wsum[i] : 0;
        tot += wsum[i];
    }
    __syncthreads();
    *total = tot;
    return pre + __popcll(bal & ((1ull << lane) - 1ull));
}

__global__ __launch_bounds__(kCloudThreads) void k_cloud_voxel(const uint8_t* __restrict__ bgr,
                                                               const uint16_t* __restrict__ depth,
                                                               const float* __restrict__ depthf,
                                                               const int* __restrict__ frames, CloudCfg cfg,
                                                               CloudPoint* __restrict__ pts, CloudPoint* __restrict__ vox,
                                                               int* __restrict__ nvox)
{
    extern __shared__ __attribute__((aligned(16))) unsigned long long keys[];   // cfg.sort_cap
    __shared__ int wsum[kCloudWaves];
    __shared__ float red[kCloudWaves][6];
    const int kf = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int f = frames[kf];
    const uint8_t* img = bgr + (size_t)f * cfg.W * cfg.H * 3;
    const size_t fo = (size_t)f * cfg.W * cfg.H;
    CloudPoint* P = pts + (size_t)kf * cfg.cap;
    CloudPoint* V = vox + (size_t)kf * cfg.cap;
    // 1. createCloud + PassThrough, raster order
    float mn[3] = {3.4e38f, 3.4e38f, 3.4e38f}, mx[3] = {-3.4e38f, -3.4e38f, -3.4e38f};
    int n = 0;
    const int S = cfg.rows * cfg.cols;
    for (int s0 = 0; s0 < S; s0 += kCloudThreads) {
        const int s = s0 + tid;
        bool keep = false;
        CloudPoint p{};
        if (s < S) {
            const int r = s / cfg.cols, c = s - r * cfg.cols;
            const int m = r * cfg.res, col = c * cfg.res;
            const size_t o = fo + (size_t)m * cfg.W + col;
            // convertTo(CV_32F, 1/factor) as float(d) * scale (Core/Frame.cpp:48), or the converted image itself
            const float z = depthf ? depthf[o] : (float)depth[o] * cfg.depth_factor + 0.0f;
            keep = z > 0 && z >= cfg.zmin && z <= cfg.zmax;
            if (keep) {
                const uint8_t* px = img + ((size_t)m * cfg.W + col) * 3;
                p.x = ((float)col - cfg.cx) * z * cfg.invfx;
                p.y = ((float)m - cfg.cy) * z * cfg.invfy;
                p.z = z;
                p.b = px[0];
                p.g = px[1];
                p.r = px[2];
                p.pad = 0;
                mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
                mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
            }
        }
        int tot;
        const int off = block_excl_scan_flag(keep, wsum, &tot);
        if (keep) P[n + off] = p;
        n += tot;
    }
    // bounds (getMinMax3D)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
#pragma unroll
        for (int d = 0; d < 3; d++) {
            mn[d] = fminf(mn[d], __shfl_xor(mn[d], o, 64));
            mx[d] = fmaxf(mx[d], __shfl_xor(mx[d], o, 64));
        }
    if (lane == 0)
        for (int d = 0; d < 3; d++) { red[w][d] = mn[d]; red[w][3 + d] = mx[d]; }
    __threadfence_block();
    __syncthreads();
    for (int i = 0; i < kCloudWaves; i++)
        for (int d = 0; d < 3; d++) { mn[d] = fminf(mn[d], red[i][d]); mx[d] = fmaxf(mx[d], red[i][3 + d]); }
    if (n == 0) {
        if (tid == 0) nvox[kf] = 0;
        return;
    }
    // 2. VoxelGrid keys (PCL 1.8 applyFilter): floor indices relative to the bounds
    const float inv = cfg.inv_leaf;
    long long dd = 1;
    int minb[3], mul[3];
    int divb[3];
    for (int d = 0; d < 3; d++) {
        dd *= (long long)((mx[d] - mn[d]) * inv) + 1;
        minb[d] = (int)floorf(mn[d] * inv);
        divb[d] = (int)floorf(mx[d] * inv) - minb[d] + 1;
    }
    if (dd > 2147483647LL) {   // leaf too small for the int voxel index: PCL returns the input
        for (int i = tid; i < n; i += kCloudThreads) V[i] = P[i];
        if (tid == 0) nvox[kf] = n;
        return;
    }
    mul[0] = 1;
    mul[1] = divb[0];
    mul[2] = divb[0] * divb[1];
    int sc = 1;
    while (sc < n) sc <<= 1;
    for (int i = tid; i < sc; i += kCloudThreads) {
        unsigned long long k = ~0ull;
        if (i < n) {
            const CloudPoint p = P[i];
            const int i0 = (int)(floorf(p.x * inv) - (float)minb[0]);
            const int i1 = (int)(floorf(p.y * inv) - (float)minb[1]);
            const int i2 = (int)(floorf(p.z * inv) - (float)minb[2]);
            const unsigned long long idx = (unsigned long long)(i0 * mul[0] + i1 * mul[1] + i2 * mul[2]);
            k = (idx << 14) | (unsigned long long)i;
        }
        keys[i] = k;
    }
    __syncthreads();
    // bitonic sort of sc keys (sc a power of two, <= sort_cap)
    for (int size = 2; size <= sc; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int t = tid; t < (sc >> 1); t += kCloudThreads) {
                const int lo = 2 * t - (t & (stride - 1));
                const int hi = lo + stride;
                const bool up = (lo & size) == 0;
                const unsigned long long a = keys[lo], b = keys[hi];
                if ((a > b) == up) {
                    keys[lo] = b;
                    keys[hi] = a;
                }
            }
            __syncthreads();
        }
    }
    // 3. one thread per voxel (the first key of a run): float sums in point order, centroid, colours
    int nv = 0;
    for (int j0 = 0; j0 < n; j0 += kCloudThreads) {
        const int j = j0 + tid;
        const bool first = j < n && (j == 0 || (keys[j] >> 14) != (keys[j - 1] >> 14));
        int tot;
        const int off = block_excl_scan_flag(first, wsum, &tot);
        if (first) {
            const unsigned long long v = keys[j] >> 14;
            float sx = 0.f, sy = 0.f, sz = 0.f, sr = 0.f, sg = 0.f, sb = 0.f;
            int e = j;
            while (e < n && (keys[e] >> 14) == v) {
                const CloudPoint p = P[(int)(keys[e] & 16383ull)];
                sx += p.x; sy += p.y; sz += p.z;
                sr += (float)p.r; sg += (float)p.g; sb += (float)p.b;
                e++;
            }
            const float c = (float)(e - j);
            CloudPoint o;
            o.x = sx / c; o.y = sy / c; o.z = sz / c;
            o.r = (uint8_t)(int)(sr / c); o.g = (uint8_t)(int)(sg / c); o.b = (uint8_t)(int)(sb / c);
            o.pad = 0;
            V[nv + off] = o;
        }
        nv += tot;
    }
    if (tid == 0) nvox[kf] = nv;
}

// one wave per voxel point; the keyframe's voxel points' squared distances to it in this wave's LDS row
constexpr int kSorWaves = 4;   // at most; fewer when a distance row is long
__global__ __launch_bounds__(64 * kSorWaves) void k_sor_dist(const CloudPoint* __restrict__ vox,
                                                             const int* __restrict__ nvox, CloudCfg cfg,
                                                             float* __restrict__ dist)
{
    extern __shared__ __attribute__((aligned(16))) float d2all[];   // kSorWaves x cfg.cap
    __shared__ float kth[kSorWaves][64];
    const int kf = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int n = nvox[kf];
    const int i = blockIdx.x * (int)(blockDim.x >> 6) + w;
    if (i >= n) return;
    const CloudPoint* V = vox + (size_t)kf * cfg.cap;
    float* d2 = d2all + (size_t)w * cfg.cap;
    const CloudPoint q = V[i];
    for (int j = lane; j < n; j += 64) {   // FLANN L2_Simple<float>: ((dx^2 + dy^2) + dz^2)
        const CloudPoint p = V[j];
        const float dx = q.x - p.x, dy = q.y - p.y, dz = q.z - p.z;
        float r = dx * dx;
        r += dy * dy;
        r += dz * dz;
        d2[j] = r;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    const int kk = min(cfg.sor_k + 1, n);   // the query itself is one of the kk nearest (distance 0)
    // T = the kk-th smallest value: the largest T with count(d2 < T) < kk (bitwise on the float bits)
    unsigned int T = 0;
    for (int b = 30; b >= 0; b--) {
        const unsigned int cand = T | (1u << b);
        int cnt = 0;
        for (int j = lane; j < n; j += 64) cnt += __float_as_uint(d2[j]) < cand ? 1 : 0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
        if (cnt < kk) T = cand;
    }
    // the kk smallest: every value below T, then copies of T; sorted across the lanes (kk <= 64)
    int below = 0;
    for (int j0 = 0; j0 < n; j0 += 64) {
        const int j = j0 + lane;
        const bool f = j < n && __float_as_uint(d2[j]) < T;
        const unsigned long long bal = __ballot(f);
        if (f) kth[w][below + __popcll(bal & ((1ull << lane) - 1ull))] = d2[j];
        below += __popcll(bal);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    float v = lane < below ? kth[w][lane] : (lane < kk ? __uint_as_float(T) : 3.4e38f);
    // bitonic sort of one value per lane (ascending by lane)
    for (int size = 2; size <= 64; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            const float o = __shfl_xor(v, stride, 64);
            const bool up = (lane & size) == 0;
            const bool lower = (lane & stride) == 0;
            v = (lower == up) ? fminf(v, o) : fmaxf(v, o);
        }
    // sum sqrt of ranks 1 .. kk-1 in ascending order (rank 0 is the query), on lane 0
    double s = 0.0;
    for (int k = 1; k < kk; k++) s += sqrt((double)__shfl(v, k, 64));
    if (lane == 0) dist[(size_t)kf * cfg.cap + i] = (float)(s / cfg.sor_k);
}

__global__ __launch_bounds__(kCloudThreads) void k_sor_filter(const CloudPoint* __restrict__ vox,
                                                              const int* __restrict__ nvox, const float* __restrict__ dist,
                                                              CloudCfg cfg, CloudPoint* __restrict__ out,
                                                              int* __restrict__ nout)
{
    __shared__ int wsum[kCloudWaves];
    __shared__ double s_thr;
    const int kf = blockIdx.x, tid = threadIdx.x;
    const int n = nvox[kf];
    const float* D = dist + (size_t)kf * cfg.cap;
    if (tid == 0) {   // PCL: sums over the points in order; squares as float products
        double sum = 0.0, sq = 0.0;
        for (int i = 0; i < n; i++) {
            const float d = D[i];
            sum += d;
            sq += d * d;
        }
        const double mean = sum / (double)n;
        const double var = (sq - sum * sum / (double)n) / ((double)n - 1);
        s_thr = mean + cfg.sor_std * sqrt(var);
    }
    __syncthreads();
    const double thr = s_thr;
    const CloudPoint* V = vox + (size_t)kf * cfg.cap;
    CloudPoint* O = out + (size_t)kf * cfg.cap;
    int m = 0;
    for (int i0 = 0; i0 < n; i0 += kCloudThreads) {
        const int i = i0 + tid;
        const bool keep = i < n && !((double)D[i] > thr);
        int tot;
        const int off = block_excl_scan_flag(keep, wsum, &tot);
        if (keep) O[m + off] = V[i];
        m += tot;
    }
    if (tid == 0) nout[kf] = m;
}

hipError_t launch_cloud(const uint8_t* bgr, const uint16_t* depth, const float* depthf, const int* frames, int nkf,
                  const CloudCfg& cfg, CloudPoint* pts, CloudPoint* vox, int* nvox, float* dist, CloudPoint* out, int* nout, hipStream_t st)
{
    hipError_t e = dispatch(k_cloud_voxel, dim3(nkf), dim3(kCloudThreads), (size_t)cfg.sort_cap * 8, st, bgr, depth,
                            depthf, frames, cfg, pts, vox, nvox);
    if (e != hipSuccess) return e;
    // waves per workgroup: each holds one distance row of cap floats in LDS (<= 156 KB in all)
    const int nw = std::max(1, std::min(kSorWaves, (156 * 1024) / (cfg.cap * 4)));
    e = dispatch(k_sor_dist, dim3((cfg.cap + nw - 1) / nw, nkf), dim3(64 * nw), (size_t)nw * cfg.cap * 4, st, vox, nvox,
                 cfg, dist);
    if (e != hipSuccess) return e;
    return dispatch(k_sor_filter, dim3(nkf), dim3(kCloudThreads), 0, st, vox, nvox, dist, cfg, out, nout);
}

}  // namespace rgbd

// ransac.hip -- RansacSE3 hypothesis chains on gfx950.
//
// Reference: RansacSE3::compute, Solver/SolverSE3.cpp:23-133.  Each RANSAC iteration n draws a
// sample (sampleMatches :135-159) and refines it up to 19 times (:60-86):
//     T   = getTransformFromMatches(inliers)        (:161-179, PCL TransformationFromCorrespondences)
//     err = computeInliersAndError(all, T, inliers) (:181-214, errorFunction2 :216-280)
// The chain of iteration n depends only on its sample, not on the global best, so all chains run
// in parallel: one workgroup per hypothesis.  The host replays the sequential accept / n += 10 /
// break logic (:88-102) over the chain results and advances the RNG by exactly the samples used.
//
// Numerics follow the oracle's restatement exactly (no FMA): online f32 weighted-correspondence
// update in inlier order, f64 Jacobi SVD (Eigen 3.3 JacobiSVD<Matrix3d> sweeps), f64 Mahalanobis
// with a 3x3 LLT (Eigen unrolled triangular solves), sequential f64 error sum in match order.
#include <hip/hip_runtime.h>

#include "dispatch.h"

#include <cstdio>
#include <cstring>

#include "lanes_dev.h"
#include "lane_replay_dev.h"
#include "launch.h"
#include "ransac_dev.h"
#include "svd3_dev.h"

#ifdef RGBD_PNP_PROFILE
// lane 0's first hypothesis block of every k_ransac_hyp_lanes launch: wall-clock (10 ns) per refinement stage,
// summed over the call (0: refinements, 1 compaction, 2 weights + prefix, 3 alpha, 4 recurrences,
// 5 transform, 6 inliers + the pipelined error sum; 7, 8 unused since the sum is pipelined)
__device__ long long g_hyp_prof[16];
__device__ long long g_svd_prof[8];   // the same block's transform: svd3 stages (svd3_dev.h) + [5] R, t from U, V
#define HYP_PROF(k) do { if (hprof) { const long long t_ = wall_clock64(); g_hyp_prof[(k)] += t_ - t_prev; t_prev = t_; } } while (0)
#else
#define HYP_PROF(k) do { } while (0)
#endif

namespace rgbd {

namespace {

using namespace svd3d;

__device__ double det3(const double m[3][3])
{
    const double h0 = m[0][0] * (m[1][1] * m[2][2] - m[1][2] * m[2][1]);
    const double h1 = m[0][1] * (m[1][0] * m[2][2] - m[1][2] * m[2][0]);
    const double h2 = m[0][2] * (m[1][0] * m[2][1] - m[1][1] * m[2][0]);
    return h0 - h1 + h2;
}

// PCL TransformationFromCorrespondences::getTransformation (f64 SVD of the f32 covariance)
__device__ void tfc_transform(const float cov[3][3], const float m1[3], const float m2[3], float T[16],
                              long long* prof = nullptr)
{
    double C[3][3], U[3][3], V[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C[i][j] = (double)cov[i][j];
    svd3(C, U, V, nullptr, prof);
    const long long t_svd = prof ? (long long)wall_clock64() : 0;
    double s22 = 1.0;
    if (det3(U) * det3(V) < 0.0f) s22 = -1.0;
    const double s[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, s22}};
    double us[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) us[i][j] = (U[i][0] * s[0][j] + U[i][1] * s[1][j]) + U[i][2] * s[2][j];
    for (int i = 0; i < 3; i++) {
        float rf[3];
        for (int j = 0; j < 3; j++) rf[j] = (float)((us[i][0] * V[j][0] + us[i][1] * V[j][1]) + us[i][2] * V[j][2]);
        const float rm = (rf[0] * m1[0] + rf[1] * m1[1]) + rf[2] * m1[2];
        T[4 * i + 0] = rf[0];
        T[4 * i + 1] = rf[1];
        T[4 * i + 2] = rf[2];
        T[4 * i + 3] = m2[i] - rm;
    }
    T[12] = 0.0f; T[13] = 0.0f; T[14] = 0.0f; T[15] = 1.0f;
    if (prof) prof[5] += (long long)wall_clock64() - t_svd;
}

// errorFunction2 (:216-280) with the sticky depth covariance C
__device__ double mahalanobis2(const float* o, const float* t, const double T[12], double C, double rcx, double rcy)
{
    if (isnan(o[2]) || isnan(t[2])) return kDblMax;
    const double x0 = o[0], x1 = o[1], x2 = o[2];
    const double mu2[3] = {t[0], t[1], t[2]};
    double m[3], d[3];
    for (int i = 0; i < 3; i++) m[i] = ((T[4 * i] * x0 + T[4 * i + 1] * x1) + T[4 * i + 2] * x2) + T[4 * i + 3] * 1.0;
    for (int i = 0; i < 3; i++) d[i] = m[i] - mu2[i];
    const double dsq = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
    const double smax = fmax(rcx, C);
    if (dsq > 2.0 * (smax + smax)) return kDblMax;
    const double c1[3] = {rcx * x2, rcy * x2, C};
    const double c2[3] = {rcx * mu2[2], rcy * mu2[2], C};
    double Mx[3][3], S[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            const double a0 = T[0 * 4 + i] * (j == 0 ? c1[0] : 0.0);
            const double a1 = T[1 * 4 + i] * (j == 1 ? c1[1] : 0.0);
            const double a2 = T[2 * 4 + i] * (j == 2 ? c1[2] : 0.0);
            Mx[i][j] = (a0 + a1) + a2;
        }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            const double v = (Mx[i][0] * T[0 * 4 + j] + Mx[i][1] * T[1 * 4 + j]) + Mx[i][2] * T[2 * 4 + j];
            S[i][j] = v + (i == j ? c2[i] : 0.0);
        }
    if (isnan(d[2])) return kDblMax;
    double L[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) L[i][j] = S[i][j];
    for (int kk = 0; kk < 3; ++kk) {
        double x = L[kk][kk];
        if (kk == 1) x -= L[1][0] * L[1][0];
        if (kk == 2) x -= L[2][0] * L[2][0] + L[2][1] * L[2][1];
        if (x <= 0.0) break;
        L[kk][kk] = x = sqrt(x);
        if (kk == 1) L[2][1] -= L[2][0] * L[1][0];
        for (int r = kk + 1; r < 3; r++) L[r][kk] /= x;
    }
    double y0 = d[0] / L[0][0];
    double y1 = (d[1] - L[1][0] * y0) / L[1][1];
    double y2 = (d[2] - (L[2][0] * y0 + L[2][1] * y1)) / L[2][2];
    y2 = y2 / L[2][2];
    y1 = (y1 - L[2][1] * y2) / L[1][1];
    y0 = (y0 - (L[1][0] * y1 + L[2][0] * y2)) / L[0][0];
    const double sq = (d[0] * y0 + d[1] * y1) + d[2] * y2;
    if (!(sq >= 0.0)) return kDblMax;
    return sq;
}

}  // namespace

constexpr int kRansacThreads = 256;

// exclusive scan of a[0..n) in place (LDS), 256 threads; returns the total
__device__ int rs_scan_excl(int* a, int n, int* wsum)
{
    const int tid = threadIdx.x;
    const int per = (n + kRansacThreads - 1) / kRansacThreads;
    const int beg = min(tid * per, n), end = min(beg + per, n);
    int s = 0;
    for (int i = beg; i < end; i++) s += a[i];
    const int lane = tid & 63, w = tid >> 6;
    int x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    int wpre = 0, total = 0;
#pragma unroll
    for (int i = 0; i < kRansacThreads / 64; i++) {
        if (i < w) wpre += wsum[i];
        total += wsum[i];
    }
    int run = wpre + x - s;
    for (int i = beg; i < end; i++) {
        const int v = a[i];
        a[i] = run;
        run += v;
    }
    __syncthreads();
    return total;
}

// grid.x = hypotheses + 1; the last block evaluates the identity transform once (:105-117).
//
// The PCL online update  acc += w; a = w/acc; d1 = p - m1; d2 = q - m2;
//                        cov = (1-a)*(cov + d1^T*(a*d2)); m1 += a*d1; m2 += a*d2
// is evaluated as exact pieces: acc prefix (1 lane), a_i = w_i/acc_i (parallel), then nine lanes, each
// running one covariance recurrence c <- (1-a_i)*(c + d1_b*(a_i*d2_a)) beside the two mean recurrences
// m <- m + a_i*(x_i - m) it reads.  Every float operation is the reference's, in the reference's order,
// so the result is bit-identical to the sequential update.
// One hypothesis chain per workgroup: `sample` = its n_samp sampled ids (ignored for the identity slot),
// the result in *out and its inlier bitmask in mask_out[0 .. MW).
__device__ void ransac_hyp_block(const float* __restrict__ pts_g, const int* __restrict__ sample, int n_samp,
                                 const RansacDev& prm, bool identity, HypOut* __restrict__ out,
                                 uint32_t* __restrict__ mask_out, unsigned char* smem)
{
    const int M = prm.M;
    const int MW = (M + 31) >> 5;
    float* P = reinterpret_cast<float*>(smem);                                      // 6M
    unsigned char* un = smem + (size_t)24 * M;                                      // union, 32M bytes
    float* Wt = reinterpret_cast<float*>(un);                                       //   fit: w   (M)
    float* Al = Wt + M;                                                             //   fit: acc -> alpha (M)
    float* D = Al + M;                                                              //   fit: compaction scratch (6M)
    double* md = reinterpret_cast<double*>(un);                                     //   scan: md (M)
    int* list = reinterpret_cast<int*>(un + (size_t)32 * M);                        // M
    uint32_t* cur = reinterpret_cast<uint32_t*>(list + M);                          // MW
    uint32_t* nw = cur + MW;                                                        // MW
    uint32_t* refm = nw + MW;                                                       // MW
    int* wbase = reinterpret_cast<int*>(refm + MW);                                 // MW
    __shared__ float Tsh[16];
    __shared__ float refT[16];
    __shared__ float s_cov[9];
    __shared__ float s_mean[6];
    __shared__ int s_nfit;
    __shared__ int s_prog1, s_prog2;   // pipelined fit: blocks of 64 with the prefix / with alpha done
    __shared__ double s_err;
    __shared__ int s_ready[kRansacMaxM / 64], s_ccnt[kRansacMaxM / 64], s_cnt;   // the pipelined error sum's chunks
    __shared__ int wsum[kRansacThreads / 64];
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    for (int i = tid; i < 6 * M; i += kRansacThreads) P[i] = pts_g[i];
    for (int w = tid; w < MW; w += kRansacThreads) { cur[w] = 0u; refm[w] = 0u; }
    for (int k = tid; k < kRansacMaxM / 64; k += kRansacThreads) s_ready[k] = 0;
    __syncthreads();
    if (tid == 0 && !identity) {
        for (int i = 0; i < n_samp; i++) {
            const int id = sample[i];
            cur[id >> 5] |= 1u << (id & 31);
        }
    }
    double refinedError = 1e6;
    int nRef = 0;
    const float maxd = prm.maxMahal * prm.maxMahal;
#ifdef RGBD_PNP_PROFILE
    const bool hprof = blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0;   // (lane 0's first hypothesis)
    long long t_prev = wall_clock64();
#endif
    for (int refinement = 1; refinement < 20; refinement++) {
        __syncthreads();
#ifdef RGBD_PNP_PROFILE
        if (hprof) { g_hyp_prof[0]++; t_prev = wall_clock64(); }
#endif
        if (identity) {
            if (tid < 16) Tsh[tid] = (tid % 5 == 0) ? 1.0f : 0.0f;
        } else {
            // ---- compact the current set (index order), keeping only points with a usable weight
            for (int w = tid; w < MW; w += kRansacThreads) wbase[w] = __popc(cur[w]);
            __syncthreads();
            const int nset = rs_scan_excl(wbase, MW, wsum);
            for (int w = tid; w < MW; w += kRansacThreads) {
                uint32_t bits = cur[w];
                int pos = wbase[w];
                while (bits) {
                    const int b = __ffs(bits) - 1;
                    list[pos++] = (w << 5) + b;
                    bits &= bits - 1u;
                }
            }
            __syncthreads();
            HYP_PROF(1);
            // weights (:171-175) -- PCL add() returns early on weight 0
            for (int i = tid; i < nset; i += kRansacThreads) {
                const float* p = P + 6 * list[i];
                const float* q = p + 3;
                float w = 0.0f;
                if (!(isnan(p[2]) || isnan(q[2]))) w = 1.0f / (p[2] * q[2]);
                Wt[i] = w;
            }
            __syncthreads();
            // keep the order; drop zero weights (rare: NaN/inf depths): wave 0 compacts with a ballot prefix
            if (wave == 0) {
                int k = 0;
                for (int b0 = 0; b0 < nset; b0 += 64) {
                    const int i = b0 + lane;
                    const float w = (i < nset) ? Wt[i] : 0.0f;
                    const int li = (i < nset) ? list[i] : 0;
                    const bool keep = (i < nset) && (w != 0.0f);
                    const unsigned long long bal = __ballot(keep);
                    const int pos = k + __popcll(bal & ((1ull << lane) - 1ull));
                    __builtin_amdgcn_wave_barrier();
                    if (keep) { Al[pos] = w; reinterpret_cast<int*>(D)[pos] = li; }
                    k += __popcll(bal);
                }
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                for (int i = lane; i < k; i += 64) { Wt[i] = Al[i]; list[i] = reinterpret_cast<int*>(D)[i]; }
                if (lane == 0) {
                    s_nfit = k;
                    s_prog1 = 0;
                    s_prog2 = 0;
                }
            }
            __syncthreads();
            HYP_PROF(2);
            const int nf = s_nfit;
            // the fit points' six coordinates gathered in fit order (D[k M + i] = P[6 list[i] + k]: the compaction
            // scratch is free again), so the serial recurrences below read them directly
            for (int i = tid; i < nf; i += kRansacThreads) {
                const float* pp = P + 6 * list[i];
#pragma unroll
                for (int k = 0; k < 6; k++) D[k * M + i] = pp[k];
            }
            __syncthreads();
            HYP_PROF(3);
            // three serial stages pipelined over blocks of 64 fit points, one wave each: wave 1 (lane 0) forms the
            // accumulated-weight prefix (float adds in order), wave 2 turns a finished block into alpha_i = w_i /
            // acc_i, wave 0 runs the recurrences below on the blocks whose alphas are there -- the same operations
            // in the same order, the prefix and the divisions now beside the recurrence chain instead of before it
            const int nblk = (nf + 63) >> 6;
            if (wave == 1) {
                if (lane == 0) {
                    float acc = 0.0f;
                    for (int blk = 0; blk < nblk; blk++) {
                        const int i1 = min(blk * 64 + 64, nf);
                        int i = blk * 64;
                        for (; i + 8 <= i1; i += 8) {
                            float w8[8];
#pragma unroll
                            for (int u = 0; u < 8; u++) w8[u] = Wt[i + u];
#pragma unroll
                            for (int u = 0; u < 8; u++) { acc += w8[u]; w8[u] = acc; }
#pragma unroll
                            for (int u = 0; u < 8; u++) Al[i + u] = w8[u];
                        }
                        for (; i < i1; i++) { acc += Wt[i]; Al[i] = acc; }
                        __hip_atomic_store(&s_prog1, blk + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
            } else if (wave == 2) {
                for (int blk = 0; blk < nblk; blk++) {
                    while (__hip_atomic_load(&s_prog1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= blk)
                        __builtin_amdgcn_s_sleep(1);
                    const int i = blk * 64 + lane;
                    if (i < nf) Al[i] = Wt[i] / Al[i];
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == 0) __hip_atomic_store(&s_prog2, blk + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            // the six mean recurrences m <- m + a*(x - m) and the nine covariance recurrences
            // c <- (1-a)*(c + d1[b]*(a*d2[a])) in one pass: lane (a, b) of wave 0 runs the two means its
            // covariance entry reads (source component b, target component a) beside it, so the d's never go
            // through LDS and the covariance chain overlaps the mean chains (same operations, same order)
            if (wave == 0 && lane < 9) {
                // the two means as one packed f32 pair (m1, m2): d = x - m, t = a d, m += t are each one
                // v_pk_add / v_pk_mul for both (the same IEEE operations per component), so a point costs
                // 7 instructions instead of 10 on this serial chain
                typedef float f32x2 __attribute__((ext_vector_type(2)));
                const int ra = lane / 3, cb = lane - 3 * (lane / 3);
                f32x2 m = {0.0f, 0.0f};
                float c = 0.0f;
                auto step = [&](float x1, float x2, float a) __attribute__((always_inline)) {
                    const f32x2 X = {x1, x2}, A2 = {a, a};
                    const f32x2 d = X - m;    // (d1, d2)
                    const f32x2 t = A2 * d;   // (a d1, a d2 = ad2)
                    m = m + t;
                    c = (1.0f - a) * (c + d.x * t.y);
                };
                const float* const X1 = D + cb * M;
                const float* const X2 = D + (3 + ra) * M;
                for (int blk = 0; blk < nblk; blk++) {
                    while (__hip_atomic_load(&s_prog2, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= blk)
                        __builtin_amdgcn_s_sleep(1);
                    const int i1 = min(blk * 64 + 64, nf);
                    int i = blk * 64;
                    for (; i + 8 <= i1; i += 8) {
                        float x1[8], x2[8], a8[8];
#pragma unroll
                        for (int u = 0; u < 8; u++) {
                            x1[u] = X1[i + u];
                            x2[u] = X2[i + u];
                            a8[u] = Al[i + u];
                        }
#pragma unroll
                        for (int u = 0; u < 8; u++) step(x1[u], x2[u], a8[u]);
                    }
                    for (; i < i1; i++) step(X1[i], X2[i], Al[i]);
                }
                s_cov[lane] = c;
                if (ra == 0) s_mean[cb] = m.x;
                if (cb == 0) s_mean[3 + ra] = m.y;
            }
            __syncthreads();
            HYP_PROF(4);
            if (tid == 0) {
                float cov[3][3], m1[3], m2[3];
                for (int i = 0; i < 9; i++) cov[i / 3][i % 3] = s_cov[i];
                for (int i = 0; i < 3; i++) { m1[i] = s_mean[i]; m2[i] = s_mean[3 + i]; }
                float T[16];
#ifdef RGBD_PNP_PROFILE
                tfc_transform(cov, m1, m2, T, hprof ? g_svd_prof : nullptr);
#else
                tfc_transform(cov, m1, m2, T);
#endif
                for (int i = 0; i < 16; i++) Tsh[i] = T[i];
            }
        }
        __syncthreads();
        HYP_PROF(5);
        double T[12];
        for (int i = 0; i < 12; i++) T[i] = (double)Tsh[i];
        // ---- computeInliersAndError over all used matches: waves 1..3 evaluate the matches in chunks of 64 (chunk
        // k by wave 1 + k % 3), compact each chunk's inlier distances in match order at md[64 k ..] and publish
        // its count; wave 0's lane 0 adds them in match order as the chunks arrive -- the same sequence of f64 adds
        // as over the packed array, now beside the Mahalanobis evaluations instead of after them and a scan
        const int nch = (M + 63) >> 6;
        if (wave > 0) {
            for (int k = wave - 1; k < nch; k += kRansacThreads / 64 - 1) {
                const int c0 = 64 * k, j = c0 + lane;
                bool inl = false;
                double v = 0.0;
                if (j < M) {
                    const float* o = P + 6 * j;
                    const float* t = o + 3;
                    if (!(o[2] == 0.0f || t[0] == 0.0f)) {
                        v = mahalanobis2(o, t, T, prm.C, prm.rcx, prm.rcy);
                        inl = !(v > (double)maxd) && v >= 0.0;
                    }
                }
                const unsigned long long bal = __ballot(inl);
                if (inl) md[c0 + __popcll(bal & ((1ull << lane) - 1ull))] = v;
                if (lane == 0) {
                    nw[c0 >> 5] = (uint32_t)bal;
                    if ((c0 >> 5) + 1 < MW) nw[(c0 >> 5) + 1] = (uint32_t)(bal >> 32);
                    s_ccnt[k] = __popcll(bal);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) __hip_atomic_store(&s_ready[k], refinement, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        } else if (lane == 0) {
            double sum = 0.0;
            int cnt = 0;
            for (int k = 0; k < nch; k++) {
                while (__hip_atomic_load(&s_ready[k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != refinement)
                    __builtin_amdgcn_s_sleep(1);
                const int n = s_ccnt[k];
                const double* q = md + 64 * k;
                int i = 0;
                for (; i + 8 <= n; i += 8) {
                    double v8[8];
#pragma unroll
                    for (int u = 0; u < 8; u++) v8[u] = q[i + u];
#pragma unroll
                    for (int u = 0; u < 8; u++) sum += v8[u];
                }
                for (; i < n; i++) sum += q[i];
                cnt += n;
            }
            double err;
            if (cnt < 3)
                err = 1e9;
            else {
                err = sum / cnt;
                err = sqrt(err);
            }
            s_err = err;
            s_cnt = cnt;
        }
        __syncthreads();
        HYP_PROF(6);
        const int count = s_cnt;
        const double err = s_err;
        if (identity) {
            for (int w = tid; w < MW; w += kRansacThreads) mask_out[w] = nw[w];
            if (tid == 0) {
                for (int i = 0; i < 16; i++) out->T[i] = Tsh[i];
                out->err = err;
                out->n = count;
            }
            return;
        }
        if ((uint32_t)count < prm.minTh || err > (double)prm.maxMahal) break;
        if (count >= nRef && err <= refinedError) {
            const int prev = nRef;
            if (tid < 16) refT[tid] = Tsh[tid];
            for (int w = tid; w < MW; w += kRansacThreads) refm[w] = nw[w];
            refinedError = err;
            nRef = count;
            if (count == prev) break;
        } else {
            break;
        }
        for (int w = tid; w < MW; w += kRansacThreads) cur[w] = nw[w];
    }
    __syncthreads();
    for (int w = tid; w < MW; w += kRansacThreads) mask_out[w] = refm[w];
    if (tid == 0) {
        for (int i = 0; i < 16; i++) out->T[i] = nRef > 0 ? refT[i] : ((i % 5 == 0) ? 1.0f : 0.0f);
        out->err = refinedError;
        out->n = nRef;
    }
}

__global__ __launch_bounds__(kRansacThreads) void k_ransac_hyp(const float* __restrict__ pts_g,
                                                               const int* __restrict__ samples,
                                                               const int* __restrict__ scount, RansacDev prm,
                                                               HypOut* __restrict__ out,
                                                               uint32_t* __restrict__ masks_out)
{
    extern __shared__ __align__(16) unsigned char smem[];
    const int h = blockIdx.x;
    const bool identity = (h == prm.H);
    ransac_hyp_block(pts_g, samples + (size_t)h * prm.SS, identity ? 0 : scount[h], prm, identity, out + h,
                     masks_out + (size_t)h * prm.MWcap, smem);
}

// Lanes (lanes_dev.h): grid (chunk hypotheses [+ the identity slot in chunk 0], L).  Chunk 0 evaluates
// hypotheses [0, e0) and the identity transform (block e0) of every lane whose RANSAC runs; chunk 1
// [e0, e1) and chunk 2 [e1, H) of the lanes whose replay ran past the previous chunk.
__global__ __launch_bounds__(kRansacThreads) void k_ransac_hyp_lanes(LaneBufs lb, LaneCfg lc, int chunk)
{
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int s_last;
    const int l = blockIdx.y;
    const LaneCtl& c = lb.ctl[l];
    bool active = c.run && !(chunk > 0 && c.need_more != chunk);   // uniform per block
    bool identity = false;
    int h = 0;
    if (active) {
        if (chunk == 0) {
            identity = (int)blockIdx.x == lc.e0;
            if (!identity && (int)blockIdx.x >= min(lc.e0, c.H)) active = false;
            h = identity ? lc.H : (int)blockIdx.x;
        } else {
            h = (chunk == 1 ? lc.e0 : lc.e1) + (int)blockIdx.x;
            if (h >= min(chunk == 1 ? lc.e1 : lc.H, c.H)) active = false;
        }
    }
    if (active) {
        RansacDev prm{};
        prm.M = c.m;
        prm.H = lc.H;
        prm.SS = lc.SS;
        prm.MWcap = lc.MWcap;
        prm.minTh = lc.minTh;
        prm.maxMahal = lc.maxMahal;
        prm.C = c.cov;
        prm.rcx = lc.rcx;
        prm.rcy = lc.rcy;
        const size_t hs = (size_t)l * lc.H + (identity ? 0 : h);
        ransac_hyp_block(lb.pts + (size_t)l * lc.Mcap * 6, lb.samples + hs * lc.SS, identity ? 0 : lb.scount[hs], prm,
                         identity, lb.hyp + (size_t)l * (lc.H + 1) + h,
                         lb.masks + ((size_t)l * (lc.H + 1) + h) * lc.MWcap, smem);
    }
    if (!lc.fuse) return;
    // the lane's replay of this phase, in the last of its active workgroups to finish: every thread's stores
    // released at agent scope (the workgroups of a lane sit on different XCDs, each with its own L2), one atomic
    // count per active workgroup, and the last one acquires before it reads the hypotheses.  Inactive workgroups
    // leave at once (a phase-2 launch is ~H workgroups, almost all idle).  The count is the lane's active
    // workgroups as read at this workgroup's start: c changes only in the replay, which runs after every
    // active workgroup has read it.
    int nact = 0;
    if (c.run) {
        if (chunk == 0)
            nact = min(lc.e0, c.H) + 1;   // hypotheses [0, min(e0, H)) + the identity slot
        else if (c.need_more == chunk)
            nact = min(chunk == 1 ? lc.e1 : lc.H, c.H) - (chunk == 1 ? lc.e0 : lc.e1);
    }
    if (nact <= 0) {
        // no hypothesis of this lane in the launch: phase 0 still writes an early (or finished) lane's outcome,
        // from the identity slot's workgroup; later phases have nothing to replay
        if (chunk == 0 && (int)blockIdx.x == lc.e0) lane_replay(lb, lc, l, 0);
        return;
    }
    if (!active) return;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
        const int prev = atomicAdd(&lb.done[l], 1);
        s_last = prev == nact - 1;
        if (s_last) lb.done[l] = 0;   // every active workgroup of this launch has counted: ready for the next
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    lane_replay(lb, lc, l, chunk);
}

size_t ransac_lds_bytes(int M)
{
    const int MW = (M + 31) >> 5;
    // P 24M + union 32M + list 4M + cur/nw/refm/wbase (MW words each)
    return (size_t)24 * M + (size_t)32 * M + (size_t)4 * M + (size_t)4 * MW * 4 + 64;
}

hipError_t launch_ransac_hyp_lanes(const LaneBufs& lb, const LaneCfg& lc, int chunk, hipStream_t st)
{
    const size_t lds = ransac_lds_bytes(lc.Mcap);
    const int gx = chunk == 0 ? lc.e0 + 1 : (chunk == 1 ? lc.e1 - lc.e0 : lc.H - lc.e1);
    if (gx <= 0) return hipSuccess;
    return dispatch(k_ransac_hyp_lanes, dim3(gx, lc.L), dim3(kRansacThreads), lds, st, lb, lc, chunk);
}

hipError_t launch_ransac_hyp(const float* pts, const int* samples, const int* scount, const RansacDev& prm, HypOut* out,
                       uint32_t* masks, hipStream_t st)
{
    const size_t lds = ransac_lds_bytes(prm.M);
    return dispatch(k_ransac_hyp, dim3(prm.H + 1), dim3(kRansacThreads), lds, st, pts,
                       samples, scount, prm, out, masks);
}

#ifdef RGBD_PNP_PROFILE
void hyp_prof_dump(hipStream_t st)
{
    long long b[16];
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(b, HIP_SYMBOL(g_hyp_prof), sizeof(b));
    fprintf(stderr, "[hyp_prof] refinements %lld us: compact %.1f weights+prefix %.1f alpha %.1f recur %.1f transform %.1f inliers+sum %.1f\n",
            b[0], b[1] * 0.01, b[2] * 0.01, b[3] * 0.01, b[4] * 0.01, b[5] * 0.01, b[6] * 0.01);
    std::memset(b, 0, sizeof(b));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_hyp_prof), b, sizeof(b));
    long long v[8];
    (void)hipMemcpyFromSymbol(v, HIP_SYMBOL(g_svd_prof), sizeof(v));
    fprintf(stderr, "[svd_prof] us: scale+W %.1f sweeps %.1f S+sort %.1f R,t %.1f | sweeps %lld steps %lld\n", v[0] * 0.01,
            v[1] * 0.01, v[2] * 0.01, v[5] * 0.01, v[3], v[4]);
    std::memset(v, 0, sizeof(v));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_svd_prof), v, sizeof(v));
}
#endif

}  // namespace rgbd

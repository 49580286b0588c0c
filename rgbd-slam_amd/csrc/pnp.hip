// pnp.hip -- PnPRansac on gfx950: EPnP hypotheses, inlier counting, Gauss-Newton refinement, and the
// fused match-filter + 3D-2D gather of the tracking chain.
//
// Reference: PnPRansac::compute (Solver/PnPRansac.cpp:14-56) ->
//   cv::solvePnPRansac(v3D, v2D, K, noDist, r, t, false, 500, 3.0f, 0.85, inliers)   (:39)
// OpenCV is not available, so the operator is the definition restated in oracle/orc_pnp.cpp
// (DESIGN.md "PnPRansac definition"); this file computes the same IEEE operations in the same order.
//
// Parallel structure (the RANSAC sample stream of cv::RNG((uint64)-1) depends only on the point
// count, never on results, so every iteration's hypothesis is independent):
//   k_pnp_hyp     one 64-lane workgroup per hypothesis.  Serial pieces (3x3 PCA, sorting) on lane 0;
//                 M^T M (144 entries) across lanes; the 12x12 eigen-solve is a round-robin Jacobi whose
//                 6 disjoint rotations per round are applied by 72 (pair, row) tasks; the three beta
//                 candidates (N = 1, 2, 3) run on lanes 0..2; inlier counting over all points with ballots.
//   host          replays solvePnPRansac's sequential best / RANSACUpdateNumIters loop (pnp_host.cpp).
//   k_pnp_refine  one 256-thread workgroup per problem: order-preserving inlier compaction, then 10
//                 Gauss-Newton steps; J^T J / J^T r in 256 strided lanes + a binary tree (fixed order).
#include <hip/hip_runtime.h>

#include "dispatch.h"

#include <climits>
#include <cstddef>

#include "pnp_dev.h"
#include "exact_dev.h"

namespace rgbd {

#ifdef RGBD_PNP_PROFILE
__device__ long long g_pnp_prof[8192 * 10];   // stage timestamps of lane 0 per hypothesis (profiling builds)
#define PNP_PROF(k) do { if (threadIdx.x == 0 && blockIdx.x < 8192) g_pnp_prof[blockIdx.x * 10 + (k)] = clock64(); } while (0)
#define PNP_PROF_VAL(k, v) do { if (threadIdx.x == 0 && blockIdx.x < 8192) g_pnp_prof[blockIdx.x * 10 + (k)] = (v); } while (0)
// (one record per workgroup: group 0 of each wave)
__device__ long long g_ref_prof[64 * 48];     // k_pnp_refine stage timestamps of thread 0, problems 0..63
#define REF_PROF(k) do { if (threadIdx.x == 0 && blockIdx.x < 64) g_ref_prof[blockIdx.x * 48 + (k)] = clock64(); } while (0)
#else
#define REF_PROF(k) do { } while (0)
#define PNP_PROF(k) do { } while (0)
#define PNP_PROF_VAL(k, v) do { } while (0)
#endif

namespace {

// ------------------------------------------------------------------ small dense helpers (double)
// oracle negligible(): 100|a_pq| changes neither |a_pp| nor |a_qq| in double
__device__ __forceinline__ bool negligible(double apq, double app, double aqq)
{
    const double g = 100.0 * fabs(apq);
    return fabs(app) + g == fabs(app) && fabs(aqq) + g == fabs(aqq);
}

// sqrt_ge1 / div_plain: exact_dev.h

// t = sign(theta) / (|theta| + sqrt(theta^2 + 1)): theta^2 + 1 >= 1 is +inf only for |theta| > 2^512
// (sqrt(inf) = inf, t = +-0); otherwise the denominator is in [1, 2^513] and 1 / den normal.  Both arms are
// computed and selected, so a caller's round stays one basic block.
__device__ __forceinline__ double rot_t(double theta)
{
    const double x1 = theta * theta + 1.0;
    const double s1 = sqrt_ge1(x1);
    const double den = fabs(theta) + (x1 == INFINITY ? x1 : s1);
    const double sg = theta >= 0.0 ? 1.0 : -1.0;
    const double q1 = div_plain(sg, den);
    return den == INFINITY ? sg * 0.0 : q1;
}

// cyclic Jacobi on a symmetric 3 x 3 (row-major, in place); eigenvectors in the columns of V
// (oracle jacobi_eig, n = 3).  Every index is static after unrolling: A and V live in registers.
__device__ __forceinline__ void jacobi_eig3(double* A, double* V)
{
    constexpr int n = 3;
#pragma unroll
    for (int i = 0; i < n; i++)
#pragma unroll
        for (int j = 0; j < n; j++) V[i * n + j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; sweep++) {
        double sm = 0.0;
#pragma unroll
        for (int p = 0; p < n; p++)
#pragma unroll
            for (int q = p + 1; q < n; q++) sm += fabs(A[p * n + q]);
        if (sm == 0.0) break;
#pragma unroll
        for (int p = 0; p < n - 1; p++)
#pragma unroll
            for (int q = p + 1; q < n; q++) {
                const double apq = A[p * n + q];
                if (negligible(apq, A[p * n + p], A[q * n + q])) {
                    A[p * n + q] = 0.0;
                    A[q * n + p] = 0.0;
                    continue;
                }
                const double theta = (A[q * n + q] - A[p * n + p]) / (2.0 * apq);
                const double t = rot_t(theta);
                const double c = div_plain(1.0, sqrt_ge1(t * t + 1.0));   // t^2 + 1 in [1, 2]
                const double s = t * c;
#pragma unroll
                for (int k = 0; k < n; k++) {
                    const double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = c * akp - s * akq;
                    A[k * n + q] = s * akp + c * akq;
                }
#pragma unroll
                for (int k = 0; k < n; k++) {
                    const double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = (k == q) ? 0.0 : c * apk - s * aqk;
                    A[q * n + k] = (k == p) ? 0.0 : s * apk + c * aqk;
                }
#pragma unroll
                for (int k = 0; k < n; k++) {
                    const double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - s * vkq;
                    V[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
}

// The oracle's index sort of 3 eigenvalues, descending by compare-and-swap over (0,1), (0,2), (1,2),
// carried on (value, index) pairs in registers.  idx[c] = original index of the c-th largest.
__device__ __forceinline__ void sort3_desc(double e0, double e1, double e2, int idx[3])
{
    double v[3] = {e0, e1, e2};
    int id[3] = {0, 1, 2};
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
        for (int b = a + 1; b < 3; b++)
            if (v[b] > v[a]) {
                const double tv = v[a]; v[a] = v[b]; v[b] = tv;
                const int ti = id[a]; id[a] = id[b]; id[b] = ti;
            }
#pragma unroll
    for (int c = 0; c < 3; c++) idx[c] = id[c];
}

// column idx (0..2, run-time) of a register-resident row-major 3 x 3
__device__ __forceinline__ double col3(const double* M, int r, int idx)
{
    return idx == 0 ? M[r * 3] : (idx == 1 ? M[r * 3 + 1] : M[r * 3 + 2]);
}

// min |A x - b|, A 6 x N (row-major), Householder QR; N is a template constant so that every
// array index is static and the factorisation stays in registers.
template <int N>
__device__ __forceinline__ void lsq_qr(const double* Ain, const double* bin, double* x)
{
    constexpr int m = 6, n = N;
    double A[m * n], b[m];
#pragma unroll
    for (int i = 0; i < m * n; i++) A[i] = Ain[i];
#pragma unroll
    for (int i = 0; i < m; i++) b[i] = bin[i];
#pragma unroll
    for (int k = 0; k < n; k++) {
        double nrm = 0.0;
#pragma unroll
        for (int i = k; i < m; i++) nrm += A[i * n + k] * A[i * n + k];
        nrm = sqrt(nrm);
        if (nrm == 0.0) continue;
        const double alpha = A[k * n + k] > 0 ? -nrm : nrm;
        double v[m];
#pragma unroll
        for (int i = 0; i < m; i++) v[i] = (i < k) ? 0.0 : A[i * n + k];
        v[k] -= alpha;
        double vn = 0.0;
#pragma unroll
        for (int i = k; i < m; i++) vn += v[i] * v[i];
        if (vn == 0.0) continue;
#pragma unroll
        for (int j = k; j < n; j++) {
            double d = 0.0;
#pragma unroll
            for (int i = k; i < m; i++) d += v[i] * A[i * n + j];
            const double f = 2.0 * d / vn;
#pragma unroll
            for (int i = k; i < m; i++) A[i * n + j] -= f * v[i];
        }
        double d = 0.0;
#pragma unroll
        for (int i = k; i < m; i++) d += v[i] * b[i];
        const double f = 2.0 * d / vn;
#pragma unroll
        for (int i = k; i < m; i++) b[i] -= f * v[i];
    }
#pragma unroll
    for (int k = n - 1; k >= 0; k--) {
        double sacc = b[k];
#pragma unroll
        for (int j = k + 1; j < n; j++) sacc -= A[k * n + j] * x[j];
        x[k] = (A[k * n + k] != 0.0) ? sacc / A[k * n + k] : 0.0;
    }
}

// lsq_qr<n> with a run-time column count n <= NMAX, so that lanes with different n run one instruction
// stream side by side instead of one after another: A is 6 x NMAX row-major (columns >= n ignored); every
// lane performs exactly lsq_qr<n>'s operations in lsq_qr<n>'s order.
template <int NMAX>
__device__ __forceinline__ void lsq_qr_n(const double* Ain, const double* bin, int n, double* x)
{
    constexpr int m = 6;
    double A[m * NMAX], b[m];
#pragma unroll
    for (int i = 0; i < m * NMAX; i++) A[i] = Ain[i];
#pragma unroll
    for (int i = 0; i < m; i++) b[i] = bin[i];
#pragma unroll
    for (int k = 0; k < NMAX; k++) {
        if (k >= n) continue;
        double nrm = 0.0;
#pragma unroll
        for (int i = k; i < m; i++) nrm += A[i * NMAX + k] * A[i * NMAX + k];
        nrm = sqrt(nrm);
        if (nrm == 0.0) continue;
        const double alpha = A[k * NMAX + k] > 0 ? -nrm : nrm;
        double v[m];
#pragma unroll
        for (int i = 0; i < m; i++) v[i] = (i < k) ? 0.0 : A[i * NMAX + k];
        v[k] -= alpha;
        double vn = 0.0;
#pragma unroll
        for (int i = k; i < m; i++) vn += v[i] * v[i];
        if (vn == 0.0) continue;
#pragma unroll
        for (int j = k; j < NMAX; j++) {
            if (j >= n) continue;
            double d = 0.0;
#pragma unroll
            for (int i = k; i < m; i++) d += v[i] * A[i * NMAX + j];
            const double f = 2.0 * d / vn;
#pragma unroll
            for (int i = k; i < m; i++) A[i * NMAX + j] -= f * v[i];
        }
        double d = 0.0;
#pragma unroll
        for (int i = k; i < m; i++) d += v[i] * b[i];
        const double f = 2.0 * d / vn;
#pragma unroll
        for (int i = k; i < m; i++) b[i] -= f * v[i];
    }
#pragma unroll
    for (int k = NMAX - 1; k >= 0; k--) {
        if (k >= n) continue;
        double sacc = b[k];
#pragma unroll
        for (int j = k + 1; j < NMAX; j++)
            if (j < n) sacc -= A[k * NMAX + j] * x[j];
        x[k] = (A[k * NMAX + k] != 0.0) ? sacc / A[k * NMAX + k] : 0.0;
    }
}

__device__ __forceinline__ void svd3_jacobi(const double M[9], double U[9], double S[3], double V[9])
{
    double MtM[9];
    #pragma unroll
    for (int i = 0; i < 3; i++)
        #pragma unroll
        for (int j = 0; j < 3; j++) {
            double s = 0.0;
            #pragma unroll
            for (int k = 0; k < 3; k++) s += M[k * 3 + i] * M[k * 3 + j];
            MtM[i * 3 + j] = s;
        }
    double Vt[9];
    jacobi_eig3(MtM, Vt);
    int idx[3];
    sort3_desc(MtM[0], MtM[4], MtM[8], idx);
    #pragma unroll
    for (int c = 0; c < 3; c++) {
        const double ev = idx[c] == 0 ? MtM[0] : (idx[c] == 1 ? MtM[4] : MtM[8]);
        S[c] = ev > 0.0 ? sqrt(ev) : 0.0;
        #pragma unroll
        for (int r = 0; r < 3; r++) V[r * 3 + c] = col3(Vt, r, idx[c]);
    }
    #pragma unroll
    for (int c = 0; c < 3; c++) {
        double u[3];
        #pragma unroll
        for (int r = 0; r < 3; r++)
            u[r] = (M[r * 3 + 0] * V[0 * 3 + c] + M[r * 3 + 1] * V[1 * 3 + c]) + M[r * 3 + 2] * V[2 * 3 + c];
        #pragma unroll
        for (int p = 0; p < c; p++) {
            const double d = (u[0] * U[0 * 3 + p] + u[1] * U[1 * 3 + p]) + u[2] * U[2 * 3 + p];
            #pragma unroll
            for (int r = 0; r < 3; r++) u[r] -= d * U[r * 3 + p];
        }
        double nn = sqrt((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
        if (nn < 1e-300) {
            if (c == 2) {
                u[0] = U[1 * 3 + 0] * U[2 * 3 + 1] - U[2 * 3 + 0] * U[1 * 3 + 1];
                u[1] = U[2 * 3 + 0] * U[0 * 3 + 1] - U[0 * 3 + 0] * U[2 * 3 + 1];
                u[2] = U[0 * 3 + 0] * U[1 * 3 + 1] - U[1 * 3 + 0] * U[0 * 3 + 1];
            } else {
                u[0] = (c == 0) ? 1.0 : 0.0;
                u[1] = (c == 1) ? 1.0 : 0.0;
                u[2] = 0.0;
                #pragma unroll
                for (int p = 0; p < c; p++) {
                    const double d = (u[0] * U[0 * 3 + p] + u[1] * U[1 * 3 + p]) + u[2] * U[2 * 3 + p];
                    #pragma unroll
                    for (int r = 0; r < 3; r++) u[r] -= d * U[r * 3 + p];
                }
            }
            nn = sqrt((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
        }
        #pragma unroll
        for (int r = 0; r < 3; r++) U[r * 3 + c] = u[r] / nn;
    }
}

__device__ double det3(const double R[9])
{
    return R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) + R[2] * (R[3] * R[7] - R[4] * R[6]);
}

__device__ bool inv3(const double M[9], double Mi[9])
{
    const double d = det3(M);
    if (d == 0.0 || !isfinite(d)) return false;
    Mi[0] = (M[4] * M[8] - M[5] * M[7]) / d;
    Mi[1] = (M[2] * M[7] - M[1] * M[8]) / d;
    Mi[2] = (M[1] * M[5] - M[2] * M[4]) / d;
    Mi[3] = (M[5] * M[6] - M[3] * M[8]) / d;
    Mi[4] = (M[0] * M[8] - M[2] * M[6]) / d;
    Mi[5] = (M[2] * M[3] - M[0] * M[5]) / d;
    Mi[6] = (M[3] * M[7] - M[4] * M[6]) / d;
    Mi[7] = (M[1] * M[6] - M[0] * M[7]) / d;
    Mi[8] = (M[0] * M[4] - M[1] * M[3]) / d;
    return true;
}

// EPnP's 5-step Gauss-Newton on the betas (L: 6 x 10, row-major)
__device__ void gauss_newton(const double* L, const double* rho, double betas[4])
{
#pragma unroll 1
    for (int it = 0; it < 5; it++) {
        double A[6 * 4], b[6];
        #pragma unroll
        for (int i = 0; i < 6; i++) {
            const double* l = L + 10 * i;
            A[i * 4 + 0] = 2 * l[0] * betas[0] + l[1] * betas[1] + l[3] * betas[2] + l[6] * betas[3];
            A[i * 4 + 1] = l[1] * betas[0] + 2 * l[2] * betas[1] + l[4] * betas[2] + l[7] * betas[3];
            A[i * 4 + 2] = l[3] * betas[0] + l[4] * betas[1] + 2 * l[5] * betas[2] + l[8] * betas[3];
            A[i * 4 + 3] = l[6] * betas[0] + l[7] * betas[1] + l[8] * betas[2] + 2 * l[9] * betas[3];
            const double bb[10] = {betas[0] * betas[0], betas[0] * betas[1], betas[1] * betas[1], betas[0] * betas[2],
                                   betas[1] * betas[2], betas[2] * betas[2], betas[0] * betas[3], betas[1] * betas[3],
                                   betas[2] * betas[3], betas[3] * betas[3]};
            double s = 0.0;
            #pragma unroll
            for (int k = 0; k < 10; k++) s += l[k] * bb[k];
            b[i] = rho[i] - s;
        }
        double x[4];
        lsq_qr<4>(A, b, x);
        #pragma unroll
        for (int k = 0; k < 4; k++) betas[k] += x[k];
    }
}

// R, t from betas over the 5 sample points; returns the mean reprojection error
__device__ double compute_R_and_t(const double* pw, const double* us, const double* alphas, const PnpCam& K,
                                  const double* ut, const double betas[4], double R[9], double t[3])
{
    const int n = kPnpModel;
    double ccs[4][3];
    #pragma unroll
    for (int i = 0; i < 4; i++)
        #pragma unroll
        for (int j = 0; j < 3; j++) ccs[i][j] = 0.0;
    #pragma unroll
    for (int k = 0; k < 4; k++)
        #pragma unroll
        for (int i = 0; i < 4; i++)
            #pragma unroll
            for (int j = 0; j < 3; j++) ccs[i][j] += betas[k] * ut[k * 12 + 3 * i + j];
    double pcs[3 * kPnpModel];
    #pragma unroll
    for (int i = 0; i < n; i++)
        #pragma unroll
        for (int j = 0; j < 3; j++)
            pcs[3 * i + j] = ((alphas[4 * i] * ccs[0][j] + alphas[4 * i + 1] * ccs[1][j]) + alphas[4 * i + 2] * ccs[2][j])
                             + alphas[4 * i + 3] * ccs[3][j];
    if (pcs[2] < 0.0) {
        #pragma unroll
        for (int i = 0; i < 4; i++)
            #pragma unroll
            for (int j = 0; j < 3; j++) ccs[i][j] = -ccs[i][j];
        #pragma unroll
        for (int i = 0; i < 3 * n; i++) pcs[i] = -pcs[i];
    }
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    #pragma unroll
    for (int i = 0; i < n; i++)
        #pragma unroll
        for (int j = 0; j < 3; j++) {
            pc0[j] += pcs[3 * i + j];
            pw0[j] += pw[3 * i + j];
        }
    #pragma unroll
    for (int j = 0; j < 3; j++) {
        pc0[j] /= n;
        pw0[j] /= n;
    }
    double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    #pragma unroll
    for (int i = 0; i < n; i++)
        #pragma unroll
        for (int a = 0; a < 3; a++)
            #pragma unroll
            for (int b = 0; b < 3; b++) abt[a * 3 + b] += (pcs[3 * i + a] - pc0[a]) * (pw[3 * i + b] - pw0[b]);
    double U[9], S[3], V[9];
    svd3_jacobi(abt, U, S, V);
    #pragma unroll
    for (int a = 0; a < 3; a++)
        #pragma unroll
        for (int b = 0; b < 3; b++)
            R[a * 3 + b] = (U[a * 3 + 0] * V[b * 3 + 0] + U[a * 3 + 1] * V[b * 3 + 1]) + U[a * 3 + 2] * V[b * 3 + 2];
    if (det3(R) < 0.0)
        #pragma unroll
        for (int b = 0; b < 3; b++) R[6 + b] = -R[6 + b];
    #pragma unroll
    for (int a = 0; a < 3; a++) t[a] = pc0[a] - ((R[a * 3 + 0] * pw0[0] + R[a * 3 + 1] * pw0[1]) + R[a * 3 + 2] * pw0[2]);
    double sum = 0.0;
    #pragma unroll
    for (int i = 0; i < n; i++) {
        const double* p = pw + 3 * i;
        const double Xc = ((R[0] * p[0] + R[1] * p[1]) + R[2] * p[2]) + t[0];
        const double Yc = ((R[3] * p[0] + R[4] * p[1]) + R[5] * p[2]) + t[1];
        const double inv = 1.0 / (((R[6] * p[0] + R[7] * p[1]) + R[8] * p[2]) + t[2]);
        const double ue = K.uc + K.fu * Xc * inv, ve = K.vc + K.fv * Yc * inv;
        const double du = us[2 * i] - ue, dv = us[2 * i + 1] - ve;
        sum += sqrt(du * du + dv * dv);
    }
    return sum / n;
}

// PnPRansacCallback::computeError: float squared distance to the float-stored projection
__device__ __forceinline__ float reproj_err2(const float* P, const float* uv, const double* R, const double* t,
                                             const PnpCam& K)
{
    const double X = ((R[0] * (double)P[0] + R[1] * (double)P[1]) + R[2] * (double)P[2]) + t[0];
    const double Y = ((R[3] * (double)P[0] + R[4] * (double)P[1]) + R[5] * (double)P[2]) + t[1];
    const double Z = ((R[6] * (double)P[0] + R[7] * (double)P[1]) + R[8] * (double)P[2]) + t[2];
    const double iz = Z != 0.0 ? 1.0 / Z : 1.0;
    const float pu = (float)(K.fu * (X * iz) + K.uc);
    const float pv = (float)(K.fv * (Y * iz) + K.vc);
    const float du = uv[0] - pu, dv = uv[1] - pv;
    return du * du + dv * dv;
}

// round-robin pair table of the 12 x 12 Jacobi (oracle rr_pairs12), a compile-time constant
struct RRTable {
    int p[11][6], q[11][6];
};
constexpr RRTable make_rr()
{
    RRTable t{};
    int arr[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
    for (int r = 0; r < 11; r++) {
        for (int k = 0; k < 6; k++) {
            const int a = arr[k], b = arr[11 - k];
            t.p[r][k] = a < b ? a : b;
            t.q[r][k] = a < b ? b : a;
        }
        const int last = arr[11];
        for (int i = 11; i > 1; i--) arr[i] = arr[i - 1];
        arr[1] = last;
    }
    return t;
}
constexpr RRTable kRR = make_rr();
// partner of index k in round r (the lane whose row's element k is zeroed in round r is the lane g == part[r][k])
struct RRPart {
    int part[11][12];
};
constexpr RRPart make_part()
{
    RRPart t{};
    for (int r = 0; r < 11; r++)
        for (int j = 0; j < 6; j++) {
            t.part[r][kRR.p[r][j]] = kRR.q[r][j];
            t.part[r][kRR.q[r][j]] = kRR.p[r][j];
        }
    return t;
}
constexpr RRPart kPart = make_part();

constexpr int kGroup = 12;                 // lanes per hypothesis (one per row of the 12 x 12 matrix)
constexpr int kGroupsPerWave = 64 / kGroup;

// The outlier-flag chain's layout (k_pnp_chain, latency-bound: one pair's EPnP is its critical path): 21 lanes
// per hypothesis, three per wave.  In round r the 12 indices form 6 pairs (kRR), and the matrix is a 6 x 6
// grid of 2 x 2 blocks (rows of pair I, columns of pair J) whose round update reads only that block and the
// (c, s) of pairs I and J.  Lane g < 6 owns the diagonal block (g, g) -- and computes pair g's rotation from
// it -- and lane 6 + k the k-th pair I < J with both blocks (I, J) and (J, I) (A is not kept symmetric: the
// oracle's column-then-row pass rounds a_ij and a_ji differently).  A stays in the group's LDS copy (stride
// 12); a round is: read the lane's 8 elements, the diagonal lanes' (c, s) through LDS, the block updates,
// write back -- ~210 instructions and ~1,240 cycles per round (measured) against ~370 and ~1,870 for the
// row layout, which needs 12 lanes per hypothesis and 5 hypotheses per wave.
constexpr int kBlkGroup = 21;
constexpr int kBlkGroupsPerWave = 64 / kBlkGroup;
// LDS byte offsets (relative to the group's A) of lane g's 8 elements in round r, two u16 per dword:
// X = (pI, pJ), (pI, qJ), (qI, pJ), (qI, qJ); Y = (pJ, pI), (pJ, qI), (qJ, pI), (qJ, qI); and the lane's
// round-0 mask of those in the upper triangle (the convergence test sums |a_pq|, p < q, as the oracle)
struct BlkTab {
    uint32_t o[11][kBlkGroup][4];
    uint32_t up0[kBlkGroup];
    uint32_t ij[kBlkGroup];   // the lane's block (I, J): I | J << 8
};
constexpr BlkTab make_blk()
{
    BlkTab t{};
    int bi[kBlkGroup] = {}, bj[kBlkGroup] = {};
    int n = 0;
    for (int i = 0; i < 6; i++) { bi[n] = i; bj[n] = i; n++; }
    for (int i = 0; i < 6; i++)
        for (int j = i + 1; j < 6; j++) { bi[n] = i; bj[n] = j; n++; }
    for (int g = 0; g < kBlkGroup; g++) t.ij[g] = (uint32_t)(bi[g] | (bj[g] << 8));
    for (int r = 0; r < 11; r++)
        for (int g = 0; g < kBlkGroup; g++) {
            const int pI = kRR.p[r][bi[g]], qI = kRR.q[r][bi[g]], pJ = kRR.p[r][bj[g]], qJ = kRR.q[r][bj[g]];
            const int rc[8][2] = {{pI, pJ}, {pI, qJ}, {qI, pJ}, {qI, qJ}, {pJ, pI}, {pJ, qI}, {qJ, pI}, {qJ, qI}};
            uint32_t e[8] = {};
            for (int k = 0; k < 8; k++) {
                e[k] = (uint32_t)(8 * (rc[k][0] * 12 + rc[k][1]));
                if (r == 0 && rc[k][0] < rc[k][1]) t.up0[g] |= 1u << k;
            }
            for (int k = 0; k < 4; k++) t.o[r][g][k] = e[2 * k] | (e[2 * k + 1] << 16);
        }
    return t;
}
__device__ const BlkTab kBlkTab = make_blk();

// Row stride of the group's LDS copy of A during the Jacobi sweeps: 14 doubles (112 B), so the eight
// lanes of a ds_write_b128 group cover the 32 banks once, and a struct stride of 880 dwords (= 48 mod
// 64) keeps neighbouring groups' rows off each other's banks in the ds_read_b128 partner-row reads
// (bank model: 1755 LDS cycles per sweep against the 1430 conflict-free minimum; 2985 at stride 12)
constexpr int kRowStride = 14;

struct alignas(16) HypLds {
    double V[12 * kRowStride];   // V (stride 12) after the sweeps; the rows of A (stride 14) during them
    double diag[12];
    double pw[15], us[10], alphas[20], cw[12];
    double ut[48], L[60], rho[6];
    double candR[3][9], candT[3][3], candE[3];
    double R[9], t[3];
    int order[4];
    int cnt[24];   // per-lane inlier counts (12 or 21 lanes)
    int ok;
    int pad_[47];
};
static_assert(sizeof(HypLds) == 880 * 4, "HypLds stride is part of the LDS bank layout");
static_assert(offsetof(HypLds, candE) - offsetof(HypLds, ut) >= 120 * sizeof(double), "hyp_eval's M tables over ut..");

// element e of a register-resident row as a 4-level select tree on the bits of e (b0 = e & 1 ... b3 = e & 8):
// the same 11 selects as a linear chain, 4 deep instead of 11 on the Jacobi round's critical path
__device__ __forceinline__ double row_sel(const double (&r)[12], bool b0, bool b1, bool b2, bool b3)
{
    const double x0 = b0 ? r[1] : r[0], x1 = b0 ? r[3] : r[2], x2 = b0 ? r[5] : r[4];
    const double x3 = b0 ? r[7] : r[6], x4 = b0 ? r[9] : r[8], x5 = b0 ? r[11] : r[10];
    const double y0 = b1 ? x1 : x0, y1 = b1 ? x3 : x2, y2 = b1 ? x5 : x4;
    const double z0 = b2 ? y1 : y0;
    return b3 ? y2 : z0;
}

// x of lane l - S within each 16-lane row (DPP row_shr:S); lanes with no source get 0.  Only lane
// 15 of each row is consumed after the S = 1, 2, 4, 8 levels, and its sources are always valid.
template <int S>
__device__ __forceinline__ double dpp_row_shr(double x)
{
    const unsigned long long u = __builtin_bit_cast(unsigned long long, x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(u & 0xFFFFFFFFull), 0x110 + S, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(u >> 32), 0x110 + S, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// ordering of LDS traffic between the lanes of one wave (the workgroup is one wave)
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// EPnP of the hypothesis of one G-lane group (G = kGroup: lane g owns row g; G = kBlkGroup: the block layout
// of the Jacobi, BlkTab), then its inlier count over the problem's
// points: *good_dst = count or -1 (no model), model_dst[0..11] = R (row-major), t.  Every lane of the
// workgroup calls it: k_pnp_hyp's one-wave workgroups and the four waves of k_pnp_chain.  has = a hypothesis exists in this slot; valid = write the results.  A group lies
// inside one wave and its HypLds is its own, so the stages are ordered by wave-level syncs: the waves of a
// k_pnp_chain pass drift apart (each finishes after its own slowest stages, not after every stage's slowest
// wave) and meet at the caller's barrier.
template <int G>
__device__ __forceinline__ void hyp_eval(HypLds& s, double2* CS, const uint4* __restrict__ blk_off, int g, int base,
                                         bool live, bool valid, bool has,
                                         const int* __restrict__ smp, const float* __restrict__ P3,
                                         const float* __restrict__ P2, int count, const PnpCam& K, float thr,
                                         int* __restrict__ good_dst, double* __restrict__ model_dst)
{
    PNP_PROF(0);
    // ---- group lane 0: sample points, control points (PCA), barycentric coordinates
    if (live && g == 0 && !has) s.ok = 0;
    if (live && g == 0 && has) {
        const int n = kPnpModel;
        for (int i = 0; i < n; i++) {
            const int id = smp[i];
            for (int j = 0; j < 3; j++) s.pw[3 * i + j] = (double)P3[3 * id + j];
            for (int j = 0; j < 2; j++) s.us[2 * i + j] = (double)P2[2 * id + j];
        }
        double cw[4][3];
#pragma unroll
        for (int j = 0; j < 3; j++) cw[0][j] = 0.0;
#pragma unroll
        for (int i = 0; i < n; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) cw[0][j] += s.pw[3 * i + j];
#pragma unroll
        for (int j = 0; j < 3; j++) cw[0][j] /= n;
        double A[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < n; i++) {
            double d[3];
#pragma unroll
            for (int j = 0; j < 3; j++) d[j] = s.pw[3 * i + j] - cw[0][j];
#pragma unroll
            for (int a = 0; a < 3; a++)
#pragma unroll
                for (int b = 0; b < 3; b++) A[a * 3 + b] += d[a] * d[b];
        }
        double V[9];
        jacobi_eig3(A, V);
        int idx[3];
        sort3_desc(A[0], A[4], A[8], idx);
#pragma unroll
        for (int i = 1; i < 4; i++) {
            const int ii = idx[i - 1];
            const double ev = ii == 0 ? A[0] : (ii == 1 ? A[4] : A[8]);
            const double k = sqrt((ev > 0.0 ? ev : 0.0) / n);
#pragma unroll
            for (int j = 0; j < 3; j++) cw[i][j] = cw[0][j] + k * col3(V, j, ii);
        }
        double CC[9], CCi[9];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 1; j < 4; j++) CC[i * 3 + (j - 1)] = cw[j][i] - cw[0][i];
        s.ok = inv3(CC, CCi) ? 1 : 0;
#pragma unroll
        for (int i = 0; i < n; i++) {
            double d[3];
#pragma unroll
            for (int j = 0; j < 3; j++) d[j] = s.pw[3 * i + j] - cw[0][j];
#pragma unroll
            for (int j = 0; j < 3; j++)
                s.alphas[4 * i + 1 + j] = (CCi[j * 3 + 0] * d[0] + CCi[j * 3 + 1] * d[1]) + CCi[j * 3 + 2] * d[2];
            s.alphas[4 * i] = 1.0 - s.alphas[4 * i + 1] - s.alphas[4 * i + 2] - s.alphas[4 * i + 3];
        }
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) s.cw[3 * i + j] = cw[i][j];
    }
    wave_sync();
    PNP_PROF(1);
    const bool ok0 = s.ok != 0;

    // ---- row g of M^T M: sum over the 5 points of r1a r1b + r2a r2b, point order
    double A[12], Vr[12];
    if constexpr (G == kBlkGroup) {
        // block layout: M's two rows per point as tables T1[i][b] = r1_b, T2[i][b] = r2_b (scratch over ut, L,
        // rho, candR, which are written after the sweeps), then every element of M^T M on its own lane,
        // straight into the group's LDS copy of A (a short rolled loop: this code is fetched cold per pass)
        double* const T1 = reinterpret_cast<double*>(reinterpret_cast<char*>(&s) + offsetof(HypLds, ut));
        double* const T2 = T1 + 60;
        if (live)
#pragma unroll 1
            for (int e = g; e < 12 * kPnpModel; e += G) {
                const int i = e / 12, b = e - 12 * i, c = b % 3;
                const double al = s.alphas[4 * i + b / 3], u = s.us[2 * i], v = s.us[2 * i + 1];
                T1[e] = c == 0 ? al * K.fu : (c == 1 ? 0.0 : al * (K.uc - u));
                T2[e] = c == 0 ? 0.0 : (c == 1 ? al * K.fv : al * (K.vc - v));
            }
        wave_sync();
        if (live)
#pragma unroll 1
            for (int e = g; e < 144; e += G) {
                const int a = e / 12, b = e - 12 * a;
                double acc = 0.0;
#pragma unroll
                for (int i = 0; i < kPnpModel; i++)
                    acc += T1[12 * i + a] * T1[12 * i + b] + T2[12 * i + a] * T2[12 * i + b];
                s.V[e] = acc;
            }
#pragma unroll
        for (int b = 0; b < 12; b++) Vr[b] = (g == b) ? 1.0 : 0.0;
    } else {
        const int a = g;
#pragma unroll
        for (int b = 0; b < 12; b++) {
            double acc = 0.0;
#pragma unroll
            for (int i = 0; i < kPnpModel; i++) {
                const double u = s.us[2 * i], v = s.us[2 * i + 1];
                const double aa = s.alphas[4 * i + a / 3], ab = s.alphas[4 * i + b / 3];
                const int ca = a % 3, cb = b % 3;
                const double r1a = ca == 0 ? aa * K.fu : (ca == 1 ? 0.0 : aa * (K.uc - u));
                const double r1b = cb == 0 ? ab * K.fu : (cb == 1 ? 0.0 : ab * (K.uc - u));
                const double r2a = ca == 0 ? 0.0 : (ca == 1 ? aa * K.fv : aa * (K.vc - v));
                const double r2b = cb == 0 ? 0.0 : (cb == 1 ? ab * K.fv : ab * (K.vc - v));
                acc += r1a * r1b + r2a * r2b;
            }
            A[b] = acc;
            Vr[b] = (a == b) ? 1.0 : 0.0;
        }
    }
    PNP_PROF(2);

    int sweep = 0;
    if constexpr (G == kGroup) {
    // ---- round-robin Jacobi (oracle jacobi_eig12): lane g keeps row g of A and of V in registers;
    //      every pair's (c, s) and the partner row go through the group's LDS copy of A (aliased on s.V,
    //      which is only written after the sweeps)
    double2* RA2 = reinterpret_cast<double2*>(s.V);
    unsigned long long mtab = 0;           // partner of row g in round r: bits [4r, 4r + 4)
#pragma unroll
    for (int r = 0; r < 11; r++) {
        int m = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) {
            m = (g == kRR.p[r][j]) ? kRR.q[r][j] : m;
            m = (g == kRR.q[r][j]) ? kRR.p[r][j] : m;
        }
        mtab |= (unsigned long long)m << (4 * r);
    }
    // (c, s) of the previous round's six pairs: their V column updates are applied during the next round's
    // (c, s) chain, which does not read V (identity rotations before the first round: exact no-ops on the
    // initial identity V)
    double2 csv[6];
#pragma unroll
    for (int j = 0; j < 6; j++) csv[j] = make_double2(1.0, 0.0);
    auto apply_v = [&](int rr) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 6; j++) {
            const int pj = kRR.p[rr][j], qj = kRR.q[rr][j];
            const double vkp = Vr[pj], vkq = Vr[qj];
            Vr[pj] = csv[j].x * vkp - csv[j].y * vkq;
            Vr[qj] = csv[j].y * vkp + csv[j].x * vkq;
        }
    };
    const bool gb0 = (g & 1) != 0, gb1 = (g & 2) != 0, gb2 = (g & 4) != 0, gb3 = (g & 8) != 0;
    const double* RAd = reinterpret_cast<const double*>(s.V);   // the same rows as doubles (stride kRowStride)
    if (live && ok0) {
        // a_gg (dmine), a_gm (apq) and the partner's a_mm (dpart) of the coming round, carried from round to
        // round as scalars: each round computes its successors with the same operations (and operands) as
        // the static-slot updates below, so no run-time-indexed select of the row is needed
        const int m0 = (int)(mtab & 15ull);
        double dmine = row_sel(A, gb0, gb1, gb2, gb3);
        double apq = row_sel(A, (m0 & 1) != 0, (m0 & 2) != 0, (m0 & 4) != 0, (m0 & 8) != 0);
        double dpart = __shfl(dmine, base + m0, 64);
        // the row pass of a round is applied at the start of the next one (or before the sweep's convergence
        // test), beside that round's (c, s) chain: pc, ps and the partner's row pe of the pending pass
        double pe[12], pc = 1.0, ps = 0.0;
#pragma unroll
        for (int k = 0; k < 12; k++) pe[k] = 0.0;
        // rows p, q of a pair against the partner's column-updated row, then a_pq = a_qp = 0: lane g zeroes
        // its element m, i.e. slot k where g is k's partner in round rr (a compile-time lane set: the 12
        // masks g == j serve every round).  p: c a - s b,  q: s b + c a  ==  c a + (-s) b exactly
        int gq = g;
        auto row_pass = [&](int rr) __attribute__((always_inline)) {
#pragma unroll
            for (int k = 0; k < 12; k++) A[k] = pc * A[k] + ps * pe[k];
#pragma unroll
            for (int k = 0; k < 12; k++) A[k] = (gq == kPart.part[rr][k]) ? 0.0 : A[k];
        };
        for (; sweep < 50; sweep++) {
            asm volatile("" : "+v"(gq));   // per-sweep value: the 12 (g == j) masks are formed once per sweep
            if (sweep > 0) row_pass(10);   // the previous sweep's last round
            // sum |a_pq| == 0  <=>  every off-diagonal element is exactly zero (order-free)
            bool nz = false;
#pragma unroll
            for (int e = 0; e < 12; e++) nz |= (e > g) && (A[e] != 0.0);
            const unsigned long long gm = ((1ull << kGroup) - 1ull) << base;
            if ((__ballot(nz) & gm) == 0ull) break;
            unsigned long long mt = mtab;
            asm volatile("" : "+v"(mt));   // per-sweep value: keeps the 11 x 12 (e == m) masks out of SGPRs
#pragma unroll
            for (int r = 0; r < 11; r++) {
                const int m = (int)((mt >> (4 * r)) & 15ull);
                const int mn = (int)((mt >> (4 * ((r + 1) % 11))) & 15ull);   // the next round's partner
                const bool isp = g < m;
                apply_v(r == 0 ? 10 : r - 1);   // the previous round's V columns (beside the chain below)
                if (r > 0) row_pass(r - 1);     // the previous round's row pass (beside the chain below)
                // p lane of each pair: (c, s); identity for a negligible a_pq.  Branchless, so the round is
                // one block the scheduler can interleave: every lane evaluates the chain, the rotating p lanes
                // keep it (inf / NaN elsewhere are discarded)
                const bool rot = isp && !negligible(apq, dmine, dpart);
                const double theta = (dpart - dmine) / (2.0 * apq);
                const double tq = rot_t(theta);
                const double cq = div_plain(1.0, sqrt_ge1(tq * tq + 1.0));   // tq^2 + 1 in [1, 2]
                const double c = rot ? cq : 1.0, sn = rot ? tq * cq : 0.0;
                CS[g] = make_double2(c, sn);   // read back only at the p rows
                wave_sync();
                // columns p, q of every pair (own row of A; V's in the next round)
#pragma unroll
                for (int j = 0; j < 6; j++) {
                    const int pj = kRR.p[r][j], qj = kRR.q[r][j];
                    csv[j] = CS[pj];
                    const double akp = A[pj], akq = A[qj];
                    A[pj] = csv[j].x * akp - csv[j].y * akq;
                    A[qj] = csv[j].y * akp + csv[j].x * akq;
                }
                const double2 my = CS[isp ? g : m];
                const double mys = isp ? -my.y : my.y;
                // own slot g after the column pass: p: c a_gg - s a_gm;  q: s a_gm + c a_gg
                const double dcol = my.x * dmine + mys * apq;
#pragma unroll
                for (int k = 0; k < 6; k++) RA2[g * (kRowStride / 2) + k] = make_double2(A[2 * k], A[2 * k + 1]);
                wave_sync();
                // the partner's column-updated row, kept for this round's row pass
#pragma unroll
                for (int k = 0; k < 6; k++) {
                    double2 v = RA2[m * (kRowStride / 2) + k];
                    asm("" : "+v"(v.x), "+v"(v.y));   // the whole row is read (no branch around a zeroed slot)
                    pe[2 * k] = v.x;
                    pe[2 * k + 1] = v.y;
                }
                pc = my.x;
                ps = mys;
                // the next round's a_gg, a_gm' (m' != m: never zeroed) and the partner's diagonal: the row pass
                // of slots g and m' from the column-updated values in LDS (own row, partner row)
                dmine = my.x * dcol + mys * RAd[m * kRowStride + g];
                apq = my.x * RAd[g * kRowStride + mn] + mys * RAd[m * kRowStride + mn];
                dpart = __shfl(dmine, base + mn, 64);
                wave_sync();   // this round's LDS reads are consumed before the next round's writes
            }
        }
        if (sweep == 50) row_pass(10);   // (a break at the convergence test has applied it)
        apply_v(10);   // the last round of the last sweep
    }
    wave_sync();
    if (live) {
#pragma unroll
        for (int e = 0; e < 12; e++)   // static indices only: a run-time index would put A in scratch
            if (e == g) s.diag[e] = A[e];
#pragma unroll
        for (int e = 0; e < 12; e++) s.V[g * 12 + e] = Vr[e];
    }
    } else {
        // ---- the block layout (BlkTab): A in the group's LDS copy (stride 12), lane g < 12 keeps row g of V
        char* const Ab = reinterpret_cast<char*>(s.V);
        const int gg = live ? g : 0;
        const bool dg = gg < 6;   // the lane of a diagonal block (pair gg's rotation)
        // the lane's element offsets come from the workgroup's LDS copy of BlkTab (blk_off[r * 21 + g]), each
        // round's read one round ahead (44 registers fewer than holding all 11 rounds)
        uint4 oc = blk_off[gg];
        const uint32_t ij = kBlkTab.ij[gg], up0 = kBlkTab.up0[gg];
        const int bI = (int)(ij & 255u), bJ = (int)(ij >> 8);
        wave_sync();   // M^T M in the LDS copy
        if (live && ok0) {
            double x[4], y[4];
            // V's update of a round runs at the start of the next one, between the issue of that round's block
            // loads and their use (the empty asm ties the loaded values to V's new rows, so the update fills the
            // LDS latency instead of following it); identity before the first round (exact no-ops on V = I)
            double2 cvp[6];
#pragma unroll
            for (int j = 0; j < 6; j++) cvp[j] = make_double2(1.0, 0.0);
            auto apply_v = [&](int rr) __attribute__((always_inline)) {
#pragma unroll
                for (int j = 0; j < 6; j++) {
                    const int pj = kRR.p[rr][j], qj = kRR.q[rr][j];
                    const double vkp = Vr[pj], vkq = Vr[qj];
                    Vr[pj] = cvp[j].x * vkp - cvp[j].y * vkq;
                    Vr[qj] = cvp[j].y * vkp + cvp[j].x * vkq;
                }
            };
            auto ld = [&](uint32_t o) { return *reinterpret_cast<const double*>(Ab + o); };
            auto st = [&](uint32_t o, double v) { *reinterpret_cast<double*>(Ab + o) = v; };
            auto load_blocks = [&](const uint4& o) __attribute__((always_inline)) {
                x[0] = ld(o.x & 0xffffu); x[1] = ld(o.x >> 16); x[2] = ld(o.y & 0xffffu); x[3] = ld(o.y >> 16);
                y[0] = ld(o.z & 0xffffu); y[1] = ld(o.z >> 16); y[2] = ld(o.w & 0xffffu); y[3] = ld(o.w >> 16);
            };
            for (; sweep < 50; sweep++) {
                load_blocks(oc);
                // sum |a_pq| (p < q) == 0: the upper-triangle elements among the lane's round-0 blocks
                bool nz = false;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    nz |= ((up0 >> k) & 1u) != 0u && x[k] != 0.0;
                    nz |= ((up0 >> (4 + k)) & 1u) != 0u && y[k] != 0.0;
                }
                const unsigned long long gm = ((1ull << kBlkGroup) - 1ull) << base;
                if ((__ballot(nz) & gm) == 0ull) break;
#pragma unroll
                for (int r = 0; r < 11; r++) {
                    if (r > 0) load_blocks(oc);
                    asm volatile("" ::: "memory");   // the loads issue before V's update
                    apply_v(r == 0 ? 10 : r - 1);
#pragma unroll
                    for (int k = 0; k < 12; k++) asm volatile("" : "+v"(Vr[k]));
#pragma unroll
                    for (int k = 0; k < 4; k++) asm volatile("" : "+v"(x[k]), "+v"(y[k]));
                    const uint4 on = blk_off[((r + 1) % 11) * kBlkGroup + gg];
                    // pair bI's (c, s) from its diagonal block (a_pp, a_pq, a_qq); identity for a negligible a_pq
                    const double app = x[0], apq = x[1], aqq = x[3];
                    const bool rot = !negligible(apq, app, aqq);
                    const double theta = (aqq - app) / (2.0 * apq);
                    const double tq = rot_t(theta);
                    const double cq = div_plain(1.0, sqrt_ge1(tq * tq + 1.0));   // tq^2 + 1 in [1, 2]
                    const double c = rot ? cq : 1.0, sn = rot ? tq * cq : 0.0;
                    if (dg) CS[bI] = make_double2(c, sn);
                    wave_sync();
                    const double2 cI = CS[bI], cJ = CS[bJ];
#pragma unroll
                    for (int j = 0; j < 6; j++) cvp[j] = CS[j];
                    // X (rows of pair I, columns of pair J): the column pass with J's rotation, then the row
                    // pass with I's (oracle order and operations); the diagonal block's a_pq, a_qp become 0
                    const double x0 = cJ.x * x[0] - cJ.y * x[1], x1 = cJ.y * x[0] + cJ.x * x[1];
                    const double x2 = cJ.x * x[2] - cJ.y * x[3], x3 = cJ.y * x[2] + cJ.x * x[3];
                    const double X0 = cI.x * x0 - cI.y * x2, X3 = cI.y * x1 + cI.x * x3;
                    const double X1 = dg ? 0.0 : cI.x * x1 - cI.y * x3, X2 = dg ? 0.0 : cI.y * x0 + cI.x * x2;
                    // Y (rows of pair J, columns of pair I): columns with I's rotation, then rows with J's
                    const double y0 = cI.x * y[0] - cI.y * y[1], y1 = cI.y * y[0] + cI.x * y[1];
                    const double y2 = cI.x * y[2] - cI.y * y[3], y3 = cI.y * y[2] + cI.x * y[3];
                    const double Y0 = cJ.x * y0 - cJ.y * y2, Y2 = cJ.y * y0 + cJ.x * y2;
                    const double Y1 = cJ.x * y1 - cJ.y * y3, Y3 = cJ.y * y1 + cJ.x * y3;
                    const uint4 o = oc;
                    st(o.x & 0xffffu, X0); st(o.x >> 16, X1); st(o.y & 0xffffu, X2); st(o.y >> 16, X3);
                    if (!dg) {   // (a diagonal lane's Y is its X)
                        st(o.z & 0xffffu, Y0); st(o.z >> 16, Y1); st(o.w & 0xffffu, Y2); st(o.w >> 16, Y3);
                    }
                    oc = on;
                    wave_sync();   // the round's writes before the next round's reads (and CS reads before writes)
                }
            }
            apply_v(10);   // the last round of the last sweep (V rows g < 12; the other lanes' are unused)
        }
        wave_sync();
        double dgv = 0.0;
        if (live && g < 12) dgv = reinterpret_cast<const double*>(Ab)[g * 13];
        wave_sync();   // every diagonal read before V overwrites the LDS copy of A
        if (live && g < 12) {
            s.diag[g] = dgv;
#pragma unroll
            for (int e = 0; e < 12; e++) s.V[g * 12 + e] = Vr[e];
        }
    }
    wave_sync();
    PNP_PROF(8);
    PNP_PROF_VAL(9, sweep);

    // ---- the four smallest eigenvalues (ascending, ties by index), null-space basis ut, L and rho
    if (live && g == 0) {   // (value, index) compare-and-swap in registers, the oracle's order
        double ev[12];
        int id[12];
#pragma unroll
        for (int i = 0; i < 12; i++) {
            ev[i] = s.diag[i];
            id[i] = i;
        }
#pragma unroll
        for (int a = 0; a < 12; a++)
#pragma unroll
            for (int b = a + 1; b < 12; b++)
                if (ev[b] < ev[a]) {
                    const double tv = ev[a]; ev[a] = ev[b]; ev[b] = tv;
                    const int ti = id[a]; id[a] = id[b]; id[b] = ti;
                }
#pragma unroll
        for (int k = 0; k < 4; k++) s.order[k] = id[k];
    }
    wave_sync();
    PNP_PROF(3);
    if (live)
        for (int e = g; e < 48; e += G) {
            const int k = e / 12, i = e % 12;
            s.ut[e] = s.V[i * 12 + s.order[k]];
        }
    wave_sync();
    if (live && g < 6) {
        const int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
        const int a = pa[g], b = pb[g];
        double dv[4][3];
        for (int k = 0; k < 4; k++)
            for (int j = 0; j < 3; j++) dv[k][j] = s.ut[k * 12 + 3 * a + j] - s.ut[k * 12 + 3 * b + j];
        auto dot = [&](int x, int y) { return (dv[x][0] * dv[y][0] + dv[x][1] * dv[y][1]) + dv[x][2] * dv[y][2]; };
        double* L = s.L + 10 * g;
        L[0] = dot(0, 0);
        L[1] = 2 * dot(0, 1);
        L[2] = dot(1, 1);
        L[3] = 2 * dot(0, 2);
        L[4] = 2 * dot(1, 2);
        L[5] = dot(2, 2);
        L[6] = 2 * dot(0, 3);
        L[7] = 2 * dot(1, 3);
        L[8] = 2 * dot(2, 3);
        L[9] = dot(3, 3);
        const double dx = s.cw[3 * a + 0] - s.cw[3 * b + 0], dy = s.cw[3 * a + 1] - s.cw[3 * b + 1],
                     dz = s.cw[3 * a + 2] - s.cw[3 * b + 2];
        s.rho[g] = (dx * dx + dy * dy) + dz * dz;
    }
    wave_sync();
    PNP_PROF(4);

    // ---- beta candidates N = 1, 2, 3 on group lanes 0, 1, 2
    if (live && g < 3) {
        const int N = g + 1;
        double x[5], b4[4];
        // the three least-squares problems side by side on the three lanes (one instruction stream):
        // N = 1: betas 11, 12, 13, 14 -> L columns 0, 1, 3, 6; N = 2: betas 11, 12, 22 -> columns 0..2;
        // N = 3: betas 11, 12, 22, 13, 23 -> columns 0..4
        const int nc = N == 1 ? 4 : (N == 2 ? 3 : 5);
        double A5[30];
#pragma unroll
        for (int i = 0; i < 6; i++)
#pragma unroll
            for (int k = 0; k < 5; k++) {
                const int col = (N == 1) ? (k == 2 ? 3 : (k == 3 ? 6 : k)) : k;
                A5[i * 5 + k] = k < nc ? s.L[10 * i + col] : 0.0;
            }
        lsq_qr_n<5>(A5, s.rho, nc, x);
        if (N == 1) {
            if (x[0] < 0) {
                const double b0 = sqrt(-x[0]);
                b4[0] = b0; b4[1] = -x[1] / b0; b4[2] = -x[2] / b0; b4[3] = -x[3] / b0;
            } else {
                const double b0 = sqrt(x[0]);
                b4[0] = b0; b4[1] = x[1] / b0; b4[2] = x[2] / b0; b4[3] = x[3] / b0;
            }
        } else {
            if (x[0] < 0) {
                b4[0] = sqrt(-x[0]);
                b4[1] = (x[2] < 0) ? sqrt(-x[2]) : 0.0;
            } else {
                b4[0] = sqrt(x[0]);
                b4[1] = (x[2] > 0) ? sqrt(x[2]) : 0.0;
            }
            if (x[1] < 0) b4[0] = -b4[0];
            b4[2] = (N == 3) ? x[3] / b4[0] : 0.0;
            b4[3] = 0.0;
        }
        gauss_newton(s.L, s.rho, b4);
        s.candE[g] = compute_R_and_t(s.pw, s.us, s.alphas, K, s.ut, b4, s.candR[g], s.candT[g]);
    }
    wave_sync();
    PNP_PROF(5);
    if (live && g == 0) {
        double best = INFINITY;
        int bi = -1;
        for (int c = 0; c < 3; c++)
            if (s.candE[c] < best) { best = s.candE[c]; bi = c; }
        s.ok = (ok0 && bi >= 0) ? 1 : 0;
        if (bi >= 0) {
            for (int i = 0; i < 9; i++) s.R[i] = s.candR[bi][i];
            for (int i = 0; i < 3; i++) s.t[i] = s.candT[bi][i];
        }
    }
    wave_sync();
    PNP_PROF(6);
    // ---- findInliers over every point of the problem
    const bool okm = s.ok != 0;
    double R[9], t[3];
#pragma unroll
    for (int i = 0; i < 9; i++) R[i] = s.R[i];
#pragma unroll
    for (int i = 0; i < 3; i++) t[i] = s.t[i];
    int cnt = 0;
    if (live && okm) {   // four points in flight per lane (independent division chains)
        int i = g;
        // (rolled loops: the pass's code is fetched cold for every hypothesis, so its size is time)
#pragma unroll 1
        for (; i + 3 * G < count; i += 4 * G) {
            const bool i0 = reproj_err2(P3 + 3 * i, P2 + 2 * i, R, t, K) <= thr;
            const bool i1 = reproj_err2(P3 + 3 * (i + G), P2 + 2 * (i + G), R, t, K) <= thr;
            const bool i2 = reproj_err2(P3 + 3 * (i + 2 * G), P2 + 2 * (i + 2 * G), R, t, K) <= thr;
            const bool i3 = reproj_err2(P3 + 3 * (i + 3 * G), P2 + 2 * (i + 3 * G), R, t, K) <= thr;
            cnt += (int)i0 + (int)i1 + (int)i2 + (int)i3;
        }
#pragma unroll 1
        for (; i < count; i += G) cnt += reproj_err2(P3 + 3 * i, P2 + 2 * i, R, t, K) <= thr ? 1 : 0;
    }
    if (live) s.cnt[g] = cnt;
    wave_sync();
    if (valid && g == 0) {
        int tot = 0;
        for (int k = 0; k < G; k++) tot += s.cnt[k];
        *good_dst = okm ? tot : -1;
    }
    if (valid && okm && g < 12) model_dst[g] = g < 9 ? R[g] : t[g - 9];
    PNP_PROF(7);
}

}  // namespace

// test hook: sqrt_ge1 / div_plain / rot_t over arrays (rgbd_debug_rotation_ops)
__global__ __launch_bounds__(256) void k_debug_rotation_ops(const double* __restrict__ x, const double* __restrict__ num,
                                                            const double* __restrict__ den, const double* __restrict__ theta,
                                                            int n, double* __restrict__ sq, double* __restrict__ q,
                                                            double* __restrict__ t)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    sq[i] = sqrt_ge1(x[i]);
    q[i] = div_plain(num[i], den[i]);
    t[i] = rot_t(theta[i]);
}

hipError_t launch_debug_rotation_ops(const double* x, const double* num, const double* den, const double* theta, int n,
                                     double* sq, double* q, double* t, hipStream_t st)
{
    return dispatch(k_debug_rotation_ops, dim3((n + 255) / 256), dim3(256), 0, st, x, num, den, theta, n, sq, q, t);
}

// Five hypotheses per 64-lane wave, 12 lanes each (lanes 60..63 idle): lane g of a group owns row g
// of the 12 x 12 M^T M and of V during the round-robin Jacobi, which then runs in registers with the
// partner rows exchanged by ds_bpermute; the pair table is unrolled, so all indices are static.
#define RGBD_HYP_EU 1   // waves per SIMD: r04 mid-round 2 (256 VGPRs, 336 B scratch) beat 1 (354 registers): 219.0-220.1k vs 217.7-218.1k; at the round's final build (k_describe at 8 waves per SIMD) 1 beats 2: 233.4k vs 232.1k (profiles/r04_ab_hyp_eu_final)
__global__ __launch_bounds__(64, RGBD_HYP_EU) void k_pnp_hyp(const float* __restrict__ p3, const float* __restrict__ p2,
                                                const PnpProbDev* __restrict__ probs, const int* __restrict__ hyp_prob,
                                                const int* __restrict__ samples, PnpCam K, float thr, int H,
                                                int* __restrict__ good_out, PnpModel* __restrict__ model_out)
{
    __shared__ HypLds sh[kGroupsPerWave];
    __shared__ double2 cs_sh[kGroupsPerWave][12];
    const int lane = threadIdx.x;
    const int grp = lane / kGroup < kGroupsPerWave ? lane / kGroup : kGroupsPerWave - 1;
    const bool live = lane < kGroupsPerWave * kGroup;
    const int g = live ? lane - grp * kGroup : 0;          // row owned by this lane
    const int h_raw = blockIdx.x * kGroupsPerWave + grp;
    const bool valid = live && h_raw < H;
    const int h = h_raw < H ? h_raw : H - 1;             // tail groups recompute the last hypothesis
    const int hp = hyp_prob[h];                         // -1: no hypothesis in this slot
    if (__ballot(live && hp >= 0) == 0ull) {            // a workgroup (one wave) without hypotheses
        if (valid && g == 0) good_out[h] = -1;          // every slot gets its count or -1 (pnp_dev.h)
        return;
    }
    const PnpProbDev pr = hp >= 0 ? probs[hp] : PnpProbDev{0, 0};
    hyp_eval<kGroup>(sh[grp], cs_sh[grp], nullptr, g, grp * kGroup, live, valid, hp >= 0, samples + (size_t)h * kPnpModel,
             p3 + 3 * (size_t)pr.off, p2 + 2 * (size_t)pr.off, pr.count, K, thr, good_out + h, &model_out[h].R[0]);
}

namespace {

__device__ void sincos_poly(double x, double* s_out, double* c_out)
{
    const double PIO2_1 = 1.57079632673412561417e+00, PIO2_1T = 6.07710050650619224932e-11;
    const double INV_PIO2 = 6.36619772367581382433e-01;
    const double kd = floor(x * INV_PIO2 + 0.5);
    const long k = (long)kd;
    const double r = (x - kd * PIO2_1) - kd * PIO2_1T;
    const double r2 = r * r;
    double s = -1.0 / 121645100408832000.0;
    s = s * r2 + 1.0 / 355687428096000.0;
    s = s * r2 - 1.0 / 1307674368000.0;
    s = s * r2 + 1.0 / 6227020800.0;
    s = s * r2 - 1.0 / 39916800.0;
    s = s * r2 + 1.0 / 362880.0;
    s = s * r2 - 1.0 / 5040.0;
    s = s * r2 + 1.0 / 120.0;
    s = s * r2 - 1.0 / 6.0;
    s = s * r2 + 1.0;
    const double sr = s * r;
    double c = -1.0 / 6402373705728000.0;
    c = c * r2 + 1.0 / 20922789888000.0;
    c = c * r2 - 1.0 / 87178291200.0;
    c = c * r2 + 1.0 / 479001600.0;
    c = c * r2 - 1.0 / 3628800.0;
    c = c * r2 + 1.0 / 40320.0;
    c = c * r2 - 1.0 / 720.0;
    c = c * r2 + 1.0 / 24.0;
    c = c * r2 - 0.5;
    c = c * r2 + 1.0;
    switch ((int)(k & 3)) {
    case 0: *c_out = c; *s_out = sr; break;
    case 1: *c_out = -sr; *s_out = c; break;
    case 2: *c_out = -c; *s_out = -sr; break;
    default: *c_out = sr; *s_out = -c; break;
    }
}

__device__ void rodrigues_exp(const double w[3], double R[9])
{
    const double th2 = (w[0] * w[0] + w[1] * w[1]) + w[2] * w[2];
    const double th = sqrt(th2);
    if (th < 1e-300) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    double sn, c;
    sincos_poly(th, &sn, &c);
    const double k[3] = {w[0] / th, w[1] / th, w[2] / th};
    const double c1 = 1.0 - c;
    R[0] = c + c1 * k[0] * k[0];         R[1] = c1 * k[0] * k[1] - sn * k[2]; R[2] = c1 * k[0] * k[2] + sn * k[1];
    R[3] = c1 * k[1] * k[0] + sn * k[2]; R[4] = c + c1 * k[1] * k[1];         R[5] = c1 * k[1] * k[2] - sn * k[0];
    R[6] = c1 * k[2] * k[0] - sn * k[1]; R[7] = c1 * k[2] * k[1] + sn * k[0]; R[8] = c + c1 * k[2] * k[2];
}

__device__ __forceinline__ bool solve6(const double* H, const double* g, double x[6])
{
    double A[6][7];
#pragma unroll
    for (int i = 0; i < 6; i++) {
#pragma unroll
        for (int j = 0; j < 6; j++) A[i][j] = H[i * 6 + j];
        A[i][6] = -g[i];
    }
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 6; k++) {
        int p = k;
        double ap = fabs(A[k][k]);
#pragma unroll
        for (int i = k + 1; i < 6; i++)
            if (fabs(A[i][k]) > ap) { p = i; ap = fabs(A[i][k]); }
        // row swap k <-> p with static indices (p is run-time)
#pragma unroll
        for (int i = k + 1; i < 6; i++)
            if (i == p)
#pragma unroll
                for (int j = 0; j < 7; j++) { const double tt = A[k][j]; A[k][j] = A[i][j]; A[i][j] = tt; }
        if (A[k][k] == 0.0) ok = false;
#pragma unroll
        for (int i = k + 1; i < 6; i++) {
            const double f = A[i][k] / A[k][k];
#pragma unroll
            for (int j = k; j < 7; j++) A[i][j] -= f * A[k][j];
        }
    }
    if (!ok) return false;
#pragma unroll
    for (int k = 5; k >= 0; k--) {
        double sacc = A[k][6];
#pragma unroll
        for (int j = k + 1; j < 6; j++) sacc -= A[k][j] * x[j];
        x[k] = sacc / A[k][k];
    }
    return true;
}

// 21 upper-triangle entries of J^T J and 6 of J^T r for one correspondence (left SE(3) increment)
__device__ __forceinline__ void gn_terms(const float* P, const float* uv, const double* R, const double* t,
                                         const PnpCam& K, double out[27])
{
    const double X = ((R[0] * (double)P[0] + R[1] * (double)P[1]) + R[2] * (double)P[2]) + t[0];
    const double Y = ((R[3] * (double)P[0] + R[4] * (double)P[1]) + R[5] * (double)P[2]) + t[1];
    const double Z = ((R[6] * (double)P[0] + R[7] * (double)P[1]) + R[8] * (double)P[2]) + t[2];
    const double iz = 1.0 / Z, iz2 = iz * iz;
    const double ru = (K.fu * X * iz + K.uc) - (double)uv[0];
    const double rv = (K.fv * Y * iz + K.vc) - (double)uv[1];
    const double du[3] = {K.fu * iz, 0.0, -K.fu * X * iz2};
    const double dv[3] = {0.0, K.fv * iz, -K.fv * Y * iz2};
    const double Ju[6] = {Y * du[2] - Z * du[1], Z * du[0] - X * du[2], X * du[1] - Y * du[0], du[0], du[1], du[2]};
    const double Jv[6] = {Y * dv[2] - Z * dv[1], Z * dv[0] - X * dv[2], X * dv[1] - Y * dv[0], dv[0], dv[1], dv[2]};
    int k = 0;
    for (int a = 0; a < 6; a++)
        for (int b = a; b < 6; b++) out[k++] = Ju[a] * Ju[b] + Jv[a] * Jv[b];
    for (int a = 0; a < 6; a++) out[k++] = Ju[a] * ru + Jv[a] * rv;
}

constexpr int kRefineThreads = 256;

struct RefLds {
    int idx[kPnpMaxM];
    double red[27 * 16];
    double sums[27];
    double R[9], t[3];
    int wtot[kRefineThreads / 64];
    int stop;
};

// solvePnPRansac's refinement of one problem by the first 256 threads of the workgroup (threads past them
// only join the barriers): the RANSAC inlier mask of the model R0 = {R[9], t[3]} (all ones when `all`),
// compacted in index order, then 10 Gauss-Newton steps.  The result is left in L.R / L.t (and in out[12]
// when given); mask = the problem's u8 mask row.
__device__ __forceinline__ void refine_eval(RefLds& L, const float* __restrict__ P3, const float* __restrict__ P2,
                                            int count, bool all, const double* R0, const PnpCam& K, float thr,
                                            uint8_t* __restrict__ mask, double* __restrict__ out)
{
    int* idx = L.idx;
    double* red = L.red;
    double* sums = L.sums;
    double* R = L.R;
    double* t = L.t;
    int* wtot = L.wtot;
    int& stop = L.stop;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool on = tid < kRefineThreads;
    REF_PROF(0);
    if (tid < 9) R[tid] = R0[tid];
    if (tid < 3) t[tid] = R0[9 + tid];
    __syncthreads();
    double Rr[9], tr[3];
    for (int i = 0; i < 9; i++) Rr[i] = R[i];
    for (int i = 0; i < 3; i++) tr[i] = t[i];

    // ---- RANSAC inlier mask of the best model, compacted in index order
    int nI = 0;
    for (int base = 0; base < count; base += kRefineThreads) {
        const int i = base + tid;
        bool m = false;
        if (on && i < count) {
            m = all || reproj_err2(P3 + 3 * i, P2 + 2 * i, Rr, tr, K) <= thr;
            mask[i] = m ? 1 : 0;
        }
        const unsigned long long bal = __ballot(m);
        const int below = __popcll(bal & ((1ull << lane) - 1ull));
        if (on && lane == 0) wtot[wave] = __popcll(bal);
        __syncthreads();
        int pre = 0, tot = 0;
        for (int w = 0; w < kRefineThreads / 64; w++) {
            pre += w < wave ? wtot[w] : 0;
            tot += wtot[w];
        }
        if (m) idx[nI + pre + below] = i;
        nI += tot;
        __syncthreads();
    }

    REF_PROF(1);
    // ---- 10 Gauss-Newton steps (oracle orc_pnp_ransac refinement order)
    for (int it = 0; it < 10; it++) {
        double acc[27];
        for (int k = 0; k < 27; k++) acc[k] = 0.0;
        for (int i = tid; on && i < nI; i += kRefineThreads) {
            const int id = idx[i];
            double term[27];
            gn_terms(P3 + 3 * id, P2 + 2 * id, Rr, tr, K, term);
            for (int k = 0; k < 27; k++) acc[k] += term[k];
        }
        REF_PROF(2 + 3 * it);
        // natural-order binary tree over the 256 lanes (oracle order): the 16-lane row trees with
        // DPP row shifts (lane 15 of each row ends with its row's sum), then lanes 0..26 of wave 0
        // add the 16 row sums of one term each
#pragma unroll
        for (int k = 0; k < 27; k++) {
            acc[k] += dpp_row_shr<1>(acc[k]);
            acc[k] += dpp_row_shr<2>(acc[k]);
            acc[k] += dpp_row_shr<4>(acc[k]);
            acc[k] += dpp_row_shr<8>(acc[k]);
        }
        if (on && (lane & 15) == 15)
#pragma unroll
            for (int k = 0; k < 27; k++) red[k * 16 + (tid >> 4)] = acc[k];
        __syncthreads();
        if (tid < 27) {
            double r[16];
#pragma unroll
            for (int i = 0; i < 16; i++) r[i] = red[tid * 16 + i];
#pragma unroll
            for (int s2 = 1; s2 < 16; s2 <<= 1)
#pragma unroll
                for (int i = 0; i < 16; i += 2 * s2) r[i] += r[i + s2];
            sums[tid] = r[0];
        }
        __syncthreads();
        REF_PROF(3 + 3 * it);
        if (tid == 0) {
            double Hm[36], g[6], dx[6];
            int k = 0;
            for (int a = 0; a < 6; a++)
                for (int b = a; b < 6; b++) {
                    Hm[a * 6 + b] = sums[k];
                    Hm[b * 6 + a] = sums[k];
                    k++;
                }
            for (int a = 0; a < 6; a++) g[a] = sums[k++];
            stop = solve6(Hm, g, dx) ? 0 : 1;
            if (!stop) {
                double dR[9], Rn[9], tn[3];
                rodrigues_exp(dx, dR);
                for (int a = 0; a < 3; a++) {
                    for (int b = 0; b < 3; b++)
                        Rn[a * 3 + b] = (dR[a * 3 + 0] * R[0 * 3 + b] + dR[a * 3 + 1] * R[1 * 3 + b]) + dR[a * 3 + 2] * R[2 * 3 + b];
                    tn[a] = ((dR[a * 3 + 0] * t[0] + dR[a * 3 + 1] * t[1]) + dR[a * 3 + 2] * t[2]) + dx[3 + a];
                }
                for (int i = 0; i < 9; i++) R[i] = Rn[i];
                for (int i = 0; i < 3; i++) t[i] = tn[i];
            }
        }
        __syncthreads();
        REF_PROF(4 + 3 * it);
        if (stop) break;
        for (int i = 0; i < 9; i++) Rr[i] = R[i];
        for (int i = 0; i < 3; i++) tr[i] = t[i];
    }
    if (out && tid < 12) out[tid] = tid < 9 ? R[tid] : t[tid - 9];
}

}  // namespace

__global__ __launch_bounds__(kRefineThreads) void k_pnp_refine(
    const float* __restrict__ p3, const float* __restrict__ p2, const PnpProbDev* __restrict__ probs,
    const int* __restrict__ best, const int* __restrict__ force_all, const PnpModel* __restrict__ models, PnpCam K,
    float thr, uint8_t* __restrict__ mask, PnpModel* __restrict__ out)
{
    __shared__ RefLds L;
    const int p = blockIdx.x;
    const int bh = best[p];
    if (bh < 0) return;   // uniform
    const PnpProbDev pr = probs[p];
    refine_eval(L, p3 + 3 * (size_t)pr.off, p2 + 2 * (size_t)pr.off, pr.count, force_all[p] != 0, &models[bh].R[0], K,
                thr, mask + pr.off, &out[p].R[0]);
}

// ------------------------------------------------------------------ match filter + 3D-2D gather
constexpr int kGatherThreads = 1024;
constexpr int kMaxTrain = 8192;

// Matcher::match (Features/Matcher.cpp:106-139) of one pair from its knn-2 rows kr, fused with the PnP
// 3D-2D gather, by the NT threads of the workgroup: P3 = the query frame's xyz (zq), P2 = the train frame's
// undistorted pixels (kun_t), mq / mt = the kept (queryIdx, trainIdx), in query order.  fq = the query
// frame's outlier flags (discardOutliers = true) or nullptr.  Returns the kept count (uniform).
template <int NT>
__device__ __forceinline__ int gather_eval(int* winner, int* wtot, const int4* __restrict__ kr, int nq, int nt,
                                           const float* __restrict__ zq, const float* __restrict__ zt,
                                           const float* __restrict__ kun_t, const uint8_t* __restrict__ fq,
                                           float nnratio, float* __restrict__ P3, float* __restrict__ P2,
                                           int* __restrict__ mq, int* __restrict__ mt)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < nt && i < kMaxTrain; i += NT) winner[i] = INT_MAX;
    __syncthreads();
    // candidate = ratio test passed and both depths valid (Features/Matcher.cpp:118-131; the
    // "train index already used" test only ever sees earlier candidates, so the kept match of a
    // train index is its lowest-index candidate query)
    auto candidate = [&](int i, int* i2o) -> bool {
        const int4 r = kr[i];
        if (r.w < 0) return false;   // fewer than 2 train rows: skipped (reference UB)
        const float d1 = (float)r.x, d2 = (float)r.z;
        if (!(d1 < nnratio * d2)) return false;
        if (fq && fq[i]) return false;   // ref->isOutlier(i1) (:125-128), before the train index is taken
        if (!(zq[3 * i + 2] > 0) || !(zt[3 * r.y + 2] > 0)) return false;
        *i2o = r.y;
        return true;
    };
    if (nq > 0 && nt > 0) {
        for (int i = tid; i < nq; i += NT) {
            int i2;
            if (candidate(i, &i2)) atomicMin(&winner[i2], i);
        }
    }
    __syncthreads();
    int m = 0;
    const int nql = (nq > 0 && nt > 0) ? nq : 0;
    for (int base = 0; base < nql; base += NT) {
        const int i = base + tid;
        int i2 = -1;
        const bool keep = i < nql && candidate(i, &i2) && winner[i2] == i;
        const unsigned long long bal = __ballot(keep);
        const int below = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wtot[wave] = __popcll(bal);
        __syncthreads();
        int pre = 0, tot = 0;
        for (int w = 0; w < NT / 64; w++) {
            pre += w < wave ? wtot[w] : 0;
            tot += wtot[w];
        }
        if (keep) {
            const int o = m + pre + below;
            const float* X = zq + 3 * i;
            const float* U = kun_t + 7 * i2;
            P3[3 * o] = X[0];
            P3[3 * o + 1] = X[1];
            P3[3 * o + 2] = X[2];
            P2[2 * o] = U[0];
            P2[2 * o + 1] = U[1];
            mq[o] = i;
            mt[o] = i2;
        }
        m += tot;
        __syncthreads();
    }
    return m;
}

// gather_eval for a workgroup that holds every query of the pair in registers (nq <= NT * QM): each
// query's loads issued together for the thread's QM queries (the knn-2 row, the flag, both depths, and
// the kept match's 3D point and pixel ahead of the winner test), the candidate test evaluated once, and
// the kept matches compacted in query order by one block-wide scan.  Same results as gather_eval.
template <int NT, int QM>
__device__ __forceinline__ int gather_regs(int* winner, int* wtot, const int4* __restrict__ kr, int nq, int nt,
                                           const float* __restrict__ zq, const float* __restrict__ zt,
                                           const float* __restrict__ kun_t, const uint8_t* __restrict__ fq,
                                           float nnratio, float* __restrict__ P3, float* __restrict__ P2,
                                           int* __restrict__ mq, int* __restrict__ mt, float* LP3 = nullptr,
                                           float* LP2 = nullptr)
{
    constexpr int NW = NT / 64;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    for (int i = tid; i < nt && i < kMaxTrain; i += NT) winner[i] = INT_MAX;
    const bool live = nq > 0 && nt > 0;
    int4 r[QM];
#pragma unroll
    for (int u = 0; u < QM; u++) {
        const int i = tid + u * NT;
        r[u] = (live && i < nq) ? kr[i] : make_int4(0, -1, 0, -1);
    }
    bool cand[QM];
    float X[QM][3], U[QM][2];
#pragma unroll
    for (int u = 0; u < QM; u++) {
        const int i = tid + u * NT;
        const bool pre = r[u].w >= 0 && r[u].y >= 0;
        const bool fl = (fq && pre) ? fq[i] != 0 : false;
#pragma unroll
        for (int j = 0; j < 3; j++) X[u][j] = pre ? zq[3 * i + j] : 0.0f;
        const float ztv = pre ? zt[3 * r[u].y + 2] : 0.0f;
        U[u][0] = pre ? kun_t[7 * r[u].y] : 0.0f;
        U[u][1] = pre ? kun_t[7 * r[u].y + 1] : 0.0f;
        // Matcher.cpp:118-131: ratio test, ref->isOutlier(i1) (:125-128), both depths valid
        const float d1 = (float)r[u].x, d2 = (float)r[u].z;
        cand[u] = pre && (d1 < nnratio * d2) && !fl && (X[u][2] > 0) && (ztv > 0);
    }
    __syncthreads();   // winner initialised
#pragma unroll
    for (int u = 0; u < QM; u++)
        if (cand[u]) atomicMin(&winner[r[u].y], tid + u * NT);
    __syncthreads();
    bool keep[QM];
    int below[QM];
#pragma unroll
    for (int u = 0; u < QM; u++) {
        keep[u] = cand[u] && winner[r[u].y] == tid + u * NT;
        const unsigned long long bal = __ballot(keep[u]);
        below[u] = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wtot[u * NW + wave] = __popcll(bal);
    }
    __syncthreads();
    int m = 0, pre_u[QM];
#pragma unroll
    for (int u = 0; u < QM; u++) {
        int pre = m;
#pragma unroll
        for (int w = 0; w < NW; w++) {
            const int c = wtot[u * NW + w];
            pre += w < wave ? c : 0;
            m += c;
        }
        pre_u[u] = pre + below[u];
    }
#pragma unroll
    for (int u = 0; u < QM; u++) {
        if (!keep[u]) continue;
        const int o = pre_u[u];
        P3[3 * o] = X[u][0];
        P3[3 * o + 1] = X[u][1];
        P3[3 * o + 2] = X[u][2];
        P2[2 * o] = U[u][0];
        P2[2 * o + 1] = U[u][1];
        mq[o] = tid + u * NT;
        mt[o] = r[u].y;
        if (LP3) {
            LP3[3 * o] = X[u][0];
            LP3[3 * o + 1] = X[u][1];
            LP3[3 * o + 2] = X[u][2];
            LP2[2 * o] = U[u][0];
            LP2[2 * o + 1] = U[u][1];
        }
    }
    return m;
}

__global__ __launch_bounds__(kGatherThreads) void k_match_gather(
    const int4* __restrict__ knn, const int* __restrict__ counts, const int* __restrict__ qf,
    const int* __restrict__ tf, const float* __restrict__ xyz, const float* __restrict__ kun, int kp_cap,
    float nnratio, float* __restrict__ p3, float* __restrict__ p2, PnpProbDev* __restrict__ probs,
    int* __restrict__ mq, int* __restrict__ mt, const uint8_t* __restrict__ qflags, const int* __restrict__ krow)
{
    __shared__ int winner[kMaxTrain];
    __shared__ int wtot[kGatherThreads / 64];
    const int p = blockIdx.x;
    const int rf = qf[p], cf = tf[p];
    const size_t po = (size_t)p * kp_cap;
    const int m = gather_eval<kGatherThreads>(
        winner, wtot, knn + (size_t)(krow ? krow[p] : p) * kp_cap, counts[rf], counts[cf], xyz + (size_t)rf * kp_cap * 3,
        xyz + (size_t)cf * kp_cap * 3, kun + (size_t)cf * kp_cap * 7, qflags ? qflags + (size_t)rf * kp_cap : nullptr,
        nnratio, p3 + 3 * po, p2 + 2 * po, mq + po, mt + po);
    if (threadIdx.x == 0) probs[p] = PnpProbDev{(int)po, m};
}

// ------------------------------------------------------------------ device sampling and replay
namespace {

struct CvRngDev {   // cv::RNG multiply-with-carry
    uint64_t state;
    __device__ unsigned next()
    {
        state = (uint64_t)(unsigned)state * 4164903690u + (unsigned)(state >> 32);
        return (unsigned)state;
    }
    __device__ int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + a); }
};

// oracle log_det: + - * / and exact frexp only
__device__ double log_det(double x)
{
    int e = 0;
    double m = frexp(x, &e);
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

// oracle update_num_iters (RANSACUpdateNumIters, portable log / power)
__device__ int update_num_iters(double p, double ep, int modelPoints, int maxIters)
{
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    const double DBLMIN = 2.2250738585072014e-308;
    double num = 1. - p > DBLMIN ? 1. - p : DBLMIN;
    const double q = 1. - ep;
    double qm = 1.0;
    for (int i = 0; i < modelPoints; i++) qm = qm * q;
    double denom = 1. - qm;
    if (denom < DBLMIN) return 0;
    num = log_det(num);
    denom = log_det(denom);
    return denom >= 0 || -num >= maxIters * (-denom) ? maxIters : (int)rint(num / denom);
}

}  // namespace

__global__ void k_pnp_sample(const PnpProbDev* __restrict__ probs, int P, PnpPrm prm, int* __restrict__ samples,
                             int* __restrict__ hyp_prob, PnpRep* __restrict__ rep)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const int count = probs[p].count;
    const int K0 = prm.chunk;
    const int minc = prm.min_matches > kPnpModel ? prm.min_matches : kPnpModel;
    PnpRep r{};
    r.best = -1;
    r.count = count;
    CvRngDev rng{~0ull};
    int nh = 0;
    if (count >= minc) {
        if (count == kPnpModel) {
            r.force_all = 1;
            nh = 1;
            for (int j = 0; j < kPnpModel; j++) samples[(size_t)p * K0 * kPnpModel + j] = j;
        } else {
            const int iters = prm.iterations > 1 ? prm.iterations : 1;
            nh = K0 < iters ? K0 : iters;
            for (int i = 0; i < nh; i++) {
                // the subset lives in registers while it is drawn (the duplicate test reads it)
                int cur[kPnpModel];
#pragma unroll
                for (int k = 0; k < kPnpModel; k++) {
                    for (;;) {
                        const int v = rng.uniform(0, count);
                        bool dup = false;
#pragma unroll
                        for (int j = 0; j < k; j++) dup |= cur[j] == v;
                        if (!dup) { cur[k] = v; break; }
                    }
                }
                int* idx = samples + ((size_t)p * K0 + i) * kPnpModel;
#pragma unroll
                for (int k = 0; k < kPnpModel; k++) idx[k] = cur[k];
            }
        }
    }
    for (int i = 0; i < K0; i++) hyp_prob[(size_t)p * K0 + i] = i < nh ? p : -1;
    r.nh = nh;
    r.rng = rng.state;
    rep[p] = r;
}

__global__ void k_pnp_replay(const int* __restrict__ good, int P, PnpPrm prm, PnpRep* __restrict__ rep,
                             int* __restrict__ best)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    PnpRep r = rep[p];
    const int base = p * prm.chunk;
    r.maxGood = 0;
    r.iter = 0;
    r.best = -1;
    if (r.nh == 0) {
        r.niters = 0;
        r.done = 1;
    } else if (r.force_all) {   // runKernel once, every point an inlier, no RANSAC loop
        const int g = good[base];
        if (g >= 0) {
            r.maxGood = r.count;
            r.best = base;
        }
        r.niters = 0;
        r.done = 1;
    } else {
        r.niters = prm.iterations > 1 ? prm.iterations : 1;
        while (r.iter < r.niters && r.iter < r.nh) {
            const int g = good[base + r.iter];
            if (g >= 0 && g > (r.maxGood > kPnpModel - 1 ? r.maxGood : kPnpModel - 1)) {
                r.maxGood = g;
                r.best = base + r.iter;
                r.niters = update_num_iters(prm.confidence, (double)(r.count - g) / r.count, kPnpModel, r.niters);
            }
            r.iter++;
        }
        r.done = r.iter >= r.niters ? 1 : 0;
    }
    rep[p] = r;
    best[p] = (r.done && r.best >= 0 && r.maxGood > 0) ? r.best : -1;
    best[P + p] = r.force_all;
}

// the second chunk's subsets, continuing each unfinished problem's cv::RNG stream (getSubset as k_pnp_sample)
__global__ void k_pnp_sample2(int P, PnpPrm prm, int* __restrict__ samples, int* __restrict__ hyp_prob,
                              PnpRep* __restrict__ rep)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    PnpRep r = rep[p];
    const int K1 = prm.chunk2;
    int k = 0;
    if (!r.done && !r.force_all && r.nh > 0) {   // the replay consumed every drawn subset: iter == nh < niters
        k = r.niters - r.nh;
        k = k < K1 ? k : K1;
        CvRngDev rng{r.rng};
        for (int i = 0; i < k; i++) {
            int cur[kPnpModel];
#pragma unroll
            for (int q = 0; q < kPnpModel; q++) {
                for (;;) {
                    const int v = rng.uniform(0, r.count);
                    bool dup = false;
#pragma unroll
                    for (int j = 0; j < q; j++) dup |= cur[j] == v;
                    if (!dup) { cur[q] = v; break; }
                }
            }
            int* idx = samples + ((size_t)p * K1 + i) * kPnpModel;
#pragma unroll
            for (int q = 0; q < kPnpModel; q++) idx[q] = cur[q];
        }
        r.rng = rng.state;
    }
    for (int i = 0; i < K1; i++) hyp_prob[(size_t)p * K1 + i] = i < k ? p : -1;
    r.nh2 = k;
    rep[p] = r;
}

// the replay over the second chunk (slots h01 + p * chunk2 + i), from the state k_pnp_replay left
__global__ void k_pnp_replay2(const int* __restrict__ good, int h01, int P, PnpPrm prm, PnpRep* __restrict__ rep,
                              int* __restrict__ best)
{
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    PnpRep r = rep[p];
    if (r.nh2 > 0) {
        const int base = h01 + p * prm.chunk2, e0 = r.nh;
        r.nh += r.nh2;
        while (r.iter < r.niters && r.iter < r.nh) {
            const int g = good[base + r.iter - e0];
            if (g >= 0 && g > (r.maxGood > kPnpModel - 1 ? r.maxGood : kPnpModel - 1)) {
                r.maxGood = g;
                r.best = base + r.iter - e0;
                r.niters = update_num_iters(prm.confidence, (double)(r.count - g) / r.count, kPnpModel, r.niters);
            }
            r.iter++;
        }
        r.done = r.iter >= r.niters ? 1 : 0;
        r.nh2 = 0;
    }
    rep[p] = r;
    best[p] = (r.done && r.best >= 0 && r.maxGood > 0) ? r.best : -1;
}

hipError_t launch_pnp_sample2(int P, const PnpPrm& prm, int* samples, int* hyp_prob, PnpRep* rep, hipStream_t st)
{
    if (P <= 0) return hipSuccess;
    return dispatch(k_pnp_sample2, dim3((P + 63) / 64), dim3(64), 0, st, P, prm, samples, hyp_prob, rep);
}

hipError_t launch_pnp_replay2(const int* good, int h01, int P, const PnpPrm& prm, PnpRep* rep, int* best, hipStream_t st)
{
    if (P <= 0) return hipSuccess;
    return dispatch(k_pnp_replay2, dim3((P + 63) / 64), dim3(64), 0, st, good, h01, P, prm, rep, best);
}

hipError_t launch_pnp_sample(const PnpProbDev* probs, int P, const PnpPrm& prm, int* samples, int* hyp_prob, PnpRep* rep,
                       hipStream_t st)
{
    if (P <= 0) return hipSuccess;
    return dispatch(k_pnp_sample, dim3((P + 63) / 64), dim3(64), 0, st, probs, P, prm, samples, hyp_prob, rep);
}

hipError_t launch_pnp_replay(const int* good, int P, const PnpPrm& prm, PnpRep* rep, int* best, hipStream_t st)
{
    if (P <= 0) return hipSuccess;
    return dispatch(k_pnp_replay, dim3((P + 63) / 64), dim3(64), 0, st, good, P, prm, rep, best);
}

hipError_t launch_pnp_hyp(const float* p3, const float* p2, const PnpProbDev* probs, const int* hyp_prob,
                    const int* samples, const PnpCam& cam, float thr, int H, int* good, PnpModel* models,
                    hipStream_t st)
{
    if (H <= 0) return hipSuccess;
    return dispatch(k_pnp_hyp, dim3((H + kGroupsPerWave - 1) / kGroupsPerWave), dim3(64), 0, st, p3, p2, probs, hyp_prob, samples, cam, thr, H, good,
                       models);
}

#ifdef RGBD_PNP_PROFILE
}  // namespace rgbd
#include <cstdio>
namespace rgbd {
void pnp_prof_dump(int H, hipStream_t st)
{
    static long long buf[8192 * 10];
    const int n = H < 8192 ? H : 8192;
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(buf, HIP_SYMBOL(g_pnp_prof), sizeof(long long) * 10 * n);
    double acc[10] = {0};
    for (int h = 0; h < n; h++) {
        const long long* b = buf + h * 10;
        acc[1] += b[1] - b[0]; acc[2] += b[2] - b[1]; acc[8] += b[8] - b[2]; acc[3] += b[3] - b[8];
        acc[4] += b[4] - b[3]; acc[5] += b[5] - b[4]; acc[6] += b[6] - b[5]; acc[7] += b[7] - b[6];
        acc[9] += b[9];
    }
    static long long rb[64 * 48];
    (void)hipMemcpyFromSymbol(rb, HIP_SYMBOL(g_ref_prof), sizeof(rb));
    double gn = 0, red = 0, sol = 0;
    for (int it = 0; it < 10; it++) {
        gn += rb[2 + 3 * it] - (it ? rb[1 + 3 * it] : rb[1]);
        red += rb[3 + 3 * it] - rb[2 + 3 * it];
        sol += rb[4 + 3 * it] - rb[3 + 3 * it];
    }
    fprintf(stderr, "[ref_prof] problem 0: mask+compact %lld  10 its: terms %.0f reduce %.0f solve %.0f  total %lld\n",
            rb[1] - rb[0], gn, red, sol, rb[31] - rb[0]);
    fprintf(stderr, "[pnp_prof] H=%d mean cycles: stageA %.0f MtM %.0f jacobi %.0f (sweeps %.2f) sort %.0f L %.0f cand %.0f sel %.0f score %.0f\n",
            n, acc[1] / n, acc[2] / n, acc[8] / n, acc[9] / n, acc[3] / n, acc[4] / n, acc[5] / n, acc[6] / n, acc[7] / n);
}
#endif

hipError_t launch_pnp_refine(const float* p3, const float* p2, const PnpProbDev* probs, const int* best,
                       const int* force_all, const PnpModel* models, const PnpCam& cam, float thr, int P,
                       uint8_t* mask, PnpModel* out, hipStream_t st)
{
    if (P <= 0) return hipSuccess;
    return dispatch(k_pnp_refine, dim3(P), dim3(kRefineThreads), 0, st, p3, p2, probs, best, force_all, models,
                       cam, thr, mask, out);
}

hipError_t launch_match_gather(const int4* knn, const int* counts, const int* qf, const int* tf, const float* xyz,
                         const float* kun, int kp_cap, float nnratio, int npairs, float* p3, float* p2,
                         PnpProbDev* probs, int* mq, int* mt, hipStream_t st, const uint8_t* qflags, const int* krow)
{
    if (npairs <= 0) return hipSuccess;
    return dispatch(k_match_gather, dim3(npairs), dim3(kGatherThreads), 0, st, knn, counts, qf, tf, xyz, kun,
                       kp_cap, nnratio, p3, p2, probs, mq, mt, qflags, krow);
}

// ------------------------------------------------------------------ the outlier-flag chain, one run per workgroup
// Every stage of a pair on the chain's critical path (gather, subsets, hypotheses, replay, the RANSAC inlier
// mask, flags) runs inside one workgroup per run, with the device functions the batched kernels use, so a
// run's pairs follow each other with no launch or host round trip between them.  The Gauss-Newton
// refinement is off that path (the flags read the RANSAC mask and ok, never the refined pose), so every
// pair's refinement runs afterwards in one k_pnp_refine launch over the whole batch.  Four waves:
// three 21-lane groups per wave in the block layout of the Jacobi (BlkTab: a hypothesis's EPnP, the pair's
// critical path, about twice as fast as in k_pnp_hyp's five 12-lane groups), 12 hypotheses per pass (the
// synthetic fr1 chain needs 3-15 RANSAC iterations per pair: ~1.04 passes per pair).
constexpr int kChainThreads = kRefineThreads;
constexpr int kChainHyp = (kChainThreads / 64) * kBlkGroupsPerWave;
constexpr int kChainRaw = 512;   // raw RNG outputs kept in LDS
constexpr int kChainGQ = 8;      // queries per thread held in registers by the chain's gather (nq <= 2048)
static_assert(kChainThreads == 256, "the refinement's reduction tree is over 256 lanes");

#ifdef RGBD_PNP_PROFILE
// workgroup 0 (the first run): per-stage wall-clock sums (100 MHz ticks) over its pairs, pairs, passes
__device__ long long g_chain_prof[10];
#define CHAIN_T(v) long long v = 0; if (threadIdx.x == 0 && blockIdx.x == 0) v = wall_clock64()
#define CHAIN_ADD(k, t0, t1) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_chain_prof[(k)] += (t1) - (t0); } while (0)
#define CHAIN_CNT(k) do { if (threadIdx.x == 0 && blockIdx.x == 0) g_chain_prof[(k)] += 1; } while (0)
#else
#define CHAIN_T(v) do { } while (0)
#define CHAIN_ADD(k, t0, t1) do { } while (0)
#define CHAIN_CNT(k) do { } while (0)
#endif

namespace {
struct ChainLds {
    union {
        struct { int winner[kMaxTrain]; int wtot[kChainGQ * (kChainThreads / 64)]; } g;
        struct { HypLds sh[kChainThreads / 64][kBlkGroupsPerWave]; double2 cs[kChainThreads / 64][kBlkGroupsPerWave][12]; } h;
    } u;
    int samples[kChainHyp * kPnpModel];
    int good[kChainHyp];
    PnpModel models[kChainHyp];
    double best[12];
    alignas(8) unsigned short vals[kChainThreads];   // raw RNG outputs pos0 .. pos0 + 255 mod count (a pass's draws)
    uint32_t raw[kChainRaw];                          // the first raw outputs (the same stream for every pair)
    uint4 blk_off[11 * kBlkGroup];                    // BlkTab's element offsets (per round, lane)
    int k, ok, pos;
};
}  // namespace

// Every pair's points are also staged in LDS (dynamic, 20 B per kp_cap slot), where the hypotheses' samples,
// their inlier counts and the RANSAC mask read them (kp_cap <= kPnpMaxM = 4096: <= 80 KB beside ChainLds)
__global__ __launch_bounds__(kChainThreads, 1) void k_pnp_chain(
    const int4* __restrict__ knn, const int* __restrict__ counts, const float* __restrict__ xyz,
    const float* __restrict__ kun, int kp_cap, float nnratio, const int* __restrict__ seg, PnpCam K, float thr,
    PnpPrm prm, float* __restrict__ p3, float* __restrict__ p2, int* __restrict__ mq, int* __restrict__ mt,
    uint8_t* __restrict__ mask, uint8_t* __restrict__ flags, PnpChainRes* __restrict__ res,
    const uint32_t* __restrict__ rngtab, int ntab, unsigned long long rng_end, PnpProbDev* __restrict__ probs,
    int* __restrict__ best, PnpModel* __restrict__ models, int P)
{
    __shared__ ChainLds L;
    extern __shared__ __align__(16) float chain_pts[];   // [3 kp_cap] xyz, [2 kp_cap] uv
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int s = blockIdx.x;
    const int pa = seg[s], pb = seg[s + 1];
    float* const LP3 = chain_pts;
    float* const LP2 = chain_pts + 3 * kp_cap;
    // this lane's hypothesis group (k_pnp_hyp's layout) and its slot in a pass
    const int grp = lane / kBlkGroup < kBlkGroupsPerWave ? lane / kBlkGroup : kBlkGroupsPerWave - 1;
    const bool live = lane < kBlkGroupsPerWave * kBlkGroup;
    const int g = live ? lane - grp * kBlkGroup : 0;
    const int hs = wave * kBlkGroupsPerWave + grp;
    const int minc = prm.min_matches > kPnpModel ? prm.min_matches : kPnpModel;
    for (int j = tid; j < kChainRaw; j += kChainThreads) L.raw[j] = j < ntab ? rngtab[j] : 0u;
    for (int j = tid; j < 11 * kBlkGroup; j += kChainThreads)
        L.blk_off[j] = *reinterpret_cast<const uint4*>(&kBlkTab.o[j / kBlkGroup][j % kBlkGroup][0]);
    for (int p = pa; p < pb; p++) {
        const int rf = p, cf = p + 1;
        const size_t po = (size_t)p * kp_cap;   // the pair's points, kept for the refinement
        float* P3 = p3 + 3 * po;
        float* P2 = p2 + 2 * po;
        int* MQ = mq + po;
        int* MT = mt + po;
        uint8_t* MK = mask + po;
        CHAIN_T(t0);
        // Matcher::match(ref = frame p, cur = frame p + 1, discardOutliers = true) + the 3D-2D gather
        const int nq = counts[rf], nt = counts[cf];
        const int count = nq <= kChainGQ * kChainThreads
            ? gather_regs<kChainThreads, kChainGQ>(L.u.g.winner, L.u.g.wtot, knn + (size_t)p * kp_cap, nq, nt,
                                                   xyz + (size_t)rf * kp_cap * 3, xyz + (size_t)cf * kp_cap * 3,
                                                   kun + (size_t)cf * kp_cap * 7, flags + (size_t)rf * kp_cap, nnratio,
                                                   P3, P2, MQ, MT, LP3, LP2)
            : gather_eval<kChainThreads>(L.u.g.winner, L.u.g.wtot, knn + (size_t)p * kp_cap, nq, nt,
                                         xyz + (size_t)rf * kp_cap * 3, xyz + (size_t)cf * kp_cap * 3,
                                         kun + (size_t)cf * kp_cap * 7, flags + (size_t)rf * kp_cap, nnratio, P3, P2,
                                         MQ, MT);
        if (nq > kChainGQ * kChainThreads) {   // the loop form wrote HBM only
            __syncthreads();
            for (int i = tid; i < count; i += kChainThreads) {
#pragma unroll
                for (int j = 0; j < 3; j++) LP3[3 * i + j] = P3[3 * i + j];
#pragma unroll
                for (int j = 0; j < 2; j++) LP2[2 * i + j] = P2[2 * i + j];
            }
        }
        __syncthreads();
        const float* const Q3 = LP3;   // the solve reads the points from LDS
        const float* const Q2 = LP2;
        CHAIN_T(t1);
        CHAIN_ADD(0, t0, t1);
        CHAIN_CNT(8);
        // solvePnPRansac: thread 0 keeps the RANSACPointSetRegistrator::run state (k_pnp_sample / k_pnp_replay
        // and the host continuation, one pass of up to 20 iterations at a time)
        const bool force = count == kPnpModel && count >= minc;   // runKernel once, every point an inlier
        // the cv::RNG((uint64)-1) stream of every call is the same: rngtab[j] = its (j + 1)-th raw output (host
        // table), rng_end = the state after the table (draws past it continue sequentially on wave 0)
        CvRngDev rng{rng_end};
        int maxGood = 0, iter = 0, ev = 0, have = 0, pos = 0;
        int niters = count >= minc ? (force ? 1 : (prm.iterations > 1 ? prm.iterations : 1)) : 0;
        if (tid == 0) L.pos = 0;
        __syncthreads();
        for (;;) {
            CHAIN_T(a0);
            {   // uniform(0, count) of the next 256 raw outputs, one per thread
                const int j = L.pos + tid;
                const uint32_t rv = j < kChainRaw ? L.raw[j] : (j < ntab ? rngtab[j] : 0u);
                L.vals[tid] = (unsigned short)(j < ntab && count > 0 ? rv % (unsigned)count : 0u);
            }
            __syncthreads();
            // wave 0 keeps the RANSACPointSetRegistrator::run state (every lane the same values)
            if (wave == 0) {
                int k = iter < niters ? niters - ev : 0;
                k = k < kChainHyp ? k : kChainHyp;
                if (force) {
                    if (lane < kPnpModel) L.samples[lane] = lane;
                } else {
                    // getSubset: 5 distinct indices per iteration, a repeated index redrawn.  The subsets
                    // that need no redraw are formed side by side (lane j takes the 5 values after the j
                    // subsets before it); the first subset with a repeated value, and any value past the
                    // pass's window or the table, by the sequential rule
                    const int p0 = pos;
                    int I = 0, o = 0;
                    while (I < k) {
                        const int rem = k - I;
                        if (o + kPnpModel * rem <= kChainThreads && p0 + o + kPnpModel * rem <= ntab) {
                            const bool on = lane < rem;
                            const int b0 = o + kPnpModel * (on ? lane : 0);
                            int cv[kPnpModel];
#pragma unroll
                            for (int q = 0; q < kPnpModel; q++) cv[q] = L.vals[b0 + q];
                            bool dup = false;
#pragma unroll
                            for (int q = 1; q < kPnpModel; q++)
#pragma unroll
                                for (int j = 0; j < q; j++) dup |= cv[j] == cv[q];
                            const unsigned long long bad = __ballot(on && dup);
                            const int f = bad ? __ffsll((long long)bad) - 1 : rem;
                            if (on && lane < f)
#pragma unroll
                                for (int q = 0; q < kPnpModel; q++) L.samples[(I + lane) * kPnpModel + q] = cv[q];
                            I += f;
                            o += kPnpModel * f;
                            if (I == k) break;
                        }
                        int cur[kPnpModel];
#pragma unroll
                        for (int q = 0; q < kPnpModel; q++) {
                            for (;;) {
                                const int at = p0 + o;
                                int v;
                                if (at < ntab)
                                    v = o < kChainThreads ? (int)L.vals[o] : (int)(rngtab[at] % (unsigned)count);
                                else
                                    v = (int)(rng.next() % (unsigned)count);
                                o++;
                                bool dup = false;
#pragma unroll
                                for (int j = 0; j < q; j++) dup |= cur[j] == v;
                                if (!dup) { cur[q] = v; break; }
                            }
                        }
                        if (lane == 0)
#pragma unroll
                            for (int q = 0; q < kPnpModel; q++) L.samples[I * kPnpModel + q] = cur[q];
                        I++;
                    }
                    pos = p0 + o;
                    if (lane == 0) L.pos = pos;
                }
                if (lane == 0) L.k = k;
            }
            __syncthreads();
            CHAIN_T(a1);
            CHAIN_ADD(1, a0, a1);
            const int kk = L.k;
            if (kk <= 0) break;   // uniform
            CHAIN_CNT(9);
            hyp_eval<kBlkGroup>(L.u.h.sh[wave][grp], L.u.h.cs[wave][grp], L.blk_off, g, grp * kBlkGroup, live, live && hs < kk, hs < kk,
                     L.samples + hs * kPnpModel, Q3, Q2, count, K, thr, &L.good[hs], &L.models[hs].R[0]);
            __syncthreads();
            CHAIN_T(a2);
            CHAIN_ADD(2, a1, a2);
            if (wave == 0) {   // the sequential replay of this pass (accept, RANSACUpdateNumIters)
                const int e0 = ev;
                ev += kk;
                if (force) {
                    if (L.good[0] >= 0) {
                        maxGood = count;
                        have = 1;
                        if (lane < 12) L.best[lane] = (&L.models[0].R[0])[lane];
                    }
                    niters = 0;
                } else {
                    while (iter < niters && iter < ev) {
                        const int gd = L.good[iter - e0];
                        if (gd >= 0 && gd > (maxGood > kPnpModel - 1 ? maxGood : kPnpModel - 1)) {
                            maxGood = gd;
                            have = 1;
                            if (lane < 12) L.best[lane] = (&L.models[iter - e0].R[0])[lane];
                            niters = update_num_iters(prm.confidence, (double)(count - gd) / count, kPnpModel, niters);
                        }
                        iter++;
                    }
                }
            }
            CHAIN_T(a3);
            CHAIN_ADD(3, a2, a3);
        }
        if (tid == 0) L.ok = have && maxGood > 0;
        __syncthreads();
        const bool ok = L.ok != 0;
        CHAIN_T(t2);
        // the RANSAC inlier mask of the best model (k_pnp_refine's first stage; every point when force)
        if (ok) {
            double Rb[9], tb[3];
#pragma unroll
            for (int j = 0; j < 9; j++) Rb[j] = L.best[j];
#pragma unroll
            for (int j = 0; j < 3; j++) tb[j] = L.best[9 + j];
            for (int i = tid; i < count; i += kChainThreads)
                MK[i] = (force || reproj_err2(Q3 + 3 * i, Q2 + 2 * i, Rb, tb, K) <= thr) ? 1 : 0;
        }
        if (tid == 0) {
            PnpChainRes r{};
            r.count = count;
            r.ok = ok ? 1 : 0;
            r.n_inliers = ok ? maxGood : 0;
            r.iters = iter;
            res[p] = r;
            probs[p] = PnpProbDev{(int)po, count};
            best[p] = ok ? p : -1;   // k_pnp_refine's inputs
            best[P + p] = force ? 1 : 0;
        }
        if (ok && tid < 12) (&models[p].R[0])[tid] = L.best[tid];
        __syncthreads();   // the mask is read across threads below
        CHAIN_T(t3);
        CHAIN_ADD(4, t2, t3);
        // PnPRansac::compute's flag writes on frame p + 1 (read by the run's next pair)
        if (p + 1 < pb && count >= prm.min_matches) {
            uint8_t* f = flags + (size_t)cf * kp_cap;
            for (int o = tid; o < count; o += kChainThreads) f[MT[o]] = (ok && MK[o]) ? 0 : 1;
        }
        __threadfence_block();
        __syncthreads();
        CHAIN_T(t4);
        CHAIN_ADD(5, t3, t4);
        CHAIN_ADD(6, t0, t4);
    }
}

#ifdef RGBD_PNP_PROFILE
}  // namespace rgbd
#include <cstdio>
namespace rgbd {
void chain_prof_dump(hipStream_t st)
{
    long long b[10];
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(b, HIP_SYMBOL(g_chain_prof), sizeof(b));
    const double n = b[8] > 0 ? (double)b[8] : 1.0, us = 0.01;   // 100 MHz ticks
    fprintf(stderr, "[chain_prof] run 0: %lld pairs, %.2f passes/pair; us per pair: gather %.2f subsets %.2f "
            "hypotheses %.2f replay %.2f mask %.2f result+flags %.2f total %.2f\n", b[8], b[9] / n, b[0] * us / n,
            b[1] * us / n, b[2] * us / n, b[3] * us / n, b[4] * us / n, b[5] * us / n, b[6] * us / n);
    long long z[10] = {0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_chain_prof), z, sizeof(z));
}
#endif

hipError_t launch_pnp_chain(const int4* knn, const int* counts, const float* xyz, const float* kun, int kp_cap,
                      float nnratio, const int* seg, int S, const PnpCam& cam, float thr, const PnpPrm& prm, float* p3,
                      float* p2, int* mq, int* mt, uint8_t* mask, uint8_t* flags, PnpChainRes* res,
                      const uint32_t* rngtab, int ntab, unsigned long long rng_end, PnpProbDev* probs, int* best,
                      PnpModel* models, int P, hipStream_t st)
{
    if (S <= 0) return hipSuccess;
    static_assert(sizeof(ChainLds) + (size_t)kPnpMaxM * 5 * sizeof(float) <= 160 * 1024, "k_pnp_chain LDS");
    if (kp_cap > kPnpMaxM) return hipErrorInvalidValue;   // the caller checks first (pnp_host.cpp track_submit)
    return dispatch(k_pnp_chain, dim3(S), dim3(kChainThreads), (size_t)kp_cap * 5 * sizeof(float), st, knn, counts,
                       xyz, kun, kp_cap, nnratio, seg, cam, thr, prm, p3, p2, mq, mt, mask, flags, res, rngtab, ntab,
                       rng_end, probs, best, models, P);
}

}  // namespace rgbd

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

#include <climits>

#include "pnp_dev.h"

namespace rgbd {

namespace {

// ------------------------------------------------------------------ small dense helpers (double)
// cyclic Jacobi on a symmetric 3 x 3 (row-major, in place); eigenvectors in the columns of V
__device__ void jacobi_eig3(double* A, double* V)
{
    const int n = 3;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) V[i * n + j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; sweep++) {
        double off = 0.0, diag = 0.0;
        for (int p = 0; p < n; p++) {
            diag += A[p * n + p] * A[p * n + p];
            for (int q = p + 1; q < n; q++) off += A[p * n + q] * A[p * n + q];
        }
        if (!(off > 1e-36 * diag) || off == 0.0) break;
        for (int p = 0; p < n - 1; p++)
            for (int q = p + 1; q < n; q++) {
                const double apq = A[p * n + q];
                if (fabs(apq) < 1e-300) continue;
                const double theta = (A[q * n + q] - A[p * n + p]) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0);
                const double s = t * c;
                for (int k = 0; k < n; k++) {
                    const double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = c * akp - s * akq;
                    A[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; k++) {
                    const double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = c * apk - s * aqk;
                    A[q * n + k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; k++) {
                    const double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - s * vkq;
                    V[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
}

// min |A x - b|, A 6 x n (n <= 5, row-major), Householder QR
__device__ void lsq_qr(const double* Ain, const double* bin, int n, double* x)
{
    const int m = 6;
    double A[6 * 5], b[6];
    for (int i = 0; i < m * n; i++) A[i] = Ain[i];
    for (int i = 0; i < m; i++) b[i] = bin[i];
    for (int k = 0; k < n; k++) {
        double nrm = 0.0;
        for (int i = k; i < m; i++) nrm += A[i * n + k] * A[i * n + k];
        nrm = sqrt(nrm);
        if (nrm == 0.0) continue;
        const double alpha = A[k * n + k] > 0 ? -nrm : nrm;
        double v[6];
        for (int i = 0; i < m; i++) v[i] = (i < k) ? 0.0 : A[i * n + k];
        v[k] -= alpha;
        double vn = 0.0;
        for (int i = k; i < m; i++) vn += v[i] * v[i];
        if (vn == 0.0) continue;
        for (int j = k; j < n; j++) {
            double d = 0.0;
            for (int i = k; i < m; i++) d += v[i] * A[i * n + j];
            const double f = 2.0 * d / vn;
            for (int i = k; i < m; i++) A[i * n + j] -= f * v[i];
        }
        double d = 0.0;
        for (int i = k; i < m; i++) d += v[i] * b[i];
        const double f = 2.0 * d / vn;
        for (int i = k; i < m; i++) b[i] -= f * v[i];
    }
    for (int k = n - 1; k >= 0; k--) {
        double s = b[k];
        for (int j = k + 1; j < n; j++) s -= A[k * n + j] * x[j];
        x[k] = (A[k * n + k] != 0.0) ? s / A[k * n + k] : 0.0;
    }
}

__device__ void svd3_jacobi(const double M[9], double U[9], double S[3], double V[9])
{
    double MtM[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0.0;
            for (int k = 0; k < 3; k++) s += M[k * 3 + i] * M[k * 3 + j];
            MtM[i * 3 + j] = s;
        }
    double Vt[9];
    jacobi_eig3(MtM, Vt);
    int idx[3] = {0, 1, 2};
    for (int a = 0; a < 3; a++)
        for (int b = a + 1; b < 3; b++)
            if (MtM[idx[b] * 4] > MtM[idx[a] * 4]) { const int t = idx[a]; idx[a] = idx[b]; idx[b] = t; }
    for (int c = 0; c < 3; c++) {
        const double ev = MtM[idx[c] * 4];
        S[c] = ev > 0.0 ? sqrt(ev) : 0.0;
        for (int r = 0; r < 3; r++) V[r * 3 + c] = Vt[r * 3 + idx[c]];
    }
    for (int c = 0; c < 3; c++) {
        double u[3];
        for (int r = 0; r < 3; r++)
            u[r] = (M[r * 3 + 0] * V[0 * 3 + c] + M[r * 3 + 1] * V[1 * 3 + c]) + M[r * 3 + 2] * V[2 * 3 + c];
        for (int p = 0; p < c; p++) {
            const double d = (u[0] * U[0 * 3 + p] + u[1] * U[1 * 3 + p]) + u[2] * U[2 * 3 + p];
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
                for (int p = 0; p < c; p++) {
                    const double d = (u[0] * U[0 * 3 + p] + u[1] * U[1 * 3 + p]) + u[2] * U[2 * 3 + p];
                    for (int r = 0; r < 3; r++) u[r] -= d * U[r * 3 + p];
                }
            }
            nn = sqrt((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
        }
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
    for (int it = 0; it < 5; it++) {
        double A[6 * 4], b[6];
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
            for (int k = 0; k < 10; k++) s += l[k] * bb[k];
            b[i] = rho[i] - s;
        }
        double x[4];
        lsq_qr(A, b, 4, x);
        for (int k = 0; k < 4; k++) betas[k] += x[k];
    }
}

// R, t from betas over the 5 sample points; returns the mean reprojection error
__device__ double compute_R_and_t(const double* pw, const double* us, const double* alphas, const PnpCam& K,
                                  const double* ut, const double betas[4], double R[9], double t[3])
{
    const int n = kPnpModel;
    double ccs[4][3];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 3; j++) ccs[i][j] = 0.0;
    for (int k = 0; k < 4; k++)
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 3; j++) ccs[i][j] += betas[k] * ut[k * 12 + 3 * i + j];
    double pcs[3 * kPnpModel];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++)
            pcs[3 * i + j] = ((alphas[4 * i] * ccs[0][j] + alphas[4 * i + 1] * ccs[1][j]) + alphas[4 * i + 2] * ccs[2][j])
                             + alphas[4 * i + 3] * ccs[3][j];
    if (pcs[2] < 0.0) {
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 3; j++) ccs[i][j] = -ccs[i][j];
        for (int i = 0; i < 3 * n; i++) pcs[i] = -pcs[i];
    }
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) {
            pc0[j] += pcs[3 * i + j];
            pw0[j] += pw[3 * i + j];
        }
    for (int j = 0; j < 3; j++) {
        pc0[j] /= n;
        pw0[j] /= n;
    }
    double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; i++)
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) abt[a * 3 + b] += (pcs[3 * i + a] - pc0[a]) * (pw[3 * i + b] - pw0[b]);
    double U[9], S[3], V[9];
    svd3_jacobi(abt, U, S, V);
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++)
            R[a * 3 + b] = (U[a * 3 + 0] * V[b * 3 + 0] + U[a * 3 + 1] * V[b * 3 + 1]) + U[a * 3 + 2] * V[b * 3 + 2];
    if (det3(R) < 0.0)
        for (int b = 0; b < 3; b++) R[6 + b] = -R[6 + b];
    for (int a = 0; a < 3; a++) t[a] = pc0[a] - ((R[a * 3 + 0] * pw0[0] + R[a * 3 + 1] * pw0[1]) + R[a * 3 + 2] * pw0[2]);
    double sum = 0.0;
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

struct HypLds {
    double A[144];
    double V[144];
    double pw[15], us[10], alphas[20], cw[12];
    double cs[6][2];
    double ut[48], L[60], rho[6];
    double candR[3][9], candT[3][3], candE[3];
    double R[9], t[3];
    int act[6];
    int pairs[11][6][2];
    int order[4];
    int flag;
    int ok;
};

}  // namespace

__global__ __launch_bounds__(64) void k_pnp_hyp(const float* __restrict__ p3, const float* __restrict__ p2,
                                                const PnpProbDev* __restrict__ probs, const int* __restrict__ hyp_prob,
                                                const int* __restrict__ samples, PnpCam K, float thr, int H,
                                                int* __restrict__ good_out, PnpModel* __restrict__ model_out)
{
    __shared__ HypLds s;
    const int h = blockIdx.x;
    if (h >= H) return;
    const int lane = threadIdx.x;
    const PnpProbDev pr = probs[hyp_prob[h]];
    const float* P3 = p3 + 3 * (size_t)pr.off;
    const float* P2 = p2 + 2 * (size_t)pr.off;

    // ---- lane 0: sample points, control points (PCA), barycentric coordinates, Jacobi pair table
    if (lane == 0) {
        const int n = kPnpModel;
        for (int i = 0; i < n; i++) {
            const int id = samples[(size_t)h * kPnpModel + i];
            for (int j = 0; j < 3; j++) s.pw[3 * i + j] = (double)P3[3 * id + j];
            for (int j = 0; j < 2; j++) s.us[2 * i + j] = (double)P2[2 * id + j];
        }
        double cw[4][3];
        for (int j = 0; j < 3; j++) cw[0][j] = 0.0;
        for (int i = 0; i < n; i++)
            for (int j = 0; j < 3; j++) cw[0][j] += s.pw[3 * i + j];
        for (int j = 0; j < 3; j++) cw[0][j] /= n;
        double A[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < n; i++) {
            double d[3];
            for (int j = 0; j < 3; j++) d[j] = s.pw[3 * i + j] - cw[0][j];
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) A[a * 3 + b] += d[a] * d[b];
        }
        double V[9];
        jacobi_eig3(A, V);
        int idx[3] = {0, 1, 2};
        for (int a = 0; a < 3; a++)
            for (int b = a + 1; b < 3; b++)
                if (A[idx[b] * 4] > A[idx[a] * 4]) { const int t = idx[a]; idx[a] = idx[b]; idx[b] = t; }
        for (int i = 1; i < 4; i++) {
            const double ev = A[idx[i - 1] * 4];
            const double k = sqrt((ev > 0.0 ? ev : 0.0) / n);
            for (int j = 0; j < 3; j++) cw[i][j] = cw[0][j] + k * V[j * 3 + idx[i - 1]];
        }
        double CC[9], CCi[9];
        for (int i = 0; i < 3; i++)
            for (int j = 1; j < 4; j++) CC[i * 3 + (j - 1)] = cw[j][i] - cw[0][i];
        s.ok = inv3(CC, CCi) ? 1 : 0;
        for (int i = 0; i < n; i++) {
            double d[3];
            for (int j = 0; j < 3; j++) d[j] = s.pw[3 * i + j] - cw[0][j];
            for (int j = 0; j < 3; j++)
                s.alphas[4 * i + 1 + j] = (CCi[j * 3 + 0] * d[0] + CCi[j * 3 + 1] * d[1]) + CCi[j * 3 + 2] * d[2];
            s.alphas[4 * i] = 1.0 - s.alphas[4 * i + 1] - s.alphas[4 * i + 2] - s.alphas[4 * i + 3];
        }
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 3; j++) s.cw[3 * i + j] = cw[i][j];
        int arr[12];
        for (int i = 0; i < 12; i++) arr[i] = i;
        for (int r = 0; r < 11; r++) {
            for (int k = 0; k < 6; k++) {
                const int a = arr[k], b = arr[11 - k];
                s.pairs[r][k][0] = a < b ? a : b;
                s.pairs[r][k][1] = a < b ? b : a;
            }
            const int last = arr[11];
            for (int i = 11; i > 1; i--) arr[i] = arr[i - 1];
            arr[1] = last;
        }
    }
    __syncthreads();
    if (!s.ok) {
        if (lane == 0) good_out[h] = -1;
        return;
    }

    // ---- M^T M (12 x 12): entry (a, b) = sum over the 5 points of r1a r1b + r2a r2b, point order
    for (int e = lane; e < 144; e += 64) {
        const int a = e / 12, b = e % 12;
        double acc = 0.0;
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
        s.A[e] = acc;
        s.V[e] = (a == b) ? 1.0 : 0.0;
    }
    __syncthreads();

    // ---- round-robin Jacobi (oracle jacobi_eig12)
    for (int sweep = 0; sweep < 60; sweep++) {
        if (lane == 0) {
            double off = 0.0, diag = 0.0;
            for (int p = 0; p < 12; p++) {
                diag += s.A[p * 12 + p] * s.A[p * 12 + p];
                for (int q = p + 1; q < 12; q++) off += s.A[p * 12 + q] * s.A[p * 12 + q];
            }
            s.flag = (!(off > 1e-36 * diag) || off == 0.0) ? 0 : 1;
        }
        __syncthreads();
        if (!s.flag) break;
        for (int r = 0; r < 11; r++) {
            if (lane < 6) {
                const int p = s.pairs[r][lane][0], q = s.pairs[r][lane][1];
                const double apq = s.A[p * 12 + q];
                const int act = !(fabs(apq) < 1e-300);
                s.act[lane] = act;
                if (act) {
                    const double theta = (s.A[q * 12 + q] - s.A[p * 12 + p]) / (2.0 * apq);
                    const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                    const double c = 1.0 / sqrt(t * t + 1.0);
                    s.cs[lane][0] = c;
                    s.cs[lane][1] = t * c;
                }
            }
            __syncthreads();
            for (int u = lane; u < 72; u += 64) {       // columns p, q of every active pair
                const int j = u / 12, k = u % 12;
                if (s.act[j]) {
                    const int p = s.pairs[r][j][0], q = s.pairs[r][j][1];
                    const double c = s.cs[j][0], sn = s.cs[j][1];
                    const double akp = s.A[k * 12 + p], akq = s.A[k * 12 + q];
                    s.A[k * 12 + p] = c * akp - sn * akq;
                    s.A[k * 12 + q] = sn * akp + c * akq;
                }
            }
            __syncthreads();
            for (int u = lane; u < 144; u += 64) {      // rows p, q (u < 72) and V columns (u >= 72)
                const int uu = u < 72 ? u : u - 72;
                const int j = uu / 12, k = uu % 12;
                if (s.act[j]) {
                    const int p = s.pairs[r][j][0], q = s.pairs[r][j][1];
                    const double c = s.cs[j][0], sn = s.cs[j][1];
                    if (u < 72) {
                        const double apk = s.A[p * 12 + k], aqk = s.A[q * 12 + k];
                        s.A[p * 12 + k] = c * apk - sn * aqk;
                        s.A[q * 12 + k] = sn * apk + c * aqk;
                    } else {
                        const double vkp = s.V[k * 12 + p], vkq = s.V[k * 12 + q];
                        s.V[k * 12 + p] = c * vkp - sn * vkq;
                        s.V[k * 12 + q] = sn * vkp + c * vkq;
                    }
                }
            }
            __syncthreads();
        }
    }

    // ---- the four smallest eigenvalues (ascending, ties by index), null-space basis ut, L and rho
    if (lane == 0) {
        int order[12];
        for (int i = 0; i < 12; i++) order[i] = i;
        for (int a = 0; a < 12; a++)
            for (int b = a + 1; b < 12; b++)
                if (s.A[order[b] * 13] < s.A[order[a] * 13]) { const int tt = order[a]; order[a] = order[b]; order[b] = tt; }
        for (int k = 0; k < 4; k++) s.order[k] = order[k];
    }
    __syncthreads();
    if (lane < 48) {
        const int k = lane / 12, i = lane % 12;
        s.ut[lane] = s.V[i * 12 + s.order[k]];
    }
    __syncthreads();
    if (lane < 6) {
        const int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
        const int a = pa[lane], b = pb[lane];
        double dv[4][3];
        for (int k = 0; k < 4; k++)
            for (int j = 0; j < 3; j++) dv[k][j] = s.ut[k * 12 + 3 * a + j] - s.ut[k * 12 + 3 * b + j];
        auto dot = [&](int x, int y) { return (dv[x][0] * dv[y][0] + dv[x][1] * dv[y][1]) + dv[x][2] * dv[y][2]; };
        double* L = s.L + 10 * lane;
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
        s.rho[lane] = (dx * dx + dy * dy) + dz * dz;
    }
    __syncthreads();

    // ---- beta candidates N = 1, 2, 3 on lanes 0, 1, 2
    if (lane < 3) {
        const int N = lane + 1;
        const int ncol = N == 1 ? 4 : (N == 2 ? 3 : 5);
        const int cols1[4] = {0, 1, 3, 6};
        double A[30], x[5], b4[4];
        for (int i = 0; i < 6; i++)
            for (int k = 0; k < ncol; k++) A[i * ncol + k] = s.L[10 * i + (N == 1 ? cols1[k] : k)];
        lsq_qr(A, s.rho, ncol, x);
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
        s.candE[lane] = compute_R_and_t(s.pw, s.us, s.alphas, K, s.ut, b4, s.candR[lane], s.candT[lane]);
    }
    __syncthreads();
    if (lane == 0) {
        double best = INFINITY;
        int bi = -1;
        for (int c = 0; c < 3; c++)
            if (s.candE[c] < best) { best = s.candE[c]; bi = c; }
        s.ok = bi >= 0 ? 1 : 0;
        if (bi >= 0) {
            for (int i = 0; i < 9; i++) s.R[i] = s.candR[bi][i];
            for (int i = 0; i < 3; i++) s.t[i] = s.candT[bi][i];
        }
    }
    __syncthreads();
    if (!s.ok) {
        if (lane == 0) good_out[h] = -1;
        return;
    }
    // ---- findInliers over every point of the problem
    double R[9], t[3];
    for (int i = 0; i < 9; i++) R[i] = s.R[i];
    for (int i = 0; i < 3; i++) t[i] = s.t[i];
    int cnt = 0;
    for (int i = lane; i < pr.count; i += 64) cnt += reproj_err2(P3 + 3 * i, P2 + 2 * i, R, t, K) <= thr ? 1 : 0;
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if (lane == 0) good_out[h] = cnt;
    if (lane < 12) {
        double* dst = lane < 9 ? &model_out[h].R[lane] : &model_out[h].t[lane - 9];
        *dst = lane < 9 ? R[lane] : t[lane - 9];
    }
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

__device__ bool solve6(const double* H, const double* g, double x[6])
{
    double A[6][7];
    for (int i = 0; i < 6; i++) {
        for (int j = 0; j < 6; j++) A[i][j] = H[i * 6 + j];
        A[i][6] = -g[i];
    }
    for (int k = 0; k < 6; k++) {
        int p = k;
        for (int i = k + 1; i < 6; i++)
            if (fabs(A[i][k]) > fabs(A[p][k])) p = i;
        if (A[p][k] == 0.0) return false;
        if (p != k)
            for (int j = 0; j < 7; j++) { const double tt = A[k][j]; A[k][j] = A[p][j]; A[p][j] = tt; }
        for (int i = k + 1; i < 6; i++) {
            const double f = A[i][k] / A[k][k];
            for (int j = k; j < 7; j++) A[i][j] -= f * A[k][j];
        }
    }
    for (int k = 5; k >= 0; k--) {
        double sacc = A[k][6];
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
constexpr int kRedBatch = 9;   // reduced components per LDS pass (27 = 3 x 9)

}  // namespace

__global__ __launch_bounds__(kRefineThreads) void k_pnp_refine(
    const float* __restrict__ p3, const float* __restrict__ p2, const PnpProbDev* __restrict__ probs,
    const int* __restrict__ best, const int* __restrict__ force_all, const PnpModel* __restrict__ models, PnpCam K,
    float thr, uint8_t* __restrict__ mask, PnpModel* __restrict__ out)
{
    __shared__ int idx[kPnpMaxM];
    __shared__ double red[kRedBatch * kRefineThreads];
    __shared__ double sums[27];
    __shared__ double R[9], t[3];
    __shared__ int wtot[kRefineThreads / 64];
    __shared__ int stop;
    const int p = blockIdx.x;
    const int bh = best[p];
    if (bh < 0) return;   // uniform
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const PnpProbDev pr = probs[p];
    const float* P3 = p3 + 3 * (size_t)pr.off;
    const float* P2 = p2 + 2 * (size_t)pr.off;
    const bool all = force_all[p] != 0;
    if (tid < 9) R[tid] = models[bh].R[tid];
    if (tid < 3) t[tid] = models[bh].t[tid];
    __syncthreads();
    double Rr[9], tr[3];
    for (int i = 0; i < 9; i++) Rr[i] = R[i];
    for (int i = 0; i < 3; i++) tr[i] = t[i];

    // ---- RANSAC inlier mask of the best model, compacted in index order
    int nI = 0;
    for (int base = 0; base < pr.count; base += kRefineThreads) {
        const int i = base + tid;
        bool m = false;
        if (i < pr.count) {
            m = all || reproj_err2(P3 + 3 * i, P2 + 2 * i, Rr, tr, K) <= thr;
            mask[pr.off + i] = m ? 1 : 0;
        }
        const unsigned long long bal = __ballot(m);
        const int below = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wtot[wave] = __popcll(bal);
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

    // ---- 10 Gauss-Newton steps (oracle orc_pnp_ransac refinement order)
    for (int it = 0; it < 10; it++) {
        double acc[27];
        for (int k = 0; k < 27; k++) acc[k] = 0.0;
        for (int i = tid; i < nI; i += kRefineThreads) {
            const int id = idx[i];
            double term[27];
            gn_terms(P3 + 3 * id, P2 + 2 * id, Rr, tr, K, term);
            for (int k = 0; k < 27; k++) acc[k] += term[k];
        }
        for (int k0 = 0; k0 < 27; k0 += kRedBatch) {
            for (int kk = 0; kk < kRedBatch; kk++) red[kk * kRefineThreads + tid] = acc[k0 + kk];
            __syncthreads();
            for (int sdist = kRefineThreads / 2; sdist > 0; sdist >>= 1) {
                if (tid < sdist)
                    for (int kk = 0; kk < kRedBatch; kk++)
                        red[kk * kRefineThreads + tid] += red[kk * kRefineThreads + tid + sdist];
                __syncthreads();
            }
            if (tid < kRedBatch) sums[k0 + tid] = red[tid * kRefineThreads];
            __syncthreads();
        }
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
        if (stop) break;
        for (int i = 0; i < 9; i++) Rr[i] = R[i];
        for (int i = 0; i < 3; i++) tr[i] = t[i];
    }
    if (tid < 9) out[p].R[tid] = R[tid];
    if (tid < 3) out[p].t[tid] = t[tid];
}

// ------------------------------------------------------------------ match filter + 3D-2D gather
constexpr int kGatherThreads = 1024;
constexpr int kMaxTrain = 8192;

__global__ __launch_bounds__(kGatherThreads) void k_match_gather(
    const int4* __restrict__ knn, const int* __restrict__ counts, const int* __restrict__ qf,
    const int* __restrict__ tf, const float* __restrict__ xyz, const float* __restrict__ kun, int kp_cap,
    float nnratio, float* __restrict__ p3, float* __restrict__ p2, PnpProbDev* __restrict__ probs,
    int* __restrict__ mq, int* __restrict__ mt)
{
    __shared__ int winner[kMaxTrain];
    __shared__ int wtot[kGatherThreads / 64];
    const int p = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int rf = qf[p], cf = tf[p];
    const int nq = counts[rf], nt = counts[cf];
    const int4* kr = knn + (size_t)p * kp_cap;
    const float* zq = xyz + (size_t)rf * kp_cap * 3;
    const float* zt = xyz + (size_t)cf * kp_cap * 3;
    for (int i = tid; i < nt && i < kMaxTrain; i += kGatherThreads) winner[i] = INT_MAX;
    __syncthreads();
    // candidate = ratio test passed and both depths valid (Features/Matcher.cpp:118-131; the
    // "train index already used" test only ever sees earlier candidates, so the kept match of a
    // train index is its lowest-index candidate query)
    auto candidate = [&](int i, int* i2o) -> bool {
        const int4 r = kr[i];
        if (r.w < 0) return false;   // fewer than 2 train rows: skipped (reference UB)
        const float d1 = (float)r.x, d2 = (float)r.z;
        if (!(d1 < nnratio * d2)) return false;
        if (!(zq[3 * i + 2] > 0) || !(zt[3 * r.y + 2] > 0)) return false;
        *i2o = r.y;
        return true;
    };
    if (nq > 0 && nt > 0) {
        for (int i = tid; i < nq; i += kGatherThreads) {
            int i2;
            if (candidate(i, &i2)) atomicMin(&winner[i2], i);
        }
    }
    __syncthreads();
    int m = 0;
    float* P3 = p3 + 3 * (size_t)p * kp_cap;
    float* P2 = p2 + 2 * (size_t)p * kp_cap;
    const int nql = (nq > 0 && nt > 0) ? nq : 0;
    for (int base = 0; base < nql; base += kGatherThreads) {
        const int i = base + tid;
        int i2 = -1;
        const bool keep = i < nql && candidate(i, &i2) && winner[i2] == i;
        const unsigned long long bal = __ballot(keep);
        const int below = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wtot[wave] = __popcll(bal);
        __syncthreads();
        int pre = 0, tot = 0;
        for (int w = 0; w < kGatherThreads / 64; w++) {
            pre += w < wave ? wtot[w] : 0;
            tot += wtot[w];
        }
        if (keep) {
            const int o = m + pre + below;
            const float* X = xyz + ((size_t)rf * kp_cap + i) * 3;
            const float* U = kun + ((size_t)cf * kp_cap + i2) * 7;
            P3[3 * o] = X[0];
            P3[3 * o + 1] = X[1];
            P3[3 * o + 2] = X[2];
            P2[2 * o] = U[0];
            P2[2 * o + 1] = U[1];
            mq[(size_t)p * kp_cap + o] = i;
            mt[(size_t)p * kp_cap + o] = i2;
        }
        m += tot;
        __syncthreads();
    }
    if (tid == 0) probs[p] = PnpProbDev{(int)((size_t)p * kp_cap), m};
}

void launch_pnp_hyp(const float* p3, const float* p2, const PnpProbDev* probs, const int* hyp_prob,
                    const int* samples, const PnpCam& cam, float thr, int H, int* good, PnpModel* models,
                    hipStream_t st)
{
    if (H <= 0) return;
    hipLaunchKernelGGL(k_pnp_hyp, dim3(H), dim3(64), 0, st, p3, p2, probs, hyp_prob, samples, cam, thr, H, good,
                       models);
}

void launch_pnp_refine(const float* p3, const float* p2, const PnpProbDev* probs, const int* best,
                       const int* force_all, const PnpModel* models, const PnpCam& cam, float thr, int P,
                       uint8_t* mask, PnpModel* out, hipStream_t st)
{
    if (P <= 0) return;
    hipLaunchKernelGGL(k_pnp_refine, dim3(P), dim3(kRefineThreads), 0, st, p3, p2, probs, best, force_all, models,
                       cam, thr, mask, out);
}

void launch_match_gather(const int4* knn, const int* counts, const int* qf, const int* tf, const float* xyz,
                         const float* kun, int kp_cap, float nnratio, int npairs, float* p3, float* p2,
                         PnpProbDev* probs, int* mq, int* mt, hipStream_t st)
{
    if (npairs <= 0) return;
    hipLaunchKernelGGL(k_match_gather, dim3(npairs), dim3(kGatherThreads), 0, st, knn, counts, qf, tf, xyz, kun,
                       kp_cap, nnratio, p3, p2, probs, mq, mt);
}

}  // namespace rgbd

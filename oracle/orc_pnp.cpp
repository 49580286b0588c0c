// orc_pnp.cpp -- ORACLE (test infrastructure only; see rgbd_oracle.h header).
//
// PnPRansac::compute (Solver/PnPRansac.cpp:14-56) calls
//   cv::solvePnPRansac(v3D, v2D, K, noDist, r, t, false, 500, 3.0f, 0.85, inliers)   (:39)
// OpenCV is absent, so the operator is DEFINED here (DESIGN.md "PnPRansac definition") and the
// HIP path must equal this definition bit for bit:
//   * RANSAC driver = OpenCV 3.4 RANSACPointSetRegistrator::run: cv::RNG((uint64)-1) multiply-with-
//     carry stream, getSubset (5 distinct indices), findInliers (float err <= (float)(thr*thr)),
//     best = goodCount > max(best, modelPoints-1), niters = RANSACUpdateNumIters(conf, ep, 5, niters)
//     (its log / pow restated portably: log_det, repeated products).
//   * minimal solver = EPnP (Lepetit, Moreno-Noguer, Fua 2009) on the 5 sampled points: PCA control
//     points, barycentric coordinates, 12x12 M^T M null space (round-robin Jacobi), betas for N = 1, 2, 3
//     (+ 5 Gauss-Newton steps), Procrustes R,t; the lowest-reprojection-error candidate wins.
//   * model error = float squared pixel distance of the pinhole projection (no distortion).
//   * final refinement on the RANSAC inliers = 10 Gauss-Newton steps on SE(3) (left increment),
//     normal equations accumulated in a fixed 256-lane strided order + a natural-order binary tree
//     over the lanes (the device order).
// All arithmetic is IEEE double/float without contraction; sin/cos are polynomial evaluations built
// from + - * / only, so host and device agree exactly.
#include "rgbd_oracle.h"
#include "orc_common.h"

#include <cfloat>
#include <climits>
#include <cmath>
#include <cstring>
#include <vector>

namespace {

using orc::rodrigues_exp;
using orc::solve6;
using orc::sincos_poly;

// ------------------------------------------------------------ cv::RNG (multiply-with-carry)
struct CvRng {
    uint64_t state;
    explicit CvRng(uint64_t s) : state(s ? s : 0xffffffffull) {}
    unsigned next()
    {
        state = (uint64_t)(unsigned)state * 4164903690u + (unsigned)(state >> 32);
        return (unsigned)state;
    }
    int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + a); }
};

// natural log from + - * / and exact frexp only, so host and device agree bit for bit:
// x = m 2^e, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s), s = (m - 1) / (m + 1), series to s^23
double log_det(double x)
{
    int e = 0;
    double m = std::frexp(x, &e);
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

// RANSACUpdateNumIters (OpenCV 3.4 ptsetreg.cpp) with std::log -> log_det and std::pow(q, 5) -> q^5
// as four products (the portable definition the device replay also computes)
int update_num_iters(double p, double ep, int modelPoints, int maxIters)
{
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    const double q = 1. - ep;
    double qm = 1.0;
    for (int i = 0; i < modelPoints; i++) qm = qm * q;
    double denom = 1. - qm;
    if (denom < DBL_MIN) return 0;
    num = log_det(num);
    denom = log_det(denom);
    return denom >= 0 || -num >= maxIters * (-denom) ? maxIters : (int)std::nearbyint(num / denom);
}

// ------------------------------------------------------------ small dense helpers
// cyclic Jacobi eigen-decomposition of a symmetric n x n matrix (row-major, in place):
// eigenvalues on the diagonal, eigenvectors in the columns of V.  Deterministic definition
// (Numerical Recipes style): a sweep visits (p, q), p < q, in row order; an element whose 100|a_pq|
// does not change |a_pp| nor |a_qq| in double is set to zero and skipped; after a rotation a_pq and
// a_qp are set to exactly zero; sweeps stop when the sum of |a_pq| is exactly zero (<= 50 sweeps).
bool negligible(double apq, double app, double aqq)
{
    const double g = 100.0 * std::fabs(apq);
    return std::fabs(app) + g == std::fabs(app) && std::fabs(aqq) + g == std::fabs(aqq);
}

void jacobi_eig(double* A, double* V, int n)
{
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) V[i * n + j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; sweep++) {
        double sm = 0.0;
        for (int p = 0; p < n; p++)
            for (int q = p + 1; q < n; q++) sm += std::fabs(A[p * n + q]);
        if (sm == 0.0) break;
        for (int p = 0; p < n - 1; p++)
            for (int q = p + 1; q < n; q++) {
                const double apq = A[p * n + q];
                if (negligible(apq, A[p * n + p], A[q * n + q])) {
                    A[p * n + q] = 0.0;
                    A[q * n + p] = 0.0;
                    continue;
                }
                const double theta = (A[q * n + q] - A[p * n + p]) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0);
                const double s = t * c;
                for (int k = 0; k < n; k++) {   // columns p, q
                    const double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = c * akp - s * akq;
                    A[k * n + q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; k++) {   // rows p, q; the rotated pair itself becomes exactly zero
                    const double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = (k == q) ? 0.0 : c * apk - s * aqk;
                    A[q * n + k] = (k == p) ? 0.0 : s * apk + c * aqk;
                }
                for (int k = 0; k < n; k++) {
                    const double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - s * vkq;
                    V[k * n + q] = s * vkp + c * vkq;
                }
            }
    }
}

// Round-robin (tournament) ordered Jacobi for the 12 x 12 EPnP matrix.  One sweep = 11 rounds of
// 6 disjoint pairs: arr = [0..11]; round pairs (arr[k], arr[11-k]), k = 0..5 (as (min, max)); then
// arr[1..11] rotates right by one.  Within a round every active pair's (c, s) comes from the same
// matrix, then ALL column updates, then ALL row updates, then the V updates are applied (disjoint
// pairs, so each element's arithmetic is fixed).  A pair is inactive (and its a_pq zeroed) when
// negligible() holds; rotated pairs end with a_pq = a_qp = 0 exactly; sweeps stop at sum |a_pq| == 0
// (<= 50).  This order is the definition the device follows (one rotation pair per lane group).
void rr_pairs12(int P[11][6][2])
{
    int arr[12];
    for (int i = 0; i < 12; i++) arr[i] = i;
    for (int r = 0; r < 11; r++) {
        for (int k = 0; k < 6; k++) {
            const int a = arr[k], b = arr[11 - k];
            P[r][k][0] = a < b ? a : b;
            P[r][k][1] = a < b ? b : a;
        }
        const int last = arr[11];
        for (int i = 11; i > 1; i--) arr[i] = arr[i - 1];
        arr[1] = last;
    }
}

void jacobi_eig12(double* A, double* V)
{
    const int n = 12;
    int P[11][6][2];
    rr_pairs12(P);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) V[i * n + j] = (i == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 50; sweep++) {
        double sm = 0.0;
        for (int p = 0; p < n; p++)
            for (int q = p + 1; q < n; q++) sm += std::fabs(A[p * n + q]);
        if (sm == 0.0) break;
        for (int r = 0; r < 11; r++) {
            double cs[6][2];
            bool act[6];
            for (int j = 0; j < 6; j++) {
                const int p = P[r][j][0], q = P[r][j][1];
                const double apq = A[p * n + q];
                // a negligible a_pq gets the identity rotation (c, s) = (1, 0); the row pass below
                // then sets a_pq = a_qp = 0 as Numerical Recipes does (bit-identical but for the
                // sign of zero elements, which the device's branch-free update needs)
                act[j] = !negligible(apq, A[p * n + p], A[q * n + q]);
                if (!act[j]) {
                    cs[j][0] = 1.0;
                    cs[j][1] = 0.0;
                    continue;
                }
                const double theta = (A[q * n + q] - A[p * n + p]) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                cs[j][0] = 1.0 / std::sqrt(t * t + 1.0);
                cs[j][1] = t * cs[j][0];
            }
            for (int j = 0; j < 6; j++) {
                const int p = P[r][j][0], q = P[r][j][1];
                const double c = cs[j][0], s = cs[j][1];
                for (int k = 0; k < n; k++) {
                    const double akp = A[k * n + p], akq = A[k * n + q];
                    A[k * n + p] = c * akp - s * akq;
                    A[k * n + q] = s * akp + c * akq;
                }
            }
            for (int j = 0; j < 6; j++) {
                const int p = P[r][j][0], q = P[r][j][1];
                const double c = cs[j][0], s = cs[j][1];
                for (int k = 0; k < n; k++) {
                    const double apk = A[p * n + k], aqk = A[q * n + k];
                    A[p * n + k] = (k == q) ? 0.0 : c * apk - s * aqk;
                    A[q * n + k] = (k == p) ? 0.0 : s * apk + c * aqk;
                }
            }
            for (int j = 0; j < 6; j++) {
                const int p = P[r][j][0], q = P[r][j][1];
                const double c = cs[j][0], s = cs[j][1];
                for (int k = 0; k < n; k++) {
                    const double vkp = V[k * n + p], vkq = V[k * n + q];
                    V[k * n + p] = c * vkp - s * vkq;
                    V[k * n + q] = s * vkp + c * vkq;
                }
            }
        }
    }
}

// least squares min |A x - b| for A m x n (m >= n, row-major) by Householder QR; x[n]
void lsq_qr(const double* Ain, const double* bin, int m, int n, double* x)
{
    double A[6 * 5], b[6];
    std::memcpy(A, Ain, sizeof(double) * m * n);
    std::memcpy(b, bin, sizeof(double) * m);
    for (int k = 0; k < n; k++) {
        double nrm = 0.0;
        for (int i = k; i < m; i++) nrm += A[i * n + k] * A[i * n + k];
        nrm = std::sqrt(nrm);
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

// 3x3 SVD-based Procrustes: R = U V^T of abt (via eigen of abt^T abt), det fix on the last row
void svd3_jacobi(const double M[9], double U[9], double S[3], double V[9])
{
    // V, S^2 from the eigen-decomposition of M^T M; U = M V / S (Gram-Schmidt completion for tiny S)
    double MtM[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0.0;
            for (int k = 0; k < 3; k++) s += M[k * 3 + i] * M[k * 3 + j];
            MtM[i * 3 + j] = s;
        }
    double Vt[9];
    jacobi_eig(MtM, Vt, 3);
    // sort eigenvalues descending (stable by index)
    int idx[3] = {0, 1, 2};
    for (int a = 0; a < 3; a++)
        for (int b = a + 1; b < 3; b++)
            if (MtM[idx[b] * 4] > MtM[idx[a] * 4]) { int t = idx[a]; idx[a] = idx[b]; idx[b] = t; }
    for (int c = 0; c < 3; c++) {
        const double ev = MtM[idx[c] * 4];
        S[c] = ev > 0.0 ? std::sqrt(ev) : 0.0;
        for (int r = 0; r < 3; r++) V[r * 3 + c] = Vt[r * 3 + idx[c]];
    }
    for (int c = 0; c < 3; c++) {
        double u[3];
        for (int r = 0; r < 3; r++) u[r] = (M[r * 3 + 0] * V[0 * 3 + c] + M[r * 3 + 1] * V[1 * 3 + c]) + M[r * 3 + 2] * V[2 * 3 + c];
        // orthogonalise against previous columns, then normalise
        for (int p = 0; p < c; p++) {
            const double d = (u[0] * U[0 * 3 + p] + u[1] * U[1 * 3 + p]) + u[2] * U[2 * 3 + p];
            for (int r = 0; r < 3; r++) u[r] -= d * U[r * 3 + p];
        }
        double nn = std::sqrt((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
        if (nn < 1e-300) {   // complete the basis with a cross product (c == 2) or a canonical axis
            if (c == 2) {
                u[0] = U[1 * 3 + 0] * U[2 * 3 + 1] - U[2 * 3 + 0] * U[1 * 3 + 1];
                u[1] = U[2 * 3 + 0] * U[0 * 3 + 1] - U[0 * 3 + 0] * U[2 * 3 + 1];
                u[2] = U[0 * 3 + 0] * U[1 * 3 + 1] - U[1 * 3 + 0] * U[0 * 3 + 1];
            } else {
                u[0] = (c == 0) ? 1.0 : 0.0; u[1] = (c == 1) ? 1.0 : 0.0; u[2] = 0.0;
                for (int p = 0; p < c; p++) {
                    const double d = (u[0] * U[0 * 3 + p] + u[1] * U[1 * 3 + p]) + u[2] * U[2 * 3 + p];
                    for (int r = 0; r < 3; r++) u[r] -= d * U[r * 3 + p];
                }
            }
            nn = std::sqrt((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]);
        }
        for (int r = 0; r < 3; r++) U[r * 3 + c] = u[r] / nn;
    }
}

double det3(const double R[9])
{
    return R[0] * (R[4] * R[8] - R[5] * R[7]) - R[1] * (R[3] * R[8] - R[5] * R[6]) + R[2] * (R[3] * R[7] - R[4] * R[6]);
}

struct Cam { double fu, fv, uc, vc; };

// ------------------------------------------------------------ EPnP
void epnp_control_points(int n, const double* pw, double cw[4][3])
{
    for (int j = 0; j < 3; j++) cw[0][j] = 0.0;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) cw[0][j] += pw[3 * i + j];
    for (int j = 0; j < 3; j++) cw[0][j] /= n;
    double A[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        double d[3];
        for (int j = 0; j < 3; j++) d[j] = pw[3 * i + j] - cw[0][j];
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) A[a * 3 + b] += d[a] * d[b];
    }
    double V[9];
    jacobi_eig(A, V, 3);
    int idx[3] = {0, 1, 2};
    for (int a = 0; a < 3; a++)
        for (int b = a + 1; b < 3; b++)
            if (A[idx[b] * 4] > A[idx[a] * 4]) { int t = idx[a]; idx[a] = idx[b]; idx[b] = t; }
    for (int i = 1; i < 4; i++) {
        const double ev = A[idx[i - 1] * 4];
        const double k = std::sqrt((ev > 0.0 ? ev : 0.0) / n);
        for (int j = 0; j < 3; j++) cw[i][j] = cw[0][j] + k * V[j * 3 + idx[i - 1]];
    }
}

bool inv3(const double M[9], double Mi[9])
{
    const double d = det3(M);
    if (d == 0.0 || !std::isfinite(d)) return false;
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

const int kPairs[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};

void compute_ccs(const double betas[4], const double ut[4][12], double ccs[4][3])
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 3; j++) ccs[i][j] = 0.0;
    for (int k = 0; k < 4; k++)
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 3; j++) ccs[i][j] += betas[k] * ut[k][3 * i + j];
}

// R, t from betas; returns the mean reprojection error
double compute_R_and_t(int n, const double* pw, const double* us, const double* alphas, const Cam& K,
                       const double ut[4][12], const double betas[4], double R[9], double t[3])
{
    double ccs[4][3];
    compute_ccs(betas, ut, ccs);
    std::vector<double> pcs(3 * n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++)
            pcs[3 * i + j] = ((alphas[4 * i] * ccs[0][j] + alphas[4 * i + 1] * ccs[1][j]) + alphas[4 * i + 2] * ccs[2][j])
                             + alphas[4 * i + 3] * ccs[3][j];
    if (pcs[2] < 0.0) {                                  // solve_for_sign
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 3; j++) ccs[i][j] = -ccs[i][j];
        for (int i = 0; i < 3 * n; i++) pcs[i] = -pcs[i];
    }
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int i = 0; i < n; i++)
        for (int j = 0; j < 3; j++) { pc0[j] += pcs[3 * i + j]; pw0[j] += pw[3 * i + j]; }
    for (int j = 0; j < 3; j++) { pc0[j] /= n; pw0[j] /= n; }
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
        sum += std::sqrt(du * du + dv * dv);
    }
    return sum / n;
}

void gauss_newton(const double L[6][10], const double rho[6], double betas[4])
{
    for (int it = 0; it < 5; it++) {
        double A[6 * 4], b[6];
        for (int i = 0; i < 6; i++) {
            const double* l = L[i];
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
        lsq_qr(A, b, 6, 4, x);
        for (int k = 0; k < 4; k++) betas[k] += x[k];
    }
}

// EPnP on n points: returns false only for degenerate input (singular control points)
bool epnp(int n, const double* pw, const double* us, const Cam& K, double R[9], double t[3])
{
    double cw[4][3];
    epnp_control_points(n, pw, cw);
    double CC[9], CCi[9];
    for (int i = 0; i < 3; i++)
        for (int j = 1; j < 4; j++) CC[i * 3 + (j - 1)] = cw[j][i] - cw[0][i];
    if (!inv3(CC, CCi)) return false;
    std::vector<double> alphas(4 * n);
    for (int i = 0; i < n; i++) {
        double d[3];
        for (int j = 0; j < 3; j++) d[j] = pw[3 * i + j] - cw[0][j];
        for (int j = 0; j < 3; j++)
            alphas[4 * i + 1 + j] = (CCi[j * 3 + 0] * d[0] + CCi[j * 3 + 1] * d[1]) + CCi[j * 3 + 2] * d[2];
        alphas[4 * i] = 1.0 - alphas[4 * i + 1] - alphas[4 * i + 2] - alphas[4 * i + 3];
    }
    double MtM[144];
    for (int i = 0; i < 144; i++) MtM[i] = 0.0;
    for (int i = 0; i < n; i++) {
        double r1[12], r2[12];
        const double u = us[2 * i], v = us[2 * i + 1];
        for (int j = 0; j < 4; j++) {
            const double a = alphas[4 * i + j];
            r1[3 * j] = a * K.fu; r1[3 * j + 1] = 0.0; r1[3 * j + 2] = a * (K.uc - u);
            r2[3 * j] = 0.0; r2[3 * j + 1] = a * K.fv; r2[3 * j + 2] = a * (K.vc - v);
        }
        for (int a = 0; a < 12; a++)
            for (int b = 0; b < 12; b++) MtM[a * 12 + b] += r1[a] * r1[b] + r2[a] * r2[b];
    }
    double V[144];
    jacobi_eig12(MtM, V);
    // the four smallest eigenvalues (ascending, stable by index)
    int order[12];
    for (int i = 0; i < 12; i++) order[i] = i;
    for (int a = 0; a < 12; a++)
        for (int b = a + 1; b < 12; b++)
            if (MtM[order[b] * 13] < MtM[order[a] * 13]) { int tt = order[a]; order[a] = order[b]; order[b] = tt; }
    double ut[4][12];
    for (int k = 0; k < 4; k++)
        for (int i = 0; i < 12; i++) ut[k][i] = V[i * 12 + order[k]];
    // L (6 x 10) and rho
    double L[6][10], rho[6];
    for (int p = 0; p < 6; p++) {
        const int a = kPairs[p][0], b = kPairs[p][1];
        double dv[4][3];
        for (int k = 0; k < 4; k++)
            for (int j = 0; j < 3; j++) dv[k][j] = ut[k][3 * a + j] - ut[k][3 * b + j];
        auto dot = [&](int x, int y) { return (dv[x][0] * dv[y][0] + dv[x][1] * dv[y][1]) + dv[x][2] * dv[y][2]; };
        L[p][0] = dot(0, 0);
        L[p][1] = 2 * dot(0, 1);
        L[p][2] = dot(1, 1);
        L[p][3] = 2 * dot(0, 2);
        L[p][4] = 2 * dot(1, 2);
        L[p][5] = dot(2, 2);
        L[p][6] = 2 * dot(0, 3);
        L[p][7] = 2 * dot(1, 3);
        L[p][8] = 2 * dot(2, 3);
        L[p][9] = dot(3, 3);
        const double dx = cw[a][0] - cw[b][0], dy = cw[a][1] - cw[b][1], dz = cw[a][2] - cw[b][2];
        rho[p] = (dx * dx + dy * dy) + dz * dz;
    }
    for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
    t[0] = t[1] = t[2] = 0.0;
    double best = INFINITY;
    // N = 1 (betas 11, 12, 13, 14 -> columns 0, 1, 3, 6)
    {
        double A[24], x[4], b4[4];
        for (int i = 0; i < 6; i++) { A[i * 4] = L[i][0]; A[i * 4 + 1] = L[i][1]; A[i * 4 + 2] = L[i][3]; A[i * 4 + 3] = L[i][6]; }
        lsq_qr(A, rho, 6, 4, x);
        if (x[0] < 0) {
            const double b0 = std::sqrt(-x[0]);
            b4[0] = b0; b4[1] = -x[1] / b0; b4[2] = -x[2] / b0; b4[3] = -x[3] / b0;
        } else {
            const double b0 = std::sqrt(x[0]);
            b4[0] = b0; b4[1] = x[1] / b0; b4[2] = x[2] / b0; b4[3] = x[3] / b0;
        }
        gauss_newton(L, rho, b4);
        double Rc[9], tc[3];
        const double e = compute_R_and_t(n, pw, us, alphas.data(), K, ut, b4, Rc, tc);
        if (e < best) { best = e; std::memcpy(R, Rc, sizeof(Rc)); std::memcpy(t, tc, sizeof(tc)); }
    }
    // N = 2 (betas 11, 12, 22 -> columns 0, 1, 2)
    {
        double A[18], x[3], b4[4];
        for (int i = 0; i < 6; i++) { A[i * 3] = L[i][0]; A[i * 3 + 1] = L[i][1]; A[i * 3 + 2] = L[i][2]; }
        lsq_qr(A, rho, 6, 3, x);
        if (x[0] < 0) {
            b4[0] = std::sqrt(-x[0]);
            b4[1] = (x[2] < 0) ? std::sqrt(-x[2]) : 0.0;
        } else {
            b4[0] = std::sqrt(x[0]);
            b4[1] = (x[2] > 0) ? std::sqrt(x[2]) : 0.0;
        }
        if (x[1] < 0) b4[0] = -b4[0];
        b4[2] = 0.0;
        b4[3] = 0.0;
        gauss_newton(L, rho, b4);
        double Rc[9], tc[3];
        const double e = compute_R_and_t(n, pw, us, alphas.data(), K, ut, b4, Rc, tc);
        if (e < best) { best = e; std::memcpy(R, Rc, sizeof(Rc)); std::memcpy(t, tc, sizeof(tc)); }
    }
    // N = 3 (betas 11, 12, 22, 13, 23 -> columns 0..4)
    {
        double A[30], x[5], b4[4];
        for (int i = 0; i < 6; i++)
            for (int k = 0; k < 5; k++) A[i * 5 + k] = L[i][k];
        lsq_qr(A, rho, 6, 5, x);
        if (x[0] < 0) {
            b4[0] = std::sqrt(-x[0]);
            b4[1] = (x[2] < 0) ? std::sqrt(-x[2]) : 0.0;
        } else {
            b4[0] = std::sqrt(x[0]);
            b4[1] = (x[2] > 0) ? std::sqrt(x[2]) : 0.0;
        }
        if (x[1] < 0) b4[0] = -b4[0];
        b4[2] = x[3] / b4[0];
        b4[3] = 0.0;
        gauss_newton(L, rho, b4);
        double Rc[9], tc[3];
        const double e = compute_R_and_t(n, pw, us, alphas.data(), K, ut, b4, Rc, tc);
        if (e < best) { best = e; std::memcpy(R, Rc, sizeof(Rc)); std::memcpy(t, tc, sizeof(tc)); }
    }
    return best < INFINITY;   // some candidate had a finite mean reprojection error
}

// PnPRansacCallback::computeError: float squared distance to the (float-stored) projection
float reproj_err2(const float* P, const float* uv, const double R[9], const double t[3], const Cam& K)
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

// Jacobian of the projection residual at one point wrt the left SE(3) increment (w, v):
// r = (u_hat - u, v_hat - v); 21 upper-triangle entries of J^T J and 6 of J^T r.
void gn_terms(const float* P, const float* uv, const double R[9], const double t[3], const Cam& K, double out[27])
{
    const double X = ((R[0] * (double)P[0] + R[1] * (double)P[1]) + R[2] * (double)P[2]) + t[0];
    const double Y = ((R[3] * (double)P[0] + R[4] * (double)P[1]) + R[5] * (double)P[2]) + t[1];
    const double Z = ((R[6] * (double)P[0] + R[7] * (double)P[1]) + R[8] * (double)P[2]) + t[2];
    const double iz = 1.0 / Z, iz2 = iz * iz;
    const double ru = (K.fu * X * iz + K.uc) - (double)uv[0];
    const double rv = (K.fv * Y * iz + K.vc) - (double)uv[1];
    // d(u)/dX = fu/Z, d(u)/dZ = -fu X/Z^2 ; dX/d(w,v) = [-[X]x, I]
    const double du[3] = {K.fu * iz, 0.0, -K.fu * X * iz2};
    const double dv[3] = {0.0, K.fv * iz, -K.fv * Y * iz2};
    // J row = d * [ -[p]x | I ] with p = (X, Y, Z): d*(-[p]x) = p x d
    const double Ju[6] = {Y * du[2] - Z * du[1], Z * du[0] - X * du[2], X * du[1] - Y * du[0], du[0], du[1], du[2]};
    const double Jv[6] = {Y * dv[2] - Z * dv[1], Z * dv[0] - X * dv[2], X * dv[1] - Y * dv[0], dv[0], dv[1], dv[2]};
    int k = 0;
    for (int a = 0; a < 6; a++)
        for (int b = a; b < 6; b++) out[k++] = Ju[a] * Ju[b] + Jv[a] * Jv[b];
    for (int a = 0; a < 6; a++) out[k++] = Ju[a] * ru + Jv[a] * rv;
}

}  // namespace

static int g_refine_iters = 10;   // orc_pnp_set_refine_iters(0): the RANSAC model itself (optimiser comparisons)

extern "C" {

void orc_pnp_set_refine_iters(int n) { g_refine_iters = n < 0 ? 0 : n; }

int orc_cvrng_uniform_stream(uint64_t seed, int count, int n, int32_t* out)
{
    CvRng r(seed);
    for (int i = 0; i < n; i++) out[i] = r.uniform(0, count);
    return n;
}

int orc_update_num_iters(double p, double ep, int modelPoints, int maxIters)
{
    return update_num_iters(p, ep, modelPoints, maxIters);
}

int orc_epnp(const float* p3, const float* p2, int n, const float* K4, double* R9, double* t3)
{
    std::vector<double> pw(3 * n), us(2 * n);
    for (int i = 0; i < 3 * n; i++) pw[i] = p3[i];
    for (int i = 0; i < 2 * n; i++) us[i] = p2[i];
    const Cam K{K4[0], K4[1], K4[2], K4[3]};
    return epnp(n, pw.data(), us.data(), K, R9, t3) ? 1 : 0;
}

// solvePnPRansac restated (definition above).  K4 = (fx, fy, cx, cy).  Outputs R (row-major 3x3, double),
// t (double), the RANSAC inlier mask, the number of iterations run.  Returns 1 on success.
int orc_pnp_ransac(const float* p3, const float* p2, int count, const float* K4, int iterationsCount,
                   float reprojectionError, double confidence, double* R9, double* t3, uint8_t* inlier_mask,
                   int32_t* n_inliers, int32_t* iters_run)
{
    const Cam K{K4[0], K4[1], K4[2], K4[3]};
    const int modelPoints = 5;
    *n_inliers = 0;
    *iters_run = 0;
    for (int i = 0; i < 9; i++) R9[i] = (i % 4 == 0) ? 1.0 : 0.0;
    t3[0] = t3[1] = t3[2] = 0.0;
    if (count < modelPoints) return 0;
    CvRng rng(~0ull);
    int niters = iterationsCount > 1 ? iterationsCount : 1;
    int maxGood = 0;
    double bestR[9], bestT[3];
    std::vector<uint8_t> mask(count), bestMask(count, 0);
    if (count == modelPoints) {   // runKernel once, every point an inlier (ptsetreg.cpp)
        double pw[15], us[10];
        for (int i = 0; i < 15; i++) pw[i] = p3[i];
        for (int i = 0; i < 10; i++) us[i] = p2[i];
        if (!epnp(5, pw, us, K, bestR, bestT)) return 0;
        for (int i = 0; i < count; i++) bestMask[i] = 1;
        maxGood = count;
        niters = 0;
    }
    const float thr = (float)((double)reprojectionError * (double)reprojectionError);
    int iter;
    for (iter = 0; iter < niters; iter++) {
        int idx[5];
        {
            for (int i = 0; i < modelPoints; i++) {
                for (;;) {
                    const int v = rng.uniform(0, count);
                    int j;
                    for (j = 0; j < i; j++)
                        if (idx[j] == v) break;
                    if (j == i) { idx[i] = v; break; }
                }
            }
        }
        double pw[15], us[10];
        for (int i = 0; i < 5; i++) {
            for (int j = 0; j < 3; j++) pw[3 * i + j] = p3[3 * idx[i] + j];
            for (int j = 0; j < 2; j++) us[2 * i + j] = p2[2 * idx[i] + j];
        }
        double R[9], t[3];
        if (!epnp(5, pw, us, K, R, t)) continue;
        int good = 0;
        for (int i = 0; i < count; i++) {
            const float e = reproj_err2(p3 + 3 * i, p2 + 2 * i, R, t, K);
            mask[i] = e <= thr ? 1 : 0;
            good += mask[i];
        }
        if (good > (maxGood > modelPoints - 1 ? maxGood : modelPoints - 1)) {
            bestMask = mask;
            std::memcpy(bestR, R, sizeof(R));
            std::memcpy(bestT, t, sizeof(t));
            maxGood = good;
            niters = update_num_iters(confidence, (double)(count - good) / count, modelPoints, niters);
        }
    }
    *iters_run = iter;
    if (maxGood <= 0) return 0;
    // refinement on the RANSAC inliers: 10 Gauss-Newton steps, device reduction order
    double R[9], t[3];
    std::memcpy(R, bestR, sizeof(R));
    std::memcpy(t, bestT, sizeof(t));
    std::vector<int> inl;
    for (int i = 0; i < count; i++)
        if (bestMask[i]) inl.push_back(i);
    const int nI = (int)inl.size();
    for (int it = 0; it < g_refine_iters; it++) {
        double lane[256][27];
        for (int l = 0; l < 256; l++)
            for (int k = 0; k < 27; k++) lane[l][k] = 0.0;
        for (int l = 0; l < 256; l++)
            for (int i = l; i < nI; i += 256) {
                double term[27];
                gn_terms(p3 + 3 * inl[i], p2 + 2 * inl[i], R, t, K, term);
                for (int k = 0; k < 27; k++) lane[l][k] += term[k];
            }
        // balanced binary tree over the lanes in natural order: blocks of 2, 4, ..., 256 lanes,
        // each the sum of its left and right halves
        for (int s = 1; s < 256; s <<= 1)
            for (int l = 0; l < 256; l += 2 * s)
                for (int k = 0; k < 27; k++) lane[l][k] += lane[l + s][k];
        double H[36], g[6], dx[6];
        int k = 0;
        for (int a = 0; a < 6; a++)
            for (int b = a; b < 6; b++) { H[a * 6 + b] = lane[0][k]; H[b * 6 + a] = lane[0][k]; k++; }
        for (int a = 0; a < 6; a++) g[a] = lane[0][k++];
        if (!solve6(H, g, dx)) break;
        double dR[9];
        rodrigues_exp(dx, dR);
        double Rn[9], tn[3];
        for (int a = 0; a < 3; a++) {
            for (int b = 0; b < 3; b++)
                Rn[a * 3 + b] = (dR[a * 3 + 0] * R[0 * 3 + b] + dR[a * 3 + 1] * R[1 * 3 + b]) + dR[a * 3 + 2] * R[2 * 3 + b];
            tn[a] = ((dR[a * 3 + 0] * t[0] + dR[a * 3 + 1] * t[1]) + dR[a * 3 + 2] * t[2]) + dx[3 + a];
        }
        std::memcpy(R, Rn, sizeof(R));
        std::memcpy(t, tn, sizeof(t));
    }
    std::memcpy(R9, R, sizeof(R));
    std::memcpy(t3, t, sizeof(t));
    for (int i = 0; i < count; i++) inlier_mask[i] = bestMask[i];
    *n_inliers = maxGood;
    return 1;
}

}  // extern "C"

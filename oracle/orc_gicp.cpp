// orc_gicp.cpp -- ORACLE (test infrastructure only; see rgbd_oracle.h header).
//
// Gicp::compute / align (Solver/Gicp.cpp:21-66), called from Tracking::visualOdometry when
// RansacSE3's rmse >= 0.8 (System/Tracking.cpp:145-151) with max correspondence distance 0.07 and
// 10 iterations.  The clouds are the RANSAC inlier pairs: source = F1 mvKeys3Dc[queryIdx], target =
// F2 mvKeys3Dc[trainIdx] (Gicp::createCloudsFromMatches :37-52).  PCL is absent; this restates
// pcl::GeneralizedIterativeClosestPoint<PointXYZ, PointXYZ> (PCL 1.8) -- see DESIGN.md "GICP":
//   * computeCovariances: k = 20 nearest neighbours of every point in its own cloud (exact, ties
//     by index; the kd-tree's order is ascending distance), mean / covariance accumulated in double
//     from float products, Eigen JacobiSVD U, covariance rebuilt with singular values (1, 1, eps);
//   * computeTransformation: output = guess * source (float); per outer iteration the 1-NN of
//     transformation_ * output[i] in the target (float squared distance, ties by index), a
//     correspondence when nn_dist < max_corr^2, Mahalanobis M_i = (R C1_i R^T + C2_nn)^-1 (Eigen
//     3 x 3 cofactor inverse) with R = rot(transformation_ * guess) in double;
//   * the per-iteration optimiser (PCL: BFGS) is DEFINED as gn_iterations Gauss-Newton steps on
//     sum r_i^T M_i r_i with a left SE(3) increment, J^T M J / J^T M r accumulated in 256 strided
//     lanes + a binary tree (the device order), 6 x 6 solve with partial pivoting;
//   * fewer than 4 correspondences -> PCL's NotEnoughPointsException -> not converged; delta =
//     max(|dR| / rotation_eps, |dt| / transformation_eps) over the float matrices; converged when
//     iterations >= max or delta < 1; final = transformation_ * guess (float).
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "orc_common.h"
#include "rgbd_oracle.h"

namespace {

// FLANN L2_Simple<float>: ((0 + dx^2) + dy^2) + dz^2 in float
inline float dist2f(const float* a, const float* b)
{
    const float dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
    float r = 0.0f;
    r = r + dx * dx;
    r = r + dy * dy;
    r = r + dz * dz;
    return r;
}

// k nearest (ascending distance, ties by index) of point q among pts[0..n)
void knn(const float* pts, int n, const float* q, int k, int* out)
{
    std::vector<std::pair<float, int>> best;   // sorted ascending by (d, idx)
    best.reserve(k + 1);
    for (int j = 0; j < n; j++) {
        const float d = dist2f(q, pts + 3 * j);
        if ((int)best.size() == k && !(d < best.back().first)) continue;   // ties: the earlier index stays
        size_t pos = best.size();
        while (pos > 0 && d < best[pos - 1].first) pos--;
        best.insert(best.begin() + pos, {d, j});
        if ((int)best.size() > k) best.pop_back();
    }
    for (int i = 0; i < k; i++) out[i] = best[i].second;
}

// PCL computeCovariances for one point: cov (row-major 3 x 3 double)
void covariance(const float* pts, int n, int i, int k, double eps, double* C)
{
    std::vector<int> nn(k);
    knn(pts, n, pts + 3 * i, k, nn.data());
    double mean[3] = {0, 0, 0};
    double cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int j = 0; j < k; j++) {
        const float* p = pts + 3 * nn[j];
        mean[0] += p[0];
        mean[1] += p[1];
        mean[2] += p[2];
        cov[0][0] += p[0] * p[0];
        cov[1][0] += p[1] * p[0];
        cov[1][1] += p[1] * p[1];
        cov[2][0] += p[2] * p[0];
        cov[2][1] += p[2] * p[1];
        cov[2][2] += p[2] * p[2];
    }
    for (int a = 0; a < 3; a++) mean[a] /= (double)k;
    for (int a = 0; a < 3; a++)
        for (int b = 0; b <= a; b++) {
            cov[a][b] /= (double)k;
            cov[a][b] -= mean[a] * mean[b];
            cov[b][a] = cov[a][b];
        }
    double A[9], U[9], S[3], V[9];
    for (int r = 0; r < 9; r++) A[r] = cov[r / 3][r % 3];
    orc_svd3(A, U, S, V);
    double out[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int c = 0; c < 3; c++) {
        const double v = (c == 2) ? eps : 1.0;
        double col[3] = {U[0 * 3 + c], U[1 * 3 + c], U[2 * 3 + c]};
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) out[a * 3 + b] += (v * col[a]) * col[b];
    }
    std::memcpy(C, out, sizeof(out));
}

// Eigen 3.3 compute_inverse<3>: result(r, c) = cofactor(c, r) / det, det = sum cofactor(i,0) m(i,0)
inline double cof(const double* m, int i, int j)
{
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m[i1 * 3 + j1] * m[i2 * 3 + j2] - m[i1 * 3 + j2] * m[i2 * 3 + j1];
}

void inverse3(const double* m, double* r)
{
    const double c0 = cof(m, 0, 0), c1 = cof(m, 1, 0), c2 = cof(m, 2, 0);
    const double det = (c0 * m[0] + c1 * m[3]) + c2 * m[6];
    const double invdet = 1.0 / det;
    r[0] = c0 * invdet;
    r[1] = c1 * invdet;
    r[2] = c2 * invdet;
    r[3] = cof(m, 0, 1) * invdet;
    r[4] = cof(m, 1, 1) * invdet;
    r[5] = cof(m, 2, 1) * invdet;
    r[6] = cof(m, 0, 2) * invdet;
    r[7] = cof(m, 1, 2) * invdet;
    r[8] = cof(m, 2, 2) * invdet;
}

// float 4x4 (row-major) times (x, y, z, 1): ((m0 x + m1 y) + m2 z) + m3
inline void xform_f(const float* T, const float* p, float* o)
{
    for (int r = 0; r < 3; r++) o[r] = ((T[4 * r] * p[0] + T[4 * r + 1] * p[1]) + T[4 * r + 2] * p[2]) + T[4 * r + 3];
}

// Eigen Matrix4f product, k order: ((a0 b0 + a1 b1) + a2 b2) + a3 b3
void matmul4f(const float* A, const float* B, float* C)
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            C[4 * i + j] = ((A[4 * i] * B[j] + A[4 * i + 1] * B[4 + j]) + A[4 * i + 2] * B[8 + j]) + A[4 * i + 3] * B[12 + j];
}

// one correspondence's J^T M J (21, upper triangle) and J^T M r (6); J = [-[y]x | I], r = y - q
void gn_terms(const double* y, const double* q, const double* M, double out[27])
{
    const double r[3] = {y[0] - q[0], y[1] - q[1], y[2] - q[2]};
    const double J[3][6] = {{0.0, y[2], -y[1], 1.0, 0.0, 0.0},
                            {-y[2], 0.0, y[0], 0.0, 1.0, 0.0},
                            {y[1], -y[0], 0.0, 0.0, 0.0, 1.0}};
    double Mr[3], MJ[3][6];
    for (int a = 0; a < 3; a++) {
        Mr[a] = (M[a * 3] * r[0] + M[a * 3 + 1] * r[1]) + M[a * 3 + 2] * r[2];
        for (int b = 0; b < 6; b++) MJ[a][b] = (M[a * 3] * J[0][b] + M[a * 3 + 1] * J[1][b]) + M[a * 3 + 2] * J[2][b];
    }
    int k = 0;
    for (int a = 0; a < 6; a++)
        for (int b = a; b < 6; b++) out[k++] = (J[0][a] * MJ[0][b] + J[1][a] * MJ[1][b]) + J[2][a] * MJ[2][b];
    for (int a = 0; a < 6; a++) out[k++] = (J[0][a] * Mr[0] + J[1][a] * Mr[1]) + J[2][a] * Mr[2];
}

constexpr int kLanes = 256;

}  // namespace

extern "C" {

int orc_gicp_covariances(const float* pts, int n, int k, double eps, double* cov /* n x 9 */)
{
    if (n < k) return 0;
    for (int i = 0; i < n; i++) covariance(pts, n, i, k, eps, cov + 9 * i);
    return 1;
}

int orc_gicp(const float* src, const float* tgt, int M, const float* guess, const orc_gicp_params* prm, float* T_out,
             int32_t* converged, int32_t* iters, int32_t* n_corr)
{
    for (int i = 0; i < 16; i++) T_out[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    *converged = 0;
    *iters = 0;
    if (n_corr) *n_corr = 0;
    const int k = prm->k_correspondences;
    if (M < k || M < 1) return 0;
    std::vector<double> C1(9 * (size_t)M), C2(9 * (size_t)M);
    orc_gicp_covariances(tgt, M, k, prm->gicp_epsilon, C2.data());
    orc_gicp_covariances(src, M, k, prm->gicp_epsilon, C1.data());
    std::vector<float> out(3 * (size_t)M);
    for (int i = 0; i < M; i++) xform_f(guess, src + 3 * i, &out[3 * i]);
    float T[16], prev[16];
    for (int i = 0; i < 16; i++) T[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    const double thr = prm->max_corr_dist * prm->max_corr_dist;
    std::vector<int> nn(M);
    std::vector<char> has(M);
    std::vector<double> Mi(9 * (size_t)M);
    int it = 0;
    bool conv = false;
    while (!conv) {
        // R = rot(transformation_ * guess), double accumulation in k order
        double Rg[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                double s = 0.0;
                for (int kk = 0; kk < 4; kk++) s += (double)T[4 * i + kk] * (double)guess[4 * kk + j];
                Rg[3 * i + j] = s;
            }
        int cnt = 0;
        for (int i = 0; i < M; i++) {
            float qv[3];
            xform_f(T, &out[3 * i], qv);
            int best = 0;
            float bd = dist2f(qv, tgt);
            for (int j = 1; j < M; j++) {
                const float d = dist2f(qv, tgt + 3 * j);
                if (d < bd) { bd = d; best = j; }
            }
            has[i] = (double)bd < thr;
            nn[i] = best;
            if (!has[i]) continue;
            cnt++;
            // M = R C1, temp = M R^T + C2, M_i = temp^-1
            const double* c1 = &C1[9 * (size_t)i];
            const double* c2 = &C2[9 * (size_t)best];
            double RC[9], tmp[9];
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) RC[3 * a + b] = (Rg[3 * a] * c1[b] + Rg[3 * a + 1] * c1[3 + b]) + Rg[3 * a + 2] * c1[6 + b];
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++)
                    tmp[3 * a + b] = ((RC[3 * a] * Rg[3 * b] + RC[3 * a + 1] * Rg[3 * b + 1]) + RC[3 * a + 2] * Rg[3 * b + 2]) + c2[3 * a + b];
            inverse3(tmp, &Mi[9 * (size_t)i]);
        }
        if (n_corr) *n_corr = cnt;
        std::memcpy(prev, T, sizeof(T));
        if (cnt < 4) break;   // NotEnoughPointsException: the loop ends without convergence
        // Gauss-Newton on the fixed correspondences, from the current transformation_
        double Rd[9], td[3];
        for (int a = 0; a < 3; a++) {
            for (int b = 0; b < 3; b++) Rd[3 * a + b] = (double)T[4 * a + b];
            td[a] = (double)T[4 * a + 3];
        }
        for (int g = 0; g < prm->gn_iterations; g++) {
            static double lane[kLanes][27];
            for (int l = 0; l < kLanes; l++)
                for (int kk = 0; kk < 27; kk++) lane[l][kk] = 0.0;
            for (int i = 0; i < M; i++) {
                if (!has[i]) continue;
                const double p[3] = {(double)out[3 * i], (double)out[3 * i + 1], (double)out[3 * i + 2]};
                double y[3];
                for (int a = 0; a < 3; a++) y[a] = ((Rd[3 * a] * p[0] + Rd[3 * a + 1] * p[1]) + Rd[3 * a + 2] * p[2]) + td[a];
                const float* qt = tgt + 3 * nn[i];
                const double q[3] = {(double)qt[0], (double)qt[1], (double)qt[2]};
                double term[27];
                gn_terms(y, q, &Mi[9 * (size_t)i], term);
                for (int kk = 0; kk < 27; kk++) lane[i % kLanes][kk] += term[kk];
            }
            for (int sd = kLanes / 2; sd > 0; sd >>= 1)
                for (int l = 0; l < sd; l++)
                    for (int kk = 0; kk < 27; kk++) lane[l][kk] += lane[l + sd][kk];
            double H[36], gv[6], dx[6];
            int kk = 0;
            for (int a = 0; a < 6; a++)
                for (int b = a; b < 6; b++) { H[a * 6 + b] = lane[0][kk]; H[b * 6 + a] = lane[0][kk]; kk++; }
            for (int a = 0; a < 6; a++) gv[a] = lane[0][kk++];
            if (!orc::solve6(H, gv, dx)) break;
            double dR[9], Rn[9], tn[3];
            orc::rodrigues_exp(dx, dR);
            for (int a = 0; a < 3; a++) {
                for (int b = 0; b < 3; b++)
                    Rn[3 * a + b] = (dR[3 * a] * Rd[b] + dR[3 * a + 1] * Rd[3 + b]) + dR[3 * a + 2] * Rd[6 + b];
                tn[a] = ((dR[3 * a] * td[0] + dR[3 * a + 1] * td[1]) + dR[3 * a + 2] * td[2]) + dx[3 + a];
            }
            std::memcpy(Rd, Rn, sizeof(Rd));
            std::memcpy(td, tn, sizeof(td));
        }
        for (int a = 0; a < 3; a++) {
            for (int b = 0; b < 3; b++) T[4 * a + b] = (float)Rd[3 * a + b];
            T[4 * a + 3] = (float)td[a];
        }
        double delta = 0.0;
        for (int a = 0; a < 4; a++)
            for (int b = 0; b < 4; b++) {
                const double ratio = (a < 3 && b < 3) ? 1.0 / prm->rotation_epsilon : 1.0 / prm->transformation_epsilon;
                const double cd = ratio * (double)std::fabs(prev[4 * a + b] - T[4 * a + b]);
                if (cd > delta) delta = cd;
            }
        it++;
        if (it >= prm->max_iterations || delta < 1) {
            conv = true;
            std::memcpy(prev, T, sizeof(T));
        }
    }
    *iters = it;
    if (!conv) return 0;
    *converged = 1;
    matmul4f(prev, guess, T_out);
    return 1;
}

// Gicp::compute (Solver/Gicp.cpp:21-35): < 20 matches -> false; not converged -> identity -> false;
// Eigen isIdentity (float dummy precision 1e-5) -> false
int orc_gicp_compute(const float* src, const float* tgt, int M, const float* guess, const orc_gicp_params* prm,
                     float* T_out)
{
    for (int i = 0; i < 16; i++) T_out[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    if (M < 20) return 0;
    int32_t conv = 0, it = 0;
    orc_gicp(src, tgt, M, guess, prm, T_out, &conv, &it, nullptr);
    if (!conv) {
        for (int i = 0; i < 16; i++) T_out[i] = (i % 5 == 0) ? 1.0f : 0.0f;
        return 0;
    }
    const float prec = 1e-5f;
    bool ident = true;
    for (int i = 0; i < 4 && ident; i++)
        for (int j = 0; j < 4; j++) {
            const float c = T_out[4 * i + j];
            if (i == j) {
                if (!(std::fabs(c - 1.0f) <= prec * std::fmin(std::fabs(c), 1.0f))) { ident = false; break; }
            } else if (!(std::fabs(c) <= prec)) {
                ident = false;
                break;
            }
        }
    return ident ? 0 : 1;
}

}  // extern "C"

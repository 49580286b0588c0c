// orc_solver.cpp -- ORACLE (test infrastructure only; see rgbd_oracle.h header).
//
// Scalar restatement of the reference Matcher and RansacSE3:
//   Features/Matcher.cpp:106-139 (knn-2 + ratio + dedup + outlier + depth filters)
//   Solver/SolverSE3.cpp:23-297 (RansacSE3), System/Random.cpp:7-20 (rand wrapper)
// External semantics restated (not in /root/reference; DESIGN.md "Oracle definitions"):
//   OpenCV BFMatcher::knnMatch / batchDistance(K=2) insertion rule,
//   glibc srand/rand (random_r TYPE_3), libstdc++ std::sort (called for real),
//   PCL TransformationFromCorrespondences (online f32 update + f64 JacobiSVD),
//   Eigen 3.3 JacobiSVD<Matrix3d> (2x2 real Jacobi sweeps) and LLT<Matrix3d>.
// No FMA contraction anywhere (-ffp-contract=off).
#include "rgbd_oracle.h"

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstring>
#include <limits>
#include <set>
#include <vector>

namespace {

inline int popcnt32(uint32_t v) { return __builtin_popcount(v); }

int hamming(const uint8_t* a, const uint8_t* b)
{
    int d = 0;
    for (int i = 0; i < 32; i += 4) {
        uint32_t x, y;
        std::memcpy(&x, a + i, 4);
        std::memcpy(&y, b + i, 4);
        d += popcnt32(x ^ y);
    }
    return d;
}

struct DMatch {
    int queryIdx, trainIdx, imgIdx;
    float distance;
    bool operator<(const DMatch& m) const { return distance < m.distance; }   // cv::DMatch::operator<
};

// ------------------------------------------------------------------ glibc rand
void rng_seed(orc_rng* st, uint32_t seed)
{
    if (seed == 0)
        seed = 1;
    st->state[0] = (int32_t)seed;
    int32_t word = (int32_t)seed;
    for (int i = 1; i < 31; ++i) {
        long hi = word / 127773;
        long lo = word % 127773;
        word = (int32_t)(16807 * lo - 2836 * hi);
        if (word < 0)
            word += 2147483647;
        st->state[i] = word;
    }
    st->f = 3;
    st->r = 0;
    for (int k = 0; k < 310; k++)
        orc_rng_rand(st);
}

// ------------------------------------------------------------------ Eigen 3x3 SVD
struct JRot { double c, s; };

// apply_rotation_in_the_plane(x, y, j): x' = c x + s y ; y' = -s x + c y
inline void rot_rows(double A[3][3], int p, int q, JRot j)
{
    if (j.c == 1.0 && j.s == 0.0) return;
    for (int i = 0; i < 3; i++) {
        const double xi = A[p][i], yi = A[q][i];
        A[p][i] = j.c * xi + j.s * yi;
        A[q][i] = -j.s * xi + j.c * yi;
    }
}
inline void rot_cols(double A[3][3], int p, int q, JRot j)   // applyOnTheRight(p,q,j): uses j.transpose()
{
    const JRot t{j.c, -j.s};
    if (t.c == 1.0 && t.s == 0.0) return;
    for (int i = 0; i < 3; i++) {
        const double xi = A[i][p], yi = A[i][q];
        A[i][p] = t.c * xi + t.s * yi;
        A[i][q] = -t.s * xi + t.c * yi;
    }
}

JRot make_jacobi(double x, double y, double z)
{
    const double deno = 2.0 * std::fabs(y);
    if (deno < DBL_MIN)
        return JRot{1.0, 0.0};
    const double tau = (x - z) / deno;
    const double w = std::sqrt(tau * tau + 1.0);
    double t;
    if (tau > 0.0)
        t = 1.0 / (tau + w);
    else
        t = 1.0 / (tau - w);
    const double sign_t = t > 0.0 ? 1.0 : -1.0;
    const double n = 1.0 / std::sqrt(t * t + 1.0);
    JRot r;
    r.s = -sign_t * (y / std::fabs(y)) * std::fabs(t) * n;
    r.c = n;
    return r;
}

void real_2x2_jacobi_svd(const double A[3][3], int p, int q, JRot* jl, JRot* jr)
{
    double m[2][2] = {{A[p][p], A[p][q]}, {A[q][p], A[q][q]}};
    JRot rot1;
    const double t = m[0][0] + m[1][1];
    const double d = m[1][0] - m[0][1];
    if (std::fabs(d) < DBL_MIN) {
        rot1.s = 0.0;
        rot1.c = 1.0;
    } else {
        const double u = t / d;
        const double tmp = std::sqrt(1.0 + u * u);
        rot1.s = 1.0 / tmp;
        rot1.c = u / tmp;
    }
    if (!(rot1.c == 1.0 && rot1.s == 0.0)) {
        for (int i = 0; i < 2; i++) {
            const double xi = m[0][i], yi = m[1][i];
            m[0][i] = rot1.c * xi + rot1.s * yi;
            m[1][i] = -rot1.s * xi + rot1.c * yi;
        }
    }
    *jr = make_jacobi(m[0][0], m[0][1], m[1][1]);
    const JRot jt{jr->c, -jr->s};
    jl->c = rot1.c * jt.c - rot1.s * jt.s;
    jl->s = rot1.c * jt.s + rot1.s * jt.c;
}

void svd3(const double M[3][3], double U[3][3], double S[3], double V[3][3])
{
    const double precision = 2.0 * DBL_EPSILON;
    const double considerAsZero = DBL_MIN;
    double scale = 0.0;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++)
            scale = std::max(scale, std::fabs(M[i][j]));
    if (!std::isfinite(scale)) {   // Eigen 3.3: InvalidInput; defined here as NaN factors
        for (int i = 0; i < 3; i++) {
            S[i] = NAN;
            for (int j = 0; j < 3; j++) U[i][j] = V[i][j] = NAN;
        }
        return;
    }
    if (scale == 0.0)
        scale = 1.0;
    double W[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            W[i][j] = M[i][j] / scale;
            U[i][j] = V[i][j] = (i == j) ? 1.0 : 0.0;
        }
    double maxDiag = std::max(std::max(std::fabs(W[0][0]), std::fabs(W[1][1])), std::fabs(W[2][2]));
    bool finished = false;
    int sweeps = 0;
    while (!finished && sweeps < 64) {
        finished = true;
        sweeps++;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                const double threshold = std::max(considerAsZero, precision * maxDiag);
                if (std::fabs(W[p][q]) > threshold || std::fabs(W[q][p]) > threshold) {
                    finished = false;
                    JRot jl, jr;
                    real_2x2_jacobi_svd(W, p, q, &jl, &jr);
                    rot_rows(W, p, q, jl);
                    rot_cols(U, p, q, JRot{jl.c, -jl.s});
                    rot_cols(W, p, q, jr);
                    rot_cols(V, p, q, jr);
                    maxDiag = std::max(maxDiag, std::max(std::fabs(W[p][p]), std::fabs(W[q][q])));
                }
            }
    }
    for (int i = 0; i < 3; i++) {
        const double a = W[i][i];
        S[i] = std::fabs(a);
        if (a < 0.0)
            for (int r = 0; r < 3; r++) U[r][i] = -U[r][i];
    }
    for (int i = 0; i < 3; i++) S[i] *= scale;
    for (int i = 0; i < 3; i++) {
        int pos = i;
        double mx = S[i];
        for (int j = i + 1; j < 3; j++)
            if (S[j] > mx) { mx = S[j]; pos = j; }
        if (mx == 0.0)
            break;
        if (pos != i) {
            std::swap(S[i], S[pos]);
            for (int r = 0; r < 3; r++) {
                std::swap(U[r][i], U[r][pos]);
                std::swap(V[r][i], V[r][pos]);
            }
        }
    }
}

double det3(const double m[3][3])
{
    // Eigen determinant_impl<3>: bruteforce_det3_helper(0,1,2) - (1,0,2) + (2,0,1)
    auto h = [&](int a, int b, int c) { return m[0][a] * (m[1][b] * m[2][c] - m[1][c] * m[2][b]); };
    return h(0, 1, 2) - h(1, 0, 2) + h(2, 0, 1);
}

// ------------------------------------------------------------------ PCL TFC
struct TFC {
    float acc = 0.0f;
    float mean1[3] = {0, 0, 0}, mean2[3] = {0, 0, 0};
    float cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    void add(const float p[3], const float q[3], float weight)
    {
        if (weight == 0.0f)
            return;
        acc += weight;
        const float alpha = weight / acc;
        float d1[3], d2[3];
        for (int i = 0; i < 3; i++) { d1[i] = p[i] - mean1[i]; d2[i] = q[i] - mean2[i]; }
        const float oma = 1.0f - alpha;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                // Eigen 3.3 rewrites alpha*(d2*d1^T) as (alpha*d2)*d1^T (ProductEvaluators.h)
                const float outer = d1[j] * (alpha * d2[i]);
                cov[i][j] = oma * (cov[i][j] + outer);
            }
        for (int i = 0; i < 3; i++) {
            mean1[i] += alpha * d1[i];
            mean2[i] += alpha * d2[i];
        }
    }
    void transformation(float T[16]) const
    {
        double C[3][3], U[3][3], S[3], V[3][3];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) C[i][j] = (double)cov[i][j];
        svd3(C, U, S, V);
        double s[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
        if (det3(U) * det3(V) < 0.0f)
            s[2][2] = -1.0;
        double us[3][3], r[3][3];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                us[i][j] = (U[i][0] * s[0][j] + U[i][1] * s[1][j]) + U[i][2] * s[2][j];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++)
                r[i][j] = (us[i][0] * V[j][0] + us[i][1] * V[j][1]) + us[i][2] * V[j][2];
        for (int i = 0; i < 3; i++) {
            const float rf0 = (float)r[i][0], rf1 = (float)r[i][1], rf2 = (float)r[i][2];
            const float rm = (rf0 * mean1[0] + rf1 * mean1[1]) + rf2 * mean1[2];
            T[4 * i + 0] = rf0; T[4 * i + 1] = rf1; T[4 * i + 2] = rf2;
            T[4 * i + 3] = mean2[i] - rm;
        }
        T[12] = 0.0f; T[13] = 0.0f; T[14] = 0.0f; T[15] = 1.0f;
    }
};

// ------------------------------------------------------------------ errorFunction2
struct Consts { double rcx, rcy; };
Consts raster_consts()
{
    // Solver/SolverSE3.cpp:218-225
    const double cam_angle_x = 58.0 / 180.0 * M_PI;
    const double cam_angle_y = 45.0 / 180.0 * M_PI;
    const double cam_resol_x = 640, cam_resol_y = 480;
    const double sx = 3 * std::tan(cam_angle_x / cam_resol_x);
    const double sy = 3 * std::tan(cam_angle_y / cam_resol_y);
    return Consts{sx * sx, sy * sy};
}

double error_function2(const float x1f[3], const float x2f[3], const double T[4][4], double C, const Consts& k)
{
    if (std::isnan(x1f[2]) || std::isnan(x2f[2]))
        return std::numeric_limits<double>::max();
    const double x1[4] = {x1f[0], x1f[1], x1f[2], 1.0};
    const double mu2[3] = {x2f[0], x2f[1], x2f[2]};
    double m1f2[3];
    for (int i = 0; i < 3; i++)
        m1f2[i] = ((T[i][0] * x1[0] + T[i][1] * x1[1]) + T[i][2] * x1[2]) + T[i][3] * x1[3];
    double d[3];
    for (int i = 0; i < 3; i++) d[i] = m1f2[i] - mu2[i];
    const double dsq = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
    const double smax = std::max(k.rcx, C);
    if (dsq > 2.0 * (smax + smax))
        return std::numeric_limits<double>::max();
    const double c1[3] = {k.rcx * x1[2], k.rcy * x1[2], C};
    const double c2[3] = {k.rcx * mu2[2], k.rcy * mu2[2], C};
    // cov1_in_frame_2 = R^T * cov1 * R  (evaluated as (R^T cov1) R, zeros included)
    double M[3][3], S[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            const double a0 = T[0][i] * (j == 0 ? c1[0] : 0.0);
            const double a1 = T[1][i] * (j == 1 ? c1[1] : 0.0);
            const double a2 = T[2][i] * (j == 2 ? c1[2] : 0.0);
            M[i][j] = (a0 + a1) + a2;
        }
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            const double v = (M[i][0] * T[0][j] + M[i][1] * T[1][j]) + M[i][2] * T[2][j];
            S[i][j] = v + (i == j ? c2[i] : 0.0);
        }
    if (std::isnan(d[2]))
        return std::numeric_limits<double>::max();
    // Eigen LLT<Matrix3d> (lower, unblocked, in place) + solve
    double L[3][3];
    std::memcpy(L, S, sizeof(L));
    for (int kk = 0; kk < 3; ++kk) {
        double x = L[kk][kk];
        if (kk == 1) x -= L[1][0] * L[1][0];
        if (kk == 2) x -= L[2][0] * L[2][0] + L[2][1] * L[2][1];
        if (x <= 0.0)
            break;
        L[kk][kk] = x = std::sqrt(x);
        if (kk == 1)
            L[2][1] -= L[2][0] * L[1][0];
        for (int r = kk + 1; r < 3; r++) L[r][kk] /= x;
    }
    // solveInPlace with Eigen's triangular_solver_unroller (fixed size <= 8): row oriented,
    // forward on L then backward on L^T, sums of products formed before the subtraction.
    double y[3];
    y[0] = d[0] / L[0][0];
    y[1] = (d[1] - L[1][0] * y[0]) / L[1][1];
    y[2] = (d[2] - (L[2][0] * y[0] + L[2][1] * y[1])) / L[2][2];
    y[2] = y[2] / L[2][2];
    y[1] = (y[1] - L[2][1] * y[2]) / L[1][1];
    y[0] = (y[0] - (L[1][0] * y[1] + L[2][0] * y[2])) / L[0][0];
    const double sq = (d[0] * y[0] + d[1] * y[1]) + d[2] * y[2];
    if (!(sq >= 0.0))
        return std::numeric_limits<double>::max();
    return sq;
}

struct Ransac {
    const float* xyz1;
    const float* xyz2;
    orc_ransac_params prm;
    orc_rng* rng;
    orc_sticky* sticky;
    Consts k;

    double cov()
    {
        // depthCovariance: function-static, initialised by the first call in the process
        return sticky->cov;
    }
    void touch(double depth)
    {
        if (!sticky->set) {
            const double stddev = 0.01 * depth * depth;
            sticky->cov = stddev * stddev;
            sticky->set = 1;
        }
    }
    int randomInt(int mn, int mx) { return orc_random_int(rng, mn, mx); }
    std::vector<DMatch> sample(const std::vector<DMatch>& v)
    {
        std::set<size_t> ids;
        int safety = 0;
        while (ids.size() < prm.sample_size && v.size() >= prm.sample_size) {
            int id1 = randomInt(0, (int)v.size() - 1);
            int id2 = randomInt(0, (int)v.size() - 1);
            if (id1 > id2)
                id1 = id2;
            ids.insert(id1);
            if (++safety > 10000)
                break;
        }
        std::vector<DMatch> out;
        for (size_t id : ids) out.push_back(v[id]);
        return out;
    }
    void fit(const std::vector<DMatch>& v, float T[16])
    {
        TFC t;
        for (const DMatch& m : v) {
            const float* from = xyz1 + 3 * m.queryIdx;
            const float* to = xyz2 + 3 * m.trainIdx;
            if (std::isnan(from[2]) || std::isnan(to[2]))
                continue;
            const float w = 1.0f / (from[2] * to[2]);
            t.add(from, to, w);
        }
        t.transformation(T);
    }
    double inliers_and_error(const std::vector<DMatch>& m12, const float Tf[16], std::vector<DMatch>& inl)
    {
        inl.clear();
        double meanError = 0.0;
        double T[4][4];
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) T[i][j] = (double)Tf[4 * i + j];
        const float maxd = prm.max_mahalanobis * prm.max_mahalanobis;
        for (const DMatch& m : m12) {
            const float* o = xyz1 + 3 * m.queryIdx;
            const float* t = xyz2 + 3 * m.trainIdx;
            if (o[2] == 0.0f || t[0] == 0.0f)
                continue;
            if (!std::isnan(o[2]) && !std::isnan(t[2]))
                touch((double)o[2]);
            const double md = error_function2(o, t, T, cov(), k);
            if (md > (double)maxd)
                continue;
            if (!(md >= 0.0))
                continue;
            meanError += md;
            inl.push_back(m);
        }
        if (inl.size() < 3)
            meanError = 1e9;
        else {
            meanError /= inl.size();
            meanError = std::sqrt(meanError);
        }
        return meanError;
    }
};

}  // namespace

extern "C" {

void orc_knn2(const uint8_t* dq, int nq, const uint8_t* dt, int nt, int32_t* out)
{
    // BFMatcher::knnMatch(k=2) -> batchDistance(K=2, CV_32S): strict '<' insertion,
    // equal distances keep the lower train index first.
    for (int q = 0; q < nq; q++) {
        int dist[2] = {INT_MAX, INT_MAX}, idx[2] = {-1, -1};
        for (int j = 0; j < nt; j++) {
            const int d = hamming(dq + 32 * (size_t)q, dt + 32 * (size_t)j);
            if (d < dist[1]) {
                int k = 0;
                for (k = 0; k >= 0 && dist[k] > d; k--) {
                    idx[k + 1] = idx[k];
                    dist[k + 1] = dist[k];
                }
                idx[k + 1] = j;
                dist[k + 1] = d;
            }
        }
        out[4 * q + 0] = dist[0]; out[4 * q + 1] = idx[0];
        out[4 * q + 2] = dist[1]; out[4 * q + 3] = idx[1];
    }
}

int orc_match(const uint8_t* dq, int nq, const uint8_t* dt, int nt, const uint8_t* outlier_q, const float* z_q,
              const float* z_t, float nnratio, int discard_outliers, orc_dmatch* out)
{
    // Matcher::match, Features/Matcher.cpp:106-139
    if (nq <= 0 || nt <= 0)
        return 0;
    std::vector<int32_t> knn((size_t)nq * 4);
    orc_knn2(dq, nq, dt, nt, knn.data());
    std::set<int> trainIdxs;
    int m = 0;
    for (int i = 0; i < nq; i++) {
        const int i2b = knn[4 * i + 3];
        if (i2b < 0)
            continue;   // <2 train descriptors: reference indexes matchesKnn[i][1] (UB); defined as skip
        const float d1 = (float)knn[4 * i + 0], d2 = (float)knn[4 * i + 2];
        if (d1 < nnratio * d2) {
            const int i1 = i;
            const int i2 = knn[4 * i + 1];
            if (trainIdxs.count(i2))
                continue;
            if (discard_outliers && outlier_q && outlier_q[i1])
                continue;
            if (!(z_q[i1] > 0) || !(z_t[i2] > 0))   // Frame::isValidObs, Core/Frame.cpp:415-418
                continue;
            trainIdxs.insert(i2);
            out[m].queryIdx = i1;
            out[m].trainIdx = i2;
            out[m].imgIdx = 0;
            out[m].distance = d1;
            m++;
        }
    }
    return m;
}

void orc_rng_seed(orc_rng* st, uint32_t seed) { rng_seed(st, seed); }

// Random::randomInt (System/Random.cpp:16-21) on the restated rand(); pinned against the reference's own
// Random.cpp compiled into oracle/_ref (tests/test_oracle_ref.py)
int orc_random_int(orc_rng* st, int mn, int mx)
{
    const int d = mx - mn + 1;
    return int(((double)orc_rng_rand(st) / ((double)2147483647 + 1.0)) * d) + mn;
}

int32_t orc_rng_rand(orc_rng* st)
{
    // glibc __random_r, TYPE_3 (deg 31, sep 3)
    uint32_t val = (uint32_t)st->state[st->f] + (uint32_t)st->state[st->r];
    st->state[st->f] = (int32_t)val;
    const int32_t result = (int32_t)(val >> 1);
    st->f++;
    if (st->f >= 31) {
        st->f = 0;
        st->r++;
    } else {
        st->r++;
        if (st->r >= 31)
            st->r = 0;
    }
    return result;
}

void orc_tfc_fit(const float* p1, const float* p2, const float* w, int n, float* T44)
{
    TFC t;
    for (int i = 0; i < n; i++) t.add(p1 + 3 * i, p2 + 3 * i, w[i]);
    t.transformation(T44);
}

void orc_svd3(const double* A, double* U, double* S, double* V)
{
    double M[3][3], u[3][3], v[3][3];
    for (int i = 0; i < 9; i++) M[i / 3][i % 3] = A[i];
    svd3(M, u, S, v);
    for (int i = 0; i < 9; i++) { U[i] = u[i / 3][i % 3]; V[i] = v[i / 3][i % 3]; }
}

double orc_mahalanobis2(const float* x1, const float* x2, const float* T44, double sticky_cov)
{
    double T[4][4];
    for (int i = 0; i < 16; i++) T[i / 4][i % 4] = (double)T44[i];
    return error_function2(x1, x2, T, sticky_cov, raster_consts());
}

// std::sort(vUsedMatches) (Solver/SolverSE3.cpp:52) on distances alone: order[i] = the input index at sorted
// position i.  depth_limit >= 0 runs libstdc++'s own __introsort_loop with that depth limit (0: the heap-sort
// fallback at once) + __final_insertion_sort -- the branches std::sort takes only on adversarial inputs.
int orc_sort_dmatch(const float* dist, int n, int depth_limit, int32_t* order)
{
    std::vector<DMatch> v((size_t)n);
    for (int i = 0; i < n; i++) v[i] = DMatch{0, 0, i, dist[i]};
    if (depth_limit < 0) {
        std::sort(v.begin(), v.end());
    } else if (n > 1) {
        std::__introsort_loop(v.begin(), v.end(), depth_limit, __gnu_cxx::__ops::__iter_less_iter());
        std::__final_insertion_sort(v.begin(), v.end(), __gnu_cxx::__ops::__iter_less_iter());
    }
    for (int i = 0; i < n; i++) order[i] = v[i].imgIdx;
    return n;
}

int orc_ransac_se3(const float* xyz1, const float* xyz2, const orc_dmatch* m12p, int m, const orc_ransac_params* prm,
                   orc_rng* rng, orc_sticky* sticky, int update_f2, uint8_t* flags2, float* T21, orc_dmatch* inliers_out,
                   int32_t* n_inliers, float* rmse_out)
{
    // RansacSE3::compute, Solver/SolverSE3.cpp:23-133
    Ransac R{xyz1, xyz2, *prm, rng, sticky, raster_consts()};
    std::vector<DMatch> mvInliers;
    float rmse = 1e6;
    float mT21[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    auto finish = [&](bool ok) {
        std::memcpy(T21, mT21, sizeof(mT21));
        *n_inliers = (int)mvInliers.size();
        for (size_t i = 0; i < mvInliers.size(); i++) {
            inliers_out[i].queryIdx = mvInliers[i].queryIdx;
            inliers_out[i].trainIdx = mvInliers[i].trainIdx;
            inliers_out[i].imgIdx = mvInliers[i].imgIdx;
            inliers_out[i].distance = mvInliers[i].distance;
        }
        *rmse_out = rmse;
        return ok ? 1 : 0;
    };
    if ((uint32_t)m < prm->min_inlier_th)
        return finish(false);
    std::vector<DMatch> vUsed;
    vUsed.reserve(m);
    for (int i = 0; i < m; i++) {
        vUsed.push_back(DMatch{m12p[i].queryIdx, m12p[i].trainIdx, m12p[i].imgIdx, m12p[i].distance});
        if (update_f2 && flags2)
            flags2[m12p[i].trainIdx] = 1;
    }
    if (vUsed.size() < prm->min_inlier_th)
        return finish(false);
    int validIters = 0;
    double inlierError;
    std::sort(vUsed.begin(), vUsed.end());
    for (int n = 0; (n < prm->iterations && vUsed.size() >= prm->sample_size); n++) {
        double refinedError = 1e6;
        std::vector<DMatch> vRefined;
        std::vector<DMatch> vInl = R.sample(vUsed);
        float refinedT[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        for (int refinements = 1; refinements < 20; refinements++) {
            float T[16];
            R.fit(vInl, T);
            inlierError = R.inliers_and_error(vUsed, T, vInl);
            if (vInl.size() < prm->min_inlier_th || inlierError > prm->max_mahalanobis)
                break;
            if (vInl.size() >= vRefined.size() && inlierError <= refinedError) {
                const size_t prevNum = vRefined.size();
                std::memcpy(refinedT, T, sizeof(T));
                vRefined = vInl;
                refinedError = inlierError;
                if (vInl.size() == prevNum)
                    break;
            } else
                break;
        }
        if (vRefined.size() > 0) {
            validIters++;
            if (refinedError <= rmse && vRefined.size() >= mvInliers.size() && vRefined.size() >= prm->min_inlier_th) {
                rmse = (float)refinedError;
                std::memcpy(mT21, refinedT, sizeof(refinedT));
                mvInliers = vRefined;
                if (vRefined.size() > vUsed.size() * 0.5)
                    n += 10;
                if (vRefined.size() > vUsed.size() * 0.75)
                    n += 10;
                if (vRefined.size() > vUsed.size() * 0.8)
                    break;
            }
        }
    }
    if (validIters == 0) {
        const float I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        std::vector<DMatch> vInl;
        inlierError = R.inliers_and_error(vUsed, I, vInl);
        if (vInl.size() > prm->min_inlier_th && inlierError < prm->max_mahalanobis) {
            std::memcpy(mT21, I, sizeof(I));
            mvInliers = vInl;
            rmse = (float)((double)rmse + inlierError);
            validIters++;
        }
    }
    if (mvInliers.size() >= prm->min_inlier_th) {
        if (update_f2 && flags2)
            for (const DMatch& mm : mvInliers) flags2[mm.trainIdx] = 0;
        return finish(true);
    }
    return finish(false);
}

}  // extern "C"

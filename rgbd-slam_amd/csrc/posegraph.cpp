// posegraph.cpp -- the keyframe pose graph of the reference's PoseGraph thread (Solver/PoseGraph.cpp),
// host side as in the reference: g2o::SparseOptimizer with VertexSE3 / EdgeSE3 (information 100 I,
// RobustKernelHuber) and OptimizationAlgorithmLevenberg (:40-57, :184-244, :368-386).
//
// g2o is not available here, so the optimiser is restated (DESIGN.md "Pose graph"):
//   * vertex = Twc (Isometry3d), oplus X <- X * fromVectorMQT(dx) (right increment, dx = [t; q_xyz]);
//   * edge (from, to, Z): e = toVectorMQT(Z^-1 * X_from^-1 * X_to) (translation + the vector part of
//     the unit quaternion with w >= 0); setMeasurementFromState: Z = X_from^-1 X_to;
//   * Huber kernel on chi2 = e^T Omega e (delta 1): weight rho'(chi2) on Omega and the gradient;
//   * Jacobians by central differences of the oplus (step 1e-6);
//   * Levenberg-Marquardt as g2o's: lambda0 = 1e-5 max diag(H), up to 10 trials per iteration,
//     gain ratio rho = (chi2 - chi2_new) / (dx^T (lambda dx + b) + 1e-3), lambda *= max(1/3,
//     min(2/3, 1 - (2 rho - 1)^3)) on success, lambda *= ni, ni *= 2 on failure; vertex 0 (or any
//     vertex set fixed) is held; dense Cholesky of the 6(n - fixed) system.
#include <cmath>
#include <cstring>
#include <limits>
#include <map>
#include <set>
#include <utility>
#include <vector>

#include "../../include/rgbd_hip.h"

namespace {

struct Iso {
    double R[9];
    double t[3];
};

Iso iso_identity()
{
    Iso a{};
    a.R[0] = a.R[4] = a.R[8] = 1.0;
    return a;
}

Iso mul(const Iso& a, const Iso& b)
{
    Iso c{};
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) c.R[3 * i + j] = a.R[3 * i] * b.R[j] + a.R[3 * i + 1] * b.R[3 + j] + a.R[3 * i + 2] * b.R[6 + j];
        c.t[i] = a.R[3 * i] * b.t[0] + a.R[3 * i + 1] * b.t[1] + a.R[3 * i + 2] * b.t[2] + a.t[i];
    }
    return c;
}

Iso inv(const Iso& a)
{
    Iso c{};
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) c.R[3 * i + j] = a.R[3 * j + i];
    for (int i = 0; i < 3; i++) c.t[i] = -(c.R[3 * i] * a.t[0] + c.R[3 * i + 1] * a.t[1] + c.R[3 * i + 2] * a.t[2]);
    return c;
}

Iso from_mat(const double* T)
{
    Iso a{};
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) a.R[3 * i + j] = T[4 * i + j];
        a.t[i] = T[4 * i + 3];
    }
    return a;
}

void to_mat(const Iso& a, double* T)
{
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[4 * i + j] = a.R[3 * i + j];
        T[4 * i + 3] = a.t[i];
    }
    T[12] = T[13] = T[14] = 0.0;
    T[15] = 1.0;
}

// Eigen::Quaterniond(Matrix3d) (x, y, z, w)
void quat_from_R(const double* m, double q[4])
{
    const double t = m[0] + m[4] + m[8];
    if (t > 0) {
        double s = std::sqrt(t + 1.0);
        q[3] = 0.5 * s;
        s = 0.5 / s;
        q[0] = (m[7] - m[5]) * s;
        q[1] = (m[2] - m[6]) * s;
        q[2] = (m[3] - m[1]) * s;
        return;
    }
    int i = 0;
    if (m[4] > m[0]) i = 1;
    if (m[8] > m[3 * i + i]) i = 2;
    const int j = (i + 1) % 3, k = (i + 2) % 3;
    double s = std::sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
    q[i] = 0.5 * s;
    s = 0.5 / s;
    q[3] = (m[3 * k + j] - m[3 * j + k]) * s;
    q[j] = (m[3 * j + i] + m[3 * i + j]) * s;
    q[k] = (m[3 * k + i] + m[3 * i + k]) * s;
}

void R_from_quat(double x, double y, double z, double w, double* R)
{
    R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w);     R[2] = 2 * (x * z + y * w);
    R[3] = 2 * (x * y + z * w);     R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
    R[6] = 2 * (x * z - y * w);     R[7] = 2 * (y * z + x * w);     R[8] = 1 - 2 * (x * x + y * y);
}

// g2o internal::toVectorMQT
void to_mqt(const Iso& a, double v[6])
{
    double q[4];
    quat_from_R(a.R, q);
    const double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
    double s = 1.0 / n;
    if (q[3] < 0) s = -s;
    for (int i = 0; i < 3; i++) v[i] = a.t[i];
    for (int i = 0; i < 3; i++) v[3 + i] = q[i] * s;
}

// g2o internal::fromVectorMQT
Iso from_mqt(const double v[6])
{
    Iso a{};
    for (int i = 0; i < 3; i++) a.t[i] = v[i];
    double w = 1.0 - (v[3] * v[3] + v[4] * v[4] + v[5] * v[5]);
    if (w < 0) {
        a.R[0] = a.R[4] = a.R[8] = 1.0;
        for (int i : {1, 2, 3, 5, 6, 7}) a.R[i] = 0.0;
        return a;
    }
    w = std::sqrt(w);
    R_from_quat(v[3], v[4], v[5], w, a.R);
    return a;
}

struct Edge {
    int from, to;
    Iso Zinv;
    double info, delta;
};

}  // namespace

struct rgbd_posegraph {
    std::map<int, Iso> X;          // vertex id -> Twc estimate
    std::set<int> fixed;
    std::vector<Edge> edges;
    std::set<std::pair<int, int>> edge_ids;
};

namespace {

void edge_error(const rgbd_posegraph* g, const Edge& e, const Iso& Xf, const Iso& Xt, double err[6])
{
    (void)g;
    to_mqt(mul(e.Zinv, mul(inv(Xf), Xt)), err);
}

double robust_chi2(const Edge& e, const double err[6], double* weight)
{
    double chi2 = 0.0;
    for (int i = 0; i < 6; i++) chi2 += err[i] * err[i] * e.info;
    const double d2 = e.delta * e.delta;
    if (e.delta <= 0 || chi2 <= d2) {
        if (weight) *weight = 1.0;
        return chi2;
    }
    const double s = std::sqrt(chi2);
    if (weight) *weight = e.delta / s;
    return 2.0 * s * e.delta - d2;
}

double total_chi2(const rgbd_posegraph* g, const std::map<int, Iso>& X)
{
    double c = 0.0;
    for (const Edge& e : g->edges) {
        double err[6];
        edge_error(g, e, X.at(e.from), X.at(e.to), err);
        c += robust_chi2(e, err, nullptr);
    }
    return c;
}

// dense Cholesky solve of (H + lambda I) x = b, in place; false if not positive definite
bool chol_solve(std::vector<double> A, int n, const std::vector<double>& b, std::vector<double>& x)
{
    for (int j = 0; j < n; j++) {
        double d = A[(size_t)j * n + j];
        for (int k = 0; k < j; k++) d -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
        if (!(d > 0.0)) return false;
        d = std::sqrt(d);
        A[(size_t)j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double s = A[(size_t)i * n + j];
            for (int k = 0; k < j; k++) s -= A[(size_t)i * n + k] * A[(size_t)j * n + k];
            A[(size_t)i * n + j] = s / d;
        }
    }
    x.assign(b.begin(), b.end());
    for (int i = 0; i < n; i++) {
        double s = x[i];
        for (int k = 0; k < i; k++) s -= A[(size_t)i * n + k] * x[k];
        x[i] = s / A[(size_t)i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = x[i];
        for (int k = i + 1; k < n; k++) s -= A[(size_t)k * n + i] * x[k];
        x[i] = s / A[(size_t)i * n + i];
    }
    return true;
}

}  // namespace

extern "C" {

rgbd_status rgbd_pg_create(rgbd_posegraph** out)
{
    if (!out) return RGBD_ERR_ARG;
    *out = new rgbd_posegraph();
    return RGBD_OK;
}

void rgbd_pg_destroy(rgbd_posegraph* g) { delete g; }

rgbd_status rgbd_pg_add_vertex(rgbd_posegraph* g, int32_t id, const double* Twc, int32_t fixed)
{
    if (!g || !Twc || g->X.count(id)) return RGBD_ERR_ARG;
    g->X[id] = from_mat(Twc);
    if (fixed) g->fixed.insert(id);
    return RGBD_OK;
}

rgbd_status rgbd_pg_set_fixed(rgbd_posegraph* g, int32_t id, int32_t fixed)
{
    if (!g || !g->X.count(id)) return RGBD_ERR_ARG;
    if (fixed) g->fixed.insert(id);
    else g->fixed.erase(id);
    return RGBD_OK;
}

rgbd_status rgbd_pg_add_edge(rgbd_posegraph* g, int32_t from, int32_t to, const double* Z, double info,
                             double huber_delta, double* chi2)
{
    if (!g || !g->X.count(from) || !g->X.count(to) || from == to || !(info > 0)) return RGBD_ERR_ARG;
    Edge e;
    e.from = from;
    e.to = to;
    e.info = info;
    e.delta = huber_delta;
    const Iso Zm = Z ? from_mat(Z) : mul(inv(g->X[from]), g->X[to]);   // setMeasurementFromState
    e.Zinv = inv(Zm);
    g->edges.push_back(e);
    g->edge_ids.insert({std::min(from, to), std::max(from, to)});
    if (chi2) {
        double err[6];
        edge_error(g, e, g->X[from], g->X[to], err);
        *chi2 = robust_chi2(e, err, nullptr);
    }
    return RGBD_OK;
}

int32_t rgbd_pg_exist_edge(const rgbd_posegraph* g, int32_t a, int32_t b)
{
    if (!g) return 0;
    if (a == b) return 1;   // PoseGraph::existEdge (:389-399)
    return g->edge_ids.count({std::min(a, b), std::max(a, b)}) ? 1 : 0;
}

rgbd_status rgbd_pg_counts(const rgbd_posegraph* g, int32_t* vertices, int32_t* edges)
{
    if (!g) return RGBD_ERR_ARG;
    if (vertices) *vertices = (int32_t)g->X.size();
    if (edges) *edges = (int32_t)g->edges.size();
    return RGBD_OK;
}

rgbd_status rgbd_pg_vertex(const rgbd_posegraph* g, int32_t id, double* Twc)
{
    if (!g || !Twc || !g->X.count(id)) return RGBD_ERR_ARG;
    to_mat(g->X.at(id), Twc);
    return RGBD_OK;
}

rgbd_status rgbd_pg_chi2(const rgbd_posegraph* g, double* chi2)
{
    if (!g || !chi2) return RGBD_ERR_ARG;
    *chi2 = total_chi2(g, g->X);
    return RGBD_OK;
}

rgbd_status rgbd_pg_optimize(rgbd_posegraph* g, int32_t iterations, double* chi2_out, int32_t* iterations_done)
{
    if (!g || iterations < 0) return RGBD_ERR_ARG;
    // free vertices in id order -> block index
    std::map<int, int> blk;
    for (const auto& kv : g->X)
        if (!g->fixed.count(kv.first)) {
            const int b = (int)blk.size();
            blk[kv.first] = b;
        }
    const int n = 6 * (int)blk.size();
    double chi = total_chi2(g, g->X);
    int done = 0;
    if (n == 0 || g->edges.empty()) {
        if (chi2_out) *chi2_out = chi;
        if (iterations_done) *iterations_done = 0;
        return RGBD_OK;
    }
    double lambda = 0.0, ni = 2.0;
    const double step = 1e-6;
    for (int it = 0; it < iterations; it++) {
        // build H, b (b = -J^T w Omega e)
        std::vector<double> H((size_t)n * n, 0.0), bv(n, 0.0);
        for (const Edge& e : g->edges) {
            const Iso& Xf = g->X.at(e.from);
            const Iso& Xt = g->X.at(e.to);
            double err[6];
            edge_error(g, e, Xf, Xt, err);
            double w = 1.0;
            robust_chi2(e, err, &w);
            double J[2][6][6] = {};
            const int vid[2] = {e.from, e.to};
            bool act[2];
            for (int s = 0; s < 2; s++) {
                act[s] = blk.count(vid[s]) > 0;
                if (!act[s]) continue;
                for (int d = 0; d < 6; d++) {
                    double dx[6] = {0, 0, 0, 0, 0, 0};
                    double ep[6], em[6];
                    dx[d] = step;
                    const Iso Xp = mul(s == 0 ? Xf : Xt, from_mqt(dx));
                    edge_error(g, e, s == 0 ? Xp : Xf, s == 0 ? Xt : Xp, ep);
                    dx[d] = -step;
                    const Iso Xm = mul(s == 0 ? Xf : Xt, from_mqt(dx));
                    edge_error(g, e, s == 0 ? Xm : Xf, s == 0 ? Xt : Xm, em);
                    for (int r = 0; r < 6; r++) J[s][r][d] = (ep[r] - em[r]) / (2.0 * step);
                }
            }
            const double wi = w * e.info;
            for (int s = 0; s < 2; s++) {
                if (!act[s]) continue;
                const int bs = 6 * blk.at(vid[s]);
                for (int a = 0; a < 6; a++) {
                    double g_ = 0.0;
                    for (int r = 0; r < 6; r++) g_ += J[s][r][a] * err[r];
                    bv[bs + a] -= wi * g_;
                }
                for (int s2 = 0; s2 < 2; s2++) {
                    if (!act[s2]) continue;
                    const int bs2 = 6 * blk.at(vid[s2]);
                    for (int a = 0; a < 6; a++)
                        for (int c = 0; c < 6; c++) {
                            double h = 0.0;
                            for (int r = 0; r < 6; r++) h += J[s][r][a] * J[s2][r][c];
                            H[(size_t)(bs + a) * n + bs2 + c] += wi * h;
                        }
                }
            }
        }
        if (it == 0) {   // computeLambdaInit: tau * max diagonal
            double mx = 0.0;
            for (int i = 0; i < n; i++) mx = std::max(mx, std::fabs(H[(size_t)i * n + i]));
            lambda = 1e-5 * mx;
            ni = 2.0;
        }
        double rho = 0.0;
        int q = 0;
        do {
            std::vector<double> A = H, x;
            for (int i = 0; i < n; i++) A[(size_t)i * n + i] += lambda;
            const bool ok = chol_solve(A, n, bv, x);
            std::map<int, Iso> Xn = g->X;
            if (ok)
                for (const auto& kv : blk) Xn[kv.first] = mul(g->X.at(kv.first), from_mqt(&x[6 * kv.second]));
            const double chi_new = ok ? total_chi2(g, Xn) : std::numeric_limits<double>::max();
            double scale = 0.0;
            if (ok)
                for (int j = 0; j < n; j++) scale += x[j] * (lambda * x[j] + bv[j]);
            scale += 1e-3;
            rho = (chi - chi_new) / scale;
            if (rho > 0 && std::isfinite(chi_new)) {
                const double alpha = std::min(1.0 - std::pow(2.0 * rho - 1.0, 3), 2.0 / 3.0);
                lambda *= std::max(1.0 / 3.0, alpha);
                ni = 2.0;
                chi = chi_new;
                g->X = Xn;
            } else {
                lambda *= ni;
                ni *= 2.0;
            }
            q++;
        } while (rho < 0 && q < 10);
        done++;
        if (q == 10 || rho == 0 || !std::isfinite(lambda)) break;   // OptimizationAlgorithm::Terminate
    }
    if (chi2_out) *chi2_out = chi;
    if (iterations_done) *iterations_done = done;
    return RGBD_OK;
}

}  // extern "C"

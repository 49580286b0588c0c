// svd3_dev.h -- Eigen 3.3 JacobiSVD<Matrix3d> (two-sided Jacobi, 3 x 3) on the device, the same
// operation sequence as the oracle's restatement (oracle/orc_solver.cpp svd3).  Used by RansacSE3
// (PCL TransformationFromCorrespondences) and GICP (PCL computeCovariances).
#pragma once
#include <hip/hip_runtime.h>

#include "exact_dev.h"

namespace rgbd {
namespace svd3d {

constexpr double kDblMax = 1.7976931348623157e308;
constexpr double kDblMin = 2.2250738585072014e-308;
constexpr double kDblEps = 2.220446049250313e-16;

struct JR { double c, s; };

__device__ __forceinline__ void rot_rows(double A[3][3], int p, int q, JR j)
{
    if (j.c == 1.0 && j.s == 0.0) return;
    for (int i = 0; i < 3; i++) {
        const double xi = A[p][i], yi = A[q][i];
        A[p][i] = j.c * xi + j.s * yi;
        A[q][i] = -j.s * xi + j.c * yi;
    }
}

__device__ __forceinline__ void rot_cols(double A[3][3], int p, int q, JR j)
{
    const double c = j.c, s = -j.s;
    if (c == 1.0 && s == 0.0) return;
    for (int i = 0; i < 3; i++) {
        const double xi = A[i][p], yi = A[i][q];
        A[i][p] = c * xi + s * yi;
        A[i][q] = -s * xi + c * yi;
    }
}

// The rotation's sqrts and reciprocals through exact_dev.h's sequences where their operands are in range (the
// same IEEE bits: sqrt of x in [1, inf), 1 / d for 1 <= |d| < 2^1000), the general operations otherwise; y / |y|
// (y != 0) is +-1 exactly, so copysign
__device__ __forceinline__ double sqrt_ge1_inf(double x) { return x == INFINITY ? x : sqrt_ge1(x); }   // x >= 1 or NaN
__device__ __forceinline__ double recip_ge1(double d) { return fabs(d) < 0x1p1000 ? div_plain(1.0, d) : 1.0 / d; }   // |d| >= 1
__device__ __forceinline__ JR make_jacobi(double x, double y, double z)
{
    const double deno = 2.0 * fabs(y);
    if (deno < kDblMin) return JR{1.0, 0.0};
    const double tau = (x - z) / deno;
    const double w = sqrt_ge1_inf(tau * tau + 1.0);
    const double t = (tau > 0.0) ? recip_ge1(tau + w) : recip_ge1(tau - w);
    const double sign_t = t > 0.0 ? 1.0 : -1.0;
    const double n = div_plain(1.0, sqrt_ge1(t * t + 1.0));   // t^2 + 1 in [1, 2]
    JR r;
    r.s = -sign_t * copysign(1.0, y) * fabs(t) * n;
    r.c = n;
    return r;
}

__device__ __forceinline__ void jacobi_2x2(const double A[3][3], int p, int q, JR* jl, JR* jr)
{
    double m00 = A[p][p], m01 = A[p][q], m10 = A[q][p], m11 = A[q][q];
    JR r1;
    const double t = m00 + m11;
    const double d = m10 - m01;
    if (fabs(d) < kDblMin) {
        r1.s = 0.0;
        r1.c = 1.0;
    } else {
        const double u = t / d;
        const double tmp = sqrt_ge1_inf(1.0 + u * u);
        r1.s = recip_ge1(tmp);
        const double au = fabs(u);
        r1.c = (au >= 0x1p-1000 && au < 0x1p999) ? div_plain(u, tmp) : u / tmp;   // |u / tmp| normal there
    }
    if (!(r1.c == 1.0 && r1.s == 0.0)) {
        const double a0 = r1.c * m00 + r1.s * m10, b0 = -r1.s * m00 + r1.c * m10;
        const double a1 = r1.c * m01 + r1.s * m11, b1 = -r1.s * m01 + r1.c * m11;
        m00 = a0; m10 = b0; m01 = a1; m11 = b1;
    }
    *jr = make_jacobi(m00, m01, m11);
    const double jtc = jr->c, jts = -jr->s;
    jl->c = r1.c * jtc - r1.s * jts;
    jl->s = r1.c * jts + r1.s * jtc;
}

// Eigen 3.3 JacobiSVD<Matrix3d>(ComputeFullU | ComputeFullV), square path (no preconditioner)
// prof (profiling builds): wall-clock (10 ns) accumulated per stage [0] scale + W, [1] sweeps, [2] S + sort,
// [3] sweeps run, [4] rotation steps run
__device__ __forceinline__ void svd3(const double M[3][3], double U[3][3], double V[3][3], double* Sout = nullptr,
                                     long long* prof = nullptr)
{
    long long t_prev = prof ? (long long)wall_clock64() : 0;
    auto mark = [&](int k) {
        if (prof) {
            const long long t = (long long)wall_clock64();
            prof[k] += t - t_prev;
            t_prev = t;
        }
    };
    double scale = 0.0;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) scale = fmax(scale, fabs(M[i][j]));
    if (!isfinite(scale)) {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) U[i][j] = V[i][j] = __builtin_nan("");
        return;
    }
    if (scale == 0.0) scale = 1.0;
    double W[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            W[i][j] = M[i][j] / scale;
            U[i][j] = V[i][j] = (i == j) ? 1.0 : 0.0;
        }
    double maxDiag = fmax(fmax(fabs(W[0][0]), fabs(W[1][1])), fabs(W[2][2]));
    mark(0);
    bool finished = false;
    int sweeps = 0;
    while (!finished && sweeps < 64) {
        finished = true;
        sweeps++;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                const double threshold = fmax(kDblMin, 2.0 * kDblEps * maxDiag);
                if (fabs(W[p][q]) > threshold || fabs(W[q][p]) > threshold) {
                    finished = false;
                    if (prof) prof[4]++;
                    JR jl, jr;
                    jacobi_2x2(W, p, q, &jl, &jr);
                    rot_rows(W, p, q, jl);
                    rot_cols(U, p, q, JR{jl.c, -jl.s});
                    rot_cols(W, p, q, jr);
                    rot_cols(V, p, q, jr);
                    maxDiag = fmax(maxDiag, fmax(fabs(W[p][p]), fabs(W[q][q])));
                }
            }
    }
    if (prof) prof[3] += sweeps;
    mark(1);
    double S[3];
    for (int i = 0; i < 3; i++) {
        const double a = W[i][i];
        S[i] = fabs(a);
        if (a < 0.0)
            for (int r = 0; r < 3; r++) U[r][i] = -U[r][i];
    }
    for (int i = 0; i < 3; i++) S[i] *= scale;   // singular values are sorted after rescaling (Eigen)
    for (int i = 0; i < 3; i++) {
        int pos = i;
        double mx = S[i];
        for (int j = i + 1; j < 3; j++)
            if (S[j] > mx) { mx = S[j]; pos = j; }
        if (mx == 0.0) break;
        if (pos != i) {
            const double ts = S[i]; S[i] = S[pos]; S[pos] = ts;
            for (int r = 0; r < 3; r++) {
                double t1 = U[r][i]; U[r][i] = U[r][pos]; U[r][pos] = t1;
                double t2 = V[r][i]; V[r][i] = V[r][pos]; V[r][pos] = t2;
            }
        }
    }
    if (Sout)
        for (int i = 0; i < 3; i++) Sout[i] = S[i];
    mark(2);
}

}  // namespace svd3d
}  // namespace rgbd

// orc_common.h -- ORACLE helpers shared by the PnPRansac and GICP restatements (test infrastructure
// only; see rgbd_oracle.h).  Deterministic definitions built from + - * / sqrt only.
#pragma once
#include <cmath>

namespace orc {

// ------------------------------------------------------------ deterministic sin/cos (double)
inline void sincos_poly(double x, double* s_out, double* c_out)
{
    const double PIO2_1 = 1.57079632673412561417e+00, PIO2_1T = 6.07710050650619224932e-11;
    const double INV_PIO2 = 6.36619772367581382433e-01;
    const double kd = std::floor(x * INV_PIO2 + 0.5);
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

inline void rodrigues_exp(const double w[3], double R[9])
{
    const double th2 = (w[0] * w[0] + w[1] * w[1]) + w[2] * w[2];
    const double th = std::sqrt(th2);
    if (th < 1e-300) {
        for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.0 : 0.0;
        return;
    }
    double s, c;
    sincos_poly(th, &s, &c);
    const double k[3] = {w[0] / th, w[1] / th, w[2] / th};
    const double c1 = 1.0 - c;
    R[0] = c + c1 * k[0] * k[0];        R[1] = c1 * k[0] * k[1] - s * k[2]; R[2] = c1 * k[0] * k[2] + s * k[1];
    R[3] = c1 * k[1] * k[0] + s * k[2]; R[4] = c + c1 * k[1] * k[1];        R[5] = c1 * k[1] * k[2] - s * k[0];
    R[6] = c1 * k[2] * k[0] - s * k[1]; R[7] = c1 * k[2] * k[1] + s * k[0]; R[8] = c + c1 * k[2] * k[2];
}

// 6x6 solve H x = -g by Gaussian elimination with partial pivoting (deterministic)
inline bool solve6(double H[36], double g[6], double x[6])
{
    double A[6][7];
    for (int i = 0; i < 6; i++) {
        for (int j = 0; j < 6; j++) A[i][j] = H[i * 6 + j];
        A[i][6] = -g[i];
    }
    for (int k = 0; k < 6; k++) {
        int p = k;
        for (int i = k + 1; i < 6; i++)
            if (std::fabs(A[i][k]) > std::fabs(A[p][k])) p = i;
        if (A[p][k] == 0.0) return false;
        if (p != k)
            for (int j = 0; j < 7; j++) { const double tt = A[k][j]; A[k][j] = A[p][j]; A[p][j] = tt; }
        for (int i = k + 1; i < 6; i++) {
            const double f = A[i][k] / A[k][k];
            for (int j = k; j < 7; j++) A[i][j] -= f * A[k][j];
        }
    }
    for (int k = 5; k >= 0; k--) {
        double s = A[k][6];
        for (int j = k + 1; j < 6; j++) s -= A[k][j] * x[j];
        x[k] = s / A[k][k];
    }
    return true;
}

}  // namespace orc

// gicp.hip -- GICP refinement of the tracking chain on gfx950.
//
// Reference: Gicp::compute / align (Solver/Gicp.cpp:21-66) = pcl::GeneralizedIterativeClosestPoint
// <PointXYZ, PointXYZ>, run by Tracking::visualOdometry when RansacSE3's rmse >= 0.8 with max
// correspondence distance 0.07 and 10 iterations (System/Tracking.cpp:145-151).  PCL is absent: the
// operator is the definition restated in oracle/orc_gicp.cpp (DESIGN.md "GICP"), computed here with
// the same IEEE operations in the same order.
//   k_gicp_cov    one wave per point of either cloud: its 20 nearest neighbours (exact, ascending
//                 (distance, index)) by 20 rounds of a wave-wide 64-bit key minimum, then PCL's
//                 mean / covariance, Eigen JacobiSVD U and the (1, 1, eps) rebuild on lane 0.
//   k_gicp_align  one 512-thread workgroup per problem runs every outer iteration: 1-NN of each
//                 transformed source point over the LDS-resident target (a thread per point), then
//                 Gauss-Newton steps whose J^T M J / J^T M r sums (M = (R C1 R^T + C2)^-1 per
//                 correspondence) run in 256 strided lanes + a binary tree (the oracle's order).
#include <hip/hip_runtime.h>

#include "dispatch.h"

#include <climits>

#include "gicp_dev.h"
#include "lanes_dev.h"
#include "svd3_dev.h"

namespace rgbd {

namespace {

__device__ __forceinline__ float dist2f(float ax, float ay, float az, float bx, float by, float bz)
{
    const float dx = ax - bx, dy = ay - by, dz = az - bz;
    float r = 0.0f;
    r = r + dx * dx;
    r = r + dy * dy;
    r = r + dz * dz;
    return r;
}

// 64-bit min of one DPP step (lanes without a source keep ~0, which the min ignores)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ unsigned long long dpp_min_u64(unsigned long long v)
{
    const unsigned tlo = (unsigned)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)(unsigned)v, CTRL, ROWMASK, 0xf, false);
    const unsigned thi = (unsigned)__builtin_amdgcn_update_dpp((int)0xffffffff, (int)(unsigned)(v >> 32), CTRL, ROWMASK, 0xf, false);
    const unsigned long long t = ((unsigned long long)thi << 32) | tlo;
    return t < v ? t : v;
}

// the wave's minimum (uniform): row_shr 1, 2, 4, 8 leave each 16-lane row's minimum in its lane 15, row_bcast 15
// and 31 carry them up to lane 63 (DPP only: no LDS round trips in the k-NN rounds)
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v)
{
    v = dpp_min_u64<0x111, 0xf>(v);
    v = dpp_min_u64<0x112, 0xf>(v);
    v = dpp_min_u64<0x114, 0xf>(v);
    v = dpp_min_u64<0x118, 0xf>(v);
    v = dpp_min_u64<0x142, 0xa>(v);
    v = dpp_min_u64<0x143, 0xc>(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, 63);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), 63);
    return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ double cof(const double* m, int i, int j)
{
    const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
    return m[i1 * 3 + j1] * m[i2 * 3 + j2] - m[i1 * 3 + j2] * m[i2 * 3 + j1];
}

// Eigen 3.3 compute_inverse<3> (oracle inverse3)
__device__ __forceinline__ void inverse3(const double* m, double* r)
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

// oracle gn_terms: J = [-[y]x | I], r = y - q
__device__ __forceinline__ void gn_terms(const double* y, const double* q, const double* M, double out[27])
{
    const double r[3] = {y[0] - q[0], y[1] - q[1], y[2] - q[2]};
    const double J[3][6] = {{0.0, y[2], -y[1], 1.0, 0.0, 0.0},
                            {-y[2], 0.0, y[0], 0.0, 1.0, 0.0},
                            {y[1], -y[0], 0.0, 0.0, 0.0, 1.0}};
    double Mr[3], MJ[3][6];
#pragma unroll
    for (int a = 0; a < 3; a++) {
        Mr[a] = (M[a * 3] * r[0] + M[a * 3 + 1] * r[1]) + M[a * 3 + 2] * r[2];
#pragma unroll
        for (int b = 0; b < 6; b++) MJ[a][b] = (M[a * 3] * J[0][b] + M[a * 3 + 1] * J[1][b]) + M[a * 3 + 2] * J[2][b];
    }
    int k = 0;
#pragma unroll
    for (int a = 0; a < 6; a++)
#pragma unroll
        for (int b = a; b < 6; b++) out[k++] = (J[0][a] * MJ[0][b] + J[1][a] * MJ[1][b]) + J[2][a] * MJ[2][b];
#pragma unroll
    for (int a = 0; a < 6; a++) out[k++] = (J[0][a] * Mr[0] + J[1][a] * Mr[1]) + J[2][a] * Mr[2];
}

constexpr int kCovWaves = 4;
constexpr int kCovPer = (kGicpMaxM + 63) / 64;   // candidates per lane
constexpr int kAlignThreads = 512;
constexpr int kRedLanes = 256;                    // reduction lanes (oracle kLanes)

}  // namespace

// ---------------------------------------------------------------- covariances (PCL computeCovariances)
// A wave takes a group of up to kCovG consecutive points of [source | target]: the k-nearest-neighbour search
// of each, one after another with the whole wave (distances of every cloud point, k rounds of wave minimum
// over (distance, index) keys: ascending distance, ties by index), the neighbour ids kept in LDS; then lane s
// forms point s's covariance from its neighbours and its SVD-regularised matrix, so the f64 covariance and
// SVD run kCovG points per wave instead of one lane per wave.
constexpr int kCovK = 32;   // neighbour slots per point (k_correspondences <= 32, gicp_host.cpp)
constexpr int kCovG = 16;   // points per wave group (more waves in flight hide the k-NN rounds' latency)

// 64 u64 values across the wave sorted ascending by lane (bitonic network over lane pairs)
__device__ __forceinline__ unsigned long long wave_sort_u64(unsigned long long v)
{
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k2 = 2; k2 <= 64; k2 <<= 1)
#pragma unroll
        for (int j = k2 >> 1; j > 0; j >>= 1) {
            const unsigned long long o = __shfl_xor(v, j);
            const bool take_min = ((lane & k2) == 0) == ((lane & j) == 0);
            v = take_min ? (o < v ? o : v) : (o > v ? o : v);
        }
    return v;
}

// the neighbours of point i of cloud `pts` (M <= 64 NC points, uniform per wave), ids into nn[0 .. k) in
// ascending (distance, index) order.  The keys (distance bits, index) are unique.  t = the k-th smallest of
// the 64 lanes' minimum keys bounds the k-th smallest key overall (k lanes hold a key <= t), so the k nearest
// are among the keys <= t: those (about k of them for spatially unordered indices) are compacted through
// LDS, sorted across the wave and the first k taken.  More than 64 candidates: k rounds of wave minimum.
template <int NC>
__device__ void gicp_knn(const float* __restrict__ pts, int M, int k, int i, uint16_t* nn, unsigned long long* cand)
{
    const int lane = threadIdx.x & 63;
    const float qx = pts[3 * i], qy = pts[3 * i + 1], qz = pts[3 * i + 2];
    unsigned long long key[NC];
    unsigned long long lm = ~0ull;
#pragma unroll
    for (int c = 0; c < NC; c++) {
        const int j = lane + 64 * c;
        key[c] = ~0ull;
        if (j < M) {
            const float d = dist2f(qx, qy, qz, pts[3 * j], pts[3 * j + 1], pts[3 * j + 2]);
            key[c] = ((unsigned long long)__float_as_uint(d) << 32) | (unsigned)j;
        }
        lm = key[c] < lm ? key[c] : lm;
    }
    const unsigned long long srt = wave_sort_u64(lm);
    const unsigned long long t = ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(unsigned)(srt >> 32), k - 1) << 32) |
                                 (unsigned)__builtin_amdgcn_readlane((int)(unsigned)srt, k - 1);
    int cnt = 0;
#pragma unroll
    for (int c = 0; c < NC; c++) cnt += key[c] <= t ? 1 : 0;
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    const int total = __builtin_amdgcn_readlane(incl, 63);
    if (total <= 64) {
        int pos = incl - cnt;
#pragma unroll
        for (int c = 0; c < NC; c++)
            if (key[c] <= t) cand[pos++] = key[c];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const unsigned long long v = wave_sort_u64(lane < total ? cand[lane] : ~0ull);
        if (lane < k) nn[lane] = (uint16_t)(unsigned)v;
        __builtin_amdgcn_wave_barrier();   // cand is read before the next point overwrites it
        return;
    }
    for (int r = 0; r < k; r++) {   // rounds: the wave's minimum; its owner lane drops it and rescans
        const unsigned long long g = wave_min_u64(lm);
        const int j = (int)(g & 0xffffffffu);
        if (lane == 0) nn[r] = (uint16_t)j;
        const int cj = j >> 6;
        const bool own = lane == (j & 63);
#pragma unroll
        for (int c = 0; c < NC; c++)
            if (c == cj) key[c] = own ? ~0ull : key[c];
        if (own) {
            lm = ~0ull;
#pragma unroll
            for (int c = 0; c < NC; c++) lm = key[c] < lm ? key[c] : lm;
        }
    }
}

// dispatch on the candidate slots per lane the problem needs (M uniform per wave)
__device__ __forceinline__ void gicp_knn_any(const float* __restrict__ pts, int M, int k, int i, uint16_t* nn,
                                             unsigned long long* cand)
{
    const int nc = (M + 63) >> 6;
    if (nc <= 4) gicp_knn<4>(pts, M, k, i, nn, cand);
    else if (nc <= 8) gicp_knn<8>(pts, M, k, i, nn, cand);
    else if (nc <= 12) gicp_knn<12>(pts, M, k, i, nn, cand);
    else if (nc <= 16) gicp_knn<16>(pts, M, k, i, nn, cand);
    else if (nc <= 20) gicp_knn<20>(pts, M, k, i, nn, cand);
    else if (nc <= 24) gicp_knn<24>(pts, M, k, i, nn, cand);
    else if (nc <= 28) gicp_knn<28>(pts, M, k, i, nn, cand);
    else gicp_knn<kCovPer>(pts, M, k, i, nn, cand);
}

// point i's regularised covariance from its k neighbours (one lane; PCL computeCovariances + the SVD
// replacement of the eigenvalues by (1, 1, eps))
__device__ __forceinline__ void gicp_cov_from_nn(const float* __restrict__ pts, int k, double eps, const uint16_t* nn,
                                                 double* __restrict__ dst)
{
    double mean[3] = {0, 0, 0};
    double C[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int r = 0; r < k; r++) {
        const float* p = pts + 3 * nn[r];
        const float px = p[0], py = p[1], pz = p[2];
        mean[0] += px;
        mean[1] += py;
        mean[2] += pz;
        C[0][0] += px * px;
        C[1][0] += py * px;
        C[1][1] += py * py;
        C[2][0] += pz * px;
        C[2][1] += pz * py;
        C[2][2] += pz * pz;
    }
    for (int a = 0; a < 3; a++) mean[a] /= (double)k;
    for (int a = 0; a < 3; a++)
        for (int b = 0; b <= a; b++) {
            C[a][b] /= (double)k;
            C[a][b] -= mean[a] * mean[b];
            C[b][a] = C[a][b];
        }
    double U[3][3], V[3][3];
    svd3d::svd3(C, U, V);
    double out[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int c = 0; c < 3; c++) {
        const double v = (c == 2) ? eps : 1.0;
        const double col[3] = {U[0][c], U[1][c], U[2][c]};
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) out[a * 3 + b] += (v * col[a]) * col[b];
    }
    for (int e = 0; e < 9; e++) dst[e] = out[e];
}

// one problem (M pairs): points qi in [0, 2M) = source then target, in groups of 64 per wave
__global__ __launch_bounds__(64 * kCovWaves) void k_gicp_cov(const float* __restrict__ src, const float* __restrict__ tgt,
                                                             int M, int k, double eps, double* __restrict__ cov)
{
    __shared__ uint16_t nnb[kCovWaves][kCovG][kCovK];
    __shared__ unsigned long long candb[kCovWaves][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q0 = (blockIdx.x * kCovWaves + w) * kCovG;
    if (q0 >= 2 * M) return;   // whole wave
    const int n = min(kCovG, 2 * M - q0);
    for (int s = 0; s < n; s++) {
        const int qi = q0 + s;
        gicp_knn_any(qi < M ? src : tgt, M, k, qi < M ? qi : qi - M, nnb[w][s], candb[w]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (lane >= n) return;
    const int qi = q0 + lane;
    gicp_cov_from_nn(qi < M ? src : tgt, k, eps, nnb[w][lane], cov + (size_t)qi * 9);
}

// the deferred problems of the lane chain (lanes_dev.h): every (problem, point) item of k_gicp_list's
// prefix in groups of kCovG per wave, strided over the grid (an item's problem by binary search in the prefix)
constexpr int kCovPairBlocks = 4096;
__device__ __forceinline__ int gicp_problem_of(const LaneBufs& lb, int np, int t)
{
    int a = 0, z = np - 1;   // last problem whose prefix <= t
    while (a < z) {
        const int mid = (a + z + 1) >> 1;
        if (lb.ppre[mid] <= t) a = mid;
        else z = mid - 1;
    }
    return a;
}

__global__ __launch_bounds__(64 * kCovWaves) void k_gicp_cov_pairs(LaneBufs lb, LaneCfg lc)
{
    __shared__ uint16_t nnb[kCovWaves][kCovG][kCovK];
    __shared__ unsigned long long candb[kCovWaves][64];
    const int np = lb.pcount[0], total = lb.pcount[1];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int t0 = (blockIdx.x * kCovWaves + w) * kCovG; t0 < total; t0 += kCovPairBlocks * kCovWaves * kCovG) {
        const int n = min(kCovG, total - t0);
        for (int s = 0; s < n; s++) {
            const int t = t0 + s;
            const int a = gicp_problem_of(lb, np, t);
            const int b = lb.plist[a];
            const int M = lb.gn[b];
            const int qi = t - lb.ppre[a];
            const size_t lo = (size_t)b * lc.GM * 3;
            gicp_knn_any(qi < M ? lb.gsrc + lo : lb.gtgt + lo, M, lc.gp.k, qi < M ? qi : qi - M, nnb[w][s], candb[w]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < n) {
            const int t = t0 + lane;
            const int a = gicp_problem_of(lb, np, t);
            const int b = lb.plist[a];
            const int M = lb.gn[b];
            const int qi = t - lb.ppre[a];
            const size_t lo = (size_t)b * lc.GM * 3;
            gicp_cov_from_nn(qi < M ? lb.gsrc + lo : lb.gtgt + lo, lc.gp.k, lc.gp.gicp_eps, nnb[w][lane],
                             lb.gcov + (size_t)b * 2 * lc.GM * 9 + (size_t)qi * 9);
        }
        __builtin_amdgcn_wave_barrier();   // the group's LDS ids are read before the next group overwrites them
    }
}

// ---------------------------------------------------------------- outer iterations (computeTransformation)
// The 1-NN search runs on a uniform grid over the target with cells of 1.01 max_corr_dist: a correspondence
// needs float distance < max_corr_dist^2, so every target that can be one lies in the 27 cells around the
// query's cell (the 1 % margin covers the float rounding of the differences and of x / h), and the
// smallest (distance, index) among them is the brute-force scan's result (first index on ties) whenever
// that result is a correspondence; when it is not, neither is the grid's.  Targets are sorted by cell key,
// the nine (x, y) columns of three z cells are key ranges found by binary search.  Points beyond the
// grid's +-512-cell range fall back to the full scan.  M_i = (R C1 R^T + C2)^-1 of each correspondence is
// computed once per outer iteration (R is fixed in it) into Mi (global scratch, M x 9 doubles).
constexpr int kGridBits = 10, kGridHalf = 512;

__device__ __forceinline__ int grid_cell(float v, float inv)
{
    const float c = floorf(v * inv);
    return (c > -(float)kGridHalf && c < (float)(kGridHalf - 1)) ? (int)c + kGridHalf : -1;   // 1 .. 1022 usable
}

__device__ void gicp_align_block(const float* __restrict__ src, const float* __restrict__ tgt, int M,
                                 const double* __restrict__ cov, const float* __restrict__ guess, const GicpDevPrm& prm,
                                 GicpOut* __restrict__ out, double* __restrict__ Mi)
{
    __shared__ float ox[kGicpMaxM], oy[kGicpMaxM], oz[kGicpMaxM];   // output = guess * source
    __shared__ float tx[kGicpMaxM], ty[kGicpMaxM], tz[kGicpMaxM];   // target
    __shared__ int nn[kGicpMaxM];                                   // -1: no correspondence
    __shared__ unsigned long long skey[kGicpMaxM];                  // (cell key << 11 | target index), sorted
    __shared__ int grid_ok;
    __shared__ double red[27 * 128];
    __shared__ double sums[27];
    __shared__ float G[16], T[16], prev[16];
    __shared__ double Rg[9], Rd[9], td[3];
    __shared__ int cnt_s, stop_s, conv_s, it_s;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < 16) {
        G[tid] = guess[tid];
        T[tid] = (tid % 5 == 0) ? 1.0f : 0.0f;
    }
    if (tid == 0) { cnt_s = 0; conv_s = 0; it_s = 0; grid_ok = 1; }
    __syncthreads();
    const float hinv = 1.0f / (float)(sqrt(prm.thr) * 1.01);
    int Mp = 1;
    while (Mp < M) Mp <<= 1;
    for (int i = tid; i < Mp; i += kAlignThreads) {
        if (i >= M) {
            skey[i] = ~0ull;
            continue;
        }
        const float px = src[3 * i], py = src[3 * i + 1], pz = src[3 * i + 2];
        ox[i] = ((G[0] * px + G[1] * py) + G[2] * pz) + G[3];
        oy[i] = ((G[4] * px + G[5] * py) + G[6] * pz) + G[7];
        oz[i] = ((G[8] * px + G[9] * py) + G[10] * pz) + G[11];
        const float a = tgt[3 * i], b = tgt[3 * i + 1], c = tgt[3 * i + 2];
        tx[i] = a;
        ty[i] = b;
        tz[i] = c;
        const int kx = grid_cell(a, hinv), ky = grid_cell(b, hinv), kz = grid_cell(c, hinv);
        if (kx < 0 || ky < 0 || kz < 0) grid_ok = 0;
        const unsigned long long key = ((unsigned long long)(kx & 1023) << (2 * kGridBits)) |
                                       ((unsigned long long)(ky & 1023) << kGridBits) | (unsigned long long)(kz & 1023);
        skey[i] = (key << 11) | (unsigned long long)i;
    }
    __syncthreads();
    // bitonic sort of the Mp keys
    for (int k = 2; k <= Mp; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < Mp; i += kAlignThreads) {
                const int p = i ^ j;
                if (p > i) {
                    const unsigned long long a = skey[i], b = skey[p];
                    if (((i & k) == 0) == (a > b)) {
                        skey[i] = b;
                        skey[p] = a;
                    }
                }
            }
            __syncthreads();
        }
    bool aborted = false;
    for (;;) {
        if (tid < 9) {
            const int i = tid / 3, j = tid % 3;
            double s = 0.0;
            for (int kk = 0; kk < 4; kk++) s += (double)T[4 * i + kk] * (double)G[4 * kk + j];
            Rg[tid] = s;
        }
        if (tid == 0) cnt_s = 0;
        __syncthreads();
        // 1-NN of transformation_ * output[i] in the target; Mahalanobis matrix of a correspondence
        int mycnt = 0;
        for (int i = tid; i < M; i += kAlignThreads) {
            const float qx = ((T[0] * ox[i] + T[1] * oy[i]) + T[2] * oz[i]) + T[3];
            const float qy = ((T[4] * ox[i] + T[5] * oy[i]) + T[6] * oz[i]) + T[7];
            const float qz = ((T[8] * ox[i] + T[9] * oy[i]) + T[10] * oz[i]) + T[11];
            const int cx = grid_cell(qx, hinv), cy = grid_cell(qy, hinv), cz = grid_cell(qz, hinv);
            int best = -1;
            float bd = 0.0f;
            if (grid_ok && cx > 0 && cy > 0 && cz > 0 && cx < 1023 && cy < 1023 && cz < 1023) {
                for (int dxy = 0; dxy < 9; dxy++) {
                    const unsigned long long col = ((unsigned long long)(cx + dxy / 3 - 1) << (2 * kGridBits)) |
                                                   ((unsigned long long)(cy + dxy % 3 - 1) << kGridBits);
                    const unsigned long long lo = (col | (unsigned long long)(cz - 1)) << 11;
                    const unsigned long long hi = (col | (unsigned long long)(cz + 1)) << 11 | 2047ull;
                    int a = 0, b = M;   // first key >= lo
                    while (a < b) {
                        const int mid = (a + b) >> 1;
                        if (skey[mid] < lo) a = mid + 1;
                        else b = mid;
                    }
                    for (; a < M && skey[a] <= hi; a++) {
                        const int j = (int)(skey[a] & 2047ull);
                        const float d = dist2f(qx, qy, qz, tx[j], ty[j], tz[j]);
                        if (best < 0 || d < bd || (d == bd && j < best)) { bd = d; best = j; }
                    }
                }
            } else {   // outside the grid: the full scan
                best = 0;
                bd = dist2f(qx, qy, qz, tx[0], ty[0], tz[0]);
                for (int j = 1; j < M; j++) {
                    const float d = dist2f(qx, qy, qz, tx[j], ty[j], tz[j]);
                    if (d < bd) { bd = d; best = j; }
                }
            }
            const bool has = best >= 0 && (double)bd < prm.thr;
            nn[i] = has ? best : -1;
            mycnt += has ? 1 : 0;
            if (has) {   // M_i = (R C1_i R^T + C2_j)^-1, fixed for this outer iteration
                const double* c1 = cov + (size_t)i * 9;
                const double* c2 = cov + ((size_t)M + best) * 9;
                double RC[9], tmp[9], Mv[9];
#pragma unroll
                for (int a = 0; a < 3; a++)
#pragma unroll
                    for (int b = 0; b < 3; b++)
                        RC[3 * a + b] = (Rg[3 * a] * c1[b] + Rg[3 * a + 1] * c1[3 + b]) + Rg[3 * a + 2] * c1[6 + b];
#pragma unroll
                for (int a = 0; a < 3; a++)
#pragma unroll
                    for (int b = 0; b < 3; b++)
                        tmp[3 * a + b] = ((RC[3 * a] * Rg[3 * b] + RC[3 * a + 1] * Rg[3 * b + 1]) + RC[3 * a + 2] * Rg[3 * b + 2])
                                         + c2[3 * a + b];
                inverse3(tmp, Mv);
#pragma unroll
                for (int e = 0; e < 9; e++) Mi[(size_t)i * 9 + e] = Mv[e];
            }
        }
        if (mycnt) atomicAdd(&cnt_s, mycnt);
        __syncthreads();
        if (tid < 16) prev[tid] = T[tid];
        if (cnt_s < 4) {   // PCL NotEnoughPointsException: leave the loop unconverged
            aborted = true;
            break;
        }
        if (tid < 9) Rd[tid] = (double)T[4 * (tid / 3) + tid % 3];
        if (tid < 3) td[tid] = (double)T[4 * tid + 3];
        __syncthreads();
        for (int g = 0; g < prm.gn_iterations; g++) {
            double acc[27];
#pragma unroll
            for (int kk = 0; kk < 27; kk++) acc[kk] = 0.0;
            if (tid < kRedLanes) {
                double R[9], t3[3];
#pragma unroll
                for (int e = 0; e < 9; e++) R[e] = Rd[e];
#pragma unroll
                for (int e = 0; e < 3; e++) t3[e] = td[e];
                for (int i = tid; i < M; i += kRedLanes) {
                    const int j = nn[i];
                    if (j < 0) continue;
                    const double p[3] = {(double)ox[i], (double)oy[i], (double)oz[i]};
                    double y[3];
#pragma unroll
                    for (int a = 0; a < 3; a++) y[a] = ((R[3 * a] * p[0] + R[3 * a + 1] * p[1]) + R[3 * a + 2] * p[2]) + t3[a];
                    const double q[3] = {(double)tx[j], (double)ty[j], (double)tz[j]};
                    double Mv[9];   // M_i of this outer iteration (computed with the correspondences)
#pragma unroll
                    for (int e = 0; e < 9; e++) Mv[e] = Mi[(size_t)i * 9 + e];
                    double term[27];
                    gn_terms(y, q, Mv, term);
#pragma unroll
                    for (int kk = 0; kk < 27; kk++) acc[kk] += term[kk];
                }
            }
            // tree over the 256 lanes: s = 128, 64 through LDS, then wave 0 with shuffles
            if (wave >= 2 && wave < 4)
#pragma unroll
                for (int kk = 0; kk < 27; kk++) red[kk * 128 + (tid - 128)] = acc[kk];
            __syncthreads();
            if (wave < 2)
#pragma unroll
                for (int kk = 0; kk < 27; kk++) acc[kk] += red[kk * 128 + tid];
            __syncthreads();
            if (wave == 1)
#pragma unroll
                for (int kk = 0; kk < 27; kk++) red[kk * 128 + lane] = acc[kk];
            __syncthreads();
            if (wave == 0) {
#pragma unroll
                for (int kk = 0; kk < 27; kk++) acc[kk] += red[kk * 128 + lane];
#pragma unroll
                for (int sd = 32; sd > 0; sd >>= 1)
#pragma unroll
                    for (int kk = 0; kk < 27; kk++) acc[kk] += __shfl_down(acc[kk], sd);
                if (lane == 0)
#pragma unroll
                    for (int kk = 0; kk < 27; kk++) sums[kk] = acc[kk];
            }
            __syncthreads();
            if (tid == 0) {
                double H[36], gv[6], dx[6];
                int kk = 0;
                for (int a = 0; a < 6; a++)
                    for (int b = a; b < 6; b++) { H[a * 6 + b] = sums[kk]; H[b * 6 + a] = sums[kk]; kk++; }
                for (int a = 0; a < 6; a++) gv[a] = sums[kk++];
                stop_s = solve6(H, gv, dx) ? 0 : 1;
                if (!stop_s) {
                    double dR[9], Rn[9], tn[3];
                    rodrigues_exp(dx, dR);
                    for (int a = 0; a < 3; a++) {
                        for (int b = 0; b < 3; b++)
                            Rn[3 * a + b] = (dR[3 * a] * Rd[b] + dR[3 * a + 1] * Rd[3 + b]) + dR[3 * a + 2] * Rd[6 + b];
                        tn[a] = ((dR[3 * a] * td[0] + dR[3 * a + 1] * td[1]) + dR[3 * a + 2] * td[2]) + dx[3 + a];
                    }
                    for (int e = 0; e < 9; e++) Rd[e] = Rn[e];
                    for (int e = 0; e < 3; e++) td[e] = tn[e];
                }
            }
            __syncthreads();
            if (stop_s) break;
        }
        if (tid == 0) {
            for (int a = 0; a < 3; a++) {
                for (int b = 0; b < 3; b++) T[4 * a + b] = (float)Rd[3 * a + b];
                T[4 * a + 3] = (float)td[a];
            }
            double delta = 0.0;
            for (int a = 0; a < 4; a++)
                for (int b = 0; b < 4; b++) {
                    const double ratio = (a < 3 && b < 3) ? 1.0 / prm.rot_eps : 1.0 / prm.trans_eps;
                    const double cd = ratio * (double)fabsf(prev[4 * a + b] - T[4 * a + b]);
                    if (cd > delta) delta = cd;
                }
            it_s++;
            if (it_s >= prm.max_iterations || delta < 1) {
                conv_s = 1;
                for (int e = 0; e < 16; e++) prev[e] = T[e];
            }
        }
        __syncthreads();
        if (conv_s) break;
    }
    if (tid == 0) {
        GicpOut o;
        o.converged = (!aborted && conv_s) ? 1 : 0;
        o.iters = it_s;
        o.n_corr = cnt_s;
        for (int e = 0; e < 16; e++) o.T[e] = (e % 5 == 0) ? 1.0f : 0.0f;
        if (o.converged)
            for (int i = 0; i < 4; i++)
                for (int j = 0; j < 4; j++)
                    o.T[4 * i + j] = ((prev[4 * i] * G[j] + prev[4 * i + 1] * G[4 + j]) + prev[4 * i + 2] * G[8 + j])
                                     + prev[4 * i + 3] * G[12 + j];
        *out = o;
    }
}

__global__ __launch_bounds__(kAlignThreads) void k_gicp_align(const float* __restrict__ src, const float* __restrict__ tgt,
                                                              int M, const double* __restrict__ cov,
                                                              const float* __restrict__ guess, GicpDevPrm prm,
                                                              GicpOut* __restrict__ out, double* __restrict__ Mi)
{
    gicp_align_block(src, tgt, M, cov, guess, prm, out, Mi);
}

__global__ __launch_bounds__(kAlignThreads) void k_gicp_align_pairs(LaneBufs lb, LaneCfg lc)
{
    if ((int)blockIdx.x >= lb.pcount[0]) return;
    const int b = lb.plist[blockIdx.x];
    const int M = lb.gn[b];
    const size_t lo = (size_t)b * lc.GM * 3;
    gicp_align_block(lb.gsrc + lo, lb.gtgt + lo, M, lb.gcov + (size_t)b * 2 * lc.GM * 9, lb.gguess + (size_t)b * 16,
                     lc.gp, lb.gout + b, lb.gM + (size_t)b * lc.GM * 9);
}

hipError_t launch_gicp_cov_pairs(const LaneBufs& lb, const LaneCfg& lc, hipStream_t st)
{
    return dispatch(k_gicp_cov_pairs, dim3(kCovPairBlocks), dim3(64 * kCovWaves), 0, st, lb, lc);
}

hipError_t launch_gicp_align_pairs(const LaneBufs& lb, const LaneCfg& lc, hipStream_t st)
{
    return dispatch(k_gicp_align_pairs, dim3(lc.B), dim3(kAlignThreads), 0, st, lb, lc);
}

hipError_t launch_gicp(const float* src, const float* tgt, int M, const float* guess, const GicpDevPrm& prm, double* cov,
                 GicpOut* out, double* Mi, hipStream_t st)
{
    const hipError_t e = dispatch(k_gicp_cov, dim3((2 * M + kCovG * kCovWaves - 1) / (kCovG * kCovWaves)), dim3(64 * kCovWaves),
                                  0, st, src, tgt, M, prm.k, prm.gicp_eps, cov);
    if (e != hipSuccess) return e;
    return dispatch(k_gicp_align, dim3(1), dim3(kAlignThreads), 0, st, src, tgt, M, cov, guess, prm, out, Mi);
}

}  // namespace rgbd

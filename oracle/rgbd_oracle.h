/*
 * rgbd_oracle.h -- C API of the CPU ORACLE (test infrastructure only).
 *
 * THIS IS NOT PRODUCT CODE.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load liboracle.so, and only as the checker / the timed CPU
 * baseline.  The product path (rgbd-slam_amd/, librgbd_hip.so) never links it.
 *
 * The oracle is a scalar C++17 restatement of the reference's hot path
 * (toniortiz/rgbd-slam), function by function, with file:line citations in
 * the .cpp files.  PARITY UNPINNED: the reference ships no tests/fixtures
 *  and cannot be built here (OpenCV/PCL/Eigen absent, SURVEY
 * s8c), so the oracle is pinned only by the known-answer tables the reference
 * itself defines (pattern table, umax, per-level budgets, pyramid/cell shapes,
 * RansacSE3 constants) and by glibc rand() run live; external-library
 * semantics it restates (OpenCV 3.4 / PCL 1.8 / Eigen 3.3) are listed in
 * DESIGN.md "Oracle definitions".
 */
#ifndef RGBD_ORACLE_H
#define RGBD_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* cv::KeyPoint memory layout (28 bytes). */
typedef struct { float x, y, size, angle, response; int32_t octave, class_id; } orc_keypoint;
/* cv::DMatch memory layout (16 bytes). */
typedef struct { int32_t queryIdx, trainIdx, imgIdx; float distance; } orc_dmatch;

typedef struct {
    int32_t nfeatures;      /* Extractor::setParameters(nfeat, ...)  Features/Extractor.cpp:24 */
    float scale_factor;     /* 1.2f */
    int32_t nlevels;        /* 8 */
    int32_t ini_th_fast;    /* 20 */
    int32_t min_th_fast;    /* 7 */
} orc_orb_params;

typedef struct {
    float fx, fy, cx, cy;
    float k1, k2, p1, p2, k3;   /* IntrinsicMatrix::setDistortion order (k1,k2,k3,p1,p2) stored by name */
    float depth_map_factor;     /* RGBDcamera::mDepthMapFactor = 1/factor  Core/RGBDcamera.cpp:21 */
} orc_camera;

typedef struct { int32_t state[31]; int32_t f, r; } orc_rng;      /* glibc random_r TYPE_3 */
typedef struct { double cov; int32_t set; int32_t pad; } orc_sticky;   /* RansacSE3::depthCovariance static */

typedef struct {
    int32_t iterations;        /* 200 */
    uint32_t min_inlier_th;    /* 10 */
    float max_mahalanobis;     /* 3.0f */
    uint32_t sample_size;      /* 4 */
} orc_ransac_params;

/* ---- ORBextractor tables (ctor, Features/ORBextractor.cpp:348-406) ---- */
int orc_orb_tables(const orc_orb_params* p, int width, int height,
                   float* scale, float* inv_scale, int32_t* nfeat_per_level,
                   int32_t* lvl_w, int32_t* lvl_h, int32_t* umax16);
int orc_gauss_kernel7(int32_t* k7);

/* ---- image stages ---- */
void orc_gray(const uint8_t* bgr, int w, int h, uint8_t* gray);
/* pyramid levels written tight (row stride = level width), concatenated level-major */
int orc_pyramid(const uint8_t* gray, int w, int h, const orc_orb_params* p, uint8_t* out);
/* FAST-9 on an arbitrary image region, OpenCV semantics; out = (x,y,score) triples */
int orc_fast(const uint8_t* img, int stride, int cols, int rows, int threshold,
             int32_t* out_xys, int cap);
/* per-level candidates (vToDistributeKeys) as (x,y,score) relative to minBorder */
int orc_level_candidates(const uint8_t* level, int w, int h, const orc_orb_params* p,
                         int32_t* out_xys, int cap);
/* DistributeOctTree on given candidates; out = (x,y,score) in final list order */
int orc_distribute(const int32_t* xys, int n, int minX, int maxX, int minY, int maxY,
                   int N, int32_t* out_xys, int cap);
/* 7x7 sigma=2 fixed-point blur, REFLECT_101 */
void orc_blur(const uint8_t* src, int w, int h, uint8_t* dst);
float orc_fast_atan2(float y, float x);
void orc_cos_sin(float rad, float* c, float* s);

/* ORBextractor::operator() on a gray image */
int orc_detect_and_compute(const uint8_t* gray, int w, int h, const orc_orb_params* p,
                           orc_keypoint* kps, uint8_t* desc, int cap);
/* Frame::Frame: gray + extract + undistort + unproject */
int orc_frame(const uint8_t* bgr, const uint16_t* depth, int w, int h,
              const orc_orb_params* p, const orc_camera* cam,
              orc_keypoint* kps, orc_keypoint* kps_un, uint8_t* desc, float* xyz, int cap);

/* Frame::undistortKeyPoints + uprojectCamera (Core/Frame.cpp:251-281, :91-117) of given keypoints */
void orc_frame_geometry(const orc_keypoint* kps, int n, const uint16_t* depth, int w, const orc_camera* cam,
                        orc_keypoint* kps_un, float* xyz);

/* ---- SVO detector + BRIEF descriptor, the reference's default Extractor(SVO, BRIEF, NORMAL)
 *      (main.cpp:31; orc_svo.cpp) ---- */
typedef struct {
    int32_t nfeatures;   /* retainBest(nfeatures) in Extractor::detectAndCompute, 1000 */
    int32_t nlevels;     /* SVOextractor(nlevels, 5, 20): 8 */
    int32_t cell_size;   /* 5 */
    int32_t threshold;   /* FAST-10 barrier, 20 */
} orc_svo_params;
/* the default 256 x (y1, x1, y2, x2) BRIEF test table (rgbd-slam_amd/csrc/brief_pattern.inc) */
void orc_brief_default_pattern(int8_t* out);
/* halfSample pyramid, levels tight and concatenated; returns total bytes */
int orc_svo_pyramid(const uint8_t* gray, int w, int h, int nlevels, uint8_t* out);
/* fast_corner_detect_10 + fast_corner_score_10 + fast_nonmax_3x3 on one image: (x, y, score) */
int orc_fast10_corners(const uint8_t* img, int w, int h, int barrier, int32_t* xys, int cap);
/* score map: fast_corner_score_10 at corners, 0 elsewhere; returns the corner count */
int orc_fast10_score_map(const uint8_t* img, int w, int h, int barrier, int32_t* score);
float orc_shi_tomasi(const uint8_t* img, int w, int h, int u, int v);
/* SVOextractor::detect: the grid keypoints with response > 20 in cell order */
int orc_svo_detect(const uint8_t* gray, int w, int h, const orc_svo_params* p, orc_keypoint* kps, int cap);
/* KeyPointsFilter::retainBest on responses: order[] = original indices in the retained order */
int orc_retain_best(const float* response, int n, int n_points, int32_t* order);
/* the same with libstdc++'s std::__introselect run at an explicit depth limit (0: heap-select fallback) */
int orc_retain_best_depth(const float* response, int n, int n_points, int depth_limit, int32_t* order);
/* Extractor::detectAndCompute (SVO + BRIEF); pattern NULL = the default table */
int orc_svo_detect_and_compute(const uint8_t* gray, int w, int h, const orc_svo_params* p, const int8_t* pattern,
                               orc_keypoint* kps, uint8_t* desc, int cap);
/* Frame::Frame with the SVO + BRIEF extractor */
int orc_svo_frame(const uint8_t* bgr, const uint16_t* depth, int w, int h, const orc_svo_params* p,
                  const int8_t* pattern, const orc_camera* cam, orc_keypoint* kps, orc_keypoint* kps_un,
                  uint8_t* desc, float* xyz, int cap);

/* ---- Matcher ---- */
/* knn-2 brute force Hamming: out[q*4 + {0,1,2,3}] = d1, i1, d2, i2 (i=-1 if absent) */
void orc_knn2(const uint8_t* dq, int nq, const uint8_t* dt, int nt, int32_t* out);
int orc_match(const uint8_t* dq, int nq, const uint8_t* dt, int nt,
              const uint8_t* outlier_q, const float* z_q, const float* z_t,
              float nnratio, int discard_outliers, orc_dmatch* out);

/* ---- RNG (glibc srand/rand restated) ---- */
void orc_rng_seed(orc_rng* st, uint32_t seed);
int32_t orc_rng_rand(orc_rng* st);
int orc_random_int(orc_rng* st, int mn, int mx);   /* Random::randomInt, System/Random.cpp:16-21 */

/* ---- RansacSE3 (Solver/SolverSE3.cpp:23-297) ----
 * xyz arrays are N x 3 f32 (Frame::mvKeys3Dc).  T21 out is 4x4 row-major.
 * flags2 (optional, may be NULL): F2 outlier flags updated when update_f2. */
/* std::sort of DMatch by distance (libstdc++), order[i] = input index; depth_limit >= 0 forces introsort's limit */
int orc_sort_dmatch(const float* dist, int n, int depth_limit, int32_t* order);
int orc_ransac_se3(const float* xyz1, const float* xyz2, const orc_dmatch* m12, int m,
                   const orc_ransac_params* prm, orc_rng* rng, orc_sticky* sticky,
                   int update_f2, uint8_t* flags2,
                   float* T21, orc_dmatch* inliers, int32_t* n_inliers, float* rmse);
/* one weighted PCL-TransformationFromCorrespondences fit (sequential online update) */
void orc_tfc_fit(const float* p1, const float* p2, const float* w, int n, float* T44);
/* Eigen JacobiSVD 3x3 restatement: U, S(3), V row-major */
void orc_svd3(const double* A, double* U, double* S, double* V);
/* errorFunction2 */
double orc_mahalanobis2(const float* x1, const float* x2, const float* T44, double sticky_cov);

/* ---- PnPRansac (Solver/PnPRansac.cpp:14-56 -> cv::solvePnPRansac, restated definition) ---- */
int orc_cvrng_uniform_stream(uint64_t seed, int count, int n, int32_t* out);
int orc_update_num_iters(double p, double ep, int modelPoints, int maxIters);
int orc_epnp(const float* p3, const float* p2, int n, const float* K4, double* R9, double* t3);
void orc_pnp_set_refine_iters(int n);   /* default 10 (the definition); 0 returns the RANSAC model */
int orc_pnp_ransac(const float* p3, const float* p2, int count, const float* K4, int iterationsCount,
                   float reprojectionError, double confidence, double* R9, double* t3, uint8_t* inlier_mask,
                   int32_t* n_inliers, int32_t* iters_run);

/* ---- GICP (Solver/Gicp.cpp:21-66 -> pcl::GeneralizedIterativeClosestPoint, restated definition) ---- */
typedef struct {
    int32_t max_iterations;          /* Tracking: 10 (System/Tracking.cpp:150); Gicp ctor 15 */
    int32_t k_correspondences;       /* PCL default 20 */
    double max_corr_dist;            /* Tracking: 0.07 (:149); Gicp ctor 0.08 */
    double transformation_epsilon;   /* Gicp ctor 1e-9 (Solver/Gicp.cpp:15) */
    double rotation_epsilon;         /* PCL default 2e-3 */
    double gicp_epsilon;             /* PCL default 1e-3 */
    int32_t gn_iterations;           /* Gauss-Newton steps per outer iteration (replaces PCL's BFGS) */
    int32_t pad;
} orc_gicp_params;
int orc_gicp_covariances(const float* pts, int n, int k, double eps, double* cov);
int orc_gicp(const float* src, const float* tgt, int M, const float* guess, const orc_gicp_params* prm, float* T_out,
             int32_t* converged, int32_t* iters, int32_t* n_corr);
int orc_gicp_compute(const float* src, const float* tgt, int M, const float* guess, const orc_gicp_params* prm,
                     float* T_out);

/* ---- keyframe dense cloud (orc_cloud.cpp; System/Tracking.cpp:234-237) ---- */
/* pcl::PointXYZRGB's payload: xyz + the packed rgb word (bytes b, g, r, 0). */
typedef struct { float x, y, z; uint8_t b, g, r, pad; } orc_point;
int orc_cloud(const uint8_t* bgr, const uint16_t* depth, int W, int H, const orc_camera* cam, int res, float zmin,
              float zmax, orc_point* out, int cap);
int orc_voxel(const orc_point* in, int n, float leaf, orc_point* out);
int orc_sor(const orc_point* in, int n, int k, double std_mul, orc_point* out, float* dist_out);
int orc_keyframe_cloud(const uint8_t* bgr, const uint16_t* depth, int W, int H, const orc_camera* cam,
                       orc_point* out, int cap);

#ifdef __cplusplus
}
#endif
#endif

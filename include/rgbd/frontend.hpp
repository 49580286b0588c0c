// rgbd/frontend.hpp -- header-only C++ surfaces over the C ABI, named and shaped like the
// reference's classes so System/Tracking.cpp-style callers port line for line:
//
//   rgbd::ORBextractor   <- ORBextractor / Extractor(ORB2, ORB2, NORMAL)  Features/ORBextractor.h:9-66
//   rgbd::Extractor      <- Extractor(detector, descriptor, mode): (ORB2, ORB2) or (SVO, BRIEF), NORMAL
//                           (main.cpp:31's default)                       Features/Extractor.h:9-72
//   rgbd::Frame          <- Frame (keys, keysUn, descriptors, keys3Dc, outlier flags, pose)  Core/Frame.h
//   rgbd::Matcher        <- Matcher::match                                Features/Matcher.h:23-24
//   rgbd::RansacSE3      <- RansacSE3::compute + rmse / mvInliers / mT21   Solver/SolverSE3.h:15-57
//   rgbd::Gicp           <- Gicp::compute / align + setters                 Solver/Gicp.h:10-57
//   rgbd::PnPRansac      <- PnPRansac::compute                             Solver/PnPRansac.h
//
// No OpenCV/Eigen types: poses are row-major float[16] (cv::Mat 4x4 CV_32F layout), keypoints and
// matches are the byte-identical rgbd_keypoint / rgbd_dmatch.  INTEGRATION.md shows the thin
// cv::Feature2D / cv::Mat adapters a maintainer adds on the reference side.
#pragma once
#include <array>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../rgbd_hip.h"

namespace rgbd {

class Error : public std::runtime_error {
public:
    using std::runtime_error::runtime_error;
};

inline void check(rgbd_ctx* c, rgbd_status s, const char* what)
{
    if (s != RGBD_OK) throw Error(std::string(what) + ": " + rgbd_last_error(c));
}

using Pose = std::array<float, 16>;
inline Pose identity() { return Pose{1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}; }

// One extraction context (device workspace + camera); what Frame needs from an extractor.
class ExtractorBase {
public:
    // Extractor::detectAndCompute (mask ignored, as in the reference)
    void detectAndCompute(const uint8_t* gray, int step, std::vector<rgbd_keypoint>& kps,
                          std::vector<uint8_t>& desc)
    {
        const int cap = rgbd_max_keypoints(ctx_.get());
        kps.resize(cap);
        desc.resize((size_t)cap * 32);
        int n = 0;
        check(ctx_.get(), rgbd_detect_and_compute(ctx_.get(), gray, step, kps.data(), desc.data(), cap, &n),
              "detectAndCompute");
        kps.resize(n);
        desc.resize((size_t)n * 32);
    }
    rgbd_ctx* ctx() const { return ctx_.get(); }
    const rgbd_camera& camera() const { return cam_; }

protected:
    void adopt(rgbd_ctx* c, rgbd_status s, const rgbd_camera& cam, const char* what)
    {
        cam_ = cam;
        ctx_.reset(c, rgbd_destroy);
        check(c, s, what);
    }
    std::shared_ptr<rgbd_ctx> ctx_;
    rgbd_camera cam_{};
};

// Shared by every Frame of a sequence (main.cpp:31 shares one Extractor); one per thread.
class ORBextractor : public ExtractorBase {
public:
    ORBextractor(int width, int height, const rgbd_camera& cam, int nfeatures = 1000, float scaleFactor = 1.2f,
                 int nlevels = 8, int iniThFAST = 20, int minThFAST = 7, int device = 0, int max_batch = 1)
    {
        rgbd_orb_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST};
        rgbd_ctx* c = nullptr;
        const rgbd_status s = rgbd_create(device, width, height, max_batch, &p, &cam, &c);
        adopt(c, s, cam, "rgbd_create");
    }
};

// Extractor(eType detector, eType descriptor, eMode mode) -- Features/Extractor.cpp:15-22.  The accelerated
// pairs are (ORB2, ORB2) and (SVO, BRIEF) in NORMAL mode (main.cpp:31 runs the latter); the OpenCV stock
// detectors / descriptors and the ADAPTIVE wrappers are not on this path and throw.
class Extractor : public ExtractorBase {
public:
    enum eType { ORB = 0, ORB2, SVO, FAST, GFTT, STAR, BRISK, FREAK, BRIEF, LATCH, SURF, SIFT };
    enum eMode { NORMAL = 0, ADAPTIVE };

    Extractor(eType detector, eType descriptor, eMode mode, int width, int height, const rgbd_camera& cam,
              int device = 0, int max_batch = 1)
        : mDetectorType(detector), mDescriptorType(descriptor), mMode(mode), W_(width), H_(height),
          device_(device), maxB_(max_batch)
    {
        const bool orb2 = detector == ORB2 && descriptor == ORB2, svo = detector == SVO && descriptor == BRIEF;
        if (mode != NORMAL || !(orb2 || svo))
            throw Error("Extractor: only (ORB2, ORB2) and (SVO, BRIEF) in NORMAL mode are accelerated");
        cam_ = cam;
        setParameters(1000, 1.2f, 8, 20, 7);   // :21
    }
    // Extractor::setParameters (:24-48): recreates the context
    void setParameters(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
    {
        nfeatures_ = nfeatures;
        scale_ = scaleFactor;
        nlevels_ = nlevels;
        rgbd_ctx* c = nullptr;
        rgbd_status s;
        if (mDetectorType == SVO) {
            rgbd_svo_params p{nfeatures, nlevels, 5, 20, 0};   // SVOextractor(nlevels, 5, 20), :162-165
            s = rgbd_create_svo(device_, W_, H_, maxB_, &p, &cam_, &c);
        } else {
            rgbd_orb_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST};
            s = rgbd_create(device_, W_, H_, maxB_, &p, &cam_, &c);
        }
        adopt(c, s, cam_, "Extractor");
    }
    // getters (:97-151); the SVO branch reports init()'s tables, the ORB2 branch ORBextractor's (same values)
    int getLevels() const { return nlevels_; }
    float getScaleFactor() const { return scale_; }
    std::vector<float> getScaleFactors() const
    {
        std::vector<float> f((size_t)nlevels_, 1.0f);
        for (int i = 1; i < nlevels_; i++) f[i] = f[i - 1] * scale_;
        return f;
    }
    std::vector<float> getInverseScaleFactors() const
    {
        std::vector<float> f = getScaleFactors();
        for (float& v : f) v = 1.0f / v;
        return f;
    }
    std::vector<float> getScaleSigmaSquares() const
    {
        std::vector<float> f = getScaleFactors();
        for (float& v : f) v = v * v;
        return f;
    }
    std::vector<float> getInverseScaleSigmaSquares() const
    {
        std::vector<float> f = getScaleSigmaSquares();
        for (float& v : f) v = 1.0f / v;
        return f;
    }
    // OpenCV's own BRIEF tests (opencv_contrib generated_32.i), 256 x {y1, x1, y2, x2}; SVO contexts only
    void setBriefPattern(const int8_t* pairs) { check(ctx_.get(), rgbd_svo_set_brief_pattern(ctx_.get(), pairs), "setBriefPattern"); }

    eType mDetectorType, mDescriptorType;
    eMode mMode;

private:
    int W_, H_, device_, maxB_;
    int nfeatures_ = 1000, nlevels_ = 8;
    float scale_ = 1.2f;
};

class Frame {
public:
    using Ptr = std::shared_ptr<Frame>;
    // Frame(imRGB, imDepth, ts, Extractor, RGBDcamera*) -- Core/Frame.cpp:34-73
    Frame(const uint8_t* bgr, const uint16_t* depth, double timeStamp, const ExtractorBase& ex)
        : mTimeStamp(timeStamp), mCamera(ex.camera())
    {
        rgbd_ctx* c = ex.ctx();
        const int cap = rgbd_max_keypoints(c);
        mvKeys.resize(cap);
        mvKeysUn.resize(cap);
        mDescriptors.resize((size_t)cap * 32);
        mvKeys3Dc.resize((size_t)cap * 3);
        int n = 0;
        check(c, rgbd_frame(c, bgr, depth, mvKeys.data(), mvKeysUn.data(), mDescriptors.data(), mvKeys3Dc.data(),
                            cap, &n), "Frame");
        N = n;
        mvKeys.resize(n);
        mvKeysUn.resize(n);
        mDescriptors.resize((size_t)n * 32);
        mvKeys3Dc.resize((size_t)n * 3);
        mvbOutlier.assign(n, 0);
    }
    bool isValidObs(size_t i) const { return mvKeys3Dc[3 * i + 2] > 0; }      // Core/Frame.cpp:415-418
    bool isOutlier(size_t i) const { return mvbOutlier[i] != 0; }
    void setPose(const Pose& T) { mTcw = T; }
    const Pose& getPose() const { return mTcw; }
    std::vector<float> depths() const
    {
        std::vector<float> z(N);
        for (int i = 0; i < N; i++) z[i] = mvKeys3Dc[3 * (size_t)i + 2];
        return z;
    }

    int N = 0;
    double mTimeStamp = 0;
    rgbd_camera mCamera{};                  // mpCamera (RGBDcamera)
    std::vector<rgbd_keypoint> mvKeys, mvKeysUn;
    std::vector<uint8_t> mDescriptors;      // N x 32
    std::vector<float> mvKeys3Dc;           // N x 3
    std::vector<uint8_t> mvbOutlier;
    Pose mTcw = identity();
};

class Matcher {
public:
    explicit Matcher(rgbd_ctx* ctx, float nnratio = 0.6f) : ctx_(ctx), mfNNratio(nnratio) {}
    int match(const Frame& ref, const Frame& cur, std::vector<rgbd_dmatch>& vMatches12, bool discardOutliers = true)
    {
        vMatches12.resize(std::max(ref.N, 1));
        int m = 0;
        const std::vector<float> zq = ref.depths(), zt = cur.depths();
        check(ctx_, rgbd_match(ctx_, ref.mDescriptors.data(), ref.N, cur.mDescriptors.data(), cur.N,
                               ref.mvbOutlier.data(), zq.data(), zt.data(), mfNNratio, discardOutliers ? 1 : 0,
                               vMatches12.data(), (int)vMatches12.size(), &m), "match");
        vMatches12.resize(m);
        return m;
    }

private:
    rgbd_ctx* ctx_;
    float mfNNratio;
};

// RNG and sticky covariance are process-global in the reference (System/Random.cpp, SolverSE3.cpp:284);
// here they live in a Session object the caller owns and passes to every solver.
struct Session {
    explicit Session(uint32_t seed = 1) { rgbd_rng_seed(&rng, seed); }
    rgbd_rng rng{};
    rgbd_sticky sticky{};
};

class RansacSE3 {
public:
    RansacSE3(rgbd_ctx* ctx, Session& s, int iters = 200, unsigned minInlierTh = 20, float maxMahalanobisDist = 3.0f,
              unsigned sampleSize = 4)
        : ctx_(ctx), s_(s), prm_{iters, minInlierTh, maxMahalanobisDist, sampleSize}
    {
    }
    // x2 = mT21 * x1; on success with updateF2, F2's pose = mT21 * pose(F1) (:119-126)
    bool compute(const Frame& F1, Frame& F2, const std::vector<rgbd_dmatch>& m12, bool updateF2 = true)
    {
        mvInliers.resize(std::max<size_t>(m12.size(), 1));
        int n_in = 0, ok = 0;
        check(ctx_, rgbd_ransac_se3(ctx_, F1.mvKeys3Dc.data(), F1.N, F2.mvKeys3Dc.data(), F2.N, m12.data(),
                                    (int)m12.size(), &prm_, &s_.rng, &s_.sticky, updateF2 ? 1 : 0,
                                    F2.mvbOutlier.data(), mT21.data(), mvInliers.data(), &n_in, &rmse, &ok),
              "RansacSE3");
        mvInliers.resize(n_in);
        if (ok && updateF2) {
            Pose P;
            const Pose& A = mT21;
            const Pose& B = F1.getPose();
            for (int i = 0; i < 4; i++)
                for (int j = 0; j < 4; j++) {
                    double acc = 0.0;   // cv::Mat CV_32F gemm accumulates in double
                    for (int k = 0; k < 4; k++) acc += (double)A[4 * i + k] * (double)B[4 * k + j];
                    P[4 * i + j] = (float)acc;
                }
            F2.setPose(P);
        }
        return ok != 0;
    }

    float rmse = 1e6f;
    std::vector<rgbd_dmatch> mvInliers;
    Pose mT21 = identity();

private:
    rgbd_ctx* ctx_;
    Session& s_;
    rgbd_ransac_params prm_;
};

inline Pose pose_mul(const Pose& A, const Pose& B)   // cv::Mat CV_32F gemm: double accumulation
{
    Pose P;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double acc = 0.0;
            for (int k = 0; k < 4; k++) acc += (double)A[4 * i + k] * (double)B[4 * k + j];
            P[4 * i + j] = (float)acc;
        }
    return P;
}

// Gicp(F1, F2, matches, guess): clouds = F1 / F2 3D of the matches (createCloudsFromMatches); on
// success F2's pose = mT * pose(F1) (Solver/Gicp.cpp:21-35).  Ctor defaults: 15 iterations, 0.08 m.
class Gicp {
public:
    Gicp(rgbd_ctx* ctx, const Frame& F1, Frame& F2, const std::vector<rgbd_dmatch>& matches, const Pose& guess)
        : ctx_(ctx), F1_(F1), F2_(F2), matches_(matches), guess_(guess)
    {
    }
    void setMaximumIterations(int iters) { prm_.max_iterations = iters; }
    void setMaxCorrespondenceDistance(double dist) { prm_.max_corr_dist = dist; }
    void setTransformationEpsilon(double eps) { prm_.transformation_epsilon = eps; }
    bool compute(std::vector<rgbd_dmatch>& /*inliers*/)
    {
        const int M = (int)matches_.size();
        std::vector<float> src((size_t)std::max(M, 1) * 3), tgt((size_t)std::max(M, 1) * 3);
        for (int i = 0; i < M; i++)
            for (int k = 0; k < 3; k++) {
                src[3 * i + k] = F1_.mvKeys3Dc[3 * (size_t)matches_[i].queryIdx + k];
                tgt[3 * i + k] = F2_.mvKeys3Dc[3 * (size_t)matches_[i].trainIdx + k];
            }
        int ok = 0;
        check(ctx_, rgbd_gicp_compute(ctx_, src.data(), tgt.data(), M, guess_.data(), &prm_, mT.data(), &ok), "Gicp");
        if (ok && mbUpdate) F2_.setPose(pose_mul(mT, F1_.getPose()));
        return ok != 0;
    }

    bool mbUpdate = true;
    Pose mT = identity();

private:
    rgbd_ctx* ctx_;
    const Frame& F1_;
    Frame& F2_;
    const std::vector<rgbd_dmatch>& matches_;
    Pose guess_;
    rgbd_gicp_params prm_{15, 20, 0.08, 1e-9, 2e-3, 1e-3, 4, 1};
};

// PnPRansac(F1, F2, matches).compute(inliers) (Solver/PnPRansac.cpp:14-56).  as_written = true keeps
// the reference's code as it stands: object points = F2's own back-projection (unprojectWorld with F2's
// current pose, :28-30), and the pose Converter::toHomogeneous builds (:42, System/Converter.cpp:27-37):
// Rodrigues reallocates R as CV_64F, and R.copyTo(Tcw.rowRange(0, 3).colRange(0, 3)) hands a temporary ROI
// to an _OutputArray(const Mat&), which is FIXED_TYPE | FIXED_SIZE; Mat::copyTo into a fixed-type
// destination of another type converts in place (convertTo), so Tcw = [float(R) | float(t)] written into
// Tcw's own data (OpenCV 3.x semantics recalled, parity unpinned: OpenCV is absent) and
// F2's pose becomes that matrix -- not composed with F1's pose.  The default (as_written = false) pairs
// F1's 3D with F2's pixels -- the pairing the tracking benchmark needs -- and sets F2's pose =
// [R|t] pose(F1).  R and t (the solver's rvec / tvec as a rotation matrix) are kept in both modes.
class PnPRansac {
public:
    PnPRansac(rgbd_ctx* ctx, const Frame& F1, Frame& F2, const std::vector<rgbd_dmatch>& matches, bool as_written = false)
        : ctx_(ctx), F1_(F1), F2_(F2), matches_(matches), as_written_(as_written)
    {
    }
    bool compute(std::vector<rgbd_dmatch>& inliers)
    {
        const int M = (int)matches_.size();
        if (M < 10) return false;
        std::vector<float> p3((size_t)M * 3), p2((size_t)M * 2);
        const Pose& Tw = F2_.getPose();   // unprojectWorld: Rwc x + Ow, Twc = Tcw^-1
        for (int i = 0; i < M; i++) {
            const rgbd_dmatch& m = matches_[i];
            const rgbd_keypoint& ku = F2_.mvKeysUn[m.trainIdx];
            p2[2 * i] = ku.x;
            p2[2 * i + 1] = ku.y;
            if (as_written_) {
                // Frame::unprojectWorld (Core/Frame.cpp:317-327): mRwc * x + mOw with the float members
                // set by updatePoseMatrices (:143-153): Rwc = Rcw^T, Ow = -Rcw^T tcw (cv::Mat gemm,
                // double accumulation, one rounding; alpha = -1 for Ow, + Ow as the gemm's C term)
                const float* x = &F2_.mvKeys3Dc[3 * (size_t)m.trainIdx];
                for (int r = 0; r < 3; r++) {
                    double o = 0.0;
                    for (int k = 0; k < 3; k++) o += (double)Tw[4 * k + r] * (double)Tw[4 * k + 3];
                    const float Ow = (float)(o * -1.0);
                    double a = 0.0;
                    for (int k = 0; k < 3; k++) a += (double)Tw[4 * k + r] * (double)x[k];
                    p3[3 * i + r] = (float)(a * 1.0 + (double)Ow * 1.0);
                }
            } else {
                for (int r = 0; r < 3; r++) p3[3 * i + r] = F1_.mvKeys3Dc[3 * (size_t)m.queryIdx + r];
            }
            F2_.mvbOutlier[m.trainIdx] = 1;
        }
        const float K4[4] = {F2_.mCamera.fx, F2_.mCamera.fy, F2_.mCamera.cx, F2_.mCamera.cy};   // mpCamera->k()
        rgbd_pnp_params prm{500, 3.0f, 0.85, 10, 0};
        std::vector<uint8_t> mask(M);
        int ninl = 0, iters = 0, ok = 0;
        check(ctx_, rgbd_pnp_ransac(ctx_, p3.data(), p2.data(), M, K4, &prm, R.data(), t.data(), mask.data(), &ninl,
                                    &iters, &ok), "PnPRansac");
        if (!ok) return false;
        Pose T = identity();
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) T[4 * r + c] = (float)R[3 * r + c];
            T[4 * r + 3] = (float)t[r];
        }
        F2_.setPose(as_written_ ? T : pose_mul(T, F1_.getPose()));   // as written: toHomogeneous's [float(R) | float(t)]
        inliers.clear();
        for (int i = 0; i < M; i++)
            if (mask[i]) {
                inliers.push_back(matches_[i]);
                F2_.mvbOutlier[matches_[i].trainIdx] = 0;
            }
        return true;
    }

    std::array<double, 9> R{};
    std::array<double, 3> t{};

private:
    rgbd_ctx* ctx_;
    const Frame& F1_;
    Frame& F2_;
    const std::vector<rgbd_dmatch>& matches_;
    bool as_written_;
};

}  // namespace rgbd

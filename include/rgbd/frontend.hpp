// rgbd/frontend.hpp -- header-only C++ surfaces over the C ABI, named and shaped like the
// reference's classes so System/Tracking.cpp-style callers port line for line:
//
//   rgbd::ORBextractor   <- ORBextractor / Extractor(ORB2, ORB2, NORMAL)  Features/ORBextractor.h:9-66
//   rgbd::Frame          <- Frame (keys, keysUn, descriptors, keys3Dc, outlier flags, pose)  Core/Frame.h
//   rgbd::Matcher        <- Matcher::match                                Features/Matcher.h:23-24
//   rgbd::RansacSE3      <- RansacSE3::compute + rmse / mvInliers / mT21   Solver/SolverSE3.h:15-57
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

// Shared by every Frame of a sequence (main.cpp:31 shares one Extractor); one per thread.
class ORBextractor {
public:
    ORBextractor(int width, int height, const rgbd_camera& cam, int nfeatures = 1000, float scaleFactor = 1.2f,
                 int nlevels = 8, int iniThFAST = 20, int minThFAST = 7, int device = 0, int max_batch = 1)
    {
        rgbd_orb_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST};
        rgbd_ctx* c = nullptr;
        rgbd_status s = rgbd_create(device, width, height, max_batch, &p, &cam, &c);
        ctx_.reset(c, rgbd_destroy);
        check(c, s, "rgbd_create");
    }
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

private:
    std::shared_ptr<rgbd_ctx> ctx_;
};

class Frame {
public:
    using Ptr = std::shared_ptr<Frame>;
    // Frame(imRGB, imDepth, ts, Extractor, RGBDcamera*) -- Core/Frame.cpp:34-73
    Frame(const uint8_t* bgr, const uint16_t* depth, double timeStamp, ORBextractor& ex) : mTimeStamp(timeStamp)
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

}  // namespace rgbd

// ref_mirror.hpp -- the reference-side surface that INTEGRATION.md's bodies are written against, mirrored
// so those bodies compile and run here (OpenCV, Eigen, PCL and the rest of the reference are absent offline).
//
// The classes keep the reference's names, members and signatures for everything the bodies touch:
//   Solver                 Solver/Solver.h:10-26        (mF1, mF2, mMatches; compute(inliers))
//   PnPRansac              Solver/PnPRansac.h:6-14
//   Gicp                   Solver/Gicp.h:10-56          (mbUpdate, mT, mGuess, the setters, mGicp)
//   RansacSE3              Solver/SolverSE3.h:11-60     (rmse, mvInliers, mT21, the four parameters)
//   Matcher                Features/Matcher.h:12-40     (mfNNratio)
//   Extractor/ORBextractor Features/Extractor.h:9-60, Features/ORBextractor.h
//   Frame                  Core/Frame.h:24-170          (N, mvKeys, mvKeysUn, mvKeys3Dc, mDescriptors,
//                                                        mvbOutlier, pose members, the flag accessors)
// The integration adds one member: Extractor::context(), the device context (librgbd_hip.so) an Extractor
// owns; Frames reach it through mpExtractor.  The cv / Eigen types are the smallest stand-ins with the
// reference's names and the semantics the bodies rely on: cv::Mat is a 2-D CV_8U / CV_32F / CV_64F matrix
// (and the CV_8UC3 / CV_16U images a Frame is built from; at<T>, eye, create = reallocate unless size and
// type match, release, rowRange / colRange views, copyTo,
// clone, the CV_32F product as cv::gemm: double accumulation in k order, one rounding); cv::KeyPoint and
// cv::DMatch are byte-identical to rgbd_keypoint / rgbd_dmatch; Eigen::Matrix4f is row-indexed
// (operator()(r, c)) with isIdentity() at float precision (1e-5).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <vector>

#include "rgbd_hip.h"

constexpr int CV_8U = 0;
constexpr int CV_16U = 2;
constexpr int CV_32F = 5;
constexpr int CV_64F = 6;
constexpr int CV_8UC3 = 16;

namespace cv {

struct Point2f {
    float x = 0, y = 0;
};
struct Point3f {
    float x = 0, y = 0, z = 0;
};
struct KeyPoint {
    Point2f pt;
    float size = 0, angle = -1, response = 0;
    int octave = 0, class_id = -1;
};
struct DMatch {
    int queryIdx = -1, trainIdx = -1, imgIdx = -1;
    float distance = 0;
    bool operator<(const DMatch& m) const { return distance < m.distance; }
};
static_assert(sizeof(KeyPoint) == sizeof(rgbd_keypoint), "cv::KeyPoint == rgbd_keypoint (28 B)");
static_assert(sizeof(DMatch) == sizeof(rgbd_dmatch), "cv::DMatch == rgbd_dmatch (16 B)");

class Mat {
public:
    int rows = 0, cols = 0;
    uint8_t* data = nullptr;
    size_t step = 0;   // bytes per row

    Mat() = default;
    Mat(int r, int c, int type) { create(r, c, type); }
    static Mat eye(int r, int c, int type)
    {
        Mat m(r, c, type);
        for (int i = 0; i < r && i < c; i++) m.set(i, i, 1.0);
        return m;
    }
    int type() const { return type_; }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    size_t elemSize() const
    {
        return type_ == CV_8U ? 1 : type_ == CV_8UC3 ? 3 : type_ == CV_16U ? 2 : type_ == CV_32F ? 4 : 8;
    }
    // OpenCV: no reallocation when size and type already match
    void create(int r, int c, int type)
    {
        if (data && r == rows && c == cols && type == type_) return;
        type_ = type;
        rows = r;
        cols = c;
        step = (size_t)c * elemSize();
        buf_ = std::make_shared<std::vector<uint8_t>>((size_t)r * step + 1);
        data = buf_->data();
    }
    void release()
    {
        buf_.reset();
        data = nullptr;
        rows = cols = 0;
        step = 0;
    }
    template <typename T>
    T& at(int r, int c) { return reinterpret_cast<T*>(data + (size_t)r * step)[c]; }
    template <typename T>
    const T& at(int r, int c) const { return reinterpret_cast<const T*>(data + (size_t)r * step)[c]; }
    template <typename T>
    T& at(int i) { return rows == 1 ? at<T>(0, i) : at<T>(i, 0); }
    uint8_t* ptr(int r) { return data + (size_t)r * step; }
    Mat rowRange(int a, int b) const
    {
        Mat v = *this;
        v.rows = b - a;
        v.data = data + (size_t)a * step;
        return v;
    }
    Mat colRange(int a, int b) const
    {
        Mat v = *this;
        v.cols = b - a;
        v.data = data + (size_t)a * elemSize();
        return v;
    }
    Mat col(int c) const { return colRange(c, c + 1); }
    // copyTo: a destination of another size / type is reallocated; a fixed view of the right size converts
    // in place (Mat::copyTo's convertTo branch, the App. A-9 behaviour of toHomogeneous)
    void copyTo(Mat& dst) const
    {
        if (dst.data && dst.rows == rows && dst.cols == cols) {
            for (int r = 0; r < rows; r++)
                for (int c = 0; c < cols; c++) dst.set(r, c, get(r, c));
            return;
        }
        dst.create(rows, cols, type_);
        for (int r = 0; r < rows; r++) std::memcpy(dst.ptr(r), data + (size_t)r * step, (size_t)cols * elemSize());
    }
    Mat clone() const
    {
        Mat m;
        copyTo(m);
        return m;
    }
    double get(int r, int c) const
    {
        if (type_ == CV_32F) return at<float>(r, c);
        if (type_ == CV_64F) return at<double>(r, c);
        return at<uint8_t>(r, c);
    }
    void set(int r, int c, double v)
    {
        if (type_ == CV_32F) at<float>(r, c) = (float)v;
        else if (type_ == CV_64F) at<double>(r, c) = v;
        else at<uint8_t>(r, c) = (uint8_t)v;
    }

private:
    int type_ = CV_8U;
    std::shared_ptr<std::vector<uint8_t>> buf_;
};

// A * B of two CV_32F matrices: cv::gemm (double accumulation in k order, one rounding to float)
inline Mat operator*(const Mat& A, const Mat& B)
{
    if (A.type() != CV_32F || B.type() != CV_32F || A.cols != B.rows) throw std::runtime_error("cv::Mat product");
    Mat C(A.rows, B.cols, CV_32F);
    for (int i = 0; i < A.rows; i++)
        for (int j = 0; j < B.cols; j++) {
            double s = 0.0;
            for (int k = 0; k < A.cols; k++) s += (double)A.at<float>(i, k) * (double)B.at<float>(k, j);
            C.at<float>(i, j) = (float)s;
        }
    return C;
}

class _InputArray {
public:
    _InputArray(const Mat& m) : m_(&m) {}
    Mat getMat() const { return *m_; }
    bool empty() const { return m_->empty(); }

private:
    const Mat* m_;
};
class _OutputArray {
public:
    _OutputArray(Mat& m) : m_(&m) {}
    void create(int r, int c, int type) const { m_->create(r, c, type); }
    Mat getMat() const { return *m_; }
    void release() const { m_->release(); }

private:
    Mat* m_;
};
using InputArray = const _InputArray&;
using OutputArray = const _OutputArray&;

}  // namespace cv

namespace Eigen {
class Matrix4f {
public:
    float& operator()(int r, int c) { return a_[4 * r + c]; }
    float operator()(int r, int c) const { return a_[4 * r + c]; }
    static Matrix4f Identity()
    {
        Matrix4f m;
        for (int i = 0; i < 4; i++) m(i, i) = 1.0f;
        return m;
    }
    // DenseBase::isIdentity(prec = NumTraits<float>::dummy_precision() = 1e-5)
    bool isIdentity(float prec = 1e-5f) const
    {
        for (int r = 0; r < 4; r++)
            for (int c = 0; c < 4; c++) {
                const float v = (*this)(r, c);
                if (r == c ? !(std::fabs(v - 1.0f) <= prec * std::fmin(std::fabs(v), 1.0f)) : !(std::fabs(v) <= prec))
                    return false;
            }
        return true;
    }

private:
    float a_[16] = {};
};
}  // namespace Eigen

namespace Converter {
// Converter::toMat<float, 4, 4> (System/Converter.h): the Eigen matrix as a CV_32F cv::Mat
template <typename T, int R, int C>
cv::Mat toMat(const Eigen::Matrix4f& m)
{
    static_assert(R == 4 && C == 4, "mirror: 4x4 only");
    cv::Mat out(4, 4, CV_32F);
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) out.at<float>(r, c) = m(r, c);
    return out;
}
}  // namespace Converter

// RGBDcamera (Core/RGBDcamera.h): intrinsics, distortion and the depth factor
class RGBDcamera {
public:
    float fx = 0, fy = 0, cx = 0, cy = 0, k1 = 0, k2 = 0, p1 = 0, p2 = 0, k3 = 0;
    float mDepthMapFactor = 1.0f;   // 1 / factor (Core/RGBDcamera.cpp)
    cv::Mat k() const
    {
        cv::Mat K = cv::Mat::eye(3, 3, CV_32F);
        K.at<float>(0, 0) = fx;
        K.at<float>(1, 1) = fy;
        K.at<float>(0, 2) = cx;
        K.at<float>(1, 2) = cy;
        return K;
    }
    rgbd_camera abi() const { return rgbd_camera{fx, fy, cx, cy, k1, k2, p1, p2, k3, mDepthMapFactor}; }
};

// Extractor (Features/Extractor.h:9-60).  Integration member: context() -- the device context this Extractor
// owns, created on first use for the image size and camera of the first frame it sees.
class Extractor {
public:
    using Ptr = std::shared_ptr<Extractor>;
    enum eType { ORB = 0, ORB2, SVO, FAST, GFTT, STAR, BRISK, FREAK, BRIEF, LATCH, SURF, SIFT };
    enum eMode { NORMAL = 0, ADAPTIVE };
    eType mDetectorType, mDescriptorType;
    eMode mMode;
    Extractor(eType detector, eType descriptor, eMode mode);   // solver_bodies.cpp
    ~Extractor();
    void setParameters(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST);
    void detectAndCompute(cv::InputArray image, cv::InputArray mask, std::vector<cv::KeyPoint>& keypoints,
                          cv::OutputArray descriptors);
    rgbd_ctx* context(int width, int height, const RGBDcamera& cam);
    rgbd_ctx* context() const { return mCtx; }

    int nfeatures = 1000, nlevels = 8, iniThFAST = 20, minThFAST = 7;
    float scaleFactor = 1.2f;

private:
    rgbd_ctx* mCtx = nullptr;
};

class Frame {
public:
    using Ptr = std::shared_ptr<Frame>;
    Frame(const cv::Mat& imRGB, const cv::Mat& imDepth, const double& timeStamp, std::shared_ptr<Extractor> pExtractor,
          RGBDcamera* pRGBDcamera);   // solver_bodies.cpp

    // Core/Frame.cpp:124-147: setPose clones Tcw and updates the pose members
    void setPose(cv::Mat Tcw)
    {
        mTcw = Tcw.clone();
        updatePoseMatrices();
    }
    cv::Mat getPose() const { return mTcw.clone(); }
    // mRcw = Tcw(0:3, 0:3), mRwc = mRcw^T, mtcw = Tcw(0:3, 3), mOw = -mRcw^T mtcw (one gemm: double sums,
    // alpha -1, one rounding)
    void updatePoseMatrices()
    {
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) mRwc[3 * r + c] = mTcw.at<float>(c, r);
            double o = 0.0;
            for (int k = 0; k < 3; k++) o += (double)mTcw.at<float>(k, r) * (double)mTcw.at<float>(k, 3);
            mOw[r] = (float)(o * -1.0);
        }
    }
    // Core/Frame.cpp:317-327: mRwc * x3Dc + mOw (one gemm with mOw as its C term), empty when z <= 0
    cv::Mat unprojectWorld(const size_t& i)
    {
        if (!(mvKeys3Dc[i].z > 0)) return cv::Mat();
        const float x[3] = {mvKeys3Dc[i].x, mvKeys3Dc[i].y, mvKeys3Dc[i].z};
        cv::Mat X(3, 1, CV_32F);
        for (int r = 0; r < 3; r++) {
            double a = 0.0;
            for (int k = 0; k < 3; k++) a += (double)mRwc[3 * r + k] * (double)x[k];
            X.at<float>(r, 0) = (float)(a * 1.0 + (double)mOw[r] * 1.0);
        }
        return X;
    }
    bool isOutlier(const size_t& idx) const { return mvbOutlier[idx] == true; }
    void setInlier(const size_t& idx) { mvbOutlier[idx] = false; }
    void setOutlier(const size_t& idx) { mvbOutlier[idx] = true; }
    bool isValidObs(const size_t& idx) { return mvKeys3Dc[idx].z > 0; }

    std::shared_ptr<Extractor> mpExtractor;
    RGBDcamera* mpCamera;
    double mTimeStamp;
    size_t N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
    std::vector<cv::Point3f> mvKeys3Dc;
    cv::Mat mDescriptors;
    std::vector<bool> mvbOutlier;

private:
    cv::Mat mTcw;
    float mRwc[9] = {}, mOw[3] = {};
};

class Matcher {
public:
    using Ptr = std::shared_ptr<Matcher>;
    Matcher(float nnratio = 0.6) : mfNNratio(nnratio) {}
    int match(std::shared_ptr<Frame> ref, std::shared_ptr<Frame> cur, std::vector<cv::DMatch>& vMatches12,
              const bool discardOutliers = true);   // solver_bodies.cpp

protected:
    float mfNNratio;
};

class Solver {
public:
    using Ptr = std::shared_ptr<Solver>;
    Solver(const std::shared_ptr<Frame> F1, std::shared_ptr<Frame> F2, const std::vector<cv::DMatch>& matches)
        : mF1(F1), mF2(F2), mMatches(matches)
    {
    }
    virtual ~Solver() {}
    virtual bool compute(std::vector<cv::DMatch>& inliers) = 0;

protected:
    const std::shared_ptr<Frame> mF1;
    std::shared_ptr<Frame> mF2;
    const std::vector<cv::DMatch>& mMatches;
};

class PnPRansac : public Solver {
public:
    PnPRansac(const std::shared_ptr<Frame> F1, std::shared_ptr<Frame> F2, const std::vector<cv::DMatch>& matches)
        : Solver(F1, F2, matches)
    {
    }
    ~PnPRansac() {}
    bool compute(std::vector<cv::DMatch>& inliers) override;   // solver_bodies.cpp
};

class Gicp : public Solver {
public:
    Gicp(const std::shared_ptr<Frame> F1, std::shared_ptr<Frame> F2, const std::vector<cv::DMatch>& matches,
         Eigen::Matrix4f& guess);   // solver_bodies.cpp
    virtual ~Gicp() {}
    bool compute(std::vector<cv::DMatch>& inliers) override;
    Eigen::Matrix4f align();
    void setMaximumIterations(int iters);
    void setMaxCorrespondenceDistance(double dist);
    void setEuclideanFitnessEpsilon(double epsilon);
    void setTransformationEpsilon(double epsilon);

    bool mbUpdate;
    Eigen::Matrix4f mT;

private:
    void createCloudsFromMatches();
    rgbd_gicp_params mGicp;   // the registration's parameters (PCL's GeneralizedIterativeClosestPoint in the reference)
    Eigen::Matrix4f mGuess;

public:
    std::vector<float> mpSrcCloud, mpTgtCloud;   // M x 3 (pcl::PointCloud<pcl::PointXYZ> in the reference)
};

class RansacSE3 {
public:
    RansacSE3();
    RansacSE3(int iters, unsigned minInlierTh, float maxMahalanobisDist, unsigned sampleSize);
    ~RansacSE3() {}
    bool compute(std::shared_ptr<Frame> pF1, std::shared_ptr<Frame> pF2, const std::vector<cv::DMatch>& m12,
                 const bool& updateF2 = true);   // solver_bodies.cpp

private:
    int mIterations;
    unsigned mMinInlierTh;
    float mMaxMahalanobisDistance;
    unsigned mSampleSize;

public:
    float rmse;
    std::vector<cv::DMatch> mvInliers;
    Eigen::Matrix4f mT21;
};

// Random (System/Random.h): initSeed() seeds the process's rand() once (srand(time(NULL))).  RansacSE3 draws
// its samples from that stream and keeps a function-static depth covariance (Solver/SolverSE3.cpp:282-287);
// on the device both are explicit, so the integration keeps them here as the same process-wide state:
// initSeed() seeds the device stream with the same seed (initSeed(seed): a fixed seed, for tests).
class Random {
public:
    static void initSeed();
    static void initSeed(unsigned seed);
    static rgbd_rng& stream();            // RansacSE3's rand() stream
    static rgbd_sticky& depthCovariance();  // RansacSE3::depthCovariance's statics

protected:
    static bool SET_RAND;
};

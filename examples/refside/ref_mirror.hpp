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
//   Frame                  Core/Frame.h:24-216          (mnId / nNextId / id(), mImColor, mImGray, mImDepth, N,
//                                                        mvKeys, mvKeysUn, mvKeys3Dc, mvKeysColor, mDescriptors,
//                                                        mvbOutlier, mvpLandmarks, the grid and image bounds,
//                                                        mpReferenceKF, the pose members, the flag accessors)
//   Landmark, Map          Core/Landmark.h, Core/Map.h  (what Tracking::initialize / PoseGraph touch)
//   Tracking, PoseGraph    System/Tracking.h, Solver/PoseGraph.h (the members track() and the PoseGraph
//                                                        thread use; their code is restated in ref_system.cpp)
// The integration adds one member: Extractor::context(), the device context (librgbd_hip.so) an Extractor
// owns FOR THE CALLING THREAD (the tracking thread and the PoseGraph thread each get their own); Frames reach
// it through mpExtractor.  The cv / Eigen types are the smallest stand-ins with the
// reference's names and the semantics the bodies rely on: cv::Mat is a 2-D CV_8U / CV_32F / CV_64F matrix
// (and the CV_8UC3 / CV_16U images a Frame is built from; at<T>, eye, create = reallocate unless size and
// type match, release, rowRange / colRange views, copyTo,
// clone, the CV_32F product as cv::gemm: double accumulation in k order, one rounding); cv::KeyPoint and
// cv::DMatch are byte-identical to rgbd_keypoint / rgbd_dmatch; Eigen::Matrix4f is row-indexed
// (operator()(r, c)) with isIdentity() at float precision (1e-5).
#pragma once
#include <cmath>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <stdexcept>
#include <thread>
#include <vector>

#include "rgbd_hip.h"

constexpr int CV_8U = 0;
constexpr int CV_16U = 2;
constexpr int CV_32F = 5;
constexpr int CV_64F = 6;
constexpr int CV_8UC3 = 16;
constexpr int CV_BGR2GRAY = 6;   // cv::COLOR_BGR2GRAY
#define FRAME_GRID_ROWS 48       // Core/Frame.h:15-16
#define FRAME_GRID_COLS 64

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
struct Vec3b {
    uint8_t val[3] = {0, 0, 0};
    uint8_t& operator[](int i) { return val[i]; }
    uint8_t operator[](int i) const { return val[i]; }
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
    template <typename T>
    const T& at(int i) const { return rows == 1 ? at<T>(0, i) : at<T>(i, 0); }
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
    // reshape(cn): the mirror keeps N x 2 float points as they are (channels are not tracked)
    Mat reshape(int cn) const
    {
        (void)cn;
        return *this;
    }
    size_t total() const { return (size_t)rows * cols; }
    // convertTo(CV_32F, alpha) of a CV_16U image: float(v) * float(alpha) + 0.0f per pixel (cvtScale_ with a
    // float work type, OpenCV 3.4); the destination is (re)allocated
    void convertTo(Mat& d, int rtype, double alpha = 1.0) const
    {
        if (type_ != CV_16U || rtype != CV_32F) throw std::runtime_error("mirror convertTo: 16U -> 32F only");
        d.create(rows, cols, CV_32F);
        const float a = (float)alpha;
        for (int r = 0; r < rows; r++)
            for (int c = 0; c < cols; c++) d.at<float>(r, c) = (float)at<uint16_t>(r, c) * a + 0.0f;
    }
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

// cvtColor(BGR2GRAY) on CV_8UC3: OpenCV's fixed point, (1868 B + 9617 G + 4899 R + 2^13) >> 14
inline void cvtColor(InputArray src, OutputArray dst, int code)
{
    const Mat s = src.getMat();
    if (code != CV_BGR2GRAY || s.type() != CV_8UC3) throw std::runtime_error("mirror cvtColor: BGR2GRAY only");
    dst.create(s.rows, s.cols, CV_8U);
    Mat d = dst.getMat();
    for (int y = 0; y < s.rows; y++)
        for (int x = 0; x < s.cols; x++) {
            const uint8_t* p = s.data + (size_t)y * s.step + (size_t)x * 3;
            d.at<uint8_t>(y, x) = (uint8_t)((1868 * p[0] + 9617 * p[1] + 4899 * p[2] + 8192) >> 14);
        }
}

// undistortPoints(src, dst, K, D, noArray(), P = K) on N x 2 CV_32F points: cvUndistortPoints' 5 iterations in
// double (the same sequence the device's k_undistort runs)
inline void undistortPoints(InputArray src, OutputArray dst, InputArray K, InputArray D, InputArray R, InputArray P)
{
    (void)R;
    (void)P;
    const Mat s = src.getMat(), k = K.getMat(), dc = D.getMat();
    const double fx = k.at<float>(0, 0), fy = k.at<float>(1, 1), cx = k.at<float>(0, 2), cy = k.at<float>(1, 2);
    double kk[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < (int)dc.total() && i < 5; i++) kk[i] = dc.at<float>(i);
    std::vector<float> out(2 * (size_t)s.rows);
    for (int i = 0; i < s.rows; i++) {
        const double ifx = 1. / fx, ify = 1. / fy;
        double x = ((double)s.at<float>(i, 0) - cx) * ifx, y = ((double)s.at<float>(i, 1) - cy) * ify;
        const double x0 = x, y0 = y;
        for (int j = 0; j < 5; j++) {
            const double r2 = x * x + y * y;
            const double icdist = 1 / (1 + ((kk[4] * r2 + kk[1]) * r2 + kk[0]) * r2);
            const double deltaX = 2 * kk[2] * x * y + kk[3] * (r2 + 2 * x * x);
            const double deltaY = kk[2] * (r2 + 2 * y * y) + 2 * kk[3] * x * y;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        out[2 * i] = (float)(fx * x + cx);
        out[2 * i + 1] = (float)(fy * y + cy);
    }
    dst.create(s.rows, 2, CV_32F);
    Mat d = dst.getMat();
    for (int i = 0; i < s.rows; i++) {
        d.at<float>(i, 0) = out[2 * i];
        d.at<float>(i, 1) = out[2 * i + 1];
    }
}

// cv::norm (NORM_L2) of a CV_32F vector: double sum of squares in element order, then sqrt
inline double norm(const Mat& m)
{
    double s = 0.0;
    for (int r = 0; r < m.rows; r++)
        for (int c = 0; c < m.cols; c++) {
            const double v = m.at<float>(r, c);
            s += v * v;
        }
    return std::sqrt(s);
}

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

// RGBDcamera (Core/RGBDcamera.h, Core/IntrinsicMatrix.cpp): intrinsics, distortion (k1 k2 p1 p2 [k3]) and
// mDepthMapFactor = 1 / depthMapFactor (Core/RGBDcamera.cpp:20)
class RGBDcamera {
public:
    RGBDcamera(float fx, float fy, float cx, float cy, float k1, float k2, float p1, float p2, float k3,
               float depthMapFactor)
        : mFx(fx), mFy(fy), mCx(cx), mCy(cy), mInvfx(1.0f / fx), mInvfy(1.0f / fy), mK1(k1), mK2(k2), mP1(p1),
          mP2(p2), mK3(k3), mDepthMapFactor(1.0f / depthMapFactor)
    {
    }
    cv::Mat k()
    {
        cv::Mat K = cv::Mat::eye(3, 3, CV_32F);
        K.at<float>(0, 0) = mFx;
        K.at<float>(1, 1) = mFy;
        K.at<float>(0, 2) = mCx;
        K.at<float>(1, 2) = mCy;
        return K;
    }
    cv::Mat distCoef()   // IntrinsicMatrix::setDistortion: 4 x 1, 5 x 1 when k3 != 0
    {
        cv::Mat D(mK3 != 0.0f ? 5 : 4, 1, CV_32F);
        D.at<float>(0) = mK1;
        D.at<float>(1) = mK2;
        D.at<float>(2) = mP1;
        D.at<float>(3) = mP2;
        if (mK3 != 0.0f) D.at<float>(4) = mK3;
        return D;
    }
    float fx() { return mFx; }
    float fy() { return mFy; }
    float cx() { return mCx; }
    float cy() { return mCy; }
    float invfx() { return mInvfx; }
    float invfy() { return mInvfy; }

private:
    float mFx, mFy, mCx, mCy, mInvfx, mInvfy, mK1, mK2, mP1, mP2, mK3;

public:
    float mDepthMapFactor;
};

// Extractor (Features/Extractor.h:9-60).  Integration member: context() -- the device context this Extractor
// owns for the calling thread, created on the thread's first use for the geometry and camera of the first
// frame the Extractor saw (librgbd_hip's contexts, like ORBextractor, are not reentrant).
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
    rgbd_ctx* context(int width, int height, RGBDcamera& cam);
    rgbd_ctx* context();
    size_t contexts();   // how many threads hold a context (test hook)

    int nfeatures = 1000, nlevels = 8, iniThFAST = 20, minThFAST = 7;
    float scaleFactor = 1.2f;

private:
    rgbd_ctx* threadContext();   // under mMutexCtx
    std::mutex mMutexCtx;
    std::map<std::thread::id, rgbd_ctx*> mCtx;
    int mWidth = 0, mHeight = 0;
    rgbd_camera mCamera{};
};

class Frame;

// Landmark (Core/Landmark.h): what Tracking::initialize sets
class Landmark {
public:
    using Ptr = std::shared_ptr<Landmark>;
    Landmark(const cv::Mat& Pos, std::shared_ptr<Frame> frame, const size_t& idxF)
        : mWorldPos(Pos.clone()), mpRefKF(frame), mnFirstIdx(idxF)
    {
    }
    void addObservation(std::shared_ptr<Frame> pKF, size_t obsId)
    {
        std::lock_guard<std::mutex> lock(mMutexFeatures);
        mObservations[pKF.get()] = obsId;
    }
    void setColor(const cv::Vec3b& color) { mColor = color; }
    cv::Vec3b getColor() const { return mColor; }
    cv::Mat getWorldPos() const { return mWorldPos.clone(); }

private:
    cv::Mat mWorldPos;
    std::weak_ptr<Frame> mpRefKF;
    size_t mnFirstIdx;
    cv::Vec3b mColor;
    std::mutex mMutexFeatures;
    std::map<const Frame*, size_t> mObservations;
};

class Frame {
public:
    using Ptr = std::shared_ptr<Frame>;
    struct PointT {           // pcl::PointXYZRGB: xyz + the packed bgr bytes
        float x = 0, y = 0, z = 0;
        uint8_t b = 0, g = 0, r = 0, a = 0;
    };
    struct PointCloudT {      // pcl::PointCloud<PointT>
        std::vector<PointT> points;
        uint32_t width = 0, height = 0;
        bool is_dense = true;
    };
    Frame(const cv::Mat& imRGB, const cv::Mat& imDepth, const double& timeStamp, std::shared_ptr<Extractor> pExtractor,
          RGBDcamera* pRGBDcamera);   // solver_bodies.cpp

    // Core/Frame.cpp:124-153: setPose clones Tcw and updates the pose members under mMutexPose
    void setPose(cv::Mat Tcw)
    {
        std::lock_guard<std::mutex> lock(mMutexPose);
        mTcw = Tcw.clone();
        updatePoseMatrices();
    }
    cv::Mat getPose() const
    {
        std::lock_guard<std::mutex> lock(mMutexPose);
        return mTcw.clone();
    }
    cv::Mat getPoseInverse()
    {
        std::lock_guard<std::mutex> lock(mMutexPose);
        return mTwc.clone();
    }
    cv::Mat getCameraCenter()
    {
        std::lock_guard<std::mutex> lock(mMutexPose);
        cv::Mat O(3, 1, CV_32F);
        for (int r = 0; r < 3; r++) O.at<float>(r, 0) = mOw[r];
        return O;
    }
    // mRcw = Tcw(0:3, 0:3), mRwc = mRcw^T, mtcw = Tcw(0:3, 3), mOw = -mRcw^T mtcw (one gemm: double sums,
    // alpha -1, one rounding), mTwc = [mRwc | mOw]
    void updatePoseMatrices()
    {
        mTwc = cv::Mat::eye(4, 4, CV_32F);
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) mRwc[3 * r + c] = mTcw.at<float>(c, r);
            double o = 0.0;
            for (int k = 0; k < 3; k++) o += (double)mTcw.at<float>(k, r) * (double)mTcw.at<float>(k, 3);
            mOw[r] = (float)(o * -1.0);
            for (int c = 0; c < 3; c++) mTwc.at<float>(r, c) = mRwc[3 * r + c];
            mTwc.at<float>(r, 3) = mOw[r];
        }
    }
    // Core/Frame.cpp:317-327: mRwc * x3Dc + mOw (one gemm with mOw as its C term), empty when z <= 0
    cv::Mat unprojectWorld(const size_t& i)
    {
        if (!(mvKeys3Dc[i].z > 0)) return cv::Mat();
        const float x[3] = {mvKeys3Dc[i].x, mvKeys3Dc[i].y, mvKeys3Dc[i].z};
        std::lock_guard<std::mutex> lock(mMutexPose);
        cv::Mat X(3, 1, CV_32F);
        for (int r = 0; r < 3; r++) {
            double a = 0.0;
            for (int k = 0; k < 3; k++) a += (double)mRwc[3 * r + k] * (double)x[k];
            X.at<float>(r, 0) = (float)(a * 1.0 + (double)mOw[r] * 1.0);
        }
        return X;
    }
    // Core/Frame.cpp:231-241
    bool posInGrid(const cv::KeyPoint& kp, int& posX, int& posY)
    {
        posX = (int)std::round((kp.pt.x - mnMinX) * mfGridElementWidthInv);
        posY = (int)std::round((kp.pt.y - mnMinY) * mfGridElementHeightInv);
        return !(posX < 0 || posX >= FRAME_GRID_COLS || posY < 0 || posY >= FRAME_GRID_ROWS);
    }
    bool isInlier(const size_t& idx) const { return mvbOutlier[idx] == false; }
    bool isOutlier(const size_t& idx) const { return mvbOutlier[idx] == true; }
    void setInlier(const size_t& idx) { mvbOutlier[idx] = false; }
    void setOutlier(const size_t& idx) { mvbOutlier[idx] = true; }
    bool isValidObs(const size_t& idx) { return mvKeys3Dc[idx].z > 0; }
    void addLandmark(Landmark::Ptr pLM, const size_t& i)
    {
        std::lock_guard<std::mutex> lock(mMutexFeatures);
        mvpLandmarks[i] = pLM;
    }
    Landmark::Ptr getLandmark(const size_t& i)
    {
        std::lock_guard<std::mutex> lock(mMutexFeatures);
        return mvpLandmarks[i];
    }
    int id()
    {
        std::lock_guard<std::mutex> lock(mMutexId);
        return mnId;
    }
    // Integration member: createCloud(res) + passThroughFilter("z", zmin, zmax) + downsampleCloud(leaf) +
    // statisticalFilterCloud(k, stddev) in one device call (solver_bodies.cpp)
    void createFilteredCloud(int res, float zmin, float zmax, float leaf, int k, double stddev);
    bool isValidCloud()
    {
        std::lock_guard<std::mutex> lock(mMutexCloud);
        return mpCloud != nullptr;
    }
    std::shared_ptr<PointCloudT> cloud()   // test hook (the reference keeps mpCloud private)
    {
        std::lock_guard<std::mutex> lock(mMutexCloud);
        return mpCloud;
    }
    void setKF()
    {
        std::lock_guard<std::mutex> lock(mMutexId);
        mbIsKF = true;
    }
    bool isKF()
    {
        std::lock_guard<std::mutex> lock(mMutexId);
        return mbIsKF;
    }

    cv::Mat mImColor, mImGray, mImDepth;
    std::shared_ptr<Extractor> mpExtractor;
    RGBDcamera* mpCamera;
    double mTimeStamp;
    size_t N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
    std::vector<cv::Point3f> mvKeys3Dc;
    std::vector<cv::Vec3b> mvKeysColor;
    cv::Mat mDescriptors;
    std::vector<bool> mvbOutlier;
    static float mfGridElementWidthInv, mfGridElementHeightInv;
    std::vector<std::size_t> mGrid[FRAME_GRID_COLS][FRAME_GRID_ROWS];
    static float mnMinX, mnMaxX, mnMinY, mnMaxY;
    static bool mbInitialComputations;
    Frame::Ptr mpReferenceKF;

private:
    void computeImageBounds();     // Core/Frame.cpp:283-315 (ref_system.cpp)
    void assignFeaturesToGrid();   // Core/Frame.cpp:75-89 (ref_system.cpp)
    std::vector<Landmark::Ptr> mvpLandmarks;
    static int nNextId;
    int mnId = 0;
    bool mbIsKF = false;
    cv::Mat mTcw, mTwc;
    float mRwc[9] = {}, mOw[3] = {};
    std::mutex mMutexId, mMutexFeatures, mMutexCloud;
    mutable std::mutex mMutexPose;
    std::shared_ptr<PointCloudT> mpCloud;
};

// Map (Core/Map.h): the landmarks and keyframes Tracking and PoseGraph add
class Map {
public:
    using Ptr = std::shared_ptr<Map>;
    void addLandmark(Landmark::Ptr pLM)
    {
        std::lock_guard<std::mutex> lock(mMutexMap);
        mspLandmarks.push_back(pLM);
    }
    void addKeyFrame(Frame::Ptr pKF)
    {
        std::lock_guard<std::mutex> lock(mMutexMap);
        mvpKeyFrames.push_back(pKF);
    }
    std::vector<Frame::Ptr> getAllKeyFrames()
    {
        std::lock_guard<std::mutex> lock(mMutexMap);
        return mvpKeyFrames;
    }
    std::vector<Landmark::Ptr> getAllLandmarks()
    {
        std::lock_guard<std::mutex> lock(mMutexMap);
        return mspLandmarks;
    }

private:
    std::mutex mMutexMap;
    std::vector<Landmark::Ptr> mspLandmarks;
    std::vector<Frame::Ptr> mvpKeyFrames;
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
// initSeed() seeds the device stream with the same seed (initSeed(seed): a fixed seed, for tests), and
// mutex() serialises the threads that draw from it (glibc's rand() takes a lock per draw; a device call
// draws a whole RansacSE3's samples, so it holds the lock for the call).
class Random {
public:
    static void initSeed();
    static void initSeed(unsigned seed);
    static rgbd_rng& stream();            // RansacSE3's rand() stream
    static rgbd_sticky& depthCovariance();  // RansacSE3::depthCovariance's statics
    static std::mutex& mutex();

protected:
    static bool SET_RAND;
};

class PoseGraph;

// Tracking (System/Tracking.h): the state track() keeps (the viewer, the loop detector and the BoW vocabulary
// are absent).  track() and its helpers are restated in ref_system.cpp; createKeyFrame is INTEGRATION.md's body.
class Tracking {
public:
    enum TrackerState { NOT_INITIALIZED = 0, OK, LOST };
    Tracking(std::shared_ptr<Map> pMap, bool withPoseGraph);
    ~Tracking();
    cv::Mat track(std::shared_ptr<Frame> newFrame);
    void shutdown();
    int getMeanInliers();
    int getCurrentInliers();

    std::list<cv::Mat> mRelativeFramePoses;
    std::list<std::shared_ptr<Frame>> mReferences;
    std::list<double> mFrameTimes;

protected:
    void initialize();
    void visualOdometry();
    void recover();
    bool needKeyFrame();
    void createKeyFrame();   // solver_bodies.cpp
    void updateLastFrame();
    void updateRelativePose();

    std::shared_ptr<Frame> mpCurFrame;
    std::pair<std::shared_ptr<Frame>, std::shared_ptr<Frame>> mpRefFrame;
    TrackerState mState;
    std::shared_ptr<Map> mpMap;
    std::shared_ptr<PoseGraph> mpPoseGraph;
    std::shared_ptr<Frame> mpLastKeyFrame;
    int mnAcumInliers, mnInliers, mnMeanInliers;
    std::mutex mMutexStatistics;
    cv::Mat mVelocity;
    std::mutex mMutexTrack;
};

// PoseGraph (Solver/PoseGraph.h): the keyframe queue and the thread that runs updateGraph() on it (createNode,
// createEdgeWithReference, createLocalEdges; Solver/PoseGraph.cpp:59-155), with g2o replaced by rgbd_posegraph
// (INTEGRATION.md section 9).  Restated in ref_system.cpp; loop detection is absent (no vocabulary).
class PoseGraph {
public:
    PoseGraph(Tracking* pTracker, std::shared_ptr<Map> pMap);
    ~PoseGraph();
    void insertKeyFrame(Frame::Ptr pKF);
    void shutdown();   // processes what is queued, then joins the thread

private:
    void run();
    bool checkNewKeyFrames();
    void updateGraph();
    void createLocalEdges();
    void nearestNodes(Frame::Ptr pKF, std::vector<Frame::Ptr>& candidates);

    Tracking* mpTracker;
    std::shared_ptr<Map> mpMap;
    rgbd_posegraph* mGraph = nullptr;
    Frame::Ptr mpCurrentKF, mpReferenceKF;
    std::list<Frame::Ptr> mlpKeyFrameQueue;
    std::mutex mMutexQueue, mMutexFinish;
    bool mbFinishRequested = false;
    std::thread mRunThread;
};

// Test hooks of ref_system.cpp (not reference surfaces): every RansacSE3::compute the Tracking and PoseGraph
// restatements run goes through sac_compute, which records the calls in the order they took the process's
// rand() stream, so a test can replay both threads' draws from one stream.
namespace refside {
struct SacRecord {
    int seq;            // order in which the call held the stream
    char thread;        // 'T' tracking, 'P' pose graph
    int id1, id2;       // F1->id(), F2->id()
    int n_matches, ok, n_inliers;
    uint32_t rmse_bits, T_bits[16];
};
bool sac_compute(char thread, RansacSE3& sac, std::shared_ptr<Frame> F1, std::shared_ptr<Frame> F2,
                 const std::vector<cv::DMatch>& m12, bool updateF2);
std::vector<SacRecord> sac_log();
struct PairRecord {      // a PoseGraph candidate: the Matcher's count (RansacSE3 runs when >= 30)
    int id_cur, id_kf, n_matches;
};
std::vector<PairRecord> pair_log();
void log_pair(int id_cur, int id_kf, int n_matches);
}  // namespace refside

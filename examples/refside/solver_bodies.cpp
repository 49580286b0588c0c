// solver_bodies.cpp -- the reference-side bodies of INTEGRATION.md, compiled against the reference's own class
// surfaces (mirrored in ref_mirror.hpp) and librgbd_hip.so.  Each block between "// [body NAME]" and
// "// [end]" is quoted verbatim in INTEGRATION.md (tests/test_integration_doc.py keeps the two equal), so
// what a maintainer pastes into the reference is what tests/test_gpu_refside.py runs.
#include <ctime>
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include "ref_mirror.hpp"

static void check(rgbd_ctx* ctx, rgbd_status s, const char* what)
{
    if (s != RGBD_OK) throw std::runtime_error(std::string(what) + ": " + (ctx ? rgbd_last_error(ctx) : "no context"));
}

// [body Random]
// System/Random.cpp: the device RansacSE3 draws from the same seed as the process's rand()
bool Random::SET_RAND = false;
static rgbd_rng g_rand_stream;
static rgbd_sticky g_depth_cov = {0.0, 0, 0};

void Random::initSeed()
{
    if (!SET_RAND) initSeed((unsigned int)time(NULL));
}

void Random::initSeed(unsigned seed)
{
    srand(seed);
    rgbd_rng_seed(&g_rand_stream, seed);
    SET_RAND = true;
}

rgbd_rng& Random::stream() { return g_rand_stream; }
rgbd_sticky& Random::depthCovariance() { return g_depth_cov; }
std::mutex& Random::mutex()
{
    static std::mutex m;   // held by a RansacSE3 call for its draws (glibc's rand() locks per draw)
    return m;
}
// [end]

// [body Extractor]
// Features/Extractor.cpp:15-22, 50-61: the (ORB2, ORB2) and (SVO, BRIEF) pairs run on the device.  A device
// context is not reentrant (like ORBextractor, Features/ORBextractor.h:39), so each thread that uses this
// Extractor -- the tracking thread building Frames, the PoseGraph thread matching keyframes
// (Solver/PoseGraph.cpp:141-149) -- gets a context of its own, created for the first frame's geometry
Extractor::Extractor(eType detector, eType descriptor, eMode mode)
    : mDetectorType(detector), mDescriptorType(descriptor), mMode(mode)
{
    const bool orb2 = detector == ORB2 && descriptor == ORB2, svo = detector == SVO && descriptor == BRIEF;
    if (mode != NORMAL || !(orb2 || svo)) throw std::runtime_error("Extractor: not a device pair");
    setParameters(1000, 1.2f, 8, 20, 7);
}

Extractor::~Extractor()
{
    for (auto& kv : mCtx) rgbd_destroy(kv.second);
}

void Extractor::setParameters(int _nfeatures, float _scaleFactor, int _nlevels, int _iniThFAST, int _minThFAST)
{
    nfeatures = _nfeatures;
    scaleFactor = _scaleFactor;
    nlevels = _nlevels;
    iniThFAST = _iniThFAST;
    minThFAST = _minThFAST;
}

rgbd_ctx* Extractor::context(int width, int height, RGBDcamera& cam)
{
    std::lock_guard<std::mutex> lock(mMutexCtx);
    if (mWidth == 0) {
        const cv::Mat D = cam.distCoef();
        mCamera = rgbd_camera{cam.fx(), cam.fy(), cam.cx(), cam.cy(), D.at<float>(0), D.at<float>(1), D.at<float>(2),
                              D.at<float>(3), D.rows > 4 ? D.at<float>(4) : 0.0f, cam.mDepthMapFactor};
        mWidth = width;
        mHeight = height;
    } else if (width != mWidth || height != mHeight) {
        throw std::runtime_error("Extractor: one image size per Extractor");
    }
    return threadContext();
}

rgbd_ctx* Extractor::context()
{
    std::lock_guard<std::mutex> lock(mMutexCtx);
    if (mWidth == 0) throw std::runtime_error("Extractor: no frame has been built yet");
    return threadContext();
}

rgbd_ctx* Extractor::threadContext()
{
    rgbd_ctx*& ctx = mCtx[std::this_thread::get_id()];
    if (ctx) return ctx;
    rgbd_status s;
    if (mDetectorType == ORB2) {
        const rgbd_orb_params orb{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST};
        s = rgbd_create(0, mWidth, mHeight, 1, &orb, &mCamera, &ctx);
    } else {   // SVOextractor(nlevels, 5, 20) + retainBest(nfeatures) + BRIEF-32 (:162-165, :224-226)
        const rgbd_svo_params svo{nfeatures, nlevels, 5, 20, 0};
        s = rgbd_create_svo(0, mWidth, mHeight, 1, &svo, &mCamera, &ctx);
    }
    if (s != RGBD_OK) {
        const std::string msg = std::string("rgbd_create: ") + (ctx ? rgbd_last_error(ctx) : "no context");
        if (ctx) rgbd_destroy(ctx);
        mCtx.erase(std::this_thread::get_id());
        throw std::runtime_error(msg);
    }
    return ctx;
}

size_t Extractor::contexts()
{
    std::lock_guard<std::mutex> lock(mMutexCtx);
    return mCtx.size();
}

void Extractor::detectAndCompute(cv::InputArray image, cv::InputArray mask, std::vector<cv::KeyPoint>& keypoints,
                                 cv::OutputArray descriptors)
{
    (void)mask;                                     // ignored by both branches, as in the reference
    if (image.empty()) return;                      // ORBextractor.cpp:708-709
    cv::Mat g = image.getMat();                     // CV_8UC1 (:712)
    rgbd_ctx* ctx = context();                      // this thread's; context(W, H, camera) ran for the geometry
    const int cap = rgbd_max_keypoints(ctx);
    keypoints.resize(cap);
    cv::Mat desc(cap, 32, CV_8U);
    int n = 0;
    check(ctx, rgbd_detect_and_compute(ctx, g.data, (int)g.step, reinterpret_cast<rgbd_keypoint*>(keypoints.data()),
                                       desc.data, cap, &n), "rgbd_detect_and_compute");
    keypoints.resize(n);
    if (n == 0) {                                   // ORBextractor.cpp:726-730
        descriptors.release();
    } else {
        descriptors.create(n, 32, CV_8U);
        cv::Mat d = descriptors.getMat();
        desc.rowRange(0, n).copyTo(d);              // the n rows written above
    }
}
// [end]

// [body Frame]
// Core/Frame.cpp:34-117: the ctor sets every member it sets in the reference, in the same order (id, the three
// images, keypoints, descriptors, landmarks, flags, image bounds and grid, 3D points, colours);
// extractFeatures + undistortKeyPoints + uprojectCamera's 3D points are one device pass over imRGB / imDepth
// (CV_8UC3 BGR and CV_16U, both continuous).  mImGray and mImDepth stay host images for their readers
// (drawTackedPoints, createCloud)
Frame::Frame(const cv::Mat& imRGB, const cv::Mat& imDepth, const double& timeStamp, Extractor::Ptr pExtractor,
             RGBDcamera* pRGBDcamera)
    : mImColor(imRGB), mpExtractor(pExtractor), mpCamera(pRGBDcamera), mTimeStamp(timeStamp), mbIsKF(false)
{
    mnId = nNextId++;

    cv::cvtColor(imRGB, mImGray, CV_BGR2GRAY);
    imDepth.convertTo(mImDepth, CV_32F, static_cast<double>(mpCamera->mDepthMapFactor));

    rgbd_ctx* ctx = mpExtractor->context(imRGB.cols, imRGB.rows, *mpCamera);
    const int cap = rgbd_max_keypoints(ctx);
    mvKeys.resize(cap);
    mvKeysUn.resize(cap);
    mvKeys3Dc.resize(cap);                          // cv::Point3f == float[3]
    cv::Mat desc(cap, 32, CV_8U);
    int n = 0;
    check(ctx, rgbd_frame(ctx, imRGB.data, reinterpret_cast<const uint16_t*>(imDepth.data),
                          reinterpret_cast<rgbd_keypoint*>(mvKeys.data()), reinterpret_cast<rgbd_keypoint*>(mvKeysUn.data()),
                          desc.data, reinterpret_cast<float*>(mvKeys3Dc.data()), cap, &n), "rgbd_frame");
    N = (size_t)n;
    mvKeys.resize(N);
    mvKeysUn.resize(N);
    mvKeys3Dc.resize(N);
    if (mvKeys.empty()) return;                     // :54-55 (descriptors released, :726-730)
    desc.rowRange(0, n).copyTo(mDescriptors);

    mvpLandmarks = std::vector<Landmark::Ptr>(N, nullptr);
    mvbOutlier = std::vector<bool>(N, false);

    if (mbInitialComputations) {                    // :62-69
        computeImageBounds();
        mfGridElementWidthInv = static_cast<float>(FRAME_GRID_COLS) / static_cast<float>(mnMaxX - mnMinX);
        mfGridElementHeightInv = static_cast<float>(FRAME_GRID_ROWS) / static_cast<float>(mnMaxY - mnMinY);
        mbInitialComputations = false;
    }
    assignFeaturesToGrid();

    mvKeysColor.resize(N);                          // uprojectCamera's colour: the truncated distorted pixel (:105)
    for (size_t i = 0; i < N; i++)
        mvKeysColor[i] = mImColor.at<cv::Vec3b>((int)mvKeys[i].pt.y, (int)mvKeys[i].pt.x);
}
// [end]

// [body Matcher::match]
// Features/Matcher.cpp:106-139: knn-2 (Hamming), ratio test, first query per train index, the reference's
// outlier flag (discardOutliers) and both depths valid -- in one device call
int Matcher::match(Frame::Ptr ref, Frame::Ptr cur, std::vector<cv::DMatch>& vMatches12, const bool discardOutliers)
{
    vMatches12.clear();
    rgbd_ctx* ctx = ref->mpExtractor->context();
    std::vector<uint8_t> outl(ref->N);
    std::vector<float> zq(ref->N), zt(cur->N);
    for (size_t i = 0; i < ref->N; i++) {
        outl[i] = ref->isOutlier(i);
        zq[i] = ref->mvKeys3Dc[i].z;                // isValidObs: z > 0
    }
    for (size_t i = 0; i < cur->N; i++) zt[i] = cur->mvKeys3Dc[i].z;
    vMatches12.resize(ref->N);
    int m = 0;
    check(ctx, rgbd_match(ctx, ref->mDescriptors.data, (int)ref->N, cur->mDescriptors.data, (int)cur->N, outl.data(),
                          zq.data(), zt.data(), mfNNratio, discardOutliers, reinterpret_cast<rgbd_dmatch*>(vMatches12.data()),
                          (int)vMatches12.size(), &m), "rgbd_match");
    vMatches12.resize(m);
    return m;
}
// [end]

// [body RansacSE3]
// Solver/SolverSE3.cpp:10-133: the whole loop (sort, samples from the process's rand() stream, refinement
// chains, accept / break replay, identity fallback) on the device; flags and pose written as :40-41, :119-125.
// The tracking and PoseGraph threads share the stream and the depth covariance, so a call holds Random's lock
RansacSE3::RansacSE3() : RansacSE3(200, 20, 3.0f, 4) {}

RansacSE3::RansacSE3(int iters, unsigned minInlierTh, float maxMahalanobisDist, unsigned sampleSize)
    : mIterations(iters), mMinInlierTh(minInlierTh), mMaxMahalanobisDistance(maxMahalanobisDist), mSampleSize(sampleSize)
{
}

bool RansacSE3::compute(Frame::Ptr pF1, Frame::Ptr pF2, const std::vector<cv::DMatch>& m12, const bool& updateF2)
{
    rgbd_ctx* ctx = pF1->mpExtractor->context();   // the calling thread's context
    std::lock_guard<std::mutex> draws(Random::mutex());
    Random::initSeed();
    std::vector<uint8_t> flags(pF2->N);
    for (size_t i = 0; i < pF2->N; i++) flags[i] = pF2->isOutlier(i);
    const rgbd_ransac_params prm{mIterations, mMinInlierTh, mMaxMahalanobisDistance, mSampleSize};
    float T[16];
    int nIn = 0, ok = 0;
    mvInliers.resize(m12.size());
    check(ctx, rgbd_ransac_se3(ctx, reinterpret_cast<const float*>(pF1->mvKeys3Dc.data()), (int)pF1->N,
                               reinterpret_cast<const float*>(pF2->mvKeys3Dc.data()), (int)pF2->N,
                               reinterpret_cast<const rgbd_dmatch*>(m12.data()), (int)m12.size(), &prm, &Random::stream(),
                               &Random::depthCovariance(), updateF2, flags.data(), T,
                               reinterpret_cast<rgbd_dmatch*>(mvInliers.data()), &nIn, &rmse, &ok), "rgbd_ransac_se3");
    mvInliers.resize(nIn);
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) mT21(r, c) = T[4 * r + c];
    if (updateF2) {
        for (size_t i = 0; i < pF2->N; i++) flags[i] ? pF2->setOutlier(i) : pF2->setInlier(i);
        if (ok) {
            cv::Mat T21 = Converter::toMat<float, 4, 4>(mT21);
            T21 = T21 * pF1->getPose();
            pF2->setPose(T21);
        }
    }
    return ok != 0;
}
// [end]

// [body Gicp]
// Solver/Gicp.cpp: the ctor's parameters, the setters Tracking calls (System/Tracking.cpp:148-149), compute's
// rules (< 20 pairs, identity -> false, mbUpdate) on the host as the reference has them; align() on the device
Gicp::Gicp(const Frame::Ptr F1, Frame::Ptr F2, const std::vector<cv::DMatch>& matches, Eigen::Matrix4f& guess)
    : Solver(F1, F2, matches), mbUpdate(true), mGuess(guess)
{
    // setMaximumIterations(15), setMaxCorrespondenceDistance(0.08), setEuclideanFitnessEpsilon(1),
    // setTransformationEpsilon(1e-9) (:12-15) over PCL's defaults (k 20, rotation epsilon 2e-3, GICP epsilon 1e-3)
    mGicp = rgbd_gicp_params{15, 20, 0.08, 1e-9, 2e-3, 1e-3, 4, 1};
}

bool Gicp::compute(std::vector<cv::DMatch>& inliers)
{
    (void)inliers;   // not written by the reference either
    if (mMatches.size() < 20) return false;
    createCloudsFromMatches();
    mT = align();
    if (!mT.isIdentity()) {
        if (mbUpdate) mF2->setPose(Converter::toMat<float, 4, 4>(mT) * mF1->getPose());
        return true;
    } else
        return false;
}

void Gicp::createCloudsFromMatches()
{
    mpSrcCloud.clear();
    mpTgtCloud.clear();
    for (const auto& m : mMatches) {
        const cv::Point3f& source = mF1->mvKeys3Dc[m.queryIdx];
        const cv::Point3f& target = mF2->mvKeys3Dc[m.trainIdx];
        mpSrcCloud.insert(mpSrcCloud.end(), {source.x, source.y, source.z});
        mpTgtCloud.insert(mpTgtCloud.end(), {target.x, target.y, target.z});
    }
}

Eigen::Matrix4f Gicp::align()
{
    rgbd_ctx* ctx = mF1->mpExtractor->context();
    float guess[16], T[16];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) guess[4 * r + c] = mGuess(r, c);
    int converged = 0, iterations = 0;
    check(ctx, rgbd_gicp(ctx, mpSrcCloud.data(), mpTgtCloud.data(), (int)(mpSrcCloud.size() / 3), guess, &mGicp, T,
                         &converged, &iterations), "rgbd_gicp");
    if (!converged) return Eigen::Matrix4f::Identity();
    Eigen::Matrix4f out;
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) out(r, c) = T[4 * r + c];
    return out;
}

void Gicp::setMaximumIterations(int iters) { mGicp.max_iterations = iters; }
void Gicp::setMaxCorrespondenceDistance(double dist) { mGicp.max_corr_dist = dist; }
void Gicp::setEuclideanFitnessEpsilon(double epsilon) { (void)epsilon; }   // not a criterion of the definition (GICP)
void Gicp::setTransformationEpsilon(double epsilon) { mGicp.transformation_epsilon = epsilon; }
// [end]

// [body PnPRansac::compute]
// Solver/PnPRansac.cpp:14-56 as written: object points = F2's own unprojectWorld, pixels = F2's mvKeysUn,
// every matched train an outlier (:31), cv::solvePnPRansac(..., 500, 3.0f, 0.85) on the device (:39), then
// Tcw = Converter::toHomogeneous(r, t) = [float(R) | float(t)] and the inliers' flags (:51)
bool PnPRansac::compute(std::vector<cv::DMatch>& inliers)
{
    if (mMatches.size() < 10) return false;
    std::vector<cv::Point2f> v2D;
    v2D.reserve(mMatches.size());
    std::vector<cv::Point3f> v3D;
    v3D.reserve(mMatches.size());
    for (size_t i = 0; i < mMatches.size(); i++) {
        const cv::DMatch& m = mMatches[i];
        v2D.push_back(mF2->mvKeysUn[m.trainIdx].pt);
        cv::Mat pw = mF2->unprojectWorld(m.trainIdx);
        v3D.push_back(cv::Point3f{pw.at<float>(0), pw.at<float>(1), pw.at<float>(2)});
        mF2->setOutlier(m.trainIdx);
    }
    if (v2D.size() < 10) return false;
    rgbd_ctx* ctx = mF2->mpExtractor->context();
    const cv::Mat K = mF2->mpCamera->k();
    const float K4[4] = {K.at<float>(0, 0), K.at<float>(1, 1), K.at<float>(0, 2), K.at<float>(1, 2)};
    const rgbd_pnp_params prm{500, 3.0f, 0.85, 10, 0};
    const int M = (int)v2D.size();
    double R[9], t[3];
    std::vector<uint8_t> mask(M);
    int nIn = 0, iters = 0, status = 0;
    check(ctx, rgbd_pnp_ransac(ctx, reinterpret_cast<const float*>(v3D.data()), reinterpret_cast<const float*>(v2D.data()),
                               M, K4, &prm, R, t, mask.data(), &nIn, &iters, &status), "rgbd_pnp_ransac");
    if (status) {
        cv::Mat Rm(3, 3, CV_64F), tm(3, 1, CV_64F);
        for (int r = 0; r < 3; r++) {
            for (int c = 0; c < 3; c++) Rm.at<double>(r, c) = R[3 * r + c];
            tm.at<double>(r, 0) = t[r];
        }
        cv::Mat Tcw = cv::Mat::eye(4, 4, CV_32F);
        cv::Mat TR = Tcw.rowRange(0, 3).colRange(0, 3), Tt = Tcw.rowRange(0, 3).col(3);
        Rm.copyTo(TR);                              // CV_64F into the fixed CV_32F view: converted
        tm.copyTo(Tt);
        mF2->setPose(Tcw);
        inliers.clear();
        inliers.reserve(nIn);
        for (int i = 0; i < M; ++i) {
            if (!mask[i]) continue;
            const cv::DMatch& m = mMatches[i];
            inliers.push_back(m);
            mF2->setInlier(m.trainIdx);
        }
    }
    return status != 0;
}
// [end]

// [body Frame::createFilteredCloud]
// Core/Frame.cpp:475-549: createCloud(res) (every res-th pixel of mImDepth with z > 0, unprojected, coloured from
// mImColor) + passThroughFilter("z", zmin, zmax) + downsampleCloud(leaf) + statisticalFilterCloud(k, stddev) in
// one device call over the Frame's own images -- the four calls Tracking::createKeyFrame makes in a row
void Frame::createFilteredCloud(int res, float zmin, float zmax, float leaf, int k, double stddev)
{
    std::lock_guard<std::mutex> lock(mMutexCloud);
    if (mpCloud) return;                            // :479-480
    rgbd_ctx* ctx = mpExtractor->context();
    const rgbd_cloud_params prm{res, zmin, zmax, leaf, k, stddev};
    std::vector<rgbd_point> pts((size_t)((mImDepth.rows + res - 1) / res) * ((mImDepth.cols + res - 1) / res));
    int n = 0;
    check(ctx, rgbd_keyframe_cloud_f32(ctx, mImColor.data, reinterpret_cast<const float*>(mImDepth.data), &prm,
                                       pts.data(), (int)pts.size(), &n), "rgbd_keyframe_cloud_f32");
    mpCloud = std::make_shared<PointCloudT>();
    mpCloud->points.resize(n);
    for (int i = 0; i < n; i++) {
        PointT& p = mpCloud->points[i];
        p.x = pts[i].x;
        p.y = pts[i].y;
        p.z = pts[i].z;
        p.b = pts[i].b;
        p.g = pts[i].g;
        p.r = pts[i].r;
    }
    mpCloud->height = 1;
    mpCloud->width = (uint32_t)n;
    mpCloud->is_dense = false;
}
// [end]

// [body Tracking::createKeyFrame]
// System/Tracking.cpp:227-240 with the four cloud calls as one (computeBoW(mpVoc) stays first in the reference;
// the DBoW3 vocabulary is absent here)
void Tracking::createKeyFrame()
{
    mpLastKeyFrame = mpCurFrame;
    mpLastKeyFrame->setKF();
    mpCurFrame->mpReferenceKF = mpLastKeyFrame;

    mpLastKeyFrame->createFilteredCloud(6, 0.5f, 4.0f, 0.04f, 50, 1.0);   // :234-237

    if (mpPoseGraph) mpPoseGraph->insertKeyFrame(mpLastKeyFrame);
}
// [end]

// ref_system.cpp -- the reference code around INTEGRATION.md's bodies that a maintainer keeps as it is, restated
// over the mirrored surfaces (ref_mirror.hpp) so the bodies run inside the reference's own control flow:
//   Frame       computeImageBounds / assignFeaturesToGrid and the statics (Core/Frame.cpp:15-18, 75-89, 283-315)
//   Tracking    track / initialize / visualOdometry / recover / needKeyFrame / updateLastFrame /
//               updateRelativePose (System/Tracking.cpp:39-256); createKeyFrame is a body (solver_bodies.cpp)
//   PoseGraph   the keyframe queue and its thread: updateGraph -> createNode / createEdgeWithReference /
//               createLocalEdges (Solver/PoseGraph.cpp:59-216, 289-296) over rgbd_posegraph
// plus the test hooks declared at the end of ref_mirror.hpp.
#include <algorithm>
#include <cstdio>
#include <unistd.h>

#include "ref_mirror.hpp"

int Frame::nNextId = 0;
bool Frame::mbInitialComputations = true;
float Frame::mnMinX, Frame::mnMinY, Frame::mnMaxX, Frame::mnMaxY;
float Frame::mfGridElementWidthInv, Frame::mfGridElementHeightInv;

// ------------------------------------------------------------------ test hooks
namespace refside {
static std::mutex g_order;
static int g_seq = 0;
static std::vector<SacRecord> g_sac;
static std::mutex g_pair_mu;
static std::vector<PairRecord> g_pairs;

bool sac_compute(char thread, RansacSE3& sac, std::shared_ptr<Frame> F1, std::shared_ptr<Frame> F2,
                 const std::vector<cv::DMatch>& m12, bool updateF2)
{
    std::lock_guard<std::mutex> lock(g_order);   // fixes the order of the draws for the replay
    const bool ok = sac.compute(F1, F2, m12, updateF2);
    SacRecord r{};
    r.seq = g_seq++;
    r.thread = thread;
    r.id1 = F1->id();
    r.id2 = F2->id();
    r.n_matches = (int)m12.size();
    r.ok = ok ? 1 : 0;
    r.n_inliers = (int)sac.mvInliers.size();
    std::memcpy(&r.rmse_bits, &sac.rmse, 4);
    for (int i = 0; i < 16; i++) {
        const float v = sac.mT21(i / 4, i % 4);
        std::memcpy(&r.T_bits[i], &v, 4);
    }
    g_sac.push_back(r);
    return ok;
}
std::vector<SacRecord> sac_log()
{
    std::lock_guard<std::mutex> lock(g_order);
    return g_sac;
}
void log_pair(int id_cur, int id_kf, int n_matches)
{
    std::lock_guard<std::mutex> lock(g_pair_mu);
    g_pairs.push_back(PairRecord{id_cur, id_kf, n_matches});
}
std::vector<PairRecord> pair_log()
{
    std::lock_guard<std::mutex> lock(g_pair_mu);
    return g_pairs;
}
}  // namespace refside

// ------------------------------------------------------------------ Frame (kept reference code)
void Frame::computeImageBounds()
{
    cv::Mat D = mpCamera->distCoef(), K = mpCamera->k();
    if (D.at<float>(0) != 0.0f) {   // the four image corners, undistorted
        cv::Mat c(4, 2, CV_32F);
        const float cols = (float)mImGray.cols, rows = (float)mImGray.rows;
        const float xy[8] = {0.0f, 0.0f, cols, 0.0f, 0.0f, rows, cols, rows};
        for (int i = 0; i < 8; i++) c.at<float>(i / 2, i % 2) = xy[i];
        c = c.reshape(2);
        cv::undistortPoints(c, c, K, D, cv::Mat(), K);
        c = c.reshape(1);
        mnMinX = std::min(c.at<float>(0, 0), c.at<float>(2, 0));
        mnMaxX = std::max(c.at<float>(1, 0), c.at<float>(3, 0));
        mnMinY = std::min(c.at<float>(0, 1), c.at<float>(1, 1));
        mnMaxY = std::max(c.at<float>(2, 1), c.at<float>(3, 1));
    } else {
        mnMinX = 0.0f;
        mnMaxX = (float)mImGray.cols;
        mnMinY = 0.0f;
        mnMaxY = (float)mImGray.rows;
    }
}

void Frame::assignFeaturesToGrid()
{
    const int nReserve = (int)(0.5f * N / (FRAME_GRID_COLS * FRAME_GRID_ROWS));
    for (int i = 0; i < FRAME_GRID_COLS; i++)
        for (int j = 0; j < FRAME_GRID_ROWS; j++) mGrid[i][j].reserve(nReserve);
    for (size_t i = 0; i < N; i++) {
        int gx, gy;
        if (posInGrid(mvKeysUn[i], gx, gy)) mGrid[gx][gy].push_back(i);
    }
}

// ------------------------------------------------------------------ Tracking (kept reference code)
Tracking::Tracking(std::shared_ptr<Map> pMap, bool withPoseGraph)
    : mpCurFrame(nullptr), mState(NOT_INITIALIZED), mpMap(pMap), mnAcumInliers(0), mnInliers(0), mnMeanInliers(0)
{
    if (withPoseGraph) mpPoseGraph = std::make_shared<PoseGraph>(this, pMap);
}

Tracking::~Tracking() { shutdown(); }

void Tracking::shutdown()
{
    if (mpPoseGraph) mpPoseGraph->shutdown();
}

cv::Mat Tracking::track(std::shared_ptr<Frame> newFrame)
{
    std::lock_guard<std::mutex> lck(mMutexTrack);
    mpCurFrame = newFrame;
    if (mState == NOT_INITIALIZED) {
        initialize();
    } else if (mState == OK) {
        visualOdometry();
        updateLastFrame();
        mpCurFrame->mpReferenceKF = mpLastKeyFrame;
        mVelocity = mpCurFrame->getPose() * mpRefFrame.first->getPoseInverse();   // motion model
        if (needKeyFrame()) createKeyFrame();
        mpRefFrame.second = mpRefFrame.first;
        mpRefFrame.first = mpCurFrame;
    } else {
        recover();
        mpRefFrame.second = mpRefFrame.first;
        mpRefFrame.first = mpCurFrame;
    }
    updateRelativePose();
    return mpCurFrame->getPose();
}

void Tracking::initialize()
{
    mpCurFrame->setPose(cv::Mat::eye(4, 4, CV_32F));
    for (size_t i = 0; i < mpCurFrame->N; ++i) {   // a landmark per keypoint with depth, coloured by mvKeysColor
        if (!(mpCurFrame->mvKeys3Dc[i].z > 0)) continue;
        Landmark::Ptr pLM = std::make_shared<Landmark>(mpCurFrame->unprojectWorld(i), mpCurFrame, i);
        pLM->addObservation(mpCurFrame, i);
        pLM->setColor(mpCurFrame->mvKeysColor[i]);
        mpMap->addLandmark(pLM);
        mpCurFrame->addLandmark(pLM, i);
    }
    mpRefFrame = {mpCurFrame, mpCurFrame};
    createKeyFrame();
    mState = OK;
}

void Tracking::visualOdometry()
{
    Frame::Ptr pRefFrame = mpRefFrame.first;
    Matcher matcher(0.9f);
    std::vector<cv::DMatch> vMatches, vInliers;
    matcher.match(pRefFrame, mpCurFrame, vMatches);
    RansacSE3 sac(200, 10, 3.0f, 4);
    bool b = refside::sac_compute('T', sac, pRefFrame, mpCurFrame, vMatches, true);
    if (!b) {   // the second most recent frame
        vMatches.clear();
        pRefFrame = mpRefFrame.second;
        matcher.match(pRefFrame, mpCurFrame, vMatches);
        b = refside::sac_compute('T', sac, pRefFrame, mpCurFrame, vMatches, true);
    }
    if (sac.rmse >= 0.8f) {
        Eigen::Matrix4f guess = sac.mT21;
        Solver::Ptr solver(new Gicp(pRefFrame, mpCurFrame, sac.mvInliers, guess));
        static_cast<Gicp&>(*solver).setMaxCorrespondenceDistance(0.07);
        static_cast<Gicp&>(*solver).setMaximumIterations(10);
        b = solver->compute(vInliers);
    }
    vInliers = sac.mvInliers;
    {
        std::lock_guard<std::mutex> lock(mMutexStatistics);
        mnInliers = (int)vInliers.size();
        mnAcumInliers += (int)vInliers.size();
        mnMeanInliers = mnAcumInliers / mpCurFrame->id();
    }
    if (!b) recover();
}

void Tracking::recover()
{
    mpCurFrame->setPose(mpRefFrame.first->getPose());
    mState = OK;
}

bool Tracking::needKeyFrame()   // 20 cm or 10 degrees since the last keyframe
{
    const cv::Mat delta = mpCurFrame->getPoseInverse() * mpLastKeyFrame->getPose();
    const double tn = cv::norm(delta.rowRange(0, 3).col(3));
    const float tr = delta.at<float>(0, 0) + delta.at<float>(1, 1) + delta.at<float>(2, 2);
    const double rn = std::acos(0.5 * (tr - 1.0));
    return (tn > 0.20) | (rn > 0.1745);
}

void Tracking::updateLastFrame()
{
    Frame::Ptr pRef = mpRefFrame.first->mpReferenceKF;
    const cv::Mat Tlr = mRelativeFramePoses.back();
    mpRefFrame.first->setPose(Tlr * pRef->getPose());
}

void Tracking::updateRelativePose()
{
    mRelativeFramePoses.push_back(mpCurFrame->getPose() * mpCurFrame->mpReferenceKF->getPoseInverse());
    mReferences.push_back(mpLastKeyFrame);
    mFrameTimes.push_back(mpCurFrame->mTimeStamp);
}

int Tracking::getMeanInliers()
{
    std::lock_guard<std::mutex> lock(mMutexStatistics);
    return mnMeanInliers;
}

int Tracking::getCurrentInliers()
{
    std::lock_guard<std::mutex> lock(mMutexStatistics);
    return mnInliers;
}

// ------------------------------------------------------------------ PoseGraph (kept reference code)
PoseGraph::PoseGraph(Tracking* pTracker, std::shared_ptr<Map> pMap) : mpTracker(pTracker), mpMap(pMap)
{
    if (rgbd_pg_create(&mGraph) != RGBD_OK) throw std::runtime_error("rgbd_pg_create");
    mRunThread = std::thread(&PoseGraph::run, this);
}

PoseGraph::~PoseGraph()
{
    shutdown();
    rgbd_pg_destroy(mGraph);
}

void PoseGraph::insertKeyFrame(Frame::Ptr pKF)
{
    std::lock_guard<std::mutex> lock(mMutexQueue);
    mlpKeyFrameQueue.push_back(pKF);
}

void PoseGraph::shutdown()
{
    {
        std::lock_guard<std::mutex> lock(mMutexFinish);
        mbFinishRequested = true;
    }
    if (mRunThread.joinable()) mRunThread.join();
}

bool PoseGraph::checkNewKeyFrames()
{
    std::lock_guard<std::mutex> lock(mMutexQueue);
    return !mlpKeyFrameQueue.empty();
}

void PoseGraph::run()   // :59-103, loop detection absent; finishes the queue before it stops
{
    while (true) {
        if (checkNewKeyFrames()) {
            updateGraph();
            continue;
        }
        {
            std::lock_guard<std::mutex> lock(mMutexFinish);
            if (mbFinishRequested) break;
        }
        usleep(3000);
    }
}

void PoseGraph::updateGraph()   // :105-126 with createNode / createEdgeWithReference (:184-216)
{
    {
        std::lock_guard<std::mutex> lock(mMutexQueue);
        mpCurrentKF = mlpKeyFrameQueue.front();
        mlpKeyFrameQueue.pop_front();
    }
    mpMap->addKeyFrame(mpCurrentKF);
    const cv::Mat Twc = mpCurrentKF->getPoseInverse();
    double T[16];
    for (int i = 0; i < 16; i++) T[i] = Twc.at<float>(i / 4, i % 4);
    rgbd_pg_add_vertex(mGraph, mpCurrentKF->id(), T, mpCurrentKF->id() == 0);
    if (mpCurrentKF->id() != 0 && mpReferenceKF) {
        double chi2;
        rgbd_pg_add_edge(mGraph, mpCurrentKF->id(), mpReferenceKF->id(), nullptr, 100.0, 1.0, &chi2);
    }
    mpReferenceKF = mpCurrentKF;
    createLocalEdges();
}

void PoseGraph::createLocalEdges()   // :128-155
{
    const int matchesTh = 30;
    std::vector<Frame::Ptr> candidates;
    nearestNodes(mpCurrentKF, candidates);
    for (Frame::Ptr pKFi : candidates) {
        if (pKFi == mpCurrentKF) continue;
        if (rgbd_pg_exist_edge(mGraph, mpCurrentKF->id(), pKFi->id())) continue;
        Matcher matcher(0.9f);
        std::vector<cv::DMatch> vMatches;
        matcher.match(pKFi, mpCurrentKF, vMatches);   // this thread's device context
        refside::log_pair(mpCurrentKF->id(), pKFi->id(), (int)vMatches.size());
        if ((int)vMatches.size() < matchesTh) continue;
        RansacSE3 sac(200, matchesTh, 3.0f, 4);
        if (!refside::sac_compute('P', sac, pKFi, mpCurrentKF, vMatches, false)) continue;
        double Z[16], chi2;
        for (int i = 0; i < 16; i++) Z[i] = sac.mT21(i / 4, i % 4);
        rgbd_pg_add_edge(mGraph, mpCurrentKF->id(), pKFi->id(), Z, 100.0, 1.0, &chi2);
    }
}

// :157-182: the keyframes whose camera centres lie within 0.5 m (KdTreeFLANN radiusSearch: nearest first)
void PoseGraph::nearestNodes(Frame::Ptr pKF, std::vector<Frame::Ptr>& candidates)
{
    const std::vector<Frame::Ptr> vpKFs = mpMap->getAllKeyFrames();
    const cv::Mat Ow = pKF->getCameraCenter();
    std::vector<std::pair<float, size_t>> hits;
    for (size_t i = 0; i < vpKFs.size(); i++) {
        const cv::Mat O = vpKFs[i]->getCameraCenter();
        const float dx = O.at<float>(0) - Ow.at<float>(0), dy = O.at<float>(1) - Ow.at<float>(1),
                    dz = O.at<float>(2) - Ow.at<float>(2);
        const float d2 = dx * dx + dy * dy + dz * dz;
        if (d2 <= 0.50f * 0.50f) hits.push_back({d2, i});
    }
    std::stable_sort(hits.begin(), hits.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    for (const auto& h : hits) candidates.push_back(vpKFs[h.second]);
}

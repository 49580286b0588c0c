// refside_main.cpp -- drives INTEGRATION.md's reference-side bodies (solver_bodies.cpp) the way the reference's
// callers do, over a raw sequence written by tests/test_gpu_refside.py (N frames: BGR8 640x480, then u16 depth).
//
//   pnp     the outlier-flag chain of the benchmark path: for b = 1..N-1, F2's pose prior = F1's pose, then
//           Matcher(0.9).match(F1, F2, m) (discardOutliers = true: F1's flags, written by the previous pair's
//           PnPRansac) and PnPRansac(F1, F2, m).compute(inliers) (Solver/PnPRansac.cpp:14-56 as written)
//   vo      Tracking::visualOdometry (System/Tracking.cpp:121-163): initialize(), RansacSE3(200, 10, 3, 4),
//           the second reference, Gicp with setMaxCorrespondenceDistance(0.07) / setMaximumIterations(10),
//           recover(); Random::initSeed(2024)
//   detect  Extractor::detectAndCompute on each frame's gray image (cvtColor's fixed point) against the Frame's
//           own keypoints / descriptors, then on a constant image (no keypoints: descriptors released)
//   track   main.cpp's loop: each Frame built from its images, then Tracking::track (System/Tracking.cpp:39-75;
//           initialize's landmarks from mvKeysColor, visualOdometry's id()-based mean, createKeyFrame's cloud
//           from mImColor / mImDepth), with the PoseGraph thread (pg = 1) matching keyframes and running
//           RansacSE3(..., false) on its own device context while tracking goes on; Random::initSeed(2024)
// Output (stdout): per frame "b ok n_matches n_inliers" + the 16 pose floats as hex bits (pnp, vo), or
// "detect b n same_kps same_desc" (detect) and "empty n released"; track: see run_track.
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "ref_mirror.hpp"

static void print_pose(const cv::Mat& T)
{
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            uint32_t u;
            const float v = T.at<float>(r, c);
            std::memcpy(&u, &v, 4);
            std::printf(" %08" PRIx32, u);
        }
    std::printf("\n");
}

static void print_bits(const float* v, int n)
{
    for (int i = 0; i < n; i++) {
        uint32_t u;
        std::memcpy(&u, &v[i], 4);
        std::printf(" %08" PRIx32, u);
    }
}

static void dump(const std::string& path, const void* p, size_t bytes)
{
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f || std::fwrite(p, 1, bytes, f) != bytes) throw std::runtime_error("write " + path);
    std::fclose(f);
}

// track mode.  stdout: "t b is_kf mean_inliers cur_inliers" + track()'s pose bits per frame, "frame b id N",
// "bounds" + the six grid statics' bits, "lm n", "sac seq thread id1 id2 n_matches ok n_inliers rmse T[16]" per
// RansacSE3 call in stream order, "pair id_cur id_kf n_matches" per PoseGraph candidate, "ctx n".  Files in
// out/: lm.bin (per landmark x y z f32 + b g r pad), f<b>_color.u8 (mvKeysColor), f<b>_grid.i32 (per cell,
// column-major as mGrid[i][j]: count then indices), f<b>_cloud.pts (keyframes' rgbd_point clouds), and for
// b < 2 f<b>_gray.u8 / f<b>_depth.f32 (mImGray / mImDepth).
static int run_track(const std::vector<cv::Mat>& rgb, const std::vector<cv::Mat>& dep, RGBDcamera& cam, int nfeat,
                     const std::string& out, bool pg)
{
    Random::initSeed(2024);
    auto extractor = std::make_shared<Extractor>(Extractor::ORB2, Extractor::ORB2, Extractor::NORMAL);
    extractor->setParameters(nfeat, 1.2f, 8, 20, 7);
    auto map = std::make_shared<Map>();
    std::vector<Frame::Ptr> frames;
    {
        Tracking tracker(map, pg);
        for (size_t b = 0; b < rgb.size(); b++) {
            Frame::Ptr F = std::make_shared<Frame>(rgb[b], dep[b], b / 30.0, extractor, &cam);   // grabFrame
            frames.push_back(F);
            const cv::Mat T = tracker.track(F);
            std::printf("t %zu %d %d %d", b, F->isKF() ? 1 : 0, tracker.getMeanInliers(), tracker.getCurrentInliers());
            print_pose(T);
        }
        tracker.shutdown();   // the PoseGraph thread finishes its queue
    }
    std::printf("bounds");
    const float bnd[6] = {Frame::mnMinX, Frame::mnMaxX, Frame::mnMinY, Frame::mnMaxY, Frame::mfGridElementWidthInv,
                          Frame::mfGridElementHeightInv};
    print_bits(bnd, 6);
    std::printf("\n");
    for (size_t b = 0; b < frames.size(); b++) {
        Frame& F = *frames[b];
        std::printf("frame %zu %d %zu\n", b, F.id(), F.N);
        const std::string pre = out + "/f" + std::to_string(b);
        dump(pre + "_color.u8", F.mvKeysColor.data(), F.N * 3);
        std::vector<int32_t> grid;
        for (int i = 0; i < FRAME_GRID_COLS; i++)
            for (int j = 0; j < FRAME_GRID_ROWS; j++) {
                grid.push_back((int32_t)F.mGrid[i][j].size());
                for (size_t k : F.mGrid[i][j]) grid.push_back((int32_t)k);
            }
        dump(pre + "_grid.i32", grid.data(), grid.size() * 4);
        if (F.isKF()) {
            const auto cl = F.cloud();
            if (!cl) throw std::runtime_error("keyframe without a cloud");
            std::vector<rgbd_point> pts(cl->points.size());
            for (size_t i = 0; i < pts.size(); i++) {
                const Frame::PointT& p = cl->points[i];
                pts[i] = rgbd_point{p.x, p.y, p.z, p.b, p.g, p.r, 0};
            }
            dump(pre + "_cloud.pts", pts.data(), pts.size() * sizeof(rgbd_point));
        }
        if (b < 2) {
            dump(pre + "_gray.u8", F.mImGray.data, (size_t)F.mImGray.rows * F.mImGray.cols);
            dump(pre + "_depth.f32", F.mImDepth.data, (size_t)F.mImDepth.rows * F.mImDepth.cols * 4);
        }
    }
    std::vector<uint8_t> lm;
    for (const Landmark::Ptr& p : map->getAllLandmarks()) {
        const cv::Mat X = p->getWorldPos();
        const cv::Vec3b c = p->getColor();
        const float xyz[3] = {X.at<float>(0), X.at<float>(1), X.at<float>(2)};
        const uint8_t bgr[4] = {c[0], c[1], c[2], 0};
        lm.insert(lm.end(), reinterpret_cast<const uint8_t*>(xyz), reinterpret_cast<const uint8_t*>(xyz) + 12);
        lm.insert(lm.end(), bgr, bgr + 4);
    }
    dump(out + "/lm.bin", lm.data(), lm.size());
    std::printf("lm %zu\n", lm.size() / 16);
    for (const refside::SacRecord& r : refside::sac_log()) {
        std::printf("sac %d %c %d %d %d %d %d %08" PRIx32, r.seq, r.thread, r.id1, r.id2, r.n_matches, r.ok, r.n_inliers,
                    r.rmse_bits);
        for (int i = 0; i < 16; i++) std::printf(" %08" PRIx32, r.T_bits[i]);
        std::printf("\n");
    }
    for (const refside::PairRecord& r : refside::pair_log()) std::printf("pair %d %d %d\n", r.id_cur, r.id_kf, r.n_matches);
    std::printf("ctx %zu\n", extractor->contexts());
    return 0;
}


int main(int argc, char** argv)
{
    if (argc < 14) {
        std::fprintf(stderr, "usage: %s seq.raw n fx fy cx cy k1 k2 p1 p2 k3 factor pnp pose0.f32 | vo [nfeatures] | detect | "
                             "track nfeatures outdir pg\n", argv[0]);
        return 2;
    }
    const int n = std::atoi(argv[2]);
    float a[10];
    for (int i = 0; i < 10; i++) a[i] = (float)std::atof(argv[3 + i]);
    RGBDcamera cam(a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8], a[9]);   // depthMapFactor = factor
    const std::string mode = argv[13];
    const int W = 640, H = 480;
    std::vector<cv::Mat> rgb(n), dep(n);
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 3;
    for (int i = 0; i < n; i++) {
        rgb[i].create(H, W, CV_8UC3);
        dep[i].create(H, W, CV_16U);
        if (std::fread(rgb[i].data, 1, (size_t)W * H * 3, f) != (size_t)W * H * 3) return 4;
        if (std::fread(dep[i].data, 2, (size_t)W * H, f) != (size_t)W * H) return 4;
    }
    std::fclose(f);
    try {
        if (mode == "track")   // track nfeatures outdir pg
            return argc > 16 ? run_track(rgb, dep, cam, std::atoi(argv[14]), argv[15], std::atoi(argv[16]) != 0) : 2;
        auto extractor = std::make_shared<Extractor>(Extractor::ORB2, Extractor::ORB2, Extractor::NORMAL);
        if (mode == "vo" && argc > 14)   // Extractor::setParameters(nfeatures, 1.2f, 8, 20, 7) before the first frame
            extractor->setParameters(std::atoi(argv[14]), 1.2f, 8, 20, 7);
        std::vector<Frame::Ptr> frames;
        for (int i = 0; i < n; i++) frames.push_back(std::make_shared<Frame>(rgb[i], dep[i], i / 30.0, extractor, &cam));
        if (mode == "pnp") {
            cv::Mat pose0(4, 4, CV_32F);
            FILE* g = std::fopen(argc > 14 ? argv[14] : "", "rb");
            if (!g || std::fread(pose0.data, 4, 16, g) != 16) return 5;
            std::fclose(g);
            frames[0]->setPose(pose0);
            Matcher matcher(0.9f);
            for (int b = 1; b < n; b++) {
                Frame::Ptr F1 = frames[b - 1], F2 = frames[b];
                F2->setPose(F1->getPose());
                std::vector<cv::DMatch> m, inliers;
                matcher.match(F1, F2, m, true);
                Solver::Ptr solver(new PnPRansac(F1, F2, m));
                const bool ok = solver->compute(inliers);
                std::printf("%d %d %zu %zu", b, ok ? 1 : 0, m.size(), inliers.size());
                print_pose(F2->getPose());
            }
        } else if (mode == "vo") {
            Random::initSeed(2024);
            frames[0]->setPose(cv::Mat::eye(4, 4, CV_32F));   // Tracking::initialize (:97-99)
            Frame::Ptr first = frames[0], second = frames[0];   // mpRefFrame
            for (int b = 1; b < n; b++) {
                Frame::Ptr cur = frames[b], pRefFrame = first;
                Matcher matcher(0.9f);
                std::vector<cv::DMatch> vMatches, vInliers;
                matcher.match(pRefFrame, cur, vMatches);
                RansacSE3 sac(200, 10, 3.0f, 4);
                bool ok = sac.compute(pRefFrame, cur, vMatches);
                if (!ok) {
                    vMatches.clear();
                    pRefFrame = second;
                    matcher.match(pRefFrame, cur, vMatches);
                    ok = sac.compute(pRefFrame, cur, vMatches);
                }
                if (sac.rmse >= 0.8f) {
                    Eigen::Matrix4f guess = sac.mT21;
                    Solver::Ptr solver(new Gicp(pRefFrame, cur, sac.mvInliers, guess));
                    static_cast<Gicp&>(*solver).setMaxCorrespondenceDistance(0.07);
                    static_cast<Gicp&>(*solver).setMaximumIterations(10);
                    ok = solver->compute(vInliers);
                }
                vInliers = sac.mvInliers;
                if (!ok) cur->setPose(first->getPose());      // recover() (:195-199)
                second = first;
                first = cur;
                std::printf("%d %d %zu %zu", b, ok ? 1 : 0, vMatches.size(), vInliers.size());
                print_pose(cur->getPose());
            }
        } else if (mode == "detect") {
            for (int b = 0; b < n; b++) {
                cv::Mat gray(H, W, CV_8U);                      // cvtColor BGR2GRAY, 8U fixed point
                for (int y = 0; y < H; y++)
                    for (int x = 0; x < W; x++) {
                        const uint8_t* p = rgb[b].data + ((size_t)y * W + x) * 3;
                        gray.at<uint8_t>(y, x) = (uint8_t)((1868 * p[0] + 9617 * p[1] + 4899 * p[2] + 8192) >> 14);
                    }
                std::vector<cv::KeyPoint> kps;
                cv::Mat desc;
                extractor->detectAndCompute(gray, cv::Mat(), kps, desc);
                const Frame& F = *frames[b];
                const bool same_kps = kps.size() == F.N && std::memcmp(kps.data(), F.mvKeys.data(), F.N * sizeof(cv::KeyPoint)) == 0;
                const bool same_desc = desc.rows == (int)F.N && desc.cols == 32 &&
                                       std::memcmp(desc.data, F.mDescriptors.data, F.N * 32) == 0;
                std::printf("detect %d %zu %d %d\n", b, kps.size(), same_kps ? 1 : 0, same_desc ? 1 : 0);
            }
            cv::Mat flat(H, W, CV_8U);
            std::memset(flat.data, 128, (size_t)W * H);
            std::vector<cv::KeyPoint> kps(3);
            cv::Mat desc(5, 32, CV_8U);
            extractor->detectAndCompute(flat, cv::Mat(), kps, desc);
            std::printf("empty %zu %d\n", kps.size(), desc.empty() ? 1 : 0);
        } else {
            return 2;
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}

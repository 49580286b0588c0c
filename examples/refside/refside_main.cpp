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
// Output (stdout): per frame "b ok n_matches n_inliers" + the 16 pose floats as hex bits (pnp, vo), or
// "detect b n same_kps same_desc" (detect) and "empty n released".
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

int main(int argc, char** argv)
{
    if (argc < 14) {
        std::fprintf(stderr, "usage: %s seq.raw n fx fy cx cy k1 k2 p1 p2 k3 factor pnp pose0.f32 | vo [nfeatures] | detect\n", argv[0]);
        return 2;
    }
    const int n = std::atoi(argv[2]);
    RGBDcamera cam;
    cam.fx = (float)std::atof(argv[3]);
    cam.fy = (float)std::atof(argv[4]);
    cam.cx = (float)std::atof(argv[5]);
    cam.cy = (float)std::atof(argv[6]);
    cam.k1 = (float)std::atof(argv[7]);
    cam.k2 = (float)std::atof(argv[8]);
    cam.p1 = (float)std::atof(argv[9]);
    cam.p2 = (float)std::atof(argv[10]);
    cam.k3 = (float)std::atof(argv[11]);
    cam.mDepthMapFactor = 1.0f / (float)std::atof(argv[12]);
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

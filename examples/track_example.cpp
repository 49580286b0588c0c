// track_example.cpp -- Tracking::visualOdometry (System/Tracking.cpp:121-163) written
// against the drop-in surfaces of include/rgbd/frontend.hpp, the way System/Tracking.cpp reads.
// Input: a raw sequence file written by tests (N frames of BGR8 640x480 then u16 depth).
// Output (stdout): one line per frame "idx ok n_inliers tx ty tz" of the Tcw translation.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "rgbd/frontend.hpp"

int main(int argc, char** argv)
{
    if (argc < 13) {
        std::fprintf(stderr, "usage: %s seq.raw n fx fy cx cy k1 k2 p1 p2 k3 factor [orb|svo]\n", argv[0]);
        return 2;
    }
    const char* path = argv[1];
    const int n = std::atoi(argv[2]);
    rgbd_camera cam{(float)std::atof(argv[3]), (float)std::atof(argv[4]), (float)std::atof(argv[5]),
                    (float)std::atof(argv[6]), (float)std::atof(argv[7]), (float)std::atof(argv[8]),
                    (float)std::atof(argv[9]), (float)std::atof(argv[10]), (float)std::atof(argv[11]),
                    1.0f / (float)std::atof(argv[12])};
    const int W = 640, H = 480;
    FILE* f = std::fopen(path, "rb");
    if (!f) return 3;
    std::vector<uint8_t> bgr((size_t)W * H * 3);
    std::vector<uint16_t> depth((size_t)W * H);
    try {
        // main.cpp:31: Extractor(SVO, BRIEF, NORMAL) by default in the reference; ORB2 is the north star's
        const bool svo = argc > 13 && std::string(argv[13]) == "svo";
        rgbd::Extractor extractor(svo ? rgbd::Extractor::SVO : rgbd::Extractor::ORB2,
                                  svo ? rgbd::Extractor::BRIEF : rgbd::Extractor::ORB2, rgbd::Extractor::NORMAL, W, H, cam);
        rgbd::Session session(2024);
        rgbd::Matcher matcher(extractor.ctx(), 0.9f);                 // Tracking.cpp:126
        rgbd::Frame::Ptr last, second;
        for (int i = 0; i < n; i++) {
            if (std::fread(bgr.data(), 1, bgr.size(), f) != bgr.size()) return 4;
            if (std::fread(depth.data(), 2, depth.size(), f) != depth.size()) return 4;
            auto cur = std::make_shared<rgbd::Frame>(bgr.data(), depth.data(), i / 30.0, extractor);
            bool ok = true;
            int ninl = 0;
            if (!last) {
                cur->setPose(rgbd::identity());                       // initialize(), :97-99
                second = cur;
            } else {
                std::vector<rgbd_dmatch> m;
                rgbd::Frame::Ptr ref = last;
                matcher.match(*ref, *cur, m);
                rgbd::RansacSE3 sac(extractor.ctx(), session, 200, 10, 3.0f, 4);
                ok = sac.compute(*ref, *cur, m);
                if (!ok) {                                            // second reference, :134-143
                    m.clear();
                    ref = second;
                    matcher.match(*ref, *cur, m);
                    ok = sac.compute(*ref, *cur, m);
                }
                if (sac.rmse >= 0.8f) {                               // GICP refinement, :145-151
                    rgbd::Gicp gicp(extractor.ctx(), *ref, *cur, sac.mvInliers, sac.mT21);
                    gicp.setMaxCorrespondenceDistance(0.07);
                    gicp.setMaximumIterations(10);
                    std::vector<rgbd_dmatch> vInliers;
                    ok = gicp.compute(vInliers);
                }
                if (!ok) cur->setPose(last->getPose());               // recover(), :195-199
                ninl = (int)sac.mvInliers.size();
                second = last;
            }
            last = cur;
            const rgbd::Pose& P = cur->getPose();
            std::printf("%d %d %d %.9g %.9g %.9g\n", i, ok ? 1 : 0, ninl, P[3], P[7], P[11]);
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    std::fclose(f);
    return 0;
}

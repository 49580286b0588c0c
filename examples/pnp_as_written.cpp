// pnp_as_written.cpp -- PnPRansac::compute exactly as the reference has it (Solver/PnPRansac.cpp:14-56,
// rgbd::PnPRansac(..., as_written = true)), driven the way a caller would: two frames, F2 carrying a pose,
// Matcher(0.9).match(F1, F2) with discardOutliers, then compute().  Input: a raw file of two frames (BGR8
// 640x480 then u16 depth each) and F2's Tcw (16 floats).  Output (stdout, hex bit patterns):
//   "ok n_matches n_inliers", "R r0..r8" (f64), "t t0 t1 t2" (f64), "pose p0..p15" (F2's Tcw after, f32),
//   "inl q0 q1 ..." (queryIdx of the inliers in order), "flags k" (F2 outlier flags set after compute)
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rgbd/frontend.hpp"

static uint64_t bits64(double v) { uint64_t u; std::memcpy(&u, &v, 8); return u; }
static uint32_t bits32(float v) { uint32_t u; std::memcpy(&u, &v, 4); return u; }

int main(int argc, char** argv)
{
    if (argc < 13) {
        std::fprintf(stderr, "usage: %s pair.raw pose.f32 fx fy cx cy k1 k2 p1 p2 k3 factor\n", argv[0]);
        return 2;
    }
    rgbd_camera cam{(float)std::atof(argv[3]), (float)std::atof(argv[4]), (float)std::atof(argv[5]),
                    (float)std::atof(argv[6]), (float)std::atof(argv[7]), (float)std::atof(argv[8]),
                    (float)std::atof(argv[9]), (float)std::atof(argv[10]), (float)std::atof(argv[11]),
                    1.0f / (float)std::atof(argv[12])};
    const int W = 640, H = 480;
    std::vector<uint8_t> bgr[2];
    std::vector<uint16_t> depth[2];
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 3;
    for (int i = 0; i < 2; i++) {
        bgr[i].resize((size_t)W * H * 3);
        depth[i].resize((size_t)W * H);
        if (std::fread(bgr[i].data(), 1, bgr[i].size(), f) != bgr[i].size()) return 4;
        if (std::fread(depth[i].data(), 2, depth[i].size(), f) != depth[i].size()) return 4;
    }
    std::fclose(f);
    rgbd::Pose pose2{};
    FILE* g = std::fopen(argv[2], "rb");
    if (!g || std::fread(pose2.data(), 4, 16, g) != 16) return 5;
    std::fclose(g);
    try {
        rgbd::Extractor ex(rgbd::Extractor::ORB2, rgbd::Extractor::ORB2, rgbd::Extractor::NORMAL, W, H, cam);
        rgbd::Frame F1(bgr[0].data(), depth[0].data(), 0.0, ex);
        rgbd::Frame F2(bgr[1].data(), depth[1].data(), 1.0 / 30, ex);
        F2.setPose(pose2);
        rgbd::Matcher matcher(ex.ctx(), 0.9f);
        std::vector<rgbd_dmatch> m, inliers;
        matcher.match(F1, F2, m);
        rgbd::PnPRansac pnp(ex.ctx(), F1, F2, m, /*as_written=*/true);
        const bool ok = pnp.compute(inliers);
        std::printf("%d %zu %zu\n", ok ? 1 : 0, m.size(), inliers.size());
        std::printf("R");
        for (double v : pnp.R) std::printf(" %016" PRIx64, bits64(v));
        std::printf("\nt");
        for (double v : pnp.t) std::printf(" %016" PRIx64, bits64(v));
        std::printf("\npose");
        for (float v : F2.getPose()) std::printf(" %08" PRIx32, bits32(v));
        std::printf("\ninl");
        for (const rgbd_dmatch& d : inliers) std::printf(" %d", d.queryIdx);
        int nf = 0;
        for (uint8_t b : F2.mvbOutlier) nf += b ? 1 : 0;
        std::printf("\nflags %d\n", nf);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    return 0;
}

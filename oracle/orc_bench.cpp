// orc_bench.cpp -- the CPU baseline driver (test infrastructure only: bench.py's cpu_baseline leg).
//
// THIS IS NOT PRODUCT CODE.  It times the oracle (the scalar C++ restatement of the reference's hot
// path) the way the reference's main loop runs it (main.cpp:39-48 -> Frame::Frame, Tracking::track), so
// the whole CPU leg runs in C++ with no per-call Python orchestration:
//   * extraction: Frame::Frame (Core/Frame.cpp:34-73) = gray + ORBextractor (or SVO + BRIEF) + undistort +
//     unproject, on rendered frames walked back and forth (bench.py pingpong) from a start offset, for a
//     time budget;
//   * chain over the first `chain` extracted frames, consecutive pairs:
//       solver 0 (the north-star benchmark chain, rgbd_pnp_track_batch's definition):
//         Matcher::match(F1, F2, m, discardOutliers = false) (Features/Matcher.cpp:106-139) + PnPRansac with
//         F1's 3D and F2's undistorted pixels (Solver/PnPRansac.cpp:14-56; 500 it, 3 px, 0.85), pose chained;
//       solver 1 (Tracking::visualOdometry, System/Tracking.cpp:121-163): Matcher(0.9) with the reference
//         frame's outlier flags -> RansacSE3(200, 10, 3, 4) updating F2's flags -> second reference b - 2 on
//         failure -> GICP (0.07 m, 10 iterations) when rmse >= 0.8 -> recover().
// The same sequence as tests/chain_model.py's pnp_track / track (which the GPU tests compare against).
#include <chrono>
#include <cstring>
#include <vector>

#include "rgbd_oracle.h"

namespace {

struct FrameOut {
    std::vector<orc_keypoint> kps, kun;
    std::vector<uint8_t> desc;
    std::vector<float> xyz;
    int n = 0;
};

inline int pingpong(int g, int U)
{
    if (U <= 1) return 0;
    const int r = g % (2 * U - 2);
    return r < U ? r : 2 * U - 2 - r;
}

double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// cv::Mat CV_32F 4x4 product: double accumulation in k order, one rounding (chain_model.compose)
void compose(const float* A, const float* B, float* C)
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) {
            double s = 0.0;
            for (int k = 0; k < 4; k++) s += (double)A[4 * i + k] * (double)B[4 * k + j];
            C[4 * i + j] = (float)s;
        }
}

}  // namespace

extern "C" {

typedef struct {
    int32_t frames_extracted, chain_frames, chain_ok, pad;
    double t_extract, t_chain, t_match, t_solve;
} orc_bench_result;

// Returns 0, or -1 on bad arguments.  bgr [U][H][W][3], depth [U][H][W].
int orc_bench_run(const uint8_t* bgr, const uint16_t* depth, int U, int W, int H, const orc_orb_params* orb,
                  const orc_svo_params* svo, const orc_camera* cam, int solver, int start, double seconds, int chain,
                  orc_bench_result* out)
{
    if (!bgr || !depth || U < 1 || (!orb && !svo) || !cam || !out || chain < 2) return -1;
    const int cap = 16384;
    std::vector<FrameOut> frames;
    frames.reserve(chain);
    FrameOut scratch;
    auto extract = [&](int idx, FrameOut& f) {
        f.kps.resize(cap);
        f.kun.resize(cap);
        f.desc.resize((size_t)cap * 32);
        f.xyz.resize((size_t)cap * 3);
        const uint8_t* b = bgr + (size_t)idx * W * H * 3;
        const uint16_t* d = depth + (size_t)idx * W * H;
        f.n = svo ? orc_svo_frame(b, d, W, H, svo, nullptr, cam, f.kps.data(), f.kun.data(), f.desc.data(), f.xyz.data(), cap)
                  : orc_frame(b, d, W, H, orb, cam, f.kps.data(), f.kun.data(), f.desc.data(), f.xyz.data(), cap);
        if (f.n < 0) f.n = 0;
    };
    // untimed: the first frames pay the process's page faults
    extract(pingpong(start * 5, U), scratch);
    const double t0 = now_s();
    int nfr = 0;
    for (;;) {
        if ((int)frames.size() < chain) {
            frames.emplace_back();
            extract(pingpong(start * 5 + nfr, U), frames.back());
        } else {
            extract(pingpong(start * 5 + nfr, U), scratch);
        }
        nfr++;
        if (now_s() - t0 > seconds && (int)frames.size() >= chain) break;   // at least the chain's frames
    }
    out->frames_extracted = nfr;
    out->t_extract = now_s() - t0;
    const int B = (int)frames.size();
    out->chain_frames = B;
    out->chain_ok = 0;
    out->t_match = out->t_solve = 0.0;
    std::vector<orc_dmatch> m(cap), inl(cap);
    std::vector<float> z1(cap), z2(cap), p3((size_t)cap * 3), p2((size_t)cap * 2), src((size_t)cap * 3), tgt((size_t)cap * 3);
    std::vector<uint8_t> zero(cap, 0), mask(cap);
    std::vector<std::vector<uint8_t>> flags(B, std::vector<uint8_t>(cap, 0));
    std::vector<float> poses((size_t)B * 16, 0.0f);
    for (int i = 0; i < 4; i++) poses[5 * i] = 1.0f;
    const float K4[4] = {cam->fx, cam->fy, cam->cx, cam->cy};
    orc_rng rng;
    orc_rng_seed(&rng, 99);
    orc_sticky sticky{0.0, 0, 0};
    const orc_ransac_params rp{200, 10, 3.0f, 4};
    const orc_gicp_params gp{10, 20, 0.07, 1e-9, 2e-3, 1e-3, 4, 0};
    auto zcol = [&](const FrameOut& f, std::vector<float>& z) {
        for (int i = 0; i < f.n; i++) z[i] = f.xyz[3 * (size_t)i + 2];
    };
    const double t1 = now_s();
    for (int b = 1; b < B; b++) {
        float T[16];
        std::memset(T, 0, sizeof(T));
        for (int i = 0; i < 4; i++) T[5 * i] = 1.0f;
        bool ok = false;
        int ref = b - 1;
        if (solver == 0) {
            const FrameOut &f1 = frames[b - 1], &f2 = frames[b];
            double ta = now_s();
            zcol(f1, z1);
            zcol(f2, z2);
            const int nm = orc_match(f1.desc.data(), f1.n, f2.desc.data(), f2.n, zero.data(), z1.data(), z2.data(), 0.9f,
                                     0, m.data());
            double tb = now_s();
            out->t_match += tb - ta;
            if (nm >= 10) {
                for (int i = 0; i < nm; i++) {
                    std::memcpy(&p3[3 * (size_t)i], &f1.xyz[3 * (size_t)m[i].queryIdx], 12);
                    p2[2 * (size_t)i] = f2.kun[m[i].trainIdx].x;
                    p2[2 * (size_t)i + 1] = f2.kun[m[i].trainIdx].y;
                }
                double R9[9], t3[3];
                int32_t ni = 0, it = 0;
                ok = orc_pnp_ransac(p3.data(), p2.data(), nm, K4, 500, 3.0f, 0.85, R9, t3, mask.data(), &ni, &it) != 0;
                if (ok)
                    for (int r = 0; r < 3; r++) {
                        for (int c = 0; c < 3; c++) T[4 * r + c] = (float)R9[3 * r + c];
                        T[4 * r + 3] = (float)t3[r];
                    }
            }
            out->t_solve += now_s() - tb;
        } else {
            float rmse = 0.0f;
            int32_t ni = 0;
            for (int att = 0; att < 2 && !ok; att++) {
                ref = att == 0 ? b - 1 : (b - 2 > 0 ? b - 2 : 0);
                const FrameOut &f1 = frames[ref], &f2 = frames[b];
                double ta = now_s();
                zcol(f1, z1);
                zcol(f2, z2);
                const int nm = orc_match(f1.desc.data(), f1.n, f2.desc.data(), f2.n, flags[ref].data(), z1.data(),
                                         z2.data(), 0.9f, 1, m.data());
                double tb = now_s();
                out->t_match += tb - ta;
                ok = orc_ransac_se3(f1.xyz.data(), f2.xyz.data(), m.data(), nm, &rp, &rng, &sticky, 1, flags[b].data(), T,
                                    inl.data(), &ni, &rmse) != 0;
                out->t_solve += now_s() - tb;
            }
            if (rmse >= 0.8f) {   // Gicp(pRefFrame, cur, sac.mvInliers, sac.mT21)
                double tb = now_s();
                for (int i = 0; i < ni; i++) {
                    std::memcpy(&src[3 * (size_t)i], &frames[ref].xyz[3 * (size_t)inl[i].queryIdx], 12);
                    std::memcpy(&tgt[3 * (size_t)i], &frames[b].xyz[3 * (size_t)inl[i].trainIdx], 12);
                }
                float Tg[16];
                ok = orc_gicp_compute(src.data(), tgt.data(), ni, T, &gp, Tg) != 0;
                std::memcpy(T, Tg, sizeof(T));
                out->t_solve += now_s() - tb;
            }
        }
        if (ok) {
            compose(T, &poses[(size_t)ref * 16], &poses[(size_t)b * 16]);
            out->chain_ok++;
        } else {
            std::memcpy(&poses[(size_t)b * 16], &poses[(size_t)(b - 1) * 16], 64);
        }
    }
    out->t_chain = now_s() - t1;
    return 0;
}

}  // extern "C"

// lane_replay_dev.h -- the device RansacSE3 loop's sampler and replay (Solver/SolverSE3.cpp:54-125, 135-159),
// shared by k_lane_match / k_lane_replay (lanes.hip) and the fused replay tail of k_ransac_hyp_lanes (ransac.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lanes_dev.h"

namespace rgbd {
namespace {

// ---------------------------------------------------------------- glibc rand (System/Random.cpp:16-20)
// random_r TYPE_3 held by one wave: lane i < 31 keeps state word i, the two indices are wave-uniform, so a
// draw is two v_readlane + one add + one masked move (no LDS / memory round trip per call).  Every lane of
// the wave calls next() together and gets the same value.
struct WaveGlibc {
    int32_t sv;   // state word `lane` (lanes >= 31: unused)
    int f, r;     // wave-uniform
    __device__ void load(const int32_t* st)   // st: state[31], f, r
    {
        const int lane = threadIdx.x & 63;
        sv = lane < 31 ? st[lane] : 0;
        f = __builtin_amdgcn_readfirstlane(st[31]);
        r = __builtin_amdgcn_readfirstlane(st[32]);
    }
    __device__ void store(int32_t* st) const
    {
        const int lane = threadIdx.x & 63;
        if (lane < 31) st[lane] = sv;
        if (lane == 0) {
            st[31] = f;
            st[32] = r;
        }
    }
    __device__ int32_t next()
    {
        const uint32_t val = (uint32_t)__builtin_amdgcn_readlane(sv, f) + (uint32_t)__builtin_amdgcn_readlane(sv, r);
        sv = ((int)(threadIdx.x & 63) == f) ? (int32_t)val : sv;
        if (++f >= 31) {
            f = 0;
            ++r;
        } else if (++r >= 31) {
            r = 0;
        }
        return (int32_t)(val >> 1);
    }
    // Random::randomInt(0, M - 1)
    __device__ int random_int(int M) { return int(((double)next() / ((double)2147483647 + 1.0)) * (double)M); }
};

// hypotheses [h0, h1) of lane l: sample ids, their count, cumulative rand() calls (from `calls`); called by a
// whole wave (the generator's state is spread over its lanes), lane 0 writes
__device__ inline void sample_hyps(const LaneBufs& lb, const LaneCfg& lc, int l, WaveGlibc& g, int h0, int h1, int m, int calls)
{
    const int SS = lc.SS;
    int* smp = lb.samples + (size_t)l * lc.H * SS;
    int* scnt = lb.scount + (size_t)l * lc.H;
    int* cum = lb.snap + (size_t)l * lc.H;
    const bool w0 = (threadIdx.x & 63) == 0;
    for (int h = h0; h < h1; h++) {
        int ids[8];
        int n = 0, safety = 0;
        while (n < SS) {
            int id1 = g.random_int(m);
            const int id2 = g.random_int(m);
            calls += 2;
            if (id1 > id2) id1 = id2;
            int pos = 0;
            while (pos < n && ids[pos] < id1) pos++;
            if (pos == n || ids[pos] != id1) {
                for (int k = n; k > pos; k--) ids[k] = ids[k - 1];
                ids[pos] = id1;
                n++;
            }
            if (++safety > 10000) break;
        }
        if (w0) {
            for (int k = 0; k < n; k++) smp[(size_t)h * SS + k] = ids[k];
            scnt[h] = n;
            cum[h] = calls;
        }
    }
}

// ---------------------------------------------------------------- the sequential RANSAC loop and its outcome
// phase 0: replay over the first chunk; a lane that needs more hypotheses is left to phase 1, and phase 1
// draws the samples of the rest, [e1, H), for a lane that needs them in phase 2 (glibc rand on one wave).
// The phase that completes a lane's pair writes its result and, unless the second reference runs next round,
// moves the lane to the next frame.  Run by every thread of the calling workgroup (k_lane_replay's one wave, or
// the last-finishing k_ransac_hyp_lanes workgroup of the lane); the work is wave 0's, the barriers everyone's.
__device__ inline void lane_replay(const LaneBufs& lb, const LaneCfg& lc, int l, int phase)
{
    __shared__ int s_best, s_ok, s_n, s_hit, s_hyps, s_calls;
    __shared__ float s_rmse;
    __shared__ int s_wbase;
    const int tid = threadIdx.x, lane = tid & 63;
    const bool w0 = tid < 64;
    LaneCtl& c = lb.ctl[l];
    if (c.b > c.end) return;
    if (phase > 0 && c.need_more != phase) return;
    const int att = c.retry;   // this round's attempt (written below only after every lane has read it)
    const int b = c.b;
    const int M = c.m;
    const HypOut* ho = lb.hyp + (size_t)l * (lc.H + 1);
    if (tid == 0) {
        int bestH = -1;
        bool ok = false;
        float rmse = 1e6f;
        int nin = 0, hused = 0;
        bool need = false;
        if (!c.early) {
            const int H = c.H;
            const int evaluated = phase == 0 ? min(lc.e0, H) : (phase == 1 ? min(lc.e1, H) : H);
            int validIters = 0;
            size_t bestN = 0;
            int h = 0;
            for (int n = 0; n < lc.iters && (uint32_t)M >= (uint32_t)lc.SS; n++) {
                if (h >= evaluated) {   // the loop needs a hypothesis not evaluated yet
                    need = true;
                    break;
                }
                const HypOut& o = ho[h];
                h++;
                if (o.n > 0) {
                    validIters++;
                    const size_t nr = (size_t)o.n;
                    if (o.err <= (double)rmse && nr >= bestN && nr >= lc.minTh) {
                        rmse = (float)o.err;
                        bestH = h - 1;
                        bestN = nr;
                        if (nr > M * 0.5) n += 10;
                        if (nr > M * 0.75) n += 10;
                        if (nr > M * 0.8) break;
                    }
                }
            }
            hused = h;
            if (!need) {
                // the RNG after the h hypotheses drawn (advanced by the wave below)
                s_calls = h > 0 ? lb.snap[(size_t)l * lc.H + h - 1] : 0;
                if (validIters == 0) {   // identity fallback (:105-117)
                    const HypOut& id = ho[lc.H];
                    if ((uint32_t)id.n > lc.minTh && id.err < (double)lc.maxMahal) {
                        bestH = lc.H;
                        rmse = (float)((double)rmse + id.err);
                    }
                }
                if (bestH >= 0) nin = ho[bestH].n;
                ok = bestH >= 0 && (uint32_t)nin >= lc.minTh;
            }
        }
        s_hyps = hused;
        s_best = bestH;
        s_ok = ok ? 1 : 0;
        s_n = nin;
        s_rmse = rmse;
        s_hit = need ? 1 : 0;
        if (need) c.need_more = phase + 1;
    }
    if (tid == 0 && (c.early || s_hit)) s_calls = 0;
    __syncthreads();
    if (!w0) {
    } else if (s_hit) {   // sampleMatches for the next chunk's hypotheses, continuing the sampler's RNG (whole wave)
        const int h0 = phase == 0 ? lc.e0 : lc.e1, h1 = phase == 0 ? min(lc.e1, c.H) : c.H;
        WaveGlibc g;
        g.load(c.srng);
        sample_hyps(lb, lc, l, g, h0, h1, c.m, h0 > 0 ? lb.snap[(size_t)l * lc.H + h0 - 1] : 0);
        g.store(c.srng);
    } else if (s_calls > 0) {   // the lane's RNG advanced by the rand() calls of the hypotheses drawn
        WaveGlibc g;
        g.load(c.rng);
        for (int k = 0; k < s_calls; k++) (void)g.next();
        g.store(c.rng);
    }
    __syncthreads();
    if (s_hit) return;   // phase 0: finished by phase 1
    const int bestH = s_best;
    const bool ok = s_ok != 0;
    PairOut& po = lb.out[b];
    const float* Tb = bestH >= 0 ? ho[bestH].T : nullptr;
    // mvInliers = the best mask's matches in sorted order; updateF2: their train indices are inliers
    const uint32_t* mask = lb.masks + ((size_t)l * (lc.H + 1) + (bestH >= 0 ? bestH : 0)) * lc.MWcap;
    const int2* mt = lb.mt + (size_t)l * lc.Mcap;
    uint8_t* fcur = lb.flags + (size_t)b * lc.K;
    const bool gicp_now = lc.gicp && s_rmse >= 0.8f && !(att == 0 && !ok);
    // GICP reads nothing the chain writes later (flags, RNG and sticky state are RANSAC's), so its problem is
    // staged in pair b's slot and solved with every other pair's after the rounds (k_gicp_*_pairs)
    const size_t go = (size_t)b * lc.GM * 3;
    if (tid == 0) s_wbase = 0;
    __syncthreads();
    if (bestH >= 0 && !c.early) {
        for (int i0 = 0; i0 < M; i0 += 64) {
            const int i = i0 + lane;
            const bool in = w0 && i < M && ((mask[i >> 5] >> (i & 31)) & 1u);
            const unsigned long long bal = __ballot(in);
            const int pos = s_wbase + __popcll(bal & ((1ull << lane) - 1ull));
            if (in) {
                const int2 qt = mt[i];
                if (ok) fcur[qt.y] = 0;
                if (gicp_now && pos < lc.GM) {   // createCloudsFromMatches (Solver/Gicp.cpp:37-52)
                    const float* p = lb.pts + ((size_t)l * lc.Mcap + i) * 6;
                    for (int k = 0; k < 3; k++) {
                        lb.gsrc[go + 3 * pos + k] = p[k];
                        lb.gtgt[go + 3 * pos + k] = p[3 + k];
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (tid == 0) s_wbase += __popcll(bal);
            __syncthreads();
        }
    }
    const bool retry_next = att == 0 && !ok;   // the second reference (Tracking.cpp:134-143), in the lane's next round
    if (tid < 16) {
        const float v = Tb ? Tb[lane] : ((lane % 5 == 0) ? 1.0f : 0.0f);
        po.Tsac[lane] = v;
        if (!retry_next) po.T[lane] = v;   // a GICP pair's T is k_gicp_post's
        if (gicp_now) lb.gguess[(size_t)b * 16 + lane] = v;
    }
    if (tid == 0) {
        const int nin = (bestH >= 0) ? s_n : 0;
        po.rmse = s_rmse;
        po.sac_ok = ok ? 1 : 0;
        po.n_inliers = nin;
        po.ref = c.ref;
        po.retried = att;
        po.hyps = s_hyps;
        c.run = 0;
        c.retry = 0;
        po.gicp_run = 0;
        lb.gn[b] = 0;
        if (retry_next) {
            c.retry = 1;
            lb.rq[l] = max(b - 2, c.start);
            lb.rt[l] = b;
        } else {
            lb.rq[l] = -1;
            if (gicp_now) {   // Gicp(pRefFrame, cur, sac.mvInliers, sac.mT21): < 20 pairs -> false
                if (nin > lc.GM) c.err = 2;
                lb.gn[b] = nin >= 20 ? min(nin, lc.GM) : 0;
                po.gicp_run = 1;
            }
            po.ok = gicp_now ? 0 : (ok ? 1 : 0);   // a GICP pair's result is k_gicp_post's
            po.gicp_ok = 0;
            c.b = b + 1;
        }
    }
}

}  // namespace
}  // namespace rgbd

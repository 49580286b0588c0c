"""GPU parity: the device-resident RansacSE3 tracking chain (rgbd-slam_amd/csrc/lanes.hip, lanes_host.cpp).

  * the device std::sort(vUsedMatches) (Solver/SolverSE3.cpp:52) equals libstdc++'s order (oracle), ties,
    adversarial orders and introsort's heap-sort fallback (forced depth limits) included;
  * rgbd_track_lanes: L lanes of one batch advanced together on the device; every lane equals the oracle
    chain (tests/chain_model.py: Matcher -> RansacSE3 -> second reference -> GICP when rmse >= 0.8 ->
    recover) over its own frames with its own RNG and sticky covariance: poses, status, inliers bit for bit,
    and the RNG / sticky state after the lane.  Config 3 (fr2 camera, 2000 keypoints, GICP), with a
    noise frame in one lane so that lane takes the second-reference retry and recover().
"""
import numpy as np
import pytest

from conftest import synth_seq
import chain_model

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sctx(pkg):
    c = pkg.Context(640, 480, max_batch=1)
    yield c
    c.close()


@pytest.mark.parametrize("n", [1, 2, 7, 16, 17, 40, 64, 65, 100, 128, 333, 500, 1024, 2304])
def test_device_sort_matches_libstdcxx(oracle, sctx, n):
    rs = np.random.RandomState(100 + n)
    arrays = [rs.randint(0, 30, size=n), rs.randint(0, 256, size=n), np.sort(rs.randint(0, 60, size=n)),
              np.sort(rs.randint(0, 60, size=n))[::-1], np.full(n, 3), rs.permutation(n) % 257]
    for d in arrays:
        d = d.astype(np.float32)
        for dl in ((-1,) if n <= 16 else (-1, 0, 2, 5)):
            want = oracle.sort_dmatch(d, dl)
            got = sctx.debug_sort_matches(d, dl)
            assert np.array_equal(got, want), (n, dl)


def _lane_case(pkg, oracle, B, L, nfeat, preset, seed, noise_frame=None, step=1):
    import torch
    bgr, depth, gt, cam = synth_seq(step * (B - 1) + 1, seed=seed, preset=preset)
    bgr, depth, gt = bgr[::step].copy(), depth[::step].copy(), gt[::step]
    if noise_frame is not None:
        bgr[noise_frame] = np.random.RandomState(5).randint(0, 256, size=bgr[noise_frame].shape).astype(np.uint8)
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"], cam["k3"],
                   cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(nfeat), cam=c)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    seeds = [300 + 17 * l for l in range(L)]
    rngs = [pkg.rng(s) for s in seeds]
    sts = [pkg.Sticky() for _ in range(L)]
    pose0 = gt[0].astype(np.float32)
    poses, status, ninl, raw = ctx.track_lanes(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, pkg.ransac_params(), L, rngs,
                                               sts, pose0)
    ctx.close()
    p, oc = oracle.orb_params(nfeat), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(B)]
    base, rem = divmod(B, L)
    st = [l * base + min(l, rem) for l in range(L + 1)]
    lf = [0] + [st[l] - 1 for l in range(1, L)] + [B - 1]
    logs = []
    for l in range(L):
        a, z = lf[l], lf[l + 1]
        p0 = pose0 if l == 0 else np.eye(4, dtype=np.float32)
        log = []
        wp, ws, wn, wr, wst = chain_model.track(oracle, frames[a:z + 1], p0, seeds[l], log=log)
        rows = slice(a + l, z + l + 1)
        assert np.array_equal(raw[rows].view(np.uint32), wp.view(np.uint32)), l
        # (status / inliers of the lane-major rows: row 0 of a lane is its reference frame)
        assert list(rngs[l].state) == list(wr.state) and (rngs[l].f, rngs[l].r) == (wr.f, wr.r), l
        assert sts[l].cov == wst.cov and sts[l].set == wst.set, l
        logs.append((ws, wn, log))
    return poses, status, ninl, logs, gt, lf


def test_track_lanes_config3_matches_per_lane_oracle(pkg, oracle):
    """BASELINE config 3 shape: fr2 camera, ORB 2000 keypoints, RansacSE3 -> second reference -> GICP.
    Every third frame of the sequence (rmse >= 0.8 on some, so GICP refines them); frame 8 is noise, so
    lane 1 fails on it against frame 7, retries against frame 6, and recovers.  Frame 8 is also lane 2's
    first frame (lane_first = [0, 4, 8, 12]), so frame 9's two attempts both use frame 8 (the second
    reference is max(b - 2, lane start) = 8) and it recovers too.  A retry that succeeds against b - 2
    inside a lane is test_track_lanes_retry_inside_a_lane."""
    B, L = 13, 3
    poses, status, ninl, logs, gt, lf = _lane_case(pkg, oracle, B, L, 2000, "fr2", 29, noise_frame=8, step=3)
    want_status = np.concatenate([logs[0][0]] + [lg[0][1:] for lg in logs[1:]])
    want_inl = np.concatenate([logs[0][1]] + [lg[1][1:] for lg in logs[1:]])
    assert np.array_equal(status, want_status) and np.array_equal(ninl, want_inl)
    assert sum(g for lg in logs for (_, g) in lg[2]) >= 2, "the chain should take the GICP branch"
    assert not status[8] and status.sum() >= B - 2


def test_track_lanes_fr1_many_lanes(pkg, oracle):
    """Config 2's camera at 1000 keypoints, 8 lanes of 3-4 frames: lane boundaries, fresh flags per lane."""
    B, L = 26, 8
    poses, status, ninl, logs, gt, lf = _lane_case(pkg, oracle, B, L, 1000, "fr1", 31)
    assert status.all()
    for b in range(1, B):   # the stitched trajectory follows the ground truth frame to frame
        rel = poses[b] @ np.linalg.inv(poses[b - 1])
        rel_gt = gt[b] @ np.linalg.inv(gt[b - 1])
        assert np.linalg.norm(rel[:3, 3] - rel_gt[:3, 3]) < 0.02


def test_track_lanes_on_a_prior_extraction(pkg, oracle):
    """rgbd_track_lanes(d_bgr = d_depth = NULL) tracks the context's last rgbd_extract_batch: the same bits as
    the one-call form (the bench's two-context schedule extracts and tracks in separate calls)."""
    import torch
    B, L = 12, 3
    bgr, depth, gt, cam = synth_seq(B, seed=47, preset="fr1")
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"], cam["k3"],
                   cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(1000), cam=c)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    out = []
    for split in (False, True):
        rngs = [pkg.rng(500 + l) for l in range(L)]
        sts = [pkg.Sticky() for _ in range(L)]
        if split:
            ctx.extract_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B)
            out.append(ctx.track_lanes(0, 0, B, 0.9, pkg.ransac_params(), L, rngs, sts, gt[0].astype(np.float32)))
        else:
            out.append(ctx.track_lanes(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, pkg.ransac_params(), L, rngs, sts,
                                       gt[0].astype(np.float32)))
    with pytest.raises(pkg.RgbdError):   # no extraction of this many frames to track
        ctx.track_lanes(0, 0, B - 1, 0.9, pkg.ransac_params(), L, [pkg.rng(1) for _ in range(L)],
                        [pkg.Sticky() for _ in range(L)])
    ctx.close()
    (p1, s1, n1, r1), (p2, s2, n2, r2) = out
    assert np.array_equal(r1.view(np.uint32), r2.view(np.uint32))
    assert np.array_equal(s1, s2) and np.array_equal(n1, n2) and s1.all()


def test_track_lanes_retry_inside_a_lane(pkg, oracle):
    """A noise frame strictly inside a lane (B = 13, L = 3: lane 1 = frames 4..8, frame 6 noise): frame 6
    fails against 5 and 4 and recovers; frame 7 fails against the noise frame 6, and its retry against the
    second reference b - 2 = 5 (a real frame of the same lane) succeeds (System/Tracking.cpp:134-143)."""
    B, L = 13, 3
    poses, status, ninl, logs, gt, lf = _lane_case(pkg, oracle, B, L, 1000, "fr1", 37, noise_frame=6)
    assert lf[1] == 4 and lf[2] == 8
    log1 = logs[1][2]   # lane 1's (retried, gicp) for frames 5, 6, 7, 8
    assert log1[6 - 5][0] and not status[6]
    assert log1[7 - 5][0] and status[7], "frame 7's retry against frame 5 should succeed"
    assert status[8]

"""GPU parity: the tracking front-end chain over a device-resident batch (rgbd_track_batch) vs an
oracle-driven restatement of Tracking::visualOdometry (RansacSE3 -> second reference -> GICP when
rmse >= 0.8 -> recover; tests/chain_model.py), at the BASELINE configs 2 (fr1, 1000 kp) and 3
(fr2 / desk-like, 2000 kp, GICP refinement), and split into concurrent lanes as bench.py runs it."""
import ctypes as C

import numpy as np
import pytest

from conftest import synth_seq
import chain_model

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("preset,seed", [("fr1", 13), ("fr3", 17)])
def test_track_batch_matches_oracle_chain(pkg, oracle, preset, seed):
    import torch
    B = 6
    bgr, depth, gt, cam = synth_seq(B, seed=seed, preset=preset)
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(1000), cam=c)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pose0 = gt[0].astype(np.float32)
    r = pkg.rng(2024)
    st = pkg.Sticky()
    poses, status, ninl = ctx.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, pkg.ransac_params(), r, st,
                                          pose0)
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(B)]
    wp, ws, wn, wr, wst = chain_model.track(oracle, frames, pose0, 2024)
    assert np.array_equal(status, ws)
    assert np.array_equal(ninl, wn)
    assert np.array_equal(poses.view(np.uint32), wp.view(np.uint32))
    assert list(r.state) == list(wr.state) and st.cov == wst.cov
    assert status.all()
    # tracking quality on the synthetic sequence: relative motion error per frame
    for b in range(1, B):
        rel = poses[b] @ np.linalg.inv(poses[b - 1])
        rel_gt = gt[b] @ np.linalg.inv(gt[b - 1])
        assert np.linalg.norm(rel[:3, 3] - rel_gt[:3, 3]) < 0.02
    ctx.close()


def _ctx(pkg, cam, B, nfeat):
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    return pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(nfeat), cam=c)


def test_track_batch_config3_fr2_2000kp_gicp_retry(pkg, oracle):
    """BASELINE config 3: TUM fr2/desk-like camera (depth factor 5208), ORB 2000 keypoints, the
    reference tracker's chain with GICP refinement (System/Tracking.cpp:121-163, Solver/Gicp.cpp:21-66).
    Frame 3 is replaced by noise (valid depth), so RansacSE3 fails on it (retry, then recover()) and
    frame 4 fails against frame 3 and succeeds against the second reference, frame 2.  Poses, status,
    inliers, the RNG state and the sticky covariance equal the oracle chain bit for bit; the chain
    takes the GICP branch and the retry."""
    import torch
    B = 8
    bgr, depth, gt, cam = synth_seq(3 * B - 2, seed=29, preset="fr2")
    bgr, depth, gt = bgr[::3].copy(), depth[::3].copy(), gt[::3]   # every third frame: RANSAC rmse >= 0.8 on some
    bgr[3] = np.random.RandomState(5).randint(0, 256, size=bgr[3].shape).astype(np.uint8)
    ctx = _ctx(pkg, cam, B, 2000)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pose0 = gt[0].astype(np.float32)
    r, st = pkg.rng(77), pkg.Sticky()
    poses, status, ninl = ctx.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, pkg.ransac_params(), r, st,
                                          pose0)
    p, oc = oracle.orb_params(2000), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(B)]
    assert min(len(f["kps"]) for i, f in enumerate(frames) if i != 3) > 1500
    log = []
    wp, ws, wn, wr, wst = chain_model.track(oracle, frames, pose0, 77, log=log)
    assert np.array_equal(status, ws) and np.array_equal(ninl, wn)
    assert np.array_equal(poses.view(np.uint32), wp.view(np.uint32))
    assert list(r.state) == list(wr.state) and st.cov == wst.cov
    assert sum(g and s for (_, g), s in zip(log, status[1:])) >= 2, log   # GICP refined tracked frames
    assert log[2][0] and log[3][0], log           # log[b - 1]: frames 3 and 4 retried the second reference
    assert status[3] == 0 and status[4] == 1      # the noise frame recovered; frame 4 tracked against frame 2
    rel = poses[4] @ np.linalg.inv(poses[2])
    rel_gt = gt[4] @ np.linalg.inv(gt[2])
    assert np.linalg.norm(rel[:3, 3] - rel_gt[:3, 3]) < 0.05
    ctx.close()


def test_track_lanes_equal_per_chunk_oracle_chains(pkg, oracle):
    """bench.py --solver se3: the batch split into lanes (1-frame halo, an RNG / sticky covariance each,
    rgbd_track_lanes: all lanes advanced together on the device) equals one oracle chain per chunk, stitched
    like the multi-GPU chunks (dist.stitch)."""
    import torch
    import rgbd_slam_amd.dist as D
    B, L = 10, 3
    bgr, depth, gt, cam = synth_seq(B, seed=13, preset="fr1")
    ctx = _ctx(pkg, cam, B, 1000)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pose0 = gt[0].astype(np.float32)
    rngs = [pkg.rng(1234 + l) for l in range(L)]
    sts = [pkg.Sticky() for _ in range(L)]
    poses, status, ninl, _ = ctx.track_lanes(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, pkg.ransac_params(), L, rngs,
                                             sts, pose0)
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(B)]
    chunks, ws_all, wn_all = [], [], []
    for l in range(L):
        a, z = D.shard_range(B, L, l)
        p0 = pose0 if l == 0 else np.eye(4, dtype=np.float32)
        wp, ws, wn, wr, wst = chain_model.track(oracle, frames[a:z], p0, 1234 + l)
        assert list(rngs[l].state) == list(wr.state) and sts[l].cov == wst.cov
        chunks.append(wp)
        ws_all.append(ws if l == 0 else ws[1:])
        wn_all.append(wn if l == 0 else wn[1:])
    want = D.stitch(chunks, pose0)
    assert np.array_equal(poses.view(np.uint32), want.view(np.uint32))
    assert np.array_equal(status, np.concatenate(ws_all)) and np.array_equal(ninl, np.concatenate(wn_all))
    ctx.close()


@pytest.mark.parametrize("preset,step,B,nfeat,noise", [("fr1", 4, 12, 1000, False), ("fr2", 3, 8, 2000, True)])
def test_track_batch_kf_matches_oracle_tracking(pkg, oracle, preset, step, B, nfeat, noise):
    """rgbd_track_batch_kf = Tracking::track (System/Tracking.cpp:39-73) from initialize(): visualOdometry
    plus updateLastFrame, needKeyFrame / createKeyFrame and updateRelativePose in the reference's float
    Mat arithmetic (tests/chain_model.track_kf).  fr1 every 4th frame crosses the 20 cm keyframe
    threshold twice; on fr2 (config 3, noise frame 3) frame 4's second-reference retry reads frame 2's
    pose as updateLastFrame rewrote it, so its pose differs from the un-anchored chain's."""
    import torch
    bgr, depth, gt, cam = synth_seq(step * (B - 1) + 1, seed=29, preset=preset)
    bgr, depth, gt = bgr[::step].copy(), depth[::step].copy(), gt[::step]
    if noise:
        bgr[3] = np.random.RandomState(5).randint(0, 256, size=bgr[3].shape).astype(np.uint8)
    ctx = _ctx(pkg, cam, B, nfeat)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pose0 = gt[0].astype(np.float32)
    r, st, ts = pkg.rng(77), pkg.Sticky(), pkg.TrackState()
    poses, status, ninl, rel, kf = ctx.track_batch_kf(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9,
                                                      pkg.ransac_params(), r, st, ts, pose0)
    p, oc = oracle.orb_params(nfeat), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(B)]
    log = []
    wp, ws, wn, wrel, wkf, wr, wst = chain_model.track_kf(oracle, frames, pose0, 77, log=log)
    assert np.array_equal(status, ws) and np.array_equal(ninl, wn)
    assert np.array_equal(kf, wkf) and kf.sum() >= 2, kf
    assert np.array_equal(poses.view(np.uint32), wp.view(np.uint32))
    assert np.array_equal(rel.view(np.uint32), wrel.view(np.uint32))
    assert list(r.state) == list(wr.state) and st.cov == wst.cov
    # the state hands the last frame's bookkeeping on
    assert ts.valid == 1 and ts.first_is_kf == int(kf[-1])
    assert np.array_equal(np.ctypeslib.as_array(ts.first_rel).view(np.uint32), wrel[-1].reshape(16).view(np.uint32))
    if noise:
        assert log[3][0] and status[4] == 1
        plain, *_ = chain_model.track(oracle, frames, pose0, 77)
        assert not np.array_equal(poses[4].view(np.uint32), plain[4].view(np.uint32))
    ctx.close()


@pytest.mark.parametrize("preset,step,n,nfeat,noise,cut", [("fr1", 4, 12, 1000, False, 7), ("fr2", 3, 8, 2000, True, 4)])
def test_track_batch_kf_chunks_equal_one_chain(pkg, oracle, preset, step, n, nfeat, noise, cut):
    """Two chunks that overlap by two frames (rgbd_track_state: mpRefFrame.second / .first, their outlier
    flags, keyframe and relative pose handed on) track exactly as one chain over the sequence.  On fr2 the
    second chunk starts at frame 2, so its first tracked frame (4) fails against the noise frame 3 and
    retries against frame 2, the chunk's frame 0, with the pose and flags the first chunk left."""
    import torch
    bgr, depth, gt, cam = synth_seq(step * (n - 1) + 1, seed=29, preset=preset)
    bgr, depth, gt = bgr[::step].copy(), depth[::step].copy(), gt[::step]
    if noise:
        bgr[3] = np.random.RandomState(5).randint(0, 256, size=bgr[3].shape).astype(np.uint8)
    ctx = _ctx(pkg, cam, n, nfeat)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pose0 = gt[0].astype(np.float32)
    r, st, ts = pkg.rng(77), pkg.Sticky(), pkg.track_state(ctx.kp_cap)
    poses = np.zeros((n, 4, 4), np.float32)
    rel = np.zeros((n, 4, 4), np.float32)
    status, ninl, kf = (np.zeros(n, np.int32) for _ in range(3))
    for s, e in ((0, cut), (cut - 2, n)):
        B = e - s
        k0 = 2 if ts.valid else 1
        p, sb, ib, rb, kb = ctx.track_batch_kf(d_bgr[s:e].data_ptr(), d_dep[s:e].data_ptr(), B, 0.9,
                                               pkg.ransac_params(), r, st, ts, pose0 if s == 0 else poses[s + 1])
        lo = 0 if k0 == 1 else k0
        poses[s + lo:e], rel[s + lo:e], kf[s + lo:e] = p[lo:], rb[lo:], kb[lo:]
        status[s + lo:e], ninl[s + lo:e] = sb[lo:], ib[lo:]
    p_, oc = oracle.orb_params(nfeat), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p_, oc) for i in range(n)]
    log = []
    wp, ws, wn, wrel, wkf, wr, wst = chain_model.track_kf(oracle, frames, pose0, 77, log=log)
    assert np.array_equal(status[1:], ws[1:]) and np.array_equal(ninl[1:], wn[1:])
    assert np.array_equal(kf, wkf)
    assert np.array_equal(poses.view(np.uint32), wp.view(np.uint32))
    assert np.array_equal(rel.view(np.uint32), wrel.view(np.uint32))
    assert list(r.state) == list(wr.state) and st.cov == wst.cov
    if noise:
        assert log[3][0] and status[4] == 1   # frame 4 (the second chunk's first tracked) retried
    ctx.close()

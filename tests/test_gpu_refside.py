"""GPU: INTEGRATION.md's reference-side bodies (examples/refside/solver_bodies.cpp, compiled against the
reference's class surfaces mirrored in examples/refside/ref_mirror.hpp) driven the way the reference's callers
drive them (examples/refside/refside_main.cpp), bit for bit against the oracle chains:
  * PnPRansac::compute as written (Solver/PnPRansac.cpp:14-56) over the outlier-flag chain of Matcher::match
    (Features/Matcher.cpp:125-128): mF2->setOutlier for every match, setInlier for the RANSAC inliers (:31, :51);
  * Tracking::visualOdometry (System/Tracking.cpp:121-163) over RansacSE3::compute and Gicp::compute with the
    setters Tracking calls (0.07 m, 10 iterations) and Gicp's mbUpdate / isIdentity rules (Solver/Gicp.cpp:21-35);
  * Extractor::detectAndCompute keeps the descriptors it wrote and releases them on zero keypoints
    (Features/ORBextractor.cpp:726-730)."""
import os
import subprocess

import numpy as np
import pytest

import chain_model
from conftest import ROOT, synth_seq

pytestmark = pytest.mark.gpu

EXE = os.path.join(ROOT, "rgbd-slam_amd", "build", "refside")
CAM_KEYS = ("fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2", "k3", "factor")


def _run(tmp_path, bgr, depth, cam, mode, pose0=None, extra=()):
    assert os.path.exists(EXE), "build() must compile examples/refside"
    raw = tmp_path / "seq.raw"
    with open(raw, "wb") as f:
        for i in range(len(bgr)):
            f.write(np.ascontiguousarray(bgr[i]).tobytes())
            f.write(np.ascontiguousarray(depth[i]).tobytes())
    args = [EXE, str(raw), str(len(bgr))] + ["%r" % float(cam[k]) for k in CAM_KEYS] + [mode]
    if pose0 is not None:
        pf = tmp_path / "pose0.f32"
        pf.write_bytes(np.ascontiguousarray(pose0, np.float32).tobytes())
        args.append(str(pf))
    args += [str(e) for e in extra]
    out = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    return [l.split() for l in out.stdout.strip().splitlines()]


def _rows(rows):
    """(b, ok, n_matches, n_inliers, pose f32 4x4) per frame line."""
    out = []
    for r in rows:
        pose = np.array([int(v, 16) for v in r[4:20]], np.uint32).view(np.float32).reshape(4, 4)
        out.append((int(r[0]), int(r[1]), int(r[2]), int(r[3]), pose))
    return out


@pytest.mark.parametrize("noise", [None, 3])
def test_refside_pnp_flag_chain_matches_oracle(oracle, tmp_path, noise):
    """The flag chain through the reference-side Matcher::match and PnPRansac::compute bodies, with F2's pose
    prior = F1's pose; noise = a noise frame in the chain (few matches into and out of it)."""
    B = 7
    bgr, depth, gt, cam = synth_seq(B, seed=71, preset="fr1")
    if noise is not None:
        bgr[noise] = np.random.RandomState(5).randint(0, 256, size=bgr[noise].shape).astype(np.uint8)
    pose0 = gt[0].astype(np.float32)
    got = _rows(_run(tmp_path, bgr, depth, cam, "pnp", pose0))
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(B)]
    K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
    wp, ws, wn, wm, _ = chain_model.pnp_track_flagged(oracle, frames, pose0, K4, 1, as_written=True)
    assert [g[0] for g in got] == list(range(1, B))
    for b, ok, nm, ni, pose in got:
        assert (ok, nm, ni) == (ws[b], wm[b], wn[b]), (b, ok, nm, ni, ws[b], wm[b], wn[b])
        assert np.array_equal(pose.view(np.uint32), wp[b].view(np.uint32)), b
    # as written, the object points are F2's own back-projection, so even the noise frame's pair is
    # self-consistent: what differs is the matches (and so the flags) around it
    assert ws[1:].all()


def test_refside_visual_odometry_matches_oracle(oracle, tmp_path):
    """Tracking::visualOdometry over the reference-side RansacSE3, Matcher and Gicp bodies (process-wide rand()
    stream seeded by Random::initSeed(2024), sticky depth covariance) against the oracle chain: status, inliers
    and the pose bits of every frame.  BASELINE config 3's setting (fr2 camera, 2000 keypoints through
    Extractor::setParameters), every third frame so RansacSE3's rmse reaches 0.8 and Gicp::compute runs, and a
    noise frame so the second reference and recover() run."""
    n = 8
    bgr, depth, gt, cam = synth_seq(3 * n - 2, seed=29, preset="fr2")
    bgr, depth = bgr[::3].copy(), depth[::3].copy()
    bgr[3] = np.random.RandomState(5).randint(0, 256, size=bgr[3].shape).astype(np.uint8)
    got = _rows(_run(tmp_path, bgr, depth, cam, "vo", extra=(2000,)))
    p, oc = oracle.orb_params(2000), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(n)]
    log = []
    wp, ws, wn, _, _ = chain_model.track(oracle, frames, np.eye(4, dtype=np.float32), 2024, log=log)
    assert [g[0] for g in got] == list(range(1, n))
    for b, ok, nm, ni, pose in got:
        assert (ok, ni) == (ws[b], wn[b]), (b, ok, ni, ws[b], wn[b])
        assert np.array_equal(pose.view(np.uint32), wp[b].view(np.uint32)), b
    assert any(g for _, g in log), log   # Gicp::compute ran (rmse >= 0.8)
    assert any(r for r, _ in log), log   # the second reference ran


def test_refside_detect_and_compute_keeps_descriptors(tmp_path):
    """Extractor::detectAndCompute's body returns exactly the Frame path's keypoints and descriptors (the rows
    it wrote, not a reallocated block), and releases the descriptors when no keypoint is found."""
    n = 3
    bgr, depth, gt, cam = synth_seq(n, seed=75, preset="fr1")
    rows = _run(tmp_path, bgr, depth, cam, "detect")
    det = [r for r in rows if r[0] == "detect"]
    assert len(det) == n
    for r in det:
        assert int(r[2]) > 500 and r[3] == "1" and r[4] == "1", r
    empty = [r for r in rows if r[0] == "empty"]
    assert empty == [["empty", "0", "1"]]


def _round_half_away(v):
    return np.where(v >= 0, np.floor(v + np.float32(0.5)), -np.floor(-v + np.float32(0.5)))


def _undistort_corners(cam):
    """cv::undistortPoints of the four image corners (Core/Frame.cpp:288-307; 5 iterations in double)."""
    fx, fy, cx, cy = (float(np.float32(cam[k])) for k in ("fx", "fy", "cx", "cy"))
    k = [float(np.float32(cam[n])) for n in ("k1", "k2", "p1", "p2", "k3")]
    out = []
    for u, v in ((0.0, 0.0), (640.0, 0.0), (0.0, 480.0), (640.0, 480.0)):
        x0 = (u - cx) * (1.0 / fx)
        y0 = (v - cy) * (1.0 / fy)
        x, y = x0, y0
        for _ in range(5):
            r2 = x * x + y * y
            icd = 1 / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
            dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x)
            dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y
            x = (x0 - dx) * icd
            y = (y0 - dy) * icd
        out.append((np.float32(fx * x + cx), np.float32(fy * y + cy)))
    return out


def _track_case(oracle, tmp_path, pg):
    """main.cpp's loop over the reference-side bodies: 20 frames (every 4th of an fr2 sequence, 2000 keypoints
    as BASELINE config 3) so that needKeyFrame fires several times and the PoseGraph thread has older keyframes
    within its 0.5 m radius to match."""
    n, step = 20, 4
    bgr, depth, gt, cam = synth_seq(step * (n - 1) + 1, seed=29, preset="fr2")
    bgr, depth = bgr[::step].copy(), depth[::step].copy()
    out = tmp_path / "out"
    out.mkdir()
    rows = _run(tmp_path, bgr, depth, cam, "track", extra=(2000, out, int(pg)))
    p, oc = oracle.orb_params(2000), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(n)]
    return rows, out, bgr, depth, cam, frames


def _check_track(oracle, rows, out, bgr, depth, cam, frames, pg):
    n = len(frames)
    sac = [r for r in rows if r[0] == "sac"]
    T_calls = [r for r in sac if r[2] == "T"]
    P_calls = [r for r in sac if r[2] == "P"]
    pending = list(P_calls)
    seen = {"t": 0, "p": 0}
    prm_pg = oracle.ransac_params(200, 30, 3.0, 4)

    def replay_pg(r, st, flags, upto):
        while pending and int(pending[0][1]) < upto:
            rec = pending.pop(0)
            i1, i2, nm, ok, ni = (int(v) for v in rec[3:8])
            z = lambda i: frames[i]["xyz"][:, 2]
            m = oracle.match(frames[i1]["desc"], frames[i2]["desc"], flags[i1], z(i1), z(i2), 0.9, True)
            assert len(m) == nm, (rec[:8], len(m))
            wok, T, inl, rm = oracle.ransac_se3(frames[i1]["xyz"], frames[i2]["xyz"], m, prm_pg, r, st, None)
            assert (ok, ni) == (int(wok), len(inl)), (rec[:8], wok, len(inl))
            assert int(rec[8], 16) == np.float32(rm).view(np.uint32), rec[:9]
            assert [int(v, 16) for v in rec[9:25]] == list(T.reshape(-1).view(np.uint32)), rec[:8]
            seen["p"] += 1

    def hook(r, st, flags):
        k = seen["t"]
        seen["t"] += 1
        replay_pg(r, st, flags, int(T_calls[k][1]))
        hook.flags = flags

    wp, ws, wn, rel, kflag, r, st = chain_model.track_kf(oracle, frames, np.eye(4, dtype=np.float32), 2024, hook=hook)
    replay_pg(r, st, hook.flags, 1 << 30)
    assert seen["t"] == len(T_calls) and seen["p"] == len(P_calls) and not pending
    # track()'s poses, keyframes and visualOdometry's statistics (mnMeanInliers = mnAcumInliers / id())
    trows = [r for r in rows if r[0] == "t"]
    assert [int(r[1]) for r in trows] == list(range(n))
    acc = 0
    for r in trows:
        b = int(r[1])
        acc += int(wn[b]) if b else 0
        assert int(r[2]) == int(kflag[b]), (b, r[2], kflag[b])
        assert (int(r[3]), int(r[4])) == ((acc // b, int(wn[b])) if b else (0, 0)), (b, r[3:5])
        pose = np.array([int(v, 16) for v in r[5:21]], np.uint32)
        assert np.array_equal(pose, wp[b].reshape(-1).view(np.uint32)), b
    assert int(kflag.sum()) >= 3, kflag
    # Frame members: ids, the grid statics and the grid, mvKeysColor, mImGray / mImDepth
    fr = {int(r[1]): r for r in rows if r[0] == "frame"}
    c = _undistort_corners(cam)
    minX, maxX = min(c[0][0], c[2][0]), max(c[1][0], c[3][0])
    minY, maxY = min(c[0][1], c[1][1]), max(c[2][1], c[3][1])
    invW, invH = np.float32(64) / np.float32(maxX - minX), np.float32(48) / np.float32(maxY - minY)
    bounds = [int(v, 16) for v in next(r for r in rows if r[0] == "bounds")[1:7]]
    assert bounds == [int(np.float32(v).view(np.uint32)) for v in (minX, maxX, minY, maxY, invW, invH)]
    for b in range(n):
        kps, kun = frames[b]["kps"], frames[b]["kps_un"]
        assert (int(fr[b][2]), int(fr[b][3])) == (b, len(kps))
        col = np.fromfile(out / ("f%d_color.u8" % b), np.uint8).reshape(-1, 3)
        assert np.array_equal(col, bgr[b][kps["y"].astype(np.int32), kps["x"].astype(np.int32)]), b
        gx = _round_half_away((kun["x"] - np.float32(minX)) * invW).astype(np.int64)
        gy = _round_half_away((kun["y"] - np.float32(minY)) * invH).astype(np.int64)
        inside = (gx >= 0) & (gx < 64) & (gy >= 0) & (gy < 48)
        want = []
        for i in range(64):
            for j in range(48):
                idx = np.nonzero(inside & (gx == i) & (gy == j))[0]
                want.append(len(idx))
                want.extend(idx.tolist())
        assert np.array_equal(np.fromfile(out / ("f%d_grid.i32" % b), np.int32), np.array(want, np.int32)), b
        if kflag[b]:   # createKeyFrame's cloud from mImColor / mImDepth
            got = np.fromfile(out / ("f%d_cloud.pts" % b), oracle.POINT_DTYPE)
            assert np.array_equal(got.view(np.uint8), oracle.keyframe_cloud(bgr[b], depth[b], cam).view(np.uint8)), b
        if b < 2:
            assert np.array_equal(np.fromfile(out / ("f%d_gray.u8" % b), np.uint8).reshape(480, 640), oracle.gray(bgr[b]))
            dimg = depth[b].astype(np.float32) * (np.float32(1.0) / np.float32(cam["factor"])) + np.float32(0.0)
            assert np.array_equal(np.fromfile(out / ("f%d_depth.f32" % b), np.float32).reshape(480, 640), dimg)
    # Tracking::initialize: one landmark per frame-0 keypoint with depth, at its 3D point, in mvKeysColor
    lm = np.fromfile(out / "lm.bin", np.uint8).reshape(-1, 16)
    xyz0, k0 = frames[0]["xyz"], frames[0]["kps"]
    sel = xyz0[:, 2] > 0
    assert int(next(r for r in rows if r[0] == "lm")[1]) == len(lm) == int(sel.sum())
    assert np.array_equal(lm[:, :12].copy().view(np.float32), xyz0[sel])
    assert np.array_equal(lm[:, 12:15], bgr[0][k0["y"].astype(np.int32), k0["x"].astype(np.int32)][sel])
    ctx = int(next(r for r in rows if r[0] == "ctx")[1])
    return P_calls, [r for r in rows if r[0] == "pair"], ctx, hook.flags


def test_refside_tracking_frame_members(oracle, tmp_path):
    """Tracking::track over the reference-side Frame body: every member the callers read (mnId / id(),
    mvKeysColor, mImGray, mImDepth, the grid and its statics, the landmarks of initialize, the keyframe cloud
    createKeyFrame builds from mImColor / mImDepth) and track()'s poses, keyframes and inlier statistics equal
    the oracle's, bit for bit (Core/Frame.cpp:34-117, System/Tracking.cpp:39-256)."""
    rows, out, bgr, depth, cam, frames = _track_case(oracle, tmp_path, pg=False)
    P, pairs, ctx, _ = _check_track(oracle, rows, out, bgr, depth, cam, frames, pg=False)
    assert not P and not pairs and ctx == 1


def test_refside_posegraph_thread_own_context(oracle, tmp_path):
    """The PoseGraph thread (Solver/PoseGraph.cpp:59-155) matches keyframes and runs RansacSE3(..., false) on a
    device context of its own while the tracking thread keeps tracking: both threads' results equal the oracle,
    with their RansacSE3 draws replayed from the one process-wide rand() stream in the order they took it."""
    rows, out, bgr, depth, cam, frames = _track_case(oracle, tmp_path, pg=True)
    P, pairs, ctx, flags = _check_track(oracle, rows, out, bgr, depth, cam, frames, pg=True)
    assert ctx == 2, ctx                      # the tracking thread's and the PoseGraph thread's
    assert len(pairs) >= 1 and len(P) >= 1, (pairs, len(P))
    z = lambda i: frames[i]["xyz"][:, 2]
    for _, cur, kf, nm in pairs:              # every candidate's Matcher count (ref = the older keyframe)
        cur, kf = int(cur), int(kf)
        m = oracle.match(frames[kf]["desc"], frames[cur]["desc"], flags[kf], z(kf), z(cur), 0.9, True)
        assert len(m) == int(nm), (cur, kf, nm, len(m))

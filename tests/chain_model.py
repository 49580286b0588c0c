"""Oracle-driven restatements of the tracking chains the device runs (test infrastructure only):
Tracking::visualOdometry (System/Tracking.cpp:121-163, RansacSE3 -> second reference -> GICP) for
rgbd_track_batch, and the extract + match + PnPRansac benchmark chain for rgbd_pnp_track_*, with
independent pairs or with the reference's outlier-flag chain (Features/Matcher.cpp:125-128,
Solver/PnPRansac.cpp:31,51)."""
import numpy as np


def compose(A, B):
    """cv::Mat CV_32F product: double accumulation in k order (no FMA), one rounding."""
    A = np.asarray(A, np.float32).reshape(4, 4)
    B = np.asarray(B, np.float32).reshape(4, 4)
    C = np.zeros((4, 4), np.float32)
    for i in range(4):
        for j in range(4):
            s = 0.0
            for k in range(4):
                s += float(A[i, k]) * float(B[k, j])
            C[i, j] = np.float32(s)
    return C


def track(oracle, frames, pose0, seed, nnratio=0.9, prm=None, sticky=None, gicp=True, log=None):
    """Tracking::visualOdometry: match -> RansacSE3 -> second reference -> GICP when rmse >= 0.8 ->
    recover() (System/Tracking.cpp:121-163).  log (a list) receives (retried, gicp_ran) per frame b >= 1."""
    prm = prm or oracle.ransac_params()
    r = oracle.rng(seed)
    st = sticky or oracle.Sticky()
    B = len(frames)
    poses = np.zeros((B, 4, 4), np.float32)
    poses[0] = pose0
    status = np.zeros(B, np.int32)
    ninl = np.zeros(B, np.int32)
    status[0] = 1
    flags = [np.zeros(max(len(f["kps"]), 1), np.uint8) for f in frames]
    for b in range(1, B):
        ref = b - 1
        z = lambda i: frames[i]["xyz"][:, 2]
        m = oracle.match(frames[ref]["desc"], frames[b]["desc"], flags[ref], z(ref), z(b), nnratio, True)
        ok, T, inl, rm = oracle.ransac_se3(frames[ref]["xyz"], frames[b]["xyz"], m, prm, r, st, flags[b])
        retried = not ok
        if not ok:
            ref = max(b - 2, 0)
            m = oracle.match(frames[ref]["desc"], frames[b]["desc"], flags[ref], z(ref), z(b), nnratio, True)
            ok, T, inl, rm = oracle.ransac_se3(frames[ref]["xyz"], frames[b]["xyz"], m, prm, r, st, flags[b])
        if gicp and rm >= 0.8:   # Gicp(pRefFrame, cur, sac.mvInliers, sac.mT21), 0.07 / 10
            src = frames[ref]["xyz"][inl["queryIdx"]] if len(inl) else np.zeros((0, 3), np.float32)
            tgt = frames[b]["xyz"][inl["trainIdx"]] if len(inl) else np.zeros((0, 3), np.float32)
            ok, T = oracle.gicp_compute(src, tgt, T)
        if log is not None:
            log.append((retried, gicp and rm >= 0.8))
        poses[b] = compose(T, poses[ref]) if ok else poses[b - 1]
        status[b] = int(ok)
        ninl[b] = len(inl)
    return poses, status, ninl, r, st


def pose_inverse(T):
    """Frame::getPoseInverse (Core/Frame.cpp:137-153): [R^T | -R^T t], the translation one cv::gemm
    (GEMM_1_T, alpha -1; double accumulation in k order, one rounding)."""
    T = np.asarray(T, np.float32).reshape(4, 4)
    Ti = np.eye(4, dtype=np.float32)
    for i in range(3):
        s = 0.0
        for k in range(3):
            s += float(T[k, i]) * float(T[k, 3])
        for j in range(3):
            Ti[i, j] = T[j, i]
        Ti[i, 3] = np.float32(s * -1.0)
    return Ti


def need_keyframe(Tcur, Tkf):
    """Tracking::needKeyFrame (System/Tracking.cpp:201-225) in the reference's float / double mix:
    cv::norm of the float translation (double sums), acos(0.5 * (R00 + R11 + R22 - 1.0)) with the three
    float entries added in float; a NaN angle compares false."""
    import math
    d = compose(pose_inverse(Tcur), Tkf)
    tn = math.sqrt((float(d[0, 3]) * float(d[0, 3]) + float(d[1, 3]) * float(d[1, 3])) + float(d[2, 3]) * float(d[2, 3]))
    tr = np.float32(np.float32(d[0, 0] + d[1, 1]) + d[2, 2])
    c = 0.5 * (float(tr) - 1.0)
    rn = math.acos(c) if -1.0 <= c <= 1.0 else float("nan")
    return tn > 0.20 or rn > 0.1745


def track_kf(oracle, frames, pose0, seed, nnratio=0.9, prm=None, sticky=None, gicp=True, log=None, hook=None):
    """Tracking::track (System/Tracking.cpp:39-73) from initialize(): visualOdometry as `track`, then
    updateLastFrame (:242-247), mpReferenceKF, needKeyFrame / createKeyFrame (:201-240) and
    updateRelativePose (:249-256).  Returns track()'s poses, status, inliers, the relative poses and the
    keyframe flags (rgbd_track_batch_kf from a zeroed state).  hook(r, st, flags), when given, runs before
    every RansacSE3 draw of the chain (another thread's draws from the same stream, replayed in order)."""
    prm = prm or oracle.ransac_params()
    r = oracle.rng(seed)
    st = sticky or oracle.Sticky()
    B = len(frames)
    P = [None] * B                       # every frame's current pose (Frame::mTcw)
    P[0] = np.asarray(pose0, np.float32).reshape(4, 4).copy()
    out = np.zeros((B, 4, 4), np.float32)
    out[0] = P[0]
    rel = np.zeros((B, 4, 4), np.float32)
    kfo = [0] * B
    kflag = np.zeros(B, np.int32)
    kf = 0                               # initialize(): frame 0 is the first keyframe
    kflag[0] = 1
    rel[0] = compose(P[0], pose_inverse(P[0]))
    status = np.zeros(B, np.int32)
    ninl = np.zeros(B, np.int32)
    status[0] = 1
    flags = [np.zeros(max(len(f["kps"]), 1), np.uint8) for f in frames]
    z = lambda i: frames[i]["xyz"][:, 2]
    pre = (lambda: hook(r, st, flags)) if hook else (lambda: None)
    for b in range(1, B):
        ref = b - 1
        m = oracle.match(frames[ref]["desc"], frames[b]["desc"], flags[ref], z(ref), z(b), nnratio, True)
        pre()
        ok, T, inl, rm = oracle.ransac_se3(frames[ref]["xyz"], frames[b]["xyz"], m, prm, r, st, flags[b])
        retried = not ok
        if not ok:
            ref = max(b - 2, 0)          # mpRefFrame.second, re-anchored by the previous updateLastFrame
            m = oracle.match(frames[ref]["desc"], frames[b]["desc"], flags[ref], z(ref), z(b), nnratio, True)
            pre()
            ok, T, inl, rm = oracle.ransac_se3(frames[ref]["xyz"], frames[b]["xyz"], m, prm, r, st, flags[b])
        if gicp and rm >= 0.8:
            src = frames[ref]["xyz"][inl["queryIdx"]] if len(inl) else np.zeros((0, 3), np.float32)
            tgt = frames[b]["xyz"][inl["trainIdx"]] if len(inl) else np.zeros((0, 3), np.float32)
            ok, T = oracle.gicp_compute(src, tgt, T)
        if log is not None:
            log.append((retried, gicp and rm >= 0.8))
        P[b] = compose(T, P[ref]) if ok else P[b - 1].copy()
        status[b] = int(ok)
        ninl[b] = len(inl)
        P[b - 1] = compose(rel[b - 1], P[kfo[b - 1]])     # updateLastFrame
        kfo[b] = kf
        if need_keyframe(P[b], P[kf]):
            kf = kfo[b] = b
            kflag[b] = 1
        rel[b] = compose(P[b], pose_inverse(P[kfo[b]]))   # updateRelativePose
        out[b] = P[b]
    return out, status, ninl, rel, kflag, r, st


def pnp_pair(oracle, f1, f2, K4, nnratio=0.9, iters=500, reproj=3.0, conf=0.85, min_matches=10):
    """Matcher::match(F1, F2, m, discardOutliers=false) + PnPRansac with F1's 3D and F2's undistorted
    pixels (the rgbd_pnp_track_batch definition).  Returns (ok, T21 f32 4x4, n_inliers, n_matches)."""
    n1 = len(f1["kps"])
    m = oracle.match(f1["desc"], f2["desc"], np.zeros(max(n1, 1), np.uint8), f1["xyz"][:, 2], f2["xyz"][:, 2],
                     nnratio, False)
    if len(m) < min_matches:
        return False, np.eye(4, dtype=np.float32), 0, len(m)
    p3 = f1["xyz"][m["queryIdx"]]
    ku = f2["kps_un"][m["trainIdx"]]
    p2 = np.stack([ku["x"], ku["y"]], 1).astype(np.float32)
    ok, R, t, mask, ni, it = oracle.pnp_ransac(p3, p2, K4, iters, reproj, conf)
    T = np.eye(4, dtype=np.float32)
    if ok:
        T[:3, :3] = R.astype(np.float32)
        T[:3, 3] = t.astype(np.float32)
    return ok, T, (ni if ok else 0), len(m)


def pnp_track(oracle, frames, pose0, K4, nnratio=0.9, **kw):
    B = len(frames)
    poses = np.zeros((B, 4, 4), np.float32)
    poses[0] = pose0
    status, ninl, nm = (np.zeros(B, np.int32) for _ in range(3))
    status[0] = 1
    for b in range(1, B):
        ok, T, ni, m = pnp_pair(oracle, frames[b - 1], frames[b], K4, nnratio, **kw)
        poses[b] = compose(T, poses[b - 1]) if ok else poses[b - 1]
        status[b], ninl[b], nm[b] = int(ok), ni, m
    return poses, status, ninl, nm


def segment_starts(P, segments):
    """First pair of each of the S contiguous runs rgbd_pnp_track_* splits the B-1 pairs into."""
    S = max(1, min(segments, P))
    return {(P * k) // S for k in range(S)}


def unproject_world(Tcw, x):
    """Frame::unprojectWorld (Core/Frame.cpp:317-327) with updatePoseMatrices' float members (:137-147):
    mOw = -mRcw^T mtcw (gemm, double sums, one rounding), then mRwc x + mOw as one gemm (double sums,
    + the float C term, one rounding)."""
    T = np.asarray(Tcw, np.float32)
    out = np.zeros(3, np.float32)
    for r in range(3):
        o = 0.0
        for k in range(3):
            o += float(T[k, r]) * float(T[k, 3])
        Ow = np.float32(o * -1.0)
        a = 0.0
        for k in range(3):
            a += float(T[k, r]) * float(x[k])
        out[r] = np.float32(a * 1.0 + float(Ow) * 1.0)
    return out


def pnp_track_flagged(oracle, frames, pose0, K4, segments=1, nnratio=0.9, iters=500, reproj=3.0, conf=0.85,
                      min_matches=10, as_written=False):
    """The reference's flag chain: Matcher::match(F1, F2, m) with discardOutliers = true (flagged queries
    of F1 skipped, Features/Matcher.cpp:125-128), then PnPRansac::compute sets every matched trainIdx of
    F2 outlier (Solver/PnPRansac.cpp:31) and the RANSAC inliers inlier again (:51); < min_matches
    matches return before any flag is written (:16-17).  Pairs split into `segments` runs whose first
    pair reads a fresh (cleared) frame.  Returns poses, status, n_inliers, n_matches and the masks.
    as_written: PnPRansac::compute as the reference has it -- object points = F2's own unprojectWorld under
    F2's pose prior (F1's pose), F2's pose = toHomogeneous = [float(R) | float(t)] instead
    of F1's 3D points and T composed with F1's pose (the batched path's pairing)."""
    B = len(frames)
    P = B - 1
    starts = segment_starts(P, segments) if P > 0 else set()
    poses = np.zeros((B, 4, 4), np.float32)
    poses[0] = pose0
    status, ninl, nm = (np.zeros(B, np.int32) for _ in range(3))
    status[0] = 1
    flags = [np.zeros(max(len(f["kps"]), 1), np.uint8) for f in frames]
    masks = [None] * B
    for b in range(1, B):
        f1, f2 = frames[b - 1], frames[b]
        if b - 1 in starts:
            flags[b - 1][:] = 0
        m = oracle.match(f1["desc"], f2["desc"], flags[b - 1], f1["xyz"][:, 2], f2["xyz"][:, 2], nnratio, True)
        nm[b] = len(m)
        ok, T = False, np.eye(4, dtype=np.float32)
        if len(m) >= min_matches:
            if as_written:
                p3 = np.stack([unproject_world(poses[b - 1], f2["xyz"][j]) for j in m["trainIdx"]]).astype(np.float32)
            else:
                p3 = f1["xyz"][m["queryIdx"]]
            ku = f2["kps_un"][m["trainIdx"]]
            p2 = np.stack([ku["x"], ku["y"]], 1).astype(np.float32)
            ok, R, t, mask, ni, it = oracle.pnp_ransac(p3, p2, K4, iters, reproj, conf)
            flags[b][m["trainIdx"]] = 1
            if ok:
                flags[b][m["trainIdx"][mask]] = 0
                T[:3, :3] = R.astype(np.float32)
                T[:3, 3] = t.astype(np.float32)
                ninl[b] = ni
                masks[b] = mask
        poses[b] = (T if as_written else compose(T, poses[b - 1])) if ok else poses[b - 1]
        status[b] = int(ok)
    return poses, status, ninl, nm, masks

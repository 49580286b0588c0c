"""Oracle-driven restatement of Tracking::visualOdometry (System/Tracking.cpp:121-163) without GICP,
used to check rgbd_track_batch (test infrastructure only)."""
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


def track(oracle, frames, pose0, seed, nnratio=0.9, prm=None, sticky=None, gicp=True):
    """Tracking::visualOdometry: match -> RansacSE3 -> second reference -> GICP when rmse >= 0.8 ->
    recover() (System/Tracking.cpp:121-163)."""
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
        if not ok:
            ref = max(b - 2, 0)
            m = oracle.match(frames[ref]["desc"], frames[b]["desc"], flags[ref], z(ref), z(b), nnratio, True)
            ok, T, inl, rm = oracle.ransac_se3(frames[ref]["xyz"], frames[b]["xyz"], m, prm, r, st, flags[b])
        if gicp and rm >= 0.8:   # Gicp(pRefFrame, cur, sac.mvInliers, sac.mT21), 0.07 / 10
            src = frames[ref]["xyz"][inl["queryIdx"]] if len(inl) else np.zeros((0, 3), np.float32)
            tgt = frames[b]["xyz"][inl["trainIdx"]] if len(inl) else np.zeros((0, 3), np.float32)
            ok, T = oracle.gicp_compute(src, tgt, T)
        poses[b] = compose(T, poses[ref]) if ok else poses[b - 1]
        status[b] = int(ok)
        ninl[b] = len(inl)
    return poses, status, ninl, r, st


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

"""Oracle-driven restatement of Tracking::visualOdometry (System/Tracking.cpp:121-163) without GICP,
used to check rgbd_track_batch (test infrastructure only)."""
import numpy as np


def compose(A, B):
    """cv::Mat CV_32F product: double accumulation in k order, one rounding."""
    return (A.astype(np.float64) @ B.astype(np.float64)).astype(np.float32)


def track(oracle, frames, pose0, seed, nnratio=0.9, prm=None, sticky=None):
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
        poses[b] = compose(T, poses[ref]) if ok else poses[b - 1]
        status[b] = int(ok)
        ninl[b] = len(inl)
    return poses, status, ninl, r, st

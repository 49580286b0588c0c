"""Tracking over a whole dataset sequence (the main.cpp / Tracking loop of the reference, for this
path): frames are read from a TUM / ICL directory (datasets.py), uploaded in batches of B frames that
overlap by one frame, and chained through the device front end:

  * solver "pnp": extract + Matcher + PnPRansac per consecutive pair (the benchmark chain), pipelined
    with rgbd_pnp_track_submit / collect (three batches in flight); batch k+1 starts at the last
    frame of batch k and takes its pose, so the chain equals one batch over the whole sequence.
  * solver "se3": Tracking::track -- visualOdometry's RansacSE3 (+ GICP when rmse >= 0.8) chain with
    updateLastFrame / keyframes / relative poses (rgbd_track_batch_kf), synchronous; the RNG, the
    RansacSE3 sticky covariance and the keyframe state carry over between batches.  The outlier flags of a batch's first frame are not carried over (as for the chunks of
    rgbd-slam_amd/dist.py), and the second-reference retry of a batch's second frame (Tracking.cpp:
    134-143, frame b-2) uses the batch's first frame, not the previous batch's second-to-last one.

Returns the camera poses Tcw of every frame; write_tum_trajectory stores them in the reference's
trajectory format (System/Tracking.cpp:286-317).  Keyframe bookkeeping (poses relative to the last
keyframe) is the caller's, as in the reference's Tracking.
"""
from __future__ import annotations

import numpy as np


def batch_starts(n: int, B: int):
    """First frame of each batch: batches [s, s + B) overlap by one frame, the last may be shorter."""
    if B < 2:
        raise ValueError(f"batch size must be at least 2 (batches overlap by one frame), not {B}")
    if n <= 1:
        return [0] if n == 1 else []
    return list(range(0, n - 1, B - 1))


def track_sequence(pkg, ds, B: int = 64, solver: str = "pnp", nfeatures: int = 1000, nnratio: float = 0.9,
                   pose0=None, device: int = 0, max_frames: int | None = None, threads: int = 8, extras=None):
    """Poses Tcw [n, 4, 4] f32, per-frame status [n] (1: tracked / first frame) and inliers [n].  With
    solver "se3" and a dict `extras`, also the relative poses ('rel') and keyframe flags ('keyframe') of
    Tracking's bookkeeping (for datasets.camera_trajectory_poses)."""
    import torch
    if B < 2:
        raise ValueError(f"batch size must be at least 2 (batches overlap by one frame), not {B}")
    n = len(ds) if max_frames is None else min(len(ds), max_frames)
    cam = ds.camera
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    ctx = pkg.Context(ds.W, ds.H, max_batch=B, orb=pkg.orb_params(nfeatures), cam=c, device=device)
    dev = torch.device("cuda", device)
    poses = np.zeros((n, 4, 4), np.float32)
    status = np.zeros(n, np.int32)
    ninl = np.zeros(n, np.int32)
    p0 = np.eye(4, dtype=np.float32) if pose0 is None else np.asarray(pose0, np.float32)
    if n == 0:
        ctx.close()
        return poses, status, ninl
    poses[0], status[0] = p0, 1
    starts = batch_starts(n, B)

    def upload(s):
        cnt = min(B, n - s)
        bgr, dep, _ = ds.load(s, cnt, threads=threads)
        return (torch.from_numpy(bgr).to(dev), torch.from_numpy(dep.view(np.int16)).to(dev), cnt)

    try:
        if solver == "pnp":
            prm = pkg.pnp_params(500, 3.0, 0.85, 10)   # Solver/PnPRansac.cpp:39
            inflight = []                               # (start, device frames) in submission order
            nxt = 0
            for k, s in enumerate(starts):
                while nxt < len(starts) and len(inflight) < 3:
                    fr = upload(starts[nxt])
                    ctx.pnp_track_submit(fr[0].data_ptr(), fr[1].data_ptr(), fr[2], nnratio, prm)
                    inflight.append((starts[nxt], fr))
                    nxt += 1
                s0, fr = inflight.pop(0)
                pb, sb, ib, _ = ctx.pnp_track_collect(poses[s0])
                poses[s0:s0 + fr[2]] = pb
                status[s0 + 1:s0 + fr[2]] = sb[1:]
                ninl[s0 + 1:s0 + fr[2]] = ib[1:]
        elif solver == "se3":
            prm = pkg.ransac_params(200, 10, 3.0, 4)   # RansacSE3(200, 10, 3.0f, 4), System/Tracking.cpp:129
            rng = pkg.rng(0)
            sticky = pkg.Sticky()
            state = pkg.TrackState()                     # Tracking's keyframe bookkeeping, carried on
            rel = np.zeros((n, 4, 4), np.float32)
            kf = np.zeros(n, np.int32)
            for s in starts:
                fr = upload(s)
                pb, sb, ib, rb, kb = ctx.track_batch_kf(fr[0].data_ptr(), fr[1].data_ptr(), fr[2], nnratio, prm, rng,
                                                        sticky, state, poses[s])
                rel[s:s + fr[2]] = rb
                kf[s:s + fr[2]] = kb
                poses[s:s + fr[2]] = pb
                status[s + 1:s + fr[2]] = sb[1:]
                ninl[s + 1:s + fr[2]] = ib[1:]
            if extras is not None:
                extras["rel"], extras["keyframe"] = rel, kf
        else:
            raise ValueError(f"solver must be 'pnp' or 'se3', not {solver!r}")
    finally:
        ctx.close()
    return poses, status, ninl

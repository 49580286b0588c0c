"""Tracking over a whole dataset sequence (the main.cpp / Tracking loop of the reference, for this
path): frames are read from a TUM / ICL directory (datasets.py), uploaded in batches of B frames that
overlap by one frame, and chained through the device front end:

  * solver "pnp": extract + Matcher + PnPRansac per consecutive pair (the benchmark chain), pipelined
    with rgbd_pnp_track_submit / collect (three batches in flight); batch k+1 starts at the last
    frame of batch k and takes its pose, so the chain equals one batch over the whole sequence.
  * solver "se3": Tracking::track -- visualOdometry's RansacSE3 (+ GICP when rmse >= 0.8) chain with
    updateLastFrame / keyframes / relative poses (rgbd_track_batch_kf), synchronous; the RNG, the
    RansacSE3 sticky covariance and the keyframe state carry over between batches, which overlap by two
    frames so that the second-reference retry and the outlier flags continue exactly (the chain equals one
    batch over the sequence, rgbd_track_state).

Returns the camera poses Tcw of every frame (track()'s returns); with solver "se3" the relative poses
and keyframe flags too (extras), from which datasets.camera_trajectory_poses composes the trajectory
System/Tracking.cpp:286-317 writes.
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
    if B < 2 or (solver == "se3" and B < 3):
        raise ValueError(f"batch size must be at least 2 (pnp: batches overlap by one frame) or 3 (se3: by two), not {B}")
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
            state = pkg.track_state(ctx.kp_cap)          # Tracking's state, carried on
            rel = np.zeros((n, 4, 4), np.float32)
            kf = np.zeros(n, np.int32)
            # batches overlap by two frames (mpRefFrame.second and .first of the next one), so the chain
            # over the whole sequence is the single-batch chain bit for bit
            s = 0
            while True:
                fr = upload(s)
                k0 = 2 if state.valid else 1
                pb, sb, ib, rb, kb = ctx.track_batch_kf(fr[0].data_ptr(), fr[1].data_ptr(), fr[2], nnratio, prm, rng,
                                                        sticky, state, poses[s + k0 - 1])
                if k0 == 1:
                    rel[s], kf[s] = rb[0], kb[0]
                rel[s + k0:s + fr[2]] = rb[k0:]
                kf[s + k0:s + fr[2]] = kb[k0:]
                poses[s + k0:s + fr[2]] = pb[k0:]
                status[s + k0:s + fr[2]] = sb[k0:]
                ninl[s + k0:s + fr[2]] = ib[k0:]
                if s + fr[2] >= n:
                    break
                s += B - 2
            if extras is not None:
                extras["rel"], extras["keyframe"] = rel, kf
        else:
            raise ValueError(f"solver must be 'pnp' or 'se3', not {solver!r}")
    finally:
        ctx.close()
    return poses, status, ninl

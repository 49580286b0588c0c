"""Whole-sequence tracking from a TUM-layout directory (rgbd-slam_amd/sequence.py): batches overlap by
one frame and are chained, three in flight, so the result equals one batch over the whole sequence."""
import os

import numpy as np
import pytest

from conftest import synth_seq

pytestmark = pytest.mark.gpu


def test_sequence_pnp_equals_one_batch(pkg, tmp_path):
    import torch
    from rgbd_slam_amd import datasets as D
    from rgbd_slam_amd.sequence import track_sequence
    import ate
    n = 13
    bgr, depth, gt, cam = synth_seq(n, seed=41, preset="fr1")
    base = str(tmp_path / "rgbd_dataset_freiburg1_seq") + os.sep
    times = 100.0 + 0.033 * np.arange(n)
    D.write_dataset(base, bgr, depth, times, gt)
    ds = D.open_dataset(base)
    poses, status, ninl = track_sequence(pkg, ds, B=5, solver="pnp", pose0=gt[0])   # batches 0-4, 4-8, 8-12
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=n, orb=pkg.orb_params(1000), cam=c)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    wp, ws, wn, _ = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), n, 0.9, pkg.pnp_params(500, 3.0, 0.85, 10),
                                        gt[0].astype(np.float32))
    ctx.close()
    assert np.array_equal(poses.view(np.uint32), wp.view(np.uint32))
    assert np.array_equal(status, ws) and np.array_equal(ninl, wn)
    assert ate.ate_rmse(poses, gt) < 0.03
    out = str(tmp_path / "traj.txt")
    D.write_tum_trajectory(out, times, poses)
    t2, Twc = D.read_tum_trajectory(out)
    assert len(t2) == n and np.allclose(np.linalg.inv(Twc), poses, atol=1e-5)


def test_sequence_se3_runs(pkg, tmp_path):
    from rgbd_slam_amd import datasets as D
    from rgbd_slam_amd.sequence import track_sequence
    import ate
    n = 9
    bgr, depth, gt, _ = synth_seq(n, seed=43, preset="fr3")
    base = str(tmp_path / "rgbd_dataset_freiburg3_seq") + os.sep
    D.write_dataset(base, bgr, depth, np.arange(n) * 0.033, gt)
    extras = {}
    poses, status, _ = track_sequence(pkg, D.open_dataset(base), B=5, solver="se3", pose0=gt[0], extras=extras)
    assert status.all()
    assert ate.ate_rmse(poses, gt) < 0.05
    # Tracking's bookkeeping across the two overlapping batches: frame 0 is the first keyframe, and the
    # trajectory saveCameraTrajectory would write (relative to it) aligns to the ground truth as well
    assert extras["keyframe"][0] == 1 and extras["rel"].shape == (n, 4, 4)
    traj = D.camera_trajectory_poses(extras["rel"], extras["keyframe"], poses)
    assert np.allclose(traj[0], np.eye(4), atol=1e-5)
    assert ate.ate_rmse(traj, gt) < 0.05


def test_posegraph_over_tracked_sequence(pkg):
    """Keyframes of a tracked 80-frame sequence, local edges from the device Matcher + RansacSE3,
    host LM: more than 5 vertices, local edges beyond the reference chain, chi2 not increased, and
    the corrected trajectory stays on the ground truth."""
    import torch
    from rgbd_slam_amd.posegraph import posegraph_sequence
    import ate
    n = 80
    bgr, depth, gt, cam = synth_seq(n, seed=51, preset="fr1")
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=n, orb=pkg.orb_params(1000), cam=c)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    poses, status, _, _ = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), n, 0.9, pkg.pnp_params(),
                                              gt[0].astype(np.float32))
    ctx.close()
    corrected, kfs, (v, e, c0, c1) = posegraph_sequence(pkg, lambda i: (bgr[i], depth[i]), cam, poses)
    assert v == len(kfs) > 5 and e > v - 1
    assert c1 <= c0 + 1e-12
    assert ate.ate_rmse(corrected, gt) < 0.05
    assert np.allclose(corrected[kfs[0]], poses[kfs[0]])        # vertex 0 is fixed

"""GPU parity: the tracking front-end chain over a device-resident batch (rgbd_track_batch) vs an
oracle-driven restatement of Tracking::visualOdometry without GICP (tests/chain_model.py)."""
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

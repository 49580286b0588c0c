"""GPU parity for BASELINE config 5 (CORBS camera, pose-graph hand-off after tracking):

  * extraction and the extract + match + PnPRansac chain on the CORBS camera preset
    (IO/DatasetCORBS.cpp:36-37: fx 468.6, fy 468.61, cx 318.27, cy 243.99, no distortion, factor 5000)
    bit-exact against the oracle;
  * the pose graph's local edges (PoseGraph::createLocalEdges, Solver/PoseGraph.cpp:128-155): the device
    Matcher(0.9) + RansacSE3(200, 30, 3.0f, 4) with updateF2 = false, edge for edge against the oracle
    chain (matches, ok, T21 bits, inliers, rmse, the RNG state and the sticky depth covariance after each);
  * the pose graph's LM (rgbd_pg_optimize) over exactly that graph against the numpy restatement
    oracle/posegraph_ref.py (g2o absent: parity unpinned against g2o itself; tolerance stated below).
"""
import os
import sys

import numpy as np
import pytest

from conftest import synth_seq
import chain_model

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def _cam(pkg, cam):
    return pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                      cam["k3"], cam["factor"])


def test_corbs_frame_bit_exact(pkg, oracle):
    bgr, depth, _, cam = synth_seq(3, seed=41, preset="corbs")
    assert cam["fx"] == np.float32(468.6) or abs(cam["fx"] - 468.6) < 1e-4
    ctx = pkg.Context(640, 480, max_batch=1, orb=pkg.orb_params(1000), cam=_cam(pkg, cam))
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    for f in range(3):
        got = ctx.frame(bgr[f], depth[f])
        want = oracle.frame(bgr[f], depth[f], p, oc)
        assert len(got["kps"]) == len(want["kps"]) > 500
        for fld in ("x", "y", "size", "angle", "response", "octave"):
            assert np.array_equal(got["kps"][fld].view(np.uint32), want["kps"][fld].view(np.uint32)), fld
        assert np.array_equal(got["desc"], want["desc"])
        assert np.array_equal(got["kps_un"].view(np.uint32), want["kps_un"].view(np.uint32))
        assert np.array_equal(got["xyz"].view(np.uint32), want["xyz"].view(np.uint32))
    ctx.close()


def test_corbs_pnp_track_batch_matches_oracle_chain(pkg, oracle):
    import torch
    B = 8
    bgr, depth, gt, cam = synth_seq(B, seed=43, preset="corbs")
    ctx = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(1000), cam=_cam(pkg, cam))
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pose0 = gt[0].astype(np.float32)
    poses, status, ninl, nm = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, pkg.pnp_params(), pose0)
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(B)]
    K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
    wp, ws, wn, wm = chain_model.pnp_track(oracle, frames, pose0, K4)
    assert np.array_equal(nm, wm) and np.array_equal(status, ws) and np.array_equal(ninl, wn)
    assert np.array_equal(poses.view(np.uint32), wp.view(np.uint32))
    assert status.all()
    ctx.close()


def _tracked_corbs(pkg, n, seed):
    import torch
    bgr, depth, gt, cam = synth_seq(n, seed=seed, preset="corbs")
    ctx = pkg.Context(640, 480, max_batch=n, orb=pkg.orb_params(1000), cam=_cam(pkg, cam))
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    poses, status, _, _ = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), n, 0.9, pkg.pnp_params(),
                                              gt[0].astype(np.float32))
    ctx.close()
    return bgr, depth, gt, cam, poses


def test_posegraph_local_edges_and_lm_match_oracle(pkg, oracle):
    """createLocalEdges on the device vs the oracle chain, then the LM over the same graph vs
    posegraph_ref.  Tolerance for the LM: the optimum's vertices within 1e-7 (absolute, Twc entries) and
    chi2 within 1e-6 relative -- near the optimum the accept / reject decisions of the lambda schedule
    turn on rounding, so the two implementations may stop a few iterations apart at the same optimum."""
    from rgbd_slam_amd.posegraph import posegraph_sequence, MATCHES_TH
    import posegraph_ref as REF
    import ate
    n = 90
    bgr, depth, gt, cam, poses = _tracked_corbs(pkg, n, seed=47)
    rec = {}
    corrected, kfs, (v, e, c0, c1) = posegraph_sequence(pkg, lambda i: (bgr[i], depth[i]), cam, poses, record=rec)
    assert v == len(kfs) > 5
    att = rec["attempts"]
    assert sum(1 for a in att if a[3] is not None and a[3]["ok"]) >= 3, "too few local edges to pin"
    # ---- the oracle chain over the same keyframes: features, Matcher(0.9), RansacSE3(200, 30, 3, 4, updateF2=false)
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    feats = {k: oracle.frame(bgr[k], depth[k], p, oc) for k in kfs}
    for k in kfs:   # the graph's features are the device's extraction, bit-exact with the oracle's
        assert np.array_equal(rec["features"][k]["desc"], feats[k]["desc"])
        assert np.array_equal(rec["features"][k]["xyz"].view(np.uint32), feats[k]["xyz"].view(np.uint32))
    orng, ost = oracle.rng(0), oracle.Sticky()
    oprm = oracle.ransac_params(200, MATCHES_TH, 3.0, 4)
    for kid, cur, m, res in att:
        fk, fc = feats[kid], feats[cur]
        mw = oracle.match(fk["desc"], fc["desc"], np.zeros(len(fk["desc"]), np.uint8), fk["xyz"][:, 2],
                          fc["xyz"][:, 2], 0.9)
        assert np.array_equal(m, mw), (kid, cur)
        if len(mw) < MATCHES_TH:
            assert res is None
            continue
        ok, T, inl, rmse = oracle.ransac_se3(fk["xyz"], fc["xyz"], mw, oprm, orng, ost)   # updateF2 = false
        assert res["ok"] == ok, (kid, cur)
        assert np.array_equal(res["T21"].view(np.uint32), np.asarray(T, np.float32).view(np.uint32)), (kid, cur)
        assert np.array_equal(res["inliers"], inl) and np.float32(res["rmse"]) == np.float32(rmse)
        assert res["rng"] == list(orng.state) + [orng.f, orng.r]
        assert res["sticky"] == (ost.cov, ost.set)
    # ---- LM over the recorded graph vs the numpy restatement (vertices as the optimiser holds them:
    # VertexSE3 keeps an Isometry3d, i.e. the float Tcw's inverse re-orthonormalised)
    X0 = rec["vertices"]
    for k in kfs:
        assert np.allclose(X0[k], np.linalg.inv(np.asarray(poses[k], np.float32).astype(np.float64)), atol=1e-6)
    edges = [REF.make_edge(X0, f, t, Z) for f, t, Z in rec["edges"]]
    assert len(edges) == e
    assert c0 == pytest.approx(REF.total_chi2(edges, X0), rel=1e-12)
    Xr, chir, _ = REF.optimize(X0, {kfs[0]}, edges, 10)
    assert c1 == pytest.approx(chir, rel=1e-6, abs=1e-9)
    for k in kfs:   # corrected keyframe poses (Tcw = Twc^-1 cast to float)
        want = np.linalg.inv(Xr[k]).astype(np.float32)
        assert np.allclose(corrected[k], want, atol=1e-6), k
    assert c1 <= c0 + 1e-12
    assert ate.ate_rmse(corrected, gt) < 0.05

"""GPU: the C++ drop-in surfaces (include/rgbd/frontend.hpp) driven by a Tracking-style loop
(examples/track_example.cpp) reproduce the oracle chain exactly."""
import os
import subprocess

import numpy as np
import pytest

import chain_model
from conftest import ROOT, synth_seq

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("extractor", ["orb", "svo"])
def test_cpp_tracking_loop_matches_oracle(oracle, tmp_path, extractor):
    exe = os.path.join(ROOT, "rgbd-slam_amd", "build", "track_example")
    assert os.path.exists(exe), "build() must compile examples/track_example.cpp"
    n = 5
    bgr, depth, gt, cam = synth_seq(n, seed=13, preset="fr1")
    raw = tmp_path / "seq.raw"
    with open(raw, "wb") as f:
        for i in range(n):
            f.write(np.ascontiguousarray(bgr[i]).tobytes())
            f.write(np.ascontiguousarray(depth[i]).tobytes())
    args = [exe, str(raw), str(n)] + ["%r" % float(cam[k]) for k in ("fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2",
                                                                       "k3", "factor")] + [extractor]
    out = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    rows = [l.split() for l in out.stdout.strip().splitlines()]
    assert len(rows) == n
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    if extractor == "svo":   # Extractor(SVO, BRIEF, NORMAL), main.cpp:31
        frames = [oracle.svo_frame(bgr[i], depth[i], oracle.svo_params(), oc) for i in range(n)]
    else:
        frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(n)]
    wp, ws, wn, _, _ = chain_model.track(oracle, frames, np.eye(4, dtype=np.float32), 2024)
    for i, r in enumerate(rows):
        assert int(r[1]) == ws[i] and int(r[2]) == wn[i]
        t = np.array([float(v) for v in r[3:6]], np.float32)
        assert np.array_equal(t, wp[i][:3, 3]), (i, t, wp[i][:3, 3])


_unproject_world = chain_model.unproject_world


@pytest.mark.parametrize("preset,seed", [("fr1", 61), ("corbs", 62)])
def test_pnp_ransac_as_written_matches_oracle(oracle, tmp_path, preset, seed):
    """PnPRansac::compute as the reference has it (Solver/PnPRansac.cpp:14-56) through the C++ surface
    (rgbd::PnPRansac(..., as_written = true), examples/pnp_as_written.cpp): object points = F2's own
    unprojectWorld under F2's pose, pixels = F2's mvKeysUn, outlier flags set then the inliers cleared, and
    F2's pose = Converter::toHomogeneous's Tcw = [float(R) | float(t)] (the CV_64F Rodrigues
    matrix and tvec copied into the fixed-type CV_32F ROIs of Tcw are converted in place by Mat::copyTo's
    convertTo branch; OpenCV semantics recalled, parity unpinned).  R, t (f64 bits), the pose bits, the
    inliers and the flags equal the oracle restatement's."""
    exe = os.path.join(ROOT, "rgbd-slam_amd", "build", "pnp_as_written")
    assert os.path.exists(exe), "build() must compile examples/pnp_as_written.cpp"
    bgr, depth, gt, cam = synth_seq(2, seed=seed, preset=preset)
    raw, pf = tmp_path / "pair.raw", tmp_path / "pose.f32"
    with open(raw, "wb") as f:
        for i in range(2):
            f.write(np.ascontiguousarray(bgr[i]).tobytes())
            f.write(np.ascontiguousarray(depth[i]).tobytes())
    pose2 = np.ascontiguousarray(gt[1], np.float32)
    pf.write_bytes(pose2.tobytes())
    args = [exe, str(raw), str(pf)] + ["%r" % float(cam[k]) for k in ("fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2",
                                                                        "k3", "factor")]
    out = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.strip().splitlines()
    ok_s, nm_s, ni_s = lines[0].split()
    R = np.array([int(v, 16) for v in lines[1].split()[1:]], np.uint64)
    t = np.array([int(v, 16) for v in lines[2].split()[1:]], np.uint64)
    pose = np.array([int(v, 16) for v in lines[3].split()[1:]], np.uint32)
    inl = [int(v) for v in lines[4].split()[1:]]
    nflags = int(lines[5].split()[1])
    # the oracle restatement
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    f1, f2 = (oracle.frame(bgr[i], depth[i], p, oc) for i in range(2))
    m = oracle.match(f1["desc"], f2["desc"], np.zeros(len(f1["kps"]), np.uint8), f1["xyz"][:, 2], f2["xyz"][:, 2],
                     0.9, True)
    assert int(nm_s) == len(m) >= 10
    p3 = np.stack([_unproject_world(pose2, f2["xyz"][j]) for j in m["trainIdx"]]).astype(np.float32)
    ku = f2["kps_un"][m["trainIdx"]]
    p2 = np.stack([ku["x"], ku["y"]], 1).astype(np.float32)
    K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
    ok, Rw, tw, mask, ni, it = oracle.pnp_ransac(p3, p2, K4)
    assert int(ok_s) == int(ok) == 1
    assert int(ni_s) == ni and inl == [int(q) for q in m["queryIdx"][mask.astype(bool)]]
    assert np.array_equal(R, Rw.reshape(9).view(np.uint64)) and np.array_equal(t, tw.view(np.uint64))
    Tw = np.eye(4, dtype=np.float32)   # toHomogeneous: eye(4) with [R | t] converted to float (saturate_cast)
    Tw[:3, :3] = Rw.reshape(3, 3).astype(np.float32)
    Tw[:3, 3] = tw.astype(np.float32)
    assert np.array_equal(pose, Tw.reshape(16).view(np.uint32))
    assert nflags == len(m) - ni
    # F2's own 3D under F2's pose is (up to rounding) where F2's camera sits: the solved pose is F2's Tcw
    Tsol = np.eye(4)
    Tsol[:3, :3] = Rw.reshape(3, 3)
    Tsol[:3, 3] = tw
    assert np.allclose(Tsol, gt[1], atol=2e-3)

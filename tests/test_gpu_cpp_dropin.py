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

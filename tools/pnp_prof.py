"""Stage profile of k_pnp_hyp (profiling build): RGBD_HIP_LIB=rgbd-slam_amd/build_prof/librgbd_hip.so."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_pkg  # noqa: E402
from pnp_cases import K_TUM, problem  # noqa: E402

pkg = load_pkg()
ctx = pkg.Context(640, 480, max_batch=2)
probs = [problem(430, 900 + i, outliers=0.2)[:2] for i in range(63)]
for rep in range(3):
    res = ctx.pnp_ransac_batch(probs, K_TUM, pkg.pnp_params(min_matches=0))
print("iters", [r["iters"] for r in res[:8]], file=sys.stderr)

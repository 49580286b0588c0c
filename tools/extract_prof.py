"""Stage profile of k_distribute (profiling build): RGBD_HIP_LIB=rgbd-slam_amd/build_prof/librgbd_hip.so."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_pkg  # noqa: E402
import synth  # noqa: E402
import torch  # noqa: E402

pkg = load_pkg()
bgr, depth, gt, cam = synth.sequence(64, seed=1000, preset="fr1")
c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"], cam["k3"],
               cam["factor"])
ctx = pkg.Context(640, 480, max_batch=64, orb=pkg.orb_params(1000), cam=c)
d_bgr = torch.from_numpy(bgr).cuda()
d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
for _ in range(3):
    ctx.extract_batch(d_bgr.data_ptr(), d_dep.data_ptr(), 64)
ctx.synchronize()

"""k_distribute per level and stage (profiling build: RGBD_HIP_LIB=rgbd-slam_amd/build_prof/librgbd_hip.so prints
[dist_prof] lines for levels 0-3 of frame 0 per extraction) with the register path on and off, plus the kernel's
HIP-event time per launch.  usage: python tools/dist_prof.py [B]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_pkg  # noqa: E402
import synth  # noqa: E402
import torch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
pkg = load_pkg()
U = 32
bgr, depth, gt, cam = synth.sequence(U, seed=1000, preset="fr1")
idx = np.arange(B) % U
c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"], cam["k3"],
               cam["factor"])
ctx = pkg.Context(640, 480, max_batch=B, cam=c, orb=pkg.orb_params(1000))
d_bgr = torch.from_numpy(bgr[idx]).cuda()
d_dep = torch.from_numpy(np.ascontiguousarray(depth[idx]).view(np.int16)).cuda()
for reg in (True, False):
    ctx.debug_quadtree_registers(reg)
    for _ in range(2):
        ctx.extract_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B)
    ctx.synchronize()
    ctx.reset_timing()
    ctx.set_timing(True)
    for _ in range(3):
        ctx.extract_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B)
    ctx.synchronize()
    t = ctx.timings()
    ctx.set_timing(False)
    print(json.dumps({"registers": reg, "frames": B,
                      "us_per_launch": {k: round(v[0] * 1e3 / max(v[1], 1), 1) for k, v in sorted(t.items())}}),
          flush=True)
    sys.stderr.flush()

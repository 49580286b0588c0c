"""Kernel times of the ORB extraction alone (64 frames per batch, HIP events per kernel)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
from conftest import load_pkg  # noqa: E402
import synth  # noqa: E402
import torch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
pkg = load_pkg()
bgr, depth, gt, cam = synth.sequence(B, seed=1000, preset="fr1")
c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"], cam["k3"],
               cam["factor"])
ctx = pkg.Context(640, 480, max_batch=B, cam=c, orb=pkg.orb_params(1000))
d_bgr = torch.from_numpy(bgr).cuda()
d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
for _ in range(3):
    ctx.extract_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B)
ctx.synchronize()
ctx.reset_timing()
ctx.set_timing(True)
R = 10
for _ in range(R):
    ctx.extract_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B)
ctx.synchronize()
t = ctx.timings()
grid = []
kps = [len(ctx.batch_frame(b)["kps"]) for b in range(min(B, 8))]
print(json.dumps({"frames": B, "us_per_launch": {k: round(v[0] * 1e3 / max(v[1], 1), 1) for k, v in sorted(t.items())},
                  "grid_keypoints": grid, "kept": kps}))

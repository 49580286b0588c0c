"""Time the keyframe dense cloud (rgbd_keyframe_cloud_batch: createCloud(6) + pass-through + VoxelGrid
0.04 + SOR(50, 1)) on the device for K keyframes of a resident batch, beside the oracle on one core."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]


def main():
    import torch
    from conftest import load_pkg
    import oracle_lib as O
    import synth
    pkg = load_pkg()
    B, K = 16, 8
    bgr, depth, _, cam = synth.sequence(B, seed=1000, preset="fr1")
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(1000), cam=c)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    frames = list(range(0, B, B // K))[:K]
    for _ in range(2):
        ctx.keyframe_cloud_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, frames)
    ctx.set_timing(True)
    reps = 10
    t0 = time.perf_counter()
    for _ in range(reps):
        clouds = ctx.keyframe_cloud_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, frames)
    wall = (time.perf_counter() - t0) / reps
    tm = ctx.timings().get("k_cloud", (0.0, 1))
    t1 = time.perf_counter()
    ref = O.keyframe_cloud(bgr[0], depth[0], cam)
    cpu = time.perf_counter() - t1
    assert np.array_equal(clouds[0].view(np.uint8), ref.view(np.uint8))
    print(json.dumps({"keyframes_per_call": K, "points_per_keyframe": int(np.mean([len(x) for x in clouds])),
                      "gpu_kernel_ms_per_call": round(tm[0] / max(tm[1], 1), 3), "gpu_wall_ms_per_call": round(wall * 1e3, 3),
                      "cpu_oracle_ms_per_keyframe": round(cpu * 1e3, 1)}))
    ctx.close()


if __name__ == "__main__":
    main()

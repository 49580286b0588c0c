"""Track a TUM / ICL sequence directory with the MI355X front end, write the camera trajectory in the
reference's format (System/Tracking.cpp:286-317) and, when the directory holds groundtruth.txt, print
the ATE (TUM evaluate_ate semantics: timestamps associated within 20 ms, Horn alignment, RMSE).

  python tools/run_sequence.py <dataset dir> [--batch 64] [--solver pnp|se3] [--out traj.txt]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dataset")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--solver", choices=["pnp", "se3"], default="pnp")
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--max-frames", type=int, default=None)
    ap.add_argument("--out", default="CameraTrajectory.txt")
    ap.add_argument("--posegraph", action="store_true",
                    help="keyframe pose graph (local edges on the device, host LM) and the corrected trajectory")
    args = ap.parse_args()
    from conftest import load_pkg
    import ate
    pkg = load_pkg()
    from rgbd_slam_amd import datasets as DS
    from rgbd_slam_amd.sequence import track_sequence
    ds = DS.open_dataset(args.dataset)
    t0 = time.perf_counter()
    extras = {}
    poses, status, ninl = track_sequence(pkg, ds, B=args.batch, solver=args.solver, nfeatures=args.nfeatures,
                                         max_frames=args.max_frames, extras=extras)
    dt = time.perf_counter() - t0
    n = len(poses)
    if args.posegraph:
        from rgbd_slam_amd.posegraph import posegraph_sequence
        poses, kfs, (v, e, c0, c1) = posegraph_sequence(pkg, ds.frame, ds.camera, poses, nfeatures=args.nfeatures)
        print(f"pose graph: {v} keyframes, {e} edges, chi2 {c0:.4g} -> {c1:.4g}")
    elif "rel" in extras:   # solver se3: the poses saveCameraTrajectory composes (relative to the first keyframe)
        poses = DS.camera_trajectory_poses(extras["rel"], extras["keyframe"], poses)
    DS.write_tum_trajectory(args.out, ds.times[:n], poses)
    print(f"{ds.name}: {n} frames in {dt:.2f} s ({n / dt:.1f} frames/s incl. PNG decoding), tracked "
          f"{int(status.sum())}/{n}, mean inliers {ninl[1:].mean() if n > 1 else 0:.1f}; trajectory -> {args.out}")
    gt_path = os.path.join(args.dataset, "groundtruth.txt")
    if os.path.exists(gt_path):
        gt_t, gt_Twc = DS.read_tum_trajectory(gt_path)
        pairs = DS.associate(ds.times[:n], gt_t)
        if len(pairs) >= 3:
            est = poses[[i for i, _ in pairs]]
            gt = np.linalg.inv(gt_Twc[[j for _, j in pairs]])
            print(f"ATE RMSE {ate.ate_rmse(est, gt):.4f} m over {len(pairs)} associated frames")


if __name__ == "__main__":
    main()

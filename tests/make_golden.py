"""Regenerate tests/golden/*.npz from the oracle (run on CPU: python tests/make_golden.py).

Inputs are not stored: they are regenerated from (seed, preset) by tools/synth.py (integer
hashing + float64, deterministic); bgr_sum guards against generator drift.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
import oracle_lib as O  # noqa: E402
import synth  # noqa: E402


def main():
    out = os.path.join(HERE, "golden")
    os.makedirs(out, exist_ok=True)
    bgr, depth, _, cam = synth.sequence(2, seed=3, preset="fr1")
    p, oc = O.orb_params(1000), O.camera(cam)
    f0 = O.frame(bgr[0], depth[0], p, oc)
    f1 = O.frame(bgr[1], depth[1], p, oc)
    np.savez_compressed(os.path.join(out, "frame_fr1_seed3.npz"), bgr_sum=np.int64(bgr[0].astype(np.int64).sum()),
                        kps=f0["kps"], desc=f0["desc"], xyz=f0["xyz"])
    m = O.match(f0["desc"], f1["desc"], np.zeros(len(f0["kps"]), np.uint8), f0["xyz"][:, 2], f1["xyz"][:, 2], 0.9)
    ok, T, inl, rm = O.ransac_se3(f0["xyz"], f1["xyz"], m, O.ransac_params(), O.rng(42), O.Sticky())
    np.savez_compressed(os.path.join(out, "pair_fr1_seed3.npz"), matches=m, T21=T, inliers=inl,
                        rmse=np.float32(rm))
    print("golden written:", len(f0["kps"]), "kps,", len(m), "matches,", len(inl), "inliers")
    # Extractor(SVO, BRIEF, NORMAL) on the same frame, default BRIEF table (orc_svo.cpp)
    s0 = O.svo_frame(bgr[0], depth[0], O.svo_params(), oc)
    np.savez_compressed(os.path.join(out, "svo_frame_fr1_seed3.npz"), bgr_sum=np.int64(bgr[0].astype(np.int64).sum()),
                        kps=s0["kps"], desc=s0["desc"], xyz=s0["xyz"], pattern=O.brief_default_pattern())
    print("svo golden written:", len(s0["kps"]), "kps")


if __name__ == "__main__":
    main()

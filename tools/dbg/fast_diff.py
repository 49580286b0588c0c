"""Debug: FAST candidates of the device vs the oracle, per level and frame (missing / extra keys)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from conftest import load_pkg
import oracle_lib as O
import synth
pkg = load_pkg()
bgr, depth, _, cam = synth.sequence(4, seed=3, preset="fr1")
c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"], cam["k3"], cam["factor"])
ctx = pkg.Context(640, 480, max_batch=1, orb=pkg.orb_params(1000), cam=c)
p = O.orb_params(1000)
for f in range(4):
    ctx.frame(bgr[f], depth[f])
    ref = O.pyramid(O.gray(bgr[f]), p)
    for l in range(8):
        want = O.level_candidates(ref[l], p)
        got = ctx.debug_candidates(0, l)
        ws = set(map(tuple, want.tolist()))
        gs = set(map(tuple, got.tolist()))
        same_order = got.shape == want.shape and np.array_equal(got, want)
        print("frame", f, "level", l, len(got), len(want), "order-equal", same_order,
              "missing", sorted(ws - gs)[:6], "extra", sorted(gs - ws)[:6])
# positions where the ordered lists differ (frame 3, level 0)
ctx.frame(bgr[3], depth[3])
ref = O.pyramid(O.gray(bgr[3]), p)
for l in (0, 3):
    want = O.level_candidates(ref[l], p)
    got = ctx.debug_candidates(0, l)
    bad = np.nonzero((got != want).any(1))[0]
    print("level", l, "bad positions", len(bad), bad[:20].tolist())
    for i in bad[:12]:
        print("  pos", i, "got", got[max(0, i - 2):i + 3].tolist(), "want", want[max(0, i - 2):i + 3].tolist())

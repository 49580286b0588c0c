"""Debug: where the device blurred pyramid differs from the oracle (rows / columns per level)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from conftest import load_pkg
import oracle_lib as O
import synth
pkg = load_pkg()
bgr, depth, _, cam = synth.sequence(2, seed=3, preset="fr1")
c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"], cam["k3"], cam["factor"])
ctx = pkg.Context(640, 480, max_batch=1, orb=pkg.orb_params(1000), cam=c)
p = O.orb_params(1000); t = O.tables(p)
ctx.frame(bgr[0], depth[0])
ref = O.pyramid(O.gray(bgr[0]), p)
for l in range(8):
    got = ctx.debug_blurred(0, l, int(t["w"][l]), int(t["h"][l]))
    want = O.blur(ref[l])
    d = got != want
    rows = np.nonzero(d.any(1))[0]
    cols = np.nonzero(d.any(0))[0]
    print(l, got.shape, int(d.sum()), "rows", rows[:40].tolist(), "cols", cols[:10].tolist(), cols[-5:].tolist())
# which oracle row does each wrong device row equal (level 0 rows 0..12, level 7 rows 0..8)?
for l, rr in ((0, range(0, 13)), (7, range(0, 9)), (3, range(0, 20))):
    got = ctx.debug_blurred(0, l, int(t["w"][l]), int(t["h"][l]))
    want = O.blur(ref[l])
    for y in rr:
        m = [int(np.abs(got[y].astype(int) - want[k].astype(int)).sum()) for k in range(want.shape[0])]
        k = int(np.argmin(m))
        print("lvl", l, "row", y, "best oracle row", k, "L1", m[k], "own L1", m[y], "ndiff", int((got[y] != want[y]).sum()),
              "first cols", np.nonzero(got[y] != want[y])[0][:8].tolist())

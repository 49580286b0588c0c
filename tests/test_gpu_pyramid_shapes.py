"""GPU parity: the image pyramid at depths and widths the default config does not reach (bit-exact vs the oracle).

k_pyramid computes levels 0 .. RGBD_PYR_STRIP_LEVELS-1 in strips and k_pyr_tail the rest (one workgroup per
frame, rows looped when a level has more column quads than the workgroup has threads).  Cases: no tail
(3 levels), a one-level tail (5), a deep tail (10 levels), a 1.25 scale factor (1.5 leaves levels
whose 30-px FAST cells exceed the 48-px ROI the extractor supports), and a 3200-px-wide frame whose level 1 has
more column quads than k_pyramid has threads and level 4 more than k_pyr_tail has (4800 px exceeds the
strips' LDS budget, rgbd_create's documented error).  Seeded noise frames: the pyramid does not depend on texture.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W,H,nlevels,scale", [(640, 480, 3, 1.2), (640, 480, 5, 1.2), (640, 480, 10, 1.2),
                                                (640, 480, 6, 1.25), (3200, 240, 8, 1.2)])
def test_pyramid_levels_bit_exact(pkg, oracle, W, H, nlevels, scale):
    rng = np.random.default_rng(W + 7 * nlevels)
    bgr = rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8)
    depth = np.zeros((H, W), np.uint16)
    cam = pkg.camera(525.0, 525.0, W / 2.0, H / 2.0)
    ctx = pkg.Context(W, H, max_batch=1, orb=pkg.orb_params(1000, scale, nlevels), cam=cam)
    p = oracle.orb_params(1000, scale, nlevels)
    t = oracle.tables(p, W, H)
    ctx.frame(bgr, depth)
    ref = oracle.pyramid(oracle.gray(bgr), p)
    for l in range(nlevels):
        assert ref[l].shape == (int(t["h"][l]), int(t["w"][l]))
        got = ctx.debug_level(0, l, int(t["w"][l]), int(t["h"][l]))
        assert np.array_equal(got, ref[l]), f"level {l}: {np.count_nonzero(got != ref[l])} px differ"

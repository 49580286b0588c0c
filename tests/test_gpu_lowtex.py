"""GPU parity in the low-texture regime (tools/synth.py preset "lowtex": large blocks whose intensities differ by
<= 23 levels, no fine pattern), where FAST at iniThFAST = 20 finds almost nothing and nearly every cell of
every level takes the minThFAST = 7 fallback (Features/ORBextractor.cpp:655-661).  The rich synthetic frames of
the other tests never reach that branch in more than a few cells.  Everything bit-exact against the oracle:
per-level candidate lists, the frame outputs, and the benchmark chain (extract + knn-2 + PnPRansac) at the
bench's batch shape."""
import numpy as np
import pytest

import chain_model
from conftest import synth_seq

pytestmark = pytest.mark.gpu


def _ctx(pkg, cam, max_batch=4):
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    return pkg.Context(640, 480, max_batch=max_batch, orb=pkg.orb_params(1000), cam=c)


def _fallback_share(oracle, gray):
    """Share of level-0 30-px cells with no FAST corner at 20 among those with one at 7 (oracle side)."""
    c20 = np.asarray(oracle.fast(gray, 20)).reshape(-1, 3)
    c7 = np.asarray(oracle.fast(gray, 7)).reshape(-1, 3)
    cells = lambda c: set(zip((c[:, 0] // 30).tolist(), (c[:, 1] // 30).tolist()))
    a20, a7 = cells(c20), cells(c7)
    return len(a7 - a20) / max(len(a7), 1)


def test_lowtex_frames_bit_exact(pkg, oracle):
    bgr, depth, _, cam = synth_seq(2, seed=5, preset="lowtex")
    ctx = _ctx(pkg, cam)
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    for f in range(2):
        assert _fallback_share(oracle, oracle.gray(bgr[f])) > 0.9   # the regime: th = 7 decides almost everywhere
        got = ctx.frame(bgr[f], depth[f])
        want = oracle.frame(bgr[f], depth[f], p, oc)
        assert len(got["kps"]) == len(want["kps"]) > 500
        for fld in got["kps"].dtype.names:
            assert np.array_equal(got["kps"][fld], want["kps"][fld]), fld
        assert np.array_equal(got["desc"], want["desc"])
        assert np.array_equal(got["xyz"].view(np.uint32), want["xyz"].view(np.uint32))
        ref = oracle.pyramid(oracle.gray(bgr[f]), p)
        for l in range(8):   # the per-cell candidate lists (fallback included), every level
            wc = oracle.level_candidates(ref[l], p)
            gc = ctx.debug_candidates(0, l)
            assert np.array_equal(gc, wc), (f, l, len(gc), len(wc))
    ctx.close()


def test_lowtex_bench_chain_bit_exact(pkg, oracle):
    """The headline chain on low-texture frames at B = 256 (16 rendered frames walked back and forth, as
    bench.py): sampled frames and every pair's PnPRansac result against the oracle."""
    import torch
    import synth
    B, U = 256, 16
    ub, ud, ut, cam = synth.sequence(U, seed=2000, preset="lowtex")
    r = np.arange(B) % (2 * U - 2)
    src = np.where(r < U, r, 2 * U - 2 - r)
    ctx = _ctx(pkg, cam, max_batch=B)
    d_bgr = torch.from_numpy(ub[src]).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(ud[src]).view(np.int16)).cuda()
    pose0 = ut[0].astype(np.float32)
    poses, status, ninl, nm = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, pkg.pnp_params(), pose0)
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    frames = [oracle.frame(ub[u], ud[u], p, oc) for u in range(U)]
    K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
    pairs = {}
    for b in range(1, B):
        key = (int(src[b - 1]), int(src[b]))
        if key not in pairs:
            pairs[key] = chain_model.pnp_pair(oracle, frames[key[0]], frames[key[1]], K4)
        ok, T, ni, m = pairs[key]
        assert (status[b], ninl[b], nm[b]) == (int(ok), ni, m), b
        want = chain_model.compose(T, poses[b - 1]) if ok else poses[b - 1]
        assert np.array_equal(poses[b].view(np.uint32), want.view(np.uint32)), b
    assert status.mean() > 0.9
    for b in (0, 17, 255):
        f, w = ctx.batch_frame(b), frames[int(src[b])]
        assert np.array_equal(f["kps"], w["kps"]) and np.array_equal(f["desc"], w["desc"])
    ctx.close()

"""GPU parity at the bench's own shape: B = 1024 frames per step (the default of bench.py), three
submissions in flight through rgbd_pnp_track_submit / collect (two output sets, three workspaces,
solves on the solve stream).  Sampled frames' KeyPoints / descriptors / xyz and sampled pairs'
PnPRansac results (pose bits, inliers, matches) equal the oracle; the three steps are identical."""
import numpy as np
import pytest

import chain_model

pytestmark = pytest.mark.gpu

B = 1024
U = 16   # rendered frames walked back and forth, as bench.py does with --unique


def _pingpong(g, u):
    r = np.asarray(g) % (2 * u - 2)
    return np.where(r < u, r, 2 * u - 2 - r)


def test_bench_shape_b1024_three_in_flight(pkg, oracle):
    import torch
    import synth
    ub, ud, ut, cam = synth.sequence(U, seed=1000, preset="fr1")
    src = _pingpong(np.arange(B), U)
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(1000), cam=c)
    d_bgr = torch.from_numpy(ub[src]).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(ud[src]).view(np.int16)).cuda()
    pose0 = ut[0].astype(np.float32)
    prm = pkg.pnp_params()
    for _ in range(3):
        ctx.pnp_track_submit(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, prm)
    got = [ctx.pnp_track_collect(pose0) for _ in range(3)]
    for g in got[1:]:
        for a, b in zip(got[0], g):
            assert np.array_equal(np.asarray(a).view(np.uint32), np.asarray(b).view(np.uint32))
    poses, status, ninl, nm = got[0]
    assert status.mean() > 0.99
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    cache = {}

    def ofr(b):
        u = int(src[b])
        if u not in cache:
            cache[u] = oracle.frame(ub[u], ud[u], p, oc)
        return cache[u]

    for b in (0, 7, 8, 511, 1023):   # the latest submission's output set (rgbd_batch_frame)
        f, w = ctx.batch_frame(b), ofr(b)
        assert len(f["kps"]) == len(w["kps"]) > 500
        assert np.array_equal(f["kps"], w["kps"]) and np.array_equal(f["desc"], w["desc"])
        assert np.array_equal(f["xyz"].view(np.uint32), w["xyz"].view(np.uint32))
    K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
    for b in (1, 8, 15, 16, 512, 1023):   # 15 -> 16 walks back (rendered 15 -> 14)
        ok, T, ni, m = chain_model.pnp_pair(oracle, ofr(b - 1), ofr(b), K4)
        assert status[b] == int(ok) and ninl[b] == ni and nm[b] == m, b
        want = chain_model.compose(T, poses[b - 1]) if ok else poses[b - 1]
        assert np.array_equal(poses[b].view(np.uint32), want.view(np.uint32)), b
    ctx.close()

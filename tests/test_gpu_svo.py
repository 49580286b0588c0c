"""GPU parity: the SVO + BRIEF front end (the reference's default Extractor(SVO, BRIEF, NORMAL), main.cpp:31)
on gfx950 vs the CPU oracle (oracle/orc_svo.cpp), bit-exact: halfSample levels, the grid keypoints before
retainBest, libstdc++'s retainBest order (device restatement vs std::nth_element / std::__introselect),
final keypoints / BRIEF descriptors / undistorted keypoints / 3D points, and the extract + match + PnPRansac
chain with an SVO context.  Calls go through the C ABI; inputs are seeded synthetic RGB-D frames."""
import math

import numpy as np
import pytest

from conftest import synth_seq
import chain_model

pytestmark = pytest.mark.gpu


def _cam(pkg, cam):
    return pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                      cam["k3"], cam["factor"])


def _ctx(pkg, cam, max_batch=4, **kw):
    return pkg.Context(640, 480, max_batch=max_batch, cam=_cam(pkg, cam), svo=pkg.svo_params(**kw))


@pytest.fixture(scope="module")
def svo_ctx(pkg, seq_fr1):
    c = _ctx(pkg, seq_fr1[3])
    yield c
    c.close()


def _same_frame(got, want):
    assert len(got["kps"]) == len(want["kps"]) > 500, (len(got["kps"]), len(want["kps"]))
    assert np.array_equal(got["kps"], want["kps"])
    assert np.array_equal(got["desc"], want["desc"])
    assert np.array_equal(got["kps_un"], want["kps_un"])
    assert np.array_equal(got["xyz"].view(np.uint32), want["xyz"].view(np.uint32))


def test_svo_pyramid_and_grid(pkg, oracle, seq_fr1, svo_ctx):
    bgr, depth, _, cam = seq_fr1
    p = oracle.svo_params()
    for f in range(2):
        svo_ctx.frame(bgr[f], depth[f])
        g = oracle.gray(bgr[f])
        ref = oracle.svo_pyramid(g, 8)
        for l in range(8):
            got = svo_ctx.svo_debug_level(0, l)
            assert np.array_equal(got, ref[l]), f"frame {f} level {l}: {np.count_nonzero(got != ref[l])} px differ"
        xyl, resp = svo_ctx.svo_debug_grid(0)
        want = oracle.svo_detect(g, p)
        assert len(xyl) == len(want) > 1000
        assert np.array_equal(xyl[:, 0], want["x"].astype(np.int32)) and np.array_equal(xyl[:, 1], want["y"].astype(np.int32))
        assert np.array_equal(xyl[:, 2], want["octave"])
        assert np.array_equal(resp.view(np.uint32), want["response"].view(np.uint32))


@pytest.mark.parametrize("preset,seed", [("fr1", 3), ("fr3", 11), ("icl", 23), ("fr2", 22)])
def test_svo_frame_bit_exact(pkg, oracle, preset, seed):
    bgr, depth, _, cam = synth_seq(2, seed=seed, preset=preset)
    ctx = _ctx(pkg, cam, max_batch=1)
    p, oc = oracle.svo_params(), oracle.camera(cam)
    for f in range(2):
        _same_frame(ctx.frame(bgr[f], depth[f]), oracle.svo_frame(bgr[f], depth[f], p, oc))
    # detect_and_compute from a gray image (Extractor::detectAndCompute)
    g = oracle.gray(bgr[0])
    k, d = ctx.detect_and_compute(g)
    wk, wd = oracle.svo_detect_and_compute(g, p)
    assert np.array_equal(k, wk) and np.array_equal(d, wd)
    ctx.close()


def test_svo_batch_and_patterns(pkg, oracle):
    import torch
    B = 6
    bgr, depth, _, cam = synth_seq(B, seed=41, preset="fr1")
    ctx = _ctx(pkg, cam, max_batch=B)
    p, oc = oracle.svo_params(), oracle.camera(cam)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pat0 = ctx.brief_pattern()
    assert np.array_equal(pat0, oracle.brief_default_pattern())
    rnd = np.random.RandomState(9).randint(-24, 25, size=(256, 4)).astype(np.int8)
    for pat in (None, rnd):
        if pat is not None:
            ctx.set_brief_pattern(pat)
        for rep in range(2):   # the cell keys are reset by k_svo_select for the next batch
            ctx.extract_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B)
            for b in range(B):
                _same_frame(ctx.batch_frame(b), oracle.svo_frame(bgr[b], depth[b], p, oc, pattern=pat))
    with pytest.raises(pkg.RgbdError):
        ctx.set_brief_pattern(np.full((256, 4), 25, np.int8))   # outside the 48-px patch
    ctx.close()


def test_svo_nfeatures_variants(pkg, oracle):
    bgr, depth, _, cam = synth_seq(2, seed=5, preset="fr3")
    oc = oracle.camera(cam)
    for nf in (1, 300, 2000, 20000):
        ctx = _ctx(pkg, cam, max_batch=1, nfeatures=nf)
        want = oracle.svo_frame(bgr[1], depth[1], oracle.svo_params(nfeatures=nf), oc)
        got = ctx.frame(bgr[1], depth[1])
        assert np.array_equal(got["kps"], want["kps"]) and np.array_equal(got["desc"], want["desc"])
        ctx.close()


def test_svo_boundary_ties_capacity(pkg, oracle):
    """retainBest keeps every tie of the boundary response: a periodic image (period 10 = two grid cells)
    ties hundreds of cells; beyond max_keypoints the context fails loudly, with room it matches."""
    import synth
    rs = np.random.RandomState(4)
    patch = rs.randint(0, 256, size=(10, 10, 3)).astype(np.uint8)
    bgr = np.ascontiguousarray(np.tile(patch, (48, 64, 1)))
    depth = np.full((480, 640), 5000, np.uint16)
    cam = dict(synth.PRESETS["fr3"])
    oc = oracle.camera(cam)
    want = oracle.svo_frame(bgr, depth, oracle.svo_params(nfeatures=100), oc)
    assert len(want["kps"]) > 100 + 64
    ctx = _ctx(pkg, cam, max_batch=1, nfeatures=100)
    assert ctx.kp_cap == 164
    with pytest.raises(pkg.RgbdError):
        ctx.frame(bgr, depth)
    ctx.close()
    ctx = _ctx(pkg, cam, max_batch=1, nfeatures=100, max_keypoints=12288)
    _same_frame_n(ctx.frame(bgr, depth), want)
    ctx.close()


def test_svo_capacity_flag_per_frame_and_batched_paths(pkg, oracle):
    """The capacity flag is per frame and cleared by every extraction: in a batch only the overflowing
    frame fails, a later extraction on the same context succeeds, and the batched tracking entry points
    (rgbd_pnp_track_batch, submit / collect, rgbd_track_batch) report RGBD_ERR_CAPACITY instead of
    tracking on truncated keypoints."""
    import synth
    import torch
    rs = np.random.RandomState(4)
    patch = rs.randint(0, 256, size=(10, 10, 3)).astype(np.uint8)
    bad = np.ascontiguousarray(np.tile(patch, (48, 64, 1)))
    bgr0, dep0, _, cam = synth.sequence(2, seed=11, preset="fr3")
    bgr = np.stack([bgr0[0], bad, bgr0[1]])
    depth = np.stack([dep0[0], np.full((480, 640), 5000, np.uint16), dep0[1]])
    oc = oracle.camera(cam)
    sp = oracle.svo_params(nfeatures=100)
    ctx = _ctx(pkg, cam, max_batch=3, nfeatures=100)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    ctx.extract_batch(d_bgr.data_ptr(), d_dep.data_ptr(), 3)
    for b in (0, 2):
        _same_frame_n(ctx.batch_frame(b), oracle.svo_frame(bgr[b], depth[b], sp, oc))
    with pytest.raises(pkg.RgbdError):
        ctx.batch_frame(1)
    _same_frame_n(ctx.frame(bgr[0], depth[0]), oracle.svo_frame(bgr[0], depth[0], sp, oc))   # flag cleared
    with pytest.raises(pkg.RgbdError):
        ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), 3, 0.9, pkg.pnp_params())
    ctx.pnp_track_submit(d_bgr.data_ptr(), d_dep.data_ptr(), 3, 0.9, pkg.pnp_params())
    with pytest.raises(pkg.RgbdError):
        ctx.pnp_track_collect()
    with pytest.raises(pkg.RgbdError):
        ctx.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), 3, 0.9, pkg.ransac_params(200, 10, 3.0, 4), pkg.rng(1),
                        pkg.Sticky())
    # frames 0 and 2 alone track fine on the same context
    d2b, d2d = d_bgr[[0, 2]].contiguous(), d_dep[[0, 2]].contiguous()
    _, st, _, _ = ctx.pnp_track_batch(d2b.data_ptr(), d2d.data_ptr(), 2, 0.9, pkg.pnp_params())
    assert st[0] == 1
    ctx.close()


def _same_frame_n(got, want):
    assert len(got["kps"]) == len(want["kps"])
    assert np.array_equal(got["kps"], want["kps"]) and np.array_equal(got["desc"], want["desc"])
    assert np.array_equal(got["xyz"].view(np.uint32), want["xyz"].view(np.uint32))


def test_svo_empty_and_flat_frames(pkg, oracle, seq_fr1):
    """A flat image has no corners: zero keypoints, like the oracle (Frame returns early, Core/Frame.cpp:55);
    nfeatures 0 makes retainBest clear everything; a flat frame inside a batch leaves its neighbours intact."""
    import torch
    bgr, depth, _, cam = seq_fr1
    oc = oracle.camera(cam)
    flat = np.full_like(bgr[0], 128)
    ctx = _ctx(pkg, cam, max_batch=3)
    got = ctx.frame(flat, depth[0])
    assert len(got["kps"]) == 0 == len(oracle.svo_frame(flat, depth[0], oracle.svo_params(), oc)["kps"])
    stack = np.ascontiguousarray(np.stack([bgr[0], flat, bgr[1]]))
    d_bgr = torch.from_numpy(stack).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth[:3]).view(np.int16)).cuda()
    ctx.extract_batch(d_bgr.data_ptr(), d_dep.data_ptr(), 3)
    for b in range(3):
        _same_frame_n(ctx.batch_frame(b), oracle.svo_frame(stack[b], depth[b], oracle.svo_params(), oc))
    ctx.close()
    ctx = _ctx(pkg, cam, max_batch=1, nfeatures=0)
    assert len(ctx.frame(bgr[0], depth[0])["kps"]) == 0
    ctx.close()


def _adversarial(n, rs):
    # many duplicates, sorted / reverse-sorted runs, organ-pipe: the shapes that stress Hoare pairing
    return [rs.rand(n).astype(np.float32),
            (rs.randint(0, 7, n) * 0.5 + 21).astype(np.float32),
            np.sort(rs.rand(n)).astype(np.float32),
            np.sort(rs.rand(n))[::-1].astype(np.float32).copy(),
            np.concatenate([np.arange(n // 2), np.arange(n - n // 2)[::-1]]).astype(np.float32),
            np.full(n, 33.0, np.float32)]


def test_retain_best_matches_libstdcxx(pkg, oracle, svo_ctx):
    rs = np.random.RandomState(17)
    for n, keep in [(5, 1), (4, 3), (17, 5), (1001, 1000), (3000, 1000), (8198, 1000), (12288, 1000), (12288, 11000),
                    (2500, 64), (777, 776)]:
        for r in _adversarial(n, rs):
            got = svo_ctx.svo_retain_best(r, keep)
            want = oracle.retain_best(r, keep)
            assert np.array_equal(got, want), (n, keep)
    # the heap-select fallback and shallow depth limits (libstdc++'s own __introselect at that depth)
    for n, keep in [(3000, 1000), (999, 500), (64, 10)]:
        for depth in (0, 1, 3, 2 * int(math.log2(n))):
            for r in _adversarial(n, rs)[:3]:
                got = svo_ctx.svo_retain_best(r, keep, depth)
                want = oracle.retain_best_depth(r, keep, depth)
                assert np.array_equal(got, want), (n, keep, depth)


def test_svo_pnp_chain_matches_oracle(pkg, oracle):
    """Extract (SVO + BRIEF) + Matcher + PnPRansac per consecutive pair, bit-exact vs the oracle chain."""
    import torch
    B = 5
    bgr, depth, gt, cam = synth_seq(B, seed=21, preset="fr1")
    ctx = _ctx(pkg, cam, max_batch=B)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pose0 = gt[0].astype(np.float32)
    poses, status, ninl, nm = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, pkg.pnp_params(), pose0)
    p, oc = oracle.svo_params(), oracle.camera(cam)
    frames = [oracle.svo_frame(bgr[i], depth[i], p, oc) for i in range(B)]
    K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
    wp, ws, wn, wm = chain_model.pnp_track(oracle, frames, pose0, K4)
    assert np.array_equal(nm, wm) and np.array_equal(status, ws) and np.array_equal(ninl, wn)
    assert np.array_equal(poses.view(np.uint32), wp.view(np.uint32))
    assert status.all()
    for b in range(1, B):
        rel = poses[b] @ np.linalg.inv(poses[b - 1])
        rel_gt = gt[b] @ np.linalg.inv(gt[b - 1])
        # sanity only (parity is the bit equality above): SVO keypoints sit on 2^level pixel grids
        assert np.linalg.norm(rel[:3, 3] - rel_gt[:3, 3]) < 0.06
    ctx.close()

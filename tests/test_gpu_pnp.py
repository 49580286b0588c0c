"""GPU parity: PnPRansac on gfx950 (rgbd_pnp_ransac_batch / rgbd_pnp_track_batch) vs the oracle
restatement (oracle/orc_pnp.cpp).  Bit-exact: R, t (f64 bits), RANSAC inlier mask, inlier count and
iteration count.  Object points / pixels are seeded synthetic problems (tests/pnp_cases.py)."""
import numpy as np
import pytest

from conftest import synth_seq
from pnp_cases import K_TUM, problem
import chain_model

pytestmark = pytest.mark.gpu

CASES = [(5, 0.0, 0.0), (6, 0.0, 0.5), (10, 0.1, 0.5), (40, 0.3, 0.5), (137, 0.3, 0.5), (300, 0.5, 1.0),
         (800, 0.2, 0.5), (1500, 0.6, 0.5), (4096, 0.3, 0.5), (64, 0.85, 0.5), (200, 0.0, 0.0)]


def _check(res, want):
    ok, R, t, mask, ni, it = want
    assert res["ok"] == ok
    assert res["n_inliers"] == (ni if ok else 0)
    if ok:
        assert res["iters"] == it
        assert np.array_equal(res["mask"], mask)
        assert np.array_equal(res["R"].view(np.uint64), R.view(np.uint64)), (res["R"] - R)
        assert np.array_equal(res["t"].view(np.uint64), t.view(np.uint64)), (res["t"] - t)


@pytest.fixture(scope="module")
def ctx(pkg):
    c = pkg.Context(640, 480, max_batch=2)
    yield c
    c.close()


def test_pnp_batch_matches_oracle(pkg, oracle, ctx):
    probs = [problem(n, 100 + i, outliers=o, noise=s)[:2] for i, (n, o, s) in enumerate(CASES)]
    res = ctx.pnp_ransac_batch(probs, K_TUM, pkg.pnp_params(min_matches=0))
    for (p3, p2), r in zip(probs, res):
        _check(r, oracle.pnp_ransac(p3, p2, K_TUM))


@pytest.mark.parametrize("seed", range(6))
def test_pnp_single_matches_oracle(pkg, oracle, ctx, seed):
    n = [25, 90, 333, 1000, 2500, 61][seed]
    p3, p2, R, t, inl = problem(n, 500 + seed, outliers=[0.2, 0.4, 0.3, 0.5, 0.1, 0.7][seed])
    r = ctx.pnp_ransac(p3, p2, K_TUM, pkg.pnp_params(min_matches=0))
    _check(r, oracle.pnp_ransac(p3, p2, K_TUM))
    if r["ok"] and seed != 5:
        assert np.abs(r["R"] - R).max() < 5e-3


def test_pnp_edges(pkg, oracle, ctx):
    p3, p2, *_ = problem(12, 9, outliers=0.0)
    same3, same2 = np.repeat(p3[:1], 30, 0), np.repeat(p2[:1], 30, 0)
    probs = [(p3[:0], p2[:0]), (p3[:4], p2[:4]), (p3[:5], p2[:5]), (same3, same2), (p3, p2)]
    res = ctx.pnp_ransac_batch(probs, K_TUM, pkg.pnp_params(min_matches=0))
    for (a, b), r in zip(probs, res):
        _check(r, oracle.pnp_ransac(a, b, K_TUM))
    assert not res[0]["ok"] and not res[1]["ok"] and res[2]["ok"] and not res[3]["ok"] and res[4]["ok"]
    # PnPRansac::compute's < 10 matches rule (Solver/PnPRansac.cpp:16)
    r = ctx.pnp_ransac(p3[:9], p2[:9], K_TUM, pkg.pnp_params(min_matches=10))
    assert not r["ok"]
    # non-default operator arguments
    prm = pkg.pnp_params(iters=50, reproj=1.5, conf=0.99, min_matches=0)
    p3, p2, *_ = problem(400, 77, outliers=0.4)
    r = ctx.pnp_ransac(p3, p2, K_TUM, prm)
    _check(r, oracle.pnp_ransac(p3, p2, K_TUM, 50, 1.5, 0.99))


@pytest.mark.parametrize("preset,seed", [("fr1", 21), ("fr2", 22), ("icl", 23)])
def test_pnp_track_batch_matches_oracle_chain(pkg, oracle, preset, seed):
    import torch
    B = 5
    bgr, depth, gt, cam = synth_seq(B, seed=seed, preset=preset)
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    nfeat = 2000 if preset == "fr2" else 1000
    ctx = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(nfeat), cam=c)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pose0 = gt[0].astype(np.float32)
    poses, status, ninl, nm = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, pkg.pnp_params(),
                                                  pose0)
    p, oc = oracle.orb_params(nfeat), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(B)]
    K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
    wp, ws, wn, wm = chain_model.pnp_track(oracle, frames, pose0, K4)
    assert np.array_equal(nm, wm)
    assert np.array_equal(status, ws)
    assert np.array_equal(ninl, wn)
    assert np.array_equal(poses.view(np.uint32), wp.view(np.uint32))
    assert status.all()
    for b in range(1, B):
        rel = poses[b] @ np.linalg.inv(poses[b - 1])
        rel_gt = gt[b] @ np.linalg.inv(gt[b - 1])
        assert np.linalg.norm(rel[:3, 3] - rel_gt[:3, 3]) < 0.02
    ctx.close()


def test_pnp_track_submit_collect_pipeline(pkg):
    """Up to three outstanding submissions (three workspaces; a submission's solve is launched by the
    next one) give, batch for batch, the bits of the synchronous rgbd_pnp_track_batch; collect follows
    submission order, also when no later submission launched the solve."""
    import torch
    B = 5
    bgr, depth, gt, cam = synth_seq(2 * B, seed=31, preset="fr1")
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(1000), cam=c)
    batches = []
    for lo in (0, B, 2, 3):   # four different chunks
        d_bgr = torch.from_numpy(np.ascontiguousarray(bgr[lo:lo + B])).cuda()
        d_dep = torch.from_numpy(np.ascontiguousarray(depth[lo:lo + B]).view(np.int16)).cuda()
        batches.append((d_bgr, d_dep, gt[lo].astype(np.float32)))
    want = [ctx.pnp_track_batch(b.data_ptr(), d.data_ptr(), B, 0.9, pkg.pnp_params(), p0) for b, d, p0 in batches]
    prm = pkg.pnp_params()

    def submit(i):
        ctx.pnp_track_submit(batches[i][0].data_ptr(), batches[i][1].data_ptr(), B, 0.9, prm)

    submit(0)
    submit(1)
    submit(2)
    with pytest.raises(pkg.RgbdError):   # a fourth outstanding submission is refused
        submit(3)
    got = [ctx.pnp_track_collect(batches[0][2])]
    submit(3)
    got += [ctx.pnp_track_collect(batches[i][2]) for i in (1, 2, 3)]   # 3: solve launched by collect
    with pytest.raises(pkg.RgbdError):
        ctx.pnp_track_collect()
    submit(1)   # a lone submission
    got.append(ctx.pnp_track_collect(batches[1][2]))
    for (wp, ws, wn, wm), (gp, gs, gn, gm) in zip(want + [want[1]], got):
        assert np.array_equal(gp.view(np.uint32), wp.view(np.uint32))
        assert np.array_equal(gs, ws) and np.array_equal(gn, wn) and np.array_equal(gm, wm)
    ctx.close()


@pytest.mark.parametrize("segments", [1, 2])
def test_pnp_track_flag_chain_continuation_matches_oracle(pkg, oracle, segments):
    """The flag chain through a pair whose RANSAC does not finish in the first hypothesis chunk (the pair
    into a noise frame: no model reaches the inlier threshold, solvePnPRansac runs all its iterations on the
    host continuation) and a failed solve's flags (every matched train index an outlier).  Bit for bit
    against the oracle chain, before and after the failing pair."""
    import torch
    B = 9
    bgr, depth, gt, cam = synth_seq(B, seed=43, preset="fr1")
    bgr[4] = np.random.RandomState(9).randint(0, 256, size=bgr[4].shape).astype(np.uint8)
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(1000), cam=c)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pose0 = gt[0].astype(np.float32)
    prm = pkg.pnp_params(flag_segments=segments)
    poses, status, ninl, nm = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, prm, pose0)
    ctx.close()
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(B)]
    K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
    wp, ws, wn, wm, _ = chain_model.pnp_track_flagged(oracle, frames, pose0, K4, segments)
    assert np.array_equal(nm, wm) and np.array_equal(status, ws) and np.array_equal(ninl, wn)
    assert np.array_equal(poses.view(np.uint32), wp.view(np.uint32))
    assert not status[4] and status[1:4].all() and status[6:].all()


def test_pnp_track_flag_chain_rng_tail_matches_oracle(pkg, oracle):
    """solvePnPRansac with 3000 iterations on the pair into a noise frame: no model reaches the inlier
    threshold, so the loop draws all 3000 subsets (> 15000 cv::RNG outputs), past the 8192-entry table
    k_pnp_chain's RNG outputs are read from, and wave 0 continues the generator sequentially from the
    table's end state (pnp.hip, k_pnp_chain).  Bit for bit against the oracle chain."""
    import torch
    B, iters = 7, 3000
    bgr, depth, gt, cam = synth_seq(B, seed=45, preset="fr1")
    bgr[3] = np.random.RandomState(11).randint(0, 256, size=bgr[3].shape).astype(np.uint8)
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(1000), cam=c)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pose0 = gt[0].astype(np.float32)
    prm = pkg.pnp_params(iters=iters, flag_segments=1)
    poses, status, ninl, nm = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, prm, pose0)
    ctx.close()
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(B)]
    K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
    wp, ws, wn, wm, _ = chain_model.pnp_track_flagged(oracle, frames, pose0, K4, 1, iters=iters)
    assert np.array_equal(nm, wm) and np.array_equal(status, ws) and np.array_equal(ninl, wn)
    assert np.array_equal(poses.view(np.uint32), wp.view(np.uint32))
    assert not status[3] and nm[3] >= 10   # the noise pair ran its whole loop (>= min_matches)


def test_pnp_track_flag_chain_many_keypoints_matches_oracle(pkg, oracle):
    """More than 2048 keypoints per frame (nfeatures 2600): k_pnp_chain's gather takes its loop form (more
    queries than its 256 threads hold in registers) and copies the kept points into LDS afterwards.  Bit
    for bit against the oracle chain."""
    import torch
    B, nf = 4, 2600
    bgr, depth, gt, cam = synth_seq(B, seed=47, preset="fr1")
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(nf), cam=c)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pose0 = gt[0].astype(np.float32)
    prm = pkg.pnp_params(flag_segments=1)
    poses, status, ninl, nm = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, prm, pose0)
    ctx.close()
    p, oc = oracle.orb_params(nf), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(B)]
    assert all(len(f["kps"]) > 2048 for f in frames[:-1])   # the loop-form gather runs for every pair
    K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
    wp, ws, wn, wm, _ = chain_model.pnp_track_flagged(oracle, frames, pose0, K4, 1)
    assert np.array_equal(nm, wm) and np.array_equal(status, ws) and np.array_equal(ninl, wn)
    assert np.array_equal(poses.view(np.uint32), wp.view(np.uint32))
    assert status[1:].all()


@pytest.mark.parametrize("segments", [1, 2, 3])
def test_pnp_track_flag_chain_matches_oracle(pkg, oracle, segments):
    """flag_segments >= 1: the reference's Matcher(discardOutliers = true) on PnPRansac's outlier flags
    (Features/Matcher.cpp:125-128, Solver/PnPRansac.cpp:31,51), one chain per run of pairs, bit for bit
    against the oracle chain; the flags change the match lists against the independent-pair mode."""
    import torch
    B = 7
    bgr, depth, gt, cam = synth_seq(B, seed=41, preset="fr1")
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(1000), cam=c)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    pose0 = gt[0].astype(np.float32)
    prm = pkg.pnp_params(flag_segments=segments)
    poses, status, ninl, nm = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, prm, pose0)
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    frames = [oracle.frame(bgr[i], depth[i], p, oc) for i in range(B)]
    K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
    wp, ws, wn, wm, _ = chain_model.pnp_track_flagged(oracle, frames, pose0, K4, segments)
    assert np.array_equal(nm, wm) and np.array_equal(status, ws) and np.array_equal(ninl, wn)
    assert np.array_equal(poses.view(np.uint32), wp.view(np.uint32))
    assert status.all()
    _, _, _, free = chain_model.pnp_track(oracle, frames, pose0, K4)
    starts = chain_model.segment_starts(B - 1, segments)
    chained = [b for b in range(1, B) if (b - 1) not in starts]
    assert sum(nm[b] for b in chained) < sum(free[b] for b in chained), (nm, free)   # flagged queries dropped
    assert all(nm[b] == free[b] for b in range(1, B) if b not in chained)
    # pipelined: the same bits through submit / collect (at most two outstanding in this mode)
    ctx.pnp_track_submit(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, prm)
    ctx.pnp_track_submit(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, prm)
    with pytest.raises(pkg.RgbdError):
        ctx.pnp_track_submit(d_bgr.data_ptr(), d_dep.data_ptr(), B, 0.9, prm)
    for _ in range(2):
        gp, gs, gn, gm = ctx.pnp_track_collect(pose0)
        assert np.array_equal(gp.view(np.uint32), wp.view(np.uint32))
        assert np.array_equal(gs, ws) and np.array_equal(gn, wn) and np.array_equal(gm, wm)
    ctx.close()


def test_svd_sqrt_div_sequences_are_ieee(pkg, ctx):
    """The 3 x 3 SVD's (csrc/svd3_dev.h: RansacSE3's transform, GICP's covariances) uses of the same sequences:
    1 / d for 1 <= |d| < 2^1000 (recip_ge1), u / sqrt(1 + u^2) for 2^-1000 <= |u| < 2^999 and sqrt(1 + u^2)
    while finite -- the IEEE bits (numpy's / and sqrt)."""
    rs = np.random.RandomState(23)
    n = 1 << 20
    sgn = lambda k: rs.choice([-1.0, 1.0], k)
    d_a = np.ldexp(rs.uniform(1, 2, n // 2), rs.randint(0, 1000, n // 2)) * sgn(n // 2)    # recip_ge1
    u = np.ldexp(rs.uniform(1, 2, n // 2), rs.randint(-1000, 999, n // 2)) * sgn(n // 2)
    with np.errstate(over="ignore"):
        tmp = np.sqrt(1.0 + u * u)
    u_ok = np.isfinite(tmp)
    u, tmp = u[u_ok], tmp[u_ok]
    nums = np.concatenate([np.ones(n // 2), u])
    dens = np.concatenate([d_a, tmp])
    with np.errstate(over="ignore"):
        xs_all = 1.0 + u * u
    xs = np.resize(xs_all[np.isfinite(xs_all)], len(nums))
    nums, dens, xs = nums[:n], dens[:n], xs[:n]
    th = np.zeros(len(nums))
    sq, q, _ = ctx.debug_rotation_ops(xs, nums, dens, th)
    assert np.array_equal(sq.view(np.uint64), np.sqrt(xs).view(np.uint64))
    assert np.array_equal(q.view(np.uint64), (nums / dens).view(np.uint64))


def test_rotation_sqrt_div_sequences_are_ieee(pkg, ctx):
    """The Jacobi rotation's shortened sqrt / division sequences (csrc/pnp.hip sqrt_ge1, div_plain: the compiler's
    own sequences minus the range-scaling and special-case steps) return the IEEE bits (numpy's sqrt and /)
    over the operand ranges the rotation feeds them: theta^2 + 1 in [1, 2^1023), tq^2 + 1 in [1, 2], the
    denominator |theta| + sqrt(theta^2 + 1) in [1, 2^513] under a numerator of +-1, and 1 over [1, sqrt 2]."""
    rs = np.random.RandomState(11)
    n = 1 << 20
    theta = np.concatenate([rs.standard_normal(n // 4), 10.0 ** rs.uniform(-20, 150, n // 4) * rs.choice([-1, 1], n // 4),
                            np.ldexp(rs.uniform(1, 2, n // 4), rs.randint(-60, 511, n // 4)),
                            np.array([0.0, 1.0, -1.0, 1e-300, np.ldexp(1.0, 511), np.ldexp(1.9999, 511)])])
    theta = np.resize(theta, n)
    x1 = theta * theta + 1.0
    den = np.abs(theta) + np.sqrt(x1)
    sg = np.where(theta >= 0.0, 1.0, -1.0)
    tq = sg / den
    x2 = tq * tq + 1.0
    xs = np.concatenate([x1[: n // 2], x2[: n // 4], np.ldexp(rs.uniform(1, 2, n // 4), rs.randint(0, 1023, n // 4))])
    nums = np.concatenate([sg[: n // 2], np.ones(n // 4), rs.uniform(1, 2, n // 4) * rs.choice([-1, 1], n // 4)])
    dens = np.concatenate([den[: n // 2], np.sqrt(x2[: n // 4]), np.ldexp(rs.uniform(1, 2, n // 4), rs.randint(0, 513, n // 4))])
    assert np.isfinite(xs).all() and (xs >= 1).all() and (np.abs(dens) >= 1).all() and (np.abs(dens) < 2.0 ** 514).all()
    th = np.concatenate([theta, -theta[:8], np.array([np.inf, -np.inf, np.ldexp(1.0, 513), -np.ldexp(1.5, 600), 1e308])])
    th = np.resize(th, n) if len(th) > n else np.concatenate([th, np.zeros(n - len(th))])
    th[-5:] = [np.inf, -np.inf, np.ldexp(1.0, 513), -np.ldexp(1.5, 600), 1e308]   # theta^2 + 1 = inf: t = +-0
    sq, q, t = ctx.debug_rotation_ops(xs, nums, dens, th)
    assert np.array_equal(sq.view(np.uint64), np.sqrt(xs).view(np.uint64))
    assert np.array_equal(q.view(np.uint64), (nums / dens).view(np.uint64))
    with np.errstate(over="ignore", invalid="ignore"):
        want_t = np.where(th >= 0.0, 1.0, -1.0) / (np.abs(th) + np.sqrt(th * th + 1.0))
    assert np.array_equal(t.view(np.uint64), want_t.view(np.uint64))

"""GPU parity: RansacSE3::compute (Solver/SolverSE3.cpp:23-133) vs the CPU oracle.

Same matches, same glibc-rand seed and sticky covariance on both sides: the accepted transform
(float bits), inlier list, rmse, the RNG state afterwards, the sticky value and the F2 outlier
flags must all agree exactly (the tolerance the north star allows, 1e-4 on SE(3), is not used).
"""
import ctypes as C

import numpy as np
import pytest

from conftest import synth_seq

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frames(oracle):
    bgr, depth, poses, cam = synth_seq(5, seed=13, preset="fr1")
    p, oc = oracle.orb_params(1000), oracle.camera(cam)
    return [oracle.frame(bgr[i], depth[i], p, oc) for i in range(5)], poses


@pytest.fixture(scope="module")
def ctx(pkg):
    return pkg.Context(640, 480, max_batch=1)


def _pkg_state(pkg, orng, ost):
    r = pkg.Rng()
    C.memmove(C.byref(r), C.byref(orng), C.sizeof(r))
    s = pkg.Sticky()
    C.memmove(C.byref(s), C.byref(ost), C.sizeof(s))
    return r, s


def _compare(pkg, oracle, ctx, xyz1, xyz2, matches, seed, sticky_cov=None, n2=None, prm_args=()):
    orng = oracle.rng(seed)
    ost = oracle.Sticky()
    if sticky_cov is not None:
        ost.cov, ost.set = sticky_cov, 1
    prng, pst = _pkg_state(pkg, orng, ost)
    n2 = n2 or len(xyz2)
    of = np.zeros(n2, np.uint8)
    pf = np.zeros(n2, np.uint8)
    ok_o, T_o, inl_o, rm_o = oracle.ransac_se3(xyz1, xyz2, matches, oracle.ransac_params(*prm_args), orng, ost, of)
    ok_p, T_p, inl_p, rm_p = ctx.ransac_se3(xyz1, xyz2, matches, pkg.ransac_params(*prm_args), prng, pst, pf)
    assert ok_o == ok_p
    assert np.array_equal(T_o.view(np.uint32), T_p.view(np.uint32)), (T_o, T_p)
    assert np.array_equal(inl_o, inl_p)
    assert np.float32(rm_o).view(np.uint32) == np.float32(rm_p).view(np.uint32), (rm_o, rm_p)
    assert list(orng.state) == list(prng.state) and (orng.f, orng.r) == (prng.f, prng.r), "RNG state diverged"
    assert ost.set == pst.set and ost.cov == pst.cov
    assert np.array_equal(of, pf)
    return ok_o, T_o, len(inl_o)


def test_ransac_consecutive_frames(pkg, oracle, ctx, frames):
    fr, poses = frames
    for i in range(4):
        f0, f1 = fr[i], fr[i + 1]
        m = oracle.match(f0["desc"], f1["desc"], np.zeros(len(f0["kps"]), np.uint8), f0["xyz"][:, 2],
                         f1["xyz"][:, 2], 0.9)
        for seed in (1, 77, 12345):
            ok, T, n = _compare(pkg, oracle, ctx, f0["xyz"], f1["xyz"], m, seed)
            assert ok and n >= 10


def test_ransac_contaminated_matches(pkg, oracle, ctx, frames):
    """Many outliers: the loop runs many iterations (n += 10 / break rarely fire)."""
    fr, _ = frames
    f0, f1 = fr[0], fr[2]
    m = oracle.match(f0["desc"], f1["desc"], np.zeros(len(f0["kps"]), np.uint8), f0["xyz"][:, 2],
                     f1["xyz"][:, 2], 0.9)
    rs = np.random.default_rng(5)
    valid_t = np.flatnonzero(f1["xyz"][:, 2] > 0)
    for frac in (0.4, 0.6, 0.75):
        mm = m.copy()
        k = rs.choice(len(mm), int(frac * len(mm)), replace=False)
        mm["trainIdx"][k] = rs.choice(valid_t, len(k))
        mm["distance"][k] = rs.integers(0, 80, len(k)).astype(np.float32)
        for seed in (3, 4):
            _compare(pkg, oracle, ctx, f0["xyz"], f1["xyz"], mm, seed)


def test_ransac_sticky_preset_and_params(pkg, oracle, ctx, frames):
    fr, _ = frames
    f0, f1 = fr[1], fr[2]
    m = oracle.match(f0["desc"], f1["desc"], np.zeros(len(f0["kps"]), np.uint8), f0["xyz"][:, 2],
                     f1["xyz"][:, 2], 0.9)
    _compare(pkg, oracle, ctx, f0["xyz"], f1["xyz"], m, 9, sticky_cov=1e-4)
    _compare(pkg, oracle, ctx, f0["xyz"], f1["xyz"], m, 9, prm_args=(50, 20, 2.0, 4))
    _compare(pkg, oracle, ctx, f0["xyz"], f1["xyz"], m, 9, prm_args=(200, 10, 3.0, 6))


def test_ransac_too_few_and_fallback(pkg, oracle, ctx, frames):
    fr, _ = frames
    f0, f1 = fr[0], fr[1]
    m = oracle.match(f0["desc"], f1["desc"], np.zeros(len(f0["kps"]), np.uint8), f0["xyz"][:, 2],
                     f1["xyz"][:, 2], 0.9)
    ok, _, _ = _compare(pkg, oracle, ctx, f0["xyz"], f1["xyz"], m[:9], 2)      # < minInlierTh
    assert not ok
    # identical clouds: the identity fallback / early accept path
    _compare(pkg, oracle, ctx, f0["xyz"], f0["xyz"], np.array(
        [(i, i, 0, float(i % 7)) for i in np.flatnonzero(f0["xyz"][:, 2] > 0)[:200]], dtype=oracle.DMATCH_DTYPE), 6)
    # pure noise: nothing fits
    rs = np.random.default_rng(11)
    noise = np.array([(int(a), int(b), 0, float(d)) for a, b, d in zip(
        rs.choice(np.flatnonzero(f0["xyz"][:, 2] > 0), 120), rs.choice(np.flatnonzero(f1["xyz"][:, 2] > 0), 120),
        rs.integers(0, 60, 120))], dtype=oracle.DMATCH_DTYPE)
    _compare(pkg, oracle, ctx, f0["xyz"], f1["xyz"], noise, 8)

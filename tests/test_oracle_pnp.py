"""CPU: the PnPRansac oracle (oracle/orc_pnp.cpp) against independent formulations and geometry.

Parity of the operator itself is unpinned (OpenCV is absent; DESIGN.md "PnPRansac definition"): these
tests pin the pieces that have a published closed form -- cv::RNG's multiply-with-carry stream and
RANSACUpdateNumIters -- and check that EPnP + RANSAC + Gauss-Newton recover known poses."""
import math

import numpy as np
import pytest

from pnp_cases import K_TUM, problem


def _mwc_uniform(seed, count, n):
    """cv::RNG::next / uniform(a, b) restated independently in Python integers."""
    state = seed if seed else 0xFFFFFFFF
    out = []
    for _ in range(n):
        state = (state & 0xFFFFFFFF) * 4164903690 + (state >> 32)
        state &= (1 << 64) - 1
        out.append((state & 0xFFFFFFFF) % count)
    return out


@pytest.mark.parametrize("count", [6, 10, 137, 1000])
def test_cvrng_stream(oracle, count):
    L = oracle._pnp_sigs()
    out = np.zeros(64, np.int32)
    L.orc_cvrng_uniform_stream((1 << 64) - 1, count, 64, out)
    assert out.tolist() == _mwc_uniform((1 << 64) - 1, count, 64)


def _update_num_iters(p, ep, m, max_iters):
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, 2.2250738585072014e-308)
    denom = 1.0 - (1.0 - ep) ** m
    if denom < 2.2250738585072014e-308:
        return 0
    num, denom = math.log(num), math.log(denom)
    return max_iters if denom >= 0 or -num >= max_iters * (-denom) else int(round(num / denom))


@pytest.mark.parametrize("ep", [0.0, 0.05, 0.2, 0.3, 0.5, 0.7, 0.9, 1.0])
@pytest.mark.parametrize("max_iters", [500, 37])
def test_update_num_iters(oracle, ep, max_iters):
    L = oracle._pnp_sigs()
    assert L.orc_update_num_iters(0.85, ep, 5, max_iters) == _update_num_iters(0.85, ep, 5, max_iters)


def test_update_num_iters_table(oracle):
    L = oracle._pnp_sigs()
    # log(0.15) / log(1 - 0.8^5) = 4.99 -> 5 ; inlier ratio 0.5 -> 60
    assert L.orc_update_num_iters(0.85, 0.2, 5, 500) == 5
    assert L.orc_update_num_iters(0.85, 0.5, 5, 500) == 60
    assert L.orc_update_num_iters(0.85, 0.0, 5, 500) == 0


@pytest.mark.parametrize("seed", range(4))
def test_epnp_exact_on_clean_points(oracle, seed):
    P, uv, R, t, _ = problem(5, seed, outliers=0.0, noise=0.0)
    ok, Re, te = oracle.epnp(P, uv, K_TUM)
    assert ok
    assert np.abs(Re - R).max() < 1e-4 and np.abs(te - t).max() < 1e-4
    assert abs(np.linalg.det(Re) - 1) < 1e-9


@pytest.mark.parametrize("n,outl,seed", [(60, 0.0, 1), (200, 0.3, 2), (500, 0.5, 3), (1200, 0.2, 4)])
def test_pnp_ransac_recovers_pose(oracle, n, outl, seed):
    P, uv, R, t, inl = problem(n, seed, outliers=outl)
    ok, Re, te, mask, ni, iters = oracle.pnp_ransac(P, uv, K_TUM)
    assert ok and ni == mask.sum() and 1 <= iters <= 500
    assert np.abs(Re - R).max() < 2e-3 and np.abs(te - t).max() < 5e-3
    # RANSAC inliers: (nearly) all true inliers, no gross outlier
    assert (mask & ~inl).sum() <= max(1, n // 100)
    assert mask[inl].mean() > 0.85   # the mask is the best minimal model's, not the refined one


def test_pnp_ransac_edges(oracle):
    P, uv, R, t, _ = problem(5, 7, outliers=0.0, noise=0.0)
    ok, *_ = oracle.pnp_ransac(P[:4], uv[:4], K_TUM)
    assert not ok
    ok, Re, te, mask, ni, iters = oracle.pnp_ransac(P, uv, K_TUM)   # count == modelPoints: one fit, all inliers
    assert ok and iters == 0 and ni == 5 and mask.all()
    assert np.abs(Re - R).max() < 1e-6
    same = np.repeat(P[:1], 20, 0)                                  # degenerate: control points singular
    ok, *_ = oracle.pnp_ransac(same, np.repeat(uv[:1], 20, 0), K_TUM)
    assert not ok

"""CPU: the GICP oracle (oracle/orc_gicp.cpp) against an independent numpy formulation of PCL's
covariance stage and against known rigid motions.  Parity with PCL's BFGS optimiser is unpinned
(PCL is absent; DESIGN.md "GICP"); the correspondence / covariance / convergence rules are restated."""
import numpy as np
import pytest

from gicp_cases import clouds


def _np_covariances(P, k=20, eps=1e-3):
    P32 = P.astype(np.float32)
    out = []
    for i in range(len(P32)):
        d = P32 - P32[i]
        d2 = (((np.float32(0) + d[:, 0] * d[:, 0]) + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]).astype(np.float32)
        nn = np.lexsort((np.arange(len(P32)), d2))[:k]
        X = P32[nn]
        mu = X.astype(np.float64).sum(0) / k
        # PCL accumulates float products (pt.y * pt.x) into double sums
        S = np.array([[(X[:, a] * X[:, b]).astype(np.float64).sum() for b in range(3)] for a in range(3)])
        C = S / k - np.outer(mu, mu)
        w, V = np.linalg.eigh(C)
        out.append(V @ np.diag([eps, 1.0, 1.0]) @ V.T)
    return np.array(out)


@pytest.mark.parametrize("n,seed", [(40, 1), (150, 2)])
def test_covariances_match_independent(oracle, n, seed):
    P, _, _ = clouds(n, seed)
    ok, C = oracle.gicp_covariances(P)
    assert ok
    np.testing.assert_allclose(C, _np_covariances(P), atol=1e-9)


def test_covariances_refuse_small_cloud(oracle):
    P, _, _ = clouds(19, 3)
    ok, _ = oracle.gicp_covariances(P)
    assert not ok


@pytest.mark.parametrize("n,seed,outl", [(60, 4, 0.0), (300, 5, 0.0), (300, 6, 0.1), (800, 7, 0.05)])
def test_gicp_recovers_motion(oracle, n, seed, outl):
    P, Q, T = clouds(n, seed, outliers=outl)
    for guess in (np.eye(4, dtype=np.float32), T.astype(np.float32)):
        conv, Te, it, nc = oracle.gicp(P, Q, guess)
        assert conv and 1 <= it <= 10 and nc >= 4
        assert np.abs(Te[:3, :3] - T[:3, :3]).max() < 5e-3 and np.abs(Te[:3, 3] - T[:3, 3]).max() < 5e-3


def test_gicp_compute_rules(oracle):
    P, Q, T = clouds(100, 8)
    ok, Te = oracle.gicp_compute(P[:19], Q[:19], np.eye(4, dtype=np.float32))
    assert not ok and np.array_equal(Te, np.eye(4, dtype=np.float32))          # < 20 matches
    ok, Te = oracle.gicp_compute(P, Q, np.eye(4, dtype=np.float32))
    assert ok
    ok, Te = oracle.gicp_compute(P, P, np.eye(4, dtype=np.float32))             # result == identity -> false
    assert not ok
    far = np.eye(4, dtype=np.float32)
    far[:3, 3] = 5.0                                                            # no correspondence -> unconverged
    conv, Te, it, nc = oracle.gicp(P, Q, far)
    assert not conv and nc < 4

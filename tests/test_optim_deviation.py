"""How far the device optimisers lie from the ones they replace (north_star's SE(3)
tolerance 1e-4).  The device PnP refinement and GICP step are Gauss-Newton; the
oracle's restatements (oracle/orc_pnp.cpp, oracle/orc_gicp.cpp) equal the device bit for bit (the -m gpu
tests), so the Gauss-Newton side is taken from the oracle here and compared with restatements of
OpenCV's solvePnP(ITERATIVE) Levenberg-Marquardt (Solver/PnPRansac.cpp:39) and PCL's GICP BFGS
(Solver/Gicp.cpp:54-66) in oracle/optim_ref.py, started from the same RANSAC model / guess.
Measured maxima (this file's cases): PnP 2.4e-11, GICP 1.2e-5 -- the noise-limited error against the
ground truth is ~1e-3 for both.  Parity of the restatements themselves is unpinned (neither OpenCV nor
PCL is importable offline)."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))

import gicp_cases  # noqa: E402
import oracle_lib as O  # noqa: E402
import optim_ref as Q  # noqa: E402
import pnp_cases  # noqa: E402

TOL = 1e-4   # north_star: SE(3) element tolerance


def _T(R, t):
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return T


@pytest.mark.parametrize("n,seed,outliers", [(30, 0, 0.3), (100, 1, 0.3), (400, 2, 0.3), (1000, 3, 0.3),
                                             (200, 4, 0.5), (600, 5, 0.1)])
def test_pnp_gauss_newton_vs_levenberg_marquardt(n, seed, outliers):
    K4 = pnp_cases.K_TUM
    P, uv, _, _, _ = pnp_cases.problem(n, seed, outliers=outliers)
    ok, R, t, mask, ni, _ = O.pnp_ransac(P, uv, K4)                 # device definition: RANSAC + 10 GN steps
    ok0, R0, t0, m0 = O.pnp_ransac_model(P, uv, K4)                 # the RANSAC model both refinements start at
    assert ok and ok0 and np.array_equal(mask, m0) and ni >= 6
    Rl, tl, _ = Q.solvepnp_lm(P[m0], uv[m0], K4, R0, t0)
    d = Q.se3_max_diff(_T(R, t), _T(Rl, tl))
    assert d < TOL, f"GN vs LM {d:.3e}"


@pytest.mark.parametrize("n,seed,outliers,motion", [(60, 0, 0.0, (0.02, 0.015)), (200, 1, 0.0, (0.02, 0.015)),
                                                    (600, 2, 0.0, (0.02, 0.015)), (300, 3, 0.05, (0.03, 0.02)),
                                                    (400, 4, 0.0, (0.01, 0.01))])
def test_gicp_gauss_newton_vs_bfgs(n, seed, outliers, motion):
    src, tgt, _ = gicp_cases.clouds(n, seed, outliers=outliers, motion=motion)
    guess = np.eye(4, dtype=np.float32)
    cv, Tg, _, _ = O.gicp(src, tgt, guess)                          # device definition
    _, cs = O.gicp_covariances(src)
    _, ct = O.gicp_covariances(tgt)
    cb, Tb, _ = Q.gicp_pcl_bfgs(src, tgt, guess, cs, ct)
    assert cv and cb
    d = Q.se3_max_diff(Tg, Tb)
    assert d < TOL, f"GN vs BFGS {d:.3e}"

"""Seeded synthetic GICP problems (test infrastructure): surface-like clouds (planes + a box) with a
known rigid motion, per-point noise, and an optional fraction of gross outliers."""
import numpy as np

from pnp_cases import rot


def clouds(n, seed, noise=0.003, outliers=0.0, motion=(0.02, 0.015)):
    rs = np.random.default_rng(seed)
    k = n // 3
    a = np.c_[rs.uniform(-1, 1, k), rs.uniform(-0.8, 0.8, k), 2.2 + 0.01 * rs.normal(size=k)]
    b = np.c_[rs.uniform(-1, 1, k), 0.9 + 0.01 * rs.normal(size=k), rs.uniform(1.2, 3.0, k)]
    m = n - 2 * k
    c = np.c_[-0.7 + 0.01 * rs.normal(size=m), rs.uniform(-0.8, 0.8, m), rs.uniform(1.2, 3.0, m)]
    P = np.concatenate([a, b, c]).astype(np.float32)
    R = rot(rs.normal(size=3) * motion[0])
    t = rs.normal(size=3) * motion[1]
    Q = P.astype(np.float64) @ R.T + t + rs.normal(size=P.shape) * noise
    bad = rs.random(n) < outliers
    Q[bad] += rs.uniform(-0.5, 0.5, size=(int(bad.sum()), 3))
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return P, Q.astype(np.float32), T

"""Seeded synthetic solvePnPRansac problems (test infrastructure): object points in front of a camera,
a random pose, pixel noise and a fraction of gross outliers."""
import numpy as np

K_TUM = np.array([517.3, 516.5, 318.6, 255.3], np.float32)


def rot(w):
    th = np.linalg.norm(w)
    if th == 0:
        return np.eye(3)
    k = w / th
    Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx


def problem(n, seed, outliers=0.3, noise=0.5, K4=K_TUM):
    rs = np.random.default_rng(seed)
    P = rs.uniform([-1.5, -1.2, 0.8], [1.5, 1.2, 4.5], size=(n, 3)).astype(np.float32)
    R = rot(rs.normal(size=3) * 0.15)
    t = rs.normal(size=3) * 0.15
    Xc = P.astype(np.float64) @ R.T + t
    uv = np.stack([K4[0] * Xc[:, 0] / Xc[:, 2] + K4[2], K4[1] * Xc[:, 1] / Xc[:, 2] + K4[3]], 1)
    uv += rs.normal(size=uv.shape) * noise
    out = rs.random(n) < outliers
    uv[out] += rs.uniform(-80, 80, size=(int(out.sum()), 2))
    return P, uv.astype(np.float32), R, t, ~out

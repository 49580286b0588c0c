"""Absolute trajectory error (TUM evaluate_ate.py semantics): rigid Horn alignment of the
estimated camera centres to ground truth (no scale), RMSE of the residual translations.
Also writes TUM trajectory lines (System/Tracking.cpp:286-317 format: t tx ty tz qx qy qz qw)."""
from __future__ import annotations

import numpy as np


def centres(Tcw: np.ndarray) -> np.ndarray:
    R = Tcw[:, :3, :3].astype(np.float64)
    t = Tcw[:, :3, 3].astype(np.float64)
    return -np.einsum("nji,nj->ni", R, t)      # twc = -R^T t


def align(model: np.ndarray, data: np.ndarray):
    """R, t minimising |R model + t - data| (Horn 1987 / evaluate_ate.align)."""
    mu_m, mu_d = model.mean(0), data.mean(0)
    W = (data - mu_d).T @ (model - mu_m)
    U, _, Vt = np.linalg.svd(W)
    S = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[2, 2] = -1
    R = U @ S @ Vt
    return R, mu_d - R @ mu_m


def ate_rmse(est_Tcw: np.ndarray, gt_Tcw: np.ndarray) -> float:
    e, g = centres(est_Tcw), centres(gt_Tcw)
    R, t = align(e, g)
    err = (e @ R.T + t) - g
    return float(np.sqrt(np.mean(np.sum(err * err, axis=1))))


def quat_from_R(R: np.ndarray):
    w = np.sqrt(max(0.0, 1 + R[0, 0] + R[1, 1] + R[2, 2])) / 2
    x = np.sqrt(max(0.0, 1 + R[0, 0] - R[1, 1] - R[2, 2])) / 2
    y = np.sqrt(max(0.0, 1 - R[0, 0] + R[1, 1] - R[2, 2])) / 2
    z = np.sqrt(max(0.0, 1 - R[0, 0] - R[1, 1] + R[2, 2])) / 2
    x = np.copysign(x, R[2, 1] - R[1, 2])
    y = np.copysign(y, R[0, 2] - R[2, 0])
    z = np.copysign(z, R[1, 0] - R[0, 1])
    return x, y, z, w


def tum_lines(times, Tcw):
    lines = []
    for t, T in zip(times, Tcw):
        Rwc = T[:3, :3].T.astype(np.float64)
        twc = -Rwc @ T[:3, 3].astype(np.float64)
        q = quat_from_R(Rwc)
        lines.append("%.6f %.9f %.9f %.9f %.9f %.9f %.9f %.9f" % ((t,) + tuple(twc) + q))
    return lines

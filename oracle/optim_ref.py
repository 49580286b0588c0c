"""TEST INFRASTRUCTURE ONLY (imported by tests/, never by the product): restatements of the two optimisers
the device path replaces with Gauss-Newton, used to MEASURE how far the device results lie from them
(north_star's SE(3) tolerance 1e-4):

* OpenCV 3.4 ``solvePnP(SOLVEPNP_ITERATIVE, useExtrinsicGuess=true)`` on the RANSAC inliers, the refinement
  inside ``cv::solvePnPRansac`` (Solver/PnPRansac.cpp:39): ``cvFindExtrinsicCameraParams2``'s ``CvLevMarq``
  over (rvec, tvec) -- lambda = 10^lambdaLg10 starting at -3, JtJ diagonal scaled by (1 + lambda), the step
  solved by SVD, a rejected step raises lambdaLg10 and retries, an accepted one lowers it, stop after 20
  iterations or when |param - prevParam| / |param| < FLT_EPSILON.  The Jacobian of cvProjectPoints2 is
  taken by central differences in double (h = 1e-7), which moves the iterates by far less than the
  tolerance measured here.
* PCL 1.8 ``GeneralizedIterativeClosestPoint::computeTransformation`` with its per-iteration
  ``estimateRigidTransformationBFGS`` (Solver/Gicp.cpp:54-66): outer loop of nearest-neighbour
  correspondences (< max_corr^2), Mahalanobis M_i = (R C_src R^T + C_tgt)^-1 with R of
  transformation_ * guess, then BFGS over x = (tx, ty, tz, roll, pitch, yaw) (R = Rz(yaw) Ry(pitch)
  Rx(roll), Eigen AngleAxis order) as an increment on transformation_, of f(x) = mean_i r_i^T M_i r_i
  with PCL's analytic gradient, at most 20 inner iterations and testGradient(gicp_epsilon = 1e-3);
  delta = max(|dR| / rotation_epsilon, |dt| / transformation_epsilon); converged when delta < 1 or
  after max_iterations.  PCL's BFGS is Eigen's unsupported BFGS with a More-Thuente line search; here
  it is scipy's BFGS (a Wolfe line search) with the same caps -- both minimise the same f.

Neither library is importable here, so these are restatements of their published algorithms, not
bit-exact copies; what the tests report is the distance between the device's Gauss-Newton result and
the optimum these restatements reach from the same start.
"""
import numpy as np

FLT_EPSILON = np.finfo(np.float32).eps


# ----------------------------------------------------------------------------------------- PnP (LM)
def rodrigues(r):
    th = float(np.linalg.norm(r))
    if th < 1e-300:
        return np.eye(3)
    k = r / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) * np.cos(th) + (1 - np.cos(th)) * np.outer(k, k) + np.sin(th) * K


def rodrigues_inv(R):
    c = np.clip((np.trace(R) - 1) / 2, -1.0, 1.0)
    th = np.arccos(c)
    if th < 1e-12:
        return np.zeros(3)
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    if np.pi - th < 1e-6:   # near pi: axis from the symmetric part
        A = (R + np.eye(3)) / 2
        k = np.sqrt(np.maximum(np.diag(A), 0))
        k *= np.sign(w + (w == 0))
        return th * k / np.linalg.norm(k)
    return th * w / (2 * np.sin(th))


def _project(P, param, K4):
    R = rodrigues(param[:3])
    X = P @ R.T + param[3:]
    return np.stack([K4[0] * X[:, 0] / X[:, 2] + K4[2], K4[1] * X[:, 1] / X[:, 2] + K4[3]], 1).reshape(-1)


def solvepnp_lm(p3, p2, K4, R0, t0, max_iter=20, eps=FLT_EPSILON):
    """cvFindExtrinsicCameraParams2's CvLevMarq refinement from (R0, t0); returns (R, t, iterations)."""
    P = np.asarray(p3, np.float64)
    m = np.asarray(p2, np.float64).reshape(-1)
    K4 = np.asarray(K4, np.float64)
    param = np.concatenate([rodrigues_inv(np.asarray(R0, np.float64)), np.asarray(t0, np.float64)])

    def err_of(x):
        return _project(P, x, K4) - m

    def jac(x):
        J = np.zeros((len(m), 6))
        for j in range(6):
            h = 1e-7 * max(1.0, abs(x[j]))
            a, b = x.copy(), x.copy()
            a[j] += h
            b[j] -= h
            J[:, j] = (_project(P, a, K4) - _project(P, b, K4)) / (2 * h)
        return J

    lam_lg10 = -3
    iters = 0
    err = err_of(param)
    prev_norm = np.linalg.norm(err)
    while True:
        J = jac(param)
        JtJ, JtE = J.T @ J, J.T @ err
        prev = param.copy()
        while True:
            A = JtJ.copy()
            A[np.diag_indices(6)] *= 1.0 + 10.0 ** lam_lg10
            delta = np.linalg.lstsq(A, JtE, rcond=None)[0]   # DECOMP_SVD
            param = prev - delta
            err = err_of(param)
            norm = np.linalg.norm(err)
            if norm > prev_norm and lam_lg10 < 16:
                lam_lg10 += 1
                continue
            break
        lam_lg10 = max(lam_lg10 - 1, -16)
        iters += 1
        if iters >= max_iter or np.linalg.norm(param - prev) < eps * np.linalg.norm(param):
            break
        prev_norm = norm
    return rodrigues(param[:3]), param[3:].copy(), iters


# ---------------------------------------------------------------------------------------- GICP (BFGS)
def rpy_to_R(r, p, y):
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    return Rz @ Ry @ Rx


def T_of(x):
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = rpy_to_R(x[3], x[4], x[5]).astype(np.float32)
    T[:3, 3] = np.asarray(x[:3], np.float32)
    return T


def x_of(T):
    return np.array([T[0, 3], T[1, 3], T[2, 3], np.arctan2(T[2, 1], T[2, 2]), np.arcsin(-np.clip(T[2, 0], -1, 1)),
                     np.arctan2(T[1, 0], T[0, 0])], np.float64)


def _dR(r, p, y):
    """d(Rz(y) Ry(p) Rx(r)) / d(r, p, y)."""
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    dRz = np.array([[-sy, -cy, 0], [cy, -sy, 0], [0, 0, 0]])
    dRy = np.array([[-sp, 0, cp], [0, 0, 0], [-cp, 0, -sp]])
    dRx = np.array([[0, 0, 0], [0, -sr, -cr], [0, cr, -sr]])
    return Rz @ Ry @ dRx, Rz @ dRy @ Rx, dRz @ Ry @ Rx


def gicp_pcl_bfgs(src, tgt, guess, cov_src, cov_tgt, max_iterations=10, max_corr=0.07, transformation_epsilon=1e-9,
                  rotation_epsilon=2e-3, gicp_epsilon=1e-3, max_inner=20):
    """PCL GICP align restated with its BFGS step; cov_* = the clouds' GICP covariances (n x 3 x 3).
    The BFGS state is the increment x = (t, rpy) on the current transformation_ (applyState:
    R <- R(x) R, t <- t + x_t), f and its analytic gradient as PCL's OptimizationFunctorWithIndices (points
    transformed in float, sums in double), stopped by PCL's testGradient(|g| < gicp_epsilon) or after
    max_inner iterations.  Returns (converged, final 4x4 float32 = transformation_ * guess, outer iterations)."""
    from scipy.optimize import minimize
    src = np.asarray(src, np.float32)
    tgt = np.asarray(tgt, np.float32)
    guess = np.asarray(guess, np.float32)
    out = (src @ guess[:3, :3].T + guess[:3, 3]).astype(np.float32)   # transformPointCloud(output, guess)
    T = np.eye(4, dtype=np.float32)
    thr = max_corr * max_corr
    it = 0
    while True:
        R = (T.astype(np.float64) @ guess.astype(np.float64))[:3, :3]
        q = (out @ T[:3, :3].T + T[:3, 3]).astype(np.float32)
        d2 = ((q[:, None, :] - tgt[None, :, :]) ** 2).sum(-1)
        nn = np.argmin(d2, 1)
        ok = d2[np.arange(len(q)), nn] < thr
        si, ti = np.nonzero(ok)[0], nn[ok]
        if len(si) < 4:
            return False, np.eye(4, dtype=np.float32), it
        M = np.linalg.inv(R @ cov_src[si] @ R.T + cov_tgt[ti])
        ps, pt = out[si].astype(np.float32), tgt[ti].astype(np.float64)
        base = T.copy()

        def state(x):
            Tx = base.copy()
            Tx[:3, :3] = (rpy_to_R(x[3], x[4], x[5]).astype(np.float32) @ base[:3, :3]).astype(np.float32)
            Tx[:3, 3] = base[:3, 3] + np.asarray(x[:3], np.float32)
            return Tx

        def fg(x):
            Tx = state(x)
            pp = (ps @ Tx[:3, :3].T + Tx[:3, 3]).astype(np.float64)
            r = pp - pt
            tmp = np.einsum('nij,nj->ni', M, r)
            f = float((r * tmp).sum() / len(si))
            g = np.zeros(6)
            g[:3] = 2.0 * tmp.sum(0) / len(si)
            Rm = 2.0 * (ps.astype(np.float64).T @ tmp) / len(si)   # sum p_src temp^T (PCL: untransformed p)
            Rb = base[:3, :3].astype(np.float64)
            for k, D in enumerate(_dR(x[3], x[4], x[5])):
                g[3 + k] = float(np.sum((D @ Rb) * Rm.T))
            return f, g

        prev = T.copy()
        res = minimize(fg, np.zeros(6), jac=True, method="BFGS",
                       options={"maxiter": max_inner, "gtol": gicp_epsilon, "norm": 2})
        T = state(res.x)
        delta = max((np.abs(prev[:3, :3] - T[:3, :3]) / rotation_epsilon).max(),
                    (np.abs(prev[:3, 3] - T[:3, 3]) / transformation_epsilon).max())
        it += 1
        if it >= max_iterations or delta < 1:
            return True, (T.astype(np.float64) @ guess.astype(np.float64)).astype(np.float32), it


def se3_max_diff(A, B):
    """max |element| difference of the [R | t] blocks (the north star's SE(3) tolerance measure)."""
    A, B = np.asarray(A, np.float64), np.asarray(B, np.float64)
    return float(np.abs(A[:3, :4] - B[:3, :4]).max())

"""Keyframe pose graph (Solver/PoseGraph.cpp) over the C ABI's host optimiser (rgbd_pg_*), with the
reference's keyframe policy (Tracking::needKeyFrame, System/Tracking.cpp:201-225) and the local-edge
search that reuses the device Matcher + RansacSE3 (PoseGraph::createLocalEdges, :128-182):

  insert_keyframe  <- PoseGraph::updateGraph (:105-126) without loop detection: node, edge with the
                      reference keyframe (setMeasurementFromState), local edges to the keyframes whose
                      camera centres lie within 0.5 m (Matcher(0.9) >= 30 matches, RansacSE3(200, 30,
                      3.0f, 4).compute(pKFi, cur, matches, updateF2=false), measurement mT21)
  optimize         <- PoseGraph::optimize (:368-386): vertex 0 fixed, LM, corrected poses
Loop closure needs the DBoW3 vocabulary (PlaceRecognition/LoopDetector), which is absent: out of
scope.  Keyframe features are those of the keyframe's own extraction, with the
outlier flags all clear (the reference reads the flags its tracking left; DESIGN.md deviations), and
the pose graph owns its RNG / RansacSE3 sticky state (the reference shares the process-global ones
with the tracking thread).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

MIN_T, MIN_R = 0.20, 0.1745          # Tracking::needKeyFrame (:217-218)
RADIUS, MATCHES_TH = 0.50, 30        # PoseGraph::nearestNodes / createLocalEdges (:130, :160)
INFO, HUBER = 100.0, 1.0             # EdgeSE3 information 100 I, RobustKernelHuber() delta 1 (:203-204)


def tnorm(T):
    """Tracking.cpp:201-205: |t| of the 4x4 (float Mat, cv::norm: double sums in order)."""
    t = [float(v) for v in np.asarray(T, np.float32)[:3, 3]]
    return float(np.sqrt((t[0] * t[0] + t[1] * t[1]) + t[2] * t[2]))


def rnorm(T):
    """Tracking.cpp:207-211: acos(0.5 * (R00 + R11 + R22 - 1.0)): the three float entries add in float,
    the rest in double."""
    R = np.asarray(T, np.float32)
    c = 0.5 * (float(np.float32(np.float32(R[0, 0] + R[1, 1]) + R[2, 2])) - 1.0)
    return float(np.arccos(c)) if abs(c) <= 1.0 else float("nan")


def mat_mul(A, B):
    """cv::Mat CV_32F product (gemm: double accumulation in k order, one rounding)."""
    A = np.asarray(A, np.float32).astype(np.float64)
    B = np.asarray(B, np.float32).astype(np.float64)
    C = np.zeros((A.shape[0], B.shape[1]), np.float64)
    for k in range(A.shape[1]):
        C += A[:, k:k + 1] * B[k:k + 1, :]
    return C.astype(np.float32)


def pose_inverse(Tcw):
    """Frame::getPoseInverse (Core/Frame.cpp:137-153): [R^T | -R^T t] in float, the translation one gemm."""
    T = np.asarray(Tcw, np.float32)
    Ti = np.eye(4, dtype=np.float32)
    Ti[:3, :3] = T[:3, :3].T
    for i in range(3):
        s = 0.0
        for k in range(3):
            s += float(T[k, i]) * float(T[k, 3])
        Ti[i, 3] = np.float32(s * -1.0)
    return Ti


def need_keyframe(Tcw_cur, Tcw_lastkf):
    """Tracking::needKeyFrame: delta = cur.getPoseInverse() * lastKF.getPose() (float Mat product)."""
    delta = mat_mul(pose_inverse(Tcw_cur), Tcw_lastkf)
    return tnorm(delta) > MIN_T or rnorm(delta) > MIN_R   # a NaN angle compares false, as acos in C++


def select_keyframes(poses):
    """Frame indices that become keyframes when frames are tracked in order (the first always)."""
    kfs = [0] if len(poses) else []
    for i in range(1, len(poses)):
        if need_keyframe(poses[i], poses[kfs[-1]]):
            kfs.append(i)
    return kfs


class PoseGraph:
    def __init__(self, pkg, ctx=None, seed: int = 0):
        self.pkg = pkg
        self.ctx = ctx                      # device Matcher + RansacSE3 for local edges (None: no local edges)
        h = C.c_void_p()
        self._check(pkg.lib().rgbd_pg_create(C.byref(h)), "rgbd_pg_create")
        self._h = h
        self.kf = {}                        # id -> dict(Tcw, xyz, desc)
        self.ref = None
        self.rng = pkg.rng(seed)
        self.sticky = pkg.Sticky()
        self.prm = pkg.ransac_params(200, MATCHES_TH, 3.0, 4)
        self.edges = []                     # (from, to, Z or None) in insertion order (parity tests)
        self.attempts = []                  # local-edge attempts: (kf, cur, matches, RansacSE3 result or None)

    def _check(self, st, what):
        if st != 0:
            raise self.pkg.RgbdError(f"{what}: status {st}")

    def close(self):
        if self._h:
            self.pkg.lib().rgbd_pg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- graph primitives
    def add_vertex(self, kid: int, Tcw, fixed: bool = False):
        Twc = np.linalg.inv(np.asarray(Tcw, np.float32).astype(np.float64))   # Converter::toSE3Quat(getPoseInverse())
        Twc = np.ascontiguousarray(Twc, np.float64)
        self._check(self.pkg.lib().rgbd_pg_add_vertex(self._h, kid, Twc.ctypes.data, int(fixed)), "add_vertex")

    def add_edge(self, frm: int, to: int, Z=None) -> float:
        chi2 = C.c_double(0)
        Zp = None
        if Z is not None:
            Zm = np.ascontiguousarray(np.asarray(Z, np.float64))
            Zp = Zm.ctypes.data
        self._check(self.pkg.lib().rgbd_pg_add_edge(self._h, frm, to, Zp, INFO, HUBER, C.byref(chi2)), "add_edge")
        self.edges.append((frm, to, None if Z is None else np.array(Z, np.float64)))
        return chi2.value

    def exist_edge(self, a: int, b: int) -> bool:
        return bool(self.pkg.lib().rgbd_pg_exist_edge(self._h, a, b))

    def counts(self):
        v, e = C.c_int32(0), C.c_int32(0)
        self._check(self.pkg.lib().rgbd_pg_counts(self._h, C.byref(v), C.byref(e)), "counts")
        return v.value, e.value

    def chi2(self) -> float:
        c = C.c_double(0)
        self._check(self.pkg.lib().rgbd_pg_chi2(self._h, C.byref(c)), "chi2")
        return c.value

    def vertex_twc(self, kid: int):
        """The vertex estimate as the optimiser holds it (Twc, double 4x4)."""
        Twc = np.zeros(16, np.float64)
        self._check(self.pkg.lib().rgbd_pg_vertex(self._h, kid, Twc.ctypes.data), "vertex")
        return Twc.reshape(4, 4)

    def pose(self, kid: int):
        """Tcw of keyframe kid from the vertex estimate (Frame::correctPose: inverse, cast to float)."""
        Twc = np.zeros(16, np.float64)
        self._check(self.pkg.lib().rgbd_pg_vertex(self._h, kid, Twc.ctypes.data), "vertex")
        return np.linalg.inv(Twc.reshape(4, 4)).astype(np.float32)

    # ---- PoseGraph::updateGraph without loop detection
    def insert_keyframe(self, kid: int, Tcw, xyz=None, desc=None):
        self.add_vertex(kid, Tcw, fixed=(kid == 0))                   # createNode
        if self.ref is not None:
            self.add_edge(kid, self.ref)                               # createEdgeWithReference
        self.kf[kid] = dict(Tcw=np.asarray(Tcw, np.float32), xyz=xyz, desc=desc)
        if self.ctx is not None and xyz is not None:
            self._local_edges(kid)
        self.ref = kid

    def _centre(self, kid):
        T = self.kf[kid]["Tcw"].astype(np.float64)
        return -T[:3, :3].T @ T[:3, 3]

    def _local_edges(self, cur: int):
        """createLocalEdges: keyframes within RADIUS of the current centre (radiusSearch), in id order."""
        oc = self._centre(cur)
        c = self.kf[cur]
        for kid in sorted(self.kf):
            if kid == cur or self.exist_edge(cur, kid):
                continue
            if np.sum((self._centre(kid) - oc) ** 2) > RADIUS * RADIUS:
                continue
            k = self.kf[kid]
            m = self.ctx.match(k["desc"], c["desc"], np.zeros(len(k["desc"]), np.uint8), k["xyz"][:, 2],
                               c["xyz"][:, 2], 0.9)
            if len(m) < MATCHES_TH:
                self.attempts.append((kid, cur, m, None))
                continue
            ok, T21, inl, rmse = self.ctx.ransac_se3(k["xyz"], c["xyz"], m, self.prm, self.rng, self.sticky)
            self.attempts.append((kid, cur, m, dict(ok=ok, T21=T21.copy(), inliers=inl, rmse=rmse,
                                                    rng=list(self.rng.state) + [self.rng.f, self.rng.r],
                                                    sticky=(self.sticky.cov, self.sticky.set))))
            if not ok:
                continue
            self.add_edge(cur, kid, T21.astype(np.float64))          # createEdge(pKFi, SE3Quat(mT21))

    def optimize(self, iterations: int = 10):
        """PoseGraph::optimize: only with more than 5 vertices (:372), vertex 0 fixed."""
        v, _ = self.counts()
        if v <= 5:
            return None
        for kid in self.kf:
            self._check(self.pkg.lib().rgbd_pg_set_fixed(self._h, kid, int(kid == 0)), "set_fixed")
        chi2, done = C.c_double(0), C.c_int32(0)
        self._check(self.pkg.lib().rgbd_pg_optimize(self._h, iterations, C.byref(chi2), C.byref(done)), "optimize")
        for kid in self.kf:                                            # Frame::correctPose
            self.kf[kid]["Tcw"] = self.pose(kid)
        return chi2.value, done.value


def corrected_trajectory(poses, kfs, kf_poses):
    """Tracking::saveCameraTrajectory (System/Tracking.cpp:286-317): every frame's pose is stored
    relative to its reference keyframe (Tcr = Tcw * Tcw_kf^-1 at tracking time) and re-anchored on the
    keyframe's corrected pose."""
    out = np.array(poses, np.float32, copy=True)
    kf_of = np.zeros(len(poses), np.int64)
    j = 0
    for i in range(len(poses)):
        while j + 1 < len(kfs) and kfs[j + 1] <= i:
            j += 1
        kf_of[i] = kfs[j]
    for i in range(len(poses)):
        k = kf_of[i]
        Tcr = np.asarray(poses[i], np.float64) @ np.linalg.inv(np.asarray(poses[k], np.float64))
        out[i] = (Tcr @ np.asarray(kf_poses[k], np.float64)).astype(np.float32)
    return out


def posegraph_sequence(pkg, get_frame, camera: dict, poses, nfeatures: int = 1000, iterations: int = 10,
                       device: int = 0, W: int = 640, H: int = 480, record: dict | None = None):
    """The PoseGraph thread over a tracked sequence: keyframes by Tracking::needKeyFrame, each inserted
    with its own features (extracted again on the device: rgbd_frame), local edges by the device
    Matcher + RansacSE3, then PoseGraph::shutdown's optimize(); returns the corrected trajectory
    (saveCameraTrajectory re-anchoring), the keyframe ids and (vertices, edges, chi2 before, chi2 after)."""
    c = pkg.camera(camera["fx"], camera["fy"], camera["cx"], camera["cy"], camera["k1"], camera["k2"],
                   camera["p1"], camera["p2"], camera["k3"], camera["factor"])
    ctx = pkg.Context(W, H, max_batch=1, orb=pkg.orb_params(nfeatures), cam=c, device=device)
    g = PoseGraph(pkg, ctx)
    try:
        kfs = select_keyframes(poses)
        for k in kfs:
            bgr, depth = get_frame(k)
            f = ctx.frame(bgr, depth)
            g.insert_keyframe(k, poses[k], xyz=f["xyz"], desc=f["desc"])
        v, e = g.counts()
        chi_before = g.chi2()
        if record is not None:   # the graph as built (parity tests): vertices (Twc), edges, local-edge attempts
            record.update(vertices={k: g.vertex_twc(k) for k in kfs},
                          edges=list(g.edges), attempts=list(g.attempts),
                          features={k: dict(g.kf[k]) for k in kfs})
        res = g.optimize(iterations)
        chi_after = res[0] if res else chi_before
        kf_poses = {k: g.kf[k]["Tcw"] for k in kfs}
        return corrected_trajectory(poses, kfs, kf_poses), kfs, (v, e, chi_before, chi_after)
    finally:
        g.close()
        ctx.close()

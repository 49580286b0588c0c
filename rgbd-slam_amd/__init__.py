"""rgbd-slam_amd -- MI355X (gfx950) RGB-D tracking front end, Python host binding.

ctypes binding of build/librgbd_hip.so (C ABI: include/rgbd_hip.h) plus thin classes
that mirror the reference's operator surfaces for this path:

  ORBextractor.detect_and_compute  <- Extractor::detectAndCompute  Features/Extractor.h:40
  Frame(bgr, depth, extractor)     <- Frame::Frame                 Core/Frame.cpp:34-73
  Matcher(nnratio).match(ref, cur) <- Matcher::match               Features/Matcher.cpp:106-139
  RansacSE3(...).compute(F1, F2, m) <- RansacSE3::compute          Solver/SolverSE3.cpp:23-133

The GPU library is mandatory: there is no CPU fallback.  Importing works without a GPU
(the library loads and exports its symbols); any compute call needs a HIP device and
raises RgbdError otherwise.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
# RGBD_HIP_LIB selects another in-tree build of the same library (e.g. build_prof/, the profiling variant)
LIB_PATH = os.environ.get("RGBD_HIP_LIB") or os.path.join(PKG_DIR, "build", "librgbd_hip.so")
HEADER = os.path.join(ROOT, "include", "rgbd_hip.h")

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
DMATCH_DTYPE = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("imgIdx", "<i4"), ("distance", "<f4")])


POINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("b", "u1"), ("g", "u1"), ("r", "u1"),
                        ("pad", "u1")])   # rgbd_point = pcl::PointXYZRGB payload


class RgbdError(RuntimeError):
    pass


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class Camera(C.Structure):
    _fields_ = [(n, C.c_float) for n in ("fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2", "k3",
                                         "depth_map_factor")]


class SvoParams(C.Structure):
    """rgbd_svo_params: Extractor(SVO, BRIEF, NORMAL), the reference's default (main.cpp:31)."""
    _fields_ = [("nfeatures", C.c_int32), ("nlevels", C.c_int32), ("cell_size", C.c_int32), ("threshold", C.c_int32),
                ("max_keypoints", C.c_int32)]


def svo_params(nfeatures=1000, nlevels=8, cell_size=5, threshold=20, max_keypoints=0) -> SvoParams:
    """setParameters(1000, ...) + SVOextractor(nlevels, 5, 20) (Features/Extractor.cpp:21, :162-165);
    max_keypoints 0 = nfeatures + 64 (retainBest's boundary ties beyond that raise RGBD_ERR_CAPACITY)."""
    return SvoParams(nfeatures, nlevels, cell_size, threshold, max_keypoints)


class CloudParams(C.Structure):
    _fields_ = [("stride", C.c_int32), ("zmin", C.c_float), ("zmax", C.c_float), ("leaf", C.c_float),
                ("sor_k", C.c_int32), ("sor_std", C.c_double)]


def cloud_params(stride=6, zmin=0.5, zmax=4.0, leaf=0.04, sor_k=50, sor_std=1.0) -> CloudParams:
    """Tracking::createKeyFrame's values (System/Tracking.cpp:234-237)."""
    return CloudParams(stride, zmin, zmax, leaf, sor_k, sor_std)


class RansacParams(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("min_inlier_th", C.c_uint32), ("max_mahalanobis", C.c_float),
                ("sample_size", C.c_uint32)]


class Rng(C.Structure):
    _fields_ = [("state", C.c_int32 * 31), ("f", C.c_int32), ("r", C.c_int32)]


class Sticky(C.Structure):
    _fields_ = [("cov", C.c_double), ("set", C.c_int32), ("pad", C.c_int32)]


class TrackState(C.Structure):
    """rgbd_track_state: Tracking's state between chunks that overlap by two frames (zeroed = a new
    sequence).  Build it with track_state(), which also owns the two outlier-flag buffers."""
    _fields_ = [("kf_pose", C.c_float * 16), ("first_rel", C.c_float * 16), ("ref2_pose", C.c_float * 16),
                ("first_is_kf", C.c_int32), ("valid", C.c_int32), ("flags2", C.c_void_p), ("flags1", C.c_void_p),
                ("flags_cap", C.c_int32)]


def track_state(cap: int) -> TrackState:
    """A zeroed TrackState with caller-owned flag buffers of `cap` bytes, kept alive by the returned
    object; cap must be >= the context's keypoint capacity (Context.kp_cap; the library checks it and
    raises RGBD_ERR_CAPACITY otherwise).  Context.track_state() sizes it for the context."""
    cap = int(cap)
    if cap < 1:
        raise ValueError("track_state: cap must be >= 1 (use Context.track_state() or ctx.kp_cap)")
    ts = TrackState()
    ts._flag_buffers = (np.zeros(cap, np.uint8), np.zeros(cap, np.uint8))
    ts.flags2 = ts._flag_buffers[0].ctypes.data
    ts.flags1 = ts._flag_buffers[1].ctypes.data
    ts.flags_cap = cap
    return ts


class PnpParams(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("reprojection_error", C.c_float), ("confidence", C.c_double),
                ("min_matches", C.c_int32), ("flag_segments", C.c_int32)]


class GicpParams(C.Structure):
    _fields_ = [("max_iterations", C.c_int32), ("k_correspondences", C.c_int32), ("max_corr_dist", C.c_double),
                ("transformation_epsilon", C.c_double), ("rotation_epsilon", C.c_double),
                ("gicp_epsilon", C.c_double), ("gn_iterations", C.c_int32), ("enable", C.c_int32)]


_vp = C.c_void_p
_i32 = C.c_int32
_PI = C.POINTER(C.c_int32)
_SIGS = {
    "rgbd_create": (_i32, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(OrbParams), C.POINTER(Camera),
                           C.POINTER(_vp)]),
    "rgbd_create_svo": (_i32, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(SvoParams), C.POINTER(Camera),
                               C.POINTER(_vp)]),
    "rgbd_svo_set_brief_pattern": (_i32, [_vp, _vp]),
    "rgbd_svo_get_brief_pattern": (_i32, [_vp, _vp]),
    "rgbd_svo_debug_level": (_i32, [_vp, _i32, _i32, _vp]),
    "rgbd_svo_debug_grid": (_i32, [_vp, _i32, _vp, _vp, _i32, _PI]),
    "rgbd_svo_retain_best": (_i32, [_vp, _vp, _i32, _i32, _i32, _vp, _PI]),
    "rgbd_destroy": (None, [_vp]),
    "rgbd_last_error": (C.c_char_p, [_vp]),
    "rgbd_max_keypoints": (_i32, [_vp]),
    "rgbd_set_stream": (_i32, [_vp, _vp]),
    "rgbd_detect_and_compute": (_i32, [_vp, _vp, _i32, _vp, _vp, _i32, _PI]),
    "rgbd_frame": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _PI]),
    "rgbd_extract_batch": (_i32, [_vp, _vp, _vp, _i32]),
    "rgbd_batch_frame": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, _i32, _PI]),
    "rgbd_batch_outputs": (_i32, [_vp, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp),
                                  C.POINTER(_vp)]),
    "rgbd_debug_level": (_i32, [_vp, _i32, _i32, _vp]),
    "rgbd_debug_blurred": (_i32, [_vp, _i32, _i32, _vp]),
    "rgbd_debug_candidates": (_i32, [_vp, _i32, _i32, _vp, _i32, _PI]),
    "rgbd_debug_selected": (_i32, [_vp, _i32, _i32, _vp, _i32, _PI]),
    "rgbd_knn2": (_i32, [_vp, _vp, _i32, _vp, _i32, _vp]),
    "rgbd_match": (_i32, [_vp, _vp, _i32, _vp, _i32, _vp, _vp, _vp, C.c_float, _i32, _vp, _i32, _PI]),
    "rgbd_ransac_se3": (_i32, [_vp, _vp, _i32, _vp, _i32, _vp, _i32, C.POINTER(RansacParams), C.POINTER(Rng),
                               C.POINTER(Sticky), _i32, _vp, _vp, _vp, _PI, C.POINTER(C.c_float), _PI]),
    "rgbd_rng_seed": (None, [C.POINTER(Rng), C.c_uint32]),
    "rgbd_track_batch": (_i32, [_vp, _vp, _vp, _i32, C.c_float, C.POINTER(RansacParams), C.POINTER(Rng),
                                C.POINTER(Sticky), _vp, _vp, _vp]),
    "rgbd_track_batch_kf": (_i32, [_vp, _vp, _vp, _i32, C.c_float, C.POINTER(RansacParams), C.POINTER(Rng),
                                   C.POINTER(Sticky), C.POINTER(TrackState), _vp, _vp, _vp, _vp, _vp]),
    "rgbd_track_lanes": (_i32, [_vp, _vp, _vp, _i32, C.c_float, C.POINTER(RansacParams), _i32, _vp, _vp, _vp, _vp, _vp,
                                _vp]),
    "rgbd_debug_sort_matches": (_i32, [_vp, _vp, _i32, _i32, _vp]),
    "rgbd_debug_fast_rank16": (_i32, [_vp, _vp, _i32, _vp, _vp]),
    "rgbd_debug_rotation_ops": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp]),
    "rgbd_pnp_ransac": (_i32, [_vp, _vp, _vp, _i32, _vp, C.POINTER(PnpParams), _vp, _vp, _vp, _PI, _PI, _PI]),
    "rgbd_pnp_ransac_batch": (_i32, [_vp, _i32, _vp, _vp, _vp, _vp, C.POINTER(PnpParams), _vp, _vp, _vp, _vp, _vp,
                                     _vp]),
    "rgbd_pnp_track_batch": (_i32, [_vp, _vp, _vp, _i32, C.c_float, C.POINTER(PnpParams), _vp, _vp, _vp, _vp]),
    "rgbd_pnp_track_submit": (_i32, [_vp, _vp, _vp, _i32, C.c_float, C.POINTER(PnpParams)]),
    "rgbd_pnp_track_collect": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "rgbd_gicp": (_i32, [_vp, _vp, _vp, _i32, _vp, C.POINTER(GicpParams), _vp, _PI, _PI]),
    "rgbd_gicp_compute": (_i32, [_vp, _vp, _vp, _i32, _vp, C.POINTER(GicpParams), _vp, _PI]),
    "rgbd_set_tracking_gicp": (_i32, [_vp, C.POINTER(GicpParams)]),
    "rgbd_set_timing": (_i32, [_vp, _i32]),
    "rgbd_reset_timing": (_i32, [_vp]),
    "rgbd_set_timing_filter": (_i32, [_vp, C.c_char_p]),
    "rgbd_timing_count": (_i32, [_vp]),
    "rgbd_timing_entry": (_i32, [_vp, _i32, C.POINTER(C.c_char_p), C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "rgbd_synchronize": (_i32, [_vp]),
    "rgbd_keyframe_cloud": (_i32, [_vp, _vp, _vp, C.POINTER(CloudParams), _vp, _i32, _PI]),
    "rgbd_keyframe_cloud_f32": (_i32, [_vp, _vp, _vp, C.POINTER(CloudParams), _vp, _i32, _PI]),
    "rgbd_keyframe_cloud_batch": (_i32, [_vp, _vp, _vp, _i32, _vp, _i32, C.POINTER(CloudParams), _vp, _i32, _vp]),
    "rgbd_pg_create": (_i32, [C.POINTER(_vp)]),
    "rgbd_pg_destroy": (None, [_vp]),
    "rgbd_pg_add_vertex": (_i32, [_vp, _i32, _vp, _i32]),
    "rgbd_pg_set_fixed": (_i32, [_vp, _i32, _i32]),
    "rgbd_pg_add_edge": (_i32, [_vp, _i32, _i32, _vp, C.c_double, C.c_double, C.POINTER(C.c_double)]),
    "rgbd_pg_exist_edge": (_i32, [_vp, _i32, _i32]),
    "rgbd_pg_counts": (_i32, [_vp, _PI, _PI]),
    "rgbd_pg_chi2": (_i32, [_vp, C.POINTER(C.c_double)]),
    "rgbd_pg_optimize": (_i32, [_vp, _i32, C.POINTER(C.c_double), _PI]),
    "rgbd_pg_vertex": (_i32, [_vp, _i32, _vp]),
}

_lib = None


def build(force: bool = False) -> str:
    """Compile librgbd_hip.so for gfx950 in-tree (hipcc)."""
    args = ["make", "-s", "-C", PKG_DIR]
    if force:
        subprocess.run(args + ["clean"], check=True)
    subprocess.run(args, check=True)
    return LIB_PATH


def lib():
    """Load the HIP library; raises if it is missing (no CPU fallback exists)."""
    global _lib
    if _lib is None:
        # Bind to the same HIP runtime as torch (torch ships its own libamdhip64 with the same
        # SONAME); loading ours first would give the process two HIP runtimes.
        try:
            import torch  # noqa: F401
        except Exception:
            pass
        if not os.path.exists(LIB_PATH):
            raise RgbdError(f"{LIB_PATH} not built: run build() / __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def exported_symbols():
    return list(_SIGS)


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data) if a is not None else None


def orb_params(nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th_fast=20, min_th_fast=7) -> OrbParams:
    """Extractor(ORB2, ORB2, NORMAL) + setParameters, Features/Extractor.cpp:15-48."""
    return OrbParams(nfeatures, scale_factor, nlevels, ini_th_fast, min_th_fast)


def camera(fx, fy, cx, cy, k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0, factor=5000.0) -> Camera:
    """RGBDcamera(IntrinsicMatrix, ..., depthMapFactor=factor); mDepthMapFactor = 1/factor."""
    return Camera(fx, fy, cx, cy, k1, k2, p1, p2, k3, np.float32(1.0) / np.float32(factor))


def ransac_params(iters=200, min_inlier_th=10, max_mahalanobis=3.0, sample_size=4) -> RansacParams:
    return RansacParams(iters, min_inlier_th, max_mahalanobis, sample_size)


def pnp_params(iters=500, reproj=3.0, conf=0.85, min_matches=10, flag_segments=0) -> PnpParams:
    """PnPRansac::compute's solvePnPRansac arguments (Solver/PnPRansac.cpp:39) + its <10-match rule.
    flag_segments (rgbd_pnp_track_*): 0 = independent pairs (discardOutliers = false); S >= 1 = the
    reference's outlier-flag chain over S contiguous runs of pairs (1 = one chain)."""
    return PnpParams(iters, reproj, conf, min_matches, flag_segments)


def gicp_params(max_iterations=10, max_corr=0.07, gn_iterations=4, enable=True) -> GicpParams:
    """Tracking's GICP settings (System/Tracking.cpp:147-151) over the Gicp ctor (Solver/Gicp.cpp:12-15)."""
    return GicpParams(max_iterations, 20, max_corr, 1e-9, 2e-3, 1e-3, gn_iterations, int(enable))


def rng(seed: int) -> Rng:
    r = Rng()
    lib().rgbd_rng_seed(C.byref(r), seed)
    return r


class Context:
    """One extractor + camera + device workspace (rgbd_create)."""

    def __init__(self, width=640, height=480, max_batch=1, orb: OrbParams | None = None,
                 cam: Camera | None = None, device=0, svo: SvoParams | None = None):
        """svo: an Extractor(SVO, BRIEF, NORMAL) context (rgbd_create_svo) instead of the ORBextractor."""
        self.orb = orb or orb_params()
        self.cam = cam or camera(535.4, 539.2, 320.1, 247.6)
        self.svo = svo
        self.W, self.H = width, height
        h = C.c_void_p()
        if svo is not None:
            st = lib().rgbd_create_svo(device, width, height, max_batch, C.byref(svo), C.byref(self.cam), C.byref(h))
        else:
            st = lib().rgbd_create(device, width, height, max_batch, C.byref(self.orb), C.byref(self.cam), C.byref(h))
        self._h = h
        if st != 0:
            msg = lib().rgbd_last_error(h).decode() if h.value else "rgbd_create failed"
            self.close()
            raise RgbdError(f"rgbd_create: {msg} (status {st})")
        self.kp_cap = lib().rgbd_max_keypoints(h)
        self._pending = []   # batch sizes of outstanding pnp_track_submit calls

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().rgbd_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st, what):
        if st != 0:
            raise RgbdError(f"{what}: {lib().rgbd_last_error(self._h).decode()} (status {st})")

    # --- extraction
    def detect_and_compute(self, gray: np.ndarray):
        gray = np.ascontiguousarray(gray, dtype=np.uint8)
        kps = np.zeros(self.kp_cap, KEYPOINT_DTYPE)
        desc = np.zeros((self.kp_cap, 32), np.uint8)
        n = C.c_int32(0)
        self._check(lib().rgbd_detect_and_compute(self._h, _ptr(gray), gray.strides[0], _ptr(kps), _ptr(desc),
                                                  self.kp_cap, C.byref(n)), "detect_and_compute")
        return kps[:n.value].copy(), desc[:n.value].copy()

    def frame(self, bgr: np.ndarray, depth: np.ndarray):
        bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
        depth = np.ascontiguousarray(depth, dtype=np.uint16)
        K = self.kp_cap
        kps, kun = np.zeros(K, KEYPOINT_DTYPE), np.zeros(K, KEYPOINT_DTYPE)
        desc, xyz = np.zeros((K, 32), np.uint8), np.zeros((K, 3), np.float32)
        n = C.c_int32(0)
        self._check(lib().rgbd_frame(self._h, _ptr(bgr), _ptr(depth), _ptr(kps), _ptr(kun), _ptr(desc), _ptr(xyz),
                                     K, C.byref(n)), "frame")
        m = n.value
        return dict(kps=kps[:m].copy(), kps_un=kun[:m].copy(), desc=desc[:m].copy(), xyz=xyz[:m].copy())

    def extract_batch(self, d_bgr: int, d_depth: int, B: int):
        self._check(lib().rgbd_extract_batch(self._h, C.c_void_p(d_bgr), C.c_void_p(d_depth), B), "extract_batch")

    def batch_frame(self, b: int):
        K = self.kp_cap
        kps, kun = np.zeros(K, KEYPOINT_DTYPE), np.zeros(K, KEYPOINT_DTYPE)
        desc, xyz = np.zeros((K, 32), np.uint8), np.zeros((K, 3), np.float32)
        n = C.c_int32(0)
        self._check(lib().rgbd_batch_frame(self._h, b, _ptr(kps), _ptr(kun), _ptr(desc), _ptr(xyz), K,
                                           C.byref(n)), "batch_frame")
        m = n.value
        return dict(kps=kps[:m].copy(), kps_un=kun[:m].copy(), desc=desc[:m].copy(), xyz=xyz[:m].copy())

    # --- SVO + BRIEF (rgbd_create_svo contexts)
    def set_brief_pattern(self, pairs: np.ndarray):
        pairs = np.ascontiguousarray(pairs, dtype=np.int8).reshape(256, 4)
        self._check(lib().rgbd_svo_set_brief_pattern(self._h, _ptr(pairs)), "set_brief_pattern")

    def brief_pattern(self) -> np.ndarray:
        out = np.zeros((256, 4), np.int8)
        self._check(lib().rgbd_svo_get_brief_pattern(self._h, _ptr(out)), "brief_pattern")
        return out

    def svo_debug_level(self, b: int, level: int):
        w, h = self.W, self.H
        for _ in range(level):   # halfSample: floor halving per level
            w, h = w // 2, h // 2
        out = np.zeros((h, w), np.uint8)
        self._check(lib().rgbd_svo_debug_level(self._h, b, level, _ptr(out)), "svo_debug_level")
        return out

    def svo_debug_grid(self, b: int, cap=16384):
        xyl = np.zeros((cap, 3), np.int32)
        resp = np.zeros(cap, np.float32)
        n = C.c_int32(0)
        self._check(lib().rgbd_svo_debug_grid(self._h, b, _ptr(xyl), _ptr(resp), cap, C.byref(n)), "svo_debug_grid")
        return xyl[:n.value].copy(), resp[:n.value].copy()

    def svo_retain_best(self, resp: np.ndarray, n_points: int, depth_limit: int = -1) -> np.ndarray:
        resp = np.ascontiguousarray(resp, dtype=np.float32)
        order = np.zeros(max(len(resp), 1), np.int32)
        m = C.c_int32(0)
        self._check(lib().rgbd_svo_retain_best(self._h, _ptr(resp), len(resp), n_points, depth_limit, _ptr(order),
                                                               C.byref(m)),
                    "svo_retain_best")
        return order[:m.value].copy()

    def debug_level(self, b: int, level: int, w: int, h: int):
        out = np.zeros((h, w), np.uint8)
        self._check(lib().rgbd_debug_level(self._h, b, level, _ptr(out)), "debug_level")
        return out

    def debug_blurred(self, b: int, level: int, w: int, h: int):
        out = np.zeros((h, w), np.uint8)
        self._check(lib().rgbd_debug_blurred(self._h, b, level, _ptr(out)), "debug_blurred")
        return out

    def debug_candidates(self, b: int, level: int, cap=200000):
        out = np.zeros((cap, 3), np.int32)
        n = C.c_int32(0)
        self._check(lib().rgbd_debug_candidates(self._h, b, level, _ptr(out), cap, C.byref(n)), "debug_candidates")
        return out[:n.value].copy()

    def debug_selected(self, b: int, level: int, cap=8192):
        out = np.zeros((cap, 3), np.int32)
        n = C.c_int32(0)
        self._check(lib().rgbd_debug_selected(self._h, b, level, _ptr(out), cap, C.byref(n)), "debug_selected")
        return out[:n.value].copy()

    # --- matching
    def knn2(self, dq: np.ndarray, dt: np.ndarray):
        dq = np.ascontiguousarray(dq, np.uint8)
        dt = np.ascontiguousarray(dt, np.uint8)
        out = np.zeros((max(len(dq), 1), 4), np.int32)
        self._check(lib().rgbd_knn2(self._h, _ptr(dq), len(dq), _ptr(dt), len(dt), _ptr(out)), "knn2")
        return out[:len(dq)]

    def match(self, dq, dt, outlier_q, zq, zt, nnratio=0.9, discard_outliers=True):
        dq = np.ascontiguousarray(dq, np.uint8)
        dt = np.ascontiguousarray(dt, np.uint8)
        outlier_q = np.ascontiguousarray(outlier_q, np.uint8)
        zq = np.ascontiguousarray(zq, np.float32)
        zt = np.ascontiguousarray(zt, np.float32)
        out = np.zeros(max(len(dq), 1), DMATCH_DTYPE)
        m = C.c_int32(0)
        self._check(lib().rgbd_match(self._h, _ptr(dq), len(dq), _ptr(dt), len(dt), _ptr(outlier_q), _ptr(zq),
                                     _ptr(zt), nnratio, int(discard_outliers), _ptr(out), len(out), C.byref(m)),
                    "match")
        return out[:m.value].copy()

    # --- solvers
    def ransac_se3(self, xyz1, xyz2, matches, prm: RansacParams, r: Rng, st: Sticky, flags2=None):
        xyz1 = np.ascontiguousarray(xyz1, np.float32)
        xyz2 = np.ascontiguousarray(xyz2, np.float32)
        matches = np.ascontiguousarray(matches, DMATCH_DTYPE)
        m = len(matches)
        T = np.zeros(16, np.float32)
        inl = np.zeros(max(m, 1), DMATCH_DTYPE)
        n_in, ok = C.c_int32(0), C.c_int32(0)
        rm = C.c_float(0)
        self._check(lib().rgbd_ransac_se3(self._h, _ptr(xyz1), len(xyz1), _ptr(xyz2), len(xyz2),
                                          _ptr(matches) if m else None, m, C.byref(prm), C.byref(r), C.byref(st),
                                          int(flags2 is not None), _ptr(flags2) if flags2 is not None else None,
                                          _ptr(T), _ptr(inl), C.byref(n_in), C.byref(rm), C.byref(ok)), "ransac_se3")
        return bool(ok.value), T.reshape(4, 4), inl[:n_in.value].copy(), float(rm.value)

    def track_batch(self, d_bgr: int, d_depth: int, B: int, nnratio: float, prm: RansacParams, r: Rng,
                    st: Sticky, pose0=None):
        poses = np.zeros((B, 16), np.float32)
        poses[0] = (np.eye(4, dtype=np.float32) if pose0 is None else np.asarray(pose0, np.float32)).reshape(16)
        status = np.zeros(B, np.int32)
        ninl = np.zeros(B, np.int32)
        self._check(lib().rgbd_track_batch(self._h, C.c_void_p(d_bgr), C.c_void_p(d_depth), B, nnratio,
                                           C.byref(prm), C.byref(r), C.byref(st), _ptr(poses), _ptr(status),
                                           _ptr(ninl)), "track_batch")
        return poses.reshape(B, 4, 4), status, ninl

    def track_batch_kf(self, d_bgr: int, d_depth: int, B: int, nnratio: float, prm: RansacParams, r: Rng,
                       st: Sticky, ts: TrackState, pose0=None):
        """Tracking::track over a chunk (rgbd_track_batch_kf): poses (track()'s returns), status, inliers,
        relative poses (mRelativeFramePoses) and keyframe flags; ts carries the state on.  A continuing
        chunk (ts.valid) starts with the previous chunk's last two frames: pose0 is then the pose of
        its frame 1 (the previous chunk's last output), and rows 0-1 of the outputs are not tracked."""
        poses = np.zeros((B, 16), np.float32)
        p0 = (np.eye(4, dtype=np.float32) if pose0 is None else np.asarray(pose0, np.float32)).reshape(16)
        if ts.valid:
            poses[1] = p0
        else:
            poses[0] = p0
        status = np.zeros(B, np.int32)
        ninl = np.zeros(B, np.int32)
        rel = np.zeros((B, 16), np.float32)
        kf = np.zeros(B, np.int32)
        self._check(lib().rgbd_track_batch_kf(self._h, C.c_void_p(d_bgr), C.c_void_p(d_depth), B, nnratio,
                                              C.byref(prm), C.byref(r), C.byref(st), C.byref(ts), _ptr(poses),
                                              _ptr(status), _ptr(ninl), _ptr(rel), _ptr(kf)), "track_batch_kf")
        return poses.reshape(B, 4, 4), status, ninl, rel.reshape(B, 4, 4), kf

    def track_state(self) -> TrackState:
        """A zeroed TrackState whose flag buffers fit this context (kp_cap bytes each)."""
        return track_state(self.kp_cap)

    def track_lanes(self, d_bgr: int, d_depth: int, B: int, nnratio: float, prm: RansacParams, L: int, rngs, stickies,
                    pose0=None, lane_first=None):
        """rgbd_track_lanes: the RansacSE3 chain over L lanes of one batch, all advanced together on the
        device.  lane_first (L + 1 frame indices; default: rgbd-slam_amd/dist.py's shard_range split) ->
        per-lane chains, stitched into one trajectory like the multi-GPU chunks.  Returns (poses [B, 4, 4]
        stitched, status [B], n_inliers [B], lane-major raw poses [(B + L - 1), 4, 4])."""
        from .dist import stitch
        if lane_first is None:
            base, rem = divmod(B, L)
            st = [l * base + min(l, rem) for l in range(L + 1)]
            lane_first = [0] + [st[l] - 1 for l in range(1, L)] + [B - 1]
        lf = np.ascontiguousarray(lane_first, np.int32)
        if len(rngs) != L or len(stickies) != L or len(lf) != L + 1:
            raise ValueError("track_lanes: L rngs, L stickies and L + 1 lane_first entries")
        R = (Rng * L)(*rngs)
        S = (Sticky * L)(*stickies)
        n = B + L - 1
        poses = np.zeros((n, 16), np.float32)
        for l in range(L):
            poses[lf[l] + l] = np.eye(4, dtype=np.float32).reshape(16)
        if pose0 is not None:
            poses[0] = np.asarray(pose0, np.float32).reshape(16)
        status, ninl = np.zeros(n, np.int32), np.zeros(n, np.int32)
        self._check(lib().rgbd_track_lanes(self._h, C.c_void_p(d_bgr), C.c_void_p(d_depth), B, nnratio, C.byref(prm), L,
                                           _ptr(lf), C.cast(R, C.c_void_p), C.cast(S, C.c_void_p), _ptr(poses),
                                           _ptr(status), _ptr(ninl)), "track_lanes")
        for l in range(L):   # the caller's objects carry the lanes' RNG / sticky state on
            C.memmove(C.byref(rngs[l]), C.byref(R[l]), C.sizeof(Rng))
            C.memmove(C.byref(stickies[l]), C.byref(S[l]), C.sizeof(Sticky))
        raw = poses.reshape(n, 4, 4)
        chunks = [raw[lf[l] + l:lf[l + 1] + l + 1] for l in range(L)]
        st_all = np.concatenate([status[lf[0]:lf[1] + 1]] + [status[lf[l] + l + 1:lf[l + 1] + l + 1] for l in range(1, L)])
        ni_all = np.concatenate([ninl[lf[0]:lf[1] + 1]] + [ninl[lf[l] + l + 1:lf[l + 1] + l + 1] for l in range(1, L)])
        p0 = raw[0] if pose0 is not None else np.eye(4, dtype=np.float32)
        return stitch(chunks, p0), st_all, ni_all, raw

    def debug_sort_matches(self, dist, depth_limit: int = -1) -> np.ndarray:
        """The device's std::sort(vUsedMatches) order of integer distances (rgbd_debug_sort_matches)."""
        d = np.ascontiguousarray(dist, np.float32)
        order = np.zeros(max(len(d), 1), np.int32)
        self._check(lib().rgbd_debug_sort_matches(self._h, _ptr(d), len(d), int(depth_limit), _ptr(order)),
                    "debug_sort_matches")
        return order[:len(d)].copy()

    def debug_fast_rank16(self, flags):
        """k_fast's 16-lane emission rank on its own (rgbd_debug_fast_rank16): flags (rows, 64) 0/1 ->
        (slots (rows, 64) with 0xffffffff where clear, counts (64,)); row r of a 16-lane cell starts at 1000 r."""
        f = np.ascontiguousarray(flags, np.uint8)
        rows = f.shape[0]
        slots = np.zeros((rows, 64), np.uint32)
        counts = np.zeros(64, np.uint32)
        self._check(lib().rgbd_debug_fast_rank16(self._h, _ptr(f), rows, _ptr(slots), _ptr(counts)), "debug_fast_rank16")
        return slots, counts

    def debug_rotation_ops(self, x, num, den, theta):
        """The Jacobi rotations' short sqrt / division sequences on their own (rgbd_debug_rotation_ops):
        (sqrt(x), num / den, sign(theta) / (|theta| + sqrt(theta^2 + 1))) as computed on the device, x >= 1 finite,
        |den| in [1, 2^1000), num / den normal, |num| >= 2^-969 unless den == 1 (include/rgbd_hip.h)."""
        arrs = [np.ascontiguousarray(a, np.float64) for a in (x, num, den, theta)]
        n = len(arrs[0])
        assert n >= 1 and all(len(a) == n for a in arrs)
        sq, q, t = np.zeros(n), np.zeros(n), np.zeros(n)
        self._check(lib().rgbd_debug_rotation_ops(self._h, *[_ptr(a) for a in arrs], n, _ptr(sq), _ptr(q), _ptr(t)),
                    "debug_rotation_ops")
        return sq, q, t

    def pnp_ransac_batch(self, problems, K4, prm: PnpParams | None = None):
        """solvePnPRansac on each (p3 [n,3], p2 [n,2]) of `problems`; one pass for all of them.
        Returns a list of dicts: ok, R (3x3 f64), t (3 f64), mask (bool[n]), n_inliers, iters."""
        prm = prm or pnp_params(min_matches=0)
        P = len(problems)
        counts = np.array([len(p3) for p3, _ in problems], np.int32)
        n = int(counts.sum())
        p3 = np.ascontiguousarray(np.concatenate([np.asarray(a, np.float32).reshape(-1, 3) for a, _ in problems])
                                  if n else np.zeros((1, 3), np.float32), np.float32)
        p2 = np.ascontiguousarray(np.concatenate([np.asarray(b, np.float32).reshape(-1, 2) for _, b in problems])
                                  if n else np.zeros((1, 2), np.float32), np.float32)
        K4 = np.ascontiguousarray(K4, np.float32)
        R, t = np.zeros((max(P, 1), 9)), np.zeros((max(P, 1), 3))
        masks = np.zeros(max(n, 1), np.uint8)
        ninl, iters, ok = (np.zeros(max(P, 1), np.int32) for _ in range(3))
        self._check(lib().rgbd_pnp_ransac_batch(self._h, P, _ptr(counts), _ptr(p3), _ptr(p2), _ptr(K4),
                                                C.byref(prm), _ptr(R), _ptr(t), _ptr(masks), _ptr(ninl), _ptr(iters),
                                                _ptr(ok)), "pnp_ransac_batch")
        out, off = [], 0
        for i in range(P):
            c = int(counts[i])
            out.append(dict(ok=bool(ok[i]), R=R[i].reshape(3, 3).copy(), t=t[i].copy(),
                            mask=masks[off:off + c].astype(bool), n_inliers=int(ninl[i]), iters=int(iters[i])))
            off += c
        return out

    def pnp_ransac(self, p3, p2, K4, prm: PnpParams | None = None):
        return self.pnp_ransac_batch([(p3, p2)], K4, prm)[0]

    def pnp_track_batch(self, d_bgr: int, d_depth: int, B: int, nnratio: float, prm: PnpParams | None = None,
                        pose0=None):
        prm = prm or pnp_params()
        poses = np.zeros((B, 16), np.float32)
        poses[0] = (np.eye(4, dtype=np.float32) if pose0 is None else np.asarray(pose0, np.float32)).reshape(16)
        status, ninl, nm = (np.zeros(B, np.int32) for _ in range(3))
        self._check(lib().rgbd_pnp_track_batch(self._h, C.c_void_p(d_bgr), C.c_void_p(d_depth), B, nnratio,
                                               C.byref(prm), _ptr(poses), _ptr(status), _ptr(ninl), _ptr(nm)),
                    "pnp_track_batch")
        return poses.reshape(B, 4, 4), status, ninl, nm

    def pnp_track_submit(self, d_bgr: int, d_depth: int, B: int, nnratio: float, prm: PnpParams | None = None):
        """Enqueue one extract + match + PnPRansac step (rgbd_pnp_track_submit); at most three outstanding."""
        prm = prm or pnp_params()
        self._pending.append(B)
        try:
            self._check(lib().rgbd_pnp_track_submit(self._h, C.c_void_p(d_bgr), C.c_void_p(d_depth), B, nnratio,
                                                    C.byref(prm)), "pnp_track_submit")
        except Exception:
            self._pending.pop()
            raise

    def pnp_track_collect(self, pose0=None):
        """Results of the oldest outstanding submission: (poses, status, n_inliers, n_matches)."""
        if not self._pending:
            raise RgbdError("pnp_track_collect: nothing submitted")
        B = self._pending.pop(0)
        poses = np.zeros((B, 16), np.float32)
        poses[0] = (np.eye(4, dtype=np.float32) if pose0 is None else np.asarray(pose0, np.float32)).reshape(16)
        status, ninl, nm = (np.zeros(B, np.int32) for _ in range(3))
        self._check(lib().rgbd_pnp_track_collect(self._h, _ptr(poses), _ptr(status), _ptr(ninl), _ptr(nm)),
                    "pnp_track_collect")
        return poses.reshape(B, 4, 4), status, ninl, nm

    def keyframe_cloud(self, bgr, depth, prm: CloudParams | None = None):
        """Tracking::createKeyFrame's dense cloud of one frame (host buffers): rgbd_point array."""
        prm = prm or cloud_params()
        bgr = np.ascontiguousarray(bgr, np.uint8)
        depth = np.ascontiguousarray(depth, np.uint16)
        cap = ((depth.shape[0] + prm.stride - 1) // prm.stride) * ((depth.shape[1] + prm.stride - 1) // prm.stride)
        out = np.zeros(cap, POINT_DTYPE)
        n = C.c_int32(0)
        self._check(lib().rgbd_keyframe_cloud(self._h, _ptr(bgr), _ptr(depth), C.byref(prm), _ptr(out), cap,
                                              C.byref(n)), "keyframe_cloud")
        return out[:n.value].copy()

    def keyframe_cloud_f32(self, bgr, depth_f32, prm: CloudParams | None = None):
        """The same cloud from Frame::mImDepth (f32, already scaled by 1/factor), as Frame::createCloud reads it."""
        prm = prm or cloud_params()
        bgr = np.ascontiguousarray(bgr, np.uint8)
        depth = np.ascontiguousarray(depth_f32, np.float32)
        cap = ((depth.shape[0] + prm.stride - 1) // prm.stride) * ((depth.shape[1] + prm.stride - 1) // prm.stride)
        out = np.zeros(cap, POINT_DTYPE)
        n = C.c_int32(0)
        self._check(lib().rgbd_keyframe_cloud_f32(self._h, _ptr(bgr), _ptr(depth), C.byref(prm), _ptr(out), cap,
                                                  C.byref(n)), "keyframe_cloud_f32")
        return out[:n.value].copy()

    def keyframe_cloud_batch(self, d_bgr: int, d_depth: int, B: int, frames, prm: CloudParams | None = None,
                             W: int = 640, H: int = 480):
        """Clouds of the listed frames of a device batch: list of rgbd_point arrays."""
        prm = prm or cloud_params()
        frames = np.ascontiguousarray(frames, np.int32)
        cap = ((H + prm.stride - 1) // prm.stride) * ((W + prm.stride - 1) // prm.stride)
        out = np.zeros((max(len(frames), 1), cap), POINT_DTYPE)
        counts = np.zeros(max(len(frames), 1), np.int32)
        self._check(lib().rgbd_keyframe_cloud_batch(self._h, C.c_void_p(d_bgr), C.c_void_p(d_depth), B, _ptr(frames),
                                                    len(frames), C.byref(prm), _ptr(out), cap, _ptr(counts)),
                    "keyframe_cloud_batch")
        return [out[k, :counts[k]].copy() for k in range(len(frames))]

    def gicp(self, src, tgt, guess, prm: GicpParams | None = None):
        """GICP align: (converged, T 4x4 f32, iterations)."""
        prm = prm or gicp_params()
        src = np.ascontiguousarray(src, np.float32).reshape(-1, 3)
        tgt = np.ascontiguousarray(tgt, np.float32).reshape(-1, 3)
        guess = np.ascontiguousarray(guess, np.float32).reshape(16)
        T = np.zeros(16, np.float32)
        cv, it = C.c_int32(0), C.c_int32(0)
        self._check(lib().rgbd_gicp(self._h, _ptr(src), _ptr(tgt), len(src), _ptr(guess), C.byref(prm), _ptr(T),
                                    C.byref(cv), C.byref(it)), "gicp")
        return bool(cv.value), T.reshape(4, 4), it.value

    def gicp_compute(self, src, tgt, guess, prm: GicpParams | None = None):
        """Gicp::compute: (ok, T 4x4 f32)."""
        prm = prm or gicp_params()
        src = np.ascontiguousarray(src, np.float32).reshape(-1, 3)
        tgt = np.ascontiguousarray(tgt, np.float32).reshape(-1, 3)
        guess = np.ascontiguousarray(guess, np.float32).reshape(16)
        T = np.zeros(16, np.float32)
        ok = C.c_int32(0)
        self._check(lib().rgbd_gicp_compute(self._h, _ptr(src), _ptr(tgt), len(src), _ptr(guess), C.byref(prm),
                                            _ptr(T), C.byref(ok)), "gicp_compute")
        return bool(ok.value), T.reshape(4, 4)

    def set_tracking_gicp(self, prm: GicpParams | None):
        self._check(lib().rgbd_set_tracking_gicp(self._h, C.byref(prm) if prm is not None else None),
                    "set_tracking_gicp")

    # --- measurement
    def set_timing(self, on: bool):
        self._check(lib().rgbd_set_timing(self._h, int(on)), "set_timing")

    def set_timing_filter(self, kernel: str | None):
        self._check(lib().rgbd_set_timing_filter(self._h, kernel.encode() if kernel else None), "set_timing_filter")

    def reset_timing(self):
        self._check(lib().rgbd_reset_timing(self._h), "reset_timing")

    def timings(self):
        out = {}
        for i in range(lib().rgbd_timing_count(self._h)):
            name, ms, n = C.c_char_p(), C.c_double(), C.c_int64()
            self._check(lib().rgbd_timing_entry(self._h, i, C.byref(name), C.byref(ms), C.byref(n)), "timing")
            out[name.value.decode()] = (ms.value, n.value)
        return out

    def synchronize(self):
        self._check(lib().rgbd_synchronize(self._h), "synchronize")

    def set_stream(self, stream: int):
        """Launch on a caller's HIP stream (a torch.cuda.Stream's .cuda_stream); 0 = the context's own."""
        self._check(lib().rgbd_set_stream(self._h, C.c_void_p(stream)), "set_stream")

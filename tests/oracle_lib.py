"""ctypes binding of the CPU ORACLE (oracle/build/liboracle.so).

Test infrastructure only: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "liboracle.so")

f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
u16p = np.ctypeslib.ndpointer(dtype=np.uint16, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class Camera(C.Structure):
    _fields_ = [(n, C.c_float) for n in ("fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2", "k3",
                                         "depth_map_factor")]


class Rng(C.Structure):
    _fields_ = [("state", C.c_int32 * 31), ("f", C.c_int32), ("r", C.c_int32)]


class Sticky(C.Structure):
    _fields_ = [("cov", C.c_double), ("set", C.c_int32), ("pad", C.c_int32)]


class SvoParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("nlevels", C.c_int32), ("cell_size", C.c_int32), ("threshold", C.c_int32)]


class RansacParams(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("min_inlier_th", C.c_uint32), ("max_mahalanobis", C.c_float),
                ("sample_size", C.c_uint32)]


KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
DMATCH_DTYPE = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("imgIdx", "<i4"), ("distance", "<f4")])
kpp = np.ctypeslib.ndpointer(dtype=KEYPOINT_DTYPE, flags="C_CONTIGUOUS")
dmp = np.ctypeslib.ndpointer(dtype=DMATCH_DTYPE, flags="C_CONTIGUOUS")

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P, Cm, SP = C.POINTER(OrbParams), C.POINTER(Camera), C.POINTER(SvoParams)
        i8p = np.ctypeslib.ndpointer(dtype=np.int8, flags="C_CONTIGUOUS")
        sig = {
            "orc_orb_tables": (C.c_int, [P, C.c_int, C.c_int, f32p, f32p, i32p, i32p, i32p, i32p]),
            "orc_gauss_kernel7": (C.c_int, [i32p]),
            "orc_gray": (None, [u8p, C.c_int, C.c_int, u8p]),
            "orc_pyramid": (C.c_int, [u8p, C.c_int, C.c_int, P, u8p]),
            "orc_fast": (C.c_int, [u8p, C.c_int, C.c_int, C.c_int, C.c_int, i32p, C.c_int]),
            "orc_level_candidates": (C.c_int, [u8p, C.c_int, C.c_int, P, i32p, C.c_int]),
            "orc_distribute": (C.c_int, [i32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, i32p,
                                         C.c_int]),
            "orc_blur": (None, [u8p, C.c_int, C.c_int, u8p]),
            "orc_fast_atan2": (C.c_float, [C.c_float, C.c_float]),
            "orc_cos_sin": (None, [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
            "orc_detect_and_compute": (C.c_int, [u8p, C.c_int, C.c_int, P, kpp, u8p, C.c_int]),
            "orc_frame": (C.c_int, [u8p, u16p, C.c_int, C.c_int, P, Cm, kpp, kpp, u8p, f32p, C.c_int]),
            "orc_knn2": (None, [u8p, C.c_int, u8p, C.c_int, i32p]),
            "orc_match": (C.c_int, [u8p, C.c_int, u8p, C.c_int, u8p, f32p, f32p, C.c_float, C.c_int, dmp]),
            "orc_rng_seed": (None, [C.POINTER(Rng), C.c_uint32]),
            "orc_rng_rand": (C.c_int32, [C.POINTER(Rng)]),
            "orc_ransac_se3": (C.c_int, [f32p, f32p, dmp, C.c_int, C.POINTER(RansacParams), C.POINTER(Rng),
                                         C.POINTER(Sticky), C.c_int, C.c_void_p, f32p, dmp,
                                         C.POINTER(C.c_int32), C.POINTER(C.c_float)]),
            "orc_tfc_fit": (None, [f32p, f32p, f32p, C.c_int, f32p]),
            "orc_svd3": (None, [f64p, f64p, f64p, f64p]),
            "orc_mahalanobis2": (C.c_double, [f32p, f32p, f32p, C.c_double]),
            "orc_cloud": (C.c_int, [u8p, u16p, C.c_int, C.c_int, Cm, C.c_int, C.c_float, C.c_float, C.c_void_p,
                                    C.c_int]),
            "orc_voxel": (C.c_int, [C.c_void_p, C.c_int, C.c_float, C.c_void_p]),
            "orc_sor": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_void_p, f32p]),
            "orc_keyframe_cloud": (C.c_int, [u8p, u16p, C.c_int, C.c_int, Cm, C.c_void_p, C.c_int]),
            "orc_brief_default_pattern": (None, [i8p]),
            "orc_svo_pyramid": (C.c_int, [u8p, C.c_int, C.c_int, C.c_int, u8p]),
            "orc_fast10_corners": (C.c_int, [u8p, C.c_int, C.c_int, C.c_int, i32p, C.c_int]),
            "orc_fast10_score_map": (C.c_int, [u8p, C.c_int, C.c_int, C.c_int, i32p]),
            "orc_shi_tomasi": (C.c_float, [u8p, C.c_int, C.c_int, C.c_int, C.c_int]),
            "orc_svo_detect": (C.c_int, [u8p, C.c_int, C.c_int, SP, kpp, C.c_int]),
            "orc_retain_best": (C.c_int, [f32p, C.c_int, C.c_int, i32p]),
            "orc_retain_best_depth": (C.c_int, [f32p, C.c_int, C.c_int, C.c_int, i32p]),
            "orc_sort_dmatch": (C.c_int, [f32p, C.c_int, C.c_int, i32p]),
            "orc_svo_detect_and_compute": (C.c_int, [u8p, C.c_int, C.c_int, SP, C.c_void_p, kpp, u8p, C.c_int]),
            "orc_svo_frame": (C.c_int, [u8p, u16p, C.c_int, C.c_int, SP, C.c_void_p, Cm, kpp, kpp, u8p, f32p,
                                        C.c_int]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


# ---- CPU baseline (bench.py cpu_baseline): the same sources built for timing ----
BENCH_LIB_PATH = os.path.join(ROOT, "oracle", "build", "liboracle_bench.so")   # -O3 -march=x86-64-v3 (prebuilt)
BENCH_FLAGS_PREBUILT = "-O3 -march=x86-64-v3 -ffp-contract=off -fno-fast-math"
BENCH_FLAGS_NATIVE = "-O3 -march=native -ffp-contract=off -fno-fast-math"
BENCH_SRCS = ["orc_orb.cpp", "orc_solver.cpp", "orc_pnp.cpp", "orc_gicp.cpp", "orc_cloud.cpp", "orc_svo.cpp",
              "orc_bench.cpp"]


class BenchResult(C.Structure):
    _fields_ = [("frames_extracted", C.c_int32), ("chain_frames", C.c_int32), ("chain_ok", C.c_int32),
                ("pad", C.c_int32), ("t_extract", C.c_double), ("t_chain", C.c_double), ("t_match", C.c_double),
                ("t_solve", C.c_double)]


def build_native_bench(out_dir: str, timeout=120):
    """Compile the oracle for this host (-O3 -march=native -ffp-contract=off) into out_dir;
    returns (path, flags) or (None, error text) when no compiler is usable (the prebuilt library is then used)."""
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, "liboracle_native.so")
    od = os.path.join(ROOT, "oracle")
    cmd = (["g++"] + BENCH_FLAGS_NATIVE.split() + ["-std=c++17", "-fPIC", "-shared", "-o", path]
           + [os.path.join(od, f) for f in BENCH_SRCS])
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    except (OSError, subprocess.TimeoutExpired) as e:
        return None, str(e)
    if r.returncode != 0 or not os.path.exists(path):
        return None, r.stderr[-500:]
    return path, BENCH_FLAGS_NATIVE


def bench_run(path, bgr, depth, cam: Camera, orb=None, svo=None, solver=0, start=0, seconds=5.0, chain=16):
    """orc_bench_run (oracle/orc_bench.cpp): extraction for `seconds` from offset `start`, then the
    `chain`-frame match + solve chain, all in C++.  Returns a BenchResult."""
    L = C.CDLL(path)
    fn = L.orc_bench_run
    fn.restype = C.c_int
    fn.argtypes = [u8p, u16p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.POINTER(Camera), C.c_int, C.c_int,
                   C.c_double, C.c_int, C.POINTER(BenchResult)]
    bgr = np.ascontiguousarray(bgr, np.uint8)
    depth = np.ascontiguousarray(depth, np.uint16)
    U, H, W = bgr.shape[:3]
    res = BenchResult()
    rc = fn(bgr, depth, U, W, H, C.byref(orb) if orb is not None else None, C.byref(svo) if svo is not None else None,
            C.byref(cam), solver, start, seconds, chain, C.byref(res))
    if rc != 0:
        raise RuntimeError("orc_bench_run failed")
    return res


def orb_params(nfeatures=1000, scale=1.2, nlevels=8, ini=20, mn=7) -> OrbParams:
    return OrbParams(nfeatures, scale, nlevels, ini, mn)


def camera(cam: dict) -> Camera:
    return Camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                  cam["k3"], np.float32(1.0) / np.float32(cam["factor"]))


def tables(p: OrbParams, w=640, h=480):
    n = p.nlevels
    sc, inv = np.zeros(n, np.float32), np.zeros(n, np.float32)
    nf, lw, lh, um = (np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros(n, np.int32),
                      np.zeros(16, np.int32))
    lib().orc_orb_tables(C.byref(p), w, h, sc, inv, nf, lw, lh, um)
    return dict(scale=sc, inv_scale=inv, nfeat=nf, w=lw, h=lh, umax=um)


def gray(bgr: np.ndarray) -> np.ndarray:
    h, w = bgr.shape[:2]
    out = np.zeros((h, w), np.uint8)
    lib().orc_gray(np.ascontiguousarray(bgr), w, h, out)
    return out


def pyramid(g: np.ndarray, p: OrbParams):
    h, w = g.shape
    t = tables(p, w, h)
    total = int(np.sum(t["w"].astype(np.int64) * t["h"]))
    out = np.zeros(total, np.uint8)
    lib().orc_pyramid(np.ascontiguousarray(g), w, h, C.byref(p), out)
    levels, off = [], 0
    for l in range(p.nlevels):
        n = int(t["w"][l]) * int(t["h"][l])
        levels.append(out[off:off + n].reshape(int(t["h"][l]), int(t["w"][l])))
        off += n
    return levels


def fast(img: np.ndarray, threshold: int):
    img = np.ascontiguousarray(img)
    cap = img.size
    out = np.zeros(cap * 3, np.int32)
    n = lib().orc_fast(img, img.shape[1], img.shape[1], img.shape[0], threshold, out, cap)
    return out[:3 * n].reshape(n, 3)


def level_candidates(level: np.ndarray, p: OrbParams):
    level = np.ascontiguousarray(level)
    cap = level.size
    out = np.zeros(cap * 3, np.int32)
    n = lib().orc_level_candidates(level, level.shape[1], level.shape[0], C.byref(p), out, cap)
    return out[:3 * n].reshape(n, 3)


def distribute(cands: np.ndarray, minX, maxX, minY, maxY, N):
    c = np.ascontiguousarray(cands.reshape(-1), dtype=np.int32)
    cap = max(len(cands), 1)
    out = np.zeros(cap * 3, np.int32)
    n = lib().orc_distribute(c, len(cands), minX, maxX, minY, maxY, N, out, cap)
    return out[:3 * n].reshape(n, 3)


def blur(img: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(img)
    out = np.zeros_like(img)
    lib().orc_blur(img, img.shape[1], img.shape[0], out)
    return out


def detect_and_compute(g: np.ndarray, p: OrbParams, cap=8192):
    g = np.ascontiguousarray(g)
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = lib().orc_detect_and_compute(g, g.shape[1], g.shape[0], C.byref(p), kps, desc, cap)
    return kps[:n].copy(), desc[:n].copy()


def frame(bgr: np.ndarray, depth: np.ndarray, p: OrbParams, cam: Camera, cap=8192):
    h, w = depth.shape
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    kun = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    xyz = np.zeros((cap, 3), np.float32)
    n = lib().orc_frame(np.ascontiguousarray(bgr), np.ascontiguousarray(depth), w, h, C.byref(p), C.byref(cam),
                        kps, kun, desc, xyz, cap)
    return dict(kps=kps[:n].copy(), kps_un=kun[:n].copy(), desc=desc[:n].copy(), xyz=xyz[:n].copy())


# ------------------------------------------------------------------ SVO + BRIEF (orc_svo.cpp)
def svo_params(nfeatures=1000, nlevels=8, cell_size=5, threshold=20) -> SvoParams:
    """Extractor(SVO, BRIEF, NORMAL): setParameters(1000, ...) + SVOextractor(nlevels, 5, 20)."""
    return SvoParams(nfeatures, nlevels, cell_size, threshold)


def brief_default_pattern() -> np.ndarray:
    out = np.zeros((256, 4), np.int8)
    lib().orc_brief_default_pattern(out)
    return out


def svo_pyramid(g: np.ndarray, nlevels=8):
    h, w = g.shape
    dims, cw, ch = [], w, h
    for l in range(nlevels):
        if l:
            cw, ch = cw // 2, ch // 2
        dims.append((ch, cw))
    out = np.zeros(sum(a * b for a, b in dims), np.uint8)
    lib().orc_svo_pyramid(np.ascontiguousarray(g), w, h, nlevels, out)
    levels, off = [], 0
    for (lh, lw) in dims:
        levels.append(out[off:off + lh * lw].reshape(lh, lw))
        off += lh * lw
    return levels


def fast10_corners(img: np.ndarray, barrier=20):
    img = np.ascontiguousarray(img)
    cap = max(img.size, 1)
    out = np.zeros(cap * 3, np.int32)
    n = lib().orc_fast10_corners(img, img.shape[1], img.shape[0], barrier, out, cap)
    return out[:3 * n].reshape(n, 3)


def fast10_score_map(img: np.ndarray, barrier=20):
    img = np.ascontiguousarray(img)
    out = np.zeros(img.shape, np.int32)
    lib().orc_fast10_score_map(img, img.shape[1], img.shape[0], barrier, out)
    return out


def shi_tomasi(img: np.ndarray, u: int, v: int) -> float:
    img = np.ascontiguousarray(img)
    return float(lib().orc_shi_tomasi(img, img.shape[1], img.shape[0], u, v))


def svo_detect(g: np.ndarray, p: SvoParams):
    g = np.ascontiguousarray(g)
    cap = g.size // 4 + 16
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    n = lib().orc_svo_detect(g, g.shape[1], g.shape[0], C.byref(p), kps, cap)
    assert n >= 0, "bad SVO parameters"
    return kps[:n].copy()


def retain_best(response: np.ndarray, n_points: int) -> np.ndarray:
    r = np.ascontiguousarray(response, dtype=np.float32)
    order = np.zeros(max(len(r), 1), np.int32)
    n = lib().orc_retain_best(r, len(r), n_points, order)
    return order[:n].copy()


def retain_best_depth(response: np.ndarray, n_points: int, depth_limit: int) -> np.ndarray:
    r = np.ascontiguousarray(response, dtype=np.float32)
    order = np.zeros(max(len(r), 1), np.int32)
    n = lib().orc_retain_best_depth(r, len(r), n_points, depth_limit, order)
    return order[:n].copy()


def _pat(pattern):
    return None if pattern is None else np.ascontiguousarray(pattern, dtype=np.int8).ctypes.data_as(C.c_void_p)


def svo_detect_and_compute(g: np.ndarray, p: SvoParams, pattern=None, cap=16384):
    g = np.ascontiguousarray(g)
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    pat = None if pattern is None else np.ascontiguousarray(pattern, dtype=np.int8)
    n = lib().orc_svo_detect_and_compute(g, g.shape[1], g.shape[0], C.byref(p), _pat(pat), kps, desc, cap)
    assert n >= 0, "bad SVO parameters"
    return kps[:n].copy(), desc[:n].copy()


def svo_frame(bgr: np.ndarray, depth: np.ndarray, p: SvoParams, cam: Camera, pattern=None, cap=16384):
    h, w = depth.shape
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    kun = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    xyz = np.zeros((cap, 3), np.float32)
    pat = None if pattern is None else np.ascontiguousarray(pattern, dtype=np.int8)
    n = lib().orc_svo_frame(np.ascontiguousarray(bgr), np.ascontiguousarray(depth), w, h, C.byref(p), _pat(pat),
                            C.byref(cam), kps, kun, desc, xyz, cap)
    assert n >= 0, "bad SVO parameters"
    return dict(kps=kps[:n].copy(), kps_un=kun[:n].copy(), desc=desc[:n].copy(), xyz=xyz[:n].copy())


def knn2(dq: np.ndarray, dt: np.ndarray) -> np.ndarray:
    out = np.zeros((max(len(dq), 1), 4), np.int32)
    lib().orc_knn2(np.ascontiguousarray(dq), len(dq), np.ascontiguousarray(dt), len(dt), out)
    return out[:len(dq)]


def match(dq, dt, outlier_q, zq, zt, ratio=0.9, discard=True):
    out = np.zeros(max(len(dq), 1), DMATCH_DTYPE)
    m = lib().orc_match(np.ascontiguousarray(dq), len(dq), np.ascontiguousarray(dt), len(dt),
                        np.ascontiguousarray(outlier_q, dtype=np.uint8), np.ascontiguousarray(zq, np.float32),
                        np.ascontiguousarray(zt, np.float32), ratio, int(discard), out)
    return out[:m].copy()


def rng(seed: int) -> Rng:
    r = Rng()
    lib().orc_rng_seed(C.byref(r), seed)
    return r


def ransac_params(iters=200, min_inl=10, maxd=3.0, sample=4) -> RansacParams:
    return RansacParams(iters, min_inl, maxd, sample)


def sort_dmatch(dist, depth_limit=-1) -> np.ndarray:
    """libstdc++ std::sort order of DMatches by distance (depth_limit >= 0: introsort's limit forced)."""
    d = np.ascontiguousarray(dist, np.float32)
    order = np.zeros(max(len(d), 1), np.int32)
    lib().orc_sort_dmatch(d, len(d), int(depth_limit), order)
    return order[:len(d)].copy()


def ransac_se3(xyz1, xyz2, matches, prm: RansacParams, r: Rng, st: Sticky, flags2=None):
    m = len(matches)
    T = np.zeros(16, np.float32)
    inl = np.zeros(max(m, 1), DMATCH_DTYPE)
    n_in = C.c_int32(0)
    rm = C.c_float(0)
    fptr = None
    if flags2 is not None:
        assert flags2.dtype == np.uint8 and flags2.flags.c_contiguous
        fptr = flags2.ctypes.data
    ok = lib().orc_ransac_se3(np.ascontiguousarray(xyz1, np.float32), np.ascontiguousarray(xyz2, np.float32),
                              np.ascontiguousarray(matches) if m else np.zeros(1, DMATCH_DTYPE), m,
                              C.byref(prm), C.byref(r), C.byref(st), int(flags2 is not None), fptr, T, inl,
                              C.byref(n_in), C.byref(rm))
    return bool(ok), T.reshape(4, 4), inl[:n_in.value].copy(), float(rm.value)


def _pnp_sigs():
    L = lib()
    if getattr(L, "_pnp_sig", False):
        return L
    L.orc_cvrng_uniform_stream.restype = C.c_int
    L.orc_cvrng_uniform_stream.argtypes = [C.c_uint64, C.c_int, C.c_int, i32p]
    L.orc_update_num_iters.restype = C.c_int
    L.orc_update_num_iters.argtypes = [C.c_double, C.c_double, C.c_int, C.c_int]
    L.orc_epnp.restype = C.c_int
    L.orc_epnp.argtypes = [f32p, f32p, C.c_int, f32p, f64p, f64p]
    L.orc_pnp_ransac.restype = C.c_int
    L.orc_pnp_ransac.argtypes = [f32p, f32p, C.c_int, f32p, C.c_int, C.c_float, C.c_double, f64p, f64p, u8p,
                                 C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    L.orc_pnp_set_refine_iters.restype = None
    L.orc_pnp_set_refine_iters.argtypes = [C.c_int]
    L._pnp_sig = True
    return L


def pnp_ransac_model(p3, p2, K4, iters=500, reproj=3.0, conf=0.85):
    """solvePnPRansac's RANSAC stage alone (no refinement): (ok, R, t, inlier mask)."""
    L = _pnp_sigs()
    L.orc_pnp_set_refine_iters(0)
    try:
        ok, R, t, mask, _, _ = pnp_ransac(p3, p2, K4, iters, reproj, conf)
    finally:
        L.orc_pnp_set_refine_iters(10)
    return ok, R, t, mask


def epnp(p3, p2, K4):
    L = _pnp_sigs()
    R, t = np.zeros(9), np.zeros(3)
    ok = L.orc_epnp(np.ascontiguousarray(p3, np.float32).reshape(-1), np.ascontiguousarray(p2, np.float32).reshape(-1),
                    len(p3), np.ascontiguousarray(K4, np.float32), R, t)
    return bool(ok), R.reshape(3, 3), t


def pnp_ransac(p3, p2, K4, iters=500, reproj=3.0, conf=0.85):
    L = _pnp_sigs()
    n = len(p3)
    R, t = np.zeros(9), np.zeros(3)
    mask = np.zeros(max(n, 1), np.uint8)
    ni, it = C.c_int32(0), C.c_int32(0)
    ok = L.orc_pnp_ransac(np.ascontiguousarray(p3, np.float32).reshape(-1), np.ascontiguousarray(p2, np.float32).reshape(-1),
                          n, np.ascontiguousarray(K4, np.float32), iters, reproj, conf, R, t, mask, C.byref(ni),
                          C.byref(it))
    return bool(ok), R.reshape(3, 3), t, mask[:n].astype(bool), ni.value, it.value


class GicpParams(C.Structure):
    _fields_ = [("max_iterations", C.c_int32), ("k_correspondences", C.c_int32), ("max_corr_dist", C.c_double),
                ("transformation_epsilon", C.c_double), ("rotation_epsilon", C.c_double),
                ("gicp_epsilon", C.c_double), ("gn_iterations", C.c_int32), ("pad", C.c_int32)]


def gicp_params(max_iterations=10, max_corr=0.07, gn_iterations=4) -> GicpParams:
    """Tracking's Gicp settings (System/Tracking.cpp:147-151) over the Gicp ctor defaults (Solver/Gicp.cpp:12-15)."""
    return GicpParams(max_iterations, 20, max_corr, 1e-9, 2e-3, 1e-3, gn_iterations, 0)


def _gicp_sigs():
    L = lib()
    if getattr(L, "_gicp_sig", False):
        return L
    L.orc_gicp_covariances.restype = C.c_int
    L.orc_gicp_covariances.argtypes = [f32p, C.c_int, C.c_int, C.c_double, f64p]
    L.orc_gicp.restype = C.c_int
    L.orc_gicp.argtypes = [f32p, f32p, C.c_int, f32p, C.POINTER(GicpParams), f32p, C.POINTER(C.c_int32),
                           C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
    L.orc_gicp_compute.restype = C.c_int
    L.orc_gicp_compute.argtypes = [f32p, f32p, C.c_int, f32p, C.POINTER(GicpParams), f32p]
    L._gicp_sig = True
    return L


def gicp_covariances(pts, k=20, eps=1e-3):
    L = _gicp_sigs()
    pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 3)
    out = np.zeros((max(len(pts), 1), 9))
    ok = L.orc_gicp_covariances(pts.reshape(-1), len(pts), k, eps, out.reshape(-1))
    return bool(ok), out[:len(pts)].reshape(-1, 3, 3)


def gicp(src, tgt, guess, prm: GicpParams | None = None):
    """pcl GICP align restated: (converged, T 4x4 f32, iterations, correspondences in the last iteration)."""
    L = _gicp_sigs()
    prm = prm or gicp_params()
    src = np.ascontiguousarray(src, np.float32).reshape(-1, 3)
    tgt = np.ascontiguousarray(tgt, np.float32).reshape(-1, 3)
    T = np.zeros(16, np.float32)
    cv, it, nc = C.c_int32(0), C.c_int32(0), C.c_int32(0)
    L.orc_gicp(src.reshape(-1), tgt.reshape(-1), len(src), np.ascontiguousarray(guess, np.float32).reshape(-1),
               C.byref(prm), T, C.byref(cv), C.byref(it), C.byref(nc))
    return bool(cv.value), T.reshape(4, 4), it.value, nc.value


def gicp_compute(src, tgt, guess, prm: GicpParams | None = None):
    """Gicp::compute (Solver/Gicp.cpp:21-35): (ok, T 4x4 f32)."""
    L = _gicp_sigs()
    prm = prm or gicp_params()
    src = np.ascontiguousarray(src, np.float32).reshape(-1, 3)
    tgt = np.ascontiguousarray(tgt, np.float32).reshape(-1, 3)
    T = np.zeros(16, np.float32)
    ok = L.orc_gicp_compute(src.reshape(-1), tgt.reshape(-1), len(src),
                            np.ascontiguousarray(guess, np.float32).reshape(-1), C.byref(prm), T)
    return bool(ok), T.reshape(4, 4)


# pcl::PointXYZRGB payload of the keyframe cloud (orc_point / rgbd_point)
POINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("b", "u1"), ("g", "u1"), ("r", "u1"),
                        ("pad", "u1")])


def cloud(bgr, depth, cam: dict, res=6, zmin=0.5, zmax=4.0):
    bgr = np.ascontiguousarray(bgr, np.uint8)
    depth = np.ascontiguousarray(depth, np.uint16)
    H, W = depth.shape
    out = np.zeros(((H + res - 1) // res) * ((W + res - 1) // res), POINT_DTYPE)
    n = lib().orc_cloud(bgr, depth, W, H, C.byref(camera(cam)), res, zmin, zmax, out.ctypes.data, len(out))
    return out[:n].copy()


def voxel(points, leaf=0.04):
    points = np.ascontiguousarray(points, POINT_DTYPE)
    out = np.zeros(max(len(points), 1), POINT_DTYPE)
    n = lib().orc_voxel(points.ctypes.data, len(points), leaf, out.ctypes.data)
    return out[:n].copy()


def sor(points, k=50, std_mul=1.0):
    points = np.ascontiguousarray(points, POINT_DTYPE)
    out = np.zeros(max(len(points), 1), POINT_DTYPE)
    dist = np.zeros(max(len(points), 1), np.float32)
    n = lib().orc_sor(points.ctypes.data, len(points), k, std_mul, out.ctypes.data, dist)
    return out[:n].copy(), dist[:len(points)].copy()


def keyframe_cloud(bgr, depth, cam: dict):
    bgr = np.ascontiguousarray(bgr, np.uint8)
    depth = np.ascontiguousarray(depth, np.uint16)
    H, W = depth.shape
    out = np.zeros(((H + 5) // 6) * ((W + 5) // 6), POINT_DTYPE)
    n = lib().orc_keyframe_cloud(bgr, depth, W, H, C.byref(camera(cam)), out.ctypes.data, len(out))
    return out[:n].copy()

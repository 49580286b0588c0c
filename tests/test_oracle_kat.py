"""CPU: the oracle pinned against every known answer the reference itself defines.

The reference ships no tests or fixtures, so the pins are the constants and tables
its source states (file:line below), glibc's own rand() run live, and closed-form checks of the
external primitives the oracle restates.  Parity of the oracle with the reference binary is
otherwise unpinned.
"""
import ctypes as C
import hashlib
import math
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_per_level_budgets_1000_and_2000(oracle):
    # ORBextractor ctor, Features/ORBextractor.cpp:372-383
    assert list(oracle.tables(oracle.orb_params(1000))["nfeat"]) == [217, 181, 151, 126, 105, 87, 73, 60]
    assert list(oracle.tables(oracle.orb_params(2000))["nfeat"]) == [434, 362, 302, 251, 209, 175, 145, 122]


def test_pyramid_sizes(oracle):
    # ComputePyramid, Features/ORBextractor.cpp:776-778
    t = oracle.tables(oracle.orb_params(1000))
    assert list(zip(t["w"], t["h"])) == [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231), (257, 193),
                                         (214, 161), (179, 134)]
    assert int(np.sum(t["w"].astype(np.int64) * t["h"])) == 950532


def test_scale_factors_double_member(oracle):
    # mvScaleFactor[i] = mvScaleFactor[i-1] * scaleFactor with scaleFactor a double member (ORBextractor.h:53)
    t = oracle.tables(oracle.orb_params(1000))
    s = [np.float32(1.0)]
    for i in range(1, 8):
        s.append(np.float32(float(s[-1]) * float(np.float32(1.2))))
    assert np.array_equal(t["scale"], np.array(s, np.float32))
    assert np.array_equal(t["inv_scale"], np.float32(1.0) / np.array(s, np.float32))


def test_umax_table(oracle):
    # Features/ORBextractor.cpp:391-405
    assert list(oracle.tables(oracle.orb_params(1000))["umax"]) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10,
                                                                      9, 8, 6, 3]


def test_pattern_table_hash():
    # bit_pattern_31_, Features/ORBextractor.cpp:89-346 (data table, 256 x 4 ints)
    txt = open(os.path.join(ROOT, "rgbd-slam_amd", "csrc", "orb_pattern.inc")).read()
    nums = [int(x) for x in re.findall(r"-?\d+", "\n".join(l for l in txt.splitlines() if not l.startswith("//")))]
    assert len(nums) == 1024 and max(abs(v) for v in nums) == 13
    assert hashlib.sha256(",".join(map(str, nums)).encode()).hexdigest() == \
        "88df8ca875cc8db56799edd57bb914edad8acb2d48c202b7a464a575b55dbdb8"
    ref = "/root/reference/Features/ORBextractor.cpp"
    if os.path.exists(ref):   # build container only; the GPU box has no /root/reference
        src = open(ref).read()
        start = src.index("bit_pattern_31_[256 * 4] = {")
        body = re.sub(r"/\*.*?\*/", "", src[start:src.index("};", start)], flags=re.S).split("{", 1)[1]
        assert [int(x) for x in re.findall(r"-?\d+", body)] == nums


def test_gaussian_kernel(oracle):
    # GaussianBlur(7x7, sigma 2) 8U bit-exact kernel (ufixedpoint16): sides round(256 g), centre 256 - sides
    k = np.zeros(7, np.int32)
    oracle.lib().orc_gauss_kernel7(k)
    assert list(k) == [18, 34, 49, 54, 49, 34, 18] and k.sum() == 256


@pytest.mark.parametrize("seed", [1, 42, 12345, 0, 2 ** 31 + 5, 4294967295])
def test_rng_matches_glibc_rand(oracle, seed, pkg):
    # System/Random.cpp:10,19 -- srand/rand; checked against this host's glibc, live
    libc = C.CDLL("libc.so.6")
    r = oracle.rng(seed)
    libc.srand(C.c_uint(seed))
    assert [oracle.lib().orc_rng_rand(C.byref(r)) for _ in range(2000)] == [libc.rand() for _ in range(2000)]
    # the product's own restatement (rgbd_rng_seed + the solver's rng) starts from the same state
    pr = pkg.rng(seed)
    r2 = oracle.rng(seed)
    assert list(pr.state) == list(r2.state) and (pr.f, pr.r) == (r2.f, r2.r)


def test_raster_constants():
    # Solver/SolverSE3.cpp:218-225 (2.2516e-5, 2.4096e-5)
    sx = 3 * math.tan(58.0 / 180.0 * math.pi / 640)
    sy = 3 * math.tan(45.0 / 180.0 * math.pi / 480)
    assert abs(sx * sx - 2.2516e-5) < 1e-8 and abs(sy * sy - 2.4096e-5) < 1e-8


def test_fast_atan2_accuracy(oracle):
    # fastAtan2 polynomial: degrees in [0, 360), error < 0.01 deg (OpenCV documents ~0.3 deg worst)
    rs = np.random.default_rng(0)
    for y, x in rs.normal(size=(2000, 2)) * 1000:
        a = oracle.lib().orc_fast_atan2(float(y), float(x))
        ref = math.degrees(math.atan2(y, x)) % 360.0
        assert 0.0 <= a < 360.0
        assert min(abs(a - ref), 360 - abs(a - ref)) < 0.01


def test_cos_sin_definition(oracle):
    # float rounding of a double evaluation: equals correctly-rounded cos/sin (numpy float64 -> float32)
    c, s = C.c_float(), C.c_float()
    for deg in np.linspace(0, 359.99, 3001, dtype=np.float32):
        rad = np.float32(deg) * np.float32(np.pi / np.float32(180.0))
        oracle.lib().orc_cos_sin(float(rad), C.byref(c), C.byref(s))
        assert c.value == float(np.float32(math.cos(float(rad))))
        assert s.value == float(np.float32(math.sin(float(rad))))


def test_svd3_reconstructs(oracle):
    rs = np.random.default_rng(3)
    for _ in range(200):
        A = rs.normal(size=(3, 3))
        U, S, V = np.zeros(9), np.zeros(3), np.zeros(9)
        oracle.lib().orc_svd3(np.ascontiguousarray(A.reshape(9)), U, S, V)
        U, V = U.reshape(3, 3), V.reshape(3, 3)
        assert np.allclose(U @ np.diag(S) @ V.T, A, atol=1e-12)
        assert np.all(np.diff(S) <= 0)
        assert np.allclose(np.sort(S)[::-1], np.linalg.svd(A, compute_uv=False), atol=1e-12)


def test_tfc_fit_recovers_rigid_motion(oracle):
    rs = np.random.default_rng(4)
    p1 = rs.uniform(-1, 1, size=(50, 3)).astype(np.float32) + np.float32([0, 0, 2])
    th = 0.2
    R = np.array([[math.cos(th), -math.sin(th), 0], [math.sin(th), math.cos(th), 0], [0, 0, 1]])
    t = np.array([0.1, -0.2, 0.05])
    p2 = (p1 @ R.T + t).astype(np.float32)
    w = (1.0 / (p1[:, 2] * p2[:, 2])).astype(np.float32)
    T = np.zeros(16, np.float32)
    oracle.lib().orc_tfc_fit(np.ascontiguousarray(p1.reshape(-1)), np.ascontiguousarray(p2.reshape(-1)), w, 50, T)
    T = T.reshape(4, 4)
    assert np.allclose(T[:3, :3], R, atol=1e-5) and np.allclose(T[:3, 3], t, atol=1e-5)


def test_undistort_inverts_distortion(oracle):
    """Frame::undistortKeyPoints (cv::undistortPoints, 5 iterations): distort(undistort(p)) ~ p."""
    import synth
    cam = synth.PRESETS["fr1"]
    rays = synth._rays(640, 480, cam)
    # rays hold the normalised undistorted coordinates of every distorted pixel (same iteration)
    u = rays[..., 0] * cam["fx"] + cam["cx"]
    assert np.isfinite(u).all()

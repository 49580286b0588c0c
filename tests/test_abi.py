"""CPU: the C-ABI library builds, loads and exports every symbol include/rgbd_hip.h declares;
entry points validate arguments without touching a GPU."""
import ctypes as C
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "rgbd_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rgbd_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(pkg):
    lib = pkg.lib()
    names = declared_symbols()
    assert len(names) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", pkg.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (rgbd_\w+)", out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        getattr(lib, n)
    assert set(pkg.exported_symbols()) <= exported


def test_kernels_built_for_gfx950(pkg):
    blob = open(pkg.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for k in (b"k_pyramid", b"k_pyr_tail", b"k_gray", b"k_fast", b"k_distribute", b"k_describe", b"k_knn2", b"k_match_gather",
              b"k_ransac_hyp", b"k_pnp_sample", b"k_pnp_hyp", b"k_pnp_replay", b"k_pnp_refine", b"k_gicp_cov",
              b"k_gicp_align", b"k_undistort", b"k_cloud_voxel", b"k_sor_dist", b"k_sor_filter", b"k_svo_pyramid", b"k_svo_detect",
              b"k_svo_select", b"k_svo_brief", b"k_svo_retain_test"):
        assert k in blob, k


def test_argument_validation_without_device(pkg):
    lib = pkg.lib()
    h = C.c_void_p()
    assert lib.rgbd_create(0, 640, 480, 0, C.byref(pkg.orb_params()), C.byref(pkg.camera(500, 500, 320, 240)),
                           C.byref(h)) == 1          # max_batch < 1 -> RGBD_ERR_ARG
    assert lib.rgbd_ransac_se3(None, None, 0, None, 0, None, 0, None, None, None, 0, None, None, None, None, None,
                               None) == 1
    assert lib.rgbd_track_batch_kf(None, None, None, 2, C.c_float(0.9), None, None, None, None, None, None, None,
                                   None, None) == 1   # no state -> RGBD_ERR_ARG
    assert lib.rgbd_match(None, None, 0, None, 0, None, None, None, 0.9, 1, None, 0, None) == 1


def test_unsupported_geometry_reported(pkg):
    lib = pkg.lib()
    h = C.c_void_p()
    st = lib.rgbd_create(0, 650, 480, 1, C.byref(pkg.orb_params()), C.byref(pkg.camera(500, 500, 320, 240)),
                         C.byref(h))
    assert st == 4   # width not a multiple of 16 -> RGBD_ERR_UNSUPPORTED, before any HIP call
    assert b"multiple of 16" in lib.rgbd_last_error(h)
    lib.rgbd_destroy(h)


def test_rng_seed_matches_glibc(pkg):
    libc = C.CDLL("libc.so.6")
    r = pkg.rng(777)
    libc.srand(777)
    # first output of random_r after seeding: state[f] + state[r] >> 1
    v = ((r.state[r.f] + r.state[r.r]) & 0xFFFFFFFF) >> 1
    assert v == libc.rand()


def test_bench_blur_split_matches_build():
    """bench.py's roofline bytes split the level blur between k_pyramid and k_fast at the build's kPbLevels."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "rgbd-slam_amd", "csrc", "rgbd_internal.h")).read()
    bench = open(os.path.join(root, "bench.py")).read()
    want = int(re.search(r"#define RGBD_PB_LEVELS (\d+)", hdr).group(1))
    got = int(re.search(r"^PB_LEVELS = (\d+)", bench, re.M).group(1))
    assert got == want
    want = int(re.search(r"#define RGBD_PYR_STRIP_LEVELS (\d+)", hdr).group(1))
    got = int(re.search(r"^STRIP_LEVELS = (\d+)", bench, re.M).group(1))
    assert got == want

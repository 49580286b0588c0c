"""CPU: the cpu_baseline build of the oracle (bench.py; oracle/orc_bench.cpp) computes what the test oracle
computes.  The timing builds (-O3 -march=native and the prebuilt -O3 -march=x86-64-v3, both
-ffp-contract=off) must give the same bits as liboracle.so (-O2) for a frame's extraction, and the C++
chain driver must track a synthetic sequence the way tests/chain_model.py does."""
import ctypes as C

import numpy as np
import pytest

import chain_model
import oracle_lib as O
from conftest import synth_seq


def _frame(path, bgr, depth, p, cam, cap=8192):
    L = C.CDLL(path)
    fn = L.orc_frame
    fn.restype = C.c_int
    fn.argtypes = [O.u8p, O.u16p, C.c_int, C.c_int, C.POINTER(O.OrbParams), C.POINTER(O.Camera), O.kpp, O.kpp, O.u8p,
                   O.f32p, C.c_int]
    kps = np.zeros(cap, O.KEYPOINT_DTYPE)
    kun = np.zeros(cap, O.KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    xyz = np.zeros((cap, 3), np.float32)
    n = fn(np.ascontiguousarray(bgr), np.ascontiguousarray(depth), 640, 480, C.byref(p), C.byref(cam), kps, kun, desc, xyz,
           cap)
    return kps[:n], kun[:n], desc[:n], xyz[:n]


@pytest.fixture(scope="module")
def native_lib(tmp_path_factory):
    path, flags = O.build_native_bench(str(tmp_path_factory.mktemp("oracle_native")))
    if path is None:
        pytest.skip("no host compiler: " + flags)
    return path


def test_timing_builds_equal_test_oracle(native_lib):
    bgr, depth, _, cam = synth_seq(1, seed=71, preset="fr1")
    p, oc = O.orb_params(1000), O.camera(cam)
    want = _frame(O.LIB_PATH, bgr[0], depth[0], p, oc)
    assert len(want[0]) > 500
    for path in (native_lib, O.BENCH_LIB_PATH):
        got = _frame(path, bgr[0], depth[0], p, oc)
        for g, w in zip(got, want):
            assert np.array_equal(g.view(np.uint8), w.view(np.uint8)), path


@pytest.mark.parametrize("solver", [0, 1])
def test_cpp_chain_driver(native_lib, solver):
    """orc_bench_run's chain over a 6-frame sequence: every pair tracks (synthetic frames, small motion),
    the same status the Python chain model gives."""
    n = 6
    bgr, depth, _, cam = synth_seq(n, seed=72, preset="fr1")
    oc = O.camera(cam)
    r = O.bench_run(native_lib, bgr, depth, oc, orb=O.orb_params(1000), solver=solver, seconds=0.0, chain=n)
    assert r.frames_extracted == n and r.chain_frames == n and r.t_chain > 0   # a zero budget: the chain's frames
    # the driver walks frames 0 .. n-1 from start 0 (pingpong), so its chain is the model's
    frames = [O.frame(bgr[i], depth[i], O.orb_params(1000), oc) for i in range(n)]
    K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
    if solver == 0:
        _, st, _, _ = chain_model.pnp_track(O, frames, np.eye(4, dtype=np.float32), K4)
    else:
        _, st, _, _, _ = chain_model.track(O, frames, np.eye(4, dtype=np.float32), 99)
    assert r.chain_ok == int(st[1:].sum()) == n - 1

"""The oracle pinned against the reference's own code where it compiles here.

Only System/Random.cpp builds without the reference's external libraries (OpenCV, Eigen, PCL, g2o are
absent): `make -C oracle ref` compiles it from /root/reference into oracle/_ref.  The
reference seeds with time(NULL) once (Random::initSeed, :8-14); after that first call, srand(seed) on the
same libc fixes the stream, so randomInt (:16-21) is compared draw for draw with the oracle's restatement
(orc_random_int on the restated glibc TYPE_3 rand) that every RansacSE3 sample is drawn from
(Solver/SolverSE3.cpp:136-149).  Skipped where oracle/_ref was not built (the GPU box has no reference)."""
import ctypes as C
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "librandom_ref.so")

pytestmark = pytest.mark.skipif(not os.path.exists(REF_SO), reason="oracle/_ref not built (make -C oracle ref)")


@pytest.mark.parametrize("seed", [1, 7, 42, 12345, 2 ** 31 + 5])
@pytest.mark.parametrize("lo,hi", [(0, 999), (0, 3), (5, 5), (-10, 10), (0, 2 ** 20)])
def test_random_int_matches_reference(oracle, seed, lo, hi):
    ref = C.CDLL(REF_SO)
    libc = C.CDLL("libc.so.6")
    init = ref._ZN6Random8initSeedEv
    rint = ref._ZN6Random9randomIntEii
    rint.restype = C.c_int
    rint.argtypes = [C.c_int, C.c_int]
    init()                       # the reference's one-time srand(time(NULL)); later calls do not reseed
    libc.srand(C.c_uint(seed))
    want = [rint(lo, hi) for _ in range(3000)]
    r = oracle.rng(seed)
    f = oracle.lib().orc_random_int
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_int, C.c_int]
    got = [f(C.addressof(r), lo, hi) for _ in range(3000)]
    assert got == want
    assert all(lo <= v <= hi for v in got)

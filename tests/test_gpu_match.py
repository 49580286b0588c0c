"""GPU parity: Hamming knn-2 and Matcher::match filters vs the CPU oracle (bit-exact)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(pkg):
    return pkg.Context(640, 480, max_batch=1)


def test_knn2_random_descriptors(ctx, oracle):
    rs = np.random.default_rng(1)
    for nq, nt in [(1, 2), (5, 3), (300, 257), (1000, 1000), (2004, 1777)]:
        dq = rs.integers(0, 256, size=(nq, 32), dtype=np.uint8)
        dt = rs.integers(0, 256, size=(nt, 32), dtype=np.uint8)
        assert np.array_equal(ctx.knn2(dq, dt), oracle.knn2(dq, dt)), (nq, nt)


def test_knn2_ties_lowest_index_first(ctx, oracle):
    """Duplicated train rows produce distance ties; batchDistance keeps the lower index first."""
    rs = np.random.default_rng(2)
    base = rs.integers(0, 256, size=(40, 32), dtype=np.uint8)
    dt = np.concatenate([base, base, base[::-1]])
    dq = base.copy()
    dq[:, 0] ^= 1
    got, want = ctx.knn2(dq, dt), oracle.knn2(dq, dt)
    assert np.array_equal(got, want)
    assert np.all(got[:, 0] == got[:, 2])      # every query has a tied pair


def test_knn2_single_train_row(ctx, oracle):
    rs = np.random.default_rng(3)
    dq = rs.integers(0, 256, size=(7, 32), dtype=np.uint8)
    dt = rs.integers(0, 256, size=(1, 32), dtype=np.uint8)
    got = ctx.knn2(dq, dt)
    assert np.array_equal(got, oracle.knn2(dq, dt))
    assert np.all(got[:, 3] == -1)


def test_match_filters(ctx, oracle, seq_fr1):
    bgr, depth, _, cam = seq_fr1
    p = oracle.orb_params(1000)
    oc = oracle.camera(cam)
    f0 = oracle.frame(bgr[0], depth[0], p, oc)
    f1 = oracle.frame(bgr[1], depth[1], p, oc)
    rs = np.random.default_rng(4)
    outl = (rs.random(len(f0["kps"])) < 0.2).astype(np.uint8)
    for ratio, discard in [(0.9, True), (0.6, True), (0.9, False)]:
        got = ctx.match(f0["desc"], f1["desc"], outl, f0["xyz"][:, 2], f1["xyz"][:, 2], ratio, discard)
        want = oracle.match(f0["desc"], f1["desc"], outl, f0["xyz"][:, 2], f1["xyz"][:, 2], ratio, discard)
        assert len(want) > 50
        assert np.array_equal(got, want), (ratio, discard)


def test_match_empty_inputs(ctx):
    z = np.zeros(0, np.float32)
    d = np.zeros((0, 32), np.uint8)
    assert len(ctx.match(d, d, np.zeros(0, np.uint8), z, z)) == 0

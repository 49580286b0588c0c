"""CPU: the array model of the device's std::sort(vUsedMatches) (tests/lane_sort_model.py, the algorithm of
rgbd-slam_amd/csrc/lanes.hip lane_sort) equals libstdc++'s std::sort (Solver/SolverSE3.cpp:52, run for real
in the oracle) on tie-heavy, sorted, reversed and constant distance arrays, including introsort's heap-sort
fallback forced by explicit depth limits (libstdc++'s own __introsort_loop in the oracle)."""
import numpy as np
import pytest

import lane_sort_model as M


@pytest.mark.parametrize("n", [1, 2, 5, 16, 17, 18, 33, 100, 257, 1000, 2304])
def test_model_matches_libstdcxx(oracle, n):
    rs = np.random.RandomState(n)
    arrays = [rs.randint(0, 30, size=n), rs.randint(0, 256, size=n), np.sort(rs.randint(0, 50, size=n)),
              np.sort(rs.randint(0, 50, size=n))[::-1], np.full(n, 7)]
    for d in arrays:
        d = d.astype(np.float32)
        for dl in ((-1,) if n <= 16 else (-1, 0, 1, 3)):
            assert np.array_equal(M.lane_sort(d, dl), oracle.sort_dmatch(d, dl)), (n, dl)


def test_heap_fallback_changes_the_order(oracle):
    """The forced depth limits reach a different (still sorted) order: the heap branch is exercised."""
    d = np.random.RandomState(0).randint(0, 40, size=1000).astype(np.float32)
    a, b = oracle.sort_dmatch(d), oracle.sort_dmatch(d, 0)
    assert (d[a][1:] >= d[a][:-1]).all() and (d[b][1:] >= d[b][:-1]).all() and not np.array_equal(a, b)


@pytest.mark.parametrize("n", [17, 18, 33, 64, 65, 100, 257, 1000])
def test_small_segment_wave_model_matches_libstdcxx(oracle, n):
    """lanes.hip wave_sort_small (segments of 17..64 finished in registers by one wave: ballot ranks, bit
    selects, lane shuffles), modelled lane by lane, gives libstdc++'s order, depth-limit fallbacks included."""
    rs = np.random.RandomState(500 + n)
    arrays = [rs.randint(0, 30, size=n), rs.randint(0, 256, size=n), np.sort(rs.randint(0, 50, size=n)),
              np.sort(rs.randint(0, 50, size=n))[::-1], np.full(n, 7), rs.permutation(n) % 11]
    for d in arrays:
        d = d.astype(np.float32)
        for dl in (-1, 0, 1, 2, 3, 5):
            assert np.array_equal(M.lane_sort_small(d, dl), oracle.sort_dmatch(d, dl)), (n, dl)

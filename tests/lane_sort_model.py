"""Array model of the device's std::sort(vUsedMatches) (rgbd-slam_amd/csrc/lanes.hip lane_sort): introsort
with the Hoare partition evaluated from stopper ranks (the k-th left stopper of the original range swaps with
the k-th right stopper while it lies before it), all segments of a recursion level at once, and the final
insertion sort as a stable sort of each leaf.  Pinned against libstdc++'s std::sort (oracle) on CPU."""
import numpy as np


def median_to_first(keys, idx, r, x, y, z):
    """std::__move_median_to_first(result, a, b, c), comp = less: swaps keys and payload together."""
    if keys[x] < keys[y]:
        sel = y if keys[y] < keys[z] else (z if keys[x] < keys[z] else x)
    elif keys[x] < keys[z]:
        sel = x
    elif keys[y] < keys[z]:
        sel = z
    else:
        sel = y
    keys[r], keys[sel] = keys[sel], keys[r]
    idx[r], idx[sel] = idx[sel], idx[r]


def partition_by_ranks(keys, idx, f, l):
    p = keys[f]
    lo = f + 1
    A = [i for i in range(lo, l) if not keys[i] < p]          # left stoppers, ascending
    Bq = [i for i in range(l - 1, lo - 1, -1) if not p < keys[i]]   # right stoppers, descending
    K = 0
    while K < len(A) and K < len(Bq) and A[K] < Bq[K]:
        K += 1
    for k in range(K):
        i, j = A[k], Bq[k]
        keys[i], keys[j] = keys[j], keys[i]
        idx[i], idx[j] = idx[j], idx[i]
    LK = A[K] if K < len(A) else 1 << 30
    return LK if K == 0 else min(LK, Bq[K - 1])


def heap_sort(keys, idx, f, l):
    """libstdc++ __make_heap + __sort_heap on [f, l) with comp = less."""
    def adjust(hole, length, v):
        top, child = hole, hole
        while child < (length - 1) // 2:
            child = 2 * (child + 1)
            if keys[f + child] < keys[f + child - 1]:
                child -= 1
            keys[f + hole], idx[f + hole] = keys[f + child], idx[f + child]
            hole = child
        if length % 2 == 0 and child == (length - 2) // 2:
            child = 2 * (child + 1)
            keys[f + hole], idx[f + hole] = keys[f + child - 1], idx[f + child - 1]
            hole = child - 1
        parent = (hole - 1) // 2
        while hole > top and keys[f + parent] < v[0]:
            keys[f + hole], idx[f + hole] = keys[f + parent], idx[f + parent]
            hole = parent
            parent = (hole - 1) // 2
        keys[f + hole], idx[f + hole] = v
    n = l - f
    if n < 2:
        return
    parent = (n - 2) // 2
    while True:
        adjust(parent, n, (keys[f + parent], idx[f + parent]))
        if parent == 0:
            break
        parent -= 1
    last = l
    while last - f > 1:
        last -= 1
        v = (keys[last], idx[last])
        keys[last], idx[last] = keys[f], idx[f]
        adjust(0, last - f, v)


def lane_sort(dist, depth_limit=-1):
    keys = [int(d) for d in dist]
    idx = list(range(len(keys)))
    n = len(keys)
    leaves = []
    segs = [(0, n, depth_limit if depth_limit >= 0 else 2 * (n.bit_length() - 1))] if n > 16 else []
    if n <= 16:
        leaves.append((0, n, True))
    while segs:
        nxt = []
        for f, l, d in segs:
            if d == 0:
                heap_sort(keys, idx, f, l)
                leaves.append((f, l, False))
                continue
            median_to_first(keys, idx, f, f + 1, f + (l - f) // 2, l - 1)
            cut = partition_by_ranks(keys, idx, f, l)
            for a, b in ((f, cut), (cut, l)):
                (nxt if b - a > 16 else leaves).append((a, b, d - 1) if b - a > 16 else (a, b, True))
        segs = nxt
    out = list(idx)
    for a, b, stable in leaves:
        if stable:
            blk = sorted(range(a, b), key=lambda i: (keys[i], i))
            out[a:b] = [idx[i] for i in blk]
    return np.array(out, np.int32)

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


def _select_bit(m, n):
    """Position of set bit n (0-based from bit 0) of the 64-bit mask m (lanes.hip select_bit)."""
    pos = 0
    for sh in (32, 16, 8, 4, 2, 1):
        c = bin(m & ((1 << sh) - 1)).count("1")
        if n >= c:
            n -= c
            m >>= sh
            pos += sh
    return pos


def wave_sort_small(keys, idx, f, n, depth):
    """Lane-level model of lanes.hip wave_sort_small: the subtree of segment [f, f+n), 16 < n <= 64, with
    lane i holding position f + i; every active segment of a level partitioned at once from ballot masks and
    bit selects.  Returns (leaves, pushed): leaf segments (abs first, abs last) and depth-0 segments."""
    W = 64
    v = [(keys[f + i], idx[f + i]) if i < n else (1 << 40, -1) for i in range(W)]
    fs, ls, dep = [0] * W, [n] * W, [depth] * W
    inn = [i < n for i in range(W)]
    while True:
        act = [inn[i] and ls[i] - fs[i] > 16 and dep[i] > 0 for i in range(W)]
        if not any(act):
            break
        mid = [fs[i] + (ls[i] - fs[i]) // 2 for i in range(W)]
        ch = [0] * W
        for i in range(W):
            va, vb, vc = v[(fs[i] + 1) % W][0], v[mid[i] % W][0], v[(ls[i] - 1) % W][0]
            if va < vb:
                ch[i] = mid[i] if vb < vc else ((ls[i] - 1) if va < vc else fs[i] + 1)
            else:
                ch[i] = (fs[i] + 1) if va < vc else ((ls[i] - 1) if vb < vc else mid[i])
        src = [i if not act[i] else (ch[i] if i == fs[i] else (fs[i] if i == ch[i] else i)) for i in range(W)]
        v = [v[src[i]] for i in range(W)]
        p = [v[fs[i]][0] for i in range(W)]
        inr = [act[i] and fs[i] < i < ls[i] for i in range(W)]
        A = [inr[i] and not v[i][0] < p[i] for i in range(W)]
        Bq = [inr[i] and not p[i] < v[i][0] for i in range(W)]
        bal = lambda fl: sum(1 << i for i in range(W) if fl[i])
        balA, balB = bal(A), bal(Bq)
        new_src = list(range(W))
        cuts = [None] * W
        swapL = [False] * W
        segm = [0] * W
        for i in range(W):
            L = ls[i] - fs[i]
            segm[i] = ((1 << 64) - 1) if L >= 64 else (((1 << L) - 1) << fs[i])
        for i in range(W):
            lm, rm = balA & segm[i], balB & segm[i]
            below = (1 << i) - 1
            ka, kb = bin(lm & below).count("1"), bin(rm & below).count("1")
            TB = bin(rm).count("1")
            swapL[i] = A[i] and TB - kb - (1 if Bq[i] else 0) >= ka + 1
        balS = bal(swapL)
        for i in range(W):
            lm, rm = balA & segm[i], balB & segm[i]
            below = (1 << i) - 1
            ka, kb = bin(lm & below).count("1"), bin(rm & below).count("1")
            TA, TB = bin(lm).count("1"), bin(rm).count("1")
            K = bin(balS & segm[i]).count("1")
            rr = TB - 1 - kb
            swapR = Bq[i] and rr < K
            if swapL[i]:
                new_src[i] = _select_bit(rm, TB - 1 - ka)
            if swapR:
                new_src[i] = _select_bit(lm, rr)
            LK = _select_bit(lm, K) if K < TA else 1 << 30
            RK1 = _select_bit(rm, TB - K) if K > 0 else -1
            cuts[i] = LK if K == 0 else min(LK, RK1)
        v = [v[new_src[i]] for i in range(W)]
        for i in range(W):
            if act[i]:
                if i < cuts[i]:
                    ls[i] = cuts[i]
                else:
                    fs[i] = cuts[i]
                dep[i] -= 1
    for i in range(n):
        keys[f + i], idx[f + i] = v[i]
    leaves, pushed = set(), set()
    for i in range(n):
        if ls[i] - fs[i] <= 16:
            leaves.add((f + fs[i], f + ls[i]))
        else:
            pushed.add((f + fs[i], f + ls[i]))
    return sorted(leaves), sorted(pushed)


def lane_sort_small(dist, depth_limit=-1):
    """lane_sort with segments of <= 64 elements finished by the wave_sort_small model (the device path)."""
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
            if l - f <= 64:
                lv, pu = wave_sort_small(keys, idx, f, l - f, d)
                leaves += [(a, b, True) for a, b in lv]
                nxt += [(a, b, 0) for a, b in pu]
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

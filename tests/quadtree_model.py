"""Python model of k_distribute's parallel DistributeOctTree formulation (test infrastructure).

Round-based restatement used by the kernel: the node list is an array in list order;
one round divides a set of nodes (phase 1: every node with >1 keys, in list order;
phase 2: by (size, creation id) descending until the list reaches N).  Children go to
the front in reverse creation order, the other nodes keep their order behind them.
Checked against the oracle's literal std::list restatement (tests/test_oracle_quadtree.py)
so the kernel's formulation is validated on CPU.
"""
import numpy as np


def quad(kx, ky, box):
    x0, y0, x1, y1 = box
    mx = x0 + (x1 - x0 + 1) // 2
    my = y0 + (y1 - y0 + 1) // 2
    return (0 if ky < my else 2) if kx < mx else (1 if ky < my else 3)


def child_box(box, q):
    x0, y0, x1, y1 = box
    mx = x0 + (x1 - x0 + 1) // 2
    my = y0 + (y1 - y0 + 1) // 2
    return ((mx if q & 1 else x0), (my if q & 2 else y0), (x1 if q & 1 else mx), (y1 if q & 2 else my))


def distribute(cands: np.ndarray, minX, maxX, minY, maxY, N):
    n = len(cands)
    if n == 0:
        return np.zeros((0, 3), np.int32)
    nIni = int(np.round(np.float32(maxX - minX) / np.float32(maxY - minY)))
    hX = np.float32(maxX - minX) / np.float32(nIni)
    node_of = np.array([min(int(np.float32(x) / hX), nIni - 1) for x in cands[:, 0]])
    sizes = np.bincount(node_of, minlength=nIni)
    # nodes: list of dicts in list order
    nodes, remap = [], {}
    for i in range(nIni):
        if sizes[i] > 0:
            remap[i] = len(nodes)
            nodes.append(dict(box=(int(hX * np.float32(i)), 0, int(hX * np.float32(i + 1)), maxY - minY),
                              size=int(sizes[i]), cid=i))
    node_of = np.array([remap[v] for v in node_of])
    next_cid = nIni
    phase = 1
    while nodes:
        prev = len(nodes)
        L = len(nodes)
        childcnt = np.zeros((L, 4), np.int64)
        for k in range(n):
            nd = node_of[k]
            if nodes[nd]["size"] > 1:
                childcnt[nd, quad(cands[k, 0], cands[k, 1], nodes[nd]["box"])] += 1
        S = [i for i in range(L) if nodes[i]["size"] > 1]
        if phase == 2:
            S.sort(key=lambda i: (nodes[i]["size"], nodes[i]["cid"]), reverse=True)
        c = [int(np.count_nonzero(childcnt[i])) for i in S]
        napply = len(S)
        if phase == 2:
            run = L
            for j, cj in enumerate(c):
                run += cj - 1
                if run >= N:
                    napply = j + 1
                    break
        T = sum(c[:napply])
        applied = set(S[:napply])
        new = [None] * (T + L - napply)
        child_idx = {}
        o = 0
        for j in range(napply):
            nd = S[j]
            for q in range(4):
                if childcnt[nd, q] > 0:
                    ni = T - 1 - o
                    new[ni] = dict(box=child_box(nodes[nd]["box"], q), size=int(childcnt[nd, q]), cid=next_cid + o)
                    child_idx[(nd, q)] = ni
                    o += 1
        surv = {}
        pos = T
        for i in range(L):
            if i not in applied:
                surv[i] = pos
                new[pos] = nodes[i]
                pos += 1
        for k in range(n):
            nd = node_of[k]
            if nd in applied:
                node_of[k] = child_idx[(nd, quad(cands[k, 0], cands[k, 1], nodes[nd]["box"]))]
            else:
                node_of[k] = surv[nd]
        n_expand = sum(1 for i in range(T) if new[i]["size"] > 1)
        nodes = new
        next_cid += T
        if len(nodes) >= N or len(nodes) == prev:
            break
        if phase == 1 and len(nodes) + 3 * n_expand > N:
            phase = 2
    best = {}
    for k in range(n):
        nd = node_of[k]
        key = (cands[k, 2], -k)
        if nd not in best or key > best[nd]:
            best[nd] = key
    return np.array([cands[-best[i][1]] for i in range(len(nodes))], np.int32).reshape(-1, 3)

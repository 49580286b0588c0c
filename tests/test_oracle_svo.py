"""SVO + BRIEF oracle (oracle/orc_svo.cpp; the reference's default Extractor(SVO, BRIEF, NORMAL), main.cpp:31)
against independent numpy formulations of each stage:

* halfSample pyramid (Features/SVOextractor.cpp:16-37, :139-148): 2x2 integer means, chained;
* FAST-10 + fast_corner_score_10: the binary-searched score equals the closed form
  max over the 16 ten-pixel arcs of (min |ring - centre| on one side) - 1;
* fast_nonmax_3x3 (Rosten's row-pointer walk) equals "no 8-neighbour corner scores >= mine";
* ShiTomasiScore (:39-84) in float32 with the reference's operation order;
* the SVO grid (:86-137): per 5x5 cell the first maximal Shi-Tomasi score over levels / raster order;
* retainBest (libstdc++ nth_element + partition): the kept set is exactly the top-n responses plus
  every tie of the boundary response;
* BRIEF-32 (xfeatures2d): runByImageBorder(28) and 9x9 box-sum tests from the integral image.
"""
import numpy as np

import oracle_lib as O
from conftest import synth_seq

RING = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
        (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]   # (dx, dy), cyclic


def _gray(seed=3, f=0, preset="fr1"):
    bgr, depth, _, cam = synth_seq(2, seed=seed, preset=preset)
    return O.gray(bgr[f]), bgr[f], depth[f], cam


def _np_half(img):
    h, w = img.shape[0] // 2, img.shape[1] // 2
    a = img[:2 * h, :2 * w].astype(np.uint16)
    return ((a[0::2, 0::2] + a[0::2, 1::2] + a[1::2, 0::2] + a[1::2, 1::2]) // 4).astype(np.uint8)


def test_pyramid_matches_numpy():
    g = _gray()[0]
    lv = O.svo_pyramid(g, 8)
    want = g
    for l in range(8):
        if l:
            want = _np_half(want)
        assert lv[l].shape == want.shape and np.array_equal(lv[l], want), l
    assert [x.shape for x in lv][-1] == (3, 5)


def _np_fast10_score(img, barrier=20):
    """closed form: D = max over arcs of 10 and both polarities of min difference; corner iff D > barrier,
    Rosten's binary-searched score = D - 1."""
    h, w = img.shape
    I = img.astype(np.int32)
    out = np.zeros((h, w), np.int32)
    if h < 7 or w < 7:
        return out
    c = I[3:h - 3, 3:w - 3]
    ring = np.stack([I[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in RING], 0)
    D = np.full(c.shape, -1000, np.int32)
    for s in range(16):
        arc = ring[[(s + j) % 16 for j in range(10)]]
        D = np.maximum(D, np.maximum((arc - c).min(0), (c - arc).min(0)))
    out[3:h - 3, 3:w - 3] = np.where(D > barrier, D - 1, 0)
    return out


def test_fast10_score_closed_form():
    g = _gray()[0]
    for img in O.svo_pyramid(g, 8)[:7]:
        got = O.fast10_score_map(img, 20)
        assert np.array_equal(got, _np_fast10_score(img, 20))
    # random images hit every arc / polarity / saturation case
    rs = np.random.RandomState(7)
    for t in range(6):
        img = rs.randint(0, 256, size=(40, 57)).astype(np.uint8)
        if t % 2:
            img = (img // 64 * 64).astype(np.uint8)   # plateaus: many equal ring values
        for b in (7, 20, 60):
            assert np.array_equal(O.fast10_score_map(img, b), _np_fast10_score(img, b))


def _np_nonmax(S):
    h, w = S.shape
    P = np.zeros((h + 2, w + 2), np.int32)
    P[1:-1, 1:-1] = S
    keep = S > 0
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dx or dy:
                n = P[1 + dy:h + 1 + dy, 1 + dx:w + 1 + dx]
                keep &= ~((n > 0) & (n >= S))
    ys, xs = np.nonzero(keep)
    return np.stack([xs, ys, S[ys, xs]], 1)


def test_nonmax_matches_neighbourhood_definition():
    g = _gray()[0]
    rs = np.random.RandomState(11)
    imgs = O.svo_pyramid(g, 8)[:7] + [rs.randint(0, 256, size=(64, 80)).astype(np.uint8),
                                       (rs.randint(0, 4, size=(64, 80)) * 80).astype(np.uint8)]
    for img in imgs:
        got = O.fast10_corners(img, 20)
        want = _np_nonmax(_np_fast10_score(img, 20))
        assert np.array_equal(got, want), (img.shape, len(got), len(want))


def _np_shi_tomasi(img, u, v):
    f32 = np.float32
    h, w = img.shape
    if u - 4 < 1 or u + 4 >= w - 1 or v - 4 < 1 or v + 4 >= h - 1:
        return f32(0)
    I = img.astype(np.int32)
    ys = slice(v - 4, v + 4)
    dx = (I[ys, u - 3:u + 5] - I[ys, u - 5:u + 3]).astype(f32)
    dy = (I[v - 3:v + 5, u - 4:u + 4] - I[v - 5:v + 3, u - 4:u + 4]).astype(f32)
    # every partial sum is an integer below 2^24: exact in any order
    xx, yy, xy = f32((dx * dx).sum()), f32((dy * dy).sum()), f32((dx * dy).sum())
    xx, yy, xy = f32(xx / f32(128)), f32(yy / f32(128)), f32(xy / f32(128))
    s = f32(xx + yy)
    disc = f32(f32(s * s) - f32(f32(4) * f32(f32(xx * yy) - f32(xy * xy))))
    return f32(0.5 * float(f32(s - np.sqrt(disc, dtype=f32))))


def test_shi_tomasi_matches_numpy():
    g = _gray()[0]
    rs = np.random.RandomState(5)
    for img in O.svo_pyramid(g, 8)[:4]:
        h, w = img.shape
        for _ in range(300):
            u, v = int(rs.randint(0, w)), int(rs.randint(0, h))
            got, want = O.shi_tomasi(img, u, v), _np_shi_tomasi(img, u, v)
            assert np.float32(got).tobytes() == np.float32(want).tobytes() or (np.isnan(got) and np.isnan(want))


def _np_svo_detect(g, nlevels=8, cell=5, thresh=20):
    lv = O.svo_pyramid(g, nlevels)
    H, W = g.shape
    gc, gr = -(-W // cell), -(-H // cell)
    best = {}
    for L, img in enumerate(lv):
        sc = 1 << L
        for x, y, _ in _np_nonmax(_np_fast10_score(img, thresh)):
            k = (y * sc // cell) * gc + x * sc // cell
            s = _np_shi_tomasi(img, int(x), int(y))
            if s > best.get(k, (np.float32(0),))[0]:
                best[k] = (s, x * sc, y * sc, L)
    out = [(k,) + best[k] for k in sorted(best) if float(best[k][0]) > 20.0]
    return out, gc * gr


def test_svo_detect_matches_numpy():
    g = _gray(seed=5)[0]
    got = O.svo_detect(g, O.svo_params())
    want, _ = _np_svo_detect(g)
    assert len(got) == len(want) > 1000
    w = np.array([(x, y, s, L) for _, s, x, y, L in want], dtype=object)
    assert np.array_equal(got["x"], w[:, 0].astype(np.float32)) and np.array_equal(got["y"], w[:, 1].astype(np.float32))
    assert np.array_equal(got["response"], w[:, 2].astype(np.float32))
    assert np.array_equal(got["octave"], w[:, 3].astype(np.int32))
    assert (got["size"] == 0).all() and (got["angle"] == -1).all() and (got["class_id"] == -1).all()


def test_retain_best_sets():
    rs = np.random.RandomState(3)
    for n, keep, levels in [(5000, 1000, None), (1500, 1000, 40), (1001, 1000, 3), (300, 1000, None), (64, 7, 2)]:
        r = rs.rand(n).astype(np.float32) * 100 if levels is None else \
            (rs.randint(0, levels, n) * 1.5).astype(np.float32)
        order = O.retain_best(r, keep)
        if n <= keep:
            assert np.array_equal(order, np.arange(n))
            continue
        kth = np.sort(r)[::-1][keep - 1]
        assert len(order) == (r >= kth).sum() and len(set(order.tolist())) == len(order)
        assert (r[order] >= kth).all() and (r[order[:keep]] >= kth).all()


def _np_brief(g, kps, pat):
    H, W = g.shape
    S = np.zeros((H + 1, W + 1), np.int64)
    S[1:, 1:] = g.astype(np.int64).cumsum(0).cumsum(1)

    def box(y, x):   # 9x9 box centred at (y, x)
        return S[y + 5, x + 5] - S[y + 5, x - 4] - S[y - 4, x + 5] + S[y - 4, x - 4]

    keep = (kps["x"] >= 28) & (kps["x"] < W - 28) & (kps["y"] >= 28) & (kps["y"] < H - 28)
    k = kps[keep]
    desc = np.zeros((len(k), 32), np.uint8)
    x, y = (k["x"] + np.float32(0.5)).astype(np.int64), (k["y"] + np.float32(0.5)).astype(np.int64)
    for t in range(256):
        y1, x1, y2, x2 = (int(v) for v in pat[t])
        bit = (box(y + y1, x + x1) < box(y + y2, x + x2)).astype(np.uint8)
        desc[:, t // 8] |= bit << (7 - t % 8)
    return k, desc


def test_brief_and_extract_match_numpy():
    g = _gray(seed=3)[0]
    p = O.svo_params()
    det = O.svo_detect(g, p)
    assert len(det) > p.nfeatures
    order = O.retain_best(det["response"], p.nfeatures)
    pat = O.brief_default_pattern()
    assert np.abs(pat.astype(int)).max() <= 24
    for pattern in (None, np.random.RandomState(2).randint(-24, 25, size=(256, 4)).astype(np.int8)):
        kps, desc = O.svo_detect_and_compute(g, p, pattern)
        wk, wd = _np_brief(g, det[order], pat if pattern is None else pattern)
        assert len(kps) == len(wk) > 800
        assert np.array_equal(kps, wk) and np.array_equal(desc, wd)


def test_svo_frame_geometry():
    g, bgr, depth, cam = _gray(seed=3)
    p = O.svo_params()
    fr = O.svo_frame(bgr, depth, p, O.camera(cam))
    kps, desc = O.svo_detect_and_compute(g, p)
    assert np.array_equal(fr["kps"], kps) and np.array_equal(fr["desc"], desc)
    # uprojectCamera: z from the distorted integer pixel
    z = depth[kps["y"].astype(int), kps["x"].astype(int)].astype(np.float32) * (np.float32(1) / np.float32(cam["factor"]))
    assert np.array_equal(fr["xyz"][:, 2], np.where(z > 0, z, 0).astype(np.float32))
    assert (fr["kps_un"]["x"] != kps["x"]).any()   # fr1 distortion applied


def test_small_and_edge_images():
    rs = np.random.RandomState(1)
    for (h, w) in [(60, 64), (128, 128), (57, 64), (40, 48)]:
        g = rs.randint(0, 256, size=(h, w)).astype(np.uint8)
        p = O.svo_params(nfeatures=100000, nlevels=4)
        want, _ = _np_svo_detect(g, nlevels=4)
        kps, desc = O.svo_detect_and_compute(g, p)
        inb = [(x, y) for _, _, x, y, _ in want if 28 <= x < w - 28 and 28 <= y < h - 28]
        assert [(int(a), int(b)) for a, b in zip(kps["x"], kps["y"])] == [(int(a), int(b)) for a, b in inb]
    # an image no larger than twice the BRIEF border keeps nothing (runByImageBorder)
    g = rs.randint(0, 256, size=(56, 64)).astype(np.uint8)
    assert len(O.svo_detect_and_compute(g, O.svo_params(nlevels=4))[0]) == 0
    # odd widths above the last level are rejected (halfSample's row walk, SVOextractor.cpp:24-35)
    g = rs.randint(0, 256, size=(64, 66)).astype(np.uint8)
    kps = np.zeros(4, O.KEYPOINT_DTYPE)
    assert O.lib().orc_svo_detect(g, 66, 64, O.svo_params(), kps, 4) == -1


def test_svo_golden_frame():
    """Regression pin of the whole SVO + BRIEF frame (tests/golden/svo_frame_fr1_seed3.npz, make_golden.py)."""
    import os
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "svo_frame_fr1_seed3.npz"),
                allow_pickle=False)
    bgr, depth, _, cam = synth_seq(2, seed=3, preset="fr1")
    assert int(g["bgr_sum"]) == int(bgr[0].astype(np.int64).sum())
    assert np.array_equal(g["pattern"], O.brief_default_pattern())
    got = O.svo_frame(bgr[0], depth[0], O.svo_params(), O.camera(cam))
    assert np.array_equal(got["kps"], g["kps"]) and np.array_equal(got["desc"], g["desc"])
    assert np.array_equal(got["xyz"].view(np.uint32), g["xyz"].view(np.uint32))

"""Keyframe dense cloud oracle (oracle/orc_cloud.cpp; System/Tracking.cpp:234-237) against independent
numpy formulations of the same PCL 1.8 semantics: stride-6 back-projection + pass-through, VoxelGrid
(min/max bounds, floor indices, centroids in point order, truncated mean colours) and
StatisticalOutlierRemoval (mean distance to the 50 nearest, mean + 1 sigma threshold)."""
import numpy as np

import oracle_lib as O
from conftest import synth_seq


def _np_cloud(bgr, depth, cam, res=6, zmin=0.5, zmax=4.0):
    f32 = np.float32
    H, W = depth.shape
    m, n = np.meshgrid(np.arange(0, H, res), np.arange(0, W, res), indexing="ij")
    z = depth[m, n].astype(f32) * (f32(1.0) / f32(cam["factor"])) + f32(0.0)
    keep = (z > 0) & (z >= f32(zmin)) & (z <= f32(zmax))
    m, n, z = m[keep], n[keep], z[keep]
    x = (n.astype(f32) - f32(cam["cx"])) * z * (f32(1.0) / f32(cam["fx"]))
    y = (m.astype(f32) - f32(cam["cy"])) * z * (f32(1.0) / f32(cam["fy"]))
    col = bgr[m, n]
    return x, y, z, col


def test_cloud_matches_numpy():
    bgr, depth, _, cam = synth_seq(2, seed=5, preset="fr1")
    for f in range(2):
        got = O.cloud(bgr[f], depth[f], cam)
        x, y, z, col = _np_cloud(bgr[f], depth[f], cam)
        assert len(got) == len(x) > 3000
        assert np.array_equal(got["x"], x) and np.array_equal(got["y"], y) and np.array_equal(got["z"], z)
        assert np.array_equal(got["b"], col[:, 0]) and np.array_equal(got["r"], col[:, 2])
        assert (got["z"] >= 0.5).all() and (got["z"] <= 4.0).all()


def _np_voxel(p, leaf=0.04):
    f32 = np.float32
    inv = f32(1.0) / f32(leaf)
    xyz = np.stack([p["x"], p["y"], p["z"]], 1)
    mn, mx = xyz.min(0), xyz.max(0)
    minb = np.floor(mn * inv).astype(np.int64)
    maxb = np.floor(mx * inv).astype(np.int64)
    divb = maxb - minb + 1
    ijk = (np.floor(xyz * inv) - minb.astype(f32)).astype(np.int64)
    idx = ijk[:, 0] + ijk[:, 1] * divb[0] + ijk[:, 2] * divb[0] * divb[1]
    order = np.lexsort((np.arange(len(p)), idx))
    out = []
    s = 0
    idx_s = idx[order]
    while s < len(order):
        e = s
        while e < len(order) and idx_s[e] == idx_s[s]:
            e += 1
        acc = np.zeros(6, f32)
        for i in order[s:e]:   # float sums in point order
            acc += np.array([p["x"][i], p["y"][i], p["z"][i], p["r"][i], p["g"][i], p["b"][i]], f32)
        acc /= f32(e - s)
        out.append((acc[0], acc[1], acc[2], int(acc[5]), int(acc[4]), int(acc[3]), 0))
        s = e
    return np.array(out, O.POINT_DTYPE)


def test_voxel_matches_numpy():
    bgr, depth, _, cam = synth_seq(2, seed=5, preset="fr1")
    p = O.cloud(bgr[0], depth[0], cam)
    got = O.voxel(p)
    want = _np_voxel(p)
    assert 1000 < len(got) < len(p)
    assert np.array_equal(got, want)


def test_sor_matches_numpy():
    rs = np.random.default_rng(7)
    pts = np.zeros(700, O.POINT_DTYPE)
    xyz = rs.normal(size=(700, 3)).astype(np.float32)
    xyz[:20] *= 6.0                                       # outliers
    pts["x"], pts["y"], pts["z"] = xyz[:, 0], xyz[:, 1], xyz[:, 2]
    pts["r"] = np.arange(700) % 251
    got, dist = O.sor(pts)
    d = np.zeros(700, np.float32)
    for i in range(700):
        dx, dy, dz = xyz[i, 0] - xyz[:, 0], xyz[i, 1] - xyz[:, 1], xyz[i, 2] - xyz[:, 2]
        r = ((dx * dx) + (dy * dy)) + (dz * dz)           # float32 throughout
        s = 0.0
        for v in np.sort(r)[1:51]:
            s += np.sqrt(np.float64(v))
        d[i] = np.float32(s / 50)
    assert np.array_equal(dist, d)
    sm = sum(float(v) for v in d)
    sq = sum(float(np.float32(v * v)) for v in d)
    thr = sm / 700 + np.sqrt((sq - sm * sm / 700) / 699)
    keep = d.astype(np.float64) <= thr
    assert np.array_equal(got, pts[keep])
    assert keep[:20].sum() < 5 and keep[20:].mean() > 0.8


def test_keyframe_cloud_chain():
    bgr, depth, _, cam = synth_seq(2, seed=5, preset="fr1")
    kc = O.keyframe_cloud(bgr[1], depth[1], cam)
    v = O.voxel(O.cloud(bgr[1], depth[1], cam))
    s, _ = O.sor(v)
    assert np.array_equal(kc, s) and 0.7 * len(v) < len(kc) <= len(v)

"""Seeded synthetic RGB-D sequences (SURVEY.md s8d "Synthetic inputs").

A box room (floor, ceiling, walls at 0.5-4.5 m) plus a few free-standing
textured cards, rendered by per-pixel ray casting from a pinhole camera with
TUM-style radial/tangential distortion.  Texture = hashed blocks (corners for
FAST at threshold 20) + a finer hashed pattern + +-2 sensor noise.  Depth is
u16 = round(z * factor) with ~5 % hashed holes (value 0), like a Kinect map.

Everything is integer-hash / float64 numpy, so a (seed, frame) pair always
gives the same bytes on any host.  The camera moves <= 2 cm and <= 1 deg per
frame; ground-truth poses are returned as Tcw (world -> camera) and can be
written in TUM format for ATE.
"""
from __future__ import annotations

import numpy as np

# TUM intrinsics, IO/DatasetTUM.cpp:61-89 (fr1, fr2, fr3) and ICL, IO/DatasetICL.cpp:37-39.
PRESETS = {
    "fr1": dict(fx=517.306408, fy=516.469215, cx=318.643040, cy=255.313989,
                k1=0.262383, k2=-0.953104, p1=-0.005358, p2=0.002628, k3=1.163314, factor=5000.0),
    "fr2": dict(fx=520.908620, fy=521.007327, cx=325.141442, cy=249.701764,
                k1=0.231222, k2=-0.784899, p1=-0.003257, p2=-0.000105, k3=0.917205, factor=5208.0),
    "fr3": dict(fx=535.4, fy=539.2, cx=320.1, cy=247.6,
                k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0, factor=5000.0),
    # ICL-NUIM: negative fy (IO/DatasetICL.cpp:37-38), no distortion, depth factor 5000
    "icl": dict(fx=481.2, fy=-480.0, cx=319.5, cy=239.5,
                k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0, factor=5000.0),
    # CORBS (IO/DatasetCORBS.cpp:37-39): no distortion, depth factor 5000
    "corbs": dict(fx=468.6, fy=468.61, cx=318.27, cy=243.99,
                  k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0, factor=5000.0),
    # low texture (fr1 camera): blocks twice as large whose intensities differ by <= 23 levels, no fine
    # pattern, so FAST at iniThFAST = 20 finds corners only along the planes' tinted boundaries and most
    # cells fall back to minThFAST = 7 (Features/ORBextractor.cpp:655-661)
    "lowtex": dict(fx=517.306408, fy=516.469215, cx=318.643040, cy=255.313989,
                   k1=0.262383, k2=-0.953104, p1=-0.005358, p2=0.002628, k3=1.163314, factor=5000.0),
}
TEXTURE = {"lowtex": "low"}   # presets whose surfaces are not the default rich texture

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    x = x.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return x


def _hash3(a, b, c) -> np.ndarray:
    with np.errstate(over="ignore"):
        h = _mix(np.asarray(a, dtype=np.int64).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
                 + np.uint64(0x632BE59BD9B4E019))
        h = _mix(h ^ (np.asarray(b, dtype=np.int64).astype(np.uint64) * np.uint64(0xC2B2AE3D27D4EB4F)))
        h = _mix(h ^ (np.asarray(c, dtype=np.int64).astype(np.uint64) * np.uint64(0x165667B19E3779F9)))
    return h


def _rot(rx, ry, rz) -> np.ndarray:
    cx, sx, cy, sy, cz, sz = np.cos(rx), np.sin(rx), np.cos(ry), np.sin(ry), np.cos(rz), np.sin(rz)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


class Scene:
    """Axis-aligned finite planes: (axis, position, (lo_u, hi_u), (lo_v, hi_v), id)."""

    def __init__(self, seed: int):
        rng = np.random.default_rng(seed)
        self.seed = int(seed)
        self.planes = [
            (2, 4.5, (-2.5, 2.5), (-1.8, 1.8), 0),     # back wall  z = 4.5
            (0, -2.4, (-1.8, 1.8), (-1.0, 4.6), 1),    # left wall  x = -2.4  (u=y, v=z)
            (0, 2.4, (-1.8, 1.8), (-1.0, 4.6), 2),     # right wall
            (1, 1.5, (-2.5, 2.5), (-1.0, 4.6), 3),     # floor      y = +1.5 (u=x, v=z)
            (1, -1.7, (-2.5, 2.5), (-1.0, 4.6), 4),    # ceiling
        ]
        for k in range(4):                              # free-standing cards facing the camera
            z = float(rng.uniform(1.4, 3.2))
            x0 = float(rng.uniform(-1.5, 0.8))
            y0 = float(rng.uniform(-0.9, 0.4))
            self.planes.append((2, z, (x0, x0 + float(rng.uniform(0.4, 0.9))),
                                (y0, y0 + float(rng.uniform(0.3, 0.8))), 5 + k))
        self.block = 0.06 + 0.02 * rng.random(len(self.planes))
        self.tint = 0.75 + 0.5 * rng.random((len(self.planes), 3))


def trajectory(n: int, seed: int, start: int = 0) -> np.ndarray:
    """Tcw (4x4, world->camera) for frames start..start+n-1: smooth, <=2 cm and <=1 deg per frame."""
    rng = np.random.default_rng(seed + 7)
    ph = rng.uniform(0, 2 * np.pi, 6)
    out = np.zeros((n, 4, 4))
    for i in range(n):
        t = float(start + i)
        c = np.array([0.45 * np.sin(0.05 * t + ph[0]), 0.15 * np.sin(0.041 * t + ph[1]),
                      -0.4 + 0.3 * np.sin(0.033 * t + ph[2])])
        R = _rot(0.08 * np.sin(0.047 * t + ph[3]), 0.12 * np.sin(0.039 * t + ph[4]),
                 0.04 * np.sin(0.053 * t + ph[5]))      # Rwc
        Tcw = np.eye(4)
        Tcw[:3, :3] = R.T
        Tcw[:3, 3] = -R.T @ c
        out[i] = Tcw
    return out


def _rays(W: int, H: int, cam: dict) -> np.ndarray:
    """Normalised camera rays (x, y, 1) of every distorted pixel (inverse distortion, 5 iters)."""
    u, v = np.meshgrid(np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64))
    x0 = (u - cam["cx"]) / cam["fx"]
    y0 = (v - cam["cy"]) / cam["fy"]
    x, y = x0.copy(), y0.copy()
    k1, k2, p1, p2, k3 = cam["k1"], cam["k2"], cam["p1"], cam["p2"], cam["k3"]
    if k1 != 0.0:
        for _ in range(5):
            r2 = x * x + y * y
            icd = 1.0 / (1 + ((k3 * r2 + k2) * r2 + k1) * r2)
            dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
            dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
            x = (x0 - dx) * icd
            y = (y0 - dy) * icd
    return np.stack([x, y, np.ones_like(x)], axis=-1)


def render(scene: Scene, Tcw: np.ndarray, frame_id: int, cam: dict, W: int = 640, H: int = 480,
           rays: np.ndarray | None = None, texture: str = "rich"):
    if rays is None:
        rays = _rays(W, H, cam)
    Rwc = Tcw[:3, :3].T
    c = -Rwc @ Tcw[:3, 3]
    d = rays @ Rwc.T                       # world ray directions (H, W, 3)
    best_t = np.full((H, W), np.inf)
    best_p = np.full((H, W), -1, dtype=np.int64)
    best_uv = np.zeros((H, W, 2))
    for axis, pos, (lu, hu), (lv, hv), pid in scene.planes:
        oa = [i for i in range(3) if i != axis]
        with np.errstate(divide="ignore", invalid="ignore"):
            t = (pos - c[axis]) / d[..., axis]
        hit = c[None, None, :] + t[..., None] * d
        a, b = hit[..., oa[0]], hit[..., oa[1]]
        ok = (t > 1e-6) & (t < best_t) & (a >= lu) & (a <= hu) & (b >= lv) & (b <= hv)
        best_t = np.where(ok, t, best_t)
        best_p = np.where(ok, pid, best_p)
        best_uv[..., 0] = np.where(ok, a, best_uv[..., 0])
        best_uv[..., 1] = np.where(ok, b, best_uv[..., 1])
    valid = best_p >= 0
    pid = np.where(valid, best_p, 0)
    low = texture == "low"
    blk = scene.block[pid] * (2.0 if low else 1.0)
    ia = np.floor(best_uv[..., 0] / blk).astype(np.int64)
    ib = np.floor(best_uv[..., 1] / blk).astype(np.int64)
    h1 = _hash3(pid * 7919 + scene.seed, ia, ib)
    if low:
        base = 100.0 + (h1 % np.uint64(24)).astype(np.float64)
    else:
        base = 30.0 + (h1 % np.uint64(190)).astype(np.float64)
    fa = np.floor(best_uv[..., 0] / (blk * 0.25)).astype(np.int64)
    fb = np.floor(best_uv[..., 1] / (blk * 0.25)).astype(np.int64)
    h2 = _hash3(pid * 104729 + scene.seed + 1, fa, fb)
    fine = ((h2 % np.uint64(41)).astype(np.float64) - 20.0) * ((h1 >> np.uint64(20)) % np.uint64(2)).astype(np.float64)
    if low:
        fine = 0.0 * fine
    yy, xx = np.meshgrid(np.arange(H), np.arange(W), indexing="ij")
    hn = _hash3(frame_id * 1000003 + scene.seed, yy, xx)
    noise = (hn % np.uint64(5)).astype(np.float64) - 2.0
    inten = np.where(valid, base + fine, 20.0)
    bgr = np.empty((H, W, 3), dtype=np.uint8)
    tint = scene.tint[pid]
    for ch in range(3):
        bgr[..., ch] = np.clip(np.rint(inten * tint[..., ch] + noise), 0, 255).astype(np.uint8)
    z = np.where(valid, best_t, 0.0)       # ray has unit z in camera frame, so t == depth
    holes = (_hash3(frame_id * 31 + scene.seed + 5, yy, xx) % np.uint64(100)) < np.uint64(5)
    depth = np.clip(np.rint(z * cam["factor"]), 0, 65535).astype(np.uint16)
    depth[holes | ~valid] = 0
    return bgr, depth


def sequence(n: int, seed: int = 0, preset: str = "fr1", start: int = 0, W: int = 640, H: int = 480):
    """Returns (bgr[n,H,W,3] u8, depth[n,H,W] u16, Tcw[n,4,4] f64, cam dict)."""
    cam = dict(PRESETS[preset])
    scene = Scene(seed)
    poses = trajectory(n, seed, start)
    rays = _rays(W, H, cam)
    bgr = np.empty((n, H, W, 3), dtype=np.uint8)
    depth = np.empty((n, H, W), dtype=np.uint16)
    tex = TEXTURE.get(preset, "rich")
    for i in range(n):
        bgr[i], depth[i] = render(scene, poses[i], start + i, cam, W, H, rays, tex)
    return bgr, depth, poses, cam


if __name__ == "__main__":
    import time
    t0 = time.time()
    b, d, p, cam = sequence(4, seed=1)
    print("4 frames in %.2fs" % (time.time() - t0), b.shape, d.shape, b.mean(), (d == 0).mean())
    rel = np.linalg.inv(p[0]) @ p[1]
    print("motion/frame: %.4f m" % np.linalg.norm(rel[:3, 3]))

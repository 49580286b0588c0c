"""LDS bank model of k_describe's rBRIEF test reads (csrc/extract.hip, the `Bl[...]` byte reads).

Each test read is a `ds_read_u8`: two 32-lane groups per wave-instruction, bank = (byte address / 4) mod 32,
one LDS cycle per group plus one per extra distinct dword on a bank (MI355X_MICROARCH.md, LDS table).  A
32-lane group is one keypoint: lane hl reads point p of test 8 hl + i in instruction (i, p).  The points are
the pattern rotated by the keypoint's angle (Features/ORBextractor.cpp:45-87), rounded as cvRound, inside the
37 x 37 square staged at a row stride of `stride` bytes from column (x - 18) & ~3.

Prints, per layout, the modelled conflict share (extra cycles / all cycles) of these reads over uniformly
random angles and column phases -- the counter ratio SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE would show if
the test reads were the kernel's only LDS traffic.  Usage: python tools/desc_bank_sim.py [n_keypoints]
"""
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def pattern():
    txt = open(os.path.join(HERE, "..", "rgbd-slam_amd", "csrc", "orb_pattern.inc")).read()
    body = "\n".join(l for l in txt.splitlines() if not l.lstrip().startswith("//"))
    v = np.array([int(t) for t in re.findall(r"-?\d+", body)], np.int64)
    assert v.size == 256 * 4
    return v.reshape(256, 4).astype(np.float32)


def cycles(addr):
    """addr: (..., 32) byte addresses of one lane group -> LDS cycles of that group's ds_read_u8."""
    dw = addr // 4
    bank = dw % 32
    out = np.empty(addr.shape[:-1], np.int64)
    flat_dw, flat_bank = dw.reshape(-1, 32), bank.reshape(-1, 32)
    o = out.reshape(-1)
    for g in range(flat_dw.shape[0]):
        uniq = np.unique(flat_dw[g])
        o[g] = np.bincount(uniq % 32, minlength=32).max()
    return out


def model(n, stride, seed=0, order=None):
    P = pattern()
    rng = np.random.default_rng(seed)
    ang = rng.uniform(0, 2 * np.pi, n).astype(np.float32)
    ph = rng.integers(0, 4, n)
    a, s = np.cos(ang)[:, None], np.sin(ang)[:, None]
    tot = ext = 0
    for p in range(2):
        x, y = P[:, 2 * p][None, :], P[:, 2 * p + 1][None, :]
        r = np.rint(x * s + y * a).astype(np.int64) + 18   # rint: round half to even, as cvRound
        c = np.rint(x * a - y * s).astype(np.int64) + 18
        addr = r * stride + c + ph[:, None]                 # (n, 256): test t's byte
        idx = np.arange(256).reshape(32, 8) if order is None else order   # lane hl, instruction i
        for i in range(8):
            cyc = cycles(addr[:, idx[:, i]])
            tot += cyc.sum()
            ext += (cyc - 1).sum()
    return ext / tot, tot / (n * 16)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    for stride in (48, 40, 44, 52, 56, 64):
        share, cyc = model(n, stride)
        print(f"row stride {stride:3d} B: conflict share {share:.3f}, {cyc:.2f} LDS cycles per 32-lane read")
    # the best static lane order for one angle cannot hold for others: random permutation of the tests
    rng = np.random.default_rng(1)
    share, cyc = model(n, 48, order=rng.permutation(256).reshape(32, 8))
    print(f"row stride  48 B, tests permuted over lanes: conflict share {share:.3f}, {cyc:.2f} cycles")
    # reference point: 32 uniformly random dwords of a 444-dword square
    rnd = np.random.default_rng(2).integers(0, 444 * 4, (n * 16, 32))
    c = cycles(rnd)
    print(f"uniform random bytes: conflict share {(c - 1).sum() / c.sum():.3f}, {c.mean():.2f} cycles")


if __name__ == "__main__":
    main()

"""GPU parity: extraction stages of the HIP path vs the CPU oracle (bit-exact).

Calls go through the C ABI (librgbd_hip.so).  Inputs: seeded synthetic RGB-D frames
(tools/synth.py), TUM fr1 (distorted) and fr3 (undistorted) intrinsics.
"""
import numpy as np
import pytest

from conftest import synth_seq

pytestmark = pytest.mark.gpu


def _ctx(pkg, cam, nfeat=1000, max_batch=4):
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    return pkg.Context(640, 480, max_batch=max_batch, orb=pkg.orb_params(nfeat), cam=c)


@pytest.fixture(scope="module")
def fr1_ctx(pkg, seq_fr1):
    return _ctx(pkg, seq_fr1[3])


def test_pyramid_bit_exact(pkg, oracle, seq_fr1, fr1_ctx):
    bgr, depth, _, cam = seq_fr1
    p = oracle.orb_params(1000)
    t = oracle.tables(p)
    for f in range(2):
        fr1_ctx.frame(bgr[f], depth[f])
        ref = oracle.pyramid(oracle.gray(bgr[f]), p)
        for l in range(8):
            got = fr1_ctx.debug_level(0, l, int(t["w"][l]), int(t["h"][l]))
            assert np.array_equal(got, ref[l]), f"frame {f} level {l}: {np.count_nonzero(got != ref[l])} px differ"


def test_blurred_pyramid_bit_exact(pkg, oracle, seq_fr1, fr1_ctx):
    # k_blur: GaussianBlur 7x7 sigma 2 REFLECT_101 of every level (Features/ORBextractor.cpp:745-746)
    bgr, depth, _, cam = seq_fr1
    p = oracle.orb_params(1000)
    t = oracle.tables(p)
    fr1_ctx.frame(bgr[0], depth[0])
    ref = oracle.pyramid(oracle.gray(bgr[0]), p)
    for l in range(8):
        got = fr1_ctx.debug_blurred(0, l, int(t["w"][l]), int(t["h"][l]))
        want = oracle.blur(ref[l])
        assert np.array_equal(got, want), f"level {l}: {np.count_nonzero(got != want)} px differ"


def test_fast_candidates_bit_exact(pkg, oracle, seq_fr1, fr1_ctx):
    bgr, depth, _, cam = seq_fr1
    p = oracle.orb_params(1000)
    fr1_ctx.frame(bgr[1], depth[1])
    ref = oracle.pyramid(oracle.gray(bgr[1]), p)
    for l in range(8):
        want = oracle.level_candidates(ref[l], p)
        got = fr1_ctx.debug_candidates(0, l)
        assert got.shape == want.shape, f"level {l}: {len(got)} vs {len(want)} candidates"
        assert np.array_equal(got, want), f"level {l}"


def test_quadtree_bit_exact(pkg, oracle, seq_fr1, fr1_ctx):
    bgr, depth, _, cam = seq_fr1
    p = oracle.orb_params(1000)
    t = oracle.tables(p)
    fr1_ctx.frame(bgr[2], depth[2])
    ref = oracle.pyramid(oracle.gray(bgr[2]), p)
    for l in range(8):
        cand = oracle.level_candidates(ref[l], p)
        w, h = int(t["w"][l]), int(t["h"][l])
        want = oracle.distribute(cand, 16, w - 16, 16, h - 16, int(t["nfeat"][l]))
        got = fr1_ctx.debug_selected(0, l)
        assert np.array_equal(got, want), f"level {l}: {len(got)} vs {len(want)}"


@pytest.mark.parametrize("preset,nfeat", [("corbs", 1000), ("fr1", 1000), ("fr2", 2000)])
def test_quadtree_paths_bit_exact(pkg, oracle, preset, nfeat):
    """k_distribute's three key-state paths against the oracle's DistributeOctTree, every level: keys and node ids
    in LDS (the small levels), node ids in LDS with the keys in the HBM scratch (levels 0-3 at 1000 kp: up to
    ~11.2k candidates on CORBS level 0), both in the HBM scratch (level 0 at 2000 kp, u16 node ids)."""
    bgr, depth, _, cam = synth_seq(2, seed={"corbs": 7, "fr1": 3, "fr2": 29}[preset], preset=preset)
    ctx = _ctx(pkg, cam, nfeat=nfeat)
    p = oracle.orb_params(nfeat)
    t = oracle.tables(p)
    for f in range(2):
        ctx.frame(bgr[f], depth[f])
        ref = oracle.pyramid(oracle.gray(bgr[f]), p)
        for l in range(8):
            cand = oracle.level_candidates(ref[l], p)
            if l == 0 and preset != "fr2":
                assert len(cand) > 10000   # CORBS / fr1 seed 3: level 0 above 10k candidates
            w, h = int(t["w"][l]), int(t["h"][l])
            want = oracle.distribute(cand, 16, w - 16, 16, h - 16, int(t["nfeat"][l]))
            got = ctx.debug_selected(0, l)
            assert np.array_equal(got, want), f"{preset} frame {f} level {l}: {len(got)} vs {len(want)}"
        want_f = oracle.frame(bgr[f], depth[f], p, oracle.camera(cam))
        _assert_frame_equal(ctx.frame(bgr[f], depth[f]), want_f, f"{preset} frame {f}")
    ctx.close()


def test_quadtree_several_roots_bit_exact(pkg, oracle):
    """A 1024 x 480 frame: every level's DistributeOctTree starts from nIni = round(dX / dY) = 2 roots
    (ORBextractor.cpp:420-446), so the root split by hX, the root counts and the root compaction run (the
    640 x 480 levels all start from one root, which k_distribute gathers without them)."""
    bgr, depth, _, cam = synth_seq(2, seed=13, preset="fr1")
    wide_bgr = np.ascontiguousarray(np.concatenate([bgr[0], bgr[1][:, ::-1][:, :384]], axis=1))
    wide_dep = np.ascontiguousarray(np.concatenate([depth[0], depth[1][:, ::-1][:, :384]], axis=1))
    h, w = wide_dep.shape
    assert (w, h) == (1024, 480)
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    ctx = pkg.Context(w, h, max_batch=1, orb=pkg.orb_params(1000), cam=c)
    p = oracle.orb_params(1000)
    t = oracle.tables(p, w, h)
    got_f = ctx.frame(wide_bgr, wide_dep)
    ref = oracle.pyramid(oracle.gray(wide_bgr), p)
    roots = []
    for l in range(8):
        lw, lh = int(t["w"][l]), int(t["h"][l])
        roots.append(int(round((lw - 32) / (lh - 32))))
        cand = oracle.level_candidates(ref[l], p)
        want = oracle.distribute(cand, 16, lw - 16, 16, lh - 16, int(t["nfeat"][l]))
        got = ctx.debug_selected(0, l)
        assert np.array_equal(got, want), f"level {l}: {len(got)} vs {len(want)}"
    assert min(roots) >= 2, roots
    _assert_frame_equal(got_f, oracle.frame(wide_bgr, wide_dep, p, oracle.camera(cam)), "1024x480")
    ctx.close()


def _assert_frame_equal(got, want, tag=""):
    assert len(got["kps"]) == len(want["kps"]), f"{tag} count {len(got['kps'])} vs {len(want['kps'])}"
    for name in ("kps", "kps_un"):
        g, w = got[name], want[name]
        for fld in g.dtype.names:
            bad = np.flatnonzero(g[fld] != w[fld])
            assert len(bad) == 0, f"{tag} {name}.{fld}: {len(bad)} differ, first {bad[:5]} {g[fld][bad[:3]]} vs {w[fld][bad[:3]]}"
    bad = np.flatnonzero(np.any(got["desc"] != want["desc"], axis=1))
    assert len(bad) == 0, f"{tag} desc rows differ: {len(bad)} first {bad[:8]}"
    assert np.array_equal(got["xyz"].view(np.uint32), want["xyz"].view(np.uint32)), f"{tag} xyz"


@pytest.mark.parametrize("preset", ["fr1", "fr3", "icl"])
def test_frame_bit_exact(pkg, oracle, preset):
    bgr, depth, _, cam = synth_seq(3, seed={"fr1": 5, "fr3": 11, "icl": 17}[preset], preset=preset)
    ctx = _ctx(pkg, cam)
    p = oracle.orb_params(1000)
    oc = oracle.camera(cam)
    for f in range(3):
        got = ctx.frame(bgr[f], depth[f])
        want = oracle.frame(bgr[f], depth[f], p, oc)
        _assert_frame_equal(got, want, f"{preset} frame {f}")
    ctx.close()


def test_frame_2000kp(pkg, oracle):
    bgr, depth, _, cam = synth_seq(2, seed=21, preset="fr2")
    ctx = _ctx(pkg, cam, nfeat=2000)
    p = oracle.orb_params(2000)
    oc = oracle.camera(cam)
    got = ctx.frame(bgr[0], depth[0])
    want = oracle.frame(bgr[0], depth[0], p, oc)
    assert len(want["kps"]) > 1500
    _assert_frame_equal(got, want, "2000kp")
    ctx.close()


def test_detect_and_compute_gray(pkg, oracle, seq_fr1, fr1_ctx):
    bgr, depth, _, cam = seq_fr1
    g = oracle.gray(bgr[3])
    kps, desc = fr1_ctx.detect_and_compute(g)
    wk, wd = oracle.detect_and_compute(g, oracle.orb_params(1000))
    assert len(kps) == len(wk)
    for fld in kps.dtype.names:
        assert np.array_equal(kps[fld], wk[fld]), fld
    assert np.array_equal(desc, wd)


def test_flat_and_low_contrast_images(pkg, oracle, fr1_ctx):
    """Edge cases: flat image (no corners at any threshold) and a low-contrast image where the
    per-cell threshold fallback 20 -> 7 decides (Features/ORBextractor.cpp:655-661)."""
    p = oracle.orb_params(1000)
    flat = np.full((480, 640), 77, np.uint8)
    kps, desc = fr1_ctx.detect_and_compute(flat)
    assert len(kps) == 0
    rs = np.random.default_rng(7)
    low = (100 + rs.integers(0, 14, size=(60, 80))).astype(np.uint8)
    low = np.kron(low, np.ones((8, 8), np.uint8))
    kps, desc = fr1_ctx.detect_and_compute(low)
    wk, wd = oracle.detect_and_compute(low, p)
    assert len(kps) == len(wk) and len(wk) > 0
    for fld in kps.dtype.names:
        assert np.array_equal(kps[fld], wk[fld]), fld
    assert np.array_equal(desc, wd)


def test_batch_extract_matches_single(pkg, oracle, seq_fr1):
    import torch
    bgr, depth, _, cam = seq_fr1
    ctx = _ctx(pkg, cam, max_batch=4)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    ctx.extract_batch(d_bgr.data_ptr(), d_dep.data_ptr(), 4)
    p = oracle.orb_params(1000)
    oc = oracle.camera(cam)
    for f in range(4):
        _assert_frame_equal(ctx.batch_frame(f), oracle.frame(bgr[f], depth[f], p, oc), f"batch frame {f}")
    ctx.close()


@pytest.mark.gpu
def test_batch16_xcd_mapping_matches_oracle(pkg, oracle, seq_fr1):
    """B % 8 == 0 takes the XCD-local 1-D grids of k_fast; frames of the second group of eight must
    land on their own slots.  Frames are the fr1 sequence and its mirror images (all distinct)."""
    import torch
    bgr, depth, _, cam = seq_fr1
    fb = np.concatenate([bgr, bgr[:, :, ::-1], bgr[:, ::-1], bgr[:, ::-1, ::-1]])
    fd = np.concatenate([depth, depth[:, :, ::-1], depth[:, ::-1], depth[:, ::-1, ::-1]])
    fb, fd = np.ascontiguousarray(fb), np.ascontiguousarray(fd)
    ctx = _ctx(pkg, cam, max_batch=16)
    d_bgr = torch.from_numpy(fb).cuda()
    d_dep = torch.from_numpy(fd.view(np.int16)).cuda()
    ctx.extract_batch(d_bgr.data_ptr(), d_dep.data_ptr(), 16)
    p = oracle.orb_params(1000)
    oc = oracle.camera(cam)
    for f in (0, 5, 9, 15):
        _assert_frame_equal(ctx.batch_frame(f), oracle.frame(fb[f], fd[f], p, oc), f"batch16 frame {f}")
    ctx.close()


def test_context_over_4gib_of_pyramids_rejected(pkg):
    """k_describe addresses the pyramids with 32-bit offsets: a context whose max_batch x pyramid bytes
    passes 4 GiB is refused with RGBD_ERR_CAPACITY before any allocation (DESIGN.md hard limits)."""
    import ctypes as C
    lib = pkg.lib()
    h = C.c_void_p()
    st = lib.rgbd_create(0, 640, 480, 5000, C.byref(pkg.orb_params()), C.byref(pkg.camera(500, 500, 320, 240)),
                         C.byref(h))
    assert st == 3, st   # RGBD_ERR_CAPACITY
    assert b"4 GiB" in lib.rgbd_last_error(h)
    lib.rgbd_destroy(h)


def test_fast_rank16_row_newbcast(pkg):
    """k_fast's emission rank for 16-lane cells on its own (csrc/extract.hip fast_rank16: ballot + mbcnt,
    row_newbcast:0 / :15 DPP moves kept as v_mov_b32_dpp): every set lane's slot is its cell's running count
    in raster order (rows, then lanes), each cell (16-lane row of the wave) counting from its own base."""
    ctx = pkg.Context(640, 480, max_batch=1)
    rs = np.random.RandomState(7)
    flags = np.concatenate([(rs.rand(40, 64) < p).astype(np.uint8) for p in (0.05, 0.3, 0.7, 1.0)]
                           + [np.zeros((3, 64), np.uint8), np.eye(64, dtype=np.uint8)])
    slots, counts = ctx.debug_fast_rank16(flags)
    ctx.close()
    want = np.full(flags.shape, 0xffffffff, np.uint64)
    cnt = [1000 * g for g in range(4)]
    for r in range(flags.shape[0]):
        for lane in range(64):
            if flags[r, lane]:
                want[r, lane] = cnt[lane >> 4]
                cnt[lane >> 4] += 1
    assert np.array_equal(slots.astype(np.uint64), want)
    assert np.array_equal(counts, np.repeat(np.array(cnt, np.uint32), 16))

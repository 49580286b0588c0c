"""Keyframe dense cloud on the device (cloud.hip) against the oracle (oracle/orc_cloud.cpp): every point
bit-identical (positions, colours, order), single-frame and batched entry points."""
import numpy as np
import pytest

from conftest import synth_seq

pytestmark = pytest.mark.gpu


def _ctx(pkg, cam, B=1):
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    return pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(1000), cam=c)


@pytest.mark.parametrize("preset,seed", [("fr1", 5), ("fr2", 22), ("icl", 17)])
def test_keyframe_cloud_bit_exact(pkg, oracle, preset, seed):
    bgr, depth, _, cam = synth_seq(2, seed=seed, preset=preset)
    ctx = _ctx(pkg, cam)
    for f in range(2):
        got = ctx.keyframe_cloud(bgr[f], depth[f])
        want = oracle.keyframe_cloud(bgr[f], depth[f], cam)
        assert len(got) == len(want) > 500
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
        # Frame::createCloud's own inputs: mImDepth = imDepth.convertTo(CV_32F, 1/factor) (Core/Frame.cpp:48)
        dimg = depth[f].astype(np.float32) * (np.float32(1.0) / np.float32(cam["factor"])) + np.float32(0.0)
        got32 = ctx.keyframe_cloud_f32(bgr[f], dimg)
        assert np.array_equal(got32.view(np.uint8), want.view(np.uint8))
    ctx.close()


def test_keyframe_cloud_batch_and_stages(pkg, oracle):
    import torch
    B = 5
    bgr, depth, _, cam = synth_seq(B, seed=41, preset="fr1")
    ctx = _ctx(pkg, cam, B)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    frames = [4, 0, 2]
    got = ctx.keyframe_cloud_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, frames)
    for k, f in enumerate(frames):
        want = oracle.keyframe_cloud(bgr[f], depth[f], cam)
        assert np.array_equal(got[k].view(np.uint8), want.view(np.uint8))
    # other parameters: no pass-through limits hit, coarser voxels, k = 20
    prm = pkg.cloud_params(stride=5, zmin=0.1, zmax=10.0, leaf=0.1, sor_k=20, sor_std=2.0)
    g2 = ctx.keyframe_cloud(bgr[1], depth[1], prm)
    v = oracle.voxel(oracle.cloud(bgr[1], depth[1], cam, res=5, zmin=0.1, zmax=10.0), leaf=0.1)
    w2, _ = oracle.sor(v, k=20, std_mul=2.0)
    assert np.array_equal(g2.view(np.uint8), w2.view(np.uint8))
    ctx.close()

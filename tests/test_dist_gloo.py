"""CPU, world size 2 over gloo: sharding with halo, the pose all-gather and exact stitching used by
bench.py's multi-GPU path (RCCL on the GPU box, same code)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from conftest import load_pkg, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from conftest import load_pkg
    load_pkg()
    import rgbd_slam_amd.dist as D
    import synth
    n = 13
    gt = synth.trajectory(n, seed=5)
    lo, hi = D.shard_range(n, world, rank)
    # "track" the chunk exactly from ground truth, relative to the chunk's first frame
    local = gt[lo:hi] @ np.linalg.inv(gt[lo])
    if rank == 0:
        local = gt[lo:hi]
    pad = np.zeros((8, 4, 4), np.float32)
    pad[:len(local)] = local
    allp = D.gather_poses(torch.from_numpy(pad.reshape(8, 16)), world)
    if rank == 0:
        chunks = []
        for r in range(world):
            l2, h2 = D.shard_range(n, world, r)
            chunks.append(allp[r].numpy().reshape(8, 4, 4)[:h2 - l2])
        out_q.put(D.stitch(chunks, gt[0]))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_ranges_cover_sequence():
    load_pkg()
    import rgbd_slam_amd.dist as D
    for n in (10, 13, 64):
        for world in (1, 2, 3, 8):
            frames = []
            for r in range(world):
                lo, hi = D.shard_range(n, world, r)
                frames.extend(range(lo + (1 if r > 0 else 0), hi))
                if r > 0:
                    assert lo == D.shard_range(n, world, r - 1)[1] - 1      # one halo frame
            assert frames == list(range(n))


def test_gather_and_stitch_world2():
    import synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    traj = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    gt = synth.trajectory(13, seed=5)
    assert traj.shape == (13, 4, 4)
    assert np.allclose(traj, gt, atol=1e-5)


def test_ate_tool():
    import ate
    import synth
    gt = synth.trajectory(30, seed=2)
    assert ate.ate_rmse(gt, gt) < 1e-9
    noisy = gt.copy()
    noisy[:, :3, 3] += np.random.default_rng(0).normal(scale=0.01, size=(30, 3))
    assert 0.003 < ate.ate_rmse(noisy, gt) < 0.03
    assert len(ate.tum_lines(np.arange(3) * 0.03, gt[:3])) == 3

"""CPU, world size 2 over gloo: sharding with halo, the pose all-gather and exact stitching used by
bench.py's multi-GPU path (RCCL on the GPU box, same code), and the config-5 hand-off: the gathered,
stitched trajectory feeding the host PoseGraph on rank 0 (Solver/PoseGraph.cpp:350-368).  The hand-off
is unmeasured on hardware (no multi-GPU run is launched from here)."""
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


def _noisy_chunk(gt, lo, hi, seed):
    """VO over frames lo..hi-1 from an identity pose at lo: ground-truth relative motion with a
    seeded per-step perturbation (the same numbers on every rank and in the single-process check)."""
    rs = np.random.default_rng(seed + lo)
    out = [np.eye(4)]
    for j in range(lo + 1, hi):
        rel = gt[j] @ np.linalg.inv(gt[j - 1])
        rel[:3, 3] += rs.normal(scale=0.004, size=3)
        out.append(rel @ out[-1])
    return np.array(out, np.float32)


def _posegraph_handoff(pkg, traj, gt):
    """Rank 0 after the gather: keyframes by Tracking::needKeyFrame, reference edges from the trajectory,
    plus ground-truth 'local' edges every third keyframe (the device RansacSE3 measurements of the
    real path), then optimize(10) and re-anchor every frame on its keyframe."""
    from rgbd_slam_amd import posegraph as PG
    kfs = PG.select_keyframes(list(traj))
    g = PG.PoseGraph(pkg)
    for k in kfs:
        g.insert_keyframe(k, traj[k])
    for a, b in zip(kfs[3::3], kfs[::3]):
        g.add_edge(a, b, (gt[a] @ np.linalg.inv(gt[b])).astype(np.float64))   # T21 = Tcw_a Tcw_b^-1
    chi0 = g.chi2()
    res = g.optimize(10)
    corr = PG.corrected_trajectory(list(traj), kfs, {k: g.kf[k]["Tcw"] for k in kfs})
    g.close()
    return kfs, chi0, res, corr


def _worker_pg(rank, world, port, out_q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from conftest import load_pkg
    pkg = load_pkg()
    import rgbd_slam_amd.dist as D
    import synth
    n = 60
    gt = synth.trajectory(n, seed=7)
    lo, hi = D.shard_range(n, world, rank)
    local = _noisy_chunk(gt, lo, hi, 11)
    pad = np.zeros((40, 4, 4), np.float32)
    pad[:len(local)] = local
    allp = D.gather_poses(torch.from_numpy(pad.reshape(40, 16)), world)
    if rank == 0:
        chunks = []
        for r in range(world):
            l2, h2 = D.shard_range(n, world, r)
            chunks.append(allp[r].numpy().reshape(40, 4, 4)[:h2 - l2])
        traj = D.stitch(chunks, gt[0].astype(np.float32))
        out_q.put((traj, _posegraph_handoff(pkg, traj, gt)))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_then_posegraph_world2():
    """config 5's hand-off at world size 2 equals the single-process pipeline on the same chunks."""
    import synth
    import ate
    pkg = load_pkg()
    import rgbd_slam_amd.dist as D
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_pg, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    traj, (kfs, chi0, res, corr) = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 60
    gt = synth.trajectory(n, seed=7)
    chunks = [_noisy_chunk(gt, *D.shard_range(n, 2, r), 11) for r in range(2)]
    want = D.stitch(chunks, gt[0].astype(np.float32))
    assert np.array_equal(traj, want)                  # the gather moves the bytes unchanged
    kfs1, chi01, res1, corr1 = _posegraph_handoff(pkg, want, gt)
    assert kfs == kfs1 and chi0 == chi01 and res == res1 and np.array_equal(corr, corr1)
    assert len(kfs) > 5 and res is not None and res[0] < chi0
    assert ate.ate_rmse(corr, gt) < ate.ate_rmse(traj, gt)


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

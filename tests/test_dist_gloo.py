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


def _worker_mode(rank, world, port, out_q, mode, batch):
    """bench.py's rank path on CPU: the rank's workload (dist.workload), VO over its frames (ground-truth
    motion + seeded noise), the padded pose block all-gathered (gather_poses into a reused buffer: the bench's
    one PoseGraph hand-off after its timed region) and rank 0's trajectories (dist.trajectories)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    load_pkg()
    import rgbd_slam_amd.dist as D
    import synth
    n_global, lo, hi, seed = D.workload(mode, batch, world, rank)
    gt = synth.trajectory(n_global, seed=seed)
    local = _noisy_chunk(gt, lo, hi, seed)
    if rank == 0 or mode == "sequences":   # tracked from the sequence's own first pose
        local = np.einsum("nij,jk->nik", local, gt[lo]).astype(np.float32)
    pad = torch.zeros((batch + 1, 16), dtype=torch.float32)
    out = torch.empty((world, batch + 1, 16), dtype=torch.float32)
    for _ in range(2):   # a reused hand-off buffer gathers the same blocks again
        pad.numpy()[:hi - lo] = local.reshape(-1, 16)
        allp = D.gather_poses(pad, world, out=out)
    assert allp.data_ptr() == out.data_ptr()
    if rank == 0:
        out_q.put(D.trajectories(mode, allp.numpy(), n_global, world, gt[0].astype(np.float32)))
    dist.barrier()
    dist.destroy_process_group()


def _run_mode(mode, batch, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_mode, args=(r, world, port, q, mode, batch)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def test_sequences_mode_world2():
    """BASELINE config 4 (--mode sequences): every rank tracks its own independent sequence (seeded by its
    rank, no frame shared, no collective on the data path); rank 0 receives every rank's trajectory through
    the pose all-gather, each equal to what one process tracking that sequence alone produces."""
    import synth
    load_pkg()
    import rgbd_slam_amd.dist as D
    batch = 17
    got = _run_mode("sequences", batch)
    assert len(got) == 2
    for r in range(2):
        n_global, lo, hi, seed = D.workload("sequences", batch, 2, r)
        assert (n_global, lo, hi) == (batch, 0, batch) and seed == 1000 + 7919 * r
        gt = synth.trajectory(n_global, seed=seed)
        want = np.einsum("nij,jk->nik", _noisy_chunk(gt, 0, batch, seed), gt[0]).astype(np.float32)
        assert np.array_equal(got[r], want)
    assert not np.allclose(got[0], got[1])   # independent sequences


def test_chunks_mode_world2_through_bench_helpers():
    """--mode chunks (configs 2, 3, 5) through the same helpers: contiguous chunks with one halo frame, the
    gathered chunks stitched on rank 0 into the one sequence a single process would track."""
    import synth
    load_pkg()
    import rgbd_slam_amd.dist as D
    batch = 9
    (traj,) = _run_mode("chunks", batch)
    n_global, _, _, seed = D.workload("chunks", batch, 2, 0)
    assert n_global == 18 and D.workload("chunks", batch, 2, 1)[1:3] == D.shard_range(18, 2, 1)
    gt = synth.trajectory(n_global, seed=seed)
    chunks = []
    for r in range(2):
        lo, hi = D.shard_range(n_global, 2, r)
        c = _noisy_chunk(gt, lo, hi, seed)
        chunks.append(np.einsum("nij,jk->nik", c, gt[0]).astype(np.float32) if r == 0 else c)
    want = D.stitch(chunks, gt[0].astype(np.float32))
    assert traj.shape == (n_global, 4, 4)
    assert np.array_equal(traj, want)


def test_bench_refuses_world_size_mismatch():
    """Under a launcher (WORLD_SIZE set) a --gpus that disagrees is refused before any GPU work."""
    import subprocess
    import sys
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"] + ["--steps", "1", "--no-cpu-baseline"],
                         capture_output=True, text=True, timeout=60, env=env)
    assert out.returncode == 2 and "WORLD_SIZE=2 but --gpus 1" in out.stderr

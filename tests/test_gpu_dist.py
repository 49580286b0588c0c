"""GPU, world size 2 on the one card: the multi-GPU chunk path of bench.py / dist.py driven by the HIP
tracker itself.  Each rank extracts, matches and solves PnPRansac for its own contiguous
chunk of one sequence (rank 1 starts one frame early, at the halo frame, from an identity pose), the poses
are all-gathered (gloo here: two ranks cannot share one device under RCCL; the RCCL branch of
dist.gather_poses is the same call), and rank 0 stitches them.

Checks: every pair's PnPRansac status and inlier count on the ranks equal the single-process run over
the whole sequence bit for bit (pairs are independent with discardOutliers = false, and PnPRansac seeds
its RNG per call), and the stitched trajectory equals the single-process chained trajectory up to the
float re-association of the chunk composition (Tcw_j = T(j <- halo) Tcw_halo)."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

N_FRAMES = 17


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _track(pkg, torch, bgr, depth, cam, pose0):
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"], cam["k3"],
                   cam["factor"])
    ctx = pkg.Context(640, 480, max_batch=len(bgr), orb=pkg.orb_params(1000), cam=c)
    d_bgr = torch.from_numpy(np.ascontiguousarray(bgr)).cuda()
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).cuda()
    out = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), len(bgr), 0.9, pkg.pnp_params(500, 3.0, 0.85, 10),
                              pose0)
    torch.cuda.synchronize()
    ctx.close()
    return out


def _worker(rank, world, port, out_q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from conftest import load_pkg, synth_seq
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = load_pkg()
    import rgbd_slam_amd.dist as D
    bgr, depth, gt, cam = synth_seq(N_FRAMES, seed=41, preset="fr1")
    lo, hi = D.shard_range(N_FRAMES, world, rank)
    pose0 = gt[lo].astype(np.float32) if rank == 0 else np.eye(4, dtype=np.float32)
    poses, status, ninl, _ = _track(pkg, torch, bgr[lo:hi], depth[lo:hi], cam, pose0)
    pad = np.zeros((N_FRAMES, 16), np.float32)
    pad[:hi - lo] = poses.reshape(-1, 16)
    allp = D.gather_poses(torch.from_numpy(pad), world)
    meta = torch.zeros((N_FRAMES, 2), dtype=torch.int32)
    meta[:hi - lo, 0] = torch.from_numpy(status)
    meta[:hi - lo, 1] = torch.from_numpy(ninl)
    allm = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(allm, meta)
    if rank == 0:
        chunks, stat = [], []
        for r in range(world):
            l2, h2 = D.shard_range(N_FRAMES, world, r)
            chunks.append(allp[r].numpy().reshape(N_FRAMES, 4, 4)[:h2 - l2])
            m = allm[r].numpy()[:h2 - l2]
            stat.append(m if r == 0 else m[1:])   # row 0 of a later chunk is its halo frame (no pair)
        out_q.put((D.stitch(chunks, gt[0]), np.concatenate(stat)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_on_one_card_match_single_process(pkg):
    import torch
    import torch.multiprocessing as mp
    from conftest import synth_seq
    bgr, depth, gt, cam = synth_seq(N_FRAMES, seed=41, preset="fr1")
    want_p, want_s, want_n, _ = _track(pkg, torch, bgr, depth, cam, gt[0].astype(np.float32))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    traj, stat = q.get(timeout=110)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert np.array_equal(stat[:, 0], want_s) and np.array_equal(stat[:, 1], want_n)
    assert want_s[1:].all()
    assert traj.shape == want_p.shape
    assert np.allclose(traj, want_p, atol=2e-5), np.abs(traj - want_p).max()


_RCCL_CHILD = r"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
from conftest import load_pkg
load_pkg()
import rgbd_slam_amd.dist as D
import torch
import torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%s" % sys.argv[2], rank=0, world_size=1)
assert dist.get_backend() == "nccl"
local = torch.arange(5 * 16, dtype=torch.float32, device="cuda").reshape(5, 16) * 0.25
out = D.gather_poses(local, 1, force_collective=True)
torch.cuda.synchronize()
assert tuple(out.shape) == (1, 5, 16) and out.device.type == "cuda"
assert torch.equal(out[0], local)
dist.barrier()
dist.destroy_process_group()
print("rccl all_gather_into_tensor ok")
"""


def test_rccl_gather_call_site_world1():
    """dist.gather_poses' RCCL branch (all_gather_into_tensor over the "nccl" backend, which is RCCL on ROCm)
    executed on the card: a fresh child process (no GPU call before its own) initialises a world-1 "nccl"
    process group and gathers a pose block through the collective; the result equals the input."""
    import subprocess
    import sys
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    out = subprocess.run([sys.executable, "-c", _RCCL_CHILD, ROOT, str(_free_port())], capture_output=True, text=True,
                         timeout=110, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "rccl all_gather_into_tensor ok" in out.stdout


def _bench_line(out):
    import json
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:] + out.stderr[-3000:]
    return json.loads(lines[0])


_BENCH_SMALL = ["--steps", "2", "--warmup", "1", "--batch", "64", "--unique", "16", "--no-cpu-baseline",
                "--flag-chain-steps", "0", "--flag-chain-one-steps", "0", "--se3-chain-one-steps", "0",
                "--no-kernel-timing"]


@pytest.mark.parametrize("mode", ["chunks", "sequences"])
def test_bench_spawns_its_ranks(mode):
    """bench.py --gpus 2 without a launcher spawns its two ranks itself (here sharing card 0 over gloo: the
    box has one GPU); rank 0 prints one line whose n_gpus is the process group's size, with the whole-job
    frames of both ranks.  BASELINE configs 4 (sequences) and 2/3/5 (chunks)."""
    import subprocess
    import sys
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                          "--mode", mode] + _BENCH_SMALL, capture_output=True, text=True, timeout=110, env=env)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    line = _bench_line(out)
    assert line["n_gpus"] == 2 and line["value"] > 0 and line["tracked_frac"] > 0.9
    assert line["config"]["mode"] == mode
    # the poses are gathered once, after the timed region (the PoseGraph hand-off), never per step
    assert line["hand_off"]["collective"] == "all_gather_into_tensor" and line["hand_off"]["timed"] is False


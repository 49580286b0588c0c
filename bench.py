"""bench.py -- frames/s of the RGB-D tracking front end on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch of B synthetic 640x480 RGB-D frames that are
already resident in HBM: ORB extraction (gray, pyramid, FAST cells, quadtree, orientation, blur,
rBRIEF, undistort, unproject) -> Hamming knn-2 of consecutive frames -> Matcher filter fused with the
3D-2D gather -> PnPRansac (EPnP hypotheses, RANSAC replay, Gauss-Newton refinement) for every pair ->
poses; then the poses are all-gathered over RCCL (PoseGraph hand-off) when N > 1.  Each rank tracks
its own sequence chunk ("weak" scaling).  --solver se3 runs the reference tracker's RansacSE3 chain
(with second-reference retry) instead.

    python bench.py [--gpus N --steps K --warmup W --batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU)

Prints one JSON line (rank 0) with the roofline of the dominant kernel (HIP events on the
library stream over the timed region) and the CPU oracle timed on the host (cpu_baseline).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
VALU_PEAK_TOPS = 78.64    # 256 CUs x 4 SIMDs x 32 lanes/clk x 2.4 GHz (= FP32 vector peak 157.3 TF / 2 per FMA)


def kernel_bytes(name, nframes, n_kp, n_match, pyr_bytes, W, H):
    """Algorithmic HBM bytes of one launch (DESIGN.md 'Roofline accounting')."""
    if name == "k_gray":
        return nframes * (W * H * 3 + W * H)
    if name == "k_pyramid":       # BGR read once, gray level 0 + levels 1..7 written
        return nframes * (W * H * 3 + pyr_bytes)
    if name == "k_fast":
        return nframes * pyr_bytes
    if name == "k_describe":      # 31-row IC disk (9 dwords) + 37-row blurred square (11 dwords) + KeyPoint, desc
        return nframes * n_kp * (31 * 36 + 37 * 44 + 28 + 32)
    if name == "k_blur":          # every level read once, its blur written once
        return nframes * 2 * pyr_bytes
    if name == "k_undistort":     # KeyPoint read, depth sample, KeyPoint (undistorted) + xyz written
        return nframes * n_kp * (28 + 2 + 28 + 12)
    if name == "k_knn2":
        return nframes * (2 * n_kp * 32 + n_kp * 16)
    if name == "k_distribute":
        return nframes * n_kp * 8
    if name == "k_ransac_hyp":
        return n_match * 24
    if name == "k_match_gather":  # knn rows + depth of both frames + kept pairs' xyz/pixel gathers and writes
        return nframes * (n_kp * 16 + 2 * n_kp * 4 + n_match * (12 + 8) * 2)
    if name == "k_pnp_hyp":       # per hypothesis: its problem's points (p3 + p2) read once
        return n_match * 20
    svo_pyr = sum((W >> l) * (H >> l) for l in range(8))   # halfSample levels (even sides at 640x480)
    ncells = -(-W // 5) * -(-H // 5)
    if name == "k_svo_pyramid":   # BGR read once, gray level 0 + levels 1..7 written
        return nframes * (W * H * 3 + svo_pyr)
    if name == "k_svo_detect":    # every level read once (cell atomics: one 8-B max per surviving corner, omitted)
        return nframes * svo_pyr
    if name == "k_svo_box":       # gray read, u16 box sums written
        return nframes * (W * H + 2 * W * H)
    if name == "k_svo_select":    # cell keys read + reset, KeyPoints written
        return nframes * (2 * ncells * 8 + n_kp * 28)
    if name == "k_svo_brief":     # KeyPoint read, 512 u16 box samples, descriptor written
        return nframes * n_kp * (28 + 512 * 2 + 32)
    if name == "k_pnp_refine":    # points read for the mask + 10 Gauss-Newton passes over the inliers
        return nframes * n_match * 20 * 11
    return 0


def hyp_per_launch(timings, B):
    """k_pnp_hyp launches carry every pair's current chunk; mean hypotheses per launch is reported by the
    library only through launches, so use the first-chunk size (32 per pair) as the per-launch count."""
    return 32 * (B - 1)


def pingpong(g, U):
    """Global frame index -> rendered frame index: 0 .. U-1, U-2 .. 0, 1 .. (period 2U - 2)."""
    r = np.asarray(g) % (2 * U - 2)
    return np.where(r < U, r, 2 * U - 2 - r)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024,
                    help="frames per rank per step (64 .. 1024 measured; 1024 best, 512 within 2 %%)")
    ap.add_argument("--unique", type=int, default=64,
                    help="distinct rendered frames; larger batches walk them back and forth (see pingpong)")
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--preset", default="fr1")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true", help="no per-kernel HIP events in the timed region")
    ap.add_argument("--lanes", type=int, default=0,
                    help="0: auto (pnp 1, se3 16); pnp: contexts the pipelined steps are dealt to round-robin; se3: independent contiguous "
                         "chunks of the batch (1-frame halo, stitched like the multi-GPU shards) tracked "
                         "concurrently, one context and host thread each")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="pnp: synchronous rgbd_pnp_track_batch per step instead of submit / collect with two in flight")
    ap.add_argument("--extractor", choices=["orb", "svo"], default="orb",
                    help="orb: ORBextractor (the north star's extractor); svo: Extractor(SVO, BRIEF, NORMAL), "
                         "the reference's main.cpp default")
    ap.add_argument("--solver", choices=["pnp", "se3"], default="pnp",
                    help="pnp: extract+match+PnPRansac (the metric); se3: the reference tracker's RansacSE3 chain")
    args = ap.parse_args()
    if args.lanes <= 0:   # measured best: one pipelined context for pnp, 16 concurrent chunks for the se3 chain
        args.lanes = 16 if args.solver == "se3" else 1

    import torch
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from conftest import load_pkg
    import synth
    pkg = load_pkg()

    import rgbd_slam_amd.dist as D
    import ate as ATE
    B = args.batch
    n_global = world * B                       # one sequence, contiguous chunks + 1 halo frame (dist.py)
    lo, hi = D.shard_range(n_global, world, rank)
    nb = hi - lo
    # render at most --unique frames of the trajectory and walk them back and forth (0 .. U-1, U-2 .. 0, 1 ..)
    # to fill the batch: every consecutive pair is a real neighbouring-frame pair of the sequence, and every
    # batch slot is its own copy in HBM (no frame is shared between slots)
    U = max(2, min(args.unique, n_global))
    src = pingpong(np.arange(n_global), U)
    need = src[lo:hi]
    ub, ud, ut, cam = synth.sequence(int(need.max()) + 1, seed=1000, preset=args.preset)
    bgr, depth, gt = ub[need], ud[need], ut[need]
    del ub, ud
    gt_all = synth.trajectory(U, seed=1000)[src]
    d_bgr = torch.from_numpy(bgr).to(dev)
    d_dep = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16)).to(dev)
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    svo = pkg.svo_params(args.nfeatures) if args.extractor == "svo" else None
    ctx = pkg.Context(640, 480, max_batch=nb, orb=pkg.orb_params(args.nfeatures), cam=c,
                      device=torch.cuda.current_device(), svo=svo)
    # further contexts (their own streams and buffers) take every L-th pipelined step, so the
    # latency-bound phases of one step overlap the VALU-bound phases of another
    ctxs = [ctx] + [pkg.Context(640, 480, max_batch=nb, orb=pkg.orb_params(args.nfeatures), cam=c,
                                device=torch.cuda.current_device(), svo=svo) for _ in range(max(args.lanes, 1) - 1)]
    prm = pkg.ransac_params(200, 10, 3.0, 4)       # RansacSE3(200, 10, 3.0f, 4), System/Tracking.cpp:129
    pnp_prm = pkg.pnp_params(500, 3.0, 0.85, 10)   # solvePnPRansac(..., 500, 3.0f, 0.85), Solver/PnPRansac.cpp:39
    rng = pkg.rng(1234 + rank)
    sticky = pkg.Sticky()
    pose0 = gt[0].astype(np.float32) if rank == 0 else np.eye(4, dtype=np.float32)
    PAD = B + 1
    last = {}

    def finish(poses, status, ninl):
        if world > 1:   # PoseGraph hand-off (RCCL all-gather); a single rank already holds them all
            pad = np.zeros((PAD, 16), np.float32)
            pad[:nb] = poses.reshape(nb, 16)
            last["allp"] = D.gather_poses(torch.from_numpy(pad).to(dev), world)
        else:
            last["allp"] = poses.reshape(1, nb, 16)
        return status, ninl

    # se3 lanes: the RansacSE3 chain is sequential within a chunk (outlier flags, RNG, sticky covariance) and
    # one chain's launches fill only ~200 workgroups, so independent chunks run side by side
    se3_lanes = args.solver == "se3" and len(ctxs) > 1
    if se3_lanes:
        from concurrent.futures import ThreadPoolExecutor
        lane_rng = [pkg.rng(1234 + 64 * rank + l) for l in range(len(ctxs))]
        lane_st = [pkg.Sticky() for _ in ctxs]
        pool = ThreadPoolExecutor(len(ctxs))

    def step():
        if se3_lanes:   # ctypes drops the GIL, so the lanes' host replays run in parallel too
            poses, status, ninl = D.track_lanes(ctxs, d_bgr.data_ptr(), d_dep.data_ptr(), nb, 0.9, prm, lane_rng,
                                                lane_st, pose0, pool)
            return finish(poses, status, ninl)
        if args.solver == "pnp":
            poses, status, ninl, nm = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), nb, 0.9, pnp_prm,
                                                          pose0)
            last["nm"] = nm
        else:
            poses, status, ninl = ctx.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), nb, 0.9, prm, rng, sticky,
                                                  pose0)
        return finish(poses, status, ninl)

    # streaming form (pnp): steps i+1, i+2 are submitted before step i is collected, so the host work of a
    # step (RANSAC bookkeeping, pose chaining, Python) overlaps the device work of the next one
    pipelined = args.solver == "pnp" and not args.no_pipeline

    L = len(ctxs)
    depth_in_flight = 2 * L + 1   # <= 3 outstanding per context (rgbd_pnp_track_submit keeps up to three)

    def submit(j=0):
        ctxs[j % L].pnp_track_submit(d_bgr.data_ptr(), d_dep.data_ptr(), nb, 0.9, pnp_prm)

    def collect(j=0):
        poses, status, ninl, nm = ctxs[j % L].pnp_track_collect(pose0)
        last["nm"] = nm
        return finish(poses, status, ninl)

    # warmup with every kernel timed: the per-kernel breakdown, and the dominant kernel; the timed
    # region then records events only around that kernel's launches (an event pair per launch costs
    # a few us of stream time, so timing all ~10 kernels would slow the measured step by ~8%)
    # The pipelined form also warms up as a pipeline (its solve stream and second workspace are created
    # by the first submission), so at least 2 warmup steps: W-1 pipelined, then the serial timed one.
    nw = max(args.warmup, 2 if pipelined else 1)
    for i in range(nw):
        if i == nw - 1:   # the last warmup step (warm caches) is the one every kernel is timed in
            torch.cuda.synchronize()
            ctx.reset_timing()
            ctx.set_timing(True)
            step()
        elif pipelined:
            for j in range(3 * L):
                submit(j)
            for j in range(3 * L):
                collect(j)
        else:
            step()
    torch.cuda.synchronize()
    warm = ctx.timings()
    dominant = max(warm.items(), key=lambda kv: kv[1][0])[0] if warm else None
    ctx.reset_timing()
    ctx.set_timing(not args.no_kernel_timing)
    ctx.set_timing_filter(dominant)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tracked = 0
    inl = []
    if pipelined:   # depth_in_flight steps in flight, dealt to the contexts round-robin
        for j in range(min(depth_in_flight - 1, args.steps)):
            submit(j)
        for i in range(args.steps):
            if i + depth_in_flight - 1 < args.steps:
                submit(i + depth_in_flight - 1)
            status, ninl = collect(i)
            tracked += int(status.sum())
            inl.append(float(ninl[1:].mean()))
    else:
        for _ in range(args.steps):
            status, ninl = step()
            tracked += int(status.sum())
            inl.append(float(ninl[1:].mean()))
    for cx in ctxs:
        cx.synchronize()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_timing(False)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    timings = ctx.timings()
    ate_m = None
    if rank == 0:
        allp = last["allp"]
        allp = allp.cpu().numpy() if hasattr(allp, "cpu") else allp
        chunks = []
        for r in range(world):
            l2, h2 = D.shard_range(n_global, world, r)
            chunks.append(allp[r][:h2 - l2].reshape(-1, 4, 4))
        traj = D.stitch(chunks, gt_all[0])
        ate_m = ATE.ate_rmse(traj, gt_all)

    frames_total = n_global * args.steps
    value = frames_total / elapsed
    ms_per_step = elapsed * 1e3 / args.steps

    # ---- roofline of the dominant kernel (HIP events on the library stream around its launches in
    # the timed region; the breakdown of all kernels comes from the warmup steps)
    n_kp = ctx.kp_cap  # upper bound; replaced by the measured mean below
    f0 = ctx.batch_frame(0)
    n_kp = len(f0["kps"])
    pyr_bytes = sum(int(round(640 / 1.2 ** l)) * int(round(480 / 1.2 ** l)) for l in range(8))
    dom = max(timings.items(), key=lambda kv: kv[1][0]) if timings else ("none", (0.0, 0))
    name, (ms, launches) = dom
    avg_ms = ms / max(launches, 1)
    n_match = int(np.mean(last["nm"][1:])) if "nm" in last else 600
    per_launch_frames = {"k_gray": B, "k_pyramid": B, "k_fast": B, "k_distribute": B, "k_describe": B,
                         "k_knn2": B - 1, "k_ransac_hyp": 1, "k_match_gather": B - 1,
                         "k_pnp_refine": B - 1}.get(name, B)
    nbytes = kernel_bytes(name, per_launch_frames, n_kp, n_match, pyr_bytes, 640, 480)
    if name == "k_pnp_hyp":   # hypotheses per launch = launches' mean (all pairs' chunks)
        nbytes = n_match * 20 * hyp_per_launch(timings, B)
    bound = "hbm"
    achieved = nbytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    # measured HBM traffic of the same kernel from the committed rocprofv3 PMC passes (tools/profile.sh:
    # separate FETCH_SIZE and WRITE_SIZE passes, KB per dispatch), bytes per launch; raw counter values
    # (this kernel's loads are dword-wide, outside the guide's 16-B/lane FETCH_SIZE calibration)
    traffic = None
    valu = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if os.path.exists(pmc_path):
        pmc = json.load(open(pmc_path)).get(name, {})
        if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
            traffic = int((pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024)
        # the bound this path actually has: VALU issue.  SQ_INSTS_VALU (wave64 instructions per launch,
        # same PMC pass set) x 64 lanes / launch time vs 256 CUs x 4 SIMDs x 32 lanes/clk x 2.4 GHz
        if "SQ_INSTS_VALU" in pmc and avg_ms > 0:
            a_t = pmc["SQ_INSTS_VALU"] * 64 / (avg_ms * 1e-3) / 1e12
            valu = {"achieved": round(a_t, 3), "peak": VALU_PEAK_TOPS, "unit": "T lane-ops/s",
                    "frac": round(a_t / VALU_PEAK_TOPS, 4), "insts_per_launch": int(pmc["SQ_INSTS_VALU"]),
                    "source": "profiles/pmc_latest.json SQ_INSTS_VALU / HIP-event launch time"}
    roofline = {"bound": bound, "kernel": name, "achieved": round(achieved, 3), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 6), "traffic": traffic,
                "algorithmic_bytes": int(nbytes), "avg_launch_ms": round(avg_ms, 5), "launches": launches,
                "traffic_source": "profiles/pmc_latest.json (rocprofv3 FETCH_SIZE+WRITE_SIZE)" if traffic else None,
                "valu": valu}
    # extract stage as a whole (1,608,000 B/frame at 1000 kp)
    wsteps = 1
    ext_ms = sum(v[0] for k, v in warm.items() if k in ("k_gray", "k_pyramid", "k_fast", "k_distribute",
                                                        "k_describe", "k_undistort", "k_svo_pyramid",
                                                        "k_svo_detect", "k_svo_select", "k_svo_brief"))
    ext_per_frame = 921600 + 614400 + n_kp * (28 + 32 + 12)
    extract_stage = {"frames": B * wsteps, "kernel_ms": round(ext_ms, 3), "source": "last warmup step, all kernels timed",
                     "achieved_GBps": round(ext_per_frame * B * wsteps / (ext_ms * 1e-3) / 1e9, 2) if ext_ms else 0,
                     "frames_per_s_kernel_time": round(B * wsteps / (ext_ms * 1e-3), 1) if ext_ms else 0}

    # ---- CPU baseline: the oracle (scalar C++ restatement) on this host, bounded sample, rank 0, N = 1
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        import oracle_lib as O
        import chain_model
        p, oc = O.orb_params(args.nfeatures), O.camera(cam)
        sp = O.svo_params(args.nfeatures)
        t0 = time.perf_counter()
        nfr = 0
        frames = []
        while True:
            i = nfr % B
            frames.append(O.svo_frame(bgr[i], depth[i], sp, oc) if svo is not None else O.frame(bgr[i], depth[i], p, oc))
            nfr += 1
            if time.perf_counter() - t0 > args.cpu_seconds * 0.8 or nfr >= 4 * B:
                break
        t_ext = time.perf_counter() - t0
        t1 = time.perf_counter()
        k = min(len(frames), 64)   # a bounded chain sample
        if args.solver == "pnp":
            K4 = np.array([cam["fx"], cam["fy"], cam["cx"], cam["cy"]], np.float32)
            chain_model.pnp_track(O, frames[:k], pose0, K4)
            what = "match/PnPRansac"
        else:
            chain_model.track(O, frames[:k], pose0, 99)
            what = "match/RansacSE3"
        t_chain = time.perf_counter() - t1
        per_frame = t_ext / nfr + t_chain / k
        cpu = {"value": round(1.0 / per_frame, 3), "unit": "frames/s", "cores": 1, "kind": "port",
               "sample": f"{nfr} frames extracted + {k}-frame {what} chain, oracle (scalar C++, 1 thread)"}

    if rank == 0:
        out = {
            "metric": "RGB-D frames/sec (extract+match+PnP) at 640×480, 1/2/4/8 GPUs; ATE vs ref",
            "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": nw, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8/i32 (fp32+fp64 solver)",
            "data": (f"synthetic (tools/synth.py, seeded TUM-{args.preset}-like RGB-D, 640x480; {U} rendered frames "
                     "walked back and forth to fill the batch, each slot its own HBM copy)"),
            "config": {"workload": (f"TUM {args.preset}/desk-like, "
                                    + ("ORB" if svo is None else "SVO+BRIEF") + f" {args.nfeatures} kp + Hamming BF knn-2 + "
                                    + ("PnPRansac (500 it, 3 px, 0.85) per consecutive pair" if args.solver == "pnp"
                                       else "RansacSE3 tracking chain (reference Tracking::visualOdometry)")),
                       "solver": args.solver, "extractor": args.extractor,
                       "host_overlap": (f"submit/collect, {depth_in_flight} steps in flight over {L} context(s); solves launched "
                                        "after the context's next quadtree" if pipelined else
                                        (f"{L} independent chunks (1-frame halo) tracked concurrently" if se3_lanes
                                         else "synchronous steps")),
                       "batch_frames_per_rank": B, "nfeatures": args.nfeatures, "preset": args.preset,
                       "parallelism": f"one sequence, contiguous chunk (+1 halo frame) per GPU x{world}, "
                                      "RCCL all-gather of poses"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "extract_stage": extract_stage,
            "kernels_ms_warmup": {k: [round(v[0], 3), v[1]] for k, v in sorted(warm.items())},
            "ate_rmse_m": round(ate_m, 5) if ate_m is not None else None,
            "tracked_frac": round(tracked / (nb * args.steps), 4),
            "mean_inliers": round(float(np.mean(inl)), 1),
            "mean_matches": n_match,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""bench.py -- frames/s of the RGB-D tracking front end on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch of B synthetic 640x480 RGB-D frames that are
already resident in HBM: ORB extraction (gray, pyramid, FAST cells, quadtree, orientation, blur,
rBRIEF, undistort, unproject) -> Hamming knn-2 of consecutive frames -> Matcher filter fused with the
3D-2D gather -> PnPRansac (EPnP hypotheses, RANSAC replay, Gauss-Newton refinement) for every pair ->
poses; then the poses are all-gathered over RCCL (PoseGraph hand-off) when N > 1.  Each rank tracks
its own sequence chunk ("weak" scaling).  --solver se3 runs the reference tracker's RansacSE3 chain
(with second-reference retry) instead.

Matcher variant of the headline: every pair independent (Matcher::match with discardOutliers = false).
A second leg (flag_chain) times the reference's outlier-flag chain (discardOutliers = true on the flags
PnPRansac sets, Features/Matcher.cpp:125-128, Solver/PnPRansac.cpp:31,51) over --flag-segments
independent runs of pairs; --flag-segments-headline S makes it the headline.  flag_chain_one times ONE
unbroken flag chain over the batch (the reference's semantics exactly), and se3_chain_one the reference
tracker's RansacSE3 -> second reference -> GICP chain (Tracking::visualOdometry) as one chain.

Modes (BASELINE configs): --mode chunks (configs 2, 3, 5: one sequence in contiguous chunks per GPU,
stitched) or --mode sequences (config 4: one independent sequence per GPU); --posegraph runs the
host PoseGraph (device Matcher + RansacSE3 local edges, LM) on rank 0 over the gathered trajectory
after the timed region (config 5 hand-off); --preset fr1 / fr2 / fr3 / icl / corbs.

    python bench.py [--gpus N --steps K --warmup W --batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one rank per GPU)

--gpus N > 1 without WORLD_SIZE in the environment: this process spawns the N ranks itself (one child
process per GPU, RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, 127.0.0.1) before anything touches the
GPU, and exits with their status; rank 0's child prints the line.  Under torchrun (WORLD_SIZE set) a
WORLD_SIZE other than --gpus is refused (exit 2).  n_gpus is the process group's size.

Prints one JSON line (rank 0) with the roofline of the dominant kernel (HIP events on the
library stream over the timed region) and the CPU oracle timed on the host (cpu_baseline: one
thread, and one process per core of the box's CPU share), measured before the GPU is touched.
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


# kernels with a per-launch algorithmic byte model (kernel_bytes); the roofline is taken over these
HBM_KERNELS = ("k_gray", "k_pyramid", "k_pyr_tail", "k_fast", "k_distribute", "k_describe", "k_undistort", "k_knn2", "k_match_gather",
               "k_svo_pyramid", "k_svo_detect", "k_svo_select", "k_svo_brief")

PB_LEVELS = 1   # RGBD_PB_LEVELS (rgbd-slam_amd/csrc/rgbd_internal.h): levels blurred inside k_pyramid; k_fast blurs the rest
STRIP_LEVELS = 4   # RGBD_PYR_STRIP_LEVELS: levels computed by k_pyramid's strips; k_pyr_tail computes the rest


# what each kernels_hbm byte figure counts: "s8d" = SURVEY s8(d)'s per-frame I/O only;
# "intermediate" = also the pyramid / blurred-pyramid levels s8(d) excludes; "l2_rereads" = per-keypoint
# overlapping square and disk rows, mostly L2-served (measured FETCH_SIZE is below the figure)
KERNEL_BYTES_KIND = {"k_pyramid": "intermediate (BGR in + levels 0-3 and blur of level 0 out)",
                     "k_pyr_tail": "intermediate (level 3 in + levels 4-7 out; their re-reads by the same workgroup not counted)",
                     "k_fast": "intermediate (pyramid in + blur of levels 1-7 out)",
                     "k_distribute": "selection only (n_kp x 8 B; the FAST candidate lists it reads are intermediates)",
                     "k_describe": "l2_rereads (37x37 square + IC disk rows per keypoint, overlapping)",
                     "k_undistort": "s8d (depth samples in, KeyPoints + xyz out)",
                     "k_knn2": "s8d (2 N 32 descriptors in + knn rows out)",
                     "k_match_gather": "s8d (knn rows in, matches + 3D-2D pairs out)"}


def kernel_bytes(name, nframes, n_kp, n_match, pyr_bytes, W, H, fused_blur=False):
    """Algorithmic HBM bytes of one launch (DESIGN.md 'Roofline accounting')."""
    lv = [int(round(W / 1.2 ** l)) * int(round(H / 1.2 ** l)) for l in range(8)]
    if name == "k_gray":
        return nframes * (W * H * 3 + W * H)
    if name == "k_pyramid":       # BGR read once, gray level 0 + levels 1..STRIP-1 written, blurred levels 0..PB-1 written
        return nframes * (W * H * 3 + sum(lv[:STRIP_LEVELS]) + sum(lv[:PB_LEVELS]))
    if name == "k_pyr_tail":      # level STRIP-1 read once, levels STRIP..7 written
        return nframes * (lv[STRIP_LEVELS - 1] + sum(lv[STRIP_LEVELS:]))
    if name == "k_fast":          # pyramid read once (the fused blur of levels PB..7 reads those rows again from
        # the same launch: not counted twice) + the blurred levels PB..7 written
        return nframes * (pyr_bytes + (sum(lv[PB_LEVELS:]) if fused_blur else 0))
    if name == "k_describe":      # 31-row IC disk (9 dwords) + 37-row blurred square (11 dwords) + KeyPoint, desc
        return nframes * n_kp * (31 * 36 + 37 * 44 + 28 + 32)
    if name == "k_undistort":     # KeyPoint read, depth sample, KeyPoint (undistorted) + xyz written
        return nframes * n_kp * (28 + 2 + 28 + 12)
    if name == "k_knn2":
        return nframes * (2 * n_kp * 32 + n_kp * 16)
    if name == "k_distribute":
        return nframes * n_kp * 8
    if name == "k_match_gather":  # knn rows + depth of both frames + kept pairs' xyz/pixel gathers and writes
        return nframes * (n_kp * 16 + 2 * n_kp * 4 + n_match * (12 + 8) * 2)
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
    return 0


def pingpong(g, U):
    """Global frame index -> rendered frame index: 0 .. U-1, U-2 .. 0, 1 .. (period 2U - 2)."""
    r = np.asarray(g) % (2 * U - 2)
    return np.where(r < U, r, 2 * U - 2 - r)



_CPU = {}   # inputs of the CPU legs (set before the pool forks; workers read them)


def _cpu_leg(k):
    """Oracle (scalar C++ restatement, built for timing) on rendered frames from offset k: extraction for a
    time budget, then a consecutive-frame match + solve chain -- both inside C++ (oracle/orc_bench.cpp), no
    per-call Python.  Returns (frames extracted, s, chain frames, s, match s, solve s)."""
    import oracle_lib as O
    d = _CPU
    oc = O.camera(d["cam"])
    r = O.bench_run(d["lib"], d["bgr"], d["depth"], oc, orb=None if d["svo"] else O.orb_params(d["nf"]),
                    svo=O.svo_params(d["nf"]) if d["svo"] else None, solver=0 if d["solver"] == "pnp" else 1,
                    start=k, seconds=d["sec"], chain=d["chain"])
    return r.frames_extracted, r.t_extract, r.chain_frames, r.t_chain, r.t_match, r.t_solve


_NATIVE = {}


def native_bench_lib():
    """The oracle built for this host once (-O3 -march=native -ffp-contract=off, ~6 s), or the
    portable prebuilt -O3 build if no compiler is usable here: (path, flags)."""
    import tempfile
    import oracle_lib as O
    if "lib" not in _NATIVE:
        lib, flags = O.build_native_bench(tempfile.mkdtemp(prefix="rgbd_cpu_"))
        if lib is None:
            lib, flags = O.BENCH_LIB_PATH, O.BENCH_FLAGS_PREBUILT
        _NATIVE.update(lib=lib, flags=flags)
    return _NATIVE["lib"], _NATIVE["flags"]


def cpu_chain_single(bgr, depth, cam, nfeatures, seconds):
    """The oracle's extraction + RansacSE3 tracking chain (Tracking::visualOdometry restated, C++,
    oracle/orc_bench.cpp) on one host thread: frames/s of extract + chain over a bounded sample."""
    import oracle_lib as O
    lib, flags = native_bench_lib()
    r = O.bench_run(lib, bgr, depth, O.camera(cam), orb=O.orb_params(nfeatures), solver=1, start=0,
                    seconds=seconds, chain=min(16, len(bgr)))
    rate = 1.0 / (r.t_extract / r.frames_extracted + r.t_chain / max(r.chain_frames - 1, 1))
    return {"value": round(rate, 3), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": (f"{r.frames_extracted} frames extracted + a {r.chain_frames}-frame RansacSE3 chain (second "
                       f"reference, GICP), one thread, oracle built with g++ {flags}")}


def cpu_baseline(bgr, depth, cam, args):
    """cpu_baseline: the oracle on this host's cores, before the GPU is initialised (the all-cores leg
    forks one process per core of the CPU share: independent sequences = different start offsets)."""
    import multiprocessing as mp
    # the oracle at -O3 -march=native -ffp-contract=off, compiled on this host (~6 s); the
    # portable prebuilt -O3 build if no compiler is usable here
    lib, flags = native_bench_lib()
    _CPU.update(bgr=bgr, depth=depth, cam=cam, nf=args.nfeatures, svo=args.extractor == "svo", solver=args.solver,
                sec=args.cpu_seconds * 0.8, chain=min(16, len(bgr)), lib=lib)

    def rate(r):
        nfr, te, kc, tc = r[:4]
        return 1.0 / (te / nfr + tc / max(kc - 1, 1))

    single = _cpu_leg(0)
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    # the GPU box's CPU share for one GPU is 16 cores (OMP_NUM_THREADS there); its affinity mask and
    # os.cpu_count() show the whole machine
    share = min(affinity, int(os.environ.get("OMP_NUM_THREADS", "16") or 16))
    P = max(1, min(share, 16))
    _CPU["sec"] = args.cpu_seconds * 0.6
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(P) as pool:
        res = pool.map(_cpu_leg, range(P))
    wall = time.perf_counter() - t0
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    what = "match/PnPRansac" if args.solver == "pnp" else "match/RansacSE3"
    tot = sum(rate(r) for r in res)
    return {"value": round(tot, 3), "unit": "frames/s", "cores": P, "kind": "port",
            "sample": (f"{P} processes (one per core of the CPU share), each {sum(r[0] for r in res) // P} frames "
                       f"extracted on average + a {res[0][2]}-frame {what} chain from its own start offset, all in "
                       f"C++ (oracle/orc_bench.cpp); oracle = scalar C++ restatement built with g++ {flags}; "
                       f"{wall:.1f} s wall"),
            "compiler_flags": flags,
            "single_thread": {"value": round(rate(single), 3), "cores": 1,
                              "sample": f"{single[0]} frames extracted + {single[2]}-frame {what} chain",
                              "ms_per_frame": {"extract": round(single[1] / single[0] * 1e3, 3),
                                               "match": round(single[4] / max(single[2] - 1, 1) * 1e3, 3),
                                               "solve": round(single[5] / max(single[2] - 1, 1) * 1e3, 3)}},
            "host": {"cpu_share": share, "affinity_cpus": affinity, "os_cpu_count": os.cpu_count(), "model": model}}


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n):
    """--gpus n without a launcher: n child processes of this script, rank i on GPU i (LOCAL_RANK i), before
    this process touches the GPU (it never does).  A failed rank ends the others (by their PIDs).  Returns
    the first non-zero exit status, else 0."""
    import subprocess
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # RCCL over dmabuf IPC on this image
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    code = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and code == 0:
                code = rc if rc > 0 else 1
                for q in live:   # the group cannot finish without this rank
                    q.terminate()
        time.sleep(0.05)
    return code


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); > 1 without torchrun: spawned here")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group of N > 1 (nccl = RCCL over xGMI; gloo: CPU pose gather, e.g. ranks sharing a card)")
    ap.add_argument("--steps", type=int, default=200)   # ~1.2 s timed at B = 1024
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024,
                    help="frames per rank per step (64 .. 1024 measured; 1024 best, 512 within 2 %%)")
    ap.add_argument("--unique", type=int, default=64,
                    help="distinct rendered frames; larger batches walk them back and forth (see pingpong)")
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--preset", default="fr1", choices=["fr1", "fr2", "fr3", "icl", "corbs"])
    ap.add_argument("--mode", choices=["chunks", "sequences"], default="chunks",
                    help="chunks: one sequence, a contiguous chunk (+1 halo frame) per GPU, stitched on rank 0; "
                         "sequences: an independent sequence per GPU (BASELINE config 4)")
    ap.add_argument("--posegraph", action="store_true",
                    help="after the timed region: host PoseGraph on rank 0 over the gathered trajectory (config 5)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true", help="no per-kernel HIP events in the timed region")
    ap.add_argument("--lanes", type=int, default=0,
                    help="0: auto (pnp 1, se3 64); pnp: contexts the pipelined steps are dealt to round-robin; se3: independent "
                         "contiguous chunks of the batch (1-frame halo, stitched like the multi-GPU shards) advanced "
                         "together on the device (rgbd_track_lanes)")
    ap.add_argument("--se3-priority", type=int, default=1,
                    help="se3 lanes with several contexts: extractions on one low-priority stream, each context's "
                         "lane rounds on its own high-priority stream")
    ap.add_argument("--se3-contexts", type=int, default=3,
                    help="se3 lanes: contexts (own streams and buffers) running consecutive steps from their own host "
                         "threads, so one step's extraction overlaps another's latency-bound lane rounds")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="pnp: synchronous rgbd_pnp_track_batch per step instead of submit / collect with two in flight")
    ap.add_argument("--extractor", choices=["orb", "svo"], default="orb",
                    help="orb: ORBextractor (the north star's extractor); svo: Extractor(SVO, BRIEF, NORMAL), "
                         "the reference's main.cpp default")
    ap.add_argument("--solver", choices=["pnp", "se3"], default="pnp",
                    help="pnp: extract+match+PnPRansac (the metric); se3: the reference tracker's RansacSE3 chain")
    ap.add_argument("--flag-segments-headline", type=int, default=0,
                    help="pnp: 0 = independent pairs (headline default); S >= 1 = the outlier-flag chain over S runs")
    ap.add_argument("--flag-segments", type=int, default=64,
                    help="pnp: runs of pairs of the flag_chain leg (1 = one chain over the batch)")
    ap.add_argument("--flag-chain-steps", type=int, default=5, help="pnp: timed steps of the flag_chain leg (0: skip)")
    ap.add_argument("--se3-chain-one-steps", type=int, default=1,
                    help="timed steps of the se3_chain_one leg: the reference tracker's RansacSE3 -> second reference "
                         "-> GICP chain (Tracking::visualOdometry) as ONE unbroken chain over the batch, one context, "
                         "one device lane (rgbd_track_batch; 0: skip)")
    ap.add_argument("--cfg3-chain-steps", type=int, default=1,
                    help="timed steps of the se3_chain_one_cfg3 leg: BASELINE config 3's workload (fr2, ORB 2000 kp, "
                         "RansacSE3 -> second reference -> GICP) as ONE unbroken chain over a batch (0: skip)")
    ap.add_argument("--flag-chain-one-steps", type=int, default=3,
                    help="pnp: timed steps of the flag_chain_one leg: ONE unbroken outlier-flag chain over the batch "
                         "(flag_segments = 1; 0: skip)")
    ap.add_argument("--lowtex-steps", type=int, default=3,
                    help="pnp: timed steps of the lowtex leg: the headline pipeline on low-texture frames (tools/synth.py "
                         "preset lowtex: the minThFAST = 7 fallback in nearly every cell; 0: skip)")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    if args.lanes <= 0:   # one pipelined context for pnp; 64 device lanes for the se3 chain
        args.lanes = 64 if args.solver == "se3" else 1

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import synth
    import ate as ATE
    from conftest import load_pkg
    pkg = load_pkg()             # the HIP library itself is loaded on first use (after the CPU legs)
    import rgbd_slam_amd.dist as D
    B = args.batch
    # chunks: one sequence, contiguous chunks + 1 halo frame; sequences: an independent sequence per rank
    n_global, lo, hi, seq_seed = D.workload(args.mode, B, world, rank)
    nb = hi - lo
    # render at most --unique frames of the trajectory and walk them back and forth (0 .. U-1, U-2 .. 0, 1 ..)
    # to fill the batch: every consecutive pair is a real neighbouring-frame pair of the sequence, and every
    # batch slot is its own copy in HBM (no frame is shared between slots)
    U = max(2, min(args.unique, n_global))
    src = pingpong(np.arange(n_global), U)
    need = src[lo:hi]
    n_render = int(src.max()) + 1 if (args.posegraph and rank == 0) else int(need.max()) + 1
    ub, ud, ut, cam = synth.sequence(n_render, seed=seq_seed, preset=args.preset)
    gt_all = synth.trajectory(U, seed=seq_seed)[src]
    pose0 = gt_all[lo].astype(np.float32) if (rank == 0 or args.mode == "sequences") else np.eye(4, dtype=np.float32)

    # config 3's single chain (fr2, 2000 kp): its own sequence, rendered here (CPU) like the headline's
    U3 = 16
    if args.cfg3_chain_steps > 0:
        src3 = pingpong(np.arange(B), U3)
        ub3, ud3, _, cam3 = synth.sequence(U3, seed=3000 + 7919 * rank, preset="fr2")

    # the low-texture leg's frames (fr1 camera, the headline context's): rendered here like the headline's
    do_lowtex = args.lowtex_steps > 0 and args.solver == "pnp" and args.extractor == "orb" and args.preset == "fr1"
    if do_lowtex:
        ubl, udl, _, _ = synth.sequence(min(U, 16), seed=seq_seed + 17, preset="lowtex")
        srcl = pingpong(np.arange(nb), min(U, 16))

    # ---- CPU baseline first: the oracle on the host cores, before anything initialises the GPU
    cpu = cpu3 = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(ub[:U], ud[:U], cam, args)
        if args.cfg3_chain_steps > 0:
            cpu3 = cpu_chain_single(ub3, ud3, cam3, 2000, min(args.cpu_seconds * 0.3, 4.0))

    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local % torch.cuda.device_count())   # gloo ranks may share a card
        dist.init_process_group(args.backend)
        assert dist.get_world_size() == args.gpus == world, (dist.get_world_size(), args.gpus, world)
    else:
        dist = None
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    coll_dev = dev if args.backend == "nccl" else torch.device("cpu")   # where the pose gather runs
    d_bgr = torch.from_numpy(ub[need]).to(dev)
    d_dep = torch.from_numpy(np.ascontiguousarray(ud[need]).view(np.int16)).to(dev)
    if not (args.posegraph and rank == 0):
        del ub, ud
    c = pkg.camera(cam["fx"], cam["fy"], cam["cx"], cam["cy"], cam["k1"], cam["k2"], cam["p1"], cam["p2"],
                   cam["k3"], cam["factor"])
    svo = pkg.svo_params(args.nfeatures) if args.extractor == "svo" else None
    ctx = pkg.Context(640, 480, max_batch=nb, orb=pkg.orb_params(args.nfeatures), cam=c,
                      device=torch.cuda.current_device(), svo=svo)
    # further contexts (their own streams and buffers) take every L-th pipelined step, so the
    # latency-bound phases of one step overlap the VALU-bound phases of another
    n_ctx = (max(args.se3_contexts, 1) if args.lanes > 1 else 1) if args.solver == "se3" else max(args.lanes, 1)
    ctxs = [ctx] + [pkg.Context(640, 480, max_batch=nb, orb=pkg.orb_params(args.nfeatures), cam=c,
                                device=torch.cuda.current_device(), svo=svo) for _ in range(n_ctx - 1)]
    prm = pkg.ransac_params(200, 10, 3.0, 4)       # RansacSE3(200, 10, 3.0f, 4), System/Tracking.cpp:129
    # solvePnPRansac(..., 500, 3.0f, 0.85), Solver/PnPRansac.cpp:39
    pnp_prm = pkg.pnp_params(500, 3.0, 0.85, 10, flag_segments=args.flag_segments_headline)
    rng = pkg.rng(1234 + rank)
    sticky = pkg.Sticky()
    PAD = B + 1
    last = {}
    if world > 1:   # the hand-off buffers: a pinned host block, its device copy, the gathered blocks
        pad_h = torch.zeros((PAD, 16), dtype=torch.float32, pin_memory=coll_dev.type == "cuda")
        pad_d = torch.zeros((PAD, 16), dtype=torch.float32, device=coll_dev)
        gathered = torch.empty((world, PAD, 16), dtype=torch.float32, device=coll_dev)

    def finish(poses, status, ninl):
        # every rank keeps its chunk's poses; the PoseGraph hand-off gathers them once, after the timed region
        # (north_star: "RCCL all-gather of poses ... only for the final PoseGraph hand-off")
        last["poses"] = poses.reshape(nb, 16)
        return status, ninl

    def hand_off():
        """The PoseGraph hand-off: one RCCL all-gather of every rank's chunk poses (a single rank holds them)."""
        if world > 1:
            pad_h.numpy()[:nb] = last["poses"]
            pad_d.copy_(pad_h)
            last["allp"] = D.gather_poses(pad_d, world, out=gathered)
        else:
            last["allp"] = last["poses"].reshape(1, nb, 16)

    # se3 lanes: the RansacSE3 chain is sequential within a chunk (outlier flags, RNG, sticky covariance), so
    # the batch is split into independent chunks (lanes) that the device advances together, one pair per round
    se3_lanes = args.solver == "se3" and args.lanes > 1
    if se3_lanes:   # per context: its lanes' RNGs and sticky covariances (independent chains)
        lane_rng = [[pkg.rng(1234 + 4096 * rank + 64 * 4096 * k + l) for l in range(args.lanes)] for k in range(n_ctx)]
        lane_st = [[pkg.Sticky() for _ in range(args.lanes)] for k in range(n_ctx)]

    import threading
    ext_lock = threading.Lock()
    round_streams, ext_stream = [], None
    if se3_lanes and n_ctx > 1 and args.se3_priority:
        lo, hi = torch.cuda.Stream.priority_range()
        ext_stream = torch.cuda.Stream(priority=lo)
        round_streams = [torch.cuda.Stream(priority=hi) for _ in range(n_ctx)]

    def step(k=0, split=False):
        if se3_lanes:
            if split:   # the contexts' extractions one at a time, each beside another context's lane rounds
                with ext_lock:
                    if round_streams:
                        ctxs[k].set_stream(ext_stream.cuda_stream)
                    ctxs[k].extract_batch(d_bgr.data_ptr(), d_dep.data_ptr(), nb)
                    ctxs[k].synchronize()
                if round_streams:   # the latency-bound rounds ahead of the extraction's waves
                    ctxs[k].set_stream(round_streams[k].cuda_stream)
                poses, status, ninl, _ = ctxs[k].track_lanes(0, 0, nb, 0.9, prm, args.lanes, lane_rng[k], lane_st[k],
                                                             pose0)
            else:
                poses, status, ninl, _ = ctxs[k].track_lanes(d_bgr.data_ptr(), d_dep.data_ptr(), nb, 0.9, prm,
                                                             args.lanes, lane_rng[k], lane_st[k], pose0)
            return finish(poses.reshape(nb, 16), status, ninl)
        if args.solver == "pnp":
            poses, status, ninl, nm = ctx.pnp_track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), nb, 0.9, pnp_prm,
                                                          pose0)
            last["nm"] = nm
        else:
            poses, status, ninl = ctx.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), nb, 0.9, prm, rng, sticky,
                                                  pose0)
        return finish(poses, status, ninl)

    # streaming form (pnp): steps i+1, i+2 are submitted before step i is collected, so the host work of a
    # step (RANSAC bookkeeping, pose chaining, Python) overlaps the device work of the next one.  The
    # flag chain keeps an output set until its collect: two in flight per context.
    pipelined = args.solver == "pnp" and not args.no_pipeline

    L = len(ctxs)

    def run_pipelined(steps, prm_used, per_ctx, frames=None):
        fb, fd = frames if frames is not None else (d_bgr.data_ptr(), d_dep.data_ptr())
        depth_in_flight = per_ctx * L - (L - 1) if per_ctx == 3 else per_ctx * L
        stamps = []
        t_start = time.perf_counter()
        for j in range(min(depth_in_flight - 1, steps)):
            ctxs[j % L].pnp_track_submit(fb, fd, nb, 0.9, prm_used)
        tracked, inl = 0, []
        for i in range(steps):
            if i + depth_in_flight - 1 < steps:
                j = i + depth_in_flight - 1
                ctxs[j % L].pnp_track_submit(fb, fd, nb, 0.9, prm_used)
            poses, status, ninl, nm = ctxs[i % L].pnp_track_collect(pose0)
            last["nm"] = nm
            finish(poses, status, ninl)
            tracked += int(status.sum())
            inl.append(float(ninl[1:].mean()))
            stamps.append(time.perf_counter())
        return tracked, inl, [b - a for a, b in zip([t_start] + stamps[:-1], stamps)], depth_in_flight

    per_ctx_depth = 2 if args.flag_segments_headline > 0 else 3
    # warmup with every kernel timed: the per-kernel breakdown, and the dominant kernel; the timed
    # region then records events only around that kernel's launches (an event pair per launch costs
    # a few us of stream time, so timing all ~10 kernels would slow the measured step by ~8%)
    # The pipelined form also warms up as a pipeline (its solve stream and second workspace are created
    # by the first submission), so at least 2 warmup steps: W-1 pipelined, then the serial timed one.
    nw = max(args.warmup, 2 if pipelined else 1)
    threaded = se3_lanes and L > 1   # se3: the contexts run their steps from their own host threads

    def run_threaded(steps):
        """Steps dealt round-robin to the contexts, each context's share run in order by its own thread (the
        library calls release the GIL), so their device work overlaps."""
        import concurrent.futures as cf
        out = [None] * steps

        def worker(k):
            for i in range(k, steps, L):
                ts = time.perf_counter()
                status, ninl = step(k, split=True)
                out[i] = (int(status.sum()), float(ninl[1:].mean()), time.perf_counter() - ts)
        with cf.ThreadPoolExecutor(max_workers=L) as ex:
            for f in [ex.submit(worker, k) for k in range(L)]:
                f.result()
        return out

    for i in range(nw):
        if i == nw - 1:   # the last warmup step (warm caches) is the one every kernel is timed in
            torch.cuda.synchronize()
            ctx.reset_timing()
            ctx.set_timing(True)
            step()
        elif pipelined:
            run_pipelined(per_ctx_depth * L, pnp_prm, per_ctx_depth)
        elif threaded:
            run_threaded(L)
        else:
            step()
    torch.cuda.synchronize()
    warm = ctx.timings()
    # the roofline kernel: the longest of the kernels whose per-launch algorithmic bytes are defined (the
    # extraction / matching kernels).  The solver kernels are per-pair dependent chains (latency-bound, bytes
    # mostly LDS-resident): the longest of all is reported beside it as time_dominant, without a roofline
    hbm_warm = {k: v for k, v in warm.items() if k in HBM_KERNELS}
    dominant = max(hbm_warm.items(), key=lambda kv: kv[1][0])[0] if hbm_warm else None
    time_dom = max(warm.items(), key=lambda kv: kv[1][0]) if warm else None
    ctx.reset_timing()
    ctx.set_timing(not args.no_kernel_timing)
    ctx.set_timing_filter(dominant)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    depth_in_flight = 1
    if pipelined:   # depth_in_flight steps in flight, dealt to the contexts round-robin
        tracked, inl, step_s, depth_in_flight = run_pipelined(args.steps, pnp_prm, per_ctx_depth)
    elif threaded:
        res = run_threaded(args.steps)
        tracked, inl, step_s = sum(r[0] for r in res), [r[1] for r in res], [r[2] / L for r in res]
        depth_in_flight = L
    else:
        tracked, inl, step_s = 0, [], []
        for _ in range(args.steps):
            ts = time.perf_counter()
            status, ninl = step()
            tracked += int(status.sum())
            inl.append(float(ninl[1:].mean()))
            step_s.append(time.perf_counter() - ts)
    for cx in ctxs:
        cx.synchronize()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.set_timing(False)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    timings = ctx.timings()
    t_h = time.perf_counter()
    hand_off()   # outside the timed region: the gather of the last step's poses for the PoseGraph
    hand_off_ms = (time.perf_counter() - t_h) * 1e3
    traj = None
    ate_m = None
    if rank == 0:
        allp = last["allp"]
        allp = allp.cpu().numpy() if hasattr(allp, "cpu") else allp
        # chunks: the stitched sequence; sequences: rank 0's own (every rank's poses were gathered)
        traj = D.trajectories(args.mode, allp, n_global, world, gt_all[0])[0]
        ate_m = ATE.ate_rmse(traj, gt_all)

    # ---- the reference's outlier-flag chain (discardOutliers = true), timed legs beside the headline
    def flag_leg(segments, steps):
        fprm = pkg.pnp_params(500, 3.0, 0.85, 10, flag_segments=segments)
        run_pipelined(min(2 * L, 2), fprm, 2)   # warm the flag workspaces
        for cx in ctxs:
            cx.synchronize()
        if dist is not None:
            dist.barrier()
        tf0 = time.perf_counter()
        ftr, finl, fsteps, _ = run_pipelined(steps, fprm, 2)
        for cx in ctxs:
            cx.synchronize()
        if dist is not None:
            dist.barrier()
        fel = time.perf_counter() - tf0
        if dist is not None:
            t = torch.tensor([fel], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            fel = float(t.item())
        return {"value": round(n_global * steps / fel, 2), "unit": "frames/s",
                "steps": steps, "ms_per_step": round(fel * 1e3 / steps, 3),
                "ms_per_step_median": round(float(np.median(fsteps)) * 1e3, 3),
                "segments_per_rank": segments, "pairs_per_segment": round((nb - 1) / segments, 1),
                "tracked_frac": round(ftr / (nb * steps), 4),
                "mean_inliers": round(float(np.mean(finl)), 1),
                "definition": "Matcher::match(discardOutliers=true) on PnPRansac's setOutlier/setInlier flags "
                              "(Features/Matcher.cpp:125-128, Solver/PnPRansac.cpp:31,51); exact chain within each "
                              "run of pairs, a run's first pair reads a fresh frame's flags; two steps in flight"}

    flag_chain = flag_chain_one = None
    if pipelined and args.flag_segments_headline == 0:
        if args.flag_chain_steps > 0 and args.flag_segments > 0:
            flag_chain = flag_leg(args.flag_segments, args.flag_chain_steps)
        if args.flag_chain_one_steps > 0:   # the reference's semantics exactly: one chain, every pair in order
            flag_chain_one = flag_leg(1, args.flag_chain_one_steps)

    # ---- the reference tracker's own chain as ONE unbroken chain (config 3's semantics exactly, beside the
    # headline's independent pairs or the se3 headline's L lanes): rgbd_track_batch = Tracking::visualOdometry
    # (System/Tracking.cpp:121-163) over the whole batch on one device lane, extraction included
    se3_chain_one = None
    if args.se3_chain_one_steps > 0:
        cx = ctxs[0]
        for k in ctxs:
            k.synchronize()
        r1, s1 = pkg.rng(4321 + rank), pkg.Sticky()
        cx.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), nb, 0.9, prm, r1, s1, pose0)   # warm (workspaces)
        cx.synchronize()
        if dist is not None:
            dist.barrier()
        ts0 = time.perf_counter()
        s_tr, s_in, s_st = 0, [], []
        for _ in range(args.se3_chain_one_steps):
            t1 = time.perf_counter()
            _, st1, ni1 = cx.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), nb, 0.9, prm, r1, s1, pose0)
            s_tr += int(st1.sum())
            s_in.append(float(ni1[1:].mean()))
            s_st.append(time.perf_counter() - t1)
        cx.synchronize()
        if dist is not None:
            dist.barrier()
        sel = time.perf_counter() - ts0
        if dist is not None:
            t = torch.tensor([sel], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            sel = float(t.item())
        se3_chain_one = {"value": round(n_global * args.se3_chain_one_steps / sel, 2), "unit": "frames/s",
                         "steps": args.se3_chain_one_steps,
                         "ms_per_step": round(sel * 1e3 / args.se3_chain_one_steps, 3),
                         "us_per_pair": round(sel * 1e6 / (args.se3_chain_one_steps * max(nb - 1, 1)), 1),
                         "tracked_frac": round(s_tr / (nb * args.se3_chain_one_steps), 4),
                         "mean_inliers": round(float(np.mean(s_in)), 1),
                         "definition": "rgbd_track_batch: extraction + Tracking::visualOdometry (Matcher(0.9) with "
                                       "updateF2 outlier flags, RansacSE3(200, 10, 3, 4), the second-reference retry, "
                                       "GICP when rmse >= 0.8) as one unbroken chain per rank (one lane, one "
                                       "context; RNG and sticky covariance carried pair to pair)"}

    # ---- BASELINE config 3 as one chain: fr2, ORB 2000 kp, Tracking::visualOdometry (RansacSE3(200, 10, 3, 4),
    # second reference, GICP 0.07 m / 10 iterations) over a batch of B frames on one context and one lane
    se3_chain_one_cfg3 = None
    if args.cfg3_chain_steps > 0:
        c3 = pkg.camera(cam3["fx"], cam3["fy"], cam3["cx"], cam3["cy"], cam3["k1"], cam3["k2"], cam3["p1"], cam3["p2"],
                        cam3["k3"], cam3["factor"])
        cx3 = pkg.Context(640, 480, max_batch=B, orb=pkg.orb_params(2000), cam=c3, device=torch.cuda.current_device())
        d_bgr3 = torch.from_numpy(ub3[src3]).to(dev)
        d_dep3 = torch.from_numpy(np.ascontiguousarray(ud3[src3]).view(np.int16)).to(dev)
        gt3 = synth.trajectory(U3, seed=3000 + 7919 * rank)[src3]
        r3, s3 = pkg.rng(2024 + rank), pkg.Sticky()
        pose3 = gt3[0].astype(np.float32)
        cx3.track_batch(d_bgr3.data_ptr(), d_dep3.data_ptr(), B, 0.9, prm, r3, s3, pose3)   # warm (workspaces)
        cx3.synchronize()
        if dist is not None:
            dist.barrier()
        t3 = time.perf_counter()
        tr3, in3 = 0, []
        for _ in range(args.cfg3_chain_steps):
            p3_, st3, ni3 = cx3.track_batch(d_bgr3.data_ptr(), d_dep3.data_ptr(), B, 0.9, prm, r3, s3, pose3)
            tr3 += int(st3.sum())
            in3.append(float(ni3[1:].mean()))
        cx3.synchronize()
        if dist is not None:
            dist.barrier()
        el3 = time.perf_counter() - t3
        if dist is not None:
            t = torch.tensor([el3], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el3 = float(t.item())
        se3_chain_one_cfg3 = {"value": round(world * B * args.cfg3_chain_steps / el3, 2), "unit": "frames/s",
                              "steps": args.cfg3_chain_steps, "frames_per_rank": B,
                              "ms_per_step": round(el3 * 1e3 / args.cfg3_chain_steps, 3),
                              "us_per_pair": round(el3 * 1e6 / (args.cfg3_chain_steps * (B - 1)), 1),
                              "tracked_frac": round(tr3 / (B * args.cfg3_chain_steps), 4),
                              "mean_inliers": round(float(np.mean(in3)), 1),
                              "ate_rmse_m": round(ATE.ate_rmse(p3_.reshape(-1, 4, 4), gt3), 5),
                              "cpu_baseline": cpu3,
                              "definition": "BASELINE config 3 (TUM fr2/desk-like synthetic, ORB 2000 kp + GICP): "
                                            "rgbd_track_batch = extraction + Tracking::visualOdometry as ONE unbroken "
                                            "chain over the batch per rank (one context, one device lane; outlier flags, "
                                            "RNG and sticky covariance carried pair to pair)"}
        cx3.close()
        del d_bgr3, d_dep3

    # ---- config 5 hand-off: the host PoseGraph over the gathered trajectory, rank 0, after the timing
    posegraph = None
    if args.posegraph and rank == 0:
        from rgbd_slam_amd.posegraph import posegraph_sequence
        tp = time.perf_counter()
        corr, kfs, (v, e, c0, c1) = posegraph_sequence(pkg, lambda k: (ub[src[k]], ud[src[k]]), cam, traj,
                                                       nfeatures=args.nfeatures, device=torch.cuda.current_device())
        posegraph = {"keyframes": len(kfs), "vertices": v, "edges": e, "chi2_before": round(c0, 6),
                     "chi2_after": round(c1, 6), "ms": round((time.perf_counter() - tp) * 1e3, 1),
                     "ate_rmse_m_after": round(ATE.ate_rmse(corr, gt_all), 5),
                     "definition": "PoseGraph::updateGraph without loop edges (keyframes by Tracking::needKeyFrame, "
                                   "device Matcher + RansacSE3 local edges, host LM optimize(10)); rank 0 after the "
                                   "RCCL all-gather"}

    frames_total = (n_global if args.mode == "chunks" else world * B) * args.steps
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
    per_launch_frames = {"k_gray": B, "k_pyramid": B, "k_pyr_tail": B, "k_fast": B, "k_distribute": B, "k_describe": B,
                         "k_knn2": B - 1, "k_match_gather": B - 1}.get(name, B)
    # the level blur of levels 1-7 (RGBD_PB_LEVELS = 1 onwards) runs inside the k_fast launch (blur_thread blocks of its grid)
    fused_blur = name == "k_fast"
    nbytes = kernel_bytes(name, per_launch_frames, n_kp, n_match, pyr_bytes, 640, 480, fused_blur)
    bound = "hbm"
    achieved = nbytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    # measured HBM traffic of the same kernel from the committed rocprofv3 PMC passes (tools/profile.sh
    # with SERIAL=1: the library runs single-stream, so a dispatch's device-wide TCC counters are its own;
    # separate FETCH_SIZE and WRITE_SIZE passes, KB per dispatch), bytes per launch.  gfx950 FETCH_SIZE
    # counts half the bytes of 16-B-per-lane streaming reads (MI355X_MICROARCH.md, HBM section): kernels
    # whose global reads are 16-B/lane get the factor 2, the others (dword loads) are taken as counted.
    FETCH_16B = {"k_fast": 2.0, "k_pyramid": 2.0}
    traffic = None
    valu = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if os.path.exists(pmc_path):
        pmc = json.load(open(pmc_path)).get(name, {})
        if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
            traffic = int((FETCH_16B.get(name, 1.0) * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024)
        # the bound this path actually has: VALU issue.  SQ_INSTS_VALU (wave64 instructions per launch, same
        # PMC pass set) priced three ways against the chip's issue capacity (1024 SIMDs x 2.4 GHz cycles):
        #   at_2cyc   every instruction at the 2-cycle best case (78.6 T lane-ops/s);
        #   priced    at the measured per-class issue costs (profiles/r02_ubench/valu_rate.txt) weighted by the
        #             kernel's static VALU mix (tools/valu_mix.py -> profiles/valu_mix.json);
        #   busy      SQ_ACTIVE_INST_VALU x 4 (quad-cycles -> cycles) / SIMD-cycles: the measured VALU busy.
        if "SQ_INSTS_VALU" in pmc and avg_ms > 0:
            ninst = pmc["SQ_INSTS_VALU"]
            simd_cycles = 1024 * 2.4e9 * avg_ms * 1e-3
            a_t = ninst * 64 / (avg_ms * 1e-3) / 1e12
            valu = {"achieved": round(a_t, 3), "peak": VALU_PEAK_TOPS, "unit": "T lane-ops/s",
                    "frac": round(a_t / VALU_PEAK_TOPS, 4), "insts_per_launch": int(ninst),
                    "frac_at_2cyc": round(ninst * 2.0 / simd_cycles, 4),
                    "source": "profiles/pmc_latest.json SQ_INSTS_VALU / HIP-event launch time"}
            mix_path = os.path.join(ROOT, "profiles", "valu_mix.json")
            if os.path.exists(mix_path):
                mix = json.load(open(mix_path)).get(name)
                if mix:
                    valu["cyc_per_inst_priced"] = mix["cycles_per_inst"]
                    valu["frac_priced"] = round(ninst * mix["cycles_per_inst"] / simd_cycles, 4)
                    valu["priced_source"] = "profiles/valu_mix.json (static VALU mix x valu_rate.txt)"
            if "SQ_ACTIVE_INST_VALU" in pmc:
                valu["busy_frac"] = round(pmc["SQ_ACTIVE_INST_VALU"] * 4 / simd_cycles, 4)
                valu["busy_cyc_per_inst"] = round(pmc["SQ_ACTIVE_INST_VALU"] * 4 / ninst, 3)
    roofline = {"bound": bound, "kernel": name, "achieved": round(achieved, 3), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 6), "traffic": traffic,
                "algorithmic_bytes": int(nbytes), "avg_launch_ms": round(avg_ms, 5), "launches": launches,
                "traffic_source": ("profiles/pmc_latest.json (rocprofv3 serial pass, %s x FETCH_SIZE + WRITE_SIZE)"
                                   % FETCH_16B.get(name, 1.0)) if traffic else None,
                "valu": valu, "fused_blur": fused_blur,
                "time_dominant": ({"kernel": time_dom[0], "ms_warmup_step": round(time_dom[1][0], 4),
                                   "launches": time_dom[1][1],
                                   "bound": ("HBM / VALU issue (the roofline kernel)" if time_dom[0] == name else
                                             "latency: dependent per-pair chains (no byte roofline)")}
                                  if time_dom else None)}
    # step level (SURVEY s8d algorithmic bytes per frame: extract BGR + depth in, KeyPoints + descriptors + xyz
    # out; match 2 N 32 + M 16; solve M (2 12 + 16)) over the measured step time: the whole path's HBM fraction
    step_bpf = (921600 + 614400 + n_kp * (28 + 32 + 12)) + (2 * n_kp * 32 + n_match * 16) + n_match * 40
    # the roofline's bound: VALU issue when the measured VALU busy share exceeds the HBM fraction
    if valu and valu.get("busy_frac", 0.0) > roofline["frac"]:
        roofline["bound"] = "valu"
    # the same kernel time priced with the s8d bytes per frame (the path's algorithmic bytes, not the kernel's own)
    if avg_ms > 0:
        g8 = step_bpf * per_launch_frames / (avg_ms * 1e-3) / 1e9
        roofline["s8d"] = {"bytes_per_frame": int(step_bpf), "achieved": round(g8, 3), "frac": round(g8 / HBM_PEAK_GBPS, 6),
                           "definition": "SURVEY s8d bytes per frame x frames per launch / the kernel's launch time"}
    step_gbps = step_bpf * (n_global if args.mode == "chunks" else world * B) / (ms_per_step * 1e-3) / 1e9
    roofline["step"] = {"bytes_per_frame": int(step_bpf), "achieved": round(step_gbps, 3), "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": round(step_gbps / HBM_PEAK_GBPS, 6),
                        "definition": "SURVEY s8d bytes per frame x frames per step / ms_per_step (all GPUs)"}
    # extract stage as a whole (1,608,000 B/frame at 1000 kp)
    wsteps = 1
    ext_ms = sum(v[0] for k, v in warm.items() if k in ("k_gray", "k_pyramid", "k_pyr_tail", "k_fast", "k_distribute",
                                                        "k_describe", "k_undistort", "k_svo_pyramid",
                                                        "k_svo_detect", "k_svo_select", "k_svo_brief"))
    ext_per_frame = 921600 + 614400 + n_kp * (28 + 32 + 12)
    extract_stage = {"frames": B * wsteps, "kernel_ms": round(ext_ms, 3), "source": "last warmup step, all kernels timed",
                     "achieved_GBps": round(ext_per_frame * B * wsteps / (ext_ms * 1e-3) / 1e9, 2) if ext_ms else 0,
                     "frames_per_s_kernel_time": round(B * wsteps / (ext_ms * 1e-3), 1) if ext_ms else 0}

    # every extraction kernel's HBM fraction from the last warmup step (synchronous, one event pair per
    # launch, so each kernel's time is its own): algorithmic bytes as above / its event time
    kernels_hbm = {}
    for k in ("k_pyramid", "k_pyr_tail", "k_fast", "k_distribute", "k_describe", "k_undistort", "k_knn2", "k_match_gather"):
        if k in warm and warm[k][0] > 0:
            kb = kernel_bytes(k, {"k_knn2": B - 1, "k_match_gather": B - 1}.get(k, B), n_kp, n_match, pyr_bytes,
                              640, 480, k == "k_fast")
            g = kb / (warm[k][0] * 1e-3) / 1e9
            kernels_hbm[k] = {"ms": warm[k][0], "algorithmic_bytes": int(kb), "GBps": round(g, 1),
                              "frac": round(g / HBM_PEAK_GBPS, 4), "bytes_kind": KERNEL_BYTES_KIND.get(k, "s8d")}

    # ---- the low-texture regime beside the headline: the same pipelined chain on frames where FAST at 20 finds
    # almost nothing and the per-cell minThFAST = 7 fallback decides (Features/ORBextractor.cpp:655-661)
    lowtex = None
    if do_lowtex and pipelined:
        d_lb = torch.from_numpy(ubl[srcl]).to(dev)
        d_ld = torch.from_numpy(np.ascontiguousarray(udl[srcl]).view(np.int16)).to(dev)
        fr_l = (d_lb.data_ptr(), d_ld.data_ptr())
        run_pipelined(per_ctx_depth * L, pnp_prm, per_ctx_depth, fr_l)   # warm (first touch of the frames)
        for cx in ctxs:
            cx.synchronize()
        ctx.reset_timing()
        ctx.set_timing(True)
        ctx.set_timing_filter("k_fast")
        if dist is not None:
            dist.barrier()
        tl0 = time.perf_counter()
        ltr, linl, _, _ = run_pipelined(args.lowtex_steps, pnp_prm, per_ctx_depth, fr_l)
        for cx in ctxs:
            cx.synchronize()
        if dist is not None:
            dist.barrier()
        lel = time.perf_counter() - tl0
        if dist is not None:
            t = torch.tensor([lel], dtype=torch.float64, device=coll_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            lel = float(t.item())
        kf_ms, kf_n = ctx.timings().get("k_fast", (0.0, 0))
        ctx.set_timing(False)
        nkp = [len(ctx.batch_frame(b)["kps"]) for b in (0, nb // 2, nb - 1)]
        lowtex = {"value": round(n_global * args.lowtex_steps / lel, 2), "unit": "frames/s",
                  "steps": args.lowtex_steps, "ms_per_step": round(lel * 1e3 / args.lowtex_steps, 3),
                  "k_fast_ms": round(kf_ms / max(kf_n, 1), 3), "tracked_frac": round(ltr / (nb * args.lowtex_steps), 4),
                  "mean_inliers": round(float(np.mean(linl)), 1), "keypoints_sampled": nkp,
                  "workload": ("tools/synth.py preset lowtex (fr1 camera): blocks 2x larger, intensities within 23 "
                               "levels, no fine pattern; > 90 % of level-0 cells take the minThFAST = 7 fallback "
                               "(tests/test_gpu_lowtex.py); same pipeline, batch and contexts as the headline")}
        del d_lb, d_ld

    if rank == 0:
        out = {
            "metric": "RGB-D frames/sec (extract+match+PnP) at 640×480, 1/2/4/8 GPUs; ATE vs ref",
            "value": round(value, 2), "unit": "frames/s", "n_gpus": dist.get_world_size() if dist is not None else 1, "steps": args.steps,
            "warmup": nw, "ms_per_step": round(ms_per_step, 3),
            "ms_per_step_median": round(float(np.median(step_s)) * 1e3, 3) if step_s else None,
            "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8/i32 (fp32+fp64 solver)",
            "data": (f"synthetic (tools/synth.py, seeded {args.preset}-camera RGB-D, 640x480; {U} rendered frames "
                     "walked back and forth to fill the batch, each slot its own HBM copy)"),
            "config": {"workload": (f"{args.preset} desk-like, "
                                    + ("ORB" if svo is None else "SVO+BRIEF") + f" {args.nfeatures} kp + Hamming BF knn-2 + "
                                    + ("PnPRansac (500 it, 3 px, 0.85) per consecutive pair" if args.solver == "pnp"
                                       else "RansacSE3 tracking chain (reference Tracking::visualOdometry)")),
                       "solver": args.solver, "extractor": args.extractor,
                       "host_overlap": (f"submit/collect, {depth_in_flight} steps in flight over {L} context(s); a step's PnPRansac "
                                        "solves launched right after the next step's k_fast (beside its quadtree and "
                                        "description)" if pipelined else
                                        (f"{args.lanes} independent chunks (1-frame halo) advanced together on the device "
                                         f"(rgbd_track_lanes); {L} context(s) run consecutive steps from their own host "
                                         "threads, their extractions one at a time (rgbd_extract_batch, then "
                                         "rgbd_track_lanes on it), each beside another context's lane rounds" if se3_lanes
                                         else "synchronous steps")),
                       "batch_frames_per_rank": B, "nfeatures": args.nfeatures, "preset": args.preset,
                       "matcher": (("Matcher(0.9) on RansacSE3's updateF2 outlier flags (Features/Matcher.cpp:125-128, "
                                    "Solver/SolverSE3.cpp:38-42,119-122), exact within each lane's chain, a lane's first "
                                    "frame with clear flags") if args.solver == "se3" else
                                   "discardOutliers=false: every pair independent" if args.flag_segments_headline == 0
                                   else f"discardOutliers=true: outlier-flag chain over {args.flag_segments_headline} runs"),
                       "mode": args.mode,
                       "parallelism": (f"one sequence, contiguous chunk (+1 halo frame) per GPU x{world}, no collective "
                                       "in the timed loop; one RCCL all-gather of poses after it (PoseGraph hand-off)"
                                       if args.mode == "chunks" else
                                       f"one independent sequence per GPU x{world}, no collective in the timed loop; one "
                                       "RCCL all-gather of poses after it (PoseGraph hand-off)")},
            "hand_off": {"collective": "all_gather_into_tensor" if world > 1 else None,
                         "backend": args.backend if world > 1 else None, "bytes_per_rank": (B + 1) * 64,
                         "ms": round(hand_off_ms, 3), "timed": False},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "flag_chain": flag_chain,
            "flag_chain_one": flag_chain_one,
            "se3_chain_one": se3_chain_one,
            "se3_chain_one_cfg3": se3_chain_one_cfg3,
            "lowtex": lowtex,
            "posegraph": posegraph,
            "extract_stage": extract_stage,
            "kernels_hbm": kernels_hbm,
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

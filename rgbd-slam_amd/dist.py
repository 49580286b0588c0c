"""Multi-GPU glue for the front end: one process per GPU, frames of one sequence sharded in
contiguous chunks, RCCL all-gather of poses for the (host) PoseGraph hand-off.

The data path has no collective: each rank extracts, matches and tracks its own chunk.  A chunk
k > 0 starts one frame early (a halo frame shared with chunk k-1) and is tracked from an identity
pose there, so rank 0 can stitch the gathered chunks exactly: Tcw_j = T(j <- halo) * Tcw_halo.
(SURVEY.md s8e "throughput mode"; config 5.)  Over gloo the same code runs on CPU for tests.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_frames: int, world: int, rank: int):
    """Contiguous chunk [lo, hi) of the global frame range for `rank`; lo includes the halo frame."""
    base = n_frames // world
    rem = n_frames % world
    starts = [r * base + min(r, rem) for r in range(world + 1)]
    lo, hi = starts[rank], starts[rank + 1]
    return (lo - 1 if rank > 0 else lo), hi


def workload(mode: str, batch: int, world: int, rank: int):
    """The frames a rank tracks per step (bench.py; BASELINE configs 2-5).  Returns (n_global, lo, hi, seed):
      chunks     one sequence of world x batch frames per step, rank r tracking the contiguous chunk [lo, hi)
                 (with the halo frame of shard_range) -- configs 2, 3, 5;
      sequences  an independent sequence of `batch` frames per rank, seeded by its rank (config 4: one
                 ICL-NUIM sequence per GPU).
    No frame crosses ranks in either mode: the data path has no collective."""
    if mode == "chunks":
        n_global = world * batch
        lo, hi = shard_range(n_global, world, rank)
        return n_global, lo, hi, 1000
    if mode == "sequences":
        return batch, 0, batch, 1000 + 7919 * rank
    raise ValueError(f"unknown mode {mode!r}")


def trajectories(mode: str, allp, n_global: int, world: int, pose0: np.ndarray):
    """Rank 0 after the pose all-gather (allp: (world, >= n, 16)): chunks -> [the stitched global trajectory];
    sequences -> every rank's own trajectory (each tracked from its own first pose), in rank order."""
    allp = np.asarray(allp, np.float32)
    if mode == "chunks":
        chunks = []
        for r in range(world):
            lo, hi = shard_range(n_global, world, r)
            chunks.append(allp[r][:hi - lo].reshape(-1, 4, 4))
        return [stitch(chunks, pose0)]
    return [allp[r][:n_global].reshape(-1, 4, 4) for r in range(world)]


def gather_poses(local, world: int, force_collective: bool = False, out=None):
    """All-gather each rank's (n, 16) float32 pose block (n equal on every rank); returns (world, n, 16).
    At world 1 the block is returned as is unless force_collective (the RCCL call site's own GPU test).
    `out` ((world, n, 16), local's device) is reused when given (the bench gathers every step)."""
    import torch
    import torch.distributed as dist
    if world == 1 and not force_collective:
        return local.unsqueeze(0)
    if out is None:
        out = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, local.contiguous())     # RCCL over xGMI
    else:
        parts = list(out.unbind(0))   # gloo (CPU tests): views of out
        dist.all_gather(parts, local.contiguous())
    return out


def stitch(chunks, pose0: np.ndarray) -> np.ndarray:
    """chunks[k]: (n_k, 4, 4) poses tracked from an identity pose at the chunk's first frame
    (k == 0: from pose0 directly).  Returns the global Tcw trajectory (halo frames dropped)."""
    out = [np.asarray(chunks[0], np.float64)]
    for k in range(1, len(chunks)):
        halo = out[-1][-1]                               # Tcw of the shared frame
        loc = np.asarray(chunks[k], np.float64)
        out.append(np.einsum("nij,jk->nik", loc[1:], halo))
    return np.concatenate(out).astype(np.float32)

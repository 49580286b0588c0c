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


def gather_poses(local, world: int):
    """All-gather each rank's (n, 16) float32 pose block (n equal on every rank); returns (world, n, 16)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return local.unsqueeze(0)
    out = torch.empty((world,) + tuple(local.shape), dtype=local.dtype, device=local.device)
    if dist.get_backend() == "nccl":
        dist.all_gather_into_tensor(out, local.contiguous())     # RCCL over xGMI
    else:
        parts = [torch.empty_like(local) for _ in range(world)]
        dist.all_gather(parts, local.contiguous())
        out = torch.stack(parts)
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


def track_lanes(ctxs, d_bgr: int, d_depth: int, n: int, nnratio, prm, rngs, stickies, pose0, pool=None,
                W: int = 640, H: int = 480):
    """The RansacSE3 tracking chain (rgbd_track_batch) over n device-resident frames split into
    len(ctxs) contiguous lanes (1-frame halo, shard_range), tracked concurrently, one context, RNG and
    sticky covariance per lane (ctypes releases the GIL, so the lanes' host replays overlap), then
    stitched like the multi-GPU chunks.  Returns (poses [n,4,4], status [n], n_inliers [n])."""
    L = len(ctxs)
    spans = [shard_range(n, L, l) for l in range(L)]
    fb, fd = W * H * 3, W * H * 2

    def lane(l):
        a, z = spans[l]
        p0 = np.asarray(pose0, np.float32) if l == 0 else np.eye(4, dtype=np.float32)
        return ctxs[l].track_batch(d_bgr + a * fb, d_depth + a * fd, z - a, nnratio, prm, rngs[l], stickies[l], p0)

    res = list(pool.map(lane, range(L))) if pool is not None else [lane(l) for l in range(L)]
    poses = stitch([r[0] for r in res], pose0)
    status = np.concatenate([res[0][1]] + [r[1][1:] for r in res[1:]])
    ninl = np.concatenate([res[0][2]] + [r[2][1:] for r in res[1:]])
    return poses, status, ninl

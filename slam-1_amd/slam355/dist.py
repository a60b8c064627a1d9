"""Multi-GPU tracking and local BA.

Tracking shards by frame pairs (main.py:79-97 couples only frames i and i+1):
no collective in the loop; the global trajectory needs each pair's PnP result
only, gathered once (`gather_pose_chain`, 56 B per pair) and chained in frame
order with the stale-T rule of main.py:120-124.

Local BA: each rank owns a contiguous range of points ordered by their first
observing keyframe and all observations of those points; every rank keeps all
cameras.  Per LM iteration the ranks all-reduce the reduced camera system (RCCL
over xGMI with the "nccl" backend; gloo in the CPU tests) —
BAProblem.step_distributed.
"""
from __future__ import annotations

import numpy as np


def shard_by_anchor(n_cams, n_pts, cam_idx, pt_idx, rank, world):
    """-> (point mask [P] bool, observation mask [O] bool, local point index of
    every observation kept).  Points are sorted by anchor (first observing
    camera, then index) and cut into `world` contiguous ranges."""
    cam_idx = np.asarray(cam_idx, np.int64)
    pt_idx = np.asarray(pt_idx, np.int64)
    first = np.full(n_pts, n_cams, np.int64)
    np.minimum.at(first, pt_idx, cam_idx)
    order = np.lexsort((np.arange(n_pts), first))
    mine = np.zeros(n_pts, bool)
    mine[order[rank * n_pts // world:(rank + 1) * n_pts // world]] = True
    keep = mine[pt_idx]
    remap = -np.ones(n_pts, np.int64)
    remap[mine] = np.arange(int(mine.sum()))
    return mine, keep, remap[pt_idx[keep]]


def gather_pose_chain(rvec, tvec, ninl, pose0=None, T0=None, group=None):
    """The global trajectory of frame-pair shards: rank r tracked pairs
    r*B .. r*B + B - 1 (equal B on every rank) and holds their PnP results
    rvec, tvec [B, 3] f64 and n_inliers [B] (-1 = fewer than 5 points, the
    stale-T case).  All ranks all-gather the 7 numbers per pair and chain them
    in frame order from pose0 with the previous-T rule of main.py:94-98,
    120-124 (a shard's first stale pair reuses the last T of the shard before
    it).  CUDA tensors are chained on the device by the same k_pose_chain the
    single-GPU Tracker uses (bit-identical to one Tracker over all pairs); CPU
    tensors (gloo tests) by pipeline.chain_poses.  Returns the absolute poses
    [world * B, 4, 4] f64 of frames 1 .. world * B on every rank."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    B = rvec.shape[0]
    buf = torch.cat([rvec.reshape(B, 3).double(), tvec.reshape(B, 3).double(),
                     ninl.reshape(B, 1).double()], 1).contiguous()
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    allb = torch.cat(parts)
    n = allb.shape[0]
    p0 = np.eye(4) if pose0 is None else np.asarray(pose0, float)
    t0 = np.eye(4) if T0 is None else np.asarray(T0, float)
    if allb.is_cuda:
        from . import _lib
        from .device import ptr, stream_ptr

        dev = allb.device
        rv = allb[:, 0:3].contiguous()
        tv = allb[:, 3:6].contiguous()
        ni = allb[:, 6].round().to(torch.int32).contiguous()
        state = torch.as_tensor(np.concatenate([p0, t0]).ravel(), dtype=torch.float64,
                                device=dev).contiguous()
        poses = torch.empty((n, 4, 4), dtype=torch.float64, device=dev)
        _lib.call("slam_pose_chain", ptr(rv), ptr(tv), ptr(ni), n, ptr(state), ptr(poses),
                  stream_ptr(None))
        return poses
    from .pipeline import chain_poses

    a = allb.numpy()
    poses, _ = chain_poses(p0, a[:, 0:3], a[:, 3:6], np.rint(a[:, 6]).astype(np.int64), t0)
    return torch.from_numpy(poses)

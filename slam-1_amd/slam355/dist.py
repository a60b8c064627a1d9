"""Multi-GPU local BA: landmark sharding by anchor keyframe.

Each rank owns a contiguous range of points ordered by their first observing
keyframe and all observations of those points; every rank keeps all cameras.
Per LM iteration the ranks all-reduce the reduced camera system (RCCL over
xGMI with the "nccl" backend; gloo in the CPU tests) — BAProblem.step_distributed.
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

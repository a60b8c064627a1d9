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


# Per-rank cost of a landmark shard's linearisation, assembly and back
# substitution (k_lin_mfma + k_assemble + k_back_trial), fitted to four C5
# W = 8 shards measured alone (scripts/shard_split.py; profiles/r6/split and
# profiles/r6/shard_balance: 150k / 150k / 93k / 158k observations in 1782 /
# 782 / 1486 / 824 camera-union supergroups, 139.7 / 97.6 / 112.6 / 99.7 us):
# 25.8 us + 0.25 ns per observation + 43 ns per supergroup, within 0.9 us --
# a supergroup costs as much as SHARD_SG_OBS observations.
SHARD_SG_OBS = 172.0


def point_costs(n_cams, n_pts, cam_idx, pt_idx, world):
    """Estimated cost of each point in a landmark shard, in observation units:
    its observations plus its share of the camera-union supergroup it falls in
    (ba.plan_mfma_native of the whole problem, chunks per workgroup as a shard of
    1 / world of it would use).  A loop-closure point whose cameras span the
    sequence's two ends shares its supergroup with few others (C5: 1947 such
    points make 1000 of 7251 supergroups).  Observation counts alone when the
    problem has no camera-union plan."""
    from .ba import plan_mfma_native

    cam_idx = np.asarray(cam_idx, np.int64)
    pt_idx = np.asarray(pt_idx, np.int64)
    w = np.bincount(pt_idx, minlength=n_pts).astype(np.float64)
    pl = plan_mfma_native(n_cams, n_pts, cam_idx, pt_idx, chunks_per_wg=shard_chunks_per_wg(len(cam_idx) // world))
    if pl is None:
        return w
    pt_of_chunk = pl["grp_ptr"].astype(np.int64)
    sg = pl["sg_ptr"].astype(np.int64)
    lo, hi = pt_of_chunk[sg[:-1]], pt_of_chunk[sg[1:]]  # supergroup -> new point range
    share = np.repeat(SHARD_SG_OBS / np.maximum(hi - lo, 1), hi - lo)
    w[pl["perm"][:len(share)].astype(np.int64)] += share
    return w


def shard_by_anchor(n_cams, n_pts, cam_idx, pt_idx, rank, world, balance=True):
    """-> (point mask [P] bool, observation mask [O] bool, local point index of
    every observation kept).  Points are sorted by anchor (first observing
    camera, then index) and cut into `world` contiguous ranges -- of equal
    estimated cost (point_costs) with `balance`, of equal point counts without.
    Every rank computes the same cuts (deterministic host code)."""
    cam_idx = np.asarray(cam_idx, np.int64)
    pt_idx = np.asarray(pt_idx, np.int64)
    first = np.full(n_pts, n_cams, np.int64)
    np.minimum.at(first, pt_idx, cam_idx)
    order = np.lexsort((np.arange(n_pts), first))
    if balance and world > 1:
        cw = np.cumsum(point_costs(n_cams, n_pts, cam_idx, pt_idx, world)[order])
        cuts = np.searchsorted(cw, cw[-1] * np.arange(1, world) / world, side="right")
        bounds = np.concatenate([[0], cuts, [n_pts]])
    else:
        bounds = np.arange(world + 1) * n_pts // world
    mine = np.zeros(n_pts, bool)
    mine[order[bounds[rank]:bounds[rank + 1]]] = True
    keep = mine[pt_idx]
    remap = -np.ones(n_pts, np.int64)
    remap[mine] = np.arange(int(mine.sum()))
    return mine, keep, remap[pt_idx[keep]]


def shard_chunks_per_wg(n_obs: int):
    """Linearisation chunks per workgroup for ONE rank's landmark shard of a
    window solved alone on its GPU (BAProblem chunks_per_wg): small shards want
    more, smaller workgroups than the planner's default (which is tuned for
    windows batched together).  Measured per-rank iteration at C4 / C5
    (scripts/shard_split.py, profiles/r5/shard_split/): W = 8 (313 chunks) 1 ->
    175 us vs 184 at the default 3; W = 4 / 2 (625 / 1250 chunks) 2 -> 192 /
    232 us vs 200 / 237; None (the planner's rule) from 4096 chunks up."""
    from .ba import MF_CHUNK_OBS

    n_chunks = -(-int(n_obs) // MF_CHUNK_OBS)
    if n_chunks < 512:
        return 1
    return 2 if n_chunks < 4096 else None


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


class GlobalChain:
    """The global trajectory of frame-pair shards, advanced every tracking step
    (main.py:120-124 over all ranks' pairs): rank r of `world` tracked pairs
    r*B .. r*B + B - 1 of the step's world*B consecutive pairs; the ranks
    all-gather each pair's PnP result (rvec, tvec, n_inliers: 7 doubles) and
    every rank chains the world*B results in frame order on the device
    (k_pose_chain, the stale-T rule across shard boundaries included),
    continuing a device-resident (pose, T) state from the previous step -- the
    trajectory one Tracker over all pairs gives, bit for bit.  Asynchronous on
    `stream` with the nccl (RCCL) backend; buffers are preallocated."""

    def __init__(self, B, world, device, group=None):
        import torch

        self.B, self.world, self.group = B, world, group
        f64 = dict(dtype=torch.float64, device=device)
        self.buf = torch.empty((B, 7), **f64)
        self.all = torch.empty((world * B, 7), **f64)
        self.parts = [self.all[i * B:(i + 1) * B] for i in range(world)]
        self.rv = torch.empty((world * B, 3), **f64)
        self.tv = torch.empty((world * B, 3), **f64)
        self.ni = torch.empty((world * B,), dtype=torch.int32, device=device)
        self.state = torch.empty((32,), **f64)
        self._eye = torch.as_tensor(np.concatenate([np.eye(4), np.eye(4)]).ravel(), **f64)
        self.poses = torch.empty((world * B, 4, 4), **f64)

    def reset(self, stream=None):
        """Restart the chain at the identity (an async device copy on `stream`)."""
        import torch

        with torch.cuda.stream(stream if stream is not None else torch.cuda.current_stream()):
            self.state.copy_(self._eye, non_blocking=True)

    def step(self, rvec, tvec, ninl, stream=None):
        """Gather this step's shard results and chain the world*B pairs into
        self.poses [world*B, 4, 4] (absolute poses of the step's frames 1..)."""
        import torch
        import torch.distributed as dist

        from . import _lib
        from .device import ptr, stream_ptr

        st = stream if stream is not None else torch.cuda.current_stream()
        with torch.cuda.stream(st):
            self.buf[:, 0:3].copy_(rvec)
            self.buf[:, 3:6].copy_(tvec)
            self.buf[:, 6].copy_(ninl)
            dist.all_gather(self.parts, self.buf, group=self.group)
            self.rv.copy_(self.all[:, 0:3])
            self.tv.copy_(self.all[:, 3:6])
            self.ni.copy_(self.all[:, 6].round())
            _lib.call("slam_pose_chain", ptr(self.rv), ptr(self.tv), ptr(self.ni),
                      self.world * self.B, ptr(self.state), ptr(self.poses), stream_ptr(st))
        return self.poses


class CapiComm:
    """An RCCL communicator of the C ABI (slam_comm_*; include/slam355.h) over
    the ranks of a torch.distributed group: rank 0 creates the unique id, the
    group broadcasts it (128 bytes), every rank joins.  BAProblem.
    step_distributed(comm=...) then runs the sharded LM iteration as ONE C call
    (slam_ba_step_distributed: build, all-reduce, solve, all-reduce, decide)."""

    def __init__(self, group=None, single=False):
        """single=True: a one-rank communicator with no torch.distributed group
        (tests; a C caller's nranks = 1)."""
        import ctypes

        import torch

        from . import _lib

        idb = (ctypes.c_uint8 * 128)()
        if single:
            self.rank, self.world = 0, 1
            _lib.call("slam_comm_unique_id", ctypes.cast(idb, ctypes.c_void_p))
        else:
            import torch.distributed as dist

            self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
            if self.rank == 0:
                _lib.call("slam_comm_unique_id", ctypes.cast(idb, ctypes.c_void_p))
            t = torch.tensor(list(bytes(idb)), dtype=torch.uint8)
            if dist.get_backend(group) == "nccl":
                t = t.cuda()
            dist.broadcast(t, src=0, group=group)
            idb = (ctypes.c_uint8 * 128)(*t.cpu().tolist())
        self.handle = ctypes.c_void_p()
        _lib.call("slam_comm_init", self.world, self.rank, ctypes.cast(idb, ctypes.c_void_p),
                  ctypes.byref(self.handle))

    def allreduce_(self, t, stream=None):
        """In-place f64 sum of a contiguous device tensor over the ranks."""
        from . import _lib
        from .device import ptr, stream_ptr

        _lib.call("slam_comm_allreduce_f64", self.handle, ptr(t), t.numel(), stream_ptr(stream))

    def close(self):
        from . import _lib

        if self.handle:
            _lib.call("slam_comm_destroy", self.handle)
            self.handle = type(self.handle)()

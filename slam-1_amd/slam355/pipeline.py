"""Batched stereo tracking on the GPU — the per-frame loop of
/root/reference/main.py:76-132 restructured for MI355X.

The reference processes one frame pair per Python iteration:
  ORB(right_i), ORB(left_{i+1})                       main.py:79-80
  stereo kNN-2 + ratio + F-LMedS mask                 main.py:82-84 (keypoint.py:35-66)
  triangulate                                         main.py:86 (Point3D.py:14-19)
  temporal kNN-2 + ratio + |Q| gate                   main.py:88-90 (Point3D.py:33-53)
  PnP-RANSAC, sign flip, pose chaining                main.py:94-98, 120-124
Every step depends only on frames (i, i+1), so `Tracker.track` runs B frame
pairs per call as 13 kernel launches on one stream, with all intermediate
data resident in HBM; only the B relative poses (and counters) come back to
the host for the sequential 4x4 pose chain.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from . import _lib, geometry, matcher, orb
from .device import ptr, require_gpu, stream_ptr


class Tracker:
    """Device buffers for batches of B frame pairs of H x W images."""

    def __init__(self, B, H, W, P_l, P_r, max_kp_per_tile=56, seed=0, max_distance=500.0,
                 stream=None, orb_stream=None):
        """orb_stream: run ORB on that stream into two alternating workspaces, so
        the ORB of the next batch overlaps the matching / PnP tail of this one
        (the tail kernels are latency-bound and leave most CUs idle)."""
        self.dev = require_gpu()
        self.B, self.H, self.W = B, H, W
        self.max_kp = max_kp_per_tile
        self.seed = seed
        self.max_distance = float(max_distance)
        self.stream = stream
        self.P_l = np.asarray(P_l, np.float64)
        self.P_r = np.asarray(P_r, np.float64)
        self.K = self.P_l[:3, :3].copy()
        d = self.dev
        self.tPl = torch.as_tensor(self.P_l, device=d).contiguous()
        self.tPr = torch.as_tensor(self.P_r, device=d).contiguous()
        self.tK = torch.as_tensor(self.K, device=d).contiguous()
        # ORB on 2B+1 images: left_0..left_B then right_0..right_{B-1}
        self.ows = orb.OrbWorkspace(2 * B + 1, H, W, max_kp_per_tile)
        self.orb_stream = orb_stream
        if orb_stream is not None:  # double-buffered ORB outputs
            self.ows_pair = [self.ows, orb.OrbWorkspace(2 * B + 1, H, W, max_kp_per_tile)]
            self.orb_done = [torch.cuda.Event() for _ in range(2)]
            self.slot_free = [torch.cuda.Event() for _ in range(2)]
            self._k = 0
        cap = self.cap = self.ows.kp_cap
        i32 = dict(dtype=torch.int32, device=d)
        f64 = dict(dtype=torch.float64, device=d)
        u8 = dict(dtype=torch.uint8, device=d)
        self.s_idx2 = torch.full((B, cap, 2), -1, **i32)
        self.s_dist2 = torch.full((B, cap, 2), -1, **i32)
        self.s_good = torch.zeros((B, cap), **u8)
        self.s_pairs = torch.zeros((B, cap, 2), **i32)
        self.s_cnt = torch.zeros((B,), **i32)
        self.s_ptl = torch.zeros((B, cap, 2), **f64)
        self.s_ptr = torch.zeros((B, cap, 2), **f64)
        self.f_mask = torch.zeros((B, cap), **u8)
        self.f_F = torch.zeros((B, 9), **f64)
        self.f_ninl = torch.zeros((B,), **i32)
        self.f_pairs = torch.zeros((B, cap, 2), **i32)
        self.f_cnt = torch.zeros((B,), **i32)
        self.f_ptl = torch.zeros((B, cap, 2), **f64)
        self.f_ptr = torch.zeros((B, cap, 2), **f64)
        self.f_dl = torch.zeros((B, cap, 32), **u8)
        self.f_dr = torch.zeros((B, cap, 32), **u8)
        self.X = torch.zeros((B, cap, 3), **f64)
        self.t_idx2 = torch.full((B, cap, 2), -1, **i32)
        self.t_dist2 = torch.full((B, cap, 2), -1, **i32)
        self.t_good = torch.zeros((B, cap), **u8)
        self.t_pairs = torch.zeros((B, cap, 2), **i32)
        self.t_cnt = torch.zeros((B,), **i32)
        self.Q1 = torch.zeros((B, cap, 3), **f64)
        self.q2 = torch.zeros((B, cap, 2), **f64)
        self.q1 = torch.zeros((B, cap, 2), **f64)
        self.rvec = torch.zeros((B, 3), **f64)
        self.tvec = torch.zeros((B, 3), **f64)
        self.p_ninl = torch.zeros((B,), **i32)
        self.p_mask = torch.zeros((B, cap), **u8)
        self.p_ws = geometry.pnp_workspace(B, dev=d)  # this Tracker's PnP hypotheses
        self.imgs = torch.zeros((2 * B + 1, H, W), **u8)
        # device pose chain (main.py:120-124): (pose, T) carried across batches
        self.chain_state = torch.zeros((32,), **f64)
        # identity pose + identity stale transform, device-resident: reset_chain
        # restarts the chain with an async device copy (no host synchronisation)
        self._chain_eye = torch.from_numpy(np.concatenate([np.eye(4), np.eye(4)]).ravel()).to(d)
        self.reset_chain()
        self.poses = torch.zeros((B, 4, 4), **f64)
        # running minimum of the ORB counts since the last check(): k_orb_compact
        # writes a negative count when a tile's retained ties exceed the
        # workspace (OpenCV keeps every tie); such a frame must not silently
        # degrade into "no matches" + a stale pose
        self.orb_min = torch.full((1,), 1 << 30, **i32)
        self.orb_event = torch.cuda.Event()
        # optional host-side issue time per call site (bench.py): {site: [seconds per call]}
        self.host_times = None

    def _ht(self, site, t0):
        """Record the host time since t0 against `site`; returns the new t0."""
        t1 = time.perf_counter()
        if self.host_times is not None:
            self.host_times.setdefault(site, []).append(t1 - t0)
        return t1

    # ------------------------------------------------------------------ device step
    def track(self, frame0: int, imgs: torch.Tensor | None = None, marks=None, chain=True):
        """Run the B frame pairs (frame0 + b, frame0 + b + 1), b < B, on device.

        `imgs` [2B+1, H, W] u8 = left_{frame0..frame0+B}, right_{frame0..frame0+B-1}
        (defaults to self.imgs, filled by the caller).  Asynchronous: returns
        device tensors (rvec, tvec, n_inliers); with `chain` the absolute poses
        of frames frame0+1 .. frame0+B are chained on the device into
        self.poses [B,4,4] (main.py:120-124), continuing from the previous call."""
        B, st = self.B, self.stream
        im = self.imgs if imgs is None else imgs

        def mark(name):  # optional stage events on the launch stream (bench.py)
            if marks is not None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(st if st is not None else torch.cuda.current_stream())
                marks.append((name, ev))

        main = st if st is not None else torch.cuda.current_stream()
        ost = self.orb_stream
        h0 = time.perf_counter()
        if ost is None:
            mark("start")
            kp, octv, desc, cnt = self.ows.run(im, st)
            _lib.call("slam_count_min", ptr(cnt), cnt.numel(), ptr(self.orb_min), stream_ptr(main))
            # ORB of this batch done: a caller may hold other work back until here
            self.orb_event.record(main)
            mark("orb")
        else:
            slot = self._k % 2
            self._k += 1
            self.ows = ows = self.ows_pair[slot]
            ost.wait_event(self.slot_free[slot])  # the tail that read this slot is done
            if imgs is None:  # self.imgs was filled on `main`; a caller passing `imgs`
                ost.wait_stream(main)  # orders their upload against `orb_stream` itself
            if marks is not None:  # ORB's own lane: start (past the waits) -> done
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(ost)
            kp, octv, desc, cnt = ows.run(im, ost)
            # (a torch.minimum here blocked the host on every step: ~1.5 ms)
            _lib.call("slam_count_min", ptr(cnt), cnt.numel(), ptr(self.orb_min), stream_ptr(ost))
            if marks is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(ost)
                self.orb_marks = [("start", e0), ("orb", e1)]
            self.orb_event.record(ost)
            self.orb_done[slot].record(ost)
            main.wait_event(self.orb_done[slot])
            mark("orb_wait")
        h0 = self._ht("orb_launch", h0)
        kpL, kpR = kp[0:B], kp[B + 1:2 * B + 1]
        dL, dR = desc[0:B], desc[B + 1:2 * B + 1]
        nL, nR = cnt[0:B], cnt[B + 1:2 * B + 1]
        kpL1, dL1, nL1 = kp[1:B + 1], desc[1:B + 1], cnt[1:B + 1]
        # stereo: kNN-2 + ratio (keypoint.py:44-51), gather (:96-97)
        matcher.knn2_batch(dL, nL, dR, nR, out=(self.s_idx2, self.s_dist2, self.s_good), stream=st)
        mark("stereo_knn2")
        matcher.compact_matches(self.s_idx2, self.s_good, nL, out=(self.s_pairs, self.s_cnt),
                                stream=st)
        geometry.gather_matches(kpL, kpR, self.s_pairs, self.s_cnt,
                                out=(self.s_ptl, self.s_ptr, None, None), stream=st)
        mark("stereo_match")
        h0 = self._ht("stereo_launch", h0)
        # F-LMedS mask (keypoint.py:59-66), then the surviving pairs with descriptors
        geometry.fundamental_lmeds(self.s_ptl, self.s_ptr, self.s_cnt, seed=self.seed,
                                   item0=frame0, out=(self.f_mask, self.f_F, self.f_ninl),
                                   stream=st)
        mark("f_lmeds")
        geometry.filter_pairs(self.s_pairs, self.s_cnt, self.f_mask,
                              out=(self.f_pairs, self.f_cnt), stream=st)
        geometry.gather_matches(kpL, kpR, self.f_pairs, self.f_cnt, dL, dR,
                                out=(self.f_ptl, self.f_ptr, self.f_dl, self.f_dr), stream=st)
        # triangulate (Point3D.py:14-19)
        geometry.triangulate(self.f_ptl, self.f_ptr, self.f_cnt, self.tPl, self.tPr, out=self.X,
                             stream=st)
        # temporal: tracked left descriptors at t vs left at t+1, ratio + |Q| gate
        matcher.knn2_batch(self.f_dl, self.f_cnt, dL1, nL1,
                           out=(self.t_idx2, self.t_dist2, self.t_good), stream=st)
        matcher.compact_matches(self.t_idx2, self.t_good, self.f_cnt, gate_xyz=self.X,
                                gate=self.max_distance, out=(self.t_pairs, self.t_cnt), stream=st)
        geometry.gather_temporal(self.X, self.f_ptl, kpL1, self.t_pairs, self.t_cnt,
                                 out=(self.Q1, self.q2, self.q1), stream=st)
        if ost is not None:  # the last read of this slot's ORB outputs
            self.slot_free[slot].record(main)
        mark("triangulate_temporal")
        h0 = self._ht("flmeds_tri_temporal_launch", h0)
        # PnP-RANSAC (transformation.py:11-13)
        geometry.pnp_ransac(self.Q1, self.q2, self.t_cnt, self.tK, seed=self.seed, item0=frame0,
                            out=(self.rvec, self.tvec, self.p_ninl, self.p_mask), stream=st,
                            ws=self.p_ws)
        mark("pnp")
        h0 = self._ht("pnp_launch", h0)
        if chain:
            _lib.call("slam_pose_chain", ptr(self.rvec), ptr(self.tvec), ptr(self.p_ninl), B,
                      ptr(self.chain_state), ptr(self.poses), stream_ptr(st))
            mark("pose_chain")
            self._ht("pose_chain_launch", h0)
        return self.rvec, self.tvec, self.p_ninl

    def reset_chain(self, pose0=None, T0=None):
        """Start the device pose chain at pose0 (default identity) with T0 as the
        stale transform (default identity)."""
        # on the tracking stream, ordered after the previous batch's pose chain; a
        # host-built start state is allocated on that same stream, so the caching
        # allocator cannot hand its memory out before the copy has run
        with torch.cuda.stream(self.stream if self.stream is not None
                               else torch.cuda.current_stream()):
            if pose0 is None and T0 is None:
                src = self._chain_eye
            else:  # a host-built start state (a synchronous upload; not on the bench path)
                st = np.concatenate([np.eye(4) if pose0 is None else np.asarray(pose0, float),
                                     np.eye(4) if T0 is None else np.asarray(T0, float)]).ravel()
                src = torch.from_numpy(st).to(self.chain_state.device)
            self.chain_state.copy_(src, non_blocking=True)

    def check(self):
        """Synchronises: raise if any ORB count since the last check was negative
        (keypoint workspace overflow: too many tied responses in a tile, or more
        keypoints than kp_cap), then reset the flag."""
        cur = torch.cuda.current_stream()
        streams = [x for x in (self.stream, self.orb_stream) if x is not None]
        for x in streams:  # the host read below follows every queued ORB count update
            cur.wait_stream(x)
        m = int(self.orb_min.item())
        self.orb_min.fill_(1 << 30)
        for x in streams:  # and the next batch's updates follow the reset
            x.wait_stream(cur)
        if m < 0:
            raise _lib.SlamError("Tracker: ORB keypoint workspace overflow (a tile kept more tied "
                                 "responses than the workspace holds, or kp_cap was exceeded); "
                                 "the frame would have been tracked with no matches")

    def counters(self):
        self.check()  # also orders the current stream after the tracking / ORB streams
        return dict(orb=self.ows.count.cpu().numpy(), stereo=self.s_cnt.cpu().numpy(),
                    f_inliers=self.f_cnt.cpu().numpy(), temporal=self.t_cnt.cpu().numpy(),
                    pnp_inliers=self.p_ninl.cpu().numpy())


def relative_transform(rvec, tvec):
    """transformation.py:15-19: T = [Rodrigues(-rvec) | -tvec] (the reference's
    sign flip, not the true inverse of the PnP pose)."""
    from .transformation import translation_and_rotation_vector_to_matrix

    return translation_and_rotation_vector_to_matrix(-1 * np.asarray(rvec).reshape(3, 1),
                                                     -1 * np.asarray(tvec).reshape(3, 1))


def chain_poses(pose0, rvecs, tvecs, ninl, T_prev=None):
    """main.py:94-98, 120-124: pose_{i+1} = pose_i @ T_i; when PnP had <= 4 points
    the previous T is reused (stale).  Returns (poses [B,4,4], last T)."""
    poses = []
    pose = np.asarray(pose0, float)
    T = np.eye(4) if T_prev is None else T_prev
    for r, t, n in zip(rvecs, tvecs, ninl):
        if n >= 0:
            T = relative_transform(r, t)
        pose = pose @ T
        poses.append(pose)
    return np.stack(poses), T


class LocalMap:
    """The mapping half of main.py's loop (:120-127) on the device, for
    tracked batches: each pair's temporally matched 3-D points (Q1, relative to
    frame i) go to the world frame with the NEW pose (relative_to_abs3DPoints,
    Point3D.py:22-30: k_rel_to_abs), then appendKeyPoints (keypoint.py:101-122:
    MapStore, exact nearest landmark + the |rel|-scaled gate) adds the rows
    [frame i, landmark, u, v] (u, v = the left image coordinates at time i).
    `problem()` returns the BA problem export_data / read_bal_data would give
    (XXXport_files.problem_from_map), ready for slam355.ba.BAProblem."""

    def __init__(self, tracker: Tracker, threshold=0.01, capacity=1 << 16):
        from .mapping import MapStore

        self.trk = tracker
        self.threshold = float(threshold)
        B, cap = tracker.B, tracker.cap
        self.store = MapStore(capacity=capacity, max_queries=cap)
        d = tracker.dev
        self.abs = torch.zeros((B, cap, 3), dtype=torch.float64, device=d)
        self.rows = torch.zeros((B, cap, 4), dtype=torch.float64, device=d)
        self._rows_host = []
        self.poses = [np.eye(4)]  # camera_frames (main.py:52-54)

    def add(self, frame0: int):
        """Map the batch Tracker.track(frame0) just tracked (same stream)."""
        t = self.trk
        st = t.stream
        _lib.call("slam_rel_to_abs", ptr(t.Q1), ptr(t.t_cnt), t.cap, t.B, ptr(t.poses),
                  ptr(self.abs), stream_ptr(st))
        for b in range(t.B):
            self.store.append(self.abs[b], t.Q1[b], t.q1[b], frame0 + b, self.threshold,
                              count=t.t_cnt[b:b + 1], rows=self.rows[b], stream=st)
        if st is not None:  # the host reads below follow the launches queued on `st`
            torch.cuda.current_stream().wait_stream(st)
        cnt = t.t_cnt.cpu().numpy()
        rows = self.rows.cpu().numpy()
        self._rows_host += [rows[b, :cnt[b]] for b in range(t.B)]
        self.poses += list(t.poses.cpu().numpy())

    def optimization_matrix(self):
        return np.vstack(self._rows_host) if self._rows_host else np.empty((0, 4))

    def problem(self, P_left):
        from .XXXport_files import problem_from_map

        return problem_from_map(self.optimization_matrix(), self.poses,
                                self.store.points().cpu().numpy(), P_left)


class WindowMapper:
    """The local maps of a tracked batch's windows on the device, for local BA
    on tracked data at throughput (bench.py's tracked leg): main.py:120-127 per
    window of `n` consecutive frame pairs of one Tracker batch.

    `map_batch(stream)` (after Tracker.track on `stream`): the batch's temporal
    3-D points to the world frame (one k_rel_to_abs launch, the NEW pose as in
    LocalMap), then, window by window, a fresh device map fed the window's pairs
    in order (appendKeyPoints as MapStore does, all windows in one
    slam_map_windows call; frame index = the pair's index inside the window),
    and one device -> pinned-host copy of the rows, counts, poses and maps,
    recorded by `event`.  `problems(P_left)` (host, once the event
    has fired) forms each window's BA problem as XXXport_files.problem_from_map
    does: cameras = the window's first n frames (rotation vector, t, f, 0, 0),
    points = its map, one observation per row.  Call `save_pose0(stream)`
    before Tracker.track so the window at the batch start has its first frame's
    pose (the chain state before the batch)."""

    def __init__(self, tracker: Tracker, n: int, threshold=0.01):
        import ctypes

        self.trk, self.n = tracker, int(n)
        B, cap, d = tracker.B, tracker.cap, tracker.dev
        if self.n < 1 or B % self.n:
            raise ValueError(f"window of {n} pairs must divide the batch of {B}")
        self.n_win = B // self.n
        self.threshold = float(threshold)
        self.maps = torch.zeros((self.n_win, self.n * cap, 3), dtype=torch.float64, device=d)
        self.d_M = torch.zeros((self.n_win,), dtype=torch.int32, device=d)
        nb = ctypes.c_size_t(0)
        _lib.call("slam_map_workspace_bytes", cap, (self.n - 1) * cap, ctypes.byref(nb))
        # one workspace slice per window (slam_map_windows runs a pair of every window per launch)
        self.ws = torch.empty(max(self.n_win * int(nb.value), 1), dtype=torch.uint8, device=d)
        f64 = dict(dtype=torch.float64, device=d)
        self.abs = torch.zeros((B, cap, 3), **f64)
        self.rows = torch.zeros((B, cap, 4), **f64)
        self.pose0 = torch.eye(4, **f64)
        pin = dict(pin_memory=True)
        self.h_rows = torch.zeros((B, cap, 4), dtype=torch.float64, **pin)
        self.h_cnt = torch.zeros((B,), dtype=torch.int32, **pin)
        self.h_poses = torch.zeros((B, 4, 4), dtype=torch.float64, **pin)
        self.h_pose0 = torch.zeros((4, 4), dtype=torch.float64, **pin)
        self.h_maps = torch.zeros((self.n_win, self.n * cap, 3), dtype=torch.float64, **pin)
        self.h_M = torch.zeros((self.n_win,), dtype=torch.int32, **pin)
        self.event = torch.cuda.Event()
        self.copy_stream = torch.cuda.Stream()
        self.filled = False

    def save_pose0(self, stream):
        with torch.cuda.stream(stream):
            self.pose0.copy_(self.trk.chain_state[:16].view(4, 4), non_blocking=True)

    def map_batch(self, stream):
        t = self.trk
        stream.wait_event(self.event)  # this mapper's previous host copies have run
        with torch.cuda.stream(stream):
            _lib.call("slam_rel_to_abs", ptr(t.Q1), ptr(t.t_cnt), t.cap, t.B, ptr(t.poses),
                      ptr(self.abs), stream_ptr(stream))
            # every window's device map in one call (slam_map_windows: the
            # appendKeyPoints launches of its pairs, in order, maps restarted
            # empty; pair j of all windows per launch)
            _lib.call("slam_map_windows", ptr(self.maps), ptr(self.d_M), self.n * t.cap, self.n_win,
                      self.n, ptr(self.abs), ptr(t.Q1), ptr(t.q1), ptr(t.t_cnt), t.cap,
                      self.threshold, ptr(self.rows), ptr(self.ws), self.ws.numel(), stream_ptr(stream))
            # the tracker's buffers (rewritten by the next batch) are copied on
            # the tracking stream; the mapper's own maps and rows (~7 MB at 64
            # pairs) on a copy stream, so the next batch's tracking does not
            # queue behind them
            self.h_cnt.copy_(t.t_cnt, non_blocking=True)
            self.h_poses.copy_(t.poses, non_blocking=True)
            self.h_pose0.copy_(self.pose0, non_blocking=True)
            self.h_M.copy_(self.d_M, non_blocking=True)
        self.copy_stream.wait_stream(stream)
        with torch.cuda.stream(self.copy_stream):
            self.h_maps.copy_(self.maps, non_blocking=True)
            self.h_rows.copy_(self.rows, non_blocking=True)
            self.event.record(self.copy_stream)
        self.filled = True

    def stage(self, ws, P_left, stream, lam0=1e-4):
        """The batch's windows as BA problems in one native call
        (BAWindowSet.stage over this mapper's host copies; call after
        event.synchronize()): the same problems as ws.build(self.problems(P_left))."""
        from .XXXport_files import U_OFF, V_OFF, make_cam_params

        frames = np.concatenate([self.h_pose0.numpy()[None], self.h_poses.numpy()[:-1]])
        cams = make_cam_params(frames, P_left).reshape(-1, 9)
        return ws.stage(self.h_rows.numpy(), self.h_cnt.numpy(), self.h_maps.numpy(),
                        self.h_M.numpy(), cams, U_OFF, V_OFF, stream, lam0)

    def problems(self, P_left):
        """Every window's (cams [n,9], pts [M,3], cam_idx, pt_idx, qs [O,2]) from
        the host copy (call after event.synchronize()); the camera parameters of
        the batch's frames in one make_cam_params call."""
        from .XXXport_files import U_OFF, V_OFF, make_cam_params

        n = self.n
        cnt = self.h_cnt.numpy()
        rows = self.h_rows.numpy()
        poses = self.h_poses.numpy()
        # frame b of the batch = pose before pair b (window w: frames w n .. w n + n - 1)
        frames = np.concatenate([self.h_pose0.numpy()[None], poses[:-1]])
        allcams = make_cam_params(frames, P_left).reshape(-1, 9)
        out = []
        for w in range(self.n_win):
            b0 = w * n
            om = np.concatenate([rows[b, :max(int(cnt[b]), 0)] for b in range(b0, b0 + n)])
            pts = self.h_maps[w, :int(self.h_M[w])].numpy().copy()
            qs = np.stack([om[:, 2] - U_OFF, om[:, 3] - V_OFF], 1)
            out.append((allcams[b0:b0 + n].copy(), pts, om[:, 0].astype(np.int64),
                        om[:, 1].astype(np.int64), qs))
        return out

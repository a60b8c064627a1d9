"""Device-resident landmark map: appendKeyPoints (/root/reference/keypoint.py:101-122)
on the GPU.

`MapStore` keeps the map Qs [cap, 3] f64 and its size M in HBM.  `append`
associates one frame's new absolute points with the map (exact nearest
neighbour + the reference's |rel|-scaled gate) and appends the unmatched ones,
all on the stream, so a sequence of frames runs without host synchronisation;
the host only tracks an upper bound of M to size grids and grow the buffer.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .device import ptr, require_gpu, stream_ptr, to_dev


class MapStore:
    def __init__(self, capacity=1 << 16, max_queries=4096, Qs=None):
        self.dev = require_gpu()
        self.cap = int(capacity)
        self.max_q = int(max_queries)
        self.map = torch.zeros((self.cap, 3), dtype=torch.float64, device=self.dev)
        self.M = torch.zeros((1,), dtype=torch.int32, device=self.dev)
        self.m_bound = 0
        self._ws = None
        self._ws_for = (-1, -1)
        if Qs is not None and len(Qs):
            Qs = np.ascontiguousarray(Qs, np.float64).reshape(-1, 3)
            self._grow(len(Qs))
            self.map[: len(Qs)] = torch.from_numpy(Qs).to(self.dev)
            self.M.fill_(len(Qs))
            self.m_bound = len(Qs)

    def _grow(self, need):
        if need <= self.cap:
            return
        cap = max(need, 2 * self.cap)
        m = torch.zeros((cap, 3), dtype=torch.float64, device=self.dev)
        m[: self.cap] = self.map
        self.map, self.cap = m, cap

    def _workspace(self, n):
        key = (n, self.m_bound)
        if self._ws is None or self._ws_for[0] < n or self._ws_for[1] < self.m_bound:
            nb = ctypes.c_size_t(0)
            _lib.call("slam_map_workspace_bytes", max(n, self.max_q), max(self.m_bound, self.cap),
                      ctypes.byref(nb))
            self._ws = torch.empty(int(nb.value), dtype=torch.uint8, device=self.dev)
            self._ws_for = (max(n, self.max_q), max(self.m_bound, self.cap))
        return self._ws, key

    def append(self, abs_pts, rel_pts, pts2d, frame_index, threshold=0.01, count=None,
               rows=None, stream=None):
        """One frame: abs_pts, rel_pts [N,3] f64, pts2d [N,2] f64 (device) ->
        rows [N,4] f64 = [frame, landmark index, u, v]; the map grows in place.
        `count` (device int32 [1], optional) = number of valid points (<= N)."""
        N = int(abs_pts.shape[0])
        self._grow(self.m_bound + N)
        ws, _ = self._workspace(N)
        out = rows if rows is not None else torch.empty((max(N, 1), 4), dtype=torch.float64,
                                                        device=self.dev)
        _lib.call("slam_map_associate", ptr(self.map), ptr(self.M), self.cap, self.m_bound,
                  ptr(abs_pts), ptr(rel_pts), ptr(pts2d), ptr(count), N, float(threshold),
                  int(frame_index), ptr(out), ptr(ws), ws.numel(), stream_ptr(stream))
        self.m_bound += N
        return out[:N]

    def size(self) -> int:
        """Synchronises: the current number of landmarks."""
        m = int(self.M.item())
        self.m_bound = m
        return m

    def points(self) -> torch.Tensor:
        return self.map[: self.size()]


def appendKeyPoints(Qs, absPoint, threshold, points_2d, frame_index, rel_point):
    """(keypoint.py:101-122) -> (Qs with the new landmarks appended, rows [N,4])."""
    Qs = np.asarray(Qs, np.float64).reshape(-1, 3)
    absPoint = np.ascontiguousarray(absPoint, np.float64).reshape(-1, 3)
    rel = np.ascontiguousarray(rel_point, np.float64).reshape(-1, 3)
    p2 = np.ascontiguousarray(points_2d, np.float64).reshape(-1, 2)
    n = len(absPoint)
    store = MapStore(capacity=max(len(Qs) + n, 1), max_queries=max(n, 1), Qs=Qs)
    if n == 0:
        return Qs.copy(), np.empty((0, 4))
    rows = store.append(to_dev(absPoint), to_dev(rel), to_dev(p2[:n]), frame_index, threshold)
    return store.points().cpu().numpy(), rows.cpu().numpy()

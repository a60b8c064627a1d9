"""ORACLE (test infrastructure only): map association on the CPU.

  append_keypoints   /root/reference/keypoint.py:101-122 (appendKeyPoints)

Restated in vectorised form with the reference's own KDTree (scipy.spatial):
the tree is built on the map as it was before the call (:109), every new point
queries its nearest landmark (:110), points within threshold * |rel| (:113)
take that landmark's index, the others are appended in order and get
M, M+1, ... (:117-118) — a prefix count over the unmatched points.
"""
from __future__ import annotations

import numpy as np
from scipy.spatial import KDTree


def append_keypoints(Qs, absPoint, threshold, points_2d, frame_index, rel_point):
    Qs = np.asarray(Qs, np.float64).reshape(-1, 3)
    absPoint = np.asarray(absPoint, np.float64).reshape(-1, 3)
    rel = np.asarray(rel_point, np.float64).reshape(-1, 3)
    p2 = np.asarray(points_2d, np.float64).reshape(-1, 2)
    n, M = len(absPoint), len(Qs)
    if M == 0:
        new = np.ones(n, bool)
        ind = np.zeros(n, np.int64)
    else:
        dist, ind = KDTree(Qs).query(absPoint, k=1)
        gate = threshold * np.sqrt(np.sum(rel ** 2, axis=1))
        new = ~(dist < gate)
    idx = np.where(new, M + np.cumsum(new) - 1, ind)
    rows = np.column_stack([np.full(n, float(frame_index)), idx.astype(float), p2[:n, 0], p2[:n, 1]])
    return np.vstack([Qs, absPoint[new]]), rows.reshape(-1, 4)

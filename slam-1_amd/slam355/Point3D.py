"""Drop-in for /root/reference/Point3D.py (triangulation and 2D-3D matching on the GPU)."""
from __future__ import annotations

import numpy as np
import torch

from . import geometry, matcher
from .device import require_gpu, to_dev


def sort_3D_points(triangulated_3D_point, close_def_in_m=100, far_def_in_m=1):
    """(Point3D.py:5-10) host bookkeeping; its result is unused by the reference PnP."""
    P = np.asarray(triangulated_3D_point, float).reshape(-1, 3)
    a = np.abs(P)
    return list((a < close_def_in_m).all(1)), list((a > far_def_in_m).any(1))


def triangulate_points_local(qs_l, qs_r, P_l, P_r):
    """(Point3D.py:14-19) -> (M, 3) float64 (GPU kernel k_triangulate)."""
    ql = np.asarray(qs_l, np.float64).reshape(-1, 2)
    qr = np.asarray(qs_r, np.float64).reshape(-1, 2)
    M = len(ql)
    if M == 0:
        return np.zeros((0, 3))
    dev = require_gpu()
    X = geometry.triangulate(to_dev(ql[None]), to_dev(qr[None]),
                             torch.tensor([M], dtype=torch.int32, device=dev), P_l, P_r)
    return X[0].cpu().numpy()


def relative_to_abs3DPoints(points3D, camera_frame):
    """(Point3D.py:22-30) a single 4x4 transform of a few hundred points (host)."""
    P = np.asarray(points3D, float).reshape(-1, 3)
    hom = np.hstack((P, np.ones((len(P), 1))))
    a = np.matmul(camera_frame, hom.T)
    return (a[:3] / a[3]).T


def _pts(kps):
    if isinstance(kps, np.ndarray):
        return np.asarray(kps, np.float32).reshape(-1, 2)
    return np.asarray([k.pt for k in kps], np.float32).reshape(-1, 2)


def find_2D_and_3D_correspondenses(descriptors_time_i, keypoints_left_time_i,
                                   keypoints_left_time_i1, descriptors_left_time_i1,
                                   triangulated_3D_points, max_Distance=1000):
    """(Point3D.py:33-53) -> (q2 [L,2] f64, Q1 [L,3] f64, q1 [L,2])."""
    dq = np.ascontiguousarray(descriptors_time_i, np.uint8).reshape(-1, 32)
    dt = np.ascontiguousarray(descriptors_left_time_i1, np.uint8).reshape(-1, 32)
    Q = np.asarray(triangulated_3D_points, np.float64).reshape(-1, 3)
    dev = require_gpu()
    M, N = len(dq), len(dt)
    q = to_dev((dq if M else np.zeros((1, 32), np.uint8))[None])
    t = to_dev((dt if N else np.zeros((1, 32), np.uint8))[None])
    nq = torch.tensor([M], dtype=torch.int32, device=dev)
    nt = torch.tensor([N], dtype=torch.int32, device=dev)
    idx2, dist2, good = matcher.knn2_batch(q, nq, t, nt)
    gate = to_dev((Q if M else np.zeros((1, 3)))[None])
    pairs, cnt = matcher.compact_matches(idx2, good, nq, gate_xyz=gate, gate=float(max_Distance))
    n = int(cnt[0].item())
    p = pairs[0, :n].cpu().numpy()
    q2 = _pts(keypoints_left_time_i1)[p[:, 1]].astype(np.float64)
    Q1 = Q[p[:, 0]]
    q1 = np.asarray(keypoints_left_time_i)[p[:, 0]]
    return q2, Q1, q1

"""ORACLE (test infrastructure only): numpy restatement of the reference's
post-processing around knnMatch(k=2), driven by the exact C kNN-2 oracle.

  stereo_matches   /root/reference/keypoint.py:35-66 (F-LMedS mask excluded:
                   pass `mask` explicitly; the golden uses an all-inlier mask)
  temporal_matches /root/reference/Point3D.py:33-53
  get_matches      /root/reference/tracking.py:12-34
"""
from __future__ import annotations

import numpy as np

from . import hamming_knn2


def good_pairs(des_q, des_t):
    """The `good` list (keypoint.py:45-51) as an (M, 2) int array of (queryIdx, trainIdx).

    With an exact matcher every query has 2 neighbours iff len(des_t) >= 2; with
    fewer, the first `for m, n in matches` unpack raises ValueError and the
    reference keeps nothing.
    """
    idx2, dist2, good = hamming_knn2(des_q, des_t)
    q = np.nonzero(good)[0]
    return np.stack([q, idx2[q, 0]], 1).astype(np.int64) if len(q) else np.zeros((0, 2), np.int64)


def stereo_matches(pts_l, des_l, pts_r, des_r, mask=None):
    """keypoint.py:44-66 -> (pts_left f64 [M,2], pts_right, des_left u8 [M,32], des_right)."""
    p = good_pairs(des_l, des_r)
    pts_left = np.asarray(pts_l, np.float32)[p[:, 0]].astype(np.float64)
    pts_right = np.asarray(pts_r, np.float32)[p[:, 1]].astype(np.float64)
    dl = np.asarray(des_l, np.uint8)[p[:, 0]]
    dr = np.asarray(des_r, np.uint8)[p[:, 1]]
    if mask is not None:
        m = np.asarray(mask, bool).ravel()
        pts_left, pts_right, dl, dr = pts_left[m], pts_right[m], dl[m], dr[m]
    return pts_left, pts_right, dl, dr


def temporal_matches(des_i, pts_i, pts_i1, des_i1, Q, max_Distance=1000):
    """Point3D.py:33-53 -> (q2 [L,2] f64 from kp_{i+1}.pt, Q1 [L,3], q1 [L,2])."""
    p = good_pairs(des_i, des_i1)
    Q = np.asarray(Q, np.float64)
    if len(p):
        keep = np.all(np.abs(Q[p[:, 0]]) < max_Distance, axis=1)
        p = p[keep]
    q2 = np.asarray(pts_i1, np.float32)[p[:, 1]].astype(np.float64)
    Q1 = Q[p[:, 0]]
    q1 = np.asarray(pts_i)[p[:, 0]]
    return q2, Q1, q1


def get_matches(pts1, des1, pts2, des2):
    """tracking.py:12-34 -> float32 (q1, q2)."""
    p = good_pairs(des1, des2)
    return (np.asarray(pts1, np.float32)[p[:, 0]].reshape(-1, 2),
            np.asarray(pts2, np.float32)[p[:, 1]].reshape(-1, 2))

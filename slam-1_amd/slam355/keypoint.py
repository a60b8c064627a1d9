"""Mirror of /root/reference/keypoint.py's hot-path function, on the GPU.

track_keypoints_left_to_right_new (keypoint.py:35-80): kNN-2 of the left
descriptors against the right ones with the 0.7 ratio test (:44-51), the
matched points as float64 and descriptors (:53-57), the F-LMedS inlier mask
(:59-66).  The GUI block (:68-78) is not part of the hot path and is dropped.
FLANN-LSH is replaced by exact brute force (Oracle); the F-LMedS
fit is the seeded deterministic one of csrc/fundamental.hip.

appendKeyPoints (keypoint.py:101-122, map association) is re-exported from
slam355.mapping (GPU nearest-neighbour association, device-resident map).
"""
from __future__ import annotations

import numpy as np
import torch

from . import geometry, matcher
from .device import require_gpu, to_dev
from .mapping import appendKeyPoints  # noqa: F401  (keypoint.py:101)


def _pts(kps):
    if isinstance(kps, np.ndarray):
        return np.asarray(kps, np.float32).reshape(-1, 2)
    return np.asarray([k.pt for k in kps], np.float32).reshape(-1, 2)


def good_pairs(descriptors_q, descriptors_t):
    """The reference's `good` list as an (M, 2) int array (queryIdx, trainIdx),
    in query order (keypoint.py:44-51)."""
    dq = np.ascontiguousarray(descriptors_q, np.uint8).reshape(-1, 32)
    dt = np.ascontiguousarray(descriptors_t, np.uint8).reshape(-1, 32)
    dev = require_gpu()
    M, N = len(dq), len(dt)
    q = to_dev((dq if M else np.zeros((1, 32), np.uint8))[None])
    t = to_dev((dt if N else np.zeros((1, 32), np.uint8))[None])
    nq = torch.tensor([M], dtype=torch.int32, device=dev)
    nt = torch.tensor([N], dtype=torch.int32, device=dev)
    idx2, _, good = matcher.knn2_batch(q, nq, t, nt)
    pairs, cnt = matcher.compact_matches(idx2, good, nq)
    return pairs[0, :int(cnt[0].item())].cpu().numpy().astype(np.int64)


def track_keypoints_left_to_right_new(key_points_left, descriptors_left, key_points_right,
                                      descriptors_right, leftimg=None, rightimg=None, *,
                                      seed=0, frame=0):
    """keypoint.py:35-80 -> (pts_left [M,2] f64, pts_right [M,2] f64,
    des_left [M,32] u8, des_right [M,32] u8) after the F-LMedS mask.
    `leftimg`/`rightimg` are accepted for signature parity (GUI only)."""
    p = good_pairs(descriptors_left, descriptors_right)
    pts_left = _pts(key_points_left)[p[:, 0]].astype(np.float64)
    pts_right = _pts(key_points_right)[p[:, 1]].astype(np.float64)
    des_left = np.ascontiguousarray(descriptors_left, np.uint8).reshape(-1, 32)[p[:, 0]]
    des_right = np.ascontiguousarray(descriptors_right, np.uint8).reshape(-1, 32)[p[:, 1]]
    M = len(p)
    dev = require_gpu()
    m1 = to_dev((pts_left if M else np.zeros((1, 2)))[None])
    m2 = to_dev((pts_right if M else np.zeros((1, 2)))[None])
    cnt = torch.tensor([M], dtype=torch.int32, device=dev)
    mask, _, _ = geometry.fundamental_lmeds(m1, m2, cnt, seed=seed, item0=frame)
    keep = mask[0, :M].cpu().numpy().astype(bool)
    return pts_left[keep], pts_right[keep], des_left[keep], des_right[keep]


def track_keypoints_left_to_right(image_left, image_right, key_points_left, descriptors_left,
                                  max_error=500):
    """(keypoint.py:13-32) pyramidal LK from the left to the right image (15x15,
    3 levels, 50 iterations / 0.03), then status, err < max_error and
    0 < np.around(p2) < (w, h) -> (trackpoints1 [M,2] f32, descriptors [M,32],
    trackpoints2 [M,2] f32), all on the GPU (csrc/vofront.hip)."""
    from . import vofront

    dev = require_gpu()
    p1 = _pts(key_points_left)
    des = np.asarray(descriptors_left)
    n = len(p1)
    if n == 0:
        return p1, des[:0], p1.copy()
    H, W = np.asarray(image_right).shape
    imgs = to_dev(np.stack([np.asarray(image_left, np.uint8), np.asarray(image_right, np.uint8)]))
    pyr = vofront.LKPyramids(imgs)
    t1 = to_dev(p1[None])
    cnt = torch.tensor([n], dtype=torch.int32, device=dev)
    p2, st, err = vofront.lk_track(pyr, pyr, t1, cnt, prev0=0, next0=1)
    tp1, tp2, idx, m = vofront.lk_filter(t1, p2, st, err, cnt, H, W, max_error=max_error,
                                         lower_bounds=True)
    k = int(m[0])
    sel = idx[0, :k].cpu().numpy()
    return tp1[0, :k].cpu().numpy(), des[sel], tp2[0, :k].cpu().numpy()

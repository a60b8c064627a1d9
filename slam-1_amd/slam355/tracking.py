"""Mirror of /root/reference/tracking.py's matcher, on the GPU.

get_matches (tracking.py:12-34): kNN-2 + 0.7 ratio (:22-30) and the matched
points as float32 (:32-33).  Exact brute force replaces FLANN-LSH.
"""
from __future__ import annotations

import numpy as np

from .keypoint import _pts, good_pairs


def get_matches(kp1, des1, kp2, des2):
    """tracking.py:12-34 -> (q1 [M,2] f32, q2 [M,2] f32)."""
    p = good_pairs(des1, des2)
    return (_pts(kp1)[p[:, 0]].reshape(-1, 2).astype(np.float32),
            _pts(kp2)[p[:, 1]].reshape(-1, 2).astype(np.float32))

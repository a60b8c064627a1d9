"""Exact Hamming kNN-2 matcher on the GPU (replaces FLANN-LSH knnMatch(k=2)).

Reference call sites: /root/reference/keypoint.py:40-51,
/root/reference/Point3D.py:35-49, /root/reference/tracking.py:14-30.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .device import ptr, require_gpu, stream_ptr, to_dev


def knn2_batch(q: torch.Tensor, nq: torch.Tensor, t: torch.Tensor, nt: torch.Tensor,
               *, out=None, stream=None):
    """Batched kNN-2 + ratio test on device tensors.

    q: [B, q_cap, 32] u8, nq: [B] i32, t: [B, t_cap, 32] u8, nt: [B] i32.
    Returns (idx2 [B,q_cap,2] i32, dist2 [B,q_cap,2] i32, good [B,q_cap] u8).
    Rows >= nq[b] are left untouched (initialised to -1 / 0 when allocated here).
    """
    B, q_cap, _ = q.shape
    t_cap = t.shape[1]
    if out is None:
        idx2 = torch.full((B, q_cap, 2), -1, dtype=torch.int32, device=q.device)
        dist2 = torch.full((B, q_cap, 2), -1, dtype=torch.int32, device=q.device)
        good = torch.zeros((B, q_cap), dtype=torch.uint8, device=q.device)
    else:
        idx2, dist2, good = out
    _lib.call("slam_hamming_knn2", ptr(q), ptr(nq), q_cap, ptr(t), ptr(nt), t_cap, B,
              ptr(idx2), ptr(dist2), ptr(good), stream_ptr(stream))
    return idx2, dist2, good


def compact_matches(idx2, good, nq, *, gate_xyz=None, gate=0.0, out=None, stream=None):
    """Order-preserving list of good (queryIdx, trainIdx) pairs per batch item."""
    B, q_cap = good.shape
    if out is None:
        pairs = torch.empty((B, max(q_cap, 1), 2), dtype=torch.int32, device=good.device)
        count = torch.empty((B,), dtype=torch.int32, device=good.device)
    else:
        pairs, count = out
    _lib.call("slam_compact_matches", ptr(idx2), ptr(good), ptr(nq), q_cap, B,
              ptr(gate_xyz), float(gate), ptr(pairs), ptr(count), stream_ptr(stream))
    return pairs, count


def knn2(des_q, des_t):
    """Single (query, train) pair from host/device arrays -> numpy (idx2, dist2, good)."""
    require_gpu()
    des_q = np.ascontiguousarray(des_q if not isinstance(des_q, torch.Tensor)
                                 else des_q.cpu().numpy(), dtype=np.uint8).reshape(-1, 32)
    des_t = np.ascontiguousarray(des_t if not isinstance(des_t, torch.Tensor)
                                 else des_t.cpu().numpy(), dtype=np.uint8).reshape(-1, 32)
    nq, nt = des_q.shape[0], des_t.shape[0]
    q = to_dev(des_q.reshape(1, nq, 32) if nq else np.zeros((1, 1, 32), np.uint8))
    t = to_dev(des_t.reshape(1, nt, 32) if nt else np.zeros((1, 1, 32), np.uint8))
    nq_d = to_dev(np.array([nq], np.int32))
    nt_d = to_dev(np.array([nt], np.int32))
    idx2, dist2, good = knn2_batch(q, nq_d, t, nt_d)
    return (idx2[0, :nq].cpu().numpy(), dist2[0, :nq].cpu().numpy(),
            good[0, :nq].cpu().numpy().astype(bool))

"""Device wrappers for gather / triangulation / PnP (csrc/geometry.hip)."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .device import ptr, require_gpu, stream_ptr

PNP_DEFAULTS = dict(n_hyp=100, reproj_thresh=8.0, hyp_iters=10, refine_iters=20)


def gather_matches(kpq, kpt, pairs, count, desq=None, dest=None, out=None, stream=None):
    """kp [B,cap,5] f32 + pairs [B,p_cap,2] -> (ptq, ptt [B,p_cap,2] f64, dq, dt [B,p_cap,32])."""
    B, p_cap, _ = pairs.shape
    dev = pairs.device
    if out is None:
        ptq = torch.zeros((B, p_cap, 2), dtype=torch.float64, device=dev)
        ptt = torch.zeros((B, p_cap, 2), dtype=torch.float64, device=dev)
        dq = dt = None
        if desq is not None:
            dq = torch.zeros((B, p_cap, 32), dtype=torch.uint8, device=dev)
            dt = torch.zeros((B, p_cap, 32), dtype=torch.uint8, device=dev)
    else:
        ptq, ptt, dq, dt = out
    _lib.call("slam_gather_matches", ptr(kpq), kpq.shape[1], ptr(kpt), kpt.shape[1], ptr(desq),
              ptr(dest), ptr(pairs), ptr(count), p_cap, B, ptr(ptq), ptr(ptt), ptr(dq), ptr(dt),
              stream_ptr(stream))
    return ptq, ptt, dq, dt


def gather_temporal(X, ptl, kp_next, pairs, count, out=None, stream=None):
    """-> (Q1 [B,p,3], q2 [B,p,2], q1 [B,p,2]) f64 (Point3D.py:50-52)."""
    B, pcap, _ = pairs.shape
    dev = pairs.device
    if out is None:
        Q1 = torch.zeros((B, pcap, 3), dtype=torch.float64, device=dev)
        q2 = torch.zeros((B, pcap, 2), dtype=torch.float64, device=dev)
        q1 = torch.zeros((B, pcap, 2), dtype=torch.float64, device=dev)
    else:
        Q1, q2, q1 = out
    _lib.call("slam_gather_temporal", ptr(X), ptr(ptl), X.shape[1], ptr(kp_next), kp_next.shape[1],
              ptr(pairs), ptr(count), pcap, B, ptr(Q1), ptr(q2), ptr(q1), stream_ptr(stream))
    return Q1, q2, q1


def fundamental_lmeds(m1, m2, count, seed=0, item0=0, n_hyp=300, out=None, stream=None):
    """m1/m2 [B,cap,2] f64 -> (mask [B,cap] u8, F [B,9] f64, ninliers [B] i32)."""
    B, cap, _ = m1.shape
    dev = m1.device
    if out is None:
        mask = torch.zeros((B, max(cap, 1)), dtype=torch.uint8, device=dev)
        F = torch.zeros((B, 9), dtype=torch.float64, device=dev)
        ninl = torch.zeros((B,), dtype=torch.int32, device=dev)
    else:
        mask, F, ninl = out
    _lib.call("slam_fundamental_lmeds", ptr(m1), ptr(m2), ptr(count), cap, B,
              int(seed) & ((1 << 64) - 1), int(item0), int(n_hyp), ptr(mask), ptr(F), ptr(ninl),
              stream_ptr(stream))
    return mask, F, ninl


def filter_pairs(pairs, count, mask, out=None, stream=None):
    """Keep pairs[b][k] with mask[b][k] (order preserved) -> (pairs', count')."""
    B, cap, _ = pairs.shape
    if out is None:
        o = torch.empty_like(pairs)
        oc = torch.empty((B,), dtype=torch.int32, device=pairs.device)
    else:
        o, oc = out
    _lib.call("slam_filter_pairs", ptr(pairs), ptr(count), ptr(mask), cap, B, ptr(o), ptr(oc),
              stream_ptr(stream))
    return o, oc


def triangulate(ptl, ptr_, count, P_l, P_r, out=None, stream=None):
    """ptl/ptr [B,cap,2] f64, P 3x4 (shared) or [B,3,4] -> X [B,cap,3] f64."""
    B, cap, _ = ptl.shape
    Pl = P_l if isinstance(P_l, torch.Tensor) else torch.as_tensor(np.asarray(P_l, np.float64),
                                                                   device=ptl.device)
    Pr = P_r if isinstance(P_r, torch.Tensor) else torch.as_tensor(np.asarray(P_r, np.float64),
                                                                   device=ptl.device)
    Pl, Pr = Pl.contiguous(), Pr.contiguous()
    stride = 12 if Pl.dim() == 3 else 0
    X = out if out is not None else torch.zeros((B, cap, 3), dtype=torch.float64, device=ptl.device)
    _lib.call("slam_triangulate", ptr(ptl), ptr(ptr_), ptr(count), cap, B, ptr(Pl), ptr(Pr), stride,
              ptr(X), stream_ptr(stream))
    return X


def pnp_ransac(Q, q, count, K, seed=0, item0=0, out=None, stream=None, ws=None, **kw):
    """Q [B,cap,3], q [B,cap,2] f64 -> (rvec [B,3], tvec [B,3], ninliers [B], mask [B,cap]).

    ws: the hypothesis-pose workspace (pnp_workspace(B, n_hyp)); calls that may
    run concurrently (other streams) must each pass their own.  Without one, a
    fresh buffer is allocated for this call (and kept alive for `stream`)."""
    prm = dict(PNP_DEFAULTS, **kw)
    B, cap, _ = Q.shape
    dev = Q.device
    Kt = K if isinstance(K, torch.Tensor) else torch.as_tensor(np.asarray(K, np.float64), device=dev)
    if out is None:
        rvec = torch.zeros((B, 3), dtype=torch.float64, device=dev)
        tvec = torch.zeros((B, 3), dtype=torch.float64, device=dev)
        ninl = torch.zeros((B,), dtype=torch.int32, device=dev)
        mask = torch.zeros((B, max(cap, 1)), dtype=torch.uint8, device=dev)
    else:
        rvec, tvec, ninl, mask = out
    if ws is None:
        ws = pnp_workspace(B, prm["n_hyp"], dev)
        if stream is not None and stream != torch.cuda.current_stream(dev):
            ws.record_stream(stream)  # freed by the caching allocator only after `stream`
    _lib.call("slam_pnp_ransac", ptr(Q), ptr(q), ptr(count), cap, B, ptr(Kt.contiguous()),
              int(seed) & ((1 << 64) - 1), int(item0), prm["n_hyp"], float(prm["reproj_thresh"]),
              prm["hyp_iters"], prm["refine_iters"], ptr(rvec), ptr(tvec), ptr(ninl), ptr(mask),
              ptr(ws), ws.numel(), stream_ptr(stream))
    return rvec, tvec, ninl, mask


def pnp_workspace(B, n_hyp=PNP_DEFAULTS["n_hyp"], dev="cuda"):
    """Hypothesis-pose workspace of slam_pnp_ransac for B items (f64)."""
    n = int(_lib.lib.slam_pnp_workspace_len(B, n_hyp))
    return torch.empty(max(n, 1), dtype=torch.float64, device=dev)


VO_DEFAULTS = dict(max_iter=100, lm_iters=20, early_stop=5)


def vo_estimate_pose(q1, q2, Q1, Q2, count, P, seed=0, item0=0, out=None, stream=None, **kw):
    """visual_odometry.py:135-157 batched: q1, q2 [B,cap,2], Q1, Q2 [B,cap,3] f64,
    P 3x4 -> (pose [B,6] (rotvec, t), best [B], ntried [B], err [B])."""
    prm = dict(VO_DEFAULTS, **kw)
    B, cap, _ = Q1.shape
    dev = Q1.device
    Pt = P if isinstance(P, torch.Tensor) else torch.as_tensor(np.asarray(P, np.float64), device=dev)
    if out is None:
        pose = torch.zeros((B, 6), dtype=torch.float64, device=dev)
        best = torch.zeros((B,), dtype=torch.int32, device=dev)
        ntried = torch.zeros((B,), dtype=torch.int32, device=dev)
        err = torch.zeros((B,), dtype=torch.float64, device=dev)
    else:
        pose, best, ntried, err = out
    nb = ctypes.c_size_t(0)
    _lib.call("slam_vo_pose_workspace_bytes", B, prm["max_iter"], ctypes.byref(nb))
    ws = torch.empty(nb.value, dtype=torch.uint8, device=dev)
    _lib.call("slam_vo_estimate_pose", ptr(q1), ptr(q2), ptr(Q1), ptr(Q2), ptr(count), cap, B,
              ptr(Pt.contiguous()), int(seed) & ((1 << 64) - 1), int(item0), prm["max_iter"],
              prm["lm_iters"], prm["early_stop"], ptr(pose), ptr(best), ptr(ntried), ptr(err),
              ptr(ws), nb.value, stream_ptr(stream))
    return pose, best, ntried, err


def vo_residuals(dof, q1, q2, Q1, Q2, count, P, out=None, stream=None):
    """visual_odometry.py:65-81 batched: dof [B,6] -> f [B, 4 cap] (first 4 count[b] valid)."""
    B, cap, _ = Q1.shape
    dev = Q1.device
    Pt = P if isinstance(P, torch.Tensor) else torch.as_tensor(np.asarray(P, np.float64), device=dev)
    f = out if out is not None else torch.zeros((B, 4 * max(cap, 1)), dtype=torch.float64,
                                                device=dev)
    _lib.call("slam_vo_residuals", ptr(dof), ptr(q1), ptr(q2), ptr(Q1), ptr(Q2), ptr(count), cap,
              B, ptr(Pt.contiguous()), ptr(f), stream_ptr(stream))
    return f

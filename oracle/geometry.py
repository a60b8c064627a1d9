"""ORACLE (test infrastructure only): triangulation, pose and PnP on the CPU.

  triangulate_points_local  /root/reference/Point3D.py:14-19 (cv2.triangulatePoints:
                            per point, rows x*P[2]-P[0], y*P[2]-P[1] of both views,
                            null vector = last row of V^T of the 4x4 SVD; X = v[:3]/v[3])
  relative_to_abs3DPoints   Point3D.py:22-30
  sort_3D_points            Point3D.py:5-10
  rodrigues / form_transf / calculate_transformation_matrix
                            transformation.py:5-37 (incl. the r, t sign flip)
  pnp_ransac                oracle/geometry.c (seeded RANSAC + LM spec)
  vo_residuals / vo_estimate_pose
                            visual_odometry.py:65-81, 135-157 -> oracle/vo.c
                            (seeded 6-point samples + analytic-Jacobian LM spec)
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _ptr, lib


def triangulate_points_local(qs_l, qs_r, P_l, P_r):
    ql = np.asarray(qs_l, np.float64).reshape(-1, 2)
    qr = np.asarray(qs_r, np.float64).reshape(-1, 2)
    M = len(ql)
    A = np.empty((M, 4, 4))
    for j, (q, P) in enumerate(((ql, np.asarray(P_l, float)), (qr, np.asarray(P_r, float)))):
        A[:, 2 * j] = q[:, 0:1] * P[2][None] - P[0][None]
        A[:, 2 * j + 1] = q[:, 1:2] * P[2][None] - P[1][None]
    if M == 0:
        return np.zeros((0, 3))
    _, _, Vt = np.linalg.svd(A)
    h = Vt[:, -1, :]
    return h[:, :3] / h[:, 3:4]


def relative_to_abs3DPoints(points3D, camera_frame):
    P = np.asarray(points3D, float).reshape(-1, 3)
    hom = np.hstack((P, np.ones((len(P), 1))))
    a = np.matmul(camera_frame, hom.T)
    return (a[:3] / a[3]).T


def sort_3D_points(pts, close_def_in_m=100, far_def_in_m=1):
    close = [(abs(x[0]) < close_def_in_m and abs(x[1]) < close_def_in_m and abs(x[2]) < close_def_in_m)
             for x in pts]
    far = [(abs(x[0]) > far_def_in_m or abs(x[1]) > far_def_in_m or abs(x[2]) > far_def_in_m)
           for x in pts]
    return close, far


def rodrigues(r):
    r = np.asarray(r, float).ravel()
    th = np.linalg.norm(r)
    if th < np.finfo(float).eps:
        return np.eye(3)
    k = r / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.cos(th) * np.eye(3) + (1 - np.cos(th)) * np.outer(k, k) + np.sin(th) * K


def form_transf(R, t):
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = np.asarray(t).ravel()
    return T


def pose_matrix_from_pnp(rvec, tvec):
    """transformation.py:15-19: r <- -r, t <- -t, T = [Rodrigues(-r) | -t]."""
    r = -1 * np.asarray(rvec, float).reshape(3, 1)
    t = -1 * np.asarray(tvec, float).reshape(3, 1)
    return form_transf(rodrigues(r), t.T), r, t


_PNP = None
_FM = None


def _fm_fn():
    global _FM
    if _FM is None:
        f = lib().oracle_fm_lmeds
        p, i = ctypes.c_void_p, ctypes.c_int
        f.argtypes = [p, p, i, ctypes.c_uint64, i, i, p, p, p]
        f.restype = ctypes.c_int
        _FM = f
    return _FM


def fundamental_lmeds(m1, m2, seed=0, item=0, n_hyp=300):
    """Seeded LMedS F (oracle/fundamental.c) -> (mask [M] bool, F 3x3, n_inliers, median)."""
    m1 = np.ascontiguousarray(m1, np.float64).reshape(-1, 2)
    m2 = np.ascontiguousarray(m2, np.float64).reshape(-1, 2)
    M = len(m1)
    mask = np.zeros(max(M, 1), np.uint8)
    F = np.zeros(9)
    med = np.zeros(1, np.float32)
    n = _fm_fn()(_ptr(m1), _ptr(m2), M, seed & ((1 << 64) - 1), item, n_hyp, _ptr(mask), _ptr(F),
                 _ptr(med))
    return mask[:M].astype(bool), F.reshape(3, 3), n, float(med[0])


def _pnp_fn():
    global _PNP
    if _PNP is None:
        f = lib().oracle_pnp_ransac
        p, i, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
        f.argtypes = [p, p, i, p, ctypes.c_uint64, i, i, d, i, i, p, p, p, p, p]
        f.restype = ctypes.c_int
        _PNP = f
    return _PNP


def pnp_ransac(Q, q, K, seed=0, item=0, n_hyp=100, thresh=8.0, hyp_iters=10, refine_iters=20,
               return_hypotheses=False):
    Q = np.ascontiguousarray(Q, np.float64).reshape(-1, 3)
    q = np.ascontiguousarray(q, np.float64).reshape(-1, 2)
    K = np.ascontiguousarray(K, np.float64).reshape(3, 3)
    L = len(Q)
    rvec = np.zeros(3)
    tvec = np.zeros(3)
    mask = np.zeros(max(L, 1), np.uint8)
    hyp = np.zeros((n_hyp, 6))
    hc = np.zeros(n_hyp, np.int32)
    n = _pnp_fn()(_ptr(Q), _ptr(q), L, _ptr(K), seed & ((1 << 64) - 1), item, n_hyp, thresh,
                  hyp_iters, refine_iters, _ptr(rvec), _ptr(tvec), _ptr(mask), _ptr(hyp), _ptr(hc))
    out = (rvec, tvec, n, mask[:L].astype(bool))
    return out + (hyp, hc) if return_hypotheses else out


def epnp(pw, uv, K):
    """EPnP (oracle/epnp.h) on 4..8 points -> (rvec, t) as one array [6], or None."""
    pw = np.ascontiguousarray(pw, np.float64).reshape(-1, 3)
    uv = np.ascontiguousarray(uv, np.float64).reshape(-1, 2)
    K = np.ascontiguousarray(K, np.float64).reshape(3, 3)
    f = lib().oracle_epnp
    f.argtypes = [ctypes.c_void_p] * 2 + [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    f.restype = ctypes.c_int
    p = np.zeros(6)
    return p if f(_ptr(pw), _ptr(uv), len(pw), _ptr(K), _ptr(p)) else None


_VO = None


def _vo_fns():
    global _VO
    if _VO is None:
        L = lib()
        p, i, u = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64
        L.oracle_vo_residuals.argtypes = [p, p, p, p, p, i, p, p]
        L.oracle_vo_residuals.restype = None
        L.oracle_vo_hypothesis.argtypes = [p, p, p, p, i, p, u, i, i, i, p, p]
        L.oracle_vo_hypothesis.restype = None
        L.oracle_vo_estimate_pose.argtypes = [p, p, p, p, i, p, u, i, i, i, i, p, p, p, p]
        L.oracle_vo_estimate_pose.restype = ctypes.c_int
        _VO = L
    return _VO


def _vo_in(q1, q2, Q1, Q2, P):
    return (np.ascontiguousarray(q1, np.float64).reshape(-1, 2),
            np.ascontiguousarray(q2, np.float64).reshape(-1, 2),
            np.ascontiguousarray(Q1, np.float64).reshape(-1, 3),
            np.ascontiguousarray(Q2, np.float64).reshape(-1, 3),
            np.ascontiguousarray(P, np.float64).reshape(3, 4))


def vo_residuals(dof, q1, q2, Q1, Q2, P):
    """reprojection_residuals (visual_odometry.py:65-81): flat (4N,)."""
    q1, q2, Q1, Q2, P = _vo_in(q1, q2, Q1, Q2, P)
    N = len(q1)
    f = np.zeros(max(4 * N, 1))
    d = np.ascontiguousarray(dof, np.float64).reshape(6)
    _vo_fns().oracle_vo_residuals(_ptr(d), _ptr(q1), _ptr(q2), _ptr(Q1), _ptr(Q2), N, _ptr(P), _ptr(f))
    return f[:4 * N]


def vo_hypothesis(q1, q2, Q1, Q2, P, seed=0, item=0, h=0, lm_iters=20):
    """One hypothesis of estimate_pose: (dof after LM, its 6 sample indices)."""
    q1, q2, Q1, Q2, P = _vo_in(q1, q2, Q1, Q2, P)
    dof = np.zeros(6)
    idx = np.zeros(6, np.int32)
    _vo_fns().oracle_vo_hypothesis(_ptr(q1), _ptr(q2), _ptr(Q1), _ptr(Q2), len(q1), _ptr(P),
                                   seed & ((1 << 64) - 1), item, h, lm_iters, _ptr(dof), _ptr(idx))
    return dof, idx


def vo_estimate_pose(q1, q2, Q1, Q2, P, seed=0, item=0, max_iter=100, lm_iters=20, early_stop=5):
    """estimate_pose (visual_odometry.py:135-157) -> (dof, best, ntried, error, errs[max_iter])."""
    q1, q2, Q1, Q2, P = _vo_in(q1, q2, Q1, Q2, P)
    dof = np.zeros(6)
    nt = ctypes.c_int(0)
    err = ctypes.c_double(0.0)
    errs = np.zeros(max_iter)
    best = _vo_fns().oracle_vo_estimate_pose(
        _ptr(q1), _ptr(q2), _ptr(Q1), _ptr(Q2), len(q1), _ptr(P), seed & ((1 << 64) - 1), item,
        max_iter, lm_iters, early_stop, _ptr(dof), ctypes.byref(nt), ctypes.byref(err), _ptr(errs))
    return dof, best, nt.value, err.value, errs

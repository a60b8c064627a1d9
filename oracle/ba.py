"""ORACLE (test infrastructure only): BAL bundle adjustment on the CPU.

Restates the reference's BAL reprojection block (a string literal in
/root/reference/BundleAdjustment.py:230-466, pinned by tests/golden/ba_golden.npz):
  rotate       BundleAdjustment.py:287-298
  project      BundleAdjustment.py:317-328
  objective    BundleAdjustment.py:331-369 (incl. the two >5000 px clamps)
  sparsity     BundleAdjustment.py:380-394
plus the analytic per-observation Jacobian of `objective` and the
Levenberg-Marquardt / Schur-complement algorithm the GPU runs (the reference
calls scipy least_squares TRF at :397-402; both reach the same optimum, see
DESIGN.md §BA).
"""
from __future__ import annotations

import numpy as np

CLAMP = 5000.0
CLAMP_X = 613.0 * 2   # BundleAdjustment.py:343
CLAMP_Y = 185.0 * 2   # BundleAdjustment.py:350


def rotate(Qs, rot_vecs):
    """Rodrigues rotation of points by per-row rotation vectors (:287-298)."""
    theta = np.linalg.norm(rot_vecs, axis=1)[:, np.newaxis]
    with np.errstate(invalid="ignore", divide="ignore"):
        v = np.nan_to_num(rot_vecs / theta)
    dot = np.sum(Qs * v, axis=1)[:, np.newaxis]
    c, s = np.cos(theta), np.sin(theta)
    return c * Qs + s * np.cross(v, Qs) + dot * (1 - c) * v


def project(Qs, cam_params):
    """BAL projection, camera looking down -z, radial k1/k2 (:317-328)."""
    P = rotate(Qs, cam_params[:, :3]) + cam_params[:, 3:6]
    p = -P[:, :2] / P[:, 2, np.newaxis]
    f, k1, k2 = cam_params[:, 6:].T
    n = np.sum(p ** 2, axis=1)
    r = 1 + k1 * n + k2 * n ** 2
    return p * (r * f)[:, np.newaxis]


def clamp_rows(res):
    """The two outlier clamps of :339-350, in order (second sees the first)."""
    res = np.array(res, dtype=np.float64, copy=True)
    i0 = np.unique(np.where(np.abs(res[:, 0]) > CLAMP))
    res[i0] = res[i0] / np.abs(res[i0][:, 0][:, None]) * 613 * 2
    i1 = np.unique(np.where(np.abs(res[:, 1]) > CLAMP))
    res[i1] = res[i1] / np.abs(res[i1][:, 1][:, None]) * 185 * 2
    return res


def objective(params, n_cams, n_Qs, cam_idxs, Q_idxs, qs):
    """Residual vector [x0, y0, x1, y1, ...] (:331-369, without the print)."""
    cams = params[: n_cams * 9].reshape((n_cams, 9))
    Qs = params[n_cams * 9:].reshape((n_Qs, 3))
    res = project(Qs[Q_idxs], cams[cam_idxs]) - qs
    return clamp_rows(res).ravel()


def sparsity_coo(n_cams, n_Qs, cam_idxs, Q_idxs):
    """Row/col indices of the ones of bundle_adjustment_sparsity (:380-394), row-major."""
    cam_idxs = np.asarray(cam_idxs, np.int64)
    Q_idxs = np.asarray(Q_idxs, np.int64)
    O = len(cam_idxs)
    cols = np.concatenate([cam_idxs[:, None] * 9 + np.arange(9)[None, :],
                           n_cams * 9 + Q_idxs[:, None] * 3 + np.arange(3)[None, :]], 1)
    rows = np.repeat(np.arange(2 * O), 12)
    cols = np.repeat(cols, 2, axis=0).ravel()
    order = np.lexsort((cols, rows))
    return rows[order], cols[order], (2 * O, n_cams * 9 + n_Qs * 3)


# ----------------------------------------------------------------------------- Jacobian
def _skew(a):
    z = np.zeros(len(a))
    return np.stack([np.stack([z, -a[:, 2], a[:, 1]], 1),
                     np.stack([a[:, 2], z, -a[:, 0]], 1),
                     np.stack([-a[:, 1], a[:, 0], z], 1)], 1)


def rotation_matrices(w):
    th = np.linalg.norm(w, axis=1)
    with np.errstate(invalid="ignore", divide="ignore"):
        v = np.nan_to_num(w / th[:, None])
    K = _skew(v)
    c, s = np.cos(th)[:, None, None], np.sin(th)[:, None, None]
    return c * np.eye(3)[None] + s * K + (1 - c) * v[:, :, None] * v[:, None, :]


def jacobian(cams, X):
    """Per-observation residual and analytic Jacobian of the UNCLAMPED projection.

    cams [O,9], X [O,3] -> (proj [O,2], J [O,2,12]) with columns
    [w0 w1 w2 t0 t1 t2 f k1 k2 | X0 X1 X2].  d(RX)/dw follows Gallego & Yezzi
    (2015): -R [X]x (w w^T + (R^T - I)[w]x) / |w|^2, and -[X]x at w = 0.
    """
    w, t, f, k1, k2 = cams[:, :3], cams[:, 3:6], cams[:, 6], cams[:, 7], cams[:, 8]
    R = rotation_matrices(w)
    P = np.einsum("oij,oj->oi", R, X) + t
    th2 = np.sum(w * w, axis=1)
    RX = P - t
    Wx = _skew(w)
    dRdw = np.empty((len(X), 3, 3))
    small = th2 < 1e-24
    A = (w[:, :, None] * w[:, None, :] + np.einsum("oji,ojk->oik", R, Wx) - Wx)
    with np.errstate(invalid="ignore", divide="ignore"):
        dRdw[:] = -np.einsum("oij,ojk,okl->oil", R, _skew(X), A) / th2[:, None, None]
    dRdw[small] = -_skew(RX[small])
    p = -P[:, :2] / P[:, 2:3]
    n = np.sum(p * p, axis=1)
    rad = 1 + k1 * n + k2 * n * n
    s = rad * f
    dp_dP = np.zeros((len(X), 2, 3))
    dp_dP[:, 0, 0] = -1 / P[:, 2]
    dp_dP[:, 1, 1] = -1 / P[:, 2]
    dp_dP[:, :, 2] = P[:, :2] / (P[:, 2:3] ** 2)
    dproj_dp = s[:, None, None] * np.eye(2)[None] + \
        (2 * f * (k1 + 2 * k2 * n))[:, None, None] * p[:, :, None] * p[:, None, :]
    D = np.einsum("oij,ojk->oik", dproj_dp, dp_dP)
    J = np.empty((len(X), 2, 12))
    J[:, :, 0:3] = np.einsum("oij,ojk->oik", D, dRdw)
    J[:, :, 3:6] = D
    J[:, :, 6] = p * rad[:, None]
    J[:, :, 7] = p * (f * n)[:, None]
    J[:, :, 8] = p * (f * n * n)[:, None]
    J[:, :, 9:12] = np.einsum("oij,ojk->oik", D, R)
    return p * s[:, None], J


def clamp_with_jacobian(res, J):
    """Apply the :339-350 clamps to residual rows and their Jacobians (chain rule)."""
    res = res.copy()
    J = J.copy()
    for comp, scale in ((0, CLAMP_X), (1, CLAMP_Y)):
        m = np.abs(res[:, comp]) > CLAMP
        if not m.any():
            continue
        rc = res[m, comp]
        a = scale / np.abs(rc)
        Jc = J[m, comp, :]
        J[m] = a[:, None, None] * (J[m] - (res[m] / rc[:, None])[:, :, None] * Jc[:, None, :])
        res[m] = res[m] * a[:, None]
    return res, J


def residual_and_jacobian(cams, pts, cam_idx, pt_idx, qs):
    proj, J = jacobian(cams[cam_idx], pts[pt_idx])
    return clamp_with_jacobian(proj - qs, J)


# ----------------------------------------------------------------------------- LM
class LMState:
    def __init__(self, lam=1e-4):
        self.lam = lam
        self.nu = 2.0


DIAG_MIN, DIAG_MAX = 1e-6, 1e32
LAM_MIN, LAM_MAX = 1e-16, 1e32


def normal_equations(cams, pts, cam_idx, pt_idx, qs):
    """Dense J^T J and g = -J^T r in parameter order [cams.ravel(), pts.ravel()]."""
    C, P = len(cams), len(pts)
    r, J = residual_and_jacobian(cams, pts, cam_idx, pt_idx, qs)
    n = 9 * C + 3 * P
    Jd = np.zeros((2 * len(cam_idx), n))
    rows = np.arange(len(cam_idx))
    for q in range(2):
        Jd[(2 * rows + q)[:, None], (cam_idx * 9)[:, None] + np.arange(9)] = J[:, q, :9]
        Jd[(2 * rows + q)[:, None], (9 * C + pt_idx * 3)[:, None] + np.arange(3)] = J[:, q, 9:]
    rv = r.ravel()
    return Jd.T @ Jd, -Jd.T @ rv, 0.5 * float(rv @ rv)


def lm_iteration(cams, pts, cam_idx, pt_idx, qs, st: LMState):
    """One LM iteration exactly as the GPU runs it (dense solve; the GPU uses the
    Schur complement, identical up to round-off).  Returns new (cams, pts, info)."""
    H, g, cost = normal_equations(cams, pts, cam_idx, pt_idx, qs)
    D = np.clip(np.diag(H), DIAG_MIN, DIAG_MAX)
    Hd = H + st.lam * np.diag(D)
    delta = np.linalg.solve(Hd, g)
    C = len(cams)
    cams_n = cams + delta[: 9 * C].reshape(C, 9)
    pts_n = pts + delta[9 * C:].reshape(-1, 3)
    r = residual_and_jacobian(cams_n, pts_n, cam_idx, pt_idx, qs)[0]
    cost_new = 0.5 * float(np.sum(r * r))
    pred = 0.5 * float(delta @ (st.lam * D * delta + g))
    rho = (cost - cost_new) / pred if pred > 0 else -1.0
    accepted = rho > 0
    if accepted:
        st.lam = min(max(st.lam * max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3), LAM_MIN), LAM_MAX)
        st.nu = 2.0
        cams, pts = cams_n, pts_n
    else:
        st.lam = min(st.lam * st.nu, LAM_MAX)
        st.nu *= 2.0
    return cams, pts, dict(cost=cost, cost_new=cost_new, pred=pred, rho=rho, accepted=accepted)


def lm_solve(cams, pts, cam_idx, pt_idx, qs, iters=50, lam0=1e-4):
    st = LMState(lam0)
    hist = []
    for _ in range(iters):
        cams, pts, info = lm_iteration(cams, pts, cam_idx, pt_idx, qs, st)
        hist.append(info)
    return cams, pts, hist


def sim3_align(A, B):
    """Umeyama: s, R, t minimising |s R A + t - B| over rows of A, B [n,3]."""
    mA, mB = A.mean(0), B.mean(0)
    a, b = A - mA, B - mB
    U, S, Vt = np.linalg.svd(b.T @ a / len(A))
    d = np.sign(np.linalg.det(U @ Vt))
    Dm = np.diag([1, 1, d])
    R = U @ Dm @ Vt
    s = np.trace(np.diag(S) @ Dm) / (a * a).sum(1).mean()
    return s, R, mB - s * R @ mA


def camera_centers(cams):
    R = rotation_matrices(cams[:, :3])
    return -np.einsum("oji,oj->oi", R, cams[:, 3:6])


# ----------------------------------------------------------------------------- LM (Schur)
def _obs_pairs(cam_idx, pt_idx):
    """All ordered observation pairs (o1, o2) of the same point with cam1 <= cam2."""
    order = np.lexsort((cam_idx, pt_idx))
    pts = pt_idx[order]
    starts = np.flatnonzero(np.r_[True, pts[1:] != pts[:-1]])
    counts = np.diff(np.r_[starts, len(pts)])
    o1s, o2s = [], []
    for n in np.unique(counts):
        s = starts[counts == n]
        a = (s[:, None, None] + np.arange(n)[None, :, None]).repeat(n, 2).reshape(len(s), -1)
        b = (s[:, None, None] + np.arange(n)[None, None, :]).repeat(n, 1).reshape(len(s), -1)
        a, b = order[a], order[b]
        keep = cam_idx[a] <= cam_idx[b]
        o1s.append(a[keep])
        o2s.append(b[keep])
    return np.concatenate(o1s), np.concatenate(o2s)


def lm_iteration_schur(cams, pts, cam_idx, pt_idx, qs, st: LMState, pairs=None):
    """The same LM iteration as lm_iteration, solved through the point-block
    Schur complement (vectorised numpy; scales to the C3/C4 problems)."""
    C, P = len(cams), len(pts)
    cam_idx = np.asarray(cam_idx)
    pt_idx = np.asarray(pt_idx)
    r, J = residual_and_jacobian(cams, pts, cam_idx, pt_idx, qs)
    cost = 0.5 * float(np.sum(r * r))
    Jc, Jp = J[:, :, :9], J[:, :, 9:]
    U = np.zeros((C, 9, 9))
    np.add.at(U, cam_idx, np.einsum("oai,oaj->oij", Jc, Jc))
    V = np.zeros((P, 3, 3))
    np.add.at(V, pt_idx, np.einsum("oai,oaj->oij", Jp, Jp))
    gc = np.zeros((C, 9))
    np.add.at(gc, cam_idx, -np.einsum("oai,oa->oi", Jc, r))
    gp = np.zeros((P, 3))
    np.add.at(gp, pt_idx, -np.einsum("oai,oa->oi", Jp, r))
    Dc = np.clip(np.diagonal(U, axis1=1, axis2=2), DIAG_MIN, DIAG_MAX)
    Dp = np.clip(np.diagonal(V, axis1=1, axis2=2), DIAG_MIN, DIAG_MAX)
    Vs = V + st.lam * Dp[:, :, None] * np.eye(3)[None]
    Vi = np.linalg.inv(Vs)
    W = np.einsum("oai,oaj->oij", Jc, Jp)
    Y = np.einsum("oij,ojk->oik", W, Vi[pt_idx])
    e = np.einsum("pij,pj->pi", Vi, gp)
    if pairs is None:
        pairs = _obs_pairs(cam_idx, pt_idx)
    o1, o2 = pairs
    S = np.zeros((C, C, 9, 9))
    blk = np.einsum("oik,ojk->oij", Y[o1], W[o2])
    np.add.at(S, (cam_idx[o1], cam_idx[o2]), -blk)
    same = cam_idx[o1] == cam_idx[o2]
    S = S + np.transpose(S, (1, 0, 3, 2)) * (1 - np.eye(C))[:, :, None, None]
    del same
    S[np.arange(C), np.arange(C)] += U + st.lam * Dc[:, :, None] * np.eye(9)[None]
    Sd = S.transpose(0, 2, 1, 3).reshape(9 * C, 9 * C)
    b = gc.copy()
    np.add.at(b, cam_idx, -np.einsum("oij,oj->oi", Y, gp[pt_idx]))
    dc = np.linalg.solve(Sd, b.ravel()).reshape(C, 9)
    dp = e.copy()
    np.add.at(dp, pt_idx, -np.einsum("oji,oj->oi", Y, dc[cam_idx]))
    cams_n, pts_n = cams + dc, pts + dp
    rn = residual_and_jacobian(cams_n, pts_n, cam_idx, pt_idx, qs)[0]
    cost_new = 0.5 * float(np.sum(rn * rn))
    pred = 0.5 * (float(np.sum(dc * (st.lam * Dc * dc + gc))) +
                  float(np.sum(dp * (st.lam * Dp * dp + gp))))
    rho = (cost - cost_new) / pred if pred > 0 else -1.0
    accepted = rho > 0 and np.isfinite(cost_new)
    if accepted:
        st.lam = min(max(st.lam * max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3), LAM_MIN), LAM_MAX)
        st.nu = 2.0
        cams, pts = cams_n, pts_n
    else:
        st.lam = min(st.lam * st.nu, LAM_MAX)
        st.nu *= 2.0
    return cams, pts, dict(cost=cost, cost_new=cost_new, pred=pred, rho=rho, accepted=accepted)

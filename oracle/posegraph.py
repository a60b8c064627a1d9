"""ORACLE (test infrastructure only; imported by tests/, smoke() and bench.py's
cpu_baseline leg, never by the product path): NumPy restatement of the live
pose-chain optimisation of /root/reference/BundleAdjustment.py:79-183 and of
the loop-closure helpers of /root/reference/loop_closure.py:39-52.

Pinned by tests/golden/posegraph_golden.npz (the reference's own functions run
with a stub cv2 whose Rodrigues is OpenCV's published formula; see
tests/golden/make_posegraph_goldens.py).  The Levenberg iteration below is the
algorithm the GPU kernel k_chain_lm runs (the reference runs scipy TRF), used
to check its iterates.
"""
from __future__ import annotations

import numpy as np

W = np.array([0.5, 0.05, 1.0, 1.0, 1.0, 0.0005])  # BundleAdjustment.py:114-119


def rodrigues_cv(r):
    """cv2.Rodrigues vector -> matrix (cvRodrigues2)."""
    r = np.asarray(r, np.float64).reshape(3)
    th = float(np.sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]))
    if th < np.finfo(np.float64).eps:
        return np.eye(3)
    c, s = np.cos(th), np.sin(th)
    k = r * (1.0 / th)
    rx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return c * np.eye(3) + (1 - c) * np.outer(k, k) + s * rx


def rel_pose(p):
    """translation_and_rotation_vector_to_matrix (transformation.py:23-37)."""
    T = np.eye(4)
    T[:3, :3] = rodrigues_cv(p[:3])
    T[:3, 3] = p[3:6]
    return T


def frame_costs(x):
    """objective_without_loop_closure (BundleAdjustment.py:79-105)."""
    p = np.reshape(x, (-1, 6))
    c = np.abs(p[:, 0]) * W[0]
    c += np.abs(p[:, 1]) * W[1]
    c += np.abs(p[:, 2]) * W[2]
    c += np.abs(p[:, 3]) * W[3]
    c += np.abs(p[:, 4]) * W[4]
    c += (np.abs(p[:, 5]) - 1) * W[5]
    return c


def chain(x):
    """abs_m = Rel_0 @ ... @ Rel_{m-1} in the reference's order (:128-131)."""
    T = np.eye(4)
    for p in np.reshape(x, (-1, 6)):
        T = T @ rel_pose(p)
    return T


def objective(x):
    """BundleAdjustment.py:107-145: m frame costs + translation and rotation
    loop-closure residuals."""
    T = chain(x)
    lt = np.sum(np.abs(np.subtract(np.zeros(3), T[0:3, 3]))) * 1000
    lr = np.sum(np.abs(np.subtract(100 * np.eye(3), 100 * T[0:3, 0:3]))) * 1000
    return np.hstack((frame_costs(x), lt, lr))


def sparsity(m, loop=True):
    """bundle_adjustment_sparsity(_without_loop_closure) (:147-171) as a dense
    0/1 array."""
    A = np.zeros((m + (2 if loop else 0), 6 * m), int)
    for i in range(m):
        A[i, 6 * i:6 * i + 6] = 1
    if loop:
        A[m:] = 1
    return A


# ----------------------------------------------------------------------------- Levenberg
def _drodrigues(r, R):
    th2 = float(r @ r)
    out = np.empty((3, 3, 3))
    for k in range(3):
        e = np.zeros(3)
        e[k] = 1.0
        if th2 < 1e-30:
            out[k] = np.array([[0, -e[2], e[1]], [e[2], 0, -e[0]], [-e[1], e[0], 0]])
            continue
        v = np.cross(r, (np.eye(3) - R) @ e)
        a = r[k] * r + v
        S = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
        out[k] = S @ R / th2
    return out


def jacobian(x, loop=True):
    """Analytic (sign-subgradient) Jacobian [m (+2), 6m] of objective."""
    p = np.reshape(x, (-1, 6))
    m = len(p)
    J = np.zeros((m + (2 if loop else 0), 6 * m))
    for i in range(m):
        J[i, 6 * i:6 * i + 6] = W * np.sign(p[i])
    if not loop:
        return J
    rels = [rel_pose(q) for q in p]
    pre = [np.eye(4)]
    for T in rels:
        pre.append(pre[-1] @ T)
    suf = [np.eye(4)]
    for T in rels[::-1]:
        suf.append(T @ suf[-1])
    suf = suf[::-1]  # suf[i] = Rel_i .. Rel_{m-1}
    Tend = pre[-1]
    E1 = np.sign(Tend[:3, 3])
    E2 = np.sign(Tend[:3, :3] - np.eye(3))
    for i in range(m):
        P, S = pre[i], suf[i + 1]
        dR = _drodrigues(p[i, :3], rels[i][:3, :3])
        for k in range(3):
            J[m, 6 * i + k] = 1000 * E1 @ (P[:3, :3] @ dR[k] @ S[:3, 3])
            J[m + 1, 6 * i + k] = 1e5 * np.sum(E2 * (P[:3, :3] @ dR[k] @ S[:3, :3]))
            J[m, 6 * i + 3 + k] = 1000 * E1 @ P[:3, k]
    return J


class LMState:
    def __init__(self, lam):
        self.lam, self.nu = lam, 2.0


def lm_iteration(x, st: LMState, loop=True):
    """One Levenberg iteration as k_chain_lm runs it: delta = -J^T (J J^T +
    lam I)^-1 r, accept if the cost drops (rho > 0)."""
    r = objective(x) if loop else frame_costs(x)
    J = jacobian(x, loop)
    cost = 0.5 * float(r @ r)
    y = np.linalg.solve(J @ J.T + st.lam * np.eye(len(r)), r)
    d = -J.T @ y
    pred = cost - 0.5 * float(np.sum((r + J @ d) ** 2))
    xt = x + d
    rt = objective(xt) if loop else frame_costs(xt)
    cost_new = 0.5 * float(rt @ rt)
    rho = (cost - cost_new) / pred if pred > 0 else -1.0
    if rho > 0 and np.isfinite(cost_new):
        st.lam = min(max(st.lam * max(1 / 3, 1 - (2 * rho - 1) ** 3), 1e-16), 1e32)
        st.nu = 2.0
        return xt, dict(cost=cost, cost_new=cost_new, rho=rho, accepted=True)
    st.lam = min(st.lam * st.nu, 1e32)
    st.nu *= 2.0
    return x, dict(cost=cost, cost_new=cost_new, rho=rho, accepted=False)


def initial_lambda(x, rel0, loop=True):
    """Marquardt start of k_chain_lm: rel0 * max diag(J J^T) (frame rows and,
    with loop rows, their squared norms)."""
    J = jacobian(x, loop)
    return rel0 * max(float(np.max(np.sum(J * J, axis=1))), 1e-12)


# ----------------------------------------------------------------------------- loop closure
def find_error(correct_frame, wrong_frame):
    """loop_closure.py:39-40."""
    return correct_frame - wrong_frame


def get_distribution_error(error_frame, index_0, index_i):
    """loop_closure.py:43-44."""
    return error_frame / (index_i - index_0)


def distribute_error(poses, error_frame, index_0, index_i):
    """loop_closure.py:48-52 on an array of 4x4 poses (translation only)."""
    out = np.array(poses, np.float64, copy=True)
    for i in range(index_0, index_i):
        out[i, :3, 3] += (i - index_0) * error_frame[:3, 3]
    return out

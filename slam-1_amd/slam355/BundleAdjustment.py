"""Drop-in for the reference's BundleAdjustment module, running on the GPU
through libslam355.so.  The reference file holds two generations of the same
names: the live pose-chain optimisation (:16-225) and the BAL reprojection
block inside the string literal at :230-466.  Both are served here, told apart
by their signatures exactly as the two blocks define them.

Pose chain (live code; slam355.posegraph, csrc/posegraph.hip):
  load_data(file_name)                                          (:16)
  objective_without_loop_closure(car_params)                    (:79)
  objective(car_params)                                         (:107)
  bundle_adjustment_sparsity_without_loop_closure(car_params)   (:147)
  bundle_adjustment_sparsity(car_params)                        (:159)
  bundle_adjustment_with_sparsity_without_loop_closure(car_params, sparse_mat) (:173)
  bundle_adjustment_with_sparsity(car_params, sparse_mat)       (:179)
BAL reprojection BA (csrc/ba.hip):
  read_bal_data(file_name)                                   (:236)
  objective(params, n_cams, n_Qs, cam_idxs, Q_idxs, qs)      (:331)
  bundle_adjustment_sparsity(n_cams, n_Qs, cam_idxs, Q_idxs) (:380)
  bundle_adjustment(cam_params, Qs, cam_idxs, Q_idxs, qs)    (:372)
  bundle_adjustment_with_sparsity(..., sparse_mat)           (:397)
The BAL solver is Levenberg-Marquardt on the normal equations (Schur
complement, analytic Jacobian) instead of scipy's TRF with a finite-difference
Jacobian; it converges to the same optimum (tests/test_ba.py pins the cost
against the reference's own least_squares run).  The pose-chain solver is
scipy's TRF algorithm itself (x_scale='jac', ftol as the reference passes it)
with an analytic Jacobian and the exact trust-region subproblem
(tests/test_posegraph.py: never a worse cost than the reference's run).
"""
from __future__ import annotations

import numpy as np

from . import ba as _ba
from . import posegraph as _pg


def read_bal_data(file_name):
    """BAL text file -> (cam_params [C,9], Qs [P,3], cam_idxs, Q_idxs, qs [O,2])."""
    with open(file_name, "r") as f:
        n_cams, n_Qs, n_qs = map(int, f.readline().split())
        tok = f.read().split()
    obs = np.asarray(tok[: 4 * n_qs], dtype=float).reshape(n_qs, 4)
    rest = np.asarray(tok[4 * n_qs: 4 * n_qs + 9 * n_cams + 3 * n_Qs], dtype=float)
    cam_idxs = obs[:, 0].astype(int)
    Q_idxs = obs[:, 1].astype(int)
    qs = obs[:, 2:4].astype(float)
    cam_params = rest[: n_cams * 9].reshape((n_cams, -1))
    Qs = rest[n_cams * 9: n_cams * 9 + n_Qs * 3].reshape((n_Qs, -1))
    return cam_params, Qs, cam_idxs, Q_idxs, qs


def write_bal_data(file_name, cam_params, Qs, cam_idxs, Q_idxs, qs):
    """Inverse of read_bal_data (the layout export_data writes, XXXport_files.py:44-64)."""
    cam_params = np.asarray(cam_params, float).reshape(-1, 9)
    Qs = np.asarray(Qs, float).reshape(-1, 3)
    with open(file_name, "w") as f:
        f.write(f"{len(cam_params)} {len(Qs)} {len(qs)}\n")
        for c, p, (x, y) in zip(cam_idxs, Q_idxs, np.asarray(qs, float)):
            f.write(f"{int(c)} {int(p)} {float(x)!r} {float(y)!r}\n")
        for v in cam_params.ravel():
            f.write(f"{float(v)!r}\n")
        for v in Qs.ravel():
            f.write(f"{float(v)!r}\n")


# ----------------------------------------------------------------------------- pose chain
def load_data(file_name, number_of_frames=1100):
    """(:16-31) `number_of_frames` lines of 6 floats -> flat [6 * number_of_frames]."""
    out = np.empty((number_of_frames, 6))
    with open(file_name, "r") as f:
        for j in range(number_of_frames):
            out[j] = [float(v) for v in f.readline().split()[:6]]
    return out.ravel()


def objective_without_loop_closure(car_params):
    """(:79-105) per-frame weighted motion costs [m] (GPU k_chain_objective)."""
    return _pg.chain_objective(car_params, loop=False)


def _chain_sparsity(car_params, loop):
    from scipy.sparse import lil_matrix

    n = np.shape(car_params)[0]
    m = int(n / 6) + (2 if loop else 0)
    A = lil_matrix((m, n), dtype=int)
    i = np.arange(int(n / 6))
    for s_ in range(6):
        A[i, i * 6 + s_] = 1
    if loop:
        A[m - 2:, :] = 1
    return A


def bundle_adjustment_sparsity_without_loop_closure(car_params):
    """(:147-157) one row per frame over its 6 parameters."""
    return _chain_sparsity(car_params, loop=False)


def _chain_solve(car_params, sparse_mat, loop, ftol=1e-1):
    x0 = np.asarray(car_params, np.float64).ravel()
    n_res = x0.size // 6 + (2 if loop else 0)
    if sparse_mat is not None and tuple(sparse_mat.shape) != (n_res, x0.size):
        # scipy least_squares: "`jac_sparsity` has wrong shape."
        raise ValueError("`jac_sparsity` has wrong shape.")
    residual_init = _pg.chain_objective(x0, loop=loop)
    pc = _pg.PoseChain(x0, loop=loop)
    pc.solve(ftol=ftol)
    x = pc.params()
    return residual_init, _pg.chain_objective(x, loop=loop), x


def bundle_adjustment_with_sparsity_without_loop_closure(car_params, sparse_mat):
    """(:173-177): like the reference, this optimises `objective` (m + 2
    residuals, loop rows included) against the m-row pattern, so scipy's shape
    check raises ValueError; the same error is raised here."""
    return _chain_solve(car_params, sparse_mat, loop=True)


# ----------------------------------------------------------------------------- shared names
def objective(params, *bal_args):
    """objective(car_params) (:107, pose chain: m frame costs + 2 loop-closure
    residuals) or objective(params, n_cams, n_Qs, cam_idxs, Q_idxs, qs) (:331,
    BAL reprojection residuals)."""
    if not bal_args:
        return _pg.chain_objective(params, loop=True)
    return _bal_objective(params, *bal_args)


def bundle_adjustment_sparsity(*args):
    """bundle_adjustment_sparsity(car_params) (:159, pose chain) or
    bundle_adjustment_sparsity(n_cams, n_Qs, cam_idxs, Q_idxs) (:380, BAL)."""
    if len(args) == 1:
        return _chain_sparsity(args[0], loop=True)
    return _bal_sparsity(*args)


def bundle_adjustment_with_sparsity(*args):
    """bundle_adjustment_with_sparsity(car_params, sparse_mat) (:179, pose chain,
    ftol 0.1 as the reference) or (cam_params, Qs, cam_idxs, Q_idxs, qs,
    sparse_mat) (:397, BAL).  Both return (residual_init, res.fun, res.x)."""
    if len(args) == 2:
        return _chain_solve(args[0], args[1], loop=True)
    return _bal_with_sparsity(*args)


# ----------------------------------------------------------------------------- BAL block
def _bal_objective(params, n_cams, n_Qs, cam_idxs, Q_idxs, qs):
    """Residual vector [x0, y0, x1, y1, ...] (GPU kernel k_residual)."""
    params = np.asarray(params, np.float64)
    cams = params[: n_cams * 9].reshape((n_cams, 9))
    Qs = params[n_cams * 9:].reshape((n_Qs, 3))
    return _ba.residuals(cams, Qs, cam_idxs, Q_idxs, qs).ravel()


def _bal_sparsity(n_cams, n_Qs, cam_idxs, Q_idxs):
    """The 2x12-per-observation Jacobian pattern as a scipy lil_matrix of ints.

    Host-side index bookkeeping (the GPU solver derives the same structure
    itself, slam355/ba.py:plan)."""
    from scipy.sparse import coo_matrix

    cam_idxs = np.asarray(cam_idxs, np.int64)
    Q_idxs = np.asarray(Q_idxs, np.int64)
    O = cam_idxs.size
    m, n = O * 2, n_cams * 9 + n_Qs * 3
    cols = np.concatenate([cam_idxs[:, None] * 9 + np.arange(9)[None, :],
                           n_cams * 9 + Q_idxs[:, None] * 3 + np.arange(3)[None, :]], 1)
    rows = np.repeat(np.arange(m), 12)
    cols = np.repeat(cols, 2, axis=0).ravel()
    A = coo_matrix((np.ones(len(rows), dtype=int), (rows, cols)), shape=(m, n)).tocsr()
    # duplicate entries are summed by coo->csr; lil assignment in the reference sets 1
    return (A > 0).astype(int).tolil()


def _solve(cam_params, Qs, cam_idxs, Q_idxs, qs, max_iters=200, ftol=1e-12):
    cam_params = np.asarray(cam_params, np.float64).reshape(-1, 9)
    Qs = np.asarray(Qs, np.float64).reshape(-1, 3)
    prob = _ba.BAProblem(cam_params, Qs, cam_idxs, Q_idxs, qs)
    params0 = np.hstack((cam_params.ravel(), Qs.ravel()))
    residual_init = _bal_objective(params0, len(cam_params), len(Qs), cam_idxs, Q_idxs, qs)
    prob.solve(max_iters=max_iters, ftol=ftol)
    cams, pts = prob.params()
    x = np.hstack((cams.ravel(), pts.ravel()))
    fun = _bal_objective(x, len(cam_params), len(Qs), cam_idxs, Q_idxs, qs)
    return residual_init, fun, x


def bundle_adjustment(cam_params, Qs, cam_idxs, Q_idxs, qs):
    """(:372-377) -> (residual_init, res.fun, res.x)."""
    return _solve(cam_params, Qs, cam_idxs, Q_idxs, qs)


def _bal_with_sparsity(cam_params, Qs, cam_idxs, Q_idxs, qs, sparse_mat):
    """(:397-402) -> (residual_init, res.fun, res.x).  `sparse_mat` is checked
    for shape only: the GPU solver builds the same 2x12 block structure."""
    n = np.asarray(cam_params).size + np.asarray(Qs).size
    if sparse_mat is not None and tuple(sparse_mat.shape) != (2 * len(np.ravel(cam_idxs)), n):
        raise ValueError("sparse_mat shape does not match the problem")
    return _solve(cam_params, Qs, cam_idxs, Q_idxs, qs)

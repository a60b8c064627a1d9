"""Drop-in for the reference's BAL bundle-adjustment functions
(/root/reference/BundleAdjustment.py:236-402, the block inside the string
literal at :230-466), running on the GPU through libslam355.so.

Same names, argument meaning and return values:
  read_bal_data(file_name)                                   (:236)
  objective(params, n_cams, n_Qs, cam_idxs, Q_idxs, qs)      (:331)
  bundle_adjustment_sparsity(n_cams, n_Qs, cam_idxs, Q_idxs) (:380)
  bundle_adjustment(cam_params, Qs, cam_idxs, Q_idxs, qs)    (:372)
  bundle_adjustment_with_sparsity(..., sparse_mat)           (:397)
The solver is Levenberg-Marquardt on the normal equations (Schur complement,
analytic Jacobian) instead of scipy's TRF with a finite-difference Jacobian;
it converges to the same optimum (tests/test_ba.py pins the cost against the
reference's own least_squares run).
"""
from __future__ import annotations

import numpy as np

from . import ba as _ba


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


def objective(params, n_cams, n_Qs, cam_idxs, Q_idxs, qs):
    """Residual vector [x0, y0, x1, y1, ...] (GPU kernel k_residual)."""
    params = np.asarray(params, np.float64)
    cams = params[: n_cams * 9].reshape((n_cams, 9))
    Qs = params[n_cams * 9:].reshape((n_Qs, 3))
    return _ba.residuals(cams, Qs, cam_idxs, Q_idxs, qs).ravel()


def bundle_adjustment_sparsity(n_cams, n_Qs, cam_idxs, Q_idxs):
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
    residual_init = objective(params0, len(cam_params), len(Qs), cam_idxs, Q_idxs, qs)
    prob.solve(max_iters=max_iters, ftol=ftol)
    cams, pts = prob.params()
    x = np.hstack((cams.ravel(), pts.ravel()))
    fun = objective(x, len(cam_params), len(Qs), cam_idxs, Q_idxs, qs)
    return residual_init, fun, x


def bundle_adjustment(cam_params, Qs, cam_idxs, Q_idxs, qs):
    """(:372-377) -> (residual_init, res.fun, res.x)."""
    return _solve(cam_params, Qs, cam_idxs, Q_idxs, qs)


def bundle_adjustment_with_sparsity(cam_params, Qs, cam_idxs, Q_idxs, qs, sparse_mat):
    """(:397-402) -> (residual_init, res.fun, res.x).  `sparse_mat` is checked
    for shape only: the GPU solver builds the same 2x12 block structure."""
    n = np.asarray(cam_params).size + np.asarray(Qs).size
    if sparse_mat is not None and tuple(sparse_mat.shape) != (2 * len(np.ravel(cam_idxs)), n):
        raise ValueError("sparse_mat shape does not match the problem")
    return _solve(cam_params, Qs, cam_idxs, Q_idxs, qs)

"""Drop-in for the pose estimator of /root/reference/visual_odometry.py
(`reprojection_residuals` :65-81, `estimate_pose` :135-157), on the GPU.

The reference draws its 6-point samples from NumPy's global RNG and runs
scipy's MINPACK LM; this build draws them from a seeded splitmix64 stream
(`seed=`, `frame=` keywords) and runs LM with the analytic Jacobian, so the
selected hypothesis is reproducible (oracle/vo.c states the same spec).
"""
from __future__ import annotations

import numpy as np
import torch

from . import geometry
from .device import require_gpu, to_dev
from .transformation import form_transf, rodrigues


def _batch1(q1, q2, Q1, Q2):
    q1 = np.ascontiguousarray(q1, np.float64).reshape(-1, 2)
    q2 = np.ascontiguousarray(q2, np.float64).reshape(-1, 2)
    Q1 = np.ascontiguousarray(Q1, np.float64).reshape(-1, 3)
    Q2 = np.ascontiguousarray(Q2, np.float64).reshape(-1, 3)
    n = len(q1)
    if not (len(q2) == len(Q1) == len(Q2) == n):
        raise ValueError("q1, q2, Q1, Q2 must have the same number of points")
    pad = lambda a, w: a if n else np.zeros((1, w))  # noqa: E731
    dev = require_gpu()
    return (to_dev(pad(q1, 2)[None]), to_dev(pad(q2, 2)[None]), to_dev(pad(Q1, 3)[None]),
            to_dev(pad(Q2, 3)[None]), torch.tensor([n], dtype=torch.int32, device=dev), n)


def reprojection_residuals(dof, q1, q2, Q1, Q2, P_l):
    """(visual_odometry.py:65-81) flat (4N,) residuals
    [q1_pred - q1 (x row, y row), q2_pred - q2 (x row, y row)]."""
    tq1, tq2, tQ1, tQ2, cnt, n = _batch1(q1, q2, Q1, Q2)
    d = to_dev(np.asarray(dof, np.float64).reshape(1, 6))
    f = geometry.vo_residuals(d, tq1, tq2, tQ1, tQ2, cnt, np.asarray(P_l, np.float64))
    return f[0, :4 * n].cpu().numpy()


def estimate_pose(q1, q2, Q1, Q2, P_l, max_iter=100, seed=0, frame=0, return_info=False):
    """(visual_odometry.py:135-157) 4x4 T of the best 6-point LM hypothesis with
    the reference's early termination (5 non-improving draws)."""
    tq1, tq2, tQ1, tQ2, cnt, n = _batch1(q1, q2, Q1, Q2)
    pose, best, ntried, err = geometry.vo_estimate_pose(
        tq1, tq2, tQ1, tQ2, cnt, np.asarray(P_l, np.float64), seed=seed, item0=frame,
        max_iter=max_iter)
    p = pose[0].cpu().numpy()
    T = form_transf(rodrigues(p[:3]), p[3:])
    if return_info:
        return T, dict(dof=p, best=int(best[0]), ntried=int(ntried[0]), error=float(err[0]))
    return T

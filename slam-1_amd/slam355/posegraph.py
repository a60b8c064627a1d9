"""Pose-chain (loop-closure) optimisation on the GPU — host side of
csrc/posegraph.hip.

The reference's live bundle adjustment (/root/reference/BundleAdjustment.py:
79-225) optimises m relative poses [r0 r1 r2 t0 t1 t2] so that the weighted
per-frame motion costs stay small and the chained absolute pose closes the
loop (end pose = start pose), with scipy's TRF.  Here:
  chain_objective(params, loop)  batched objective / objective_without_loop_
                                 closure (one launch for any number of vectors)
  PoseChain                      device-resident TRF (x_scale='jac', exact
                                 trust-region subproblem, analytic Jacobian)
The drop-in names live in slam355.BundleAdjustment.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .device import ptr, require_gpu, stream_ptr

STATUS = {0: "max_nfev", 1: "gtol", 2: "ftol", 3: "xtol", 4: "ftol+xtol"}


def chain_objective(params, loop: bool = True) -> np.ndarray:
    """objective (loop=True: m + 2 residuals) or objective_without_loop_closure
    (m residuals) of one [6m] or a batch [B, 6m] of parameter vectors."""
    dev = require_gpu()
    p = np.asarray(params, np.float64)
    single = p.ndim == 1
    p = np.atleast_2d(p)
    if p.shape[1] % 6:
        raise ValueError("car_params must hold 6 values per frame")
    B, m = p.shape[0], p.shape[1] // 6
    nr = m + (2 if loop else 0)
    tp = torch.from_numpy(np.ascontiguousarray(p)).to(dev)
    out = torch.empty((B, nr), dtype=torch.float64, device=dev)
    _lib.call("slam_pose_chain_objective", ptr(tp), B, m, int(loop), ptr(out), stream_ptr())
    r = out.cpu().numpy()
    return r[0] if single else r


class PoseChain:
    """Device-resident TRF run over m relative poses (scipy least_squares
    method='trf', x_scale='jac' semantics: ftol / xtol / gtol tests, max_nfev,
    trust-radius rules, the 'exact' subproblem)."""

    def __init__(self, car_params, loop: bool = True, stream=None):
        dev = require_gpu()
        x = np.ascontiguousarray(np.asarray(car_params, np.float64).ravel())
        if x.size == 0 or x.size % 6:
            raise ValueError("car_params must hold 6 values per frame (and at least one frame)")
        self.m, self.loop, self.stream = x.size // 6, bool(loop), stream
        n = int(_lib.lib.slam_pose_chain_workspace_len(self.m))
        self.ws = torch.zeros(n, dtype=torch.float64, device=dev)
        self.ws[: x.size].copy_(torch.from_numpy(x))
        self.st = torch.zeros(16, dtype=torch.float64, device=dev)
        self._started = False

    def run(self, max_iter: int, ftol=1e-8, xtol=1e-8, gtol=1e-8, max_nfev=None):
        """Up to max_iter outer TRF iterations (resumes a previous run)."""
        max_nfev = 100 * 6 * self.m if max_nfev is None else int(max_nfev)
        _lib.call("slam_pose_chain_trf", ptr(self.ws), self.m, int(self.loop), int(max_iter),
                  int(not self._started), float(ftol), float(xtol), float(gtol), max_nfev,
                  ptr(self.st), stream_ptr(self.stream))
        self._started = True

    def solve(self, ftol=1e-8, xtol=1e-8, gtol=1e-8, max_nfev=None, chunk=64) -> dict:
        """Iterate until a termination test fires or max_nfev (host checks the
        status between chunks of `chunk` iterations)."""
        max_nfev = 100 * 6 * self.m if max_nfev is None else int(max_nfev)
        while True:
            self.run(chunk, ftol, xtol, gtol, max_nfev)
            s = self.state()
            if s["status"] != 0 or s["nfev"] >= max_nfev:
                return s

    def state(self) -> dict:
        s = self.st.cpu().numpy()
        return dict(cost0=float(s[0]), cost=float(s[1]), nfev=int(s[2]), njev=int(s[3]),
                    status=int(s[4]), message=STATUS[int(s[4])], Delta=float(s[5]),
                    alpha=float(s[6]), iterations=int(s[7]))

    def params(self) -> np.ndarray:
        return self.ws[: 6 * self.m].cpu().numpy().copy()

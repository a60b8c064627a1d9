"""ORACLE — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / CPU baseline.  The product path
(slam-1_amd/slam355) never imports it and has no CPU fallback.

Contents:
  * liboracle.so (C, gcc -ffp-contract=off): hamming.c, orb.c, ba.c
  * ba.py        numpy restatement of the BAL objective (BundleAdjustment.py:287-394)
  * geometry.py  numpy restatement of triangulation / PnP / pose chain
Every function cites the reference file:line it follows.  Pinning: see
tests/golden/make_goldens.py and DESIGN.md §Oracle.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lock = threading.Lock()
_lib = None

_p = ctypes.c_void_p
_i = ctypes.c_int
_d = ctypes.c_double

_SIGS = {
    "oracle_hamming_knn2": [_p, _i, _p, _i, _p, _p, _p],
    "oracle_hamming_knn2_batch": [_p, _p, _i, _p, _p, _i, _i, _p, _p, _p],
}


def build() -> str:
    """Compile liboracle.so with gcc (make -C oracle)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    with _lock:
        if _lib is None:
            srcs = [os.path.join(_HERE, f) for f in os.listdir(_HERE) if f.endswith((".c", ".h"))]
            stale = (not os.path.exists(LIB_PATH)) or any(
                os.path.getmtime(s) > os.path.getmtime(LIB_PATH) for s in srcs)
            if stale:
                build()
            l = ctypes.CDLL(LIB_PATH)
            for name, args in _SIGS.items():
                f = getattr(l, name)
                f.argtypes = args
                f.restype = None
            _lib = l
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def hamming_knn2(q: np.ndarray, t: np.ndarray):
    """Exact kNN-2 + ratio for one pair -> (idx2 [nq,2], dist2 [nq,2], good [nq] bool)."""
    q = np.ascontiguousarray(q, dtype=np.uint8).reshape(-1, 32)
    t = np.ascontiguousarray(t, dtype=np.uint8).reshape(-1, 32)
    nq, nt = len(q), len(t)
    idx2 = np.full((nq, 2), -1, np.int32)
    dist2 = np.full((nq, 2), -1, np.int32)
    good = np.zeros(nq, np.uint8)
    lib().oracle_hamming_knn2(_ptr(q), nq, _ptr(t), nt, _ptr(idx2), _ptr(dist2), _ptr(good))
    return idx2, dist2, good.astype(bool)


def hamming_knn2_batch(q: np.ndarray, nq: np.ndarray, t: np.ndarray, nt: np.ndarray):
    """Batched layout identical to slam_hamming_knn2 (rows >= nq left at -1/0)."""
    q = np.ascontiguousarray(q, dtype=np.uint8)
    t = np.ascontiguousarray(t, dtype=np.uint8)
    B, q_cap, _ = q.shape
    t_cap = t.shape[1]
    nq = np.ascontiguousarray(nq, dtype=np.int32)
    nt = np.ascontiguousarray(nt, dtype=np.int32)
    idx2 = np.full((B, q_cap, 2), -1, np.int32)
    dist2 = np.full((B, q_cap, 2), -1, np.int32)
    good = np.zeros((B, q_cap), np.uint8)
    lib().oracle_hamming_knn2_batch(_ptr(q), _ptr(nq), q_cap, _ptr(t), _ptr(nt), t_cap, B,
                                    _ptr(idx2), _ptr(dist2), _ptr(good))
    return idx2, dist2, good


def hamming_knn2_pylist(q: np.ndarray, t: np.ndarray):
    """Pure-Python/numpy restatement for small cases (cross-checks the C oracle).

    Sort each query's candidates by (distance, train index) — the order
    cv::BFMatcher returns — and take the first two (keypoint.py:87).
    """
    q = np.asarray(q, np.uint8).reshape(-1, 32)
    t = np.asarray(t, np.uint8).reshape(-1, 32)
    pop = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(axis=2) if len(t) else \
        np.zeros((len(q), 0), np.int64)
    out = []
    for i in range(len(q)):
        order = sorted(range(len(t)), key=lambda j: (int(pop[i, j]), j))[:2]
        out.append([(j, int(pop[i, j])) for j in order])
    return out

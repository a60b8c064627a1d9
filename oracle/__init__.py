"""ORACLE — CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / CPU baseline.  The product path
(slam-1_amd/slam355) never imports it and has no CPU fallback.

Contents:
  * liboracle.so (C, gcc -ffp-contract=off): hamming.c, orb.c, geometry.c (PnP), fundamental.c
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
    "oracle_orb_level_sizes": [_i, _i, _p, _p, _p],
    "oracle_orb_level_budget": [_i, _p],
    "oracle_resize_linear_exact": [_p, _i, _i, _i, _p, _i, _i, _i],
    "oracle_fast_score_map": [_p, _i, _i, _i, _i, _p],
    "oracle_orb_umax": [_p],
    "oracle_gauss_blur7": [_p, _i, _i, _i, _p, _i],
    "oracle_gauss_kernel7": [_p],
    "oracle_harris": [_p, _i, _i, _i],
    "oracle_ic_angle": [_p, _i, _i, _i, _p],
    "oracle_orb_tiles": [_p, _i, _i, _i, _i, _i, _i, _i, _p, _p, _p, _p, _i],
    "oracle_orb_tiles_batch": [_p, _i, _i, _i, _i, _i, _p, _p, _p, _p, _i, _p],
}
_RET = {"oracle_orb_tiles": ctypes.c_int, "oracle_fast_score": ctypes.c_int,
        "oracle_harris": ctypes.c_float, "oracle_ic_angle": ctypes.c_float,
        "oracle_fast_atan2": ctypes.c_float}


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
                f.restype = _RET.get(name)
            l.oracle_fast_atan2.argtypes = [ctypes.c_float, ctypes.c_float]
            l.oracle_fast_atan2.restype = ctypes.c_float
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
    cv::BFMatcher returns — and take the first two (keypoint.py:44).
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


# ----------------------------------------------------------------------------- ORB
PATTERN_PATH = os.path.join(_HERE, "bit_pattern_31.txt")


def orb_pattern() -> np.ndarray:
    """bit_pattern_31 as int8 [256, 4] (x1, y1, x2, y2)."""
    return np.loadtxt(PATTERN_PATH, dtype=np.int64, comments="#").astype(np.int8).reshape(256, 4)


def orb_level_sizes(w, h):
    lw = np.zeros(8, np.int32)
    lh = np.zeros(8, np.int32)
    sc = np.zeros(8, np.float32)
    lib().oracle_orb_level_sizes(w, h, _ptr(lw), _ptr(lh), _ptr(sc))
    return lw, lh, sc


def orb_level_budget(nfeatures):
    n = np.zeros(8, np.int32)
    lib().oracle_orb_level_budget(nfeatures, _ptr(n))
    return n


def resize_linear_exact(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    src = np.ascontiguousarray(src, np.uint8)
    dst = np.zeros((dh, dw), np.uint8)
    lib().oracle_resize_linear_exact(_ptr(src), src.shape[1], src.shape[0], src.shape[1],
                                     _ptr(dst), dw, dh, dw)
    return dst


def fast_score_map(img: np.ndarray, threshold: int = 20) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    sc = np.zeros((h, w), np.uint8)
    lib().oracle_fast_score_map(_ptr(img), w, h, w, threshold, _ptr(sc))
    return sc


def gauss_blur7(img: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    out = np.zeros_like(img)
    lib().oracle_gauss_blur7(_ptr(img), w, h, w, _ptr(out), w)
    return out


def gauss_kernel7() -> np.ndarray:
    k = np.zeros(7, np.float32)
    lib().oracle_gauss_kernel7(_ptr(k))
    return k


def orb_umax() -> np.ndarray:
    u = np.zeros(17, np.int32)
    lib().oracle_orb_umax(_ptr(u))
    return u


def orb_tiles(img: np.ndarray, max_number_of_kp: int = 40, overlap_div=2, height_div=5,
              width_div=10, cap: int = 1 << 16):
    """orb_detector_using_tiles restated -> (kp [N,5] f32 (x,y,size,angle,response),
    octave [N] i32, desc [N,32] u8)."""
    img = np.ascontiguousarray(img, np.uint8)
    H, W = img.shape
    pat = np.ascontiguousarray(orb_pattern())
    kp = np.zeros((cap, 5), np.float32)
    octv = np.zeros(cap, np.int32)
    desc = np.zeros((cap, 32), np.uint8)
    n = lib().oracle_orb_tiles(_ptr(img), H, W, W, max_number_of_kp, overlap_div, height_div,
                               width_div, _ptr(pat), _ptr(kp), _ptr(octv), _ptr(desc), cap)
    if n < 0:
        raise RuntimeError("oracle_orb_tiles: capacity exceeded")
    return kp[:n].copy(), octv[:n].copy(), desc[:n].copy()


def orb_tiles_batch(imgs: np.ndarray, max_number_of_kp: int, cap: int):
    """Default tiling (2, 5, 10) over a batch [B,H,W] (OpenMP over images)."""
    imgs = np.ascontiguousarray(imgs, np.uint8)
    B, H, W = imgs.shape
    pat = np.ascontiguousarray(orb_pattern())
    kp = np.zeros((B, cap, 5), np.float32)
    octv = np.zeros((B, cap), np.int32)
    desc = np.zeros((B, cap, 32), np.uint8)
    cnt = np.zeros(B, np.int32)
    lib().oracle_orb_tiles_batch(_ptr(imgs), B, H, W, W, max_number_of_kp, _ptr(pat), _ptr(kp),
                                 _ptr(octv), _ptr(desc), cap, _ptr(cnt))
    return kp, octv, desc, cnt

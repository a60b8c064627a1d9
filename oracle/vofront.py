"""ORACLE — test infrastructure only (see oracle/__init__.py).

CPU restatement of the reference's LK / SGBM stereo visual-odometry front end
(SURVEY.md §8f rank 4), composed from the C primitives of oracle/vofront.c:

  get_tiled_keypoints   /root/reference/visual_odometry.py:84-96
  track_keypoints       /root/reference/visual_odometry.py:98-112
  track_keypoints_left_to_right  /root/reference/keypoint.py:13-32
  calculate_right_qs    /root/reference/visual_odometry.py:114-127
  calc_3d               /root/reference/visual_odometry.py:129-134
  sgbm_compute          /root/reference/visual_odometry.py:22-24 (StereoSGBM .compute)
  get_pose              /root/reference/visual_odometry.py:188-195 (estimate_pose with the
                        seeded hypothesis stream of oracle/vo.c)

The NumPy glue here (filters, rounding, the negative-index wrap of
calculate_right_qs, float32 arithmetic of calc_3d) is pinned by
tests/golden/vofront_golden.npz, which runs the reference's own methods with
a stub cv2 backed by the same C primitives (tests/golden/make_vofront_goldens.py).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _ptr, lib

FAST_T = 10          # cv2.FastFeatureDetector_create() default threshold
LK_WIN = 15          # visual_odometry.py:26 winSize=(15, 15)
LK_LEVELS = 3        # maxLevel=3
LK_COUNT, LK_EPS = 50, 0.03
LK_MIN_EIG = 1e-4    # calcOpticalFlowPyrLK minEigThreshold default
SGBM = dict(minDisparity=0, numDisparities=32, blockSize=11, P1=11 * 11 * 8, P2=11 * 11 * 32)

_SIGS = {
    "oracle_fast_tiles": ([ctypes.c_void_p] + [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_int],
                          ctypes.c_int),
    "oracle_pyr_down": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                         ctypes.c_int], None),
    "oracle_lk_levels": ([ctypes.c_int] * 4 + [ctypes.c_void_p] * 2, ctypes.c_int),
    "oracle_scharr": ([ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p], None),
    "oracle_lk_track": ([ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                         ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                         ctypes.c_double, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p,
                         ctypes.c_void_p], None),
    "oracle_sgbm": ([ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 7 + [ctypes.c_void_p],
                    None),
}


def _l():
    L = lib()
    if not getattr(L, "_vofront_sigs", False):
        for name, (args, ret) in _SIGS.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = ret
        L._vofront_sigs = True
    return L


def _u8(img):
    return np.ascontiguousarray(img, np.uint8)


def fast_tiles(img, tile_h=10, tile_w=20, threshold=FAST_T, per_tile=10):
    """get_kps over the tile grid (visual_odometry.py:84-96) -> [N, 3] f32 (x, y, response)."""
    img = _u8(img)
    H, W = img.shape
    cap = ((H + tile_h - 1) // tile_h) * ((W + tile_w - 1) // tile_w) * per_tile
    out = np.zeros((max(cap, 1), 3), np.float32)
    n = _l().oracle_fast_tiles(_ptr(img), H, W, W, tile_h, tile_w, threshold, per_tile,
                               _ptr(out), cap)
    if n < 0:
        raise RuntimeError("oracle_fast_tiles: capacity exceeded")
    return out[:n].copy()


def pyr_down(img):
    img = _u8(img)
    h, w = img.shape
    dst = np.zeros(((h + 1) // 2, (w + 1) // 2), np.uint8)
    _l().oracle_pyr_down(_ptr(img), w, h, _ptr(dst), dst.shape[1], dst.shape[0])
    return dst


def lk_levels(W, H, win=LK_WIN, max_level=LK_LEVELS):
    lw = np.zeros(16, np.int32)
    lh = np.zeros(16, np.int32)
    n = _l().oracle_lk_levels(W, H, win, max_level, _ptr(lw), _ptr(lh))
    return [(int(lw[i]), int(lh[i])) for i in range(n)]


def scharr(img):
    img = _u8(img)
    h, w = img.shape
    d = np.zeros((h, w, 2), np.int16)
    _l().oracle_scharr(_ptr(img), w, h, _ptr(d))
    return d


def calc_optical_flow_pyr_lk(prev, nxt, pts, win=LK_WIN, max_level=LK_LEVELS,
                             max_count=LK_COUNT, eps=LK_EPS, min_eig=LK_MIN_EIG):
    """cv2.calcOpticalFlowPyrLK(prev, nxt, pts, None, winSize=(win, win), maxLevel,
    criteria=(EPS|COUNT, max_count, eps)) -> (pts2 [N,2] f32, status [N] u8, err [N] f32)."""
    prev, nxt = _u8(prev), _u8(nxt)
    H, W = prev.shape
    p = np.ascontiguousarray(np.asarray(pts, np.float32).reshape(-1, 2))
    n = len(p)
    out = np.zeros((max(n, 1), 2), np.float32)
    st = np.zeros(max(n, 1), np.uint8)
    err = np.zeros(max(n, 1), np.float32)
    if n:
        _l().oracle_lk_track(_ptr(prev), _ptr(nxt), H, W, _ptr(p), n, win, max_level, max_count,
                             eps, min_eig, _ptr(out), _ptr(st), _ptr(err))
    return out[:n], st[:n], err[:n]


def sgbm_compute(left, right, minDisparity=0, numDisparities=32, blockSize=11, P1=968, P2=3872):
    """StereoSGBM(...).compute(left, right) -> int16 disparity x16."""
    left, right = _u8(left), _u8(right)
    H, W = left.shape
    disp = np.zeros((H, W), np.int16)
    _l().oracle_sgbm(_ptr(left), _ptr(right), H, W, minDisparity, numDisparities, blockSize, P1,
                     P2, _ptr(disp))
    return disp


def disparity_f32(left, right):
    """np.divide(disparity.compute(l, r).astype(np.float32), 16) (visual_odometry.py:24,191)."""
    return np.divide(sgbm_compute(left, right, **SGBM).astype(np.float32), 16)


def track_keypoints(img1, img2, kp_xy, max_error=4):
    """visual_odometry.py:98-112 -> (trackpoints1 [M,2] f32, trackpoints2 [M,2] f32 rounded)."""
    tp1 = np.asarray(kp_xy, np.float32).reshape(-1, 2)
    tp2, st, err = calc_optical_flow_pyr_lk(img1, img2, tp1)
    trackable = st.astype(bool)
    under = err[trackable] < max_error
    tp1 = tp1[trackable][under]
    tp2 = np.around(tp2[trackable][under])
    h, w = np.asarray(img1).shape
    inb = np.logical_and(tp2[:, 1] < h, tp2[:, 0] < w)
    return tp1[inb], tp2[inb]


def track_keypoints_left_to_right(img_l, img_r, kp_xy, descriptors_left, max_error=500):
    """keypoint.py:13-32 -> (trackpoints1 [M,2], descriptors [M,32], trackpoints2 [M,2])."""
    tp1 = np.asarray(kp_xy, np.float32).reshape(-1, 2)
    tp2, st, err = calc_optical_flow_pyr_lk(img_l, img_r, tp1)
    trackable = st.astype(bool)
    under = err[trackable] < max_error
    des = np.asarray(descriptors_left)[trackable][under]
    tp1 = tp1[trackable][under]
    tp2 = np.around(tp2[trackable][under])
    h, w = np.asarray(img_r).shape
    inb = (tp2[:, 1] < h) & (tp2[:, 0] < w) & (tp2[:, 1] > 0) & (tp2[:, 0] > 0)
    return tp1[inb], des[inb], tp2[inb]


def calculate_right_qs(q1, q2, disp1, disp2, min_disp=0.0, max_disp=100.0):
    """visual_odometry.py:114-127 (int() truncation, disp.T[x, y] with NumPy's
    negative-index wrap)."""
    def get_idxs(q, disp):
        qi = q.astype(int)
        d = disp.T[qi[:, 0], qi[:, 1]]
        return d, np.logical_and(min_disp < d, d < max_disp)

    d1, i1 = get_idxs(q1, disp1)
    d2, i2 = get_idxs(q2, disp2)
    ok = np.logical_and(i1, i2)
    q1_l, q2_l, d1, d2 = q1[ok], q2[ok], d1[ok], d2[ok]
    q1_r, q2_r = np.copy(q1_l), np.copy(q2_l)
    q1_r[:, 0] -= d1
    q2_r[:, 0] -= d2
    return q1_l, q1_r, q2_l, q2_r


def triangulate_points(P1, P2, x1, x2):
    """cv2.triangulatePoints restated: unit null vector of the 4x4 DLT system
    (f64), returned in the input dtype (4, N)."""
    x1 = np.asarray(x1)
    dt = x1.dtype if x1.dtype in (np.float32, np.float64) else np.float64
    a = np.asarray(x1, np.float64).reshape(2, -1).T
    b = np.asarray(x2, np.float64).reshape(2, -1).T
    M = len(a)
    A = np.empty((M, 4, 4))
    for j, (q, P) in enumerate(((a, np.asarray(P1, float)), (b, np.asarray(P2, float)))):
        A[:, 2 * j] = q[:, 0:1] * P[2][None] - P[0][None]
        A[:, 2 * j + 1] = q[:, 1:2] * P[2][None] - P[1][None]
    if M == 0:
        return np.zeros((4, 0), dt)
    _, _, Vt = np.linalg.svd(A)
    return Vt[:, -1, :].T.astype(dt)


def calc_3d(q1_l, q1_r, q2_l, q2_r, P_l, P_r):
    """visual_odometry.py:129-134 (float32 in, float32 homogeneous, float32 divide)."""
    Q1 = triangulate_points(P_l, P_r, q1_l.T, q1_r.T)
    Q1 = np.transpose(Q1[:3] / Q1[3])
    Q2 = triangulate_points(P_l, P_r, q2_l.T, q2_r.T)
    Q2 = np.transpose(Q2[:3] / Q2[3])
    return Q1, Q2


def get_pose(img1_l, img2_l, disp1, disp2, P_l, P_r, seed=0, frame=0, max_iter=100):
    """visual_odometry.py:188-195 with the seeded estimate_pose of oracle/vo.c.
    disp1/disp2: float32 disparity maps of frames i-1 and i."""
    from .geometry import form_transf, rodrigues, vo_estimate_pose

    kp = fast_tiles(img1_l)
    tp1, tp2 = track_keypoints(img1_l, img2_l, kp[:, :2])
    q1_l, q1_r, q2_l, q2_r = calculate_right_qs(tp1, tp2, disp1, disp2)
    Q1, Q2 = calc_3d(q1_l, q1_r, q2_l, q2_r, P_l, P_r)
    dof, best, ntried, err, _ = vo_estimate_pose(q1_l, q2_l, Q1, Q2, P_l, seed=seed, item=frame,
                                              max_iter=max_iter)
    T = form_transf(rodrigues(dof[:3]), dof[3:])
    return T, Q1, dict(kp=kp, tp1=tp1, tp2=tp2, q1_l=q1_l, q2_l=q2_l, Q1=Q1, Q2=Q2, dof=dof,
                       best=best, ntried=ntried, error=err)

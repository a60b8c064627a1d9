"""Batched device API of the LK / SGBM stereo-VO front end.

Reference path (/root/reference/visual_odometry.py, VisualOdometry.get_pose :188-195):
    kp1  = get_tiled_keypoints(img1_l, 10, 20)            # FAST per 10x20 tile, best 10
    tp1, tp2 = track_keypoints(img1_l, img2_l, kp1)       # pyramidal LK + filters
    disp_i = StereoSGBM.compute(img_l, img_r) / 16        # per frame
    q1_l, q1_r, q2_l, q2_r = calculate_right_qs(...)      # disparity lookup
    Q1, Q2 = calc_3d(...)                                 # float32 DLT
    T = estimate_pose(q1_l, q2_l, Q1, Q2)                 # RANSAC-6 + LM
Here every stage is a HIP kernel on B frame pairs at once (csrc/vofront.hip,
csrc/geometry.hip); intermediates stay in HBM and only B relative poses come
back.  Torch tensors are device-memory containers only.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib, geometry
from .device import ptr, require_gpu, stream_ptr, to_dev

FAST_T, TILE_H, TILE_W, PER_TILE = 10, 10, 20, 10   # visual_odometry.py:24,86-91,189
LK_WIN, LK_LEVELS, LK_COUNT, LK_EPS = 15, 3, 50, 0.03  # visual_odometry.py:26-29
LK_MIN_EIG = 1e-4                                    # calcOpticalFlowPyrLK default
SGBM = dict(min_disp=0, num_disp=32, block=11, P1=11 * 11 * 8, P2=11 * 11 * 32)  # :20-23


def _ws(nbytes: int, dev) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=dev)


def fast_tiles(imgs: torch.Tensor, tile_h=TILE_H, tile_w=TILE_W, threshold=FAST_T,
               per_tile=PER_TILE, kp_cap=None, stream=None):
    """imgs [B,H,W] u8 (device) -> (kp [B,cap,3] f32 (x, y, response), count [B] i32)."""
    B, H, W = imgs.shape
    dev = imgs.device
    n_tiles = -(-H // tile_h) * -(-W // tile_w)
    cap = kp_cap or n_tiles * per_tile
    nb = ctypes.c_size_t(0)
    _lib.call("slam_fast_tiles_workspace_bytes", B, H, W, tile_h, tile_w, per_tile,
              ctypes.byref(nb))
    ws = _ws(nb.value, dev)
    kp = torch.empty((B, cap, 3), dtype=torch.float32, device=dev)
    cnt = torch.empty(B, dtype=torch.int32, device=dev)
    _lib.call("slam_fast_tiles", ptr(imgs), B, H, W, W, tile_h, tile_w, threshold, per_tile,
              ptr(ws), nb.value, ptr(kp), ptr(cnt), cap, stream_ptr(stream))
    return kp, cnt


class LKPyramids:
    """Pyramids (+ derivatives) of n images: d_pyr [n, img_bytes] u8, d_der [n, img_bytes, 2] i16."""

    def __init__(self, imgs: torch.Tensor, win=LK_WIN, max_level=LK_LEVELS, derivs=True,
                 stream=None):
        n, H, W = imgs.shape
        self.H, self.W, self.win, self.max_level = H, W, win, max_level
        nlev = ctypes.c_int(0)
        nb = ctypes.c_size_t(0)
        _lib.call("slam_lk_pyramid_layout", H, W, win, max_level, ctypes.byref(nlev),
                  ctypes.byref(nb))
        self.nlev, self.img_bytes = nlev.value, nb.value
        dev = imgs.device
        self.pyr = torch.empty((n, self.img_bytes), dtype=torch.uint8, device=dev)
        self.der = (torch.empty((n, self.img_bytes, 2), dtype=torch.int16, device=dev)
                    if derivs else None)
        _lib.call("slam_lk_build_pyramids", ptr(imgs), n, H, W, W, win, max_level,
                  ptr(self.pyr), ptr(self.der), stream_ptr(stream))


def lk_track(prev: LKPyramids, nxt: LKPyramids, pts: torch.Tensor, npts: torch.Tensor,
             prev0=0, next0=0, pair_stride=1, max_count=LK_COUNT, eps=LK_EPS,
             min_eig=LK_MIN_EIG, stream=None):
    """Pair b tracks pts[b] from image prev0 + b*pair_stride of `prev` to image
    next0 + b*pair_stride of `nxt` -> (pts2 [B,cap,2] f32, status [B,cap] u8, err [B,cap] f32)."""
    B, cap, ps = pts.shape
    if prev.der is None:
        raise ValueError("prev pyramids were built without derivatives")
    for name, pyr, i0 in (("prev", prev, prev0), ("next", nxt, next0)):
        last = i0 + (B - 1) * pair_stride
        if B > 0 and not (0 <= i0 < pyr.pyr.shape[0] and 0 <= last < pyr.pyr.shape[0]):
            raise IndexError(f"lk_track: {name} images {i0}..{last} outside the "
                             f"{pyr.pyr.shape[0]} pyramids")
    if (prev.H, prev.W, prev.win, prev.max_level) != (nxt.H, nxt.W, nxt.win, nxt.max_level):
        raise ValueError("lk_track: prev/next pyramids have different layouts")
    dev = pts.device
    out = torch.empty((B, cap, 2), dtype=torch.float32, device=dev)
    st = torch.empty((B, cap), dtype=torch.uint8, device=dev)
    err = torch.empty((B, cap), dtype=torch.float32, device=dev)
    pp = ctypes.c_void_p(prev.pyr[prev0].data_ptr())
    pd = ctypes.c_void_p(prev.der[prev0].data_ptr())
    npy = ctypes.c_void_p(nxt.pyr[next0].data_ptr())
    _lib.call("slam_lk_track", pp, pd, npy, pair_stride, B, prev.H, prev.W, prev.win,
              prev.max_level, max_count, eps, min_eig, ptr(pts), ps, ptr(npts), cap, ptr(out),
              ptr(st), ptr(err), stream_ptr(stream))
    return out, st, err


def lk_filter(p1, p2, status, err, npts, H, W, max_error=4.0, lower_bounds=False, stream=None):
    """track_keypoints' filters -> (tp1, tp2 [B,cap,2] f32, idx [B,cap] i32, count [B] i32)."""
    B, cap, ps = p1.shape
    dev = p1.device
    tp1 = torch.empty((B, cap, 2), dtype=torch.float32, device=dev)
    tp2 = torch.empty((B, cap, 2), dtype=torch.float32, device=dev)
    idx = torch.empty((B, cap), dtype=torch.int32, device=dev)
    cnt = torch.empty(B, dtype=torch.int32, device=dev)
    _lib.call("slam_lk_filter", ptr(p1), ps, ptr(p2), ptr(status), ptr(err), ptr(npts), cap, B,
              H, W, float(max_error), int(bool(lower_bounds)), ptr(tp1), ptr(tp2), ptr(idx),
              ptr(cnt), stream_ptr(stream))
    return tp1, tp2, idx, cnt


def sgbm(left: torch.Tensor, right: torch.Tensor, min_disp=0, num_disp=32, block=11, P1=968,
         P2=3872, f32=True, stream=None):
    """left/right [B,H,W] u8 -> (disp [B,H,W] i16 x16, disp/16 [B,H,W] f32 or None)."""
    B, H, W = left.shape
    dev = left.device
    nb = ctypes.c_size_t(0)
    _lib.call("slam_sgbm_workspace_bytes", B, H, W, min_disp, num_disp, block, ctypes.byref(nb))
    ws = _ws(nb.value, dev)
    d = torch.empty((B, H, W), dtype=torch.int16, device=dev)
    df = torch.empty((B, H, W), dtype=torch.float32, device=dev) if f32 else None
    _lib.call("slam_sgbm", ptr(left), ptr(right), B, H, W, W, min_disp, num_disp, block, P1, P2,
              ptr(ws), nb.value, ptr(d), ptr(df), stream_ptr(stream))
    return d, df


def right_qs_3d(tp1, tp2, cnt, disp_f32, P_l, P_r, disp1_index=0, disp2_offset=1,
                min_disp=0.0, max_disp=100.0, f64=True, stream=None):
    """calculate_right_qs + calc_3d for pair b: disparity maps disp_f32[disp1_index + b]
    and disp_f32[disp1_index + b + disp2_offset]."""
    B, cap, _ = tp1.shape
    dev = tp1.device
    nd, H, W = disp_f32.shape
    if B > 0:
        first, last = disp1_index, disp1_index + B - 1 + disp2_offset
        if not (0 <= first < nd and 0 <= disp1_index + disp2_offset and last < nd):
            raise IndexError(f"right_qs_3d: disparity maps {first}..{last} outside the "
                             f"{nd} maps")
    f = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)  # noqa: E731
    d = lambda *s: torch.empty(s, dtype=torch.float64, device=dev) if f64 else None  # noqa: E731
    o = dict(q1_l=f(B, cap, 2), q1_r=f(B, cap, 2), q2_l=f(B, cap, 2), q2_r=f(B, cap, 2),
             Q1=f(B, cap, 3), Q2=f(B, cap, 3), q1_l64=d(B, cap, 2), q2_l64=d(B, cap, 2),
             Q1_64=d(B, cap, 3), Q2_64=d(B, cap, 3),
             count=torch.empty(B, dtype=torch.int32, device=dev))
    Pl = to_dev(np.asarray(P_l, np.float64).reshape(12))
    Pr = to_dev(np.asarray(P_r, np.float64).reshape(12))
    dp = ctypes.c_void_p(disp_f32[disp1_index].data_ptr())
    _lib.call("slam_vo_right_qs_3d", ptr(tp1), ptr(tp2), ptr(cnt), cap, B, dp, H * W,
              disp2_offset * H * W, H, W, float(min_disp), float(max_disp), ptr(Pl), ptr(Pr),
              ptr(o["q1_l"]), ptr(o["q1_r"]), ptr(o["q2_l"]), ptr(o["q2_r"]), ptr(o["Q1"]),
              ptr(o["Q2"]), ptr(o["q1_l64"]), ptr(o["q2_l64"]), ptr(o["Q1_64"]), ptr(o["Q2_64"]),
              ptr(o["count"]), stream_ptr(stream))
    return o


def triangulate_f32(ql, qr, P_l, P_r):
    """cv2.triangulatePoints(P_l, P_r, ql.T, qr.T) on float32 points, then
    Q[:3] / Q[3] in float32 (visual_odometry.py:130-133) -> [N, 3] f32 (NumPy)."""
    ql = np.ascontiguousarray(ql, np.float32).reshape(-1, 2)
    qr = np.ascontiguousarray(qr, np.float32).reshape(-1, 2)
    n = len(ql)
    if n == 0:
        return np.zeros((0, 3), np.float32)
    a, b = to_dev(ql[None]), to_dev(qr[None])
    cnt = torch.tensor([n], dtype=torch.int32, device=a.device)
    X = torch.empty((1, n, 3), dtype=torch.float32, device=a.device)
    Pl = to_dev(np.asarray(P_l, np.float64).reshape(12))
    Pr = to_dev(np.asarray(P_r, np.float64).reshape(12))
    _lib.call("slam_triangulate_f32", ptr(a), ptr(b), ptr(cnt), n, 1, ptr(Pl), ptr(Pr), ptr(X),
              stream_ptr(None))
    return X[0].cpu().numpy()


class StereoVO:
    """VisualOdometry.get_pose on B consecutive frame pairs per call.

    left/right [B+1, H, W] u8 (device): frame pairs (i, i+1) for i < B.  One call
    = FAST on the B first left images, LK pyramids of all B+1 left images, SGBM
    on all B+1 stereo pairs, LK + filters, disparity lookup + triangulation, and
    the seeded RANSAC-6 + LM pose (slam_vo_estimate_pose) for every pair.
    """

    def __init__(self, P_l, P_r, seed=0, max_iter=100):
        self.P_l = np.asarray(P_l, np.float64).reshape(3, 4)
        self.P_r = np.asarray(P_r, np.float64).reshape(3, 4)
        self.seed, self.max_iter = seed, max_iter
        self._side = None

    def run(self, left: torch.Tensor, right: torch.Tensor, frame0=0, stream=None):
        require_gpu()
        B = left.shape[0] - 1
        H, W = left.shape[1:]
        main = stream if stream is not None else torch.cuda.current_stream()
        # SGBM does not depend on FAST / LK: it runs on a side stream meanwhile
        if self._side is None:
            self._side = torch.cuda.Stream(device=left.device)
        ready = torch.cuda.Event()
        ready.record(main)
        self._side.wait_event(ready)
        with torch.cuda.stream(self._side):
            _, dispf = sgbm(left, right, **SGBM, stream=self._side)
            done = torch.cuda.Event()
            done.record(self._side)
        dispf.record_stream(main)
        kp, nkp = fast_tiles(left[:B], stream=main)
        pyr = LKPyramids(left, stream=main)
        p2, st, err = lk_track(pyr, pyr, kp, nkp, prev0=0, next0=1, stream=main)
        tp1, tp2, _, ntp = lk_filter(kp, p2, st, err, nkp, H, W, max_error=4.0, stream=main)
        main.wait_event(done)
        stream = main
        o = right_qs_3d(tp1, tp2, ntp, dispf, self.P_l, self.P_r, stream=stream)
        pose, best, ntried, perr = geometry.vo_estimate_pose(
            o["q1_l64"], o["q2_l64"], o["Q1_64"], o["Q2_64"], o["count"], self.P_l,
            seed=self.seed, item0=frame0, max_iter=self.max_iter, stream=stream)
        return dict(kp=kp, nkp=nkp, p2=p2, status=st, err=err, tp1=tp1, tp2=tp2, ntp=ntp,
                    disp=dispf, pose=pose, best=best, ntried=ntried, error=perr, **o)

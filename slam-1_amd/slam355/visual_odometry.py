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


# --------------------------------------------------------------------------
# The LK / SGBM front end of VisualOdometry (visual_odometry.py:11-195) on the GPU
# (csrc/vofront.hip, batched device API in slam355.vofront).

class StereoSGBM:
    """cv2.StereoSGBM_create(minDisparity, numDisparities, blockSize, P1, P2)
    (visual_odometry.py:20-23): .compute(left, right) -> int16 disparity x16."""

    def __init__(self, minDisparity=0, numDisparities=16, blockSize=3, P1=0, P2=0):
        self.kw = dict(min_disp=minDisparity, num_disp=numDisparities, block=blockSize, P1=P1,
                       P2=P2)

    def compute(self, left, right):
        from . import vofront

        l = to_dev(np.ascontiguousarray(left, np.uint8)[None])
        r = to_dev(np.ascontiguousarray(right, np.uint8)[None])
        d, _ = vofront.sgbm(l, r, f32=False, **self.kw)
        return d[0].cpu().numpy()


def StereoSGBM_create(minDisparity=0, numDisparities=16, blockSize=3, P1=0, P2=0):
    return StereoSGBM(minDisparity, numDisparities, blockSize, P1, P2)


def calc_optical_flow_pyr_lk(img1, img2, pts, win=15, max_level=3, max_count=50, eps=0.03):
    """cv2.calcOpticalFlowPyrLK(img1, img2, pts, None, winSize=(win, win), maxLevel,
    criteria=(EPS|COUNT, max_count, eps)) -> (pts2 [N,2] f32, status [N] u8, err [N] f32)."""
    from . import vofront

    p = np.ascontiguousarray(np.asarray(pts, np.float32).reshape(-1, 2))
    n = len(p)
    if n == 0:
        return np.zeros((0, 2), np.float32), np.zeros(0, np.uint8), np.zeros(0, np.float32)
    imgs = to_dev(np.stack([np.asarray(img1, np.uint8), np.asarray(img2, np.uint8)]))
    pyr = vofront.LKPyramids(imgs, win, max_level)
    cnt = torch.tensor([n], dtype=torch.int32, device=imgs.device)
    out, st, err = vofront.lk_track(pyr, pyr, to_dev(p[None]), cnt, prev0=0, next0=1,
                                    max_count=max_count, eps=eps)
    return out[0].cpu().numpy(), st[0].cpu().numpy(), err[0].cpu().numpy()


class VisualOdometry:
    """Mirror of the reference's VisualOdometry (visual_odometry.py:11-195).

    The reference's __init__ reads KITTI-style calib.txt / poses.txt and image
    directories with cv2.imread; here the images are passed as arrays
    (images_l / images_r: sequences of [H, W] u8) and calib / poses either as
    paths in the reference's text formats or as arrays.
    """

    def __init__(self, images_l, images_r, calib=None, P_l=None, P_r=None, poses=None, seed=0):
        if calib is not None:
            self.K_l, self.P_l, self.K_r, self.P_r = self._load_calib(calib)
        else:
            self.P_l = np.asarray(P_l, np.float64).reshape(3, 4)
            self.P_r = np.asarray(P_r, np.float64).reshape(3, 4)
            self.K_l, self.K_r = self.P_l[:, :3], self.P_r[:, :3]
        self.gt_poses = self._load_poses(poses) if isinstance(poses, str) else poses
        self.images_l = [np.asarray(i, np.uint8) for i in images_l]
        self.images_r = [np.asarray(i, np.uint8) for i in images_r]
        block = 11
        self.disparity = StereoSGBM_create(minDisparity=0, numDisparities=32, blockSize=block,
                                           P1=block * block * 8, P2=block * block * 32)
        self.disparities = [np.divide(self.disparity.compute(self.images_l[0], self.images_r[0])
                                      .astype(np.float32), 16)]
        self.lk_params = dict(winSize=(15, 15), maxLevel=3, criteria=(3, 50, 0.03))
        self.seed = seed

    @staticmethod
    def _load_calib(filepath):
        """visual_odometry.py:31-40: two lines of 12 floats (P_l, P_r)."""
        with open(filepath) as f:
            P_l = np.array(f.readline().split(), dtype=float).reshape(3, 4)
            P_r = np.array(f.readline().split(), dtype=float).reshape(3, 4)
        return P_l[:, :3], P_l, P_r[:, :3], P_r

    @staticmethod
    def _load_poses(filepath):
        """visual_odometry.py:42-51: 3x4 rows -> 4x4."""
        poses = []
        with open(filepath) as f:
            for line in f:
                T = np.array(line.split(), dtype=float).reshape(3, 4)
                poses.append(np.vstack((T, [0, 0, 0, 1])))
        return poses

    @staticmethod
    def _form_transf(R, t):
        return form_transf(R, t)

    def reprojection_residuals(self, dof, q1, q2, Q1, Q2):
        return reprojection_residuals(dof, q1, q2, Q1, Q2, self.P_l)

    def get_tiled_keypoints(self, img, tile_h, tile_w):
        """visual_odometry.py:84-96 -> list of KeyPoint (.pt, .response)."""
        from . import vofront
        from .orb import KeyPoint

        t = to_dev(np.ascontiguousarray(img, np.uint8)[None])
        kp, cnt = vofront.fast_tiles(t, tile_h, tile_w)
        n = int(cnt[0])
        if n < 0:
            raise RuntimeError("slam_fast_tiles: keypoint capacity exceeded")
        k = kp[0, :n].cpu().numpy()
        return [KeyPoint(x, y, 7.0, -1.0, r, 0) for x, y, r in k]

    def track_keypoints(self, img1, img2, kp1, max_error=4):
        """visual_odometry.py:98-112 -> (trackpoints1, trackpoints2) [M, 2] f32."""
        tp1 = np.array([k.pt for k in kp1], np.float32).reshape(-1, 2)
        tp2, st, err = calc_optical_flow_pyr_lk(img1, img2, tp1, self.lk_params["winSize"][0],
                                                self.lk_params["maxLevel"])
        trackable = st.astype(bool)
        under = err[trackable] < max_error
        tp1 = tp1[trackable][under]
        tp2 = np.around(tp2[trackable][under])
        h, w = np.asarray(img1).shape
        inb = np.logical_and(tp2[:, 1] < h, tp2[:, 0] < w)
        return tp1[inb], tp2[inb]

    def calculate_right_qs(self, q1, q2, disp1, disp2, min_disp=0.0, max_disp=100.0):
        """visual_odometry.py:114-127 on the GPU (slam_vo_right_qs_3d)."""
        return self._right_qs_3d(q1, q2, disp1, disp2, min_disp, max_disp)[:4]

    def calc_3d(self, q1_l, q1_r, q2_l, q2_r):
        """visual_odometry.py:129-134: float32 DLT points (slam_triangulate_f32)."""
        from . import vofront

        return (vofront.triangulate_f32(q1_l, q1_r, self.P_l, self.P_r),
                vofront.triangulate_f32(q2_l, q2_r, self.P_l, self.P_r))

    def _right_qs_3d(self, q1, q2, disp1, disp2, min_disp, max_disp):
        from . import vofront

        q1 = np.ascontiguousarray(q1, np.float32).reshape(-1, 2)
        q2 = np.ascontiguousarray(q2, np.float32).reshape(-1, 2)
        n = len(q1)
        if n == 0:
            z2, z3 = np.zeros((0, 2), np.float32), np.zeros((0, 3), np.float32)
            return z2, z2, z2, z2, z3, z3
        disp = to_dev(np.stack([np.asarray(disp1, np.float32), np.asarray(disp2, np.float32)]))
        t1, t2 = to_dev(q1[None]), to_dev(q2[None])
        cnt = torch.tensor([n], dtype=torch.int32, device=t1.device)
        o = vofront.right_qs_3d(t1, t2, cnt, disp, self.P_l, self.P_r, min_disp=min_disp,
                                max_disp=max_disp, f64=False)
        m = int(o["count"][0])
        g = lambda k: o[k][0, :m].cpu().numpy()  # noqa: E731
        return g("q1_l"), g("q1_r"), g("q2_l"), g("q2_r"), g("Q1"), g("Q2")

    def estimate_pose(self, q1, q2, Q1, Q2, max_iter=100, frame=0):
        return estimate_pose(q1, q2, Q1, Q2, self.P_l, max_iter=max_iter, seed=self.seed,
                             frame=frame)

    def get_pose(self, i):
        """visual_odometry.py:188-195 -> (T 4x4, Q1)."""
        img1_l, img2_l = self.images_l[i - 1:i + 1]
        kp1_l = self.get_tiled_keypoints(img1_l, 10, 20)
        tp1_l, tp2_l = self.track_keypoints(img1_l, img2_l, kp1_l)
        self.disparities.append(np.divide(self.disparity.compute(img2_l, self.images_r[i])
                                          .astype(np.float32), 16))
        q1_l, q1_r, q2_l, q2_r, Q1, Q2 = self._right_qs_3d(
            tp1_l, tp2_l, self.disparities[i - 1], self.disparities[i], 0.0, 100.0)
        return self.estimate_pose(q1_l, q2_l, Q1, Q2, frame=i), Q1

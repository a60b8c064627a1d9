"""Golden fixtures for the LK / SGBM stereo-VO front end,
generated from the REFERENCE's own methods (run in the build container only;
/root/reference does not exist on the GPU box):

    python tests/golden/make_vofront_goldens.py

The reference's VisualOdometry (/root/reference/visual_odometry.py) and
keypoint.track_keypoints_left_to_right (/root/reference/keypoint.py:13-32) are
imported with a stub `cv2` (OpenCV is absent from this image: an ordinary
ModuleNotFoundError, not a permission denial).  The stub's FAST detector,
calcOpticalFlowPyrLK, StereoSGBM and triangulatePoints are the CPU
restatement in oracle/vofront.c, so these goldens pin the reference's own
Python around them: the per-tile sort/truncation and offsets of
get_tiled_keypoints (:84-96), the status/error/bounds filters and np.around of
track_keypoints (:98-112) and of track_keypoints_left_to_right, the int()
truncation and negative-index wrap of calculate_right_qs (:114-127), and the
float32 homogeneous division of calc_3d (:129-134).  OpenCV's own FAST / LK /
SGBM numerics remain "parity unpinned".  VisualOdometry.__init__ reads a
dataset directory, so the instance is made with object.__new__ and given the
attributes __init__ would set (:14-29).
Only data (inputs + outputs) is written; no reference source is copied.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

from oracle import vofront as vf  # noqa: E402


class _KP:
    def __init__(self, x, y, r):
        self.pt = (float(x), float(y))
        self.response = float(r)
        self.size = 7.0


class _Fast:
    def detect(self, patch, mask=None):
        patch = np.ascontiguousarray(patch)
        h, w = patch.shape
        k = vf.fast_tiles(patch, h, w, vf.FAST_T, h * w)  # whole patch, detection order
        return [_KP(x, y, r) for x, y, r in k]


class _SGBM:
    def __init__(self, **kw):
        self.kw = kw

    def compute(self, l, r):
        return vf.sgbm_compute(l, r, **self.kw)


def _lk(img1, img2, pts, nxt, winSize, flags, maxLevel, criteria):
    p = np.asarray(pts, np.float32).reshape(-1, 2)
    out, st, err = vf.calc_optical_flow_pyr_lk(img1, img2, p, win=winSize[0], max_level=maxLevel,
                                               max_count=criteria[1], eps=criteria[2])
    return out.reshape(-1, 1, 2), st.reshape(-1, 1), err.reshape(-1, 1)


def _stub_cv2():
    cv2 = types.ModuleType("cv2")
    cv2.MOTION_AFFINE = 2
    cv2.TERM_CRITERIA_EPS = 2
    cv2.TERM_CRITERIA_COUNT = 1
    cv2.FastFeatureDetector_create = lambda *a, **k: _Fast()
    cv2.StereoSGBM_create = lambda **kw: _SGBM(**kw)
    cv2.calcOpticalFlowPyrLK = _lk
    cv2.KeyPoint_convert = lambda kps: np.array([k.pt for k in kps], np.float32).reshape(-1, 2)
    cv2.triangulatePoints = vf.triangulate_points
    cv2.imshow = lambda *a, **k: None
    cv2.waitKey = lambda *a, **k: None
    return cv2


def import_reference():
    sys.modules["cv2"] = _stub_cv2()
    if not hasattr(np, "float"):
        np.float = float  # reference uses np.float (removed in numpy>=1.24)
    sys.path.insert(0, REF)
    import keypoint  # noqa: E402
    import visual_odometry  # noqa: E402
    return visual_odometry, keypoint


def make_vo(visual_odometry, P_l, P_r):
    vo = object.__new__(visual_odometry.VisualOdometry)
    block = 11
    vo.disparity = sys.modules["cv2"].StereoSGBM_create(
        minDisparity=0, numDisparities=32, blockSize=block, P1=block * block * 8,
        P2=block * block * 32)
    vo.fastFeatures = sys.modules["cv2"].FastFeatureDetector_create()
    vo.lk_params = dict(winSize=(15, 15), flags=2, maxLevel=3, criteria=(3, 50, 0.03))
    vo.P_l, vo.P_r = P_l, P_r
    vo.K_l, vo.K_r = P_l[:, :3], P_r[:, :3]
    return vo


def cases():
    from slam355.synthetic import StereoRig, stereo_sequence

    out = []
    L, R, _, rig = stereo_sequence(2, 320, 240, seed=11, n_landmarks=300)
    out.append(("seq", L[0], L[1], R[0], R[1], rig))
    # a pure horizontal shift of 6 px to the left: points of the first columns
    # track into the reflected border and are dropped by the error test; the
    # negative-index wrap of calculate_right_qs is pinned by the crafted "wrap" case
    L2, R2, _, rig2 = stereo_sequence(1, 360, 200, seed=12, n_landmarks=300)
    a, b = L2[0][:, 10:330], L2[0][:, 4:324]
    out.append(("shift", np.ascontiguousarray(b), np.ascontiguousarray(a),
                np.ascontiguousarray(R2[0][:, 4:324]), np.ascontiguousarray(R2[0][:, 10:330]),
                StereoRig(320, 200)))
    return out


def main():
    visual_odometry, keypoint = import_reference()
    g = {}
    for name, i1, i2, r1, r2, rig in cases():
        vo = make_vo(visual_odometry, rig.P_l, rig.P_r)
        kps = vo.get_tiled_keypoints(i1, 10, 20)
        kp = np.array([[k.pt[0], k.pt[1], k.response] for k in kps], np.float32)
        tp1, tp2 = vo.track_keypoints(i1, i2, kps)
        d1 = np.divide(vo.disparity.compute(i1, r1).astype(np.float32), 16)
        d2 = np.divide(vo.disparity.compute(i2, r2).astype(np.float32), 16)
        q1_l, q1_r, q2_l, q2_r = vo.calculate_right_qs(tp1, tp2, d1, d2)
        Q1, Q2 = vo.calc_3d(q1_l, q1_r, q2_l, q2_r)
        des = np.random.default_rng(5).integers(0, 256, (len(kps), 32), dtype=np.uint8)
        lr1, lrd, lr2 = keypoint.track_keypoints_left_to_right(i1, r1, kps, des)
        for k, v in dict(img1=i1, img2=i2, right1=r1, right2=r2, P_l=rig.P_l, P_r=rig.P_r, kp=kp,
                         tp1=tp1, tp2=tp2, disp1=d1, disp2=d2, q1_l=q1_l, q1_r=q1_r, q2_l=q2_l,
                         q2_r=q2_r, Q1=Q1, Q2=Q2, des=des, lr_tp1=lr1, lr_des=lrd,
                         lr_tp2=lr2).items():
            g[f"{name}_{k}"] = np.asarray(v)
        print(name, len(kp), len(tp1), int((tp2[:, 0] < 0).sum()), len(q1_l), len(lr1))
    # calculate_right_qs on crafted inputs: negative and fractional coordinates
    # (int() truncation toward zero, disp.T[x, y] wrapping negative indices)
    rng = np.random.default_rng(13)
    H, W = 60, 90
    d1 = rng.uniform(-1.0, 120.0, (H, W)).astype(np.float32)
    d2 = rng.uniform(-1.0, 120.0, (H, W)).astype(np.float32)
    q1 = np.stack([rng.uniform(0, W - 1, 400), rng.uniform(0, H - 1, 400)], 1).astype(np.float32)
    q2 = np.round(q1 + rng.normal(0, 4, q1.shape)).astype(np.float32)
    q2[:40, 0] = -rng.integers(1, 5, 40)
    q2[40:60, 1] = -rng.integers(1, 3, 20)
    q2 = np.minimum(q2, [[W - 1, H - 1]]).astype(np.float32)
    vo = make_vo(visual_odometry, np.eye(3, 4), np.eye(3, 4))
    out = vo.calculate_right_qs(q1, q2, d1, d2)
    for k, v in dict(q1=q1, q2=q2, disp1=d1, disp2=d2, q1_l=out[0], q1_r=out[1], q2_l=out[2],
                     q2_r=out[3]).items():
        g[f"wrap_{k}"] = v
    print("wrap", len(out[0]))
    np.savez_compressed(os.path.join(HERE, "vofront_golden.npz"), **g)


if __name__ == "__main__":
    main()

"""Generate the committed golden fixtures from the REFERENCE code (run in the
build container only; /root/reference does not exist on the GPU box).

    python tests/golden/make_goldens.py

What is pinned, and how:
  * BA (BAL reprojection block, /root/reference/BundleAdjustment.py:231-465).
    That block is a module-level string literal in the reference (opened at
    :230, closed at :466), so it is executed from its source text with numpy /
    scipy in scope.  We record `objective` residuals (incl. a zero rotation
    vector and rows that trip both >5000 px clamps, :339-350), the
    `bundle_adjustment_sparsity` pattern (:380-394) and `least_squares`
    results (:397-402) at the reference's settings (ftol=0.1) and at tight
    tolerances (the optimum the GPU LM must reach).
  * Matching post-processing (/root/reference/Point3D.py:33-53,
    keypoint.py:35-80, tracking.py:12-34) imported with a stub `cv2`
    module.  cv2 (OpenCV) is absent from this image (ModuleNotFoundError, not a
    permission denial).  The stub provides an EXACT brute-force knnMatch
    (ties -> lower train index, cv::BFMatcher order), an all-inlier
    findFundamentalMat and no-op GUI calls, so these goldens pin the ratio
    test, the |Q| gate, the ValueError truncation and the gather/dtype
    semantics of the reference around an exact matcher.  FLANN-LSH itself
    (approximate, randomised) and OpenCV's ORB / F-LMedS / PnP are NOT pinned
    here ("parity unpinned").
  * Map association and BA-problem export (/root/reference/keypoint.py:101-122
    appendKeyPoints over a growing map, Point3D.py:22-30
    relative_to_abs3DPoints, XXXport_files.py:16-64 make_cam_params /
    make_Qs_for_BA / export_data), run on a seeded synthetic sequence; the
    BA_file.txt that export_data writes is recorded byte for byte.
Only data (inputs + outputs) is written; no reference source is copied.
"""
from __future__ import annotations

import contextlib
import io
import os
import sys
import types

import numpy as np

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------- stub cv2
class _DMatch:
    def __init__(self, q, t, d):
        self.queryIdx, self.trainIdx, self.distance = q, t, float(d)


class _KeyPoint:
    def __init__(self, x, y):
        self.pt = (float(np.float32(x)), float(np.float32(y)))


class _ExactMatcher:
    def __init__(self, indexParams=None, searchParams=None):
        pass

    def knnMatch(self, d1, d2, k=2):
        d1 = np.asarray(d1, np.uint8)
        d2 = np.asarray(d2, np.uint8)
        if len(d2) == 0:
            return [[] for _ in range(len(d1))]
        ham = np.unpackbits(d1[:, None, :] ^ d2[None, :, :], axis=2).sum(axis=2)
        out = []
        for i in range(len(d1)):
            order = np.lexsort((np.arange(len(d2)), ham[i]))[:k]
            out.append([_DMatch(i, int(j), ham[i, j]) for j in order])
        return out


def _stub_cv2():
    cv2 = types.ModuleType("cv2")
    cv2.FlannBasedMatcher = _ExactMatcher
    cv2.FM_LMEDS = 4
    cv2.COLOR_GRAY2BGR = 8
    cv2.LINE_AA = 16
    cv2.findFundamentalMat = lambda a, b, m: (np.eye(3), np.ones((len(a), 1), np.uint8))
    cv2.cvtColor = lambda img, code: img
    cv2.circle = lambda *a, **k: None
    cv2.imshow = lambda *a, **k: None
    cv2.waitKey = lambda *a, **k: None
    return cv2


def import_reference():
    sys.modules["cv2"] = _stub_cv2()
    if not hasattr(np, "float"):
        np.float = float  # reference uses np.float (removed in numpy>=1.24)
    sys.path.insert(0, REF)
    import Point3D  # noqa: E402
    import keypoint  # noqa: E402
    import tracking  # noqa: E402
    return Point3D, keypoint, tracking


def import_export_modules():
    import XXXport_files  # noqa: E402  (numpy + scipy Rotation only)
    import keyframe  # noqa: E402
    return XXXport_files, keyframe


def bal_namespace():
    """Execute the BAL block (BundleAdjustment.py lines 231-465) from source text."""
    from scipy.optimize import least_squares
    from scipy.sparse import lil_matrix

    lines = open(os.path.join(REF, "BundleAdjustment.py")).read().splitlines()
    assert lines[229].strip() == '"""' and lines[465].strip() == '"""', "BAL block moved"
    src = "\n".join(lines[230:465])
    ns = {"np": np, "lil_matrix": lil_matrix, "least_squares": least_squares,
          "__name__": "bal_block"}
    exec(compile(src, "BundleAdjustment.py[231:465]", "exec"), ns)
    return ns


# --------------------------------------------------------------------------- synthetic inputs
def descriptor_sets(rng, nq, nt, frac_planted=0.6, flip_p=0.08, n_dups=0):
    t = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    if n_dups:
        src = rng.choice(nt, n_dups, replace=False)
        dst = rng.choice(np.setdiff1d(np.arange(nt), src), n_dups, replace=False)
        t[dst] = t[src]
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    planted = rng.random(nq) < frac_planted
    src = rng.integers(0, nt, nq)
    bits = np.unpackbits(t[src], axis=1)
    flips = (rng.random(bits.shape) < flip_p).astype(np.uint8)
    noisy = np.packbits(bits ^ flips, axis=1)
    q[planted] = noisy[planted]
    return q, t


def rodrigues(r):
    th = np.linalg.norm(r)
    if th == 0:
        return np.eye(3)
    k = r / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def ba_problem(rng, n_cams, n_pts, obs_per_pt, project, f=716.8, noise=0.5):
    """Cameras move along -z (BAL: camera looks down -z, BundleAdjustment.py:323)."""
    C = np.stack([rng.normal(0, 0.05, n_cams), rng.normal(0, 0.05, n_cams),
                  -np.arange(n_cams, dtype=float)], 1)
    rot = rng.normal(0, 0.02, (n_cams, 3))
    cams = np.zeros((n_cams, 9))
    for c in range(n_cams):
        R = rodrigues(rot[c])
        cams[c, :3] = rot[c]
        cams[c, 3:6] = -R @ C[c]
        cams[c, 6] = f
    anchor = rng.integers(0, n_cams - obs_per_pt + 1, n_pts)
    depth = rng.uniform(8.0, 60.0, n_pts)
    X = C[anchor] + np.stack([rng.uniform(-0.4, 0.4, n_pts) * depth,
                              rng.uniform(-0.25, 0.25, n_pts) * depth, -depth], 1)
    cam_idx = (anchor[:, None] + np.arange(obs_per_pt)[None, :]).ravel()
    pt_idx = np.repeat(np.arange(n_pts), obs_per_pt)
    perm = rng.permutation(len(cam_idx))  # the reference does not sort observations
    cam_idx, pt_idx = cam_idx[perm], pt_idx[perm]
    qs = project(X[pt_idx], cams[cam_idx]) + rng.normal(0, noise, (len(cam_idx), 2))
    return cams, X, cam_idx.astype(np.int64), pt_idx.astype(np.int64), qs


def perturb(rng, cams, X, rot_s=1e-3, t_s=1e-2, p_s=0.05):
    c = cams.copy()
    c[:, :3] += rng.normal(0, rot_s, c[:, :3].shape)
    c[:, 3:6] += rng.normal(0, t_s, c[:, 3:6].shape)
    return c, X + rng.normal(0, p_s, X.shape)


# --------------------------------------------------------------------------- goldens
def make_matcher_goldens(Point3D, keypoint, tracking):
    rng = np.random.default_rng(20240601)
    out = {}
    # A: stereo-style L->R (keypoint.py:35) + temporal 2D-3D (Point3D.py:33) + get_matches
    nL, nR, nN = 300, 320, 400
    desL, desR = descriptor_sets(rng, nL, nR, n_dups=12)
    ptsL = rng.uniform(0, [1280, 720], (nL, 2)).astype(np.float32)
    ptsR = rng.uniform(0, [1280, 720], (nR, 2)).astype(np.float32)
    kpL = [_KeyPoint(*p) for p in ptsL]
    kpR = [_KeyPoint(*p) for p in ptsR]
    img = np.zeros((4, 4), np.uint8)
    with contextlib.redirect_stdout(io.StringIO()):
        pl, pr, dl, dr = keypoint.track_keypoints_left_to_right_new(kpL, desL, kpR, desR, img, img)
    out.update(stereo_desL=desL, stereo_desR=desR, stereo_ptsL=ptsL, stereo_ptsR=ptsR,
               stereo_out_ptsL=pl, stereo_out_ptsR=pr, stereo_out_desL=dl, stereo_out_desR=dr)

    M = len(pl)
    des_i1, _ = descriptor_sets(rng, nN, M)
    # plant some true temporal matches so the ratio test passes often
    des_i1[:M // 2] = dl[rng.permutation(M)[:M // 2]] if M >= 2 else des_i1[:M // 2]
    pts_i1 = rng.uniform(0, [1280, 720], (nN, 2)).astype(np.float32)
    kp_i1 = [_KeyPoint(*p) for p in pts_i1]
    Q = rng.normal(0, 300, (M, 3))  # ~10% rows fail the |Q| < 500 gate per axis
    q2, Q1, q1 = Point3D.find_2D_and_3D_correspondenses(dl, pl, kp_i1, des_i1, Q, max_Distance=500)
    out.update(temporal_des_i=dl, temporal_pts_i=pl, temporal_des_i1=des_i1,
               temporal_pts_i1=pts_i1, temporal_Q=Q, temporal_out_q2=np.asarray(q2),
               temporal_out_Q1=np.asarray(Q1), temporal_out_q1=np.asarray(q1))

    g1, g2 = tracking.get_matches(kpL, desL, kpR, desR)
    out.update(getm_out_q1=g1, getm_out_q2=g2)

    # B: train set with a single row -> ValueError truncation -> no matches
    q2b, Q1b, q1b = Point3D.find_2D_and_3D_correspondenses(
        dl[:10], pl[:10], kp_i1[:1], des_i1[:1], Q[:10], max_Distance=500)
    out.update(trunc_out_len=np.array([len(q2b), len(Q1b), len(q1b)]))
    # pure-numpy helpers of Point3D.py (:5-10, :22-30) on the triangulated-point shape
    Qr = rng.normal(0, 40, (200, 3))
    pose = np.eye(4)
    pose[:3, :3] = np.linalg.qr(rng.normal(size=(3, 3)))[0]
    pose[:3, 3] = rng.normal(0, 5, 3)
    out.update(abs_in=Qr, abs_pose=pose, abs_out=Point3D.relative_to_abs3DPoints(Qr, pose))
    close, far = Point3D.sort_3D_points(Qr, 70)
    out.update(sort_close=np.array(close), sort_far=np.array(far))
    np.savez_compressed(os.path.join(OUT, "matcher_golden.npz"), **out)
    return {k: np.shape(v) for k, v in out.items()}


def make_ba_goldens(ns):
    rng = np.random.default_rng(7)
    project, objective = ns["project"], ns["objective"]
    out = {}
    # residual case: 6 cams x 300 pts x 4 obs; cam 0 has a zero rotation vector
    cams, X, ci, pi, qs = ba_problem(rng, 6, 300, 4, project)
    cams[0, :3] = 0.0
    cams0, X0 = perturb(rng, cams, X)
    # clamp triggers: observation far from its projection on x, then on y
    qs = qs.copy()
    qs[3, 0] += 9000.0                  # |r_x| > 5000 (BundleAdjustment.py:339-343)
    qs[5, 1] -= 7000.0                  # |r_y| > 5000 (:347-350)
    qs[8, 0] -= 6000.0
    qs[8, 1] += 20000.0                 # both; second clamp sees the first rescale
    params = np.hstack((cams0.ravel(), X0.ravel()))
    with contextlib.redirect_stdout(io.StringIO()):
        r = objective(params, 6, 300, ci, pi, qs)
    out.update(res_cams=cams0, res_pts=X0, res_cam_idx=ci, res_pt_idx=pi, res_qs=qs, res_out=r)
    out.update(rot_in_pts=X0[:50], rot_in_vecs=np.vstack([np.zeros((1, 3)), cams0[1:, :3],
                                                           rng.normal(0, 1.0, (44, 3))]))
    out.update(rot_out=ns["rotate"](out["rot_in_pts"], out["rot_in_vecs"]))
    A = ns["bundle_adjustment_sparsity"](6, 300, ci, pi).tocoo()
    order = np.lexsort((A.col, A.row))
    out.update(sp_rows=A.row[order].astype(np.int64), sp_cols=A.col[order].astype(np.int64),
               sp_shape=np.array(A.shape))

    # solver case: small local-BA problem, reference settings and tight tolerances
    from scipy.optimize import least_squares
    cams, X, ci, pi, qs = ba_problem(rng, 5, 120, 4, project)
    cams0, X0 = perturb(rng, cams, X)
    A = ns["bundle_adjustment_sparsity"](5, 120, ci, pi)
    with contextlib.redirect_stdout(io.StringIO()):
        r0, rf, xf = ns["bundle_adjustment_with_sparsity"](cams0, X0, ci, pi, qs, A)
        p0 = np.hstack((cams0.ravel(), X0.ravel()))
        tight = least_squares(objective, p0, jac_sparsity=A, x_scale="jac", method="trf",
                              ftol=1e-15, xtol=1e-15, gtol=1e-15, max_nfev=2000,
                              args=(5, 120, ci, pi, qs))
    out.update(sol_cams0=cams0, sol_pts0=X0, sol_cam_idx=ci, sol_pt_idx=pi, sol_qs=qs,
               sol_gt_cams=cams, sol_gt_pts=X,
               sol_ref_r0=r0, sol_ref_rf=rf, sol_ref_x=xf,
               sol_tight_x=tight.x, sol_tight_cost=np.array(tight.cost),
               sol_tight_nfev=np.array(tight.nfev))
    np.savez_compressed(os.path.join(OUT, "ba_golden.npz"), **out)
    return {k: np.shape(v) for k, v in out.items()}


def make_mapping_goldens(Point3D, keypoint, xport, keyframe):
    """A 6-frame sequence through appendKeyPoints (threshold 0.01, main.py:125)
    with re-observed landmarks (inside and outside the 1 % gate) and new ones,
    then export_data of the accumulated problem."""
    import tempfile

    rng = np.random.default_rng(31)
    world = np.stack([rng.uniform(-15, 15, 400), rng.uniform(-3, 3, 400), rng.uniform(8, 60, 400)], 1)
    out = {}
    Qs = np.empty((0, 3))
    opt = np.empty((0, 4))
    frames = [keyframe.KeyFrame(np.eye(4))]
    for i in range(6):
        yaw = 0.01 * i
        pose = np.eye(4)
        pose[:3, :3] = np.array([[np.cos(yaw), 0, np.sin(yaw)], [0, 1, 0], [-np.sin(yaw), 0, np.cos(yaw)]])
        pose[:3, 3] = [0.1 * i, 0.0, 1.0 * i]
        n = 70 + 5 * i
        pick = rng.choice(len(world), n, replace=False)
        Xw = world[pick] + rng.normal(0, 1, (n, 1)) * rng.choice([0.002, 0.05, 2.0], (n, 1)) * 0.1
        rel = (Xw - pose[:3, 3]) @ pose[:3, :3]  # camera coordinates of frame i
        absP = Point3D.relative_to_abs3DPoints(rel, pose)
        pts2d = rng.uniform([0, 0], [1226, 370], (n, 2))
        out[f"f{i}_Qs_in"] = Qs.copy()
        out[f"f{i}_rel"] = rel
        out[f"f{i}_pose"] = pose
        out[f"f{i}_abs"] = absP
        out[f"f{i}_pts2d"] = pts2d
        Qs, rows = keypoint.appendKeyPoints(Qs, absP, 0.01, pts2d, i, rel)
        out[f"f{i}_Qs_out"] = Qs
        out[f"f{i}_rows"] = rows
        opt = np.vstack((opt, rows))
        frames.append(keyframe.KeyFrame(pose))
    P_left = np.array([[718.856, 0, 607.1928, 0], [0, 718.856, 185.2157, 0], [0, 0, 1, 0]])
    out["P_left"] = P_left
    out["frame_poses"] = np.stack([f.pose for f in frames])
    out["cam_params"] = xport.make_cam_params(frames, P_left)
    out["Qs_for_BA"] = xport.make_Qs_for_BA(Qs)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            os.mkdir("ourCache")
            xport.export_data(opt, frames, Qs, P_left)
            out["ba_file"] = np.frombuffer(open("ourCache/BA_file.txt", "rb").read(), np.uint8)
            out["cam_frames_file"] = np.frombuffer(open("ourCache/cam_frames.txt", "rb").read(),
                                                   np.uint8)
        finally:
            os.chdir(cwd)
    np.savez_compressed(os.path.join(OUT, "mapping_golden.npz"), **out)
    return {"frames": 6, "map": len(Qs), "obs": len(opt)}


def main():
    Point3D, keypoint, tracking = import_reference()
    print("matcher:", make_matcher_goldens(Point3D, keypoint, tracking))
    xport, keyframe = import_export_modules()
    print("mapping:", make_mapping_goldens(Point3D, keypoint, xport, keyframe))
    print("ba:", make_ba_goldens(bal_namespace()))


if __name__ == "__main__":
    main()

"""Gather / triangulation / PnP: oracle pinning (CPU) and HIP parity (GPU).

Reference: Point3D.py:5-30, keypoint.py:53-57, transformation.py:5-37.
Tolerances: gather bit-exact; triangulated X rel 1e-9 (GPU one-sided Jacobi vs
numpy LAPACK SVD, both backward stable on the 4x4 DLT system); PnP: the same
hypotheses and inlier counts, final pose within 1e-8 (f64 LM on the same
inlier set, reductions in different order).
"""
import os

import numpy as np
import pytest

from oracle import geometry as og


def _scene(seed, n=400, outliers=0.2, noise=0.5, large=False):
    from slam355.synthetic import StereoRig

    rig = StereoRig(1280, 720)
    rng = np.random.default_rng(seed)
    Q = np.stack([rng.uniform(-10, 10, n), rng.uniform(-3, 3, n), rng.uniform(5, 60, n)], 1)
    r = np.array([0.002, 0.01, -0.003]) * (1 + seed % 3)
    t = np.array([0.02, -0.01, -1.0])
    if large:  # loop-closure-sized motion (0.5 rad, 5 m) in the camera frame
        r = np.array([0.1, 0.48, -0.12]) * (1 + 0.1 * (seed % 3))
        t = np.array([3.0, -1.0, 3.5])
        Xc = np.stack([rng.uniform(-12, 12, n), rng.uniform(-4, 4, n), rng.uniform(6, 60, n)], 1)
        Q = (Xc - t) @ og.rodrigues(r)  # R^T (Xc - t): world points seen in front
    Xc = Q @ og.rodrigues(r).T + t
    q = Xc[:, :2] / Xc[:, 2:3] * rig.K[0, 0] + rig.K[:2, 2] + rng.normal(0, noise, (n, 2))
    k = int(outliers * n)
    q[:k] += rng.uniform(-120, 120, (k, 2))
    return rig, Q, q, r, t


# ----------------------------------------------------------------------------- CPU
def test_point3d_helpers_match_reference(golden_dir):
    g = np.load(os.path.join(golden_dir, "matcher_golden.npz"))
    assert np.array_equal(og.relative_to_abs3DPoints(g["abs_in"], g["abs_pose"]), g["abs_out"])
    close, far = og.sort_3D_points(g["abs_in"], 70)
    assert np.array_equal(close, g["sort_close"]) and np.array_equal(far, g["sort_far"])


def test_oracle_triangulation_exact_stereo():
    rig, Q, _, _, _ = _scene(0, outliers=0, noise=0)
    ql = Q[:, :2] / Q[:, 2:3] * rig.K[0, 0] + rig.K[:2, 2]
    Qr = Q - [rig.baseline, 0, 0]
    qr = Qr[:, :2] / Qr[:, 2:3] * rig.K[0, 0] + rig.K[:2, 2]
    X = og.triangulate_points_local(ql, qr, rig.P_l, rig.P_r)
    assert np.allclose(X, Q, rtol=1e-9, atol=1e-9)


def test_oracle_pnp_recovers_pose_with_outliers():
    rig, Q, q, r, t = _scene(1)
    rv, tv, n, mask = og.pnp_ransac(Q, q, rig.K, seed=3, item=7)
    assert n >= 0.75 * len(Q) and mask[:80].sum() == 0
    assert np.abs(rv - r).max() < 2e-4 and np.abs(tv - t).max() < 5e-3
    # deterministic
    rv2, tv2, n2, m2 = og.pnp_ransac(Q, q, rig.K, seed=3, item=7)
    assert np.array_equal(rv, rv2) and np.array_equal(tv, tv2) and n == n2


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_oracle_pnp_large_motion_epnp_seed(seed):
    """0.5 rad / 5 m motion, 20 % outliers: hypotheses seeded by EPnP (the
    RANSAC kernel OpenCV's solvePnPRansac uses for ITERATIVE) recover the pose."""
    rig, Q, q, r, t = _scene(seed, n=300, large=True)
    rv, tv, n, mask = og.pnp_ransac(Q, q, rig.K, seed=5, item=seed)
    assert n >= 0.75 * len(Q)
    assert np.allclose(rv, r, atol=2e-3) and np.allclose(tv, t, atol=5e-2)
    assert mask[int(0.2 * len(Q)):].mean() > 0.95


def test_oracle_epnp_exact_points():
    rng = np.random.default_rng(3)
    K = np.array([[716.8, 0, 640], [0, 716.8, 360], [0, 0, 1.0]])
    for _ in range(20):
        r, t = rng.normal(0, 0.6, 3), rng.normal(0, 4, 3)
        Xc = np.stack([rng.uniform(-10, 10, 5), rng.uniform(-5, 5, 5), rng.uniform(5, 60, 5)], 1)
        Xw = (Xc - t) @ og.rodrigues(r)
        uv = Xc[:, :2] / Xc[:, 2:3] * 716.8 + [640, 360]
        p = og.epnp(Xw, uv, K)
        assert p is not None
        assert np.allclose(og.rodrigues(p[:3]), og.rodrigues(r), atol=1e-9)
        assert np.allclose(p[3:], t, atol=1e-8 * (1 + np.abs(t).max()))


def test_oracle_pnp_guard_and_pose_sign_convention():
    rig, Q, q, _, _ = _scene(2, n=4)
    rv, tv, n, mask = og.pnp_ransac(Q, q, rig.K)
    assert n == -1  # len(Q) <= 4: the caller keeps the previous T (main.py:94-98)
    T, r, t = og.pose_matrix_from_pnp(np.array([0.1, -0.2, 0.05]), np.array([1.0, 2.0, 3.0]))
    assert np.allclose(T[:3, 3], [-1, -2, -3]) and np.allclose(r.ravel(), [-0.1, 0.2, -0.05])
    assert np.allclose(T[:3, :3], og.rodrigues([-0.1, 0.2, -0.05]))


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_gather_bit_exact():
    import torch
    from slam355 import geometry

    rng = np.random.default_rng(4)
    B, kc, pc = 3, 500, 300
    kpq = rng.uniform(0, 1000, (B, kc, 5)).astype(np.float32)
    kpt = rng.uniform(0, 1000, (B, kc, 5)).astype(np.float32)
    dq = rng.integers(0, 256, (B, kc, 32), dtype=np.uint8)
    dt = rng.integers(0, 256, (B, kc, 32), dtype=np.uint8)
    pairs = rng.integers(0, kc, (B, pc, 2)).astype(np.int32)
    cnt = np.array([300, 17, 0], np.int32)
    T = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    a, b, c, d = geometry.gather_matches(T(kpq), T(kpt), T(pairs), T(cnt), T(dq), T(dt))
    for i in range(B):
        n = cnt[i]
        p = pairs[i, :n]
        assert np.array_equal(a[i, :n].cpu().numpy(), kpq[i, p[:, 0], :2].astype(np.float64))
        assert np.array_equal(b[i, :n].cpu().numpy(), kpt[i, p[:, 1], :2].astype(np.float64))
        assert np.array_equal(c[i, :n].cpu().numpy(), dq[i, p[:, 0]])
        assert np.array_equal(d[i, :n].cpu().numpy(), dt[i, p[:, 1]])


@pytest.mark.gpu
def test_gpu_triangulation_vs_svd():
    from slam355 import Point3D

    for seed in range(3):
        rig, Q, _, _, _ = _scene(seed, outliers=0, noise=0)
        rng = np.random.default_rng(seed)
        ql = Q[:, :2] / Q[:, 2:3] * rig.K[0, 0] + rig.K[:2, 2] + rng.normal(0, 0.7, (len(Q), 2))
        Qr = Q - [rig.baseline, 0, 0]
        qr = Qr[:, :2] / Qr[:, 2:3] * rig.K[0, 0] + rig.K[:2, 2] + rng.normal(0, 0.7, (len(Q), 2))
        X = Point3D.triangulate_points_local(ql, qr, rig.P_l, rig.P_r)
        E = og.triangulate_points_local(ql, qr, rig.P_l, rig.P_r)
        assert np.all(np.abs(X - E) <= 1e-9 * np.maximum(1.0, np.abs(E)))
    # arbitrary projection matrices / noise-only points
    P1 = rng.normal(size=(3, 4))
    P2 = rng.normal(size=(3, 4))
    a, b = rng.normal(size=(50, 2)), rng.normal(size=(50, 2))
    X = Point3D.triangulate_points_local(a, b, P1, P2)
    E = og.triangulate_points_local(a, b, P1, P2)
    assert np.all(np.abs(X - E) <= 1e-7 * np.maximum(1.0, np.abs(E)))


@pytest.mark.gpu
def test_gpu_pnp_matches_oracle():
    import torch
    from slam355 import geometry

    B = 4
    scenes = [_scene(s, n=150 + 100 * s) for s in range(B)]
    cap = max(len(s[1]) for s in scenes)
    Q = np.zeros((B, cap, 3))
    q = np.zeros((B, cap, 2))
    cnt = np.zeros(B, np.int32)
    for i, (rig, Qi, qi, _, _) in enumerate(scenes):
        Q[i, :len(Qi)], q[i, :len(qi)], cnt[i] = Qi, qi, len(Qi)
    cnt[3] = 4  # guard path
    K = scenes[0][0].K
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    rv, tv, n, mask = geometry.pnp_ransac(T(Q), T(q), T(cnt), K, seed=11, item0=100)
    rv, tv, n, mask = rv.cpu().numpy(), tv.cpu().numpy(), n.cpu().numpy(), mask.cpu().numpy()
    for i in range(B):
        L = cnt[i]
        erv, etv, en, emask = og.pnp_ransac(Q[i, :L], q[i, :L], K, seed=11, item=100 + i)
        assert n[i] == en, i
        if en < 0:
            continue
        assert np.array_equal(mask[i, :L].astype(bool), emask), i
        assert np.allclose(rv[i], erv, rtol=0, atol=1e-8) and np.allclose(tv[i], etv, atol=1e-8), i


@pytest.mark.gpu
def test_gpu_pnp_large_motion_matches_oracle():
    """EPnP-seeded hypotheses on the GPU (k_pnp_hyp) equal the oracle's on
    loop-closure-sized motion with outliers: counts, masks, pose 1e-8."""
    import torch
    from slam355 import geometry

    B = 3
    scenes = [_scene(s, n=250, large=True) for s in range(B)]
    cap = 250
    Q = np.stack([s[1] for s in scenes])
    q = np.stack([s[2] for s in scenes])
    cnt = np.full(B, cap, np.int32)
    K = scenes[0][0].K
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    rv, tv, n, mask = geometry.pnp_ransac(T(Q), T(q), T(cnt), K, seed=4, item0=20)
    rv, tv, n, mask = rv.cpu().numpy(), tv.cpu().numpy(), n.cpu().numpy(), mask.cpu().numpy()
    for i in range(B):
        erv, etv, en, emask = og.pnp_ransac(Q[i], q[i], K, seed=4, item=20 + i)
        assert n[i] == en, i
        assert np.array_equal(mask[i].astype(bool), emask), i
        assert np.allclose(rv[i], erv, rtol=0, atol=1e-8) and np.allclose(tv[i], etv, atol=1e-8), i
        assert np.allclose(tv[i], scenes[i][4], atol=5e-2)


@pytest.mark.gpu
def test_gpu_reference_api_mirrors():
    from slam355 import transformation

    rig, Q, q, r, t = _scene(5)
    T, rvec, tvec = transformation.calculate_transformation_matrix(Q, q, None, None, rig.K,
                                                                   seed=2, frame=9)
    erv, etv, _, _ = og.pnp_ransac(Q, q, rig.K, seed=2, item=9)
    ET, er, et = og.pose_matrix_from_pnp(erv, etv)
    assert rvec.shape == (3, 1) and tvec.shape == (3, 1)
    assert np.allclose(T, ET, atol=1e-8) and np.allclose(rvec, er, atol=1e-8)


def _stereo_points(seed, n=300, outliers=0.3):
    from slam355.synthetic import StereoRig

    rig = StereoRig(1280, 720)
    rng = np.random.default_rng(seed)
    Q = np.stack([rng.uniform(-15, 15, n), rng.uniform(-3, 3, n), rng.uniform(5, 80, n)], 1)
    pl = Q[:, :2] / Q[:, 2:3] * rig.K[0, 0] + rig.K[:2, 2] + rng.normal(0, 0.4, (n, 2))
    Qr = Q - [rig.baseline, 0, 0]
    pr = Qr[:, :2] / Qr[:, 2:3] * rig.K[0, 0] + rig.K[:2, 2] + rng.normal(0, 0.4, (n, 2))
    k = int(outliers * n)
    pr[:k] = rng.uniform([0, 0], [1280, 720], (k, 2))
    return pl, pr


def test_oracle_fundamental_lmeds_rejects_outliers():
    pl, pr = _stereo_points(0)
    mask, F, n, med = og.fundamental_lmeds(pl, pr, seed=1, item=3)
    assert mask[:90].sum() <= 3 and mask[90:].mean() > 0.9
    # epipolar constraint holds on inliers: median point-to-epipolar-line distance
    # in the right image at the 0.4 px noise level
    h1 = np.hstack([pl, np.ones((len(pl), 1))])[mask]
    h2 = np.hstack([pr, np.ones((len(pr), 1))])[mask]
    lines = h1 @ F.T
    d = np.abs(np.sum(lines * h2, 1)) / np.hypot(lines[:, 0], lines[:, 1])
    assert np.median(d) < 1.0
    m2, F2, n2, _ = og.fundamental_lmeds(pl[:7], pr[:7])
    assert n2 == -1 and not m2.any()  # < 8 points: no model, nothing kept


@pytest.mark.gpu
def test_gpu_fundamental_lmeds_matches_oracle():
    import torch
    from slam355 import geometry

    B, cap = 4, 400
    m1 = np.zeros((B, cap, 2))
    m2 = np.zeros((B, cap, 2))
    cnt = np.array([300, 120, 7, 399], np.int32)
    for b in range(B):
        a, c = _stereo_points(10 + b, n=int(cnt[b]), outliers=0.1 * b)
        m1[b, :cnt[b]], m2[b, :cnt[b]] = a, c
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    mask, F, n = geometry.fundamental_lmeds(T(m1), T(m2), T(cnt), seed=9, item0=20)
    mask, n = mask.cpu().numpy(), n.cpu().numpy()
    for b in range(B):
        em, eF, en, _ = og.fundamental_lmeds(m1[b, :cnt[b]], m2[b, :cnt[b]], seed=9, item=20 + b)
        assert n[b] == en, b
        assert np.array_equal(mask[b, :cnt[b]].astype(bool), em), b
    # order-preserving filter of the pairs by that mask
    pairs = np.stack([np.arange(cap), cap - np.arange(cap)], 1)[None].repeat(B, 0).astype(np.int32)
    fp, fc = geometry.filter_pairs(T(pairs), T(cnt), T(mask))
    fp, fc = fp.cpu().numpy(), fc.cpu().numpy()
    for b in range(B):
        keep = mask[b, :cnt[b]].astype(bool)
        assert fc[b] == keep.sum() and np.array_equal(fp[b, :fc[b]], pairs[b, :cnt[b]][keep])

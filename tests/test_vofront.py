"""LK / SGBM stereo-VO front end: FAST on tiles, pyramidal
LK, SGBM, calculate_right_qs + calc_3d, and the whole get_pose chain.

CPU tests pin the oracle (oracle/vofront.c + oracle/vofront.py) against the
goldens produced by the reference's own VisualOdometry / keypoint methods
(tests/golden/make_vofront_goldens.py) and check the restated OpenCV
primitives on inputs with known answers.  GPU tests require bit-exact equality
of the HIP kernels with the oracle (FAST keypoints, LK points / status / error,
SGBM disparities, filtered and looked-up points); float32 triangulation is
within 4 ulp of each point's largest coordinate (f64 Jacobi null vector vs
LAPACK SVD before the float32 rounding); poses within 1e-6.  OpenCV itself: parity unpinned.
"""
import os

import numpy as np
import pytest

from oracle import vofront as vf

GOLD = os.path.join(os.path.dirname(__file__), "golden", "vofront_golden.npz")


@pytest.fixture(scope="module")
def g():
    return np.load(GOLD)


def _frames(n, W, H, seed, n_landmarks=500):
    from slam355.synthetic import stereo_sequence

    return stereo_sequence(n, W, H, seed=seed, n_landmarks=n_landmarks)


# ------------------------------------------------------------------ CPU: oracle
@pytest.mark.parametrize("case", ["seq", "shift"])
def test_oracle_glue_matches_reference_goldens(g, case):
    G = lambda k: g[f"{case}_{k}"]  # noqa: E731
    i1, i2, r1, r2 = G("img1"), G("img2"), G("right1"), G("right2")
    kp = vf.fast_tiles(i1)
    assert np.array_equal(kp, G("kp"))
    tp1, tp2 = vf.track_keypoints(i1, i2, kp[:, :2])
    assert np.array_equal(tp1, G("tp1")) and np.array_equal(tp2, G("tp2"))
    d1, d2 = vf.disparity_f32(i1, r1), vf.disparity_f32(i2, r2)
    assert np.array_equal(d1, G("disp1")) and np.array_equal(d2, G("disp2"))
    q = vf.calculate_right_qs(tp1, tp2, d1, d2)
    for k, v in zip(("q1_l", "q1_r", "q2_l", "q2_r"), q):
        assert v.dtype == np.float32 and np.array_equal(v, G(k)), k
    Q1, Q2 = vf.calc_3d(*q, G("P_l"), G("P_r"))
    assert Q1.dtype == np.float32 and np.array_equal(Q1, G("Q1")) and np.array_equal(Q2, G("Q2"))
    a, d, b = vf.track_keypoints_left_to_right(i1, r1, kp[:, :2], G("des"))
    assert np.array_equal(a, G("lr_tp1")) and np.array_equal(d, G("lr_des"))
    assert np.array_equal(b, G("lr_tp2"))


def test_oracle_right_qs_negative_wrap_golden(g):
    G = lambda k: g[f"wrap_{k}"]  # noqa: E731
    out = vf.calculate_right_qs(G("q1"), G("q2"), G("disp1"), G("disp2"))
    for k, v in zip(("q1_l", "q1_r", "q2_l", "q2_r"), out):
        assert np.array_equal(v, G(k)), k
    assert (G("q2")[:, 0] < 0).sum() > 0


def test_oracle_pyramid_and_scharr_known_answers():
    img = np.full((37, 50), 77, np.uint8)
    assert np.array_equal(vf.pyr_down(img), np.full((19, 25), 77, np.uint8))
    ramp = np.tile(np.arange(60, dtype=np.uint8) * 3, (40, 1))
    d = vf.scharr(ramp)
    assert (d[:, 1:-1, 0] == 96).all() and (d[:, :, 1] == 0).all()  # 2*3*16, no vertical change
    assert (d[:, 0, 0] == 0).all() and (d[:, -1, 0] == 0).all()      # reflect-101 columns
    assert vf.lk_levels(1280, 720) == [(1280, 720), (640, 360), (320, 180), (160, 90)]
    assert vf.lk_levels(40, 40) == [(40, 40), (20, 20)]


def test_oracle_lk_recovers_integer_translation():
    L, _, _, _ = _frames(1, 320, 240, seed=21)
    a = L[0]
    b = np.zeros_like(a)
    b[2:, :-3] = a[:-2, 3:]  # content moves by (-3, +2)
    kp = vf.fast_tiles(a)
    m = (kp[:, 0] > 40) & (kp[:, 0] < 280) & (kp[:, 1] > 40) & (kp[:, 1] < 200)
    p2, st, err = vf.calc_optical_flow_pyr_lk(a, b, kp[m, :2])
    ok = (st > 0) & (err < 4)
    assert ok.mean() > 0.8
    dv = p2[ok] - kp[m, :2][ok]
    assert np.median(np.abs(dv - [-3, 2]), 0).max() < 0.05


def test_oracle_sgbm_recovers_constant_disparity():
    rng = np.random.default_rng(3)
    base = (rng.random((60, 140)) * 255).astype(np.uint8)
    base = np.kron(base, np.ones((2, 2), np.uint8))[:, :260]  # 120 x 260 texture
    left = base[:, 9:209].copy()
    right = base[:, 18:218].copy()  # left x == right x + 9
    d = vf.sgbm_compute(left, right)
    valid = d[:, 40:190] > 0
    assert valid.mean() > 0.9
    assert np.median(d[:, 40:190][valid]) == 9 * 16
    assert (d[:, :30] == -16).all()  # x < numDisparities: invalid


def test_oracle_fast_tiles_caps_and_order():
    rng = np.random.default_rng(9)
    img = rng.integers(0, 256, (40, 60), dtype=np.uint8)  # dense corners
    k = vf.fast_tiles(img, 10, 20, 10, 10)
    k_all = vf.fast_tiles(img, 10, 20, 10, 1000)
    assert len(k) < len(k_all)
    ti = lambda a: (a[:, 1] // 10) * 3 + a[:, 0] // 20  # noqa: E731
    assert np.all(np.diff(ti(k)) >= 0)  # tiles row-major
    for t in np.unique(ti(k_all)):
        full = k_all[ti(k_all) == t]
        kept = k[ti(k) == t]
        if len(full) > 10:
            assert len(kept) == 10
            order = np.argsort(-full[:, 2], kind="stable")[:10]
            assert np.array_equal(kept, full[order])
        else:
            assert np.array_equal(kept, full)


# ------------------------------------------------------------------ GPU
def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def test_wrappers_reject_image_indices_outside_the_tensors():
    """lk_track / right_qs_3d check their image ranges on the host before any
    launch (the kernels index prev0 + b*pair_stride and disp1_index + b +
    disp2_offset directly)."""
    import types

    import torch

    from slam355 import vofront

    B, cap = 3, 8
    pts = torch.zeros((B, cap, 2))
    npts = torch.zeros(B, dtype=torch.int32)
    pyr = types.SimpleNamespace(pyr=torch.zeros((4, 16)), der=torch.zeros((4, 16, 2)), H=8, W=8,
                                win=5, max_level=1)
    with pytest.raises(IndexError):  # next images 1..3 exist, 2..4 do not
        vofront.lk_track(pyr, pyr, pts, npts, prev0=0, next0=2)
    with pytest.raises(IndexError):
        vofront.lk_track(pyr, pyr, pts, npts, prev0=0, next0=1, pair_stride=2)
    with pytest.raises(IndexError):
        vofront.lk_track(pyr, pyr, pts, npts, prev0=-1, next0=0)
    other = types.SimpleNamespace(**{**vars(pyr), "W": 16})
    with pytest.raises(ValueError):
        vofront.lk_track(pyr, other, pts, npts, prev0=0, next0=1)
    disp = torch.zeros((4, 8, 8))
    with pytest.raises(IndexError):  # pairs 0..2 read maps 0..3; offset 2 reads map 4
        vofront.right_qs_3d(pts, pts, npts, disp, np.eye(3, 4), np.eye(3, 4), disp2_offset=2)
    with pytest.raises(IndexError):
        vofront.right_qs_3d(pts, pts, npts, disp, np.eye(3, 4), np.eye(3, 4), disp1_index=1,
                            disp2_offset=1)
    with pytest.raises(IndexError):
        vofront.right_qs_3d(pts, pts, npts, disp, np.eye(3, 4), np.eye(3, 4), disp1_index=1,
                            disp2_offset=-2)


@pytest.mark.gpu
def test_gpu_fast_tiles_bit_exact():
    import torch

    from slam355 import vofront

    L, R, _, _ = _frames(2, 640, 480, seed=22)
    rng = np.random.default_rng(23)
    imgs = np.concatenate([L, R, rng.integers(0, 256, (1, 480, 640), dtype=np.uint8),
                           np.full((1, 480, 640), 100, np.uint8)])
    kp, cnt = vofront.fast_tiles(_dev(imgs))
    for b in range(len(imgs)):
        e = vf.fast_tiles(imgs[b])
        n = int(cnt[b])
        assert n == len(e), b
        assert np.array_equal(kp[b, :n].cpu().numpy(), e), b
    assert int(cnt[-1]) == 0
    # partial edge tiles, other tile shapes and caps
    odd = rng.integers(0, 256, (2, 97, 143), dtype=np.uint8)
    for th, tw, per in ((10, 20, 10), (16, 16, 3), (7, 9, 100)):
        kp, cnt = vofront.fast_tiles(_dev(odd), th, tw, 10, per)
        for b in range(2):
            e = vf.fast_tiles(odd[b], th, tw, 10, per)
            assert np.array_equal(kp[b, :int(cnt[b])].cpu().numpy(), e), (th, tw, per, b)
    L2, _, _, _ = _frames(1, 1280, 720, seed=24)
    kp, cnt = vofront.fast_tiles(_dev(L2))
    e = vf.fast_tiles(L2[0])
    assert int(cnt[0]) == len(e) > 1000
    assert np.array_equal(kp[0, :len(e)].cpu().numpy(), e)
    del torch


@pytest.mark.gpu
def test_gpu_lk_bit_exact():
    import torch

    from slam355 import vofront

    L, _, _, _ = _frames(3, 640, 480, seed=25)
    pts = [vf.fast_tiles(L[i])[:, :2] for i in range(2)]
    # add border / outside points (status paths)
    extra = np.array([[0, 0], [639, 479], [-3.5, 10], [700, 200], [2.25, 477.75], [320.5, 0.1],
                      [1e8, 5.0], [-40.0, -3e7]],
                     np.float32)
    pts = [np.concatenate([p, extra]) for p in pts]
    cap = max(len(p) for p in pts)
    P = np.zeros((2, cap, 2), np.float32)
    for i, p in enumerate(pts):
        P[i, :len(p)] = p
    cnt = torch.tensor([len(p) for p in pts], dtype=torch.int32, device="cuda")
    pyr = vofront.LKPyramids(_dev(L))
    out, st, err = vofront.lk_track(pyr, pyr, _dev(P), cnt, prev0=0, next0=1)
    for i in range(2):
        e2, est, eerr = vf.calc_optical_flow_pyr_lk(L[i], L[i + 1], pts[i])
        n = len(pts[i])
        assert np.array_equal(st[i, :n].cpu().numpy(), est), i
        assert np.array_equal(out[i, :n].cpu().numpy().view(np.uint32), e2.view(np.uint32)), i
        assert np.array_equal(err[i, :n].cpu().numpy().view(np.uint32), eerr.view(np.uint32)), i
        assert est.mean() > 0.8
    # a small image: fewer pyramid levels than maxLevel
    small = L[:2, 100:160, 200:250].copy()
    sp = vf.fast_tiles(small[0])[:, :2]
    pyr = vofront.LKPyramids(_dev(small))
    c1 = torch.tensor([len(sp)], dtype=torch.int32, device="cuda")
    out, st, err = vofront.lk_track(pyr, pyr, _dev(sp[None]), c1, prev0=0, next0=1)
    e2, est, eerr = vf.calc_optical_flow_pyr_lk(small[0], small[1], sp)
    assert pyr.nlev == 2
    assert np.array_equal(out[0].cpu().numpy(), e2) and np.array_equal(st[0].cpu().numpy(), est)
    assert np.array_equal(err[0].cpu().numpy(), eerr)


@pytest.mark.gpu
def test_gpu_sgbm_bit_exact():
    from slam355 import vofront

    L, R, _, _ = _frames(2, 320, 240, seed=26)
    d, df = vofront.sgbm(_dev(L), _dev(R))
    for b in range(2):
        e = vf.sgbm_compute(L[b], R[b])
        assert np.array_equal(d[b].cpu().numpy(), e), b
        assert np.array_equal(df[b].cpu().numpy(), e.astype(np.float32) / 16)
    rng = np.random.default_rng(27)
    noise = rng.integers(0, 256, (2, 70, 150), dtype=np.uint8)   # saturating, inconsistent
    flat = np.full((2, 40, 90), 90, np.uint8)
    tiny = rng.integers(0, 256, (2, 20, 30), dtype=np.uint8)      # W <= numDisparities
    for (l, r), kw in (((noise[:1], noise[1:]), {}),
                       ((flat[:1], flat[1:]), {}),
                       ((tiny[:1], tiny[1:]), {}),
                       ((L[:1, :, :301], R[:1, :, :301]), dict(num_disp=64, block=5, P1=200,
                                                               P2=800)),
                       ((L[:1, :120, :200], R[:1, :120, :200]), dict(block=3)),
                       ((L[:1, :60, :150], R[:1, :60, :150]), dict(block=21)),
                       ((L[:1, :101], R[:1, :101]), dict(min_disp=3, block=7))):
        kw = dict(dict(min_disp=0, num_disp=32, block=11, P1=968, P2=3872), **kw)
        d, _ = vofront.sgbm(_dev(l), _dev(r), **kw, f32=False)
        e = vf.sgbm_compute(l[0], r[0], kw["min_disp"], kw["num_disp"], kw["block"], kw["P1"],
                            kw["P2"])
        assert np.array_equal(d[0].cpu().numpy(), e), (l.shape, kw)


@pytest.mark.gpu
def test_gpu_reference_mirror_matches_goldens(g):
    """The reference's methods (goldens) == slam355.visual_odometry.VisualOdometry /
    keypoint.track_keypoints_left_to_right on the GPU."""
    from slam355 import keypoint
    from slam355.visual_odometry import VisualOdometry

    for case in ("seq", "shift"):
        G = lambda k: g[f"{case}_{k}"]  # noqa: E731, B023
        vo = VisualOdometry([G("img1"), G("img2")], [G("right1"), G("right2")], P_l=G("P_l"),
                            P_r=G("P_r"))
        assert np.array_equal(vo.disparities[0], G("disp1"))
        kps = vo.get_tiled_keypoints(G("img1"), 10, 20)
        kp = np.array([[k.pt[0], k.pt[1], k.response] for k in kps], np.float32)
        assert np.array_equal(kp, G("kp"))
        tp1, tp2 = vo.track_keypoints(G("img1"), G("img2"), kps)
        assert np.array_equal(tp1, G("tp1")) and np.array_equal(tp2, G("tp2"))
        q = vo.calculate_right_qs(tp1, tp2, G("disp1"), G("disp2"))
        for k, v in zip(("q1_l", "q1_r", "q2_l", "q2_r"), q):
            assert np.array_equal(v, G(k)), (case, k)
        Q1, Q2 = vo.calc_3d(*q)
        for a, e in ((Q1, G("Q1")), (Q2, G("Q2"))):
            # within 4 float32 ulp of each point's largest coordinate (a near-zero
            # coordinate carries the f64 null-vector difference, not its own ulp)
            scale = np.abs(e).max(1, keepdims=True)
            assert (np.abs(a - e) <= 4 * np.finfo(np.float32).eps * scale).all(), case
        a, d, b = keypoint.track_keypoints_left_to_right(G("img1"), G("right1"), kps, G("des"))
        assert np.array_equal(a, G("lr_tp1")) and np.array_equal(d, G("lr_des"))
        assert np.array_equal(b, G("lr_tp2"))
        T, Q = vo.get_pose(1)
        assert T.shape == (4, 4) and len(Q) == len(G("q1_l"))


@pytest.mark.gpu
def test_gpu_right_qs_negative_wrap(g):
    import torch

    from slam355 import vofront

    G = lambda k: g[f"wrap_{k}"]  # noqa: E731
    q1, q2 = G("q1"), G("q2")
    disp = _dev(np.stack([G("disp1"), G("disp2")]))
    cnt = torch.tensor([len(q1)], dtype=torch.int32, device="cuda")
    o = vofront.right_qs_3d(_dev(q1[None]), _dev(q2[None]), cnt, disp, np.eye(3, 4),
                            np.eye(3, 4) - [[0, 0, 0, 0.5], [0, 0, 0, 0], [0, 0, 0, 0]])
    m = int(o["count"][0])
    for k in ("q1_l", "q1_r", "q2_l", "q2_r"):
        assert np.array_equal(o[k][0, :m].cpu().numpy(), G(k)), k


@pytest.mark.gpu
def test_gpu_stereo_vo_pipeline_matches_oracle():
    """StereoVO.run (one batched call over 4 frame pairs) == the oracle's get_pose
    chain pair by pair; poses follow the synthetic ground truth."""
    from slam355.vofront import StereoVO

    L, R, poses, rig = _frames(5, 640, 480, seed=28, n_landmarks=600)
    vo = StereoVO(rig.P_l, rig.P_r, seed=7)
    out = vo.run(_dev(L), _dev(R), frame0=1)
    disp = [vf.disparity_f32(L[i], R[i]) for i in range(5)]
    for b in range(4):
        assert np.array_equal(out["disp"][b].cpu().numpy(), disp[b])
        T, Q1, info = vf.get_pose(L[b], L[b + 1], disp[b], disp[b + 1], rig.P_l, rig.P_r, seed=7,
                                  frame=1 + b)
        assert int(out["ntp"][b]) == len(info["tp1"])
        m = int(out["count"][b])
        assert m == len(info["q1_l"]) > 50
        assert np.array_equal(out["q1_l"][b, :m].cpu().numpy(), info["q1_l"])
        assert np.array_equal(out["q2_l"][b, :m].cpu().numpy(), info["q2_l"])
        assert np.allclose(out["Q1"][b, :m].cpu().numpy(), info["Q1"], rtol=1e-6, atol=1e-6)
        dof = out["pose"][b].cpu().numpy()
        assert np.allclose(dof, info["dof"], rtol=1e-6, atol=1e-6)
        gt = np.linalg.inv(poses[b]) @ poses[b + 1]
        assert np.abs(T[:3, 3] - gt[:3, 3]).max() < 0.05

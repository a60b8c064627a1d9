"""Batched tracking pipeline (main.py:76-132) vs the per-frame CPU oracle chain."""
import numpy as np
import pytest

from oracle import pipeline as op


@pytest.fixture(scope="module")
def seq():
    from slam355.synthetic import stereo_sequence

    return stereo_sequence(4, 1280, 720, seed=3)


def test_oracle_chain_recovers_forward_motion(seq):
    L, R, poses, rig = seq
    cache = {}
    for i in range(2):
        out = op.track_pair(L[i], R[i], L[i + 1], rig.P_l, rig.P_r, seed=5, frame=i, orb_cache=cache)
        assert out["n_temporal"] >= 10 and out["n_pnp"] >= 10
        # true relative motion: frame i+1 is 1 m ahead -> points move by -1 m in z
        rel = np.linalg.inv(poses[i + 1]) @ poses[i]
        assert np.allclose(out["tvec"], rel[:3, 3], atol=0.05)


def test_chain_poses_reference_semantics():
    from slam355.pipeline import chain_poses, relative_transform

    r = np.array([[0.0, 0.01, 0.0], [0, 0, 0], [0.0, -0.02, 0.001]])
    t = np.array([[0.0, 0.0, -1.0], [1, 1, 1], [0.1, 0.0, -1.0]])
    n = np.array([50, -1, 40])  # frame 1: PnP skipped -> previous T reused (main.py:94-98)
    P, T = chain_poses(np.eye(4), r, t, n)
    T0, T2 = relative_transform(r[0], t[0]), relative_transform(r[2], t[2])
    assert np.allclose(P[0], T0) and np.allclose(P[1], T0 @ T0) and np.allclose(P[2], T0 @ T0 @ T2)
    assert np.allclose(T0[:3, 3], [0, 0, 1.0])  # the sign flip of transformation.py:15-16


@pytest.mark.gpu
def test_gpu_tracker_matches_oracle_chain(seq):
    import torch
    from slam355.pipeline import Tracker

    L, R, poses, rig = seq
    B = 3
    trk = Tracker(B, 720, 1280, rig.P_l, rig.P_r, seed=5)
    trk.imgs.copy_(torch.from_numpy(np.concatenate([L[:B + 1], R[:B]])))
    rv, tv, n = trk.track(0)
    torch.cuda.synchronize()
    c = trk.counters()
    rv, tv, n = rv.cpu().numpy(), tv.cpu().numpy(), n.cpu().numpy()
    cache = {}
    for i in range(B):
        e = op.track_pair(L[i], R[i], L[i + 1], rig.P_l, rig.P_r, seed=5, frame=i, orb_cache=cache)
        assert c["stereo"][i] == e["n_stereo"], i
        assert c["f_inliers"][i] == e["n_f"], i
        assert np.array_equal(trk.f_mask[i, :e["n_stereo"]].cpu().numpy().astype(bool), e["f_mask"])
        X = trk.X[i, :e["n_f"]].cpu().numpy()
        assert np.all(np.abs(X - e["X"]) <= 1e-9 * np.maximum(1, np.abs(e["X"])))
        assert c["temporal"][i] == e["n_temporal"], i
        assert n[i] == e["n_pnp"], i
        assert np.allclose(rv[i], e["rvec"], atol=1e-8) and np.allclose(tv[i], e["tvec"], atol=1e-8)

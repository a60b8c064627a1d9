"""Hamming kNN-2 matcher: oracle pinning (CPU) and HIP parity (GPU).

Reference: keypoint.py:35-66, Point3D.py:33-53, tracking.py:12-34.
The bar is bit-exact: indices, distances and the good mask.
"""
import os

import numpy as np
import pytest

import oracle
from oracle import matching as om


def _sets(rng, nq, nt, dup=0, planted=0.6, flip=0.08):
    t = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    if dup and nt > 1:
        src = rng.integers(0, nt, dup)
        dst = rng.integers(0, nt, dup)
        t[dst] = t[src]
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    if nt:
        pick = rng.random(nq) < planted
        src = rng.integers(0, nt, nq)
        bits = np.unpackbits(t[src], axis=1) ^ (rng.random((nq, 256)) < flip).astype(np.uint8)
        q[pick] = np.packbits(bits, axis=1)[pick]
    return q, t


# ----------------------------------------------------------------------------- CPU
def test_ratio_predicate_integer_form():
    """`m.distance < 0.7 * n.distance` (keypoint.py:48) == 10*d1 < 7*d2 on [0,256]^2."""
    d = np.arange(257)
    ref = d[:, None].astype(np.float32).astype(float) < 0.7 * d[None, :].astype(np.float32).astype(float)
    assert np.array_equal(ref, 10 * d[:, None] < 7 * d[None, :])


@pytest.mark.parametrize("nq,nt,dup", [(37, 53, 10), (64, 2, 0), (5, 1, 0), (0, 8, 0), (9, 0, 0)])
def test_c_oracle_matches_sorted_restatement(nq, nt, dup):
    rng = np.random.default_rng(nq * 1000 + nt)
    q, t = _sets(rng, nq, nt, dup=dup)
    idx2, dist2, good = oracle.hamming_knn2(q, t)
    ref = oracle.hamming_knn2_pylist(q, t)
    for i in range(nq):
        exp = ref[i] + [(-1, -1)] * (2 - len(ref[i]))
        assert tuple(idx2[i]) == (exp[0][0], exp[1][0])
        assert tuple(dist2[i]) == (exp[0][1], exp[1][1])
        g = len(ref[i]) == 2 and ref[i][0][1] < 0.7 * ref[i][1][1]
        assert bool(good[i]) == g


def test_c_oracle_batch_layout():
    rng = np.random.default_rng(3)
    B, qc, tc = 3, 40, 50
    q = rng.integers(0, 256, (B, qc, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (B, tc, 32), dtype=np.uint8)
    nq, nt = np.array([40, 7, 0]), np.array([50, 1, 20])
    i2, d2, g = oracle.hamming_knn2_batch(q, nq, t, nt)
    for b in range(B):
        a, bb, c = oracle.hamming_knn2(q[b, :nq[b]], t[b, :nt[b]])
        assert np.array_equal(i2[b, :nq[b]], a) and np.array_equal(d2[b, :nq[b]], bb)
        assert np.array_equal(g[b, :nq[b]].astype(bool), c)
        assert (i2[b, nq[b]:] == -1).all()


def test_oracle_postprocessing_matches_reference_goldens(golden_dir):
    g = np.load(os.path.join(golden_dir, "matcher_golden.npz"))
    pl, pr, dl, dr = om.stereo_matches(g["stereo_ptsL"], g["stereo_desL"], g["stereo_ptsR"],
                                       g["stereo_desR"])
    for a, b in ((pl, "stereo_out_ptsL"), (pr, "stereo_out_ptsR"), (dl, "stereo_out_desL"),
                 (dr, "stereo_out_desR")):
        assert a.dtype == g[b].dtype and np.array_equal(a, g[b]), b
    q2, Q1, q1 = om.temporal_matches(g["temporal_des_i"], g["temporal_pts_i"],
                                     g["temporal_pts_i1"], g["temporal_des_i1"], g["temporal_Q"],
                                     max_Distance=500)
    for a, b in ((q2, "temporal_out_q2"), (Q1, "temporal_out_Q1"), (q1, "temporal_out_q1")):
        assert np.array_equal(a, g[b]), b
    a1, a2 = om.get_matches(g["stereo_ptsL"], g["stereo_desL"], g["stereo_ptsR"], g["stereo_desR"])
    assert a1.dtype == np.float32 and np.array_equal(a1, g["getm_out_q1"])
    assert np.array_equal(a2, g["getm_out_q2"])
    # ValueError truncation: train set of 1 -> nothing survives
    q2b, _, _ = om.temporal_matches(g["temporal_des_i"][:10], g["temporal_pts_i"][:10],
                                    g["temporal_pts_i1"][:1], g["temporal_des_i1"][:1],
                                    g["temporal_Q"][:10], 500)
    assert len(q2b) == 0 and (g["trunc_out_len"] == 0).all()


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_knn2_ragged_batch_bit_exact():
    import torch
    from slam355 import matcher

    rng = np.random.default_rng(11)
    B, qc, tc = 5, 2100, 2050
    q = np.zeros((B, qc, 32), np.uint8)
    t = np.zeros((B, tc, 32), np.uint8)
    nq = np.array([2000, 1, 777, 0, 2100], np.int32)
    nt = np.array([2000, 2050, 1, 5, 2])
    for b in range(B):
        qq, tt = _sets(rng, int(nq[b]), int(nt[b]), dup=20)
        q[b, :nq[b]], t[b, :nt[b]] = qq, tt
    dev = torch.device("cuda")
    i2, d2, g = matcher.knn2_batch(torch.from_numpy(q).to(dev), torch.from_numpy(nq).to(dev),
                                   torch.from_numpy(t).to(dev),
                                   torch.from_numpy(nt.astype(np.int32)).to(dev))
    torch.cuda.synchronize()
    ei2, ed2, eg = oracle.hamming_knn2_batch(q, nq, t, nt)
    assert np.array_equal(i2.cpu().numpy(), ei2)
    assert np.array_equal(d2.cpu().numpy(), ed2)
    assert np.array_equal(g.cpu().numpy(), eg)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 2, 3, 4, 5, 6, 7, 8])
def test_gpu_knn2_xcd_block_order_every_grid_remainder(B):
    """knn2_mx_kernel deals a frame pair's workgroups to one XCD by a bijection
    of the block index that depends on the grid size mod 8: batches whose
    grids leave every remainder still match the oracle bit for bit (3
    workgroups of 96 queries per item: grids 3B cover every residue mod 8;
    ragged query / train counts, so some workgroups exit early)."""
    import torch
    from slam355 import matcher

    rng = np.random.default_rng(100 + B)
    qc, tc = 200, 260
    q = np.zeros((B, qc, 32), np.uint8)
    t = np.zeros((B, tc, 32), np.uint8)
    nq = rng.integers(0, qc + 1, B).astype(np.int32)
    nt = rng.integers(0, tc + 1, B).astype(np.int32)
    for b in range(B):
        qq, tt = _sets(rng, int(nq[b]), int(nt[b]), dup=10)
        q[b, :nq[b]], t[b, :nt[b]] = qq, tt
    dev = torch.device("cuda")
    i2, d2, g = matcher.knn2_batch(torch.from_numpy(q).to(dev), torch.from_numpy(nq).to(dev),
                                   torch.from_numpy(t).to(dev), torch.from_numpy(nt).to(dev))
    torch.cuda.synchronize()
    ei2, ed2, eg = oracle.hamming_knn2_batch(q, nq, t, nt)
    assert np.array_equal(i2.cpu().numpy(), ei2)
    assert np.array_equal(d2.cpu().numpy(), ed2)
    assert np.array_equal(g.cpu().numpy(), eg)


@pytest.mark.gpu
def test_gpu_knn2_max_train_and_chunk_boundaries():
    import torch
    from slam355 import matcher

    rng = np.random.default_rng(5)
    for nq, nt in ((513, 1023), (512, 1024), (1, 1025), (300, 65535)):
        qq, tt = _sets(rng, nq, nt, dup=50)
        i2, d2, g = matcher.knn2(qq, tt)
        ei2, ed2, eg = oracle.hamming_knn2(qq, tt)
        assert np.array_equal(i2, ei2) and np.array_equal(d2, ed2) and np.array_equal(g, eg), (nq, nt)


@pytest.mark.gpu
@pytest.mark.parametrize("valu", [0, 1])
def test_gpu_knn2_matrix_core_and_valu_kernels_bit_exact(valu):
    """slam_hamming_knn2's fp4 matrix-core kernel (t_cap <= 16383) and the
    integer-VALU kernel (forced) against the oracle: train sets at the 16-row
    step boundaries, empty / single rows, the 14-bit index limit, duplicated
    rows (distance ties broken by the lower train index) and all-equal sets."""
    import torch
    from slam355 import _lib, matcher

    rng = np.random.default_rng(23)
    prev = _lib.lib.slam_hamming_force_valu(valu)
    try:
        cases = [(70, 0), (70, 1), (65, 2), (64, 15), (64, 16), (63, 17), (257, 33),
                 (129, 16383), (2087, 2087)]
        for nq, nt in cases:
            qq, tt = _sets(rng, nq, nt, dup=min(nt, 40))
            if nt >= 8:
                tt[nt // 2: nt // 2 + 4] = tt[1]  # exact duplicate rows: tied distances
            i2, d2, g = matcher.knn2(qq, tt)
            ei2, ed2, eg = oracle.hamming_knn2(qq, tt)
            assert np.array_equal(i2, ei2) and np.array_equal(d2, ed2), (valu, nq, nt)
            assert np.array_equal(g, eg), (valu, nq, nt)
        same = np.full((33, 32), 0xA5, np.uint8)  # every distance 0 (or equal): all ties
        i2, d2, g = matcher.knn2(same[:17], same)
        ei2, ed2, eg = oracle.hamming_knn2(same[:17], same)
        assert np.array_equal(i2, ei2) and np.array_equal(d2, ed2) and np.array_equal(g, eg)
    finally:
        _lib.lib.slam_hamming_force_valu(prev)
        torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_compact_matches_order_and_gate():
    import torch
    from slam355 import matcher

    rng = np.random.default_rng(9)
    B, qc, tc = 3, 1500, 1600
    q = rng.integers(0, 256, (B, qc, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (B, tc, 32), dtype=np.uint8)
    for b in range(B):
        q[b], t[b] = _sets(rng, qc, tc)
    nq = np.array([1500, 1033, 0], np.int32)
    nt = np.array([1600, 1600, 1600], np.int32)
    X = rng.normal(0, 400, (B, qc, 3))
    dev = torch.device("cuda")
    tq, tt = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    tnq, tnt = torch.from_numpy(nq).to(dev), torch.from_numpy(nt).to(dev)
    i2, d2, g = matcher.knn2_batch(tq, tnq, tt, tnt)
    pairs, cnt = matcher.compact_matches(i2, g, tnq, gate_xyz=torch.from_numpy(X).to(dev), gate=500.0)
    pairs, cnt = pairs.cpu().numpy(), cnt.cpu().numpy()
    for b in range(B):
        p = om.good_pairs(q[b, :nq[b]], t[b, :nt[b]])
        if len(p):
            p = p[np.all(np.abs(X[b, p[:, 0]]) < 500.0, axis=1)]
        assert cnt[b] == len(p)
        assert np.array_equal(pairs[b, :cnt[b]], p)


@pytest.mark.gpu
def test_gpu_reference_mirrors_match_goldens(golden_dir):
    """keypoint.py / tracking.py / Point3D.py mirrors on the GPU reproduce the
    goldens generated from the reference (exact-BF knnMatch stand-in)."""
    from slam355 import Point3D, keypoint, tracking

    g = np.load(os.path.join(golden_dir, "matcher_golden.npz"))
    a1, a2 = tracking.get_matches(g["stereo_ptsL"], g["stereo_desL"], g["stereo_ptsR"],
                                  g["stereo_desR"])
    assert a1.dtype == np.float32 and np.array_equal(a1, g["getm_out_q1"])
    assert np.array_equal(a2, g["getm_out_q2"])
    q2, Q1, q1 = Point3D.find_2D_and_3D_correspondenses(
        g["temporal_des_i"], g["temporal_pts_i"], g["temporal_pts_i1"], g["temporal_des_i1"],
        g["temporal_Q"], max_Distance=500)
    for a, b in ((q2, "temporal_out_q2"), (Q1, "temporal_out_Q1"), (q1, "temporal_out_q1")):
        assert np.array_equal(a, g[b]), b
    # the stereo path adds the F-LMedS mask: pre-mask pairs equal the golden
    # (all-inlier F stand-in), the mask equals the oracle's seeded LMedS
    from oracle import geometry as og

    pl, pr, dl, dr = keypoint.track_keypoints_left_to_right_new(
        g["stereo_ptsL"], g["stereo_desL"], g["stereo_ptsR"], g["stereo_desR"], seed=4, frame=2)
    mask, _, _, _ = og.fundamental_lmeds(g["stereo_out_ptsL"], g["stereo_out_ptsR"], seed=4,
                                         item=2)
    assert np.array_equal(pl, g["stereo_out_ptsL"][mask])
    assert np.array_equal(pr, g["stereo_out_ptsR"][mask])
    assert np.array_equal(dl, g["stereo_out_desL"][mask])
    assert np.array_equal(dr, g["stereo_out_desR"][mask])

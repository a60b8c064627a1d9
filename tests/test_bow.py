"""BoW place recognition, SURVEY.md §8f row 3 (/root/reference/bag_of_words.py).

CPU: the NumPy oracle against the reference's goldens (its hist /
predict_previous / predict run with a scikit-learn vocabulary fitted from fixed
centres; scikit-learn's Lloyd centres).  GPU: k_bow_hist / k_bow_query /
k_bow_lloyd against the same goldens.
"""
import os

import numpy as np
import pytest

from oracle import bow as ob

GOLD = os.path.join(os.path.dirname(__file__), "golden", "bow_golden.npz")


@pytest.fixture(scope="module")
def g():
    return np.load(GOLD)


def test_oracle_hist_and_queries_match_reference(g):
    C = g["centers"]
    for f in range(len(g["desc"])):
        assert np.array_equal(ob.labels(g["desc"][f], C), g["labels"][f])
        assert np.array_equal(ob.hist(g["desc"][f], C), g["db"][f])
    for i, thr, idx, val in g["pp"]:
        ri, rv = ob.predict_previous(g["db"][int(i)], g["db"], int(i), int(thr))
        assert ri == idx and rv == val


def test_oracle_lloyd_matches_sklearn(g):
    pool = g["desc"].reshape(-1, 32)
    for k in (1, 3, 10):
        C, lab = ob.lloyd(pool, g["C0"], k)
        assert np.allclose(C, g[f"lloyd_{k}"], rtol=1e-12, atol=1e-12)
        assert np.array_equal(lab, g[f"lloyd_{k}_labels"])


@pytest.mark.gpu
def test_gpu_histograms_match_reference(g):
    import torch
    from slam355 import bag_of_words as bw

    dev = torch.device("cuda")
    C = torch.from_numpy(g["centers"]).to(dev)
    d = torch.from_numpy(np.ascontiguousarray(g["desc"])).to(dev)
    h, lab = bw.histograms(d, None, C, labels=True)
    assert np.array_equal(lab.cpu().numpy(), g["labels"])
    assert np.array_equal(h.cpu().numpy(), g["db"])
    # ragged counts: rows past count are ignored
    cnt = torch.tensor([100, 37, 0, 1] * 10, dtype=torch.int32, device=dev)
    h2 = bw.histograms(d, cnt, C).cpu().numpy()
    for f, n in enumerate(cnt.cpu().numpy()):
        assert np.array_equal(h2[f], ob.hist(g["desc"][f][:n], g["centers"]) if n else 0 * h2[f])


@pytest.mark.gpu
def test_gpu_queries_match_reference(g):
    import torch
    from slam355 import bag_of_words as bw

    dev = torch.device("cuda")
    db = torch.from_numpy(g["db"].astype(np.int32)).to(dev)
    q = db[[int(i) for i in g["pp"][:, 0]]]
    n = torch.tensor([int(i) + 1 - int(t) if i >= t else 0 for i, t in g["pp"][:, :2]],
                     dtype=torch.int32, device=dev)
    idx, val = bw.query(q, db, n)
    for k, (i, thr, ei, ev) in enumerate(g["pp"]):
        assert int(idx[k]) == int(ei) and float(val[k]) == float(ev)
    # predict (:49-56): whole database
    q2 = db[[0, 7, 33]]
    idx, val = bw.query(q2, db, torch.full((3,), len(db), dtype=torch.int32, device=dev))
    assert np.array_equal(idx.cpu().numpy(), g["predict"][:, 0].astype(int))
    assert np.array_equal(val.cpu().numpy(), g["predict"][:, 1])


@pytest.mark.gpu
def test_gpu_lloyd_matches_sklearn(g):
    import torch
    from slam355 import bag_of_words as bw

    X = torch.from_numpy(np.ascontiguousarray(g["desc"].reshape(-1, 32))).cuda()
    for k in (1, 3, 10):
        C, lab = bw.lloyd(X, g["C0"], k)
        assert np.allclose(C.cpu().numpy(), g[f"lloyd_{k}"], rtol=1e-12, atol=1e-12)
        assert np.array_equal(lab.cpu().numpy(), g[f"lloyd_{k}_labels"])


@pytest.mark.gpu
def test_gpu_bow_train_and_recognise_places():
    """BoW.train on GPU ORB descriptors of synthetic frames (vocabulary by
    k-means++ seeding + GPU Lloyd), then place recognition: a frame recognises
    itself with distance 0, and predict_previous respects the threshold."""
    from slam355.bag_of_words import BoW
    from slam355.synthetic import stereo_sequence

    L, _, _, _ = stereo_sequence(8, 640, 480, seed=4)
    bow = BoW(n_clusters=20, n_features=100, seed=1)
    bow.train(list(L))
    assert len(bow.db) == 8 and all(h.sum() > 0 for h in bow.db)
    for i in (0, 5):
        idx, val = bow.predict(L[i])
        assert idx == i and val == 0.0
    assert bow.predict_previous(L[2], 2, 5) == (-1, -1)
    idx, val = bow.predict_previous(L[6], 6, 2)
    assert 0 <= idx <= 4 and val >= 0.0

"""Golden fixtures for BoW place recognition (SURVEY.md §8f row 3,
/root/reference/bag_of_words.py), produced by the REFERENCE code in the build
container (/root/reference does not exist on the GPU box).

    python tests/golden/make_bow_goldens.py

What is pinned, and how:
  * BoW.hist (:24-27), predict_previous (:30-45) and predict (:49-56) of the
    reference class, run on seeded synthetic descriptor sets.  BoW.__init__
    (:11-14) cannot run here (cv2 is absent and `KMeans(n_jobs=-1)` is rejected
    by this image's scikit-learn 1.7), so the object is created without it and
    given: a stub extractor whose detectAndCompute returns the frame's
    descriptors (OpenCV ORB itself is parity-unpinned; the GPU ORB is pinned
    separately), n_clusters, and a scikit-learn KMeans fitted from fixed
    initial centres (n_init=1).  train (:16-22) then runs as written.
  * Lloyd iterations: scikit-learn KMeans(init=C0, n_init=1, max_iter=k,
    tol=0, algorithm='lloyd') centres after k = 1, 3, 10 iterations on the
    pooled descriptors (uint8 rows as float64, as sklearn converts them).
Only data (inputs + outputs) is written; no reference source is copied.
"""
from __future__ import annotations

import os
import sys
import types
import warnings

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_goldens as mg  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


class _Extractor:
    """detectAndCompute(img, mask) -> (keypoints, descriptors): `img` is a frame
    index into the fixture's descriptor sets."""

    def __init__(self, sets):
        self.sets = sets

    def detectAndCompute(self, img, mask):
        d = self.sets[int(img)]
        return [None] * len(d), d


def frames(rng, n_frames, n_desc, n_words=12):
    """Descriptor sets of a revisiting trajectory: each frame mixes noisy copies
    of a few 'place' prototypes with random rows; frames 2k and 2k + n/2 share
    a place so place recognition has true matches."""
    places = rng.integers(0, 256, (n_frames // 2 + 1, n_words, 32), dtype=np.uint8)
    out = []
    for f in range(n_frames):
        pl = places[f % (n_frames // 2)]
        src = pl[rng.integers(0, n_words, n_desc)]
        bits = np.unpackbits(src, axis=1) ^ (rng.random((n_desc, 256)) < 0.05).astype(np.uint8)
        d = np.packbits(bits, axis=1)
        rand = rng.random(n_desc) < 0.3
        d[rand] = rng.integers(0, 256, (int(rand.sum()), 32), dtype=np.uint8)
        out.append(d)
    return out


def main():
    from sklearn.cluster import KMeans

    sys.modules["cv2"] = mg._stub_cv2()
    sys.modules.setdefault("tqdm", types.SimpleNamespace(tqdm=lambda x: x))
    if mg.REF not in sys.path:
        sys.path.insert(0, mg.REF)
    import bag_of_words  # noqa: E402

    rng = np.random.default_rng(11)
    K, n_frames, n_desc = 50, 40, 100
    sets = frames(rng, n_frames, n_desc)
    pool = np.concatenate(sets)
    C0 = pool[rng.choice(len(pool), K, replace=False)].astype(np.float64)
    out = dict(desc=np.array(sets), C0=C0)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for k in (1, 3, 10):
            km = KMeans(K, init=C0, n_init=1, max_iter=k, tol=0.0, algorithm="lloyd").fit(pool)
            out[f"lloyd_{k}"] = km.cluster_centers_
            out[f"lloyd_{k}_labels"] = km.labels_
        bow = object.__new__(bag_of_words.BoW)
        bow.extractor = _Extractor(sets)
        bow.n_clusters = K
        bow.kmeans = KMeans(K, init=C0, n_init=1, max_iter=300, algorithm="lloyd")
        bow.train(list(range(n_frames)))
        out["centers"] = bow.kmeans.cluster_centers_
        out["db"] = np.array(bow.db)
        out["labels"] = np.array([bow.kmeans.predict(d) for d in sets])
        q = []
        for i, thr in ((5, 10), (20, 10), (39, 10), (39, 2), (30, 25)):
            idx, val = bow.predict_previous(i, i, thr)
            q.append((i, thr, idx, val))
        out["pp"] = np.array(q, np.float64)
        out["predict"] = np.array([bow.predict(i) for i in (0, 7, 33)], np.float64)
    np.savez_compressed(os.path.join(OUT, "bow_golden.npz"), **out)
    print({k: np.shape(v) for k, v in out.items()})


if __name__ == "__main__":
    main()

"""Drop-in for /root/reference/bag_of_words.py (BoW place recognition) on the GPU.

  BoW(n_clusters=50, n_features=100)    (:11-14)
  BoW.train(imgs)                       (:16-22)  ORB on the GPU (whole image,
                                                  one patch), k-means++ seeding
                                                  on the host, Lloyd on the GPU
  BoW.hist(descriptors)                 (:24-27)
  BoW.predict_previous(img, img_index, threshold)  (:30-45)
  BoW.predict(img)                      (:49-56)
Batched device entry points for sequences: `histograms` (one launch for a
batch of descriptor sets) and `query` (chi-squared argmin for a batch of
queries against the database).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .device import ptr, require_gpu, stream_ptr, to_dev
from .orb import orb_batch


def histograms(desc: torch.Tensor, count: torch.Tensor | None, centers: torch.Tensor,
               labels: bool = False):
    """desc [B, cap, 32] u8 (device), count [B] i32 (or None: all rows) ->
    hist [B, K] i32 (and labels [B, cap] i32)."""
    B, cap = int(desc.shape[0]), int(desc.shape[1])
    K = int(centers.shape[0])
    hist = torch.empty((B, K), dtype=torch.int32, device=desc.device)
    lab = torch.full((B, cap), -1, dtype=torch.int32, device=desc.device) if labels else None
    _lib.call("slam_bow_histograms", ptr(desc), ptr(count) if count is not None else None, cap, B,
              cap, ptr(centers), K, ptr(lab), ptr(hist), stream_ptr())
    return (hist, lab) if labels else hist


def query(qhist: torch.Tensor, db: torch.Tensor, n_db: torch.Tensor):
    """chi-squared argmin / min of each query histogram over db rows [0, n_db[q])."""
    Q, K = int(qhist.shape[0]), int(qhist.shape[1])
    idx = torch.empty(Q, dtype=torch.int32, device=qhist.device)
    val = torch.empty(Q, dtype=torch.float64, device=qhist.device)
    _lib.call("slam_bow_query", ptr(qhist.contiguous()), Q, ptr(db.contiguous()),
              ptr(n_db.contiguous()), K, ptr(idx), ptr(val), stream_ptr())
    return idx, val


def lloyd(X: torch.Tensor, centers: np.ndarray, n_iter: int):
    """n_iter Lloyd iterations on the device -> (centres [K, 32] f64, labels [N])."""
    dev = require_gpu()
    c = torch.from_numpy(np.ascontiguousarray(centers, np.float64)).to(dev)
    tmp = torch.empty_like(c)
    lab = torch.empty(int(X.shape[0]), dtype=torch.int32, device=dev)
    _lib.call("slam_bow_lloyd", ptr(X), int(X.shape[0]), ptr(c), ptr(tmp), int(c.shape[0]),
              int(n_iter), ptr(lab), None, stream_ptr())
    return c, lab


def kmeans_plus_plus(X: np.ndarray, k: int, rng) -> np.ndarray:
    """Greedy k-means++ seeding (2 + log k local trials), host side, seeded."""
    X = np.asarray(X, np.float64)
    n = len(X)
    trials = 2 + int(np.log(k))
    centers = np.empty((k, X.shape[1]))
    centers[0] = X[rng.integers(n)]
    d2 = ((X - centers[0]) ** 2).sum(1)
    for c in range(1, k):
        tot = d2.sum()
        cand = np.searchsorted(np.cumsum(d2), rng.random(trials) * tot) if tot > 0 else \
            rng.integers(n, size=trials)
        cand = np.minimum(cand, n - 1)
        dc = ((X[None, :, :] - X[cand][:, None, :]) ** 2).sum(2)
        best = int(np.argmin(np.minimum(d2[None], dc).sum(1)))
        centers[c] = X[cand[best]]
        d2 = np.minimum(d2, dc[best])
    return centers


class BoW:
    def __init__(self, n_clusters=50, n_features=100, max_iter=300, seed=0):
        self.n_clusters = n_clusters
        self.n_features = n_features
        self.max_iter = max_iter
        self.rng = np.random.default_rng(seed)
        self.centers = None  # device [K, 32] f64
        self.db = []
        self._db_dev = None

    def _orb(self, imgs):
        dev = require_gpu()
        t = torch.from_numpy(np.ascontiguousarray(np.stack(imgs), np.uint8)).to(dev)
        _, _, desc, count = orb_batch(t, self.n_features, 1, 0, 0)
        return desc, count

    def fit(self, pool: np.ndarray):
        """KMeans.fit on pooled descriptors: k-means++ seeds, then Lloyd on the
        GPU until the labels stop changing or max_iter."""
        dev = require_gpu()
        X = to_dev(np.ascontiguousarray(pool, np.uint8))
        c0 = kmeans_plus_plus(pool, self.n_clusters, self.rng)
        c, lab = lloyd(X, c0, 1)
        prev = lab.clone()
        for _ in range(self.max_iter - 1):
            c, lab = lloyd(X, c.cpu().numpy(), 1)
            if torch.equal(lab, prev):
                break
            prev = lab.clone()
        self.centers = c.to(dev)
        return self

    def train(self, imgs):
        desc, count = self._orb(imgs)
        cnt = count.cpu().numpy()
        d = desc.cpu().numpy()
        pool = np.concatenate([d[i, :cnt[i]] for i in range(len(cnt))])
        self.fit(pool)
        h = histograms(desc, count, self.centers)
        self._db_dev = h
        self.db = list(h.cpu().numpy().astype(np.int64))

    def hist(self, descriptors):
        d = to_dev(np.ascontiguousarray(descriptors, np.uint8).reshape(1, -1, 32))
        return histograms(d, None, self.centers)[0].cpu().numpy().astype(np.int64)

    def _query(self, h, n):
        dev = require_gpu()
        db = self._db_dev if self._db_dev is not None and len(self._db_dev) == len(self.db) else \
            torch.from_numpy(np.asarray(self.db, np.int32)).to(dev)
        q = torch.from_numpy(np.asarray(h, np.int32)[None]).to(dev)
        idx, val = query(q, db, torch.tensor([n], dtype=torch.int32, device=dev))
        return int(idx[0]), float(val[0])

    def predict_previous(self, img, img_index, threshold):
        if img_index < threshold:
            return -1, -1
        desc, count = self._orb([img])
        h = histograms(desc, count, self.centers)[0].cpu().numpy()
        return self._query(h, img_index + 1 - threshold)

    def predict(self, img):
        desc, count = self._orb([img])
        h = histograms(desc, count, self.centers)[0].cpu().numpy()
        return self._query(h, len(self.db))

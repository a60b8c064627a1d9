"""ORACLE (test infrastructure only): NumPy restatement of
/root/reference/bag_of_words.py:24-56 (hist, chi-squared predict_previous /
predict) and of scikit-learn's Lloyd iteration (KMeans.fit, :20).  Pinned by
tests/golden/bow_golden.npz (the reference class run with scikit-learn)."""
from __future__ import annotations

import numpy as np


def labels(desc, centers):
    """argmin_j |c_j|^2 - 2 x.c_j (scikit-learn's Lloyd / predict expression)."""
    X = np.asarray(desc, np.float64)
    C = np.asarray(centers, np.float64)
    d = np.einsum("ij,ij->i", C, C)[None, :] + -2.0 * (X @ C.T)
    return np.argmin(d, axis=1)


def hist(desc, centers):
    K = len(centers)
    h, _ = np.histogram(labels(desc, centers), bins=K, range=(0, K - 1))
    return h


def chi2(x, y):
    return np.sum(2 * (x - y) ** 2 / (np.maximum(1, x + y)))


def predict_previous(h, db, img_index, threshold):
    if img_index < threshold:
        return -1, -1
    dist = [chi2(h, db[i]) for i in range(0, img_index + 1 - threshold)]
    return np.argmin(dist), np.min(dist)


def lloyd(X, centers, n_iter):
    X = np.asarray(X, np.float64)
    C = np.asarray(centers, np.float64).copy()
    for _ in range(n_iter):
        lab = labels(X, C)
        for j in range(len(C)):
            m = lab == j
            if m.any():
                C[j] = X[m].sum(0) / m.sum()
    return C, labels(X, C)

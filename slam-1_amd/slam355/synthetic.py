"""Seeded synthetic inputs (no datasets are reachable): descriptor sets, stereo
image sequences and BA problems of the BASELINE.json config shapes.
See SURVEY.md §8d for the definitions."""
from __future__ import annotations

import numpy as np


def descriptor_set(rng, nq, nt, frac_planted=0.6, flip_p=0.08):
    """Nt uniform random 32-byte rows; Nq rows of which `frac_planted` are
    copies of random train rows with each bit flipped w.p. flip_p (d ~ 20)."""
    t = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
    q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
    if nt:
        pick = rng.random(nq) < frac_planted
        src = rng.integers(0, nt, nq)
        bits = np.unpackbits(t[src], axis=1) ^ (rng.random((nq, 256)) < flip_p).astype(np.uint8)
        q[pick] = np.packbits(bits, axis=1)[pick]
    return q, t


def descriptor_batch(B, nq, nt, seed=0):
    rng = np.random.default_rng(seed)
    q = np.empty((B, nq, 32), np.uint8)
    t = np.empty((B, nt, 32), np.uint8)
    for b in range(B):
        q[b], t[b] = descriptor_set(rng, nq, nt)
    return q, np.full(B, nq, np.int32), t, np.full(B, nt, np.int32)


def _rodrigues(r):
    th = float(np.linalg.norm(r))
    if th == 0.0:
        return np.eye(3)
    k = r / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def bal_project(X, cams):
    """BAL projection (camera looks down -z, radial k1/k2) for input synthesis."""
    R = np.stack([_rodrigues(w) for w in cams[:, :3]])
    P = np.einsum("oij,oj->oi", R, X) + cams[:, 3:6]
    p = -P[:, :2] / P[:, 2:3]
    n = np.sum(p * p, axis=1)
    rad = 1 + cams[:, 7] * n + cams[:, 8] * n * n
    return p * (rad * cams[:, 6])[:, None]


def ba_problem(rng, n_cams, n_pts, obs_per_pt, f=716.8, noise=0.5):
    """Local-BA problem of SURVEY.md §8d: cameras 1 m apart along -z (BAL: the
    camera looks down -z), each point tracked by `obs_per_pt` consecutive
    keyframes from its anchor, sigma = `noise` px.  Returns
    (cams [C,9], pts [P,3], cam_idx [O], pt_idx [O], qs [O,2]), observations in
    shuffled order (the reference does not sort them)."""
    C = np.stack([rng.normal(0, 0.05, n_cams), rng.normal(0, 0.05, n_cams),
                  -np.arange(n_cams, dtype=float)], 1)
    rot = rng.normal(0, 0.02, (n_cams, 3))
    cams = np.zeros((n_cams, 9))
    for c in range(n_cams):
        cams[c, :3] = rot[c]
        cams[c, 3:6] = -_rodrigues(rot[c]) @ C[c]
        cams[c, 6] = f
    anchor = rng.integers(0, n_cams - obs_per_pt + 1, n_pts)
    depth = rng.uniform(8.0, 60.0, n_pts)
    X = C[anchor] + np.stack([rng.uniform(-0.4, 0.4, n_pts) * depth,
                              rng.uniform(-0.25, 0.25, n_pts) * depth, -depth], 1)
    cam_idx = (anchor[:, None] + np.arange(obs_per_pt)[None, :]).ravel()
    pt_idx = np.repeat(np.arange(n_pts), obs_per_pt)
    perm = rng.permutation(len(cam_idx))
    cam_idx, pt_idx = cam_idx[perm], pt_idx[perm]
    qs = bal_project(X[pt_idx], cams[cam_idx]) + rng.normal(0, noise, (len(cam_idx), 2))
    return cams, X, cam_idx.astype(np.int64), pt_idx.astype(np.int64), qs


def perturb(rng, cams, pts, rot_s=1e-3, t_s=1e-2, p_s=0.05):
    """Initialisation noise of SURVEY.md §8d (rotvec 1e-3, t 1e-2 m, points 5 cm)."""
    c = cams.copy()
    c[:, :3] += rng.normal(0, rot_s, c[:, :3].shape)
    c[:, 3:6] += rng.normal(0, t_s, c[:, 3:6].shape)
    return c, pts + rng.normal(0, p_s, pts.shape)

"""PnP-RANSAC alone on the tracking batch shape (32 frame pairs x ~115
correspondences, 20 % outliers): mean ms per slam_pnp_ransac call, for A/B of
the hypothesis kernels (run under rocprofv3 --kernel-trace --stats for the
per-kernel split).

    python scripts/pnp_time.py [LIB_NAME]   (slam-1_amd/prof/libslam355_LIB_NAME.so)"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]
if len(sys.argv) > 1:
    os.environ["SLAM355_LIB"] = os.path.join(ROOT, "slam-1_amd", "prof", f"libslam355_{sys.argv[1]}.so")

import torch  # noqa: E402
from slam355 import geometry  # noqa: E402

B, cap = 32, 128
K = np.array([[718.856, 0, 607.19], [0, 718.856, 185.22], [0, 0, 1]])
rng = np.random.default_rng(0)
Q = np.zeros((B, cap, 3))
q = np.zeros((B, cap, 2))
cnt = np.zeros(B, np.int32)
for b in range(B):
    n = int(rng.integers(100, cap))
    X = np.c_[rng.uniform(-8, 8, n), rng.uniform(-3, 3, n), rng.uniform(4, 40, n)]
    ang = rng.normal(0, 0.02, 3)
    th = np.linalg.norm(ang)
    kx = np.array([[0, -ang[2], ang[1]], [ang[2], 0, -ang[0]], [-ang[1], ang[0], 0]]) / th
    R = np.eye(3) + np.sin(th) * kx + (1 - np.cos(th)) * kx @ kx
    t = rng.normal(0, 0.3, 3)
    Xc = X @ R.T + t
    uv = (Xc[:, :2] / Xc[:, 2:]) * [K[0, 0], K[1, 1]] + [K[0, 2], K[1, 2]]
    uv += rng.normal(0, 0.5, uv.shape)
    out = rng.random(n) < 0.2
    uv[out] += rng.uniform(-80, 80, (out.sum(), 2))
    Q[b, :n], q[b, :n], cnt[b] = X, uv, n
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
tQ, tq, tc = T(Q), T(q), T(cnt)
ws = geometry.pnp_workspace(B)
for _ in range(3):
    geometry.pnp_ransac(tQ, tq, tc, K, seed=1, item0=0, ws=ws)
torch.cuda.synchronize()
N = 30
t0 = time.perf_counter()
for i in range(N):
    rv, tv, n, mask = geometry.pnp_ransac(tQ, tq, tc, K, seed=1, item0=i, ws=ws)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) / N * 1e3
print(f"pnp_ransac B={B}: {ms:.3f} ms per call; inliers mean {n.float().mean().item():.1f}")

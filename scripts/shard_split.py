"""Per-rank kernel split of the sharded LM iteration, measured (not projected):
rank r's landmark shard of a C4 / C5 window at world size W (slam355.dist.
shard_by_anchor: the shard bench.py --gpus W gives rank r), built as the same
BAProblem the distributed step uses, and iterated ALONE on this GPU (no
collective: the all-reduce is the only part one GPU cannot run) -- run under
rocprofv3 --kernel-trace --stats, so the kernel statistics are rank r's share of
k_lin_mfma / k_assemble / k_back_trial next to the replicated camera solve.
python scripts/shard_split.py {C4|C5} W r [iters] [chunks_per_wg] [fold]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from slam355.ba import BAProblem, upper_blocks  # noqa: E402
from slam355.dist import shard_by_anchor  # noqa: E402
from slam355.synthetic import ba_problem, ba_problem_loop, perturb  # noqa: E402

name, W, r = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
cpw = (int(sys.argv[5]) or None) if len(sys.argv) > 5 else None
fold = len(sys.argv) > 6 and sys.argv[6] == "fold"  # k_lin_mfma assembles (no k_assemble launch)
C, P, gen = (64, 50000, ba_problem) if name == "C4" else (500, 200000, ba_problem_loop)
rng = np.random.default_rng(7)
cams, pts, ci, pi, qs = gen(rng, C, P, 6)
c0, p0 = perturb(rng, cams, pts)
if W > 1:
    mine, keep, local_pi = shard_by_anchor(C, P, ci, pi, r, W)
    prob = BAProblem(c0, p0[mine], ci[keep], local_pi, qs[keep], block_list=upper_blocks(C, ci, pi),
                     chunks_per_wg=cpw, fold_assembly=fold)
    n_obs, n_pts = int(keep.sum()), int(mine.sum()) if mine.dtype == bool else len(mine)
else:
    prob = BAProblem(c0, p0, ci, pi, qs, chunks_per_wg=cpw, fold_assembly=fold)
    n_obs, n_pts = len(ci), P
for _ in range(3):
    prob.iterate_graphed(1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(iters):
    prob.iterate_graphed(1)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / iters
print(json.dumps({"config": name, "world": W, "rank": r, "obs": n_obs, "points": n_pts,
                  "chunks_per_wg": prob.plan["chunks_per_wg"], "fold": fold, "n_sgrps": prob.plan["n_sgrps"],
                  "ms_per_iter_alone": dt * 1e3}))

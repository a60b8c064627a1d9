"""Pose-graph TRF solve time (500-keyframe drifted loop, BASELINE C5's pose-graph
half) for the kernel SLAM_CHAIN_TRF selects: median wall time per solve to the
ftol test, with nfev / iterations / cost.  python scripts/pg_time.py [m] [reps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from slam355.posegraph import PoseChain  # noqa: E402
from slam355.synthetic import pose_chain_loop  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 500
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
x0 = pose_chain_loop(np.random.default_rng(11), m)
PoseChain(x0).solve(ftol=1e-8)
torch.cuda.synchronize()
ts, st = [], None
for _ in range(reps):
    pc = PoseChain(x0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = pc.solve(ftol=1e-8)
    ts.append(time.perf_counter() - t0)
ms = float(np.median(ts)) * 1e3
print(json.dumps({"kernel": os.environ.get("SLAM_CHAIN_TRF", "reg"), "frames": m, "ms_per_solve": ms,
                  "ms_per_iteration": ms / max(1, st["iterations"]), "nfev": st["nfev"],
                  "iterations": st["iterations"], "status": st["message"], "cost": st["cost"]}))

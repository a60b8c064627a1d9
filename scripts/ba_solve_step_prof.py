"""Cycle split of one k_solve_reg elimination step (k = n/2) — needs a library
built with -DSLAM_SOLVE_PROFILE_STEP."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

from slam355.ba import BAProblem  # noqa: E402
from slam355.synthetic import ba_problem, perturb  # noqa: E402

for C, P, k in ((6, 1500, 4), (10, 5000, 6)):
    rng = np.random.default_rng(0)
    cams, pts, ci, pi, qs = ba_problem(rng, C, P, k)
    c0, p0 = perturb(rng, cams, pts)
    prob = BAProblem(c0, p0, ci, pi, qs)
    rows = []
    for _ in range(10):
        prob.iterate(1)
        rows.append(prob.t["state"][12:16].cpu().numpy())
    m = np.median(np.array(rows), 0)
    print(f"C={C}: (a)+barrier {m[0]:.0f} clk, (b) panel {m[1]:.0f} clk, barrier {m[2]:.0f} clk, (c) mfma {m[3]:.0f} clk  (built with -DSLAM_SOLVE_PROFILE_PANEL: the last two are the panel load and elimination)")

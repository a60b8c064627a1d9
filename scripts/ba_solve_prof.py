"""Phase timing of k_solve_blk (needs a library built with -DSLAM_SOLVE_PROFILE:
`make -C slam-1_amd clean all HIPFLAGS_EXTRA=-DSLAM_SOLVE_PROFILE`)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

from slam355.ba import BAProblem  # noqa: E402
from slam355.synthetic import ba_problem, perturb  # noqa: E402

for C, P, k in ((6, 1500, 4), (10, 5000, 6), (13, 5000, 6)):
    rng = np.random.default_rng(0)
    cams, pts, ci, pi, qs = ba_problem(rng, C, P, k)
    c0, p0 = perturb(rng, cams, pts)
    prob = BAProblem(c0, p0, ci, pi, qs)
    rows = []
    for _ in range(20):
        prob.iterate(1)
        rows.append(prob.t["state"][12:16].cpu().numpy())
    m = np.median(np.array(rows), 0)
    print(f"C={C} n={9 * C}: load {m[0]:.0f} ns  eliminate {m[1]:.0f} ns "
          f"({m[1] / (9 * C):.0f}/step)  backsub {m[2]:.0f} ns  epilogue {m[3]:.0f} ns")

"""Phase split of k_linearize for group 7 (library built with -DSLAM_LIN_PROFILE):
projections, point elimination + W, slot partials (cycles), and its slot counts."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

from slam355.ba import BAProblem  # noqa: E402
from slam355.synthetic import ba_problem, perturb  # noqa: E402

rng = np.random.default_rng(0)
cams, pts, ci, pi, qs = ba_problem(rng, 10, 5000, 6)
c0, p0 = perturb(rng, cams, pts)
prob = BAProblem(c0, p0, ci, pi, qs)
rows = []
for _ in range(10):
    prob.iterate(1)
    rows.append(prob.t["state"][12:16].cpu().numpy())
m = np.median(np.array(rows), 0)
print(f"proj {m[0]:.0f} clk, points+W {m[1]:.0f} clk, slots {m[2]:.0f} clk; "
      f"camera slots {int(m[3]) // 100}, block slots {int(m[3]) % 100}")
pl = prob.plan
print("pairs per block slot", np.mean(np.diff(pl["bslot_pair_ptr"])),
      "groups", len(pl["grp_ptr"]) - 1, "bslots", len(pl["bslot_blk"]))

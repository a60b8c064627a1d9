"""Runs 20 LM iterations of the C3 local-BA window (for rocprofv3 counter passes)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

import torch  # noqa: E402

from slam355.ba import BAProblem  # noqa: E402
from slam355.synthetic import ba_problem, perturb  # noqa: E402

C, P, k = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (10, 5000, 6)))
rng = np.random.default_rng(0)
cams, pts, ci, pi, qs = ba_problem(rng, C, P, k)
c0, p0 = perturb(rng, cams, pts)
prob = BAProblem(c0, p0, ci, pi, qs)
prob.iterate(20)
torch.cuda.synchronize()
print("cost", prob.cost())

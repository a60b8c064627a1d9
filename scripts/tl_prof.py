"""Phase timing of the tiled solver's panel kernel (k_tl_panel) on a C4-sized
system.  Needs an instrumented build:
  make -C slam-1_amd clean all HIPFLAGS_EXTRA=-DSLAM_TL_PROFILE && mv slam-1_amd/slam355/libslam355.so /tmp/...
run with SLAM355_LIB=<that .so>."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

from slam355 import _lib  # noqa: E402
from slam355.ba import BAProblem  # noqa: E402
from slam355.synthetic import ba_problem, perturb  # noqa: E402

for C, P, k in ((64, 50000, 6),):
    rng = np.random.default_rng(0)
    cams, pts, ci, pi, qs = ba_problem(rng, C, P, k)
    c0, p0 = perturb(rng, cams, pts)
    prob = BAProblem(c0, p0, ci, pi, qs)
    n = len(prob.t["chol"])
    rows = []
    for _ in range(10):
        prob.iterate(1)
        rows.append(prob.t["chol"][n - 7:n - 5].cpu().numpy())
    m = np.median(np.array(rows), 0)
    print(f"C={C}: panel WG: factor {m[0]:.0f} ns, gemm+store+b {m[1]:.0f} ns")

# sub-phases of the diagonal-tile factor (WG 1 of step 0, wall clock 100 MHz)
import ctypes  # noqa: E402

fn = getattr(_lib.lib, "slam_tl_stamps", None)
if fn is not None:
    buf = (ctypes.c_ulonglong * 8)()
    fn.argtypes = [ctypes.c_void_p]
    fn(ctypes.cast(buf, ctypes.c_void_p))
    st = [int(v) for v in buf[:4]]
    print("factor sub-phases (ns): load %d, blocked chol %d, inverse assembly %d" %
          tuple(10 * (b - a) for a, b in zip(st[:3], st[1:4])))

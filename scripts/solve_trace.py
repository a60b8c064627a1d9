"""Per-camera-step timeline of k_solve_blk (library built with
build_prof_lib.sh solvetr -DSLAM_SOLVE_TRACE): (a) panel copy + barrier,
(b) panel factor, barrier, (c) trailing MFMA update, then back substitution
and epilogue, in shader cycles."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]
os.environ["SLAM355_LIB"] = os.path.join(ROOT, "slam-1_amd", "prof", "libslam355_solvetr.so")

import torch  # noqa: E402
from slam355 import _lib  # noqa: E402
from slam355.ba import BAProblem  # noqa: E402
from slam355.synthetic import ba_problem, perturb  # noqa: E402

fn = _lib.lib.slam_solve_trace
fn.argtypes = [ctypes.c_void_p]
rng = np.random.default_rng(0)
cams, pts, ci, pi, qs = ba_problem(rng, 10, 5000, 6)
c0, p0 = perturb(rng, cams, pts)
prob = BAProblem(c0, p0, ci, pi, qs)
for it in range(4):
    prob.iterate(1)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 120)()
    fn(buf)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(20, 6).astype(np.int64)
    t0 = a[19, 0]
    print(f"iter {it}: load {a[19, 1] - t0} clk; steps (a, b, bar, c):")
    for k in range(10):
        r = a[k]
        print(f"   cam {k}: {r[1] - r[0]:6d} {r[2] - r[1]:6d} {r[3] - r[2]:6d} {r[4] - r[3]:6d}   "
              f"(to next {(a[k + 1, 0] if k < 9 else a[18, 0]) - r[0]})")
    print(f"   back subst {a[18, 1] - a[18, 0]}, epilogue {a[18, 2] - a[18, 1]}, total {a[18, 2] - t0}")

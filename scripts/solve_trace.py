"""Per-panel timeline of k_solve_blk (wave 0 of window 0, s_memtime stamps) from a
library built with -DSLAM_SOLVE_TRACE:

    scripts/build_variant.sh strace ba.hip -DSLAM_SOLVE_TRACE
    python scripts/solve_trace.py [LIB_NAME] [N_WINDOWS]

Stamp slots per panel: 0 panel start, 2 factor done, 3 after the W/L barrier,
4 after the next panel's copy, 1 after the copy barrier; slot (19, 0) the
start of the elimination, (18, 0) its end."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]
name = sys.argv[1] if len(sys.argv) > 1 else "strace"
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 8
os.environ["SLAM355_LIB"] = os.path.join(ROOT, "slam-1_amd", "prof", f"libslam355_{name}.so")

import torch  # noqa: E402
from slam355 import _lib  # noqa: E402
from slam355.ba import BABatch, BAProblem  # noqa: E402
from slam355.synthetic import ba_problem, perturb  # noqa: E402

rng = np.random.default_rng(0)
probs = []
for _ in range(nb):
    cams, pts, ci, pi, qs = ba_problem(rng, 10, 5000, 6)
    c0, p0 = perturb(rng, cams, pts)
    probs.append(BAProblem(c0, p0, ci, pi, qs))
bat = BABatch(probs) if nb > 1 else None
fn = _lib.lib.slam_solve_trace
fn.argtypes = [ctypes.c_void_p]
rows = []
for it in range(12):
    (bat.iterate(1) if bat else probs[0].iterate(1))
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 120)()
    fn(buf)
    rows.append(np.frombuffer(buf, dtype=np.uint64).reshape(20, 6).astype(np.int64))
a = np.median(np.array(rows[2:]), 0)  # per-slot median over iterations
npan = 10
print(f"{name}: elimination {a[18, 0] - a[19, 0]:.0f} clk over {npan} panels")
for k in range(npan):
    t0 = a[k, 0]
    end = a[k + 1, 0] if k + 1 < npan else a[18, 0]
    rel = {s: a[k, s] - t0 for s in (2, 3, 4, 1)}
    print(f"  panel {k}: total {end - t0:6.0f}  factor {rel[2]:6.0f}  W/L barrier {rel[3]:6.0f}  "
          f"copy {rel[4]:6.0f}  copy barrier {rel[1]:6.0f}  (stamps rel. to start)")

"""Phase split of k_lin_mfma per workgroup (library built by build_linm_prof.sh),
shader cycles summed over the workgroup's chunks: staging + load wait, projections
(A), points (B), W/Y (C), MFMA + U (D), write-out (E).

    python scripts/linm_prof.py N_WINDOWS CHUNKS_PER_WG"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]
os.environ.setdefault("SLAM355_LIB", os.path.join(ROOT, "slam-1_amd", "prof", "libslam355_linm.so"))

import torch  # noqa: E402
from slam355 import _lib  # noqa: E402
from slam355.ba import BABatch, BAProblem  # noqa: E402
from slam355.synthetic import ba_problem, perturb  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 1
cpw = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # phases are per chunk: 1 chunk per WG
rng = np.random.default_rng(0)
probs = []
for _ in range(nb):
    cams, pts, ci, pi, qs = ba_problem(rng, 10, 5000, 6)
    c0, p0 = perturb(rng, cams, pts)
    probs.append(BAProblem(c0, p0, ci, pi, qs, chunks_per_wg=cpw))
bat = BABatch(probs)
fn = _lib.lib.slam_linm_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
names = ["staging+wait", "A proj", "B points", "C W/Y", "D mfma+U", "E write"]
for it in range(5):
    bat.iterate(1)
    torch.cuda.synchronize()
    n = probs[0].plan["n_sgrps"]
    buf = (ctypes.c_ulonglong * (4096 * 8))()
    fn(buf, 4096)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8).astype(np.int64)
    rows = np.concatenate([a[1024 * y:1024 * y + n] for y in range(nb)])
    d = rows[:, 1:7]  # per-phase shader cycles summed over the workgroup's chunks
    tot = d.sum(1)
    print(f"iter {it}: WGs {len(rows)} ({cpw} chunks/WG); per-WG total median {np.median(tot):.0f} "
          f"max {tot.max()} clk")
    print("   " + "  ".join(f"{nm} {np.median(d[:, k]):.0f} ({100 * np.median(d[:, k]) / np.median(tot):.0f}%)"
                            for k, nm in enumerate(names)))

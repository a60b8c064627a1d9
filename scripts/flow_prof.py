"""Per-column phase timeline of the dataflow tiled solve (k_tl3_flow) at C4 / C5.
Run with SLAM355_LIB=slam-1_amd/prof/libslam355_flowprof.so (scripts/build_flow_prof.sh)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "slam-1_amd")]

from slam355 import _lib  # noqa: E402
from slam355.ba import BAProblem  # noqa: E402
from slam355.synthetic import ba_problem, ba_problem_loop, perturb  # noqa: E402

PH = ["diag_upd", "factor", "rows", "y", "x_wait", "x", "end"]
for name, C, P, gen in (("C4", 64, 50000, ba_problem), ("C5", 500, 200000, ba_problem_loop)):
    rng = np.random.default_rng(7)
    cams, pts, ci, pi, qs = gen(rng, C, P, 6)
    c0, p0 = perturb(rng, cams, pts)
    prob = BAProblem(c0, p0, ci, pi, qs)
    T = int(prob._sched_host[1])
    fn = _lib.lib.slam_flow_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    runs = []
    for _ in range(5):
        prob.iterate(1)
        buf = (ctypes.c_ulonglong * (8 * T))()
        fn(ctypes.cast(buf, ctypes.c_void_p), T)
        runs.append(np.array(buf[:], np.int64).reshape(T, 8))
    st = runs[-1]
    t0 = st[:, 0].min()
    rel = (st - t0) * 10 / 1000.0  # us
    dump = {"config": name, "T": T, "stamps_us": rel.round(2).tolist()}
    print(f"{name}: T={T} span {rel[:, 6].max():.1f} us (to last x), epilogue end {rel[:, 7].max():.1f}")
    sched = prob._sched_host
    rec = sched[sched[5]:sched[5] + 5 * T].reshape(-1, 5)
    for J in range(min(T, 26)):
        d = np.diff(rel[J, :7])
        print(f"  col {J:3d} rows {rec[J,1]} rs {rec[J,3]}: start {rel[J,0]:7.1f} " +
              " ".join(f"{PH[i]} {d[i]:6.1f}" for i in range(6)) + f" | x at {rel[J,6]:7.1f}")
    fs = getattr(_lib.lib, "slam_flow_sub_stamps", None)
    if fs is not None:
        fs.argtypes = [ctypes.c_void_p, ctypes.c_int]
        sb = (ctypes.c_ulonglong * (8 * T))()
        fs(ctypes.cast(sb, ctypes.c_void_p), T)
        raw = np.array(sb[:], np.uint64).reshape(T, 8).astype(np.float64)
        sub = np.where((raw > t0) & (raw < t0 + 1e8), (raw - t0) * 10 / 1000.0, np.nan)
        dump["sub_us"] = np.nan_to_num(sub, nan=-1.0).round(2).tolist()
        rec_ = prob._sched_host[prob._sched_host[5]:prob._sched_host[5] + 5 * T].reshape(-1, 5)
        sh_ = prob._sched_host
        dump["rows"] = [sh_[r[0]:r[0] + r[1]].tolist() for r in rec_]
        dump["rs"] = [sh_[r[2]:r[2] + r[3]].tolist() for r in rec_]
        if len(sys.argv) > 1:
            import json as _json
            with open(f"{sys.argv[1]}_{name}.json", "w") as fo:
                _json.dump(dump, fo)
        rs = sched  # rs(J) list at rec[J, 2], count rec[J, 3]; rows at rec[J, 0], count rec[J, 1]
        print("  row 0 of each column (us, absolute): first child in / last child in / factor end /"
              " folds done / staged / product / published | parent's last child in")
        for J in range(min(T, 26)):
            last_in = ""
            if rec[J, 1] > 0:
                P = int(rs[rec[J, 0]])
                kids = rs[rec[P, 2]:rec[P, 2] + rec[P, 3]]
                if len(kids) and int(kids[-1]) == J:
                    last_in = f"{sub[P, 1]:7.1f} (+{sub[P, 1] - sub[J, 5]:.1f})"
            print(f"  col {J:3d}: " + " ".join(f"{sub[J, i]:7.1f}" for i in (0, 1)) + f" {rel[J, 2]:7.1f} " +
                  " ".join(f"{sub[J, i]:7.1f}" for i in (2, 3, 4, 5)) + " | " + last_in +
                  f" | deferred fold: tile in view {sub[J, 6]:7.1f}, loaded {sub[J, 7]:7.1f}")
    fe = getattr(_lib.lib, "slam_flow_epi_stamps", None)
    if fe is not None:
        fe.argtypes = [ctypes.c_void_p]
        eb = (ctypes.c_ulonglong * 4)()
        fe(ctypes.cast(eb, ctypes.c_void_p))
        ev = (np.array(eb[:], np.float64) - float(t0)) * 10 / 1000.0
        print(f"  epilogue (us, absolute): start {ev[0]:.1f}, x staged {ev[1]:.1f}, pc / cost reduced {ev[2]:.1f},"
              f" cameras prepared {ev[3]:.1f}")
    ff = getattr(_lib.lib, "slam_flow_fac_stamps", None)
    if ff is not None:
        fb = (ctypes.c_ulonglong * 16)()
        ff.argtypes = [ctypes.c_void_p]
        ff(ctypes.cast(fb, ctypes.c_void_p))
        v = np.array(fb[:14], np.int64) * 10 / 1000.0
        d = np.diff(v)
        # slots: 3p + 1 wave 0's look-ahead done, 3p + 2 its pivots done,
        # 3p + 3 the block's barrier passed (p = 3: after the loop)
        print("  factor of column 0 (us): " + " ".join(
            f"p{p}: look-ahead {d[3 * p]:.2f} pivots {d[3 * p + 1]:.2f} inverse+barrier {d[3 * p + 2]:.2f}"
            for p in range(4)) + f" | inverse assembly {d[12]:.2f} | total {v[13] - v[0]:.2f}")

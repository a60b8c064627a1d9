"""Diagnostic (round 6): the dataflow solve (product tasks with deeper rows) vs
the level-scheduled solve vs the oracle's Schur LM, first LM iteration."""
import sys, numpy as np
sys.path[:0]=['.','slam-1_amd']
from oracle import ba as oba
from slam355 import ba
from slam355.synthetic import ba_problem_loop
for tiles, C, P, k in (("rows64", 60, 3000, 8), ("rows64", 60, 3000, 7), ("cams:3", 40, 2000, 7), ("cams:5", 60, 3000, 8)):
  if True:
    rng = np.random.default_rng(5)
    cams, pts, ci, pi, qs = ba_problem_loop(rng, C, P, k)
    cams0 = cams.copy()
    cams0[:, :3] += rng.normal(0, 1e-3, (C, 3))
    cams0[:, 3:6] += rng.normal(0, 1e-2, (C, 3))
    pts0 = pts + rng.normal(0, 0.05, pts.shape)
    res = {}
    for mode in ("flow", "levels"):
        prob = ba.BAProblem(cams0, pts0, ci, pi, qs, tl_mode=mode, tile_mode=tiles)
        S=prob._sched_host; T,pt=int(S[1]),int(S[10])
        na=sum(int((S[S[pt+2*J]:S[pt+2*J]+3*S[pt+2*J+1]].reshape(-1,3)[:,0]>0).sum()) for J in range(T))
        prob.iterate(1)
        res[mode] = prob.params()[0]
        del prob
    st = oba.LMState(1e-4); pairs = oba._obs_pairs(ci, pi)
    oc, op, info = oba.lm_iteration_schur(cams0.copy(), pts0.copy(), ci, pi, qs, st, pairs)
    rel = lambda a, b: np.max(np.abs(a - b) / (np.abs(b) * 1e-6 + 1e-9))
    print(tiles, C, k, "mfma plan", ba.plan_mfma(C, P, ci, pi) is not None, "a>0 tasks", na, "flow vs oracle", rel(res["flow"], oc), "levels vs oracle", rel(res["levels"], oc), "flow vs levels", rel(res["flow"], res["levels"]))

"""Bundle adjustment: oracle pinning against the reference's BAL block (CPU)
and GPU parity of the HIP LM solver.

Reference: /root/reference/BundleAdjustment.py:287-402 (BAL block, pinned by
tests/golden/ba_golden.npz made from the reference's own code).
Tolerances (float64):
  residual kernel vs reference objective: |d| <= 1e-9 * max(1, |r|)
  Jacobian kernel vs oracle analytic J:   |d| <= 1e-8 * max(1, |J|)
  LM iterates GPU vs oracle:              cost rel 1e-9, params rel 1e-6 (first 8 iters)
  converged cost vs reference least_squares (tight tol): <= ref * (1 + 1e-6)
"""
import os

import numpy as np
import pytest

from oracle import ba as oba


@pytest.fixture(scope="module")
def g(golden_dir):
    return np.load(os.path.join(golden_dir, "ba_golden.npz"))


def make_problem(seed, C, P, obs_per_pt, noise=0.5, f=716.8):
    """Local-BA-shaped synthetic problem (tracks over consecutive keyframes)."""
    from slam355.synthetic import ba_problem

    return ba_problem(np.random.default_rng(seed), C, P, obs_per_pt, f=f, noise=noise)


# ----------------------------------------------------------------------------- CPU
def test_oracle_objective_equals_reference(g):
    params = np.hstack((g["res_cams"].ravel(), g["res_pts"].ravel()))
    r = oba.objective(params, 6, 300, g["res_cam_idx"], g["res_pt_idx"], g["res_qs"])
    assert np.array_equal(r, g["res_out"])  # bit-exact: same numpy expression order
    assert np.array_equal(oba.rotate(g["rot_in_pts"], g["rot_in_vecs"]), g["rot_out"])


def test_oracle_sparsity_equals_reference(g):
    rows, cols, shape = oba.sparsity_coo(6, 300, g["res_cam_idx"], g["res_pt_idx"])
    assert np.array_equal(rows, g["sp_rows"]) and np.array_equal(cols, g["sp_cols"])
    assert tuple(shape) == tuple(g["sp_shape"])


def test_oracle_jacobian_vs_finite_differences(g):
    cams, pts = g["res_cams"].copy(), g["res_pts"].copy()
    ci, pi, qs = g["res_cam_idx"], g["res_pt_idx"], g["res_qs"]
    r, J = oba.residual_and_jacobian(cams, pts, ci, pi, qs)
    assert np.allclose(r.ravel(), g["res_out"], rtol=0, atol=1e-9)
    clamped = [3, 5, 8]
    zero_rot = int(np.nonzero(ci == 0)[0][0])
    for o in clamped + [zero_rot, 17, 100, 999]:
        c, p = ci[o], pi[o]
        for k in range(12):
            cp, cm, pp, pm = cams.copy(), cams.copy(), pts.copy(), pts.copy()
            if k < 9:
                h = 1e-6 * max(1.0, abs(cams[c, k]))
                cp[c, k] += h
                cm[c, k] -= h
            else:
                h = 1e-6 * max(1.0, abs(pts[p, k - 9]))
                pp[p, k - 9] += h
                pm[p, k - 9] -= h
            sl = slice(o, o + 1)
            fd = (oba.residual_and_jacobian(cp, pp, ci[sl], pi[sl], qs[sl])[0] -
                  oba.residual_and_jacobian(cm, pm, ci[sl], pi[sl], qs[sl])[0])[0] / (2 * h)
            assert np.allclose(fd, J[o, :, k], rtol=1e-5, atol=1e-5 * max(1, np.abs(J[o]).max()))


def test_oracle_lm_reaches_reference_optimum(g):
    cams, pts, hist = oba.lm_solve(g["sol_cams0"], g["sol_pts0"], g["sol_cam_idx"],
                                   g["sol_pt_idx"], g["sol_qs"], iters=40)
    ref_tight = float(g["sol_tight_cost"])
    ref_default = 0.5 * float(np.sum(g["sol_ref_rf"] ** 2))  # reference settings (ftol=0.1)
    assert hist[-1]["cost"] <= ref_tight * (1 + 1e-6)
    assert hist[-1]["cost"] <= ref_default


def test_planner_slots_cover_schur_structure():
    from slam355 import ba

    cams, pts, ci, pi, qs = make_problem(1, 7, 200, 4)
    # add a duplicate observation (camera sees a point twice)
    ci = np.append(ci, ci[0])
    pi = np.append(pi, pi[0])
    pl = ba.plan(7, 200, ci, pi)
    gp, ptr = pl["grp_ptr"], pl["pt_ptr"]
    G = len(gp) - 1
    o0 = ptr[gp[:-1]]
    # point groups: whole points, <= 128 obs each, covering every point once
    assert gp[0] == 0 and gp[-1] == 200 and (np.diff(gp) > 0).all()
    assert (ptr[gp[1:]] - o0 <= ba.GROUP_OBS).all()
    # camera slots: each observation exactly once, in its group and camera
    seen = np.zeros(len(ci), int)
    for g in range(G):
        for s in range(pl["grp_cslot"][g], pl["grp_cslot"][g + 1]):
            obs = o0[g] + pl["cslot_obs"][pl["cslot_obs_ptr"][s]:pl["cslot_obs_ptr"][s + 1]]
            assert (obs < ptr[gp[g + 1]]).all() and (pl["obs_cam"][obs] == pl["cslot_cam"][s]).all()
            seen[obs] += 1
    assert (seen == 1).all()
    # block slots: every within-point pair o1 < o2 once, in the block of its cameras
    exp = sum(n * (n - 1) // 2 for n in np.diff(ptr))
    tri = {tuple(b): k for k, b in enumerate(pl["blocks"])}
    got = 0
    for g in range(G):
        for s in range(pl["grp_bslot"][g], pl["grp_bslot"][g + 1]):
            pr = pl["bslot_pairs"][pl["bslot_pair_ptr"][s]:pl["bslot_pair_ptr"][s + 1]]
            a, b = o0[g] + (pr & 0xFFFF), o0[g] + (pr >> 16)
            assert (a < b).all() and (pl["obs_pt"][a] == pl["obs_pt"][b]).all()
            c1, c2 = pl["obs_cam"][a], pl["obs_cam"][b]
            assert (c1 <= c2).all()
            assert all(tri[(x, y)] == pl["bslot_blk"][s] for x, y in zip(c1, c2))
            got += len(pr)
    assert got == exp
    # partial rows: camera- / block-major, group order inside a camera / block
    for key, row, ptr_, grp in (("cslot_cam", "cslot_row", "cam_cslot_ptr", "grp_cslot"),
                                ("bslot_blk", "bslot_row", "blk_bslot_ptr", "grp_bslot")):
        owner = pl[key]
        rows = pl[row]
        assert np.array_equal(np.sort(rows), np.arange(len(rows)))
        sg = np.repeat(np.arange(G), np.diff(pl[grp]))
        for b in range(len(pl[ptr_]) - 1):
            sl = np.nonzero(owner == b)[0]
            assert np.array_equal(np.sort(rows[sl]), np.arange(pl[ptr_][b], pl[ptr_][b + 1]))
            assert (np.diff(sg[sl][np.argsort(rows[sl])]) >= 0).all()
    # the duplicate observation makes a (c, c) pair
    assert any(pl["blocks"][k][0] == pl["blocks"][k][1] for k in pl["bslot_blk"])
    assert len(pl["blocks"]) == 7 * 8 // 2 and (pl["blocks"][:, 0] <= pl["blocks"][:, 1]).all()
    assert np.array_equal(ba.block_index(pl["blocks"][:, 0], pl["blocks"][:, 1], 7),
                          np.arange(28))
    assert np.array_equal(ba.point_groups(np.array([0])), [0, 0])
    with pytest.raises(ValueError):
        ba.point_groups(np.array([0, 200]))
    # a camera with no observations still plans (sharded problems)
    pl2 = ba.plan(9, 200, ci, pi)
    assert len(pl2["blocks"]) == 45 and pl2["cam_cslot_ptr"][-1] == pl2["cam_cslot_ptr"][-2]


def test_bal_file_roundtrip(tmp_path):
    from slam355 import BundleAdjustment as B

    cams, pts, ci, pi, qs = make_problem(2, 4, 30, 3)
    fn = str(tmp_path / "p.txt")
    B.write_bal_data(fn, cams, pts, ci, pi, qs)
    c2, p2, ci2, pi2, q2 = B.read_bal_data(fn)
    assert np.array_equal(c2, cams) and np.array_equal(p2, pts)
    assert np.array_equal(ci2, ci) and np.array_equal(pi2, pi) and np.array_equal(q2, qs)


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_gpu_residual_matches_reference_objective(g):
    from slam355 import BundleAdjustment as B

    params = np.hstack((g["res_cams"].ravel(), g["res_pts"].ravel()))
    r = B.objective(params, 6, 300, g["res_cam_idx"], g["res_pt_idx"], g["res_qs"])
    ref = g["res_out"]
    assert np.all(np.abs(r - ref) <= 1e-9 * np.maximum(1.0, np.abs(ref)))


@pytest.mark.gpu
def test_gpu_jacobian_matches_oracle(g):
    from slam355 import ba

    cams, pts = g["res_cams"], g["res_pts"]
    ci, pi, qs = g["res_cam_idx"], g["res_pt_idx"], g["res_qs"]
    r, J = ba.residuals(cams, pts, ci, pi, qs, jacobian=True)
    er, eJ = oba.residual_and_jacobian(cams, pts, ci, pi, qs)
    assert np.all(np.abs(r - er) <= 1e-9 * np.maximum(1.0, np.abs(er)))
    assert np.all(np.abs(J - eJ) <= 1e-8 * np.maximum(1.0, np.abs(eJ)))


@pytest.mark.gpu
@pytest.mark.parametrize("dup,C,k,lin_mode", [(0, 6, 4, "auto"), (5, 6, 4, "auto"),
                                              (0, 6, 4, "slot"), (5, 6, 4, "slot"),
                                              (0, 12, 9, "auto")])
def test_gpu_lm_iterates_match_oracle(dup, C, k, lin_mode):
    """dup > 0: some points are observed twice by the same camera (a (c, c)
    pair inside the point's Schur block).  lin_mode "slot" runs the general
    linearisation (k_linearize) that points seen by more than MF_CAMS cameras
    need; the 9-camera tracks of the last case take it under "auto"."""
    from slam355 import ba

    cams, pts, ci, pi, qs = make_problem(3, C, 150, k)
    rng = np.random.default_rng(4)
    if dup:
        kk = rng.choice(len(ci), dup, replace=False)
        ci, pi = np.append(ci, ci[kk]), np.append(pi, pi[kk])
        qs = np.vstack([qs, qs[kk] + rng.normal(0, 0.5, (dup, 2))])
    cams0 = cams.copy()
    cams0[:, :3] += rng.normal(0, 1e-3, (C, 3))
    cams0[:, 3:6] += rng.normal(0, 1e-2, (C, 3))
    pts0 = pts + rng.normal(0, 0.05, pts.shape)
    prob = ba.BAProblem(cams0, pts0, ci, pi, qs, lin_mode=lin_mode)
    assert prob.lin_mode == ("slot" if lin_mode == "slot" or k > ba.MF_CAMS else "mfma")
    st = oba.LMState(1e-4)
    oc, op = cams0.copy(), pts0.copy()
    for it in range(8):
        prob.iterate(1)
        oc, op, info = oba.lm_iteration(oc, op, ci, pi, qs, st)
        s = prob.state()
        assert bool(s["ACCEPTED"]) == bool(info["accepted"]), it
        assert abs(s["COST_NEW"] - info["cost_new"]) <= 1e-9 * info["cost_new"] + 1e-12, it
        assert abs(s["LAMBDA"] - st.lam) <= 1e-6 * st.lam, it
        gc, gp = prob.params()
        assert np.allclose(gc, oc, rtol=1e-6, atol=1e-9), it
        assert np.allclose(gp, op, rtol=1e-6, atol=1e-9), it


@pytest.mark.gpu
def test_gpu_graph_replay_matches_eager():
    """LM iterations replayed from a captured HIP graph are bit-identical to
    eager launches (same kernels, same order)."""
    from slam355 import ba

    cams, pts, ci, pi, qs = make_problem(7, 10, 800, 5)
    rng = np.random.default_rng(8)
    cams0 = cams.copy()
    cams0[:, 3:6] += rng.normal(0, 1e-2, (10, 3))
    pts0 = pts + rng.normal(0, 0.05, pts.shape)
    a = ba.BAProblem(cams0, pts0, ci, pi, qs)
    b = ba.BAProblem(cams0, pts0, ci, pi, qs)
    a.iterate(6)
    b.iterate_graphed(3)
    b.iterate_graphed(3)
    assert a.state() == b.state()
    for x, y in zip(a.params(), b.params()):
        assert np.array_equal(x, y)
    b.restore()
    b.iterate_graphed(3)
    a.restore()
    a.iterate(3)
    assert a.state() == b.state()


@pytest.mark.gpu
def test_gpu_solver_reaches_reference_optimum(g):
    from slam355 import BundleAdjustment as B

    A = B.bundle_adjustment_sparsity(5, 120, g["sol_cam_idx"], g["sol_pt_idx"])
    r0, rf, x = B.bundle_adjustment_with_sparsity(g["sol_cams0"], g["sol_pts0"], g["sol_cam_idx"],
                                                  g["sol_pt_idx"], g["sol_qs"], A)
    assert np.allclose(r0, g["sol_ref_r0"], rtol=1e-9, atol=1e-9)
    cost = 0.5 * float(np.sum(rf ** 2))
    assert cost <= float(g["sol_tight_cost"]) * (1 + 1e-6)
    # same optimum as the oracle LM (gauge fixed identically: same start, same algorithm)
    oc, op, hist = oba.lm_solve(g["sol_cams0"], g["sol_pts0"], g["sol_cam_idx"], g["sol_pt_idx"],
                                g["sol_qs"], iters=60)
    assert abs(cost - hist[-1]["cost"]) <= 1e-6 * cost
    cams = x[:45].reshape(5, 9)
    A_ = np.vstack([oba.camera_centers(cams), x[45:].reshape(-1, 3)])
    B_ = np.vstack([oba.camera_centers(oc), op])
    s, R, t = oba.sim3_align(A_, B_)
    err = np.abs((s * (R @ A_.T)).T + t - B_).max() / np.abs(B_).max()
    assert err < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("C,P,k", [(10, 5000, 6), (13, 2500, 5), (16, 3000, 5)])
def test_gpu_local_ba_config3_converges(C, P, k):
    """C3 shape (10 KF x 5k pts x 30k obs) and 9C > 120 cases (tiled multi-workgroup Cholesky)."""
    from slam355 import ba

    cams, pts, ci, pi, qs = make_problem(5 + C, C, P, k)
    rng = np.random.default_rng(6)
    cams0 = cams.copy()
    cams0[:, :3] += rng.normal(0, 1e-3, (C, 3))
    cams0[:, 3:6] += rng.normal(0, 1e-2, (C, 3))
    pts0 = pts + rng.normal(0, 0.05, pts.shape)
    prob = ba.BAProblem(cams0, pts0, ci, pi, qs)
    c0 = 0.5 * float(np.sum(oba.residual_and_jacobian(cams0, pts0, ci, pi, qs)[0] ** 2))
    st = prob.solve(max_iters=60, ftol=1e-12)
    # converged to the noise floor: 0.5 * sum r^2 ~ 0.5 * (2O - n_params) * sigma^2
    O = len(ci)
    floor = 0.5 * (2 * O - 9 * C - 3 * P) * 0.25
    assert 0.9 * floor < st["COST"] < 1.1 * floor
    assert st["COST"] < 0.1 * c0
    gc, gp = prob.params()
    r = oba.residual_and_jacobian(gc, gp, ci, pi, qs)[0]
    assert abs(0.5 * float(np.sum(r * r)) - st["COST"]) <= 1e-8 * st["COST"]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["flow", "levels", "flow/cams:5", "levels/cams:7:2"])
@pytest.mark.parametrize("C,P,k", [(14, 400, 4), (40, 1500, 5), (130, 3000, 6)])
def test_gpu_tiled_solver_iterates_match_oracle(C, P, k, mode):
    """9C > 120: the reduced camera system goes through the tiled Cholesky
    (k_tl3_flow or k_tl2_*; 2, 6 and 19 tiles of 64 rows, or tiles of whole
    cameras with padding rows, whose blocks the factor skips).  The
    130-camera trajectory window is block-banded (points seen by 6
    consecutive keyframes), so most tiles stay structurally zero and are
    skipped.  LM iterates equal the oracle's Schur LM."""
    from slam355 import ba

    cams, pts, ci, pi, qs = make_problem(11 + C, C, P, k)
    rng = np.random.default_rng(C)
    cams0 = cams.copy()
    cams0[:, :3] += rng.normal(0, 1e-3, (C, 3))
    cams0[:, 3:6] += rng.normal(0, 1e-2, (C, 3))
    pts0 = pts + rng.normal(0, 0.05, pts.shape)
    tl, _, tiles = mode.partition("/")
    prob = ba.BAProblem(cams0, pts0, ci, pi, qs, tl_mode=tl, tile_mode=tiles or None)
    st = oba.LMState(1e-4)
    oc, op = cams0.copy(), pts0.copy()
    pairs = oba._obs_pairs(ci, pi)
    for it in range(5):
        prob.iterate(1)
        oc, op, info = oba.lm_iteration_schur(oc, op, ci, pi, qs, st, pairs)
        s = prob.state()
        assert s["CHOL_FAIL"] == 0.0, it
        assert bool(s["ACCEPTED"]) == bool(info["accepted"]), it
        assert abs(s["COST_NEW"] - info["cost_new"]) <= 1e-8 * info["cost_new"] + 1e-12, it
        assert abs(s["LAMBDA"] - st.lam) <= 1e-6 * st.lam, it
        gc, gp = prob.params()
        assert np.allclose(gc, oc, rtol=1e-6, atol=1e-9), it
        assert np.allclose(gp, op, rtol=1e-6, atol=1e-9), it


@pytest.mark.gpu
@pytest.mark.parametrize("C,P,k,tiles", [(60, 3000, 8, "rows64"), (40, 2000, 7, "cams:3"),
                                         (60, 3000, 8, "cams:5")])
def test_gpu_flow_product_tasks_of_deeper_rows_equal_level_solve(C, P, k, tiles):
    """Closed loops seen 7-8 keyframes per point: their tile columns have three
    and more row tiles, so some product tasks form L_Ik L_Jk^T for a column J
    that is not the task owner's first row tile (the owner reloads that tile
    instead of keeping it in registers).  Four LM iterates of the dataflow
    solve equal those of the level-scheduled solve, which forms every such
    term itself (k_tl2_update): accept flags, costs to 1e-8, cameras to the
    oracle tests' 1e-6 / 1e-9, points to 1e-6 of their largest coordinate
    (the sums run in other orders, and these loops amplify rounding over the
    iterations; a wrong term would show at O(1)); both solve forms are checked
    against the oracle's Schur LM above."""
    from slam355 import ba
    from slam355.synthetic import ba_problem_loop

    rng = np.random.default_rng(5)
    cams, pts, ci, pi, qs = ba_problem_loop(rng, C, P, k)
    cams0 = cams.copy()
    cams0[:, :3] += rng.normal(0, 1e-3, (C, 3))
    cams0[:, 3:6] += rng.normal(0, 1e-2, (C, 3))
    pts0 = pts + rng.normal(0, 0.05, pts.shape)
    runs = {}
    for mode in ("flow", "levels"):
        prob = ba.BAProblem(cams0, pts0, ci, pi, qs, tl_mode=mode, tile_mode=tiles)
        if mode == "flow":
            S = prob._sched_host
            T, pt = int(S[1]), int(S[10])
            tasks = np.concatenate([S[S[pt + 2 * J]:S[pt + 2 * J] + 3 * S[pt + 2 * J + 1]]
                                    for J in range(T)]).reshape(-1, 3)
            assert (tasks[:, 0] > 0).any()  # the reload path is taken
        out = []
        for _ in range(4):
            prob.iterate(1)
            s = prob.state()
            assert s["CHOL_FAIL"] == 0.0
            out.append((s["COST_NEW"], s["ACCEPTED"], *prob.params()))
        runs[mode] = out
        del prob
    for a, b in zip(runs["flow"], runs["levels"]):
        assert a[1] == b[1] and abs(a[0] - b[0]) <= 1e-8 * abs(b[0])
        assert np.allclose(a[2], b[2], rtol=1e-6, atol=1e-9)
        # points as a whole (a few low-parallax loop points are ill-determined)
        assert np.abs(a[3] - b[3]).max() <= 1e-6 * np.abs(b[3]).max()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["flow", "levels"])
def test_gpu_tiled_solve_failure_leaves_a_zero_step(mode):
    """A damping that makes the camera system indefinite (lambda = -1e6): the
    tiled factor fails (CHOL_FAIL 1, not a timed-out wait), the step is
    rejected and the parameters stay; the solve's epilogue writes a zero camera
    step and trial cameras equal to the live ones -- in the dataflow form after
    the per-tile epilogue shares have written theirs (the last retirer's
    failure path overwrites them)."""
    import torch
    from slam355 import ba

    cams, pts, ci, pi, qs = make_problem(44, 40, 1500, 5)
    prob = ba.BAProblem(cams, pts, ci, pi, qs, tl_mode=mode)
    c_before, p_before = prob.params()
    prob.reset(-1e6)
    prob.iterate(1)
    torch.cuda.synchronize()
    st = prob.state()
    assert st["CHOL_FAIL"] == 1.0 and st["ACCEPTED"] == 0.0 and st["SOLVE_FAULT"] == 0.0
    c_after, p_after = prob.params()
    assert np.array_equal(c_after, c_before) and np.array_equal(p_after, p_before)
    cur = int(st["CUR"] != 0)
    assert not prob.t["delta_c"].cpu().numpy().any()
    assert np.array_equal(prob.t[f"cams{1 - cur}"].cpu().numpy(), prob.t[f"cams{cur}"].cpu().numpy())


def test_planner_packed_block_list():
    """9C > 120: the plan lists only the diagonal and the camera pairs with a
    common point (the packed sys layout); an explicit global list is honoured
    and a list that misses a local block is rejected."""
    from slam355 import ba

    C = 20
    cams, pts, ci, pi, qs = make_problem(3, C, 300, 4)
    pl = ba.plan(C, len(pts), ci, pi)
    blocks = {tuple(b) for b in pl["blocks"]}
    pairs = {(min(a, b), max(a, b)) for p in range(len(pts))
             for a in ci[pi == p] for b in ci[pi == p]}
    assert blocks == pairs | {(c, c) for c in range(C)}
    full = ba.block_index(*np.triu_indices(C), C)
    pl2 = ba.plan(C, len(pts), ci, pi, block_list=full)
    assert len(pl2["blocks"]) == C * (C + 1) // 2
    with pytest.raises(ValueError):
        ba.plan(C, len(pts), ci, pi, block_list=ba.block_index(np.arange(C), np.arange(C), C))


# ----------------------------------------------------------------------------- batched windows
def _window(seed, C, P, k):
    cams, pts, ci, pi, qs = make_problem(seed, C, P, k)
    rng = np.random.default_rng(seed + 100)
    cams0 = cams.copy()
    cams0[:, :3] += rng.normal(0, 1e-3, (C, 3))
    cams0[:, 3:6] += rng.normal(0, 1e-2, (C, 3))
    return cams0, pts + rng.normal(0, 0.05, pts.shape), ci, pi, qs


WINDOWS = [(31, 10, 5000, 6), (32, 8, 1200, 5), (33, 6, 700, 4), (34, 10, 3000, 6), (35, 12, 900, 3)]


@pytest.mark.gpu
def test_gpu_batched_windows_equal_solo_iterates():
    """slam_ba_iterate_batch: windows of different shapes (C3 = 10 x 5000 x 30k
    among them) advanced together give, bit for bit, the LM state and
    parameters each gets from solo iterations; graph replay with restore too."""
    import torch
    from slam355 import ba

    wins = [_window(*w) for w in WINDOWS]
    solo = [ba.BAProblem(*w) for w in wins]
    for p in solo:
        p.iterate(6)
    batch = ba.BABatch([ba.BAProblem(*w) for w in wins])
    batch.iterate(4)
    batch.iterate(2)
    for a, b in zip(solo, batch.problems):
        assert a.state() == b.state()
        for x, y in zip(a.params(), b.params()):
            assert np.array_equal(x, y)
    for _ in range(2):  # replayed graph of (restore + 6 iterations), twice
        batch.iterate_graphed(6, with_restore=True)
    torch.cuda.synchronize()
    for a, b in zip(solo, batch.problems):
        assert a.state() == b.state()


@pytest.mark.gpu
def test_gpu_batched_windows_full_launch_and_split():
    """More windows than one batched launch takes (SLAM_BA_MAX_BATCH = 16: the
    descriptors travel by value in the kernel arguments): 16 windows in one
    launch, the 2 left over in a second; every window's iterates equal its solo
    iterates bit for bit."""
    from slam355 import ba

    assert ba.BABatch.MAX_BATCH == 16
    shapes = [(60 + i, 6 + (i % 3), 300 + 40 * i, 3 + (i % 2)) for i in range(18)]
    wins = [_window(*w) for w in shapes]
    solo = [ba.BAProblem(*w) for w in wins]
    for p in solo:
        p.iterate(3)
    batch = ba.BABatch([ba.BAProblem(*w) for w in wins])
    batch.iterate(3)
    for a, b in zip(solo, batch.problems):
        assert a.state() == b.state()
        for x, y in zip(a.params(), b.params()):
            assert np.array_equal(x, y)


@pytest.mark.gpu
def test_gpu_batched_windows_match_oracle_schur_lm():
    """Per window of a batch, 3 LM iterations (C3 included) equal the oracle's
    Schur LM (oracle.ba.lm_iteration_schur): accept flags, costs 1e-9, lambda,
    parameters 1e-6."""
    from slam355 import ba

    wins = [_window(*w) for w in WINDOWS[:4]]
    batch = ba.BABatch([ba.BAProblem(*w) for w in wins])
    ost = [oba.LMState(1e-4) for _ in wins]
    cur = [(w[0].copy(), w[1].copy()) for w in wins]
    pairs = [oba._obs_pairs(w[2], w[3]) for w in wins]
    for it in range(3):
        batch.iterate(1)
        for i, w in enumerate(wins):
            oc, op, info = oba.lm_iteration_schur(cur[i][0], cur[i][1], w[2], w[3], w[4], ost[i],
                                                  pairs[i])
            cur[i] = (oc, op)
            s = batch.problems[i].state()
            assert bool(s["ACCEPTED"]) == bool(info["accepted"]), (i, it)
            assert abs(s["COST_NEW"] - info["cost_new"]) <= 1e-9 * info["cost_new"], (i, it)
            assert abs(s["LAMBDA"] - ost[i].lam) <= 1e-6 * ost[i].lam, (i, it)
            gc, gp = batch.problems[i].params()
            assert np.allclose(gc, oc, rtol=1e-6, atol=1e-9), (i, it)
            assert np.allclose(gp, op, rtol=1e-6, atol=1e-9), (i, it)


@pytest.mark.gpu
def test_gpu_c4_window_iterates_match_oracle():
    """BASELINE C4 shape on one GPU (64 KF x 50k points x 300k obs, the tiled
    solver on the packed 576-unknown system): 2 LM iterations equal the
    oracle's Schur LM."""
    from slam355 import ba
    from slam355.synthetic import ba_problem, perturb

    rng = np.random.default_rng(7)
    cams, pts, ci, pi, qs = ba_problem(rng, 64, 50000, 6)
    c0, p0 = perturb(rng, cams, pts)
    prob = ba.BAProblem(c0, p0, ci, pi, qs)
    st = oba.LMState(1e-4)
    oc, op = c0.copy(), p0.copy()
    pairs = oba._obs_pairs(ci, pi)
    for it in range(2):
        prob.iterate(1)
        oc, op, info = oba.lm_iteration_schur(oc, op, ci, pi, qs, st, pairs)
        s = prob.state()
        assert s["CHOL_FAIL"] == 0.0 and bool(s["ACCEPTED"]) == bool(info["accepted"]), it
        assert abs(s["COST_NEW"] - info["cost_new"]) <= 1e-9 * info["cost_new"], it
        gc, gp = prob.params()
        assert np.allclose(gc, oc, rtol=1e-6, atol=1e-9), it
        assert np.allclose(gp, op, rtol=1e-6, atol=1e-9), it


def _masked_stream(n_cus):
    """A torch stream whose kernels may use only CUs 0 .. n_cus - 1
    (hipExtStreamCreateWithCUMask) and its destructor."""
    import ctypes
    import os

    import torch

    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"),
                      mode=ctypes.RTLD_GLOBAL)
    n_total = torch.cuda.get_device_properties(0).multi_processor_count
    mask = (ctypes.c_uint32 * ((n_total + 31) // 32))()
    for i in range(n_cus):
        mask[i // 32] |= 1 << (i % 32)
    h = ctypes.c_void_p()
    assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), len(mask), mask) == 0
    return torch.cuda.ExternalStream(h.value), lambda: (torch.cuda.synchronize(),
                                                        hip.hipStreamDestroy(h))


@pytest.mark.gpu
@pytest.mark.parametrize("n_cus", [2, 4])
def test_gpu_flow_solve_with_fewer_cus_than_columns(n_cus):
    """k_tl3_flow makes no residency assumption.  The C4 solve has
    9 tile columns (one ~100 KB-LDS workgroup per CU); on a stream masked to 2
    or 4 CUs at most that many columns are resident at a time, yet the LM
    iterates equal the unmasked solve's bit for bit and no wait times out."""
    import torch
    from slam355 import ba
    from slam355.synthetic import ba_problem, perturb

    rng = np.random.default_rng(7)
    cams, pts, ci, pi, qs = ba_problem(rng, 64, 50000, 6)
    c0, p0 = perturb(rng, cams, pts)
    solo = ba.BAProblem(c0, p0, ci, pi, qs)
    solo.iterate(3)
    st, destroy = _masked_stream(n_cus)
    try:
        with torch.cuda.stream(st):
            prob = ba.BAProblem(c0, p0, ci, pi, qs, stream=st)
            prob.iterate(3)
        torch.cuda.synchronize()
        assert prob.state() == solo.state()  # state() raises on a timed-out wait
        for x, y in zip(prob.params(), solo.params()):
            assert np.array_equal(x, y)
        del prob
    finally:
        destroy()


@pytest.mark.gpu
def test_gpu_flow_solve_under_concurrent_orb():
    """C4 LM iterations (9 tile columns of k_tl3_flow) on one stream
    while ORB batches (79 KB of LDS per workgroup, thousands of workgroups) hold
    the CUs from another stream: the iterates equal those of the same solve
    alone, bit for bit, with no timed-out wait (state() would raise)."""
    import torch
    from slam355 import ba, orb
    from slam355.synthetic import ba_problem, perturb

    rng = np.random.default_rng(7)
    cams, pts, ci, pi, qs = ba_problem(rng, 64, 50000, 6)
    c0, p0 = perturb(rng, cams, pts)
    solo = ba.BAProblem(c0, p0, ci, pi, qs)
    solo.iterate(3)
    torch.cuda.synchronize()
    imgs = torch.randint(0, 256, (65, 720, 1280), dtype=torch.uint8, device="cuda")
    ows = orb.OrbWorkspace(65, 720, 1280, 64)
    s_orb, s_ba = torch.cuda.Stream(), torch.cuda.Stream()
    with torch.cuda.stream(s_ba):
        prob = ba.BAProblem(c0, p0, ci, pi, qs, stream=s_ba)
    torch.cuda.synchronize()
    ows.run(imgs, s_orb)  # the first ORB batch is queued ahead of the solve
    with torch.cuda.stream(s_ba):
        prob.iterate(3)
    for _ in range(3):
        ows.run(imgs, s_orb)
    torch.cuda.synchronize()
    st = prob.state()
    assert st == solo.state()
    for x, y in zip(prob.params(), solo.params()):
        assert np.array_equal(x, y)


@pytest.mark.gpu
def test_gpu_c5_global_ba_first_iteration_matches_oracle():
    """BASELINE C5 shape (loop-closure global BA, 500 KF x 200k points x 1.2M
    obs, 4500-unknown reduced system): the first LM iteration's accept flag,
    trial cost and camera step equal the oracle's Schur LM."""
    from slam355 import ba
    from slam355.synthetic import ba_problem_loop, perturb

    rng = np.random.default_rng(7)
    cams, pts, ci, pi, qs = ba_problem_loop(rng, 500, 200000, 6)
    c0, p0 = perturb(rng, cams, pts)
    prob = ba.BAProblem(c0, p0, ci, pi, qs)
    prob.iterate(1)
    st = oba.LMState(1e-4)
    oc, op, info = oba.lm_iteration_schur(c0, p0, ci, pi, qs, st, oba._obs_pairs(ci, pi))
    s = prob.state()
    assert s["CHOL_FAIL"] == 0.0 and bool(s["ACCEPTED"]) == bool(info["accepted"])
    assert abs(s["COST_NEW"] - info["cost_new"]) <= 1e-9 * info["cost_new"]
    assert abs(s["COST"] - info["cost_new" if info["accepted"] else "cost"]) <= 1e-9 * s["COST"]
    gc, gp = prob.params()
    assert np.allclose(gc, oc, rtol=1e-6, atol=1e-9)
    assert np.allclose(gp, op, rtol=1e-6, atol=1e-9)


# ----------------------------------------------------------------------------- camera-union plan
def _emulate_union_linearisation(pl, C, cams, pts_new, qs_sorted, lam):
    """numpy restatement of csrc/ba.hip k_lin_mfma + k_assemble over the
    plan_mfma tables -> dense undamped reduced system S [9C, 9C], b [9C]."""
    ci = pl["obs_cam"].astype(np.int64)
    pi = pl["obs_pt"].astype(np.int64)
    r, J = oba.residual_and_jacobian(cams, pts_new, ci, pi, qs_sorted)
    Jc, Jp = J[:, :, :9], J[:, :, 9:]
    P = len(pts_new)
    V = np.zeros((P, 3, 3))
    np.add.at(V, pi, np.einsum("oai,oaj->oij", Jp, Jp))
    g = np.zeros((P, 3))
    np.add.at(g, pi, -np.einsum("oai,oa->oi", Jp, r))
    D = np.clip(np.diagonal(V, axis1=1, axis2=2), oba.DIAG_MIN, oba.DIAG_MAX)
    Vi = np.linalg.inv(V + lam * D[:, :, None] * np.eye(3)[None])
    e = np.einsum("pij,pj->pi", Vi, g)
    u = np.einsum("oai,oi->oa", Jp, e[pi])
    cpart = np.zeros((len(pl["cslot_cam"]), 112))
    bpart = np.zeros((len(pl["bslot_blk"]), 81))
    for sg in range(len(pl["sg_ptr"]) - 1):
        cams_sg = pl["sg_cams"][sg][pl["sg_cams"][sg] >= 0]
        m = len(cams_sg)
        T = np.zeros((9 * m, 9 * m))
        Ua = np.zeros((m, 9, 9))
        vec = np.zeros((m, 28))
        for ch in range(pl["sg_ptr"][sg], pl["sg_ptr"][sg + 1]):
            p0, p1 = pl["grp_ptr"][ch], pl["grp_ptr"][ch + 1]
            o0, o1 = pl["pt_ptr"][p0], pl["pt_ptr"][p1]
            assert o1 - o0 <= 120 and p1 - p0 <= 16
            for q in range(p0, p1):
                Wp = np.zeros((9 * m, 3))
                for o in range(pl["pt_ptr"][q], pl["pt_ptr"][q + 1]):
                    a = pl["obs_la"][o]
                    assert cams_sg[a] == ci[o]
                    Wp[9 * a:9 * a + 9] += Jc[o].T @ Jp[o]
                T += (Wp @ Vi[q]) @ Wp.T
            cp = pl["chk_cptr"][ch]
            for a in range(m):
                for k in pl["chk_cobs"][o0 + cp[a]:o0 + cp[a + 1]]:
                    o = o0 + k
                    assert pl["obs_la"][o] == a
                    Ua[a] += Jc[o].T @ Jc[o]
                    vec[a, :9] += Jc[o].T @ r[o]
                    vec[a, 9:18] += Jc[o].T @ u[o]
                    vec[a, 18:27] += np.einsum("ai,ai->i", Jc[o], Jc[o])
                    vec[a, 27] += r[o] @ r[o]
        for a in range(m):
            row = pl["cslot_row"][pl["grp_cslot"][sg] + a]
            cpart[row, :81] = (Ua[a] - T[9 * a:9 * a + 9, 9 * a:9 * a + 9]).ravel()
            cpart[row, 81:109] = vec[a]
        for s in range(pl["grp_bslot"][sg], pl["grp_bslot"][sg + 1]):
            a, b = pl["bslot_ab"][s] & 255, pl["bslot_ab"][s] >> 8
            bpart[pl["bslot_row"][s]] = T[9 * a:9 * a + 9, 9 * b:9 * b + 9].ravel()
    S = np.zeros((9 * C, 9 * C))
    bvec = np.zeros(9 * C)
    for k, (c1, c2) in enumerate(pl["blocks"]):
        rows_b = bpart[pl["blk_bslot_ptr"][k]:pl["blk_bslot_ptr"][k + 1]].sum(0).reshape(9, 9)
        if c1 == c2:
            cp = cpart[pl["cam_cslot_ptr"][c1]:pl["cam_cslot_ptr"][c1 + 1]].sum(0)
            S[9 * c1:9 * c1 + 9, 9 * c1:9 * c1 + 9] = cp[:81].reshape(9, 9)
            bvec[9 * c1:9 * c1 + 9] = -cp[81:90] - cp[90:99]
        else:
            S[9 * c1:9 * c1 + 9, 9 * c2:9 * c2 + 9] = -rows_b
            S[9 * c2:9 * c2 + 9, 9 * c1:9 * c1 + 9] = -rows_b.T
    return S, bvec


def _dense_reduced_system(cams, pts, ci, pi, qs, lam):
    r, J = oba.residual_and_jacobian(cams, pts, ci, pi, qs)
    C = len(cams)
    Jc, Jp = J[:, :, :9], J[:, :, 9:]
    Jd = np.zeros((2 * len(ci), 9 * C + 3 * len(pts)))
    for o in range(len(ci)):
        Jd[2 * o:2 * o + 2, 9 * ci[o]:9 * ci[o] + 9] = Jc[o]
        Jd[2 * o:2 * o + 2, 9 * C + 3 * pi[o]:9 * C + 3 * pi[o] + 3] = Jp[o]
    H = Jd.T @ Jd
    gr = -Jd.T @ r.ravel()
    n = 9 * C
    A, Bm, Dm = H[:n, :n], H[:n, n:], H[n:, n:]
    Dd = np.clip(np.diag(Dm), oba.DIAG_MIN, oba.DIAG_MAX)
    Dinv = np.linalg.inv(Dm + lam * np.diag(Dd))
    return A - Bm @ Dinv @ Bm.T, gr[:n] - Bm @ Dinv @ gr[n:]


@pytest.mark.parametrize("case", ["local", "dup", "packed", "loop"])
def test_union_plan_assembles_the_reduced_system(case):
    """ba.plan_mfma's chunks / supergroups / slot rows, run through a numpy
    restatement of k_lin_mfma + k_assemble, give the Schur-reduced camera
    system of the dense normal equations (points renumbered by camera span)."""
    from slam355 import ba
    from slam355.synthetic import ba_problem_loop

    if case == "loop":
        cams, pts, ci, pi, qs = ba_problem_loop(np.random.default_rng(3), 16, 120, 4)
    else:
        C = 16 if case == "packed" else 7
        cams, pts, ci, pi, qs = make_problem(3, C, 90, 4)
    if case == "dup":
        k = np.random.default_rng(1).choice(len(ci), 6, replace=False)
        ci, pi, qs = np.append(ci, ci[k]), np.append(pi, pi[k]), np.vstack([qs, qs[k] + 0.3])
    C = len(cams)
    pts = pts + np.random.default_rng(2).normal(0, 0.05, pts.shape)
    pl = ba.plan_mfma(C, len(pts), ci, pi, chunks_per_wg=2)
    assert pl is not None
    perm = pl["perm"]
    assert np.array_equal(np.sort(perm), np.arange(len(pts)))
    assert all((pl["sg_cams"][s] >= 0).sum() <= ba.MF_CAMS for s in range(pl["n_sgrps"]))
    S, b = _emulate_union_linearisation(pl, C, cams, pts[perm], qs[pl["order"]], 1e-3)
    Sr, br = _dense_reduced_system(cams, pts, ci, pi, qs, 1e-3)
    scale = np.abs(Sr).max()
    assert np.abs(S - Sr).max() <= 1e-9 * scale
    assert np.abs(b - br).max() <= 1e-9 * max(1.0, np.abs(br).max())


def _tiled_system(S, b, sched):
    """S, b laid out in the schedule's tiles (row map: row of S -> row of the
    tiled system; the rows past a tile's cameras are padding with a unit
    diagonal): (A [N, N], b [N], row map [n])."""
    T, n, TB = int(sched[1]), len(b), 64
    N = T * TB
    rn = sched[sched[2]:sched[2] + n].astype(np.int64)
    irow = sched[sched[3]:sched[3] + N]
    A = np.zeros((N, N))
    A[np.ix_(rn, rn)] = S
    pad = np.nonzero(irow < 0)[0]
    A[pad, pad] = 1.0
    bb = np.zeros(N)
    bb[rn] = b
    return A, bb, rn


def _emulate_tl_levels(S, b, sched):
    """The level-scheduled tiled solve (csrc/ba.hip k_tl2_*) restated in NumPy,
    launch by launch: S laid out in the schedule's tiles of whole cameras, each level's
    panels (diagonal factor + inverse, y_k; L_Ik = A_Ik L_kk^-T), then its
    updates (A_IJ -= sum_k L_Ik L_Jk^T, b_I -= sum_k L_Ik y_k), then the back
    substitution by levels in reverse, x un-permuted."""
    nlev, T = int(sched[0]), int(sched[1])
    tab = sched[sched[4]:sched[4] + 6 * nlev].reshape(-1, 6)
    n, TB = len(b), 64
    N = T * TB
    A, bb, rn = _tiled_system(S, b, sched)
    t = lambda I: slice(I * TB, (I + 1) * TB)  # noqa: E731
    dinv, y, x = {}, np.zeros(N), np.zeros(N)
    for lv in range(nlev):
        po, pc, uo, uc, bo, bc = tab[lv]
        ent = sched[po:po + 2 * pc].reshape(-1, 2)
        for k in ent[ent[:, 0] == ent[:, 1], 0]:
            Lkk = np.linalg.cholesky(A[t(k), t(k)])
            dinv[k] = np.linalg.inv(Lkk)
            y[t(k)] = dinv[k] @ bb[t(k)]
        for k, I in ent[ent[:, 0] != ent[:, 1]]:
            A[t(I), t(k)] = A[t(I), t(k)] @ dinv[k].T
        for I, J, ko, kc in sched[uo:uo + 4 * uc].reshape(-1, 4):
            ks = sched[ko:ko + kc]
            A[t(I), t(J)] -= sum(A[t(I), t(k)] @ A[t(J), t(k)].T for k in ks)
            if I == J:
                bb[t(I)] -= sum(A[t(I), t(k)] @ y[t(k)] for k in ks)
    for lv in reversed(range(nlev)):
        po, pc, uo, uc, bo, bc = tab[lv]
        for k, so, sc in sched[bo:bo + 3 * bc].reshape(-1, 3):
            r = y[t(k)].copy()
            for I in sched[so:so + sc]:
                r -= A[t(I), t(k)].T @ x[t(I)]
            x[t(k)] = dinv[k].T @ r
    return x[rn]


@pytest.mark.parametrize("mode", ["rows64", "cams:5", "cams:7:2"])
@pytest.mark.parametrize("C,loop", [(30, False), (64, False), (120, True)])
def test_tl_level_schedule_solves_the_camera_system(C, loop, mode):
    """Nested-dissection level schedule of the tiled solver: row map and
    inverse consistent, each tile's rows first and its padding after them
    (whole cameras in the "cams" tilings), every level's columns independent
    (no L between them), a banded window in ~log2(T) levels (C4's 64
    keyframes: 4), and executing the schedule tile by tile solves S x = b."""
    from slam355.ba import tl_schedule, upper_blocks
    from slam355.synthetic import ba_problem, ba_problem_loop

    rng = np.random.default_rng(C)
    cams, pts, ci, pi, qs = (ba_problem_loop if loop else ba_problem)(rng, C, 40 * C, 5)
    ub = upper_blocks(C, ci, pi)
    iu, ju = np.triu_indices(C)
    blocks = np.stack([iu[ub], ju[ub]], 1)
    sched = tl_schedule(C, blocks, mode)
    nlev, T = int(sched[0]), int(sched[1])
    assert T >= -(-9 * C // 64) and nlev <= 2 + 2 * int(np.ceil(np.log2(T)))
    if C == 64:
        assert nlev == 4
    rn = sched[sched[2]:sched[2] + 9 * C].astype(np.int64)
    irow = sched[sched[3]:sched[3] + 64 * T]
    nrow = sched[sched[6]:sched[6] + T]
    assert nrow.sum() == 9 * C and nrow.min() >= 1 and nrow.max() <= 64
    assert np.array_equal(irow[rn], np.arange(9 * C)) and (irow >= 0).sum() == 9 * C
    if mode == "rows64":
        assert T == -(-9 * C // 64)
    for I in range(T):  # the tile's rows first, padding after
        tr = irow[64 * I:64 * I + 64]
        assert (tr[:nrow[I]] >= 0).all() and (tr[nrow[I]:] < 0).all()
        if mode != "rows64":  # whole cameras
            assert nrow[I] % 9 == 0 and (tr[:nrow[I]:9] % 9 == 0).all()
    # S: random SPD with exactly the camera-block pattern
    n = 9 * C
    M = np.zeros((n, n))
    for c1, c2 in blocks:
        M[9 * c1:9 * c1 + 9, 9 * c2:9 * c2 + 9] = rng.normal(size=(9, 9))
    S = M + M.T + np.diag(np.abs(M).sum(1) + np.abs(M).sum(0) + 1.0)
    b = rng.normal(size=n)
    x = _emulate_tl_levels(S, b, sched)
    assert np.allclose(x, np.linalg.solve(S, b), rtol=0, atol=1e-10 * np.abs(x).max())


@pytest.mark.parametrize("mode", ["rows64", "cams:5"])
@pytest.mark.parametrize("C,loop", [(30, False), (120, True)])
def test_tl_gather_tables_lay_out_the_system(C, loop, mode):
    """The dataflow solve's gather tables (k_tl3_flow reads its diagonal and
    row tiles straight from the packed system): every element of every
    structural tile, looked up in a packed S with the damping on the diagonal,
    equals the tiled layout of S (unit diagonal on padding rows, zeros off the
    blocks)."""
    from slam355.ba import tl_schedule, upper_blocks
    from slam355.synthetic import ba_problem, ba_problem_loop

    rng = np.random.default_rng(C + 7)
    cams, pts, ci, pi, qs = (ba_problem_loop if loop else ba_problem)(rng, C, 20 * C, 5)
    ub = upper_blocks(C, ci, pi)
    iu, ju = np.triu_indices(C)
    blocks = np.stack([iu[ub], ju[ub]], 1)
    sched = tl_schedule(C, blocks, mode)
    n, T = 9 * C, int(sched[1])
    packed = rng.normal(size=(len(blocks), 9, 9))
    dU, lam = rng.uniform(1.0, 2.0, n), 0.37
    Sd = np.zeros((n, n))
    for k, (c1, c2) in enumerate(blocks):
        Sd[9 * c1:9 * c1 + 9, 9 * c2:9 * c2 + 9] = packed[k]
        if c1 != c2:
            Sd[9 * c2:9 * c2 + 9, 9 * c1:9 * c1 + 9] = packed[k].T
    Sd[np.arange(n), np.arange(n)] += lam * dU
    A, _, _ = _tiled_system(Sd, np.zeros(n), sched)
    flat = packed.ravel()
    rec = sched[sched[5]:sched[5] + 5 * T].reshape(-1, 5)
    for J in range(T):
        ro, rc = rec[J][:2]
        base = int(sched[sched[9] + J])
        dg = sched[base + (1 + rc) * 4096:base + (1 + rc) * 4096 + 64]
        for q, I in enumerate([J] + list(sched[ro:ro + rc])):
            g = sched[base + q * 4096:base + (q + 1) * 4096].reshape(64, 64).astype(np.int64)
            got = np.where(g >= 0, flat[np.maximum(g, 0)], np.where(g == -2, 1.0, 0.0))
            if q == 0:
                d = np.arange(64)
                got[d[dg >= 0], d[dg >= 0]] += lam * dU[dg[dg >= 0]]
            assert np.array_equal(got, A[64 * I:64 * I + 64, 64 * J:64 * J + 64]), (J, q)


def _emulate_tl_flow(S, b, sched):
    """The dataflow tiled solve (csrc/ba.hip k_tl3_flow) restated in NumPy,
    column by column from the schedule's column table: the diagonal tile's
    updates over rs(J), its factor and inverse, y_J; each row tile's updates
    over its k list (rows 0 and 1: the product slots that the k formed
    themselves, through the product task table) and L_IJ = A_IJ L_JJ^-T; then
    x_J from the rows' x_I."""
    T = int(sched[1])
    fo = int(sched[5])
    rec = sched[fo:fo + 5 * T].reshape(-1, 5)
    n, TB = len(b), 64
    N = T * TB
    A, bb, rn = _tiled_system(S, b, sched)
    t = lambda I: slice(I * TB, (I + 1) * TB)  # noqa: E731
    dinv, y, x = {}, np.zeros(N), np.zeros(N)
    pt = int(sched[10])
    prod, seen = {}, set()
    for J in range(T):
        ro, rc, so, sc, uo = rec[J]
        rs = sched[so:so + sc]
        rows = sched[ro:ro + rc]
        for k in rs:
            A[t(J), t(J)] -= A[t(J), t(k)] @ A[t(J), t(k)].T
        dinv[J] = np.linalg.inv(np.linalg.cholesky(A[t(J), t(J)]))
        r = bb[t(J)] - sum((A[t(J), t(k)] @ y[t(k)] for k in rs), np.zeros(TB))
        y[t(J)] = dinv[J] @ r
        for q, I in enumerate(rows):
            ko, kc = sched[uo + 2 * q], sched[uo + 2 * q + 1]
            if q < 2:
                for k, sl in zip(sched[ko:ko + kc], sched[ko + kc:ko + 2 * kc]):
                    assert k < J and sl in prod  # formed by column k, earlier
                    A[t(I), t(J)] -= prod[sl]
            else:
                assert (sched[ko + kc:ko + 2 * kc] == -1).all()
                for k in sched[ko:ko + kc]:
                    A[t(I), t(J)] -= A[t(I), t(k)] @ A[t(J), t(k)].T
            A[t(I), t(J)] = A[t(I), t(J)] @ dinv[J].T
        # this column's product tasks (a, b, slot), ordered by b: rows[b]'s
        # L times rows[a]'s L^T, with rows[b] among rows[a]'s first two rows
        off, cnt = sched[pt + 2 * J], sched[pt + 2 * J + 1]
        tk = sched[off:off + 3 * cnt].reshape(-1, 3)
        assert (np.diff(tk[:, 1]) >= 0).all()
        for a, b_, sl in tk:
            assert a < b_ < rc and sl not in seen
            seen.add(sl)
            Ja, Ib = rows[a], rows[b_]
            assert Ib in sched[rec[Ja][0]:rec[Ja][0] + min(2, rec[Ja][1])]
            prod[sl] = A[t(Ib), t(J)] @ A[t(Ja), t(J)].T
    assert seen == set(range(int(sched[11])))
    for J in reversed(range(T)):
        ro, rc = rec[J][:2]
        r = y[t(J)].copy()
        for I in sched[ro:ro + rc]:
            assert I > J
            r -= A[t(I), t(J)].T @ x[t(I)]
        x[t(J)] = dinv[J].T @ r
    return x[rn]


@pytest.mark.parametrize("mode", ["cams:5", "cams:7:2", "rows64"])
@pytest.mark.parametrize("C,loop", [(30, False), (64, False), (120, True), (500, True)])
def test_tl_flow_table_solves_the_camera_system(C, loop, mode):
    """Column table of the dataflow tiled solve: every dependency of column J
    is an earlier column (no waits on later workgroups before the back
    substitution), and executing it column by column solves S x = b."""
    from slam355.ba import tl_schedule, upper_blocks
    from slam355.synthetic import ba_problem, ba_problem_loop

    rng = np.random.default_rng(C + 1)
    cams, pts, ci, pi, qs = (ba_problem_loop if loop else ba_problem)(rng, C, 20 * C, 5)
    ub = upper_blocks(C, ci, pi)
    iu, ju = np.triu_indices(C)
    blocks = np.stack([iu[ub], ju[ub]], 1)
    sched = tl_schedule(C, blocks, mode)
    T = int(sched[1])
    rec = sched[sched[5]:sched[5] + 5 * T].reshape(-1, 5)
    for J, (ro, rc, so, sc, uo) in enumerate(rec):
        assert all(I > J for I in sched[ro:ro + rc]) and all(k < J for k in sched[so:so + sc])
    n = 9 * C
    M = np.zeros((n, n))
    for c1, c2 in blocks:
        M[9 * c1:9 * c1 + 9, 9 * c2:9 * c2 + 9] = rng.normal(size=(9, 9))
    S = M + M.T + np.diag(np.abs(M).sum(1) + np.abs(M).sum(0) + 1.0)
    b = rng.normal(size=n)
    x = _emulate_tl_flow(S, b, sched)
    assert np.allclose(x, np.linalg.solve(S, b), rtol=0, atol=1e-10 * np.abs(x).max())


def test_union_plan_falls_back_for_wide_tracks():
    """A point seen by more than MF_CAMS cameras: no camera-union plan (the
    slot linearisation takes such problems)."""
    from slam355 import ba

    cams, pts, ci, pi, qs = make_problem(4, 10, 50, 8)
    assert ba.plan_mfma(10, 50, ci, pi) is None
    cams, pts, ci, pi, qs = make_problem(4, 10, 50, 7)
    assert ba.plan_mfma(10, 50, ci, pi) is not None


@pytest.mark.gpu
@pytest.mark.parametrize("C,P,k", [(10, 5000, 6), (64, 50000, 6)])
def test_gpu_folded_assembly_equals_k_assemble(C, P, k):
    """VERDICT r3 #4 (the fold is measured slower and off by default, but kept
    correct): k_lin_mfma assembles the reduced camera system itself (the last
    supergroup per block sums its partial rows; blocks without partial rows
    zeroed every build) -- the same system as the separate k_assemble launch to
    rounding (the sums run in another fixed order), exact zeros where no camera
    pair shares a point, and repeated builds are bit-identical."""
    import torch
    from slam355 import ba
    from slam355.synthetic import ba_problem, perturb

    rng = np.random.default_rng(3 + C)
    cams, pts, ci, pi, qs = ba_problem(rng, C, P, k)
    c0, p0 = perturb(rng, cams, pts)
    a = ba.BAProblem(c0, p0, ci, pi, qs, fold_assembly=True)
    b = ba.BAProblem(c0, p0, ci, pi, qs)  # the k_assemble launch (default)
    assert a.lin_mode == "mfma" and "asm_tab" in a.t and "asm_tab" not in b.t
    a.t["sys"].fill_(np.nan)  # every entry must be written by the build
    a.build_system()
    b.build_system()
    sa, sb = a.t["sys"].cpu().numpy(), b.t["sys"].cpu().numpy()
    assert np.isfinite(sa).all()
    assert np.array_equal(sa == 0.0, sb == 0.0)
    assert np.allclose(sa, sb, rtol=1e-12, atol=1e-12 * np.abs(sb).max())
    a.build_system()
    torch.cuda.synchronize()
    assert np.array_equal(a.t["sys"].cpu().numpy(), sa)
    for _ in range(3):
        a.iterate(1)
        b.iterate(1)
    sta, stb = a.state(), b.state()
    assert bool(sta["ACCEPTED"]) == bool(stb["ACCEPTED"])
    assert abs(sta["COST"] - stb["COST"]) <= 1e-10 * stb["COST"]


@pytest.mark.gpu
@pytest.mark.parametrize("folds", [(True, True, True), (True, False, True)])
def test_gpu_batch_folded_assembly_equals_k_assemble(folds):
    """the folded assembly through BABatch (bench --fold): one
    multi-problem k_lin_mfma launch (blockIdx.y = problem), per-problem asm_tab
    counters re-armed across graph replays, k_assemble skipped only when every
    problem folds (all folded) or run for the unfolded ones (mixed).  Each
    window's iterates over repeated iterate_graphed replays equal the same
    windows batched with k_assemble (to rounding: the sums run in another
    fixed order), and a second replay set from the restored start repeats the
    first bit for bit (the counters were re-armed)."""
    import torch
    from slam355 import ba
    from slam355.synthetic import ba_problem, perturb

    def windows(fold):
        out = []
        for w, f in enumerate(fold):
            rng = np.random.default_rng(40 + w)
            cams, pts, ci, pi, qs = ba_problem(rng, 10, 1500 + 250 * w, 6)
            c0, p0 = perturb(rng, cams, pts)
            out.append(ba.BAProblem(c0, p0, ci, pi, qs, fold_assembly=f))
        return out

    a, b = windows(folds), windows((False,) * len(folds))
    assert all(("asm_tab" in p.t) == f for p, f in zip(a, folds))
    A, B = ba.BABatch(a), ba.BABatch(b)
    runs = []
    for _ in range(2):
        A.iterate_graphed(4, with_restore=True)
        B.iterate_graphed(4, with_restore=True)
        torch.cuda.synchronize()
        sa, sb = A.states(), B.states()
        for x, y in zip(sa, sb):
            assert bool(x["ACCEPTED"]) == bool(y["ACCEPTED"]) and x["NACCEPT"] == y["NACCEPT"]
            assert abs(x["COST"] - y["COST"]) <= 1e-10 * y["COST"]
        for pa, pb in zip(a, b):
            ca, cb = pa.params()[0], pb.params()[0]
            assert np.allclose(ca, cb, rtol=1e-9, atol=1e-12)
        runs.append([p.params()[0] for p in a])
    for x, y in zip(*runs):
        assert np.array_equal(x, y)


@pytest.mark.gpu
def test_gpu_window_set_equals_separate_problems():
    """BAWindowSet (the tracked leg's batched window build: native plans, one
    staged upload into shared device buffers, one reset launch) gives each
    window the iterates BAProblem gives it alone, bit for bit, and a second
    build into the reused buffers repeats them (a window with 9 cameras per
    point falls back to an ordinary slot-mode BAProblem)."""
    import torch
    from slam355 import ba
    from slam355.synthetic import ba_problem, perturb

    probs = []
    for w, (C, P, k) in enumerate([(8, 800, 3), (9, 600, 4), (8, 1000, 2), (10, 300, 9)]):
        rng = np.random.default_rng(60 + w)
        cams, pts, ci, pi, qs = ba_problem(rng, C, P, k)
        c0, p0 = perturb(rng, cams, pts)
        probs.append((c0, p0, ci, pi, qs))
    s = torch.cuda.Stream()
    ws = ba.BAWindowSet()
    runs, sets = [], []
    for _ in range(2):
        got = ws.build(probs, s)
        sets.append(got)
        assert [p.lin_mode for p in got] == ["mfma", "mfma", "mfma", "slot"]
        with torch.cuda.stream(s):
            ba.BABatch(got[:3], stream=s).iterate(4)
            got[3].iterate(4)
        torch.cuda.synchronize()
        runs.append([p.params() for p in got])
    # double-buffered device memory: the first call's problems are still valid
    # after the second call, and dead (they raise) once a third call reuses them
    assert all(np.array_equal(a[0], b[0]) for a, b in zip(runs[0], [p.params() for p in sets[0]]))
    b0 = ba.BABatch(sets[0][:3], stream=s)
    ws.build(probs, s)
    for bad in (lambda: sets[0][0].params(), lambda: sets[0][1].state(), lambda: b0.iterate(1),
                lambda: ba.BABatch(sets[0][:3], stream=s)):
        with pytest.raises(RuntimeError, match="reused"):
            bad()
    assert sets[0][3].params() is not None  # an ordinary BAProblem owns its buffers
    sets[1][0].params()  # the second call's set is still live
    for w, pr in enumerate(probs):
        ref = ba.BAProblem(*pr)
        ref.iterate(4)
        rc, rp = ref.params()
        for r in runs:
            assert np.array_equal(r[w][0], rc) and np.array_equal(r[w][1], rp), w


def _stage_inputs(specs, n, seed, u_off=0.5, v_off=0.25):
    """Mapper-shaped host arrays (rows [W n, cap, 4] = (frame, point, u, v),
    counts, maps, M, cams) for synthetic windows of n cameras, each window's
    observations dealt over its n pairs in order, and the problems they stand
    for (q = u - u_off: the stager's arithmetic)."""
    from slam355.synthetic import ba_problem, perturb

    wins = []
    for w, (P, k) in enumerate(specs):
        rng = np.random.default_rng(seed + w)
        cams, pts, ci, pi, qs = ba_problem(rng, n, P, k)
        c0, p0 = perturb(rng, cams, pts)
        wins.append((c0, p0, ci, pi, qs))
    W = len(wins)
    cap = max(-(-len(w[2]) // n) for w in wins)
    map_cap = max(len(w[1]) for w in wins)
    rows = np.zeros((W * n, cap, 4))
    cnt = np.zeros(W * n, np.int32)
    maps = np.zeros((W, map_cap, 3))
    M = np.zeros(W, np.int32)
    cams = np.zeros((W * n, 9))
    probs = []
    for w, (c0, p0, ci, pi, qs) in enumerate(wins):
        maps[w, :len(p0)] = p0
        M[w] = len(p0)
        cams[w * n:(w + 1) * n] = c0
        parts = np.array_split(np.arange(len(ci)), n)
        qq = []
        for j, idx in enumerate(parts):
            b = w * n + j
            cnt[b] = len(idx)
            rows[b, :len(idx)] = np.stack([ci[idx], pi[idx], qs[idx, 0] + u_off, qs[idx, 1] + v_off], 1)
            qq.append(np.stack([rows[b, :len(idx), 2] - u_off, rows[b, :len(idx), 3] - v_off], 1))
        probs.append((c0, p0, ci, pi, np.concatenate(qq)))
    return (rows, cnt, maps, M, cams, u_off, v_off), probs


def test_stage_windows_layout_matches_planner():
    """slam_ba_stage_windows (host only, fake device addresses): per window the
    native planner's tables, the float64 data in BAProblem's layout (points
    permuted by the plan, observations in plan order) and descriptor addresses
    at the staged offsets; a window the camera-union plan cannot take (every
    point seen by all 8 cameras) is left to the caller."""
    import ctypes

    from slam355 import _lib, ba

    (rows, cnt, maps, M, cams, uo, vo), probs = _stage_inputs([(800, 3), (300, 8), (1000, 2)], 8, 70)
    W = len(probs)
    meta = np.zeros((W, ba.BAWindowSet.META), np.int64)
    need = np.zeros(2, np.int64)
    args = (W, 8, rows.shape[1], rows.ctypes.data, cnt.ctypes.data, maps.ctypes.data, maps.shape[1],
            M.ctypes.data, cams.ctypes.data, uo, vo)
    _lib.call("slam_ba_stage_windows", *args, None, 0, None, 0, None, None, None, meta.ctypes.data,
              need.ctypes.data)
    assert list(meta[:, 0]) == [1, 0, 1]
    h64 = np.full(int(need[0]), np.nan)
    h32 = np.full(int(need[1]), -7, np.int32)
    d64, d32 = 1 << 40, 1 << 41
    structs = (ba._Prob * W)()
    _lib.call("slam_ba_stage_windows", *args, h64.ctypes.data, len(h64), h32.ctypes.data, len(h32),
              d64, d32, ctypes.addressof(structs), meta.ctypes.data, need.ctypes.data)
    for w in (0, 2):
        c0, p0, ci, pi, qs = probs[w]
        pl = ba.plan_mfma_native(8, len(p0), ci, pi)
        m = meta[w]
        _, _, o64, o32, nb, offs = ba.BAWindowSet._views_of(h64, h32, m)
        assert nb == len(pl["buf"]) and np.array_equal(h32[o32:o32 + nb], pl["buf"])
        assert np.all(h32[o32 + nb:o32 + nb + 8] == 0)
        get = lambda k: h64[o64[k][0]:o64[k][0] + int(np.prod(o64[k][1]))].reshape(o64[k][1])  # noqa: E731
        for k in ("cams0", "cams1", "init_c"):
            assert np.array_equal(get(k), c0)
        for k in ("pts0", "pts1", "init_p"):
            assert np.array_equal(get(k), p0[pl["perm"]])
        assert np.array_equal(get("obs_q"), qs[pl["order"]])
        for k in ba.BAWindowSet._F64[7:]:
            assert np.all(get(k) == 0.0), k
        s = structs[w]
        assert (s.n_cams, s.n_pts, s.n_obs, s.n_sgrps) == (8, len(p0), len(ci), pl["n_sgrps"])
        assert s.cams[1] == d64 + 8 * o64["cams1"][0] and s.state == d64 + 8 * o64["state"][0]
        assert s.obs_meta == d32 + 4 * (o32 + offs["obs_meta"])
        assert s.ticket == d32 + 4 * (o32 + nb + 4)


@pytest.mark.gpu
def test_gpu_window_stage_equals_separate_problems():
    """BAWindowSet.stage (the tracked leg's one-call host staging) gives every
    window the iterates BAProblem gives it alone, bit for bit, twice in a row
    into the reused buffers; the window the camera-union plan cannot take is
    an ordinary (slot-mode) problem."""
    import torch
    from slam355 import ba

    inp, probs = _stage_inputs([(800, 3), (300, 8), (1000, 2)], 8, 80)
    s = torch.cuda.Stream()
    ws = ba.BAWindowSet()
    runs = []
    for _ in range(2):
        got = ws.stage(*inp, stream=s)
        assert [p.lin_mode for p in got] == ["mfma", "slot", "mfma"]
        with torch.cuda.stream(s):
            ba.BABatch([got[0], got[2]], stream=s).iterate(4)
            got[1].iterate(4)
        torch.cuda.synchronize()
        runs.append([p.params() for p in got])
    for w, pr in enumerate(probs):
        ref = ba.BAProblem(*pr)
        ref.iterate(4)
        rc, rp = ref.params()
        for r in runs:
            assert np.array_equal(r[w][0], rc) and np.array_equal(r[w][1], rp), w


def test_assembly_table_counts_every_partial_row():
    """The folded assembly's table (slam355.ba.assembly_table): every cpart row
    is counted once at its camera's diagonal block, every bpart row once at its
    block, blocks without rows are listed empty (C3 window: camera pairs more
    than 5 keyframes apart share no point)."""
    from slam355 import ba

    cams, pts, ci, pi, qs = make_problem(5, 10, 2000, 6)
    pl = ba.plan_mfma(10, len(pts), ci, pi)
    assert pl is not None
    tab = ba.assembly_table(10, pl).astype(np.int64)
    NB = len(pl["blocks"])
    need, cnt = tab[:NB], tab[NB:2 * NB]
    cam_dblk = tab[2 * NB:2 * NB + 10]
    nbs = len(pl["bslot_blk"])
    row_blk = tab[2 * NB + 10:2 * NB + 10 + nbs]
    n_empty = tab[2 * NB + 10 + nbs]
    empty = tab[2 * NB + 11 + nbs:]
    assert not cnt.any() and len(empty) == n_empty
    assert need.sum() == len(pl["cslot_cam"]) + nbs
    blocks = pl["blocks"]
    assert all(blocks[cam_dblk[c], 0] == c == blocks[cam_dblk[c], 1] for c in range(10))
    assert np.array_equal(np.bincount(row_blk, minlength=NB), np.diff(pl["blk_bslot_ptr"]))
    assert set(empty) == set(np.nonzero(need == 0)[0])
    gaps = blocks[empty, 1] - blocks[empty, 0]
    assert (gaps > 5).all() and len(empty) == sum(10 - d for d in range(6, 10))


def _rand_structure(rng, C, P, maxk, dup=0.02, empty=0.02):
    ci, pi = [], []
    for p in range(P):
        if rng.random() < empty:
            continue
        k = min(int(rng.integers(1, maxk + 1)), C)
        cs = rng.choice(C, size=k, replace=False) if rng.random() < 0.5 else \
            (rng.integers(0, C) + np.arange(k)) % C
        for c in cs:
            ci.append(c)
            pi.append(p)
            if rng.random() < dup:  # a point observed twice by one camera
                ci.append(c)
                pi.append(p)
    idx = rng.permutation(len(ci))
    return np.asarray(ci, np.int64)[idx], np.asarray(pi, np.int64)[idx]


def _same_plan(C, P, ci, pi, block_list=None, cpw=None):
    from slam355 import _lib, ba

    a = ba.plan_mfma(C, P, ci, pi, block_list, cpw)
    b = ba.plan_mfma_native(C, P, ci, pi, block_list, cpw)
    assert (a is None) == (b is None)
    if a is None:
        return
    for k in ("n_obs", "n_grps", "n_sgrps", "chunks_per_wg"):
        assert a[k] == b[k], k
    for k in _lib.PLAN_TABLES:
        x, y = np.asarray(a[k], np.int64), np.asarray(b[k], np.int64)
        assert x.shape == y.shape and np.array_equal(x, y), k


@pytest.mark.parametrize("C,P,maxk", [(8, 950, 3), (10, 5000, 6), (20, 3000, 5), (64, 4000, 7),
                                      (3, 10, 2), (1, 5, 1), (70, 2000, 7)])
def test_native_planner_equals_plan_mfma(C, P, maxk):
    """slam_ba_plan_mfma (C++) gives plan_mfma's tables element for element:
    tracked-, C3- and packed-size structures, repeated (point, camera) pairs,
    unobserved points, every chunks_per_wg rule."""
    rng = np.random.default_rng(C * 1000 + P)
    for cpw in (None, 1, 3, 8):
        ci, pi = _rand_structure(rng, C, P, maxk)
        _same_plan(C, P, ci, pi, None, cpw)


def test_native_planner_block_list_and_edges():
    from slam355 import _lib, ba

    rng = np.random.default_rng(5)
    C = 20
    ci, pi = _rand_structure(rng, C, 2000, 4)
    bl = np.concatenate([ba.upper_blocks(C, ci, pi), [ba.block_index(0, C - 1, C)]])
    _same_plan(C, 2000, ci, pi, bl)
    with pytest.raises(_lib.SlamError, match="block_list misses"):
        ba.plan_mfma_native(C, 2000, ci, pi, ba.upper_blocks(C, ci, pi)[:C])
    # an explicitly empty block_list is "given" (ADVICE r4): both planners refuse it
    with pytest.raises(ValueError, match="block_list misses"):
        ba.plan_mfma(C, 2000, ci, pi, [])
    with pytest.raises(_lib.SlamError, match="block_list misses"):
        ba.plan_mfma_native(C, 2000, ci, pi, [])
    _same_plan(8, 300, *_rand_structure(rng, 8, 300, 3), block_list=[])  # dense: list unused
    _same_plan(10, 1, np.arange(8), np.zeros(8, np.int64))  # 8 cameras on a point: slot mode
    assert ba.plan_mfma_native(10, 1, np.arange(8), np.zeros(8, np.int64)) is None
    _same_plan(5, 0, np.zeros(0, np.int64), np.zeros(0, np.int64))
    _same_plan(5, 3, np.zeros(0, np.int64), np.zeros(0, np.int64))
    with pytest.raises(_lib.SlamError, match="out of range"):
        ba.plan_mfma_native(5, 3, np.array([5]), np.array([0]))

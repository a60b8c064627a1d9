"""Multi-rank local BA: landmark sharding + summed reduced camera systems.

CPU (gloo, world_size 2): the oracle's partial Schur systems of the two
landmark shards, all-reduced, equal the single-process system.
GPU (gloo on one device, world_size 2): BAProblem.step_distributed on two
shards follows the single-process GPU LM iterates.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(C=8, P=600, k=4, loop=False):
    from slam355.synthetic import ba_problem, ba_problem_loop, perturb

    rng = np.random.default_rng(21)
    cams, pts, ci, pi, qs = (ba_problem_loop if loop else ba_problem)(rng, C, P, k)
    c0, p0 = perturb(rng, cams, pts)
    return c0, p0, ci, pi, qs


def _partial_system(c0, p0, ci, pi, qs, lam):
    """Camera-block system of one shard: S (without camera damping), b, g, diagU."""
    from oracle import ba as oba

    C, P = len(c0), len(p0)
    r, J = oba.residual_and_jacobian(c0, p0, ci, pi, qs)
    Jc, Jp = J[:, :, :9], J[:, :, 9:]
    U = np.zeros((C, 9, 9))
    np.add.at(U, ci, np.einsum("oai,oaj->oij", Jc, Jc))
    V = np.zeros((P, 3, 3))
    np.add.at(V, pi, np.einsum("oai,oaj->oij", Jp, Jp))
    gc = np.zeros((C, 9))
    np.add.at(gc, ci, -np.einsum("oai,oa->oi", Jc, r))
    gp = np.zeros((P, 3))
    np.add.at(gp, pi, -np.einsum("oai,oa->oi", Jp, r))
    Dp = np.clip(np.diagonal(V, axis1=1, axis2=2), 1e-6, 1e32)
    Vi = np.linalg.inv(V + lam * Dp[:, :, None] * np.eye(3)[None])
    W = np.einsum("oai,oaj->oij", Jc, Jp)
    Y = np.einsum("oij,ojk->oik", W, Vi[pi])
    S = np.zeros((C, C, 9, 9))
    o1, o2 = oba._obs_pairs(ci, pi)
    np.add.at(S, (ci[o1], ci[o2]), -np.einsum("oik,ojk->oij", Y[o1], W[o2]))
    S = S + np.transpose(S, (1, 0, 3, 2)) * (1 - np.eye(C))[:, :, None, None]
    S[np.arange(C), np.arange(C)] += U
    b = gc.copy()
    np.add.at(b, ci, -np.einsum("oij,oj->oi", Y, gp[pi]))
    return np.concatenate([S.transpose(0, 2, 1, 3).ravel(), b.ravel(), gc.ravel(),
                           np.diagonal(U, axis1=1, axis2=2).ravel()])


def _cpu_worker(rank, world, port, out):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "slam-1_amd")]
    import torch
    import torch.distributed as dist
    from slam355.dist import shard_by_anchor

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    c0, p0, ci, pi, qs = _problem()
    mine, keep, lpi = shard_by_anchor(len(c0), len(p0), ci, pi, rank, world)
    sysv = torch.from_numpy(_partial_system(c0, p0[mine], ci[keep], lpi, qs[keep], 1e-3))
    dist.all_reduce(sysv)
    if rank == 0:
        np.save(out, sysv.numpy())
    dist.destroy_process_group()


def test_gloo_sharded_system_equals_full(tmp_path):
    c0, p0, ci, pi, qs = _problem()
    full = _partial_system(c0, p0, ci, pi, qs, 1e-3)
    out = str(tmp_path / "sys.npy")
    mp.spawn(_cpu_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    assert np.allclose(got, full, rtol=1e-9, atol=1e-9 * np.abs(full).max())


def test_shards_partition_points_and_observations():
    from slam355.dist import shard_by_anchor

    c0, p0, ci, pi, qs = _problem()
    masks = [shard_by_anchor(len(c0), len(p0), ci, pi, r, 3) for r in range(3)]
    assert (sum(m[0].astype(int) for m in masks) == 1).all()
    assert (sum(m[1].astype(int) for m in masks) == 1).all()


def test_shards_balance_estimated_cost_on_a_loop():
    """Landmark shards of a closed loop (its loop-closure points anchored at
    keyframe 0 share their camera-union supergroups with few others): the
    cost-balanced cuts give every rank the same estimated cost (point_costs,
    within one point's), where equal point counts leave rank 0 heavier; both
    partition the points, and every rank computes the same cuts."""
    from slam355.dist import point_costs, shard_by_anchor
    from slam355.synthetic import ba_problem_loop

    rng = np.random.default_rng(3)
    C, P, W = 120, 24000, 4
    _, _, ci, pi, _ = ba_problem_loop(rng, C, P, 6)
    w = point_costs(C, P, ci, pi, W)
    for balance in (True, False):
        masks = [shard_by_anchor(C, P, ci, pi, r, W, balance=balance)[0] for r in range(W)]
        assert (sum(m.astype(int) for m in masks) == 1).all()
        cost = np.array([w[m].sum() for m in masks])
        if balance:
            assert cost.max() - cost.min() <= 2 * w.max()
        else:
            assert cost[0] > 1.05 * cost[1:].max()
    again = shard_by_anchor(C, P, ci, pi, 1, W)[0]
    assert np.array_equal(again, shard_by_anchor(C, P, ci, pi, 1, W)[0])


def _gpu_worker(rank, world, port, out, C=8, P=600, k=4, iters=6, loop=False):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "slam-1_amd")]
    import torch
    import torch.distributed as dist
    from slam355.ba import BAProblem, upper_blocks
    from slam355.dist import shard_by_anchor

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    c0, p0, ci, pi, qs = _problem(C, P, k, loop)
    mine, keep, lpi = shard_by_anchor(len(c0), len(p0), ci, pi, rank, world)
    # packed layout (9C > 120): every rank lists the blocks of the GLOBAL problem
    prob = BAProblem(c0, p0[mine], ci[keep], lpi, qs[keep], block_list=upper_blocks(C, ci, pi))
    costs = []
    for _ in range(iters):
        prob.step_distributed()
        costs.append(prob.state()["COST_NEW"])
    cams, _ = prob.params()
    if rank == 0:
        np.savez(out, costs=np.array(costs), cams=cams)
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("C,P,k,iters,loop", [(8, 600, 4, 6, False), (30, 1500, 4, 6, False),
                                              (64, 50000, 6, 2, False),
                                              (500, 200000, 6, 1, True)])
def test_gpu_step_distributed_matches_single_rank(tmp_path, C, P, k, iters, loop):
    """C = 8: dense system, one-workgroup solver; C = 30: packed block layout
    (only camera pairs with common points are all-reduced) and tiled solver;
    C = 64, 50k points, 300k observations: the C4 window split
    over two ranks, two LM iterations; C = 500, 200k points, 1.2M observations
    on a closed loop: the C5 global BA (BASELINE config 5) split over two
    ranks, the first LM iteration."""
    from slam355.ba import BAProblem

    c0, p0, ci, pi, qs = _problem(C, P, k, loop)
    prob = BAProblem(c0, p0, ci, pi, qs)
    costs = []
    for _ in range(iters):
        prob.iterate(1)
        costs.append(prob.state()["COST_NEW"])
    cams, _ = prob.params()
    out = str(tmp_path / "d.npz")
    del prob
    mp.spawn(_gpu_worker, args=(2, _free_port(), out, C, P, k, iters, loop), nprocs=2, join=True)
    d = np.load(out)
    assert np.allclose(d["costs"], costs, rtol=1e-8)
    assert np.allclose(d["cams"], cams, rtol=1e-6, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("r", [0, 5])
def test_gpu_shard_active_block_assembly_equals_full_launch(r):
    """A landmark shard's system (rank r of 8 of a 120-keyframe loop) assembled
    over its blocks with partial rows only (asm_act; those workgroups also write
    the other blocks' zeros) equals the
    assembly over every listed block: the same values, the blocks without rows
    -0.0 bit for bit (the diagonal of a camera the shard does not observe may
    differ in the sign of its zero), and the LM iterates on it bit for bit."""
    import torch
    from slam355.ba import BAProblem, upper_blocks
    from slam355.dist import shard_by_anchor

    C, P = 120, 24000
    c0, p0, ci, pi, qs = _problem(C, P, 6, True)
    mine, keep, lpi = shard_by_anchor(C, P, ci, pi, r, 8)
    blocks = upper_blocks(C, ci, pi)
    args = (c0, p0[mine], ci[keep], lpi, qs[keep])
    act = BAProblem(*args, block_list=blocks)
    full = BAProblem(*args, block_list=blocks, active_blocks=False)
    assert act._s.asm_act != 0 and 0 < act._s.n_asm_act < act._s.n_blocks and full._s.asm_act is None
    for pr in (act, full):
        pr.build_system()
    torch.cuda.synchronize()
    a, f = act.t["sys"].cpu().numpy(), full.t["sys"].cpu().numpy()
    assert np.array_equal(a, f)  # (+0 == -0)
    nb = act._s.n_blocks
    blk = np.asarray(act.plan["blocks"]).reshape(-1, 2)
    listed = np.zeros(nb, bool)
    listed[act.t["asm_act"].cpu().numpy()[:act._s.n_asm_act]] = True
    off = ~listed & (blk[:, 0] != blk[:, 1])
    sa, sf = a[:81 * nb].reshape(nb, 81), f[:81 * nb].reshape(nb, 81)
    assert np.array_equal(sa[off].view(np.uint64), sf[off].view(np.uint64))
    assert (sa[off].view(np.uint64) == np.uint64(1 << 63)).all()  # -0.0
    for pr in (act, full):
        pr.iterate(2)
    assert act.state() == full.state()
    for x, y in zip(act.params(), full.params()):
        assert np.array_equal(x, y)


# ---------------------------------------------------------------- pose chain of frame-pair shards
def _pose_results(n, seed=5):
    """PnP results of n frame pairs: small motions, a few stale (-1) pairs."""
    rng = np.random.default_rng(seed)
    rv = rng.normal(0, 0.02, (n, 3))
    tv = np.column_stack([rng.normal(0, 0.05, n), rng.normal(0, 0.05, n), rng.uniform(0.8, 1.2, n)])
    ni = rng.integers(5, 200, n)
    ni[[3, 5, 6]] = -1  # stale pairs, one of them the first pair of shard 1 (B = 5)
    return rv, tv, ni


def _chain_worker(rank, world, port, out, B, cuda):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "slam-1_amd")]
    import torch
    import torch.distributed as dist
    from slam355.dist import gather_pose_chain

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    rv, tv, ni = _pose_results(world * B)
    sl = slice(rank * B, (rank + 1) * B)
    dev = "cuda" if cuda else "cpu"
    if cuda:
        torch.cuda.set_device(0)
    pose0 = np.diag([1.0, 1.0, 1.0, 1.0])
    pose0[:3, 3] = [0.5, -0.2, 3.0]
    poses = gather_pose_chain(torch.tensor(rv[sl], device=dev), torch.tensor(tv[sl], device=dev),
                              torch.tensor(ni[sl], dtype=torch.int32, device=dev), pose0=pose0)
    if rank == 0:
        np.save(out, poses.cpu().numpy())
    dist.destroy_process_group()


def test_gloo_gather_pose_chain_equals_one_chain(tmp_path):
    """frame-pair shards + one gather of (rvec, tvec, n_inliers)
    give the trajectory of one chain over all pairs, stale-T rule across the
    shard boundary included (main.py:94-98, 120-124)."""
    from slam355.pipeline import chain_poses

    B, world = 5, 2
    out = str(tmp_path / "poses.npy")
    mp.spawn(_chain_worker, args=(world, _free_port(), out, B, False), nprocs=world, join=True)
    rv, tv, ni = _pose_results(world * B)
    pose0 = np.diag([1.0, 1.0, 1.0, 1.0])
    pose0[:3, 3] = [0.5, -0.2, 3.0]
    want, _ = chain_poses(pose0, rv, tv, ni)
    assert np.array_equal(np.load(out), want)


@pytest.mark.gpu
def test_gpu_gather_pose_chain_equals_device_chain(tmp_path):
    """The same on the device (k_pose_chain over the gathered results) against
    one device chain over all pairs: bit-identical."""
    import torch
    from slam355 import _lib
    from slam355.device import ptr, stream_ptr

    B, world = 5, 2
    out = str(tmp_path / "poses.npy")
    mp.spawn(_chain_worker, args=(world, _free_port(), out, B, True), nprocs=world, join=True)
    rv, tv, ni = _pose_results(world * B)
    pose0 = np.diag([1.0, 1.0, 1.0, 1.0])
    pose0[:3, 3] = [0.5, -0.2, 3.0]
    n = world * B
    d = "cuda"
    trv, ttv = torch.tensor(rv, device=d), torch.tensor(tv, device=d)
    tni = torch.tensor(ni, dtype=torch.int32, device=d)
    state = torch.tensor(np.concatenate([pose0, np.eye(4)]).ravel(), device=d)
    poses = torch.empty((n, 4, 4), dtype=torch.float64, device=d)
    _lib.call("slam_pose_chain", ptr(trv), ptr(ttv), ptr(tni), n, ptr(state), ptr(poses),
              stream_ptr(None))
    assert np.array_equal(np.load(out), poses.cpu().numpy())


# ---------------------------------------------------------------- one sequence over tracking shards
def _track_shard_worker(rank, world, port, out, B, steps):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "slam-1_amd")]
    import torch
    import torch.distributed as dist
    from slam355.dist import GlobalChain
    from slam355.pipeline import Tracker
    from slam355.synthetic import corridor_sequence

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    n = steps * world * B + 1
    f0s = [(s * world + rank) * B for s in range(steps)]
    ids = [f0 + i for f0 in f0s for i in range(B + 1)]
    L, R, _, rig = corridor_sequence(n, 1280, 720, seed=77, device="cuda", as_numpy=False, frames=ids)
    trk = Tracker(B, 720, 1280, rig.P_l, rig.P_r, max_kp_per_tile=64, seed=0)
    gc = GlobalChain(B, world, torch.device("cuda", 0))
    gc.reset()
    chains = []
    for s in range(steps):
        o = s * (B + 1)
        imgs = torch.cat([L[o:o + B + 1], R[o:o + B]]).contiguous()
        trk.track(f0s[s], imgs=imgs, chain=False)
        chains.append(gc.step(trk.rvec, trk.tvec, trk.p_ninl).clone())
    torch.cuda.synchronize()
    if rank == 0:
        np.save(out, torch.cat(chains).cpu().numpy())
    dist.destroy_process_group()


@pytest.mark.gpu
def test_gpu_tracking_shards_gather_one_trajectory(tmp_path):
    """`--gpus N` tracking shards ONE sequence -- rank r tracks
    pairs r*B.. of every global step, GlobalChain all-gathers the PnP results
    and chains them on every rank each step.  Two ranks of B = 3 pairs (gloo on
    one GPU) over two global steps give, bit for bit, the trajectory of one
    Tracker of B = 6 pairs over the same frames (main.py:79-98, 120-124)."""
    import torch
    from slam355.pipeline import Tracker
    from slam355.synthetic import corridor_sequence

    B, world, steps = 3, 2, 2
    out = str(tmp_path / "chain.npy")
    mp.spawn(_track_shard_worker, args=(world, _free_port(), out, B, steps), nprocs=world, join=True)
    got = np.load(out)
    G = world * B
    n = steps * G + 1
    ids = [s * G + i for s in range(steps) for i in range(G + 1)]
    L, R, poses, rig = corridor_sequence(n, 1280, 720, seed=77, device="cuda", as_numpy=False,
                                         frames=ids)
    trk = Tracker(G, 720, 1280, rig.P_l, rig.P_r, max_kp_per_tile=64, seed=0)
    want = []
    for s in range(steps):
        o = s * (G + 1)
        trk.track(s * G, imgs=torch.cat([L[o:o + G + 1], R[o:o + G]]).contiguous())
        want.append(trk.poses.clone())
    want = torch.cat(want).cpu().numpy()
    assert np.array_equal(got, want)
    gt = np.stack([np.linalg.inv(poses[0]) @ poses[i + 1] for i in range(steps * G)])
    assert np.abs(want[:, :3, 3] - gt[:, :3, 3]).max() < 0.5


# ---------------------------------------------------------------- C-ABI communicator (RCCL)
def _rccl_loadable() -> bool:
    """A library slam_comm_* would dlopen (comm.hip: SLAM_RCCL_LIB, then
    librccl.so.1, then librccl.so)."""
    import ctypes

    for name in (os.environ.get("SLAM_RCCL_LIB"), "librccl.so.1", "librccl.so"):
        if not name:
            continue
        try:
            ctypes.CDLL(name)
            return True
        except OSError:
            pass
    return False


def test_comm_unique_id_loads_rccl_lazily():
    """slam_comm_unique_id resolves RCCL at run time (dlopen; no GPU needed for
    the id) and fills SLAM_COMM_ID_BYTES bytes.  Skipped where RCCL itself
    cannot be loaded (a CPU-only host without ROCm's RCCL).  Multi-rank parity
    of the C-ABI path (slam_ba_step_distributed on > 1 rank) stays unverified
    until a multi-GPU node runs it: RCCL refuses two ranks per device."""
    import ctypes

    from slam355 import _lib

    if not _rccl_loadable():
        pytest.skip("RCCL (librccl.so.1 / SLAM_RCCL_LIB) cannot be loaded here")

    b = (ctypes.c_uint8 * 128)()
    _lib.call("slam_comm_unique_id", ctypes.cast(b, ctypes.c_void_p))
    assert any(bytes(b))
    with pytest.raises(_lib.SlamError):  # argument checks before any RCCL call
        _lib.call("slam_comm_init", 2, 5, ctypes.cast(b, ctypes.c_void_p),
                  ctypes.byref(ctypes.c_void_p()))


@pytest.mark.gpu
@pytest.mark.parametrize("C,P,k", [(8, 600, 4), (30, 1500, 4)])
def test_gpu_capi_comm_step_distributed_single_rank_equals_iterate(C, P, k):
    """slam_ba_step_distributed (build, RCCL all-reduce of prob->sys, solve,
    all-reduce of prob->small, decide: one C call) on a one-rank RCCL
    communicator gives the single-process iterates bit for bit (dense and
    packed / tiled systems)."""
    from slam355.ba import BAProblem
    from slam355.dist import CapiComm

    c0, p0, ci, pi, qs = _problem(C, P, k)
    a, b = BAProblem(c0, p0, ci, pi, qs), BAProblem(c0, p0, ci, pi, qs)
    comm = CapiComm(single=True)
    try:
        for _ in range(4):
            a.iterate(1)
            b.step_distributed(comm=comm)
            sa, sb = a.state(), b.state()
            assert sa["COST_NEW"] == sb["COST_NEW"] and sa["LAMBDA"] == sb["LAMBDA"]
        assert np.array_equal(a.params()[0], b.params()[0])
    finally:
        comm.close()

"""slam355 benchmark — the driver contract.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload tracking|ba|matcher]

Default workload ("tracking", BASELINE.json metric "frames/sec tracking+local-BA
@1280x720"): one step = B synthetic 1280x720 stereo frame pairs, resident in
HBM before the timed region (the PCIe-inclusive rate, frames streamed from
pinned host memory, is reported beside it), through the whole tracking hot
path (ORB on 2B+1 images with 64 kp/tile ~ 2075 kp/frame, on its own CU-masked
stream pipelined against the previous batch's tail; stereo kNN-2 + ratio,
F-LMedS, triangulation, temporal kNN-2 + gate, PnP-RANSAC, device pose chain)
plus the local bundle adjustment it schedules: every `ba_every` frames one LM
solve of `ba_iters` iterations over a C3-shaped window (10 keyframes x 5k
points x 30k observations), the step's windows batched.  N > 1: one process per GPU,
each with its own frame shard and its own BA windows (weak scaling; no
collective on this path).  `--workload ba` measures local-BA LM iterations/s:
C3 on one GPU, or C4 (64 KF x 50k points) sharded by landmark over the ranks
with one RCCL all-reduce of the reduced camera system per iteration.

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "slam-1_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

# slam355 (libslam355.so) is imported inside the workloads only: with --gpus N > 1
# and no WORLD_SIZE in the environment, main() starts the N ranks as a child
# process before anything here touches HIP (launch_ranks)

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
HBM_PEAK_GBS = 8000.0
F64_PEAK_TFLOPS = 78.6        # FP64 vector == FP64 matrix on gfx950 (spec)
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 78.6 T lane-ops/s (4 x SIMD32 per CU)
MATCH_OPS_PER_PAIR = 19       # 8 v_xor + 8 v_bcnt(+acc) + v_lshl_or + v_min + v_med3 (VALU kernel)
FP4_PEAK_TFLOPS = 10000.0     # FP4 MFMA dense ~10 PF (MI355X_MICROARCH.md chip-level table)
MX_FLOPS_PER_PAIR = 2 * 256   # the fp4 matrix-core matcher: 256 MACs per descriptor pair
ORB_OUT_BYTES = 56            # per keypoint: 5 f32 + octave i32 + 32 B descriptor
W_IMG, H_IMG = 1280, 720


# ---------------------------------------------------------------------------- plumbing
def dist_init():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        # SLAM_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks
        # on one GPU (RCCL refuses two ranks per device); the driver uses nccl = RCCL
        backend = os.environ.get("SLAM_DIST_BACKEND", "nccl")
        dev = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return world, rank


def launch_ranks(n):
    """`bench.py --gpus N` without a launcher: run N ranks of this same command
    under torch.distributed.run as a CHILD process (this process has not touched
    HIP and never execs), rendezvous on 127.0.0.1; rank 0's JSON line reaches
    stdout through the child's inherited stdout.  Returns the child's exit code."""
    import socket
    import subprocess

    with socket.socket() as s:  # a free rendezvous port
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=dict(os.environ, OMP_NUM_THREADS=os.environ.get(
        "OMP_NUM_THREADS", "1"))).returncode


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def reduce_scalar(x: float, world: int, op="max") -> float:
    if world == 1:
        return x
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def timed_loop(step, steps, warmup, world, marks_every=True, dict_marks=False):
    """W untimed steps, then exactly K timed steps between barrier+synchronize
    fences; per-step stage events are recorded on the launch stream."""
    for _ in range(warmup):
        step(None)
    torch.cuda.synchronize()
    all_marks = []
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step_s = []
    for _ in range(steps):
        ts = time.perf_counter()
        marks = ({} if dict_marks else []) if marks_every else None
        step(marks)
        if marks is not None:
            all_marks.append(marks)
        step_s.append(time.perf_counter() - ts)
    # host time to issue the K steps (no synchronisation inside the loop): when
    # it approaches dt, the launches, not the GPU, set the pace
    timed_loop.host_s = time.perf_counter() - t0
    timed_loop.step_s = step_s
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    stages = {}
    for marks in all_marks:
        # a list of (name, event) on one stream, or {lane: list} for several streams
        lanes = marks.values() if isinstance(marks, dict) else [marks]
        for lane in lanes:
            for (n0, e0), (n1, e1) in zip(lane[:-1], lane[1:]):
                stages.setdefault(n1, []).append(e0.elapsed_time(e1))
    return reduce_scalar(dt, world, "max"), {k: float(np.mean(v)) for k, v in stages.items()}


def ba_flops_per_iter(C, P, O, n_per_pt):
    """O(4c^2+16c+48) + sum_p 2(3c^2 n_p^2 + 9c n_p) + (cC)^3/3, c = 9."""
    c = 9
    return O * (4 * c * c + 16 * c + 48) + P * 2 * (3 * c * c * n_per_pt ** 2 + 9 * c * n_per_pt) \
        + (c * C) ** 3 / 3


# ---------------------------------------------------------------------------- tracking
def pmc_traffic(name="pmc_traffic.json"):
    """Per-kernel HBM bytes per dispatch from a committed PMC summary
    profiles/<name> (scripts/pmc_traffic.sh: FETCH_SIZE x2 + WRITE_SIZE in
    separate rocprofv3 --pmc passes of this bench), or None."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    d = json.load(open(path))
    d["path"] = os.path.relpath(path, ROOT)
    return d


def pmc_valu(kernel, name="pmc_sq.json"):
    """(SQ_INSTS_VALU per dispatch of `kernel`, source path) from the committed
    SQ counter summary profiles/<name> (scripts/gpu_profile.sh), or None."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    k = json.load(open(path)).get("kernels", {}).get(kernel)
    if not k or "SQ_INSTS_VALU" not in k:
        return None
    return float(k["SQ_INSTS_VALU"]), os.path.relpath(path, ROOT)


def pmc_bytes(pmc, kernels):
    if pmc is None or not all(k in pmc["kernels"] for k in kernels):
        return None
    return float(sum(pmc["kernels"][k]["hbm_bytes"] for k in kernels))


def masked_stream(n_cus, first=0):
    """A HIP stream whose kernels may use only CUs [first, first + n_cus)
    (hipExtStreamCreateWithCUMask), wrapped as a torch stream: `--track-cus`
    keeps the rest of the CUs free of tracking work for the local-BA stream;
    `--ba-cus` gives the two streams disjoint CU sets."""
    import ctypes

    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"),
                      mode=ctypes.RTLD_GLOBAL)
    n_total = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    words = (n_total + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for i in range(first, min(first + n_cus, n_total)):
        mask[i // 32] |= 1 << (i % 32)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), words, mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed ({rc})")
    st = torch.cuda.ExternalStream(h.value)
    # torch does not own the stream: destroy it before the runtime tears down
    st.destroy = lambda: (torch.cuda.synchronize(), hip.hipStreamDestroy(h))
    return st


class FrameFeed:
    """The synthetic stereo sequence, pre-packed per tracking batch as
    [left_0..left_B, right_0..right_{B-1}] (2B+1 images per step).

    resident=True (the headline, the contract's "inputs already resident in
    HBM"): every batch lives in HBM before the timed region; step k reads
    batch k mod n_windows in place.
    resident=False (`pcie_inclusive` beside the headline): the sequence lives in
    pinned host memory and step k's batch is uploaded on a copy stream into one
    of two device slots while step k-1 is tracked (double buffering: the copy
    into a slot waits until the tracking that read it has finished)."""

    def __init__(self, L, R, B, n_windows, resident=True):
        self.B, self.n_windows, self.resident = B, n_windows, resident
        H, W = L.shape[1:]
        packs = torch.empty((n_windows, 2 * B + 1, H, W), dtype=torch.uint8,
                            device="cuda" if resident else "cpu")
        if not resident:
            packs = packs.pin_memory()
        for w in range(n_windows):  # L, R: window w's B + 1 frames at rows w * (B + 1) ..
            f0 = w * (B + 1)
            packs[w, :B + 1] = L[f0:f0 + B + 1].to(packs.device)
            packs[w, B + 1:] = R[f0:f0 + B].to(packs.device)
        self.packs = packs
        self.k = 0
        if resident:
            return
        self.slots = [torch.empty((2 * B + 1, H, W), dtype=torch.uint8, device="cuda")
                      for _ in range(2)]
        self.copy_stream = torch.cuda.Stream()
        self.ready = [torch.cuda.Event() for _ in range(2)]
        self.free = [torch.cuda.Event() for _ in range(2)]

    def upload(self, k):
        slot = k % 2
        cs = self.copy_stream
        cs.wait_event(self.free[slot])
        with torch.cuda.stream(cs):
            self.slots[slot].copy_(self.packs[k % self.n_windows], non_blocking=True)
        self.ready[slot].record(cs)

    def prime(self):
        self.k = 0
        if self.resident:
            return
        for e in self.free:
            e.record(torch.cuda.current_stream())
        self.upload(0)

    def next(self, stream):
        """-> (images of step k, window index).  Streamed: issues the upload of
        step k+1 and makes `stream` wait for step k's upload.  Call
        release(stream) after the launches that read the images."""
        k = self.k
        if self.resident:
            return self.packs[k % self.n_windows], k % self.n_windows
        self.upload(k + 1)
        stream.wait_event(self.ready[k % 2])
        return self.slots[k % 2], k % self.n_windows

    def release(self, stream):
        if not self.resident:
            self.free[self.k % 2].record(stream)
        self.k += 1


def matcher_roofline(pairs, ms, t_cap, where, force_valu=False):
    """Roofline of one kNN-2 launch: the fp4 matrix-core kernel (t_cap <= 16383)
    against the FP4 MFMA dense peak (256 MACs per pair), the integer-VALU kernel
    against the VALU peak (19 ops per pair); both fractions reported."""
    mx = t_cap <= 16383 and not force_valu
    valu_tops = pairs * MATCH_OPS_PER_PAIR / (ms * 1e-3) / 1e12
    if mx:
        r = {"bound": "mfma", "achieved": pairs * MX_FLOPS_PER_PAIR / (ms * 1e-3) / 1e12,
             "peak": FP4_PEAK_TFLOPS, "unit": "TFLOP/s (fp4)", "kernel": f"knn2_mx_kernel ({where})",
             "flops_per_pair": MX_FLOPS_PER_PAIR}
    else:
        r = {"bound": "valu", "achieved": valu_tops, "peak": VALU_PEAK_TOPS, "unit": "Tops/s",
             "kernel": f"knn2_kernel ({where})", "ops_per_pair": MATCH_OPS_PER_PAIR}
    r.update(ms_per_launch=ms, pairs_per_launch=pairs, gpairs_per_s=pairs / (ms * 1e-3) / 1e9,
             valu_equivalent_frac=valu_tops / VALU_PEAK_TOPS)
    return r


def run_tracking(args, world, rank):
    from slam355.ba import BABatch, BAProblem
    from slam355.pipeline import Tracker
    from slam355.synthetic import ba_problem, corridor_sequence, perturb

    B = args.batch
    n_win = args.windows
    # ONE sequence over all ranks: n_win global steps of world * B consecutive
    # frame pairs; rank r tracks pairs r*B .. r*B + B - 1 of every global step
    # (frame-pair shards, main.py:79-97), so its window w starts at frame
    # (w * world + r) * B.  Each rank renders only its own frames on the GPU
    # (untimed; per-frame seeded noise, so the images do not depend on the world
    # size) and keeps them resident in HBM.
    f0s = [(w * world + rank) * B for w in range(n_win)]
    ids = [f0 + i for f0 in f0s for i in range(B + 1)]
    L, R, poses, rig = corridor_sequence(n_win * world * B + 1, W_IMG, H_IMG, seed=1000,
                                         device="cuda", as_numpy=False, frames=ids)
    feed = FrameFeed(L, R, B, n_win, resident=True)
    # the PCIe-inclusive variant (reported beside `value`, never as it): the same
    # sequence streamed from pinned host memory inside its own timed region
    feed_h2d = None if args.no_pcie_leg else FrameFeed(L, R, B, n_win, resident=False)
    feeds = [feed]
    CPU_PAIRS = 16  # cpu_baseline sample: 16 frame pairs + 16 LM iterations (~10 s of host work)
    L_np, R_np = L[:CPU_PAIRS + 1].cpu().numpy(), R[:CPU_PAIRS].cpu().numpy()
    del L, R
    # the global trajectory of the shards (world > 1): one all-gather of the
    # step's PnP results + the device pose chain over all world * B pairs, every
    # step, inside the timed region (slam355.dist.GlobalChain)
    gchain = None
    if world > 1:
        from slam355.dist import GlobalChain

        gchain = GlobalChain(B, world, torch.device("cuda", torch.cuda.current_device()))
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    if args.ba_cus:  # disjoint CU sets: tracking on [0, n - ba_cus), local BA on the rest
        args.track_cus = n_cu - args.ba_cus
    trk_stream = masked_stream(args.track_cus) if args.track_cus else None
    if trk_stream is None and args.priority == "track":
        trk_stream = torch.cuda.Stream(priority=-1)
        trk_stream.destroy = lambda: None
    orb_stream = None
    if args.orb_pipeline and trk_stream is None:
        # tracking on an explicit stream: a CU-masked stream is a blocking stream,
        # which would serialise with work on the legacy null stream
        trk_stream = torch.cuda.Stream()
        trk_stream.destroy = lambda: None
    if args.orb_pipeline:  # ORB of batch k+1 overlaps the matching / PnP tail of batch k
        if args.orb_cus:  # ORB kept off the last CUs (left to the latency-bound BA kernels)
            orb_stream = masked_stream(args.orb_cus)
        else:
            orb_stream = torch.cuda.Stream(priority=-1 if args.priority == "track" else 0)
    if args.solve_lds_floor:
        from slam355 import _lib as slib

        slib.call("slam_ba_set_solve_lds_floor", int(args.solve_lds_floor))
    if args.orb_lds_floor:
        from slam355 import _lib as slib

        slib.call("slam_orb_set_lds_floor", int(args.orb_lds_floor))
    if args.valu:  # the integer-VALU kNN-2 kernel in the pipeline (A/B)
        from slam355 import _lib as slib

        slib.lib.slam_hamming_force_valu(1)
    # the same RANSAC seed on every rank: each pair's draws follow its global
    # frame index (item0), so a pair tracks alike whichever rank holds it
    trk = Tracker(B, H_IMG, W_IMG, rig.P_l, rig.P_r, max_kp_per_tile=args.kp_per_tile, seed=0,
                  stream=trk_stream, orb_stream=orb_stream)
    rng = np.random.default_rng(2000 + rank)
    C3 = (10, 5000, 6)
    n_solves = max(1, B // args.ba_every)
    # --ba-group G: the windows of G consecutive steps advance as one launch set
    # (local mapping lags tracking by < G steps).  Pending windows are flushed at
    # the end of the warmup and of the timed region as a whole set, so the timed
    # region holds at least its K steps' windows x iterations.
    G = max(1, args.ba_group)
    assert G == 1 or args.ba_streams == 1, "--ba-group > 1 needs --ba-streams 1"
    n_launch = n_solves * G
    windows = []
    for _ in range(n_launch):  # one C3 window per `ba_every` frames, each its own problem
        cams, pts, ci, pi, qs = ba_problem(rng, *C3)
        c0, p0 = perturb(rng, cams, pts)
        windows.append((c0, p0, ci, pi, qs))
    stream = torch.cuda.current_stream()
    # local mapping (BA) on its own HIP stream, concurrent with tracking, unless --ba-serial
    # (high priority: its short latency-bound kernels go ahead of queued ORB tiles)
    if args.ba_cus and not args.ba_serial:
        ba_stream = masked_stream(args.ba_cus, first=n_cu - args.ba_cus)
    else:
        ba_stream = (stream if args.ba_serial else
                     torch.cuda.Stream(priority=-1 if args.priority == "ba" else 0))
    # --ba-streams S: the step's windows split into S batches on S streams (one
    # batch's latency-bound camera solve overlaps another's linearisation)
    ns = max(1, min(args.ba_streams, len(windows)))
    ba_subs = [ba_stream] if ns == 1 else [torch.cuda.Stream(priority=-1 if args.priority == "ba" else 0)
                                            for _ in range(ns)]
    bas = []
    for i, s in enumerate(ba_subs):
        with torch.cuda.stream(s):
            # 16 chunks per workgroup unless set: the launch set batches 16
            # windows, so fewer, fuller workgroups still cover the chip and write
            # fewer partial rows -- round 5, alternating runs of this bench
            # (profiles/r5/cpw_ab): 8 / 16 / 32 -> 22.0-22.3k / 22.3-22.5k /
            # 21.1-21.2k frames/s, PMC traffic of a batched iteration 54.8 /
            # 44.7 / 39.6 MB (the 16-window set alone is faster at 8: 65k vs
            # 57k window-iterations/s, but beside tracking it is not)
            cpw = args.chunks_per_wg if args.chunks_per_wg is not None else 16
            bas.append(BABatch([BAProblem(*w, stream=s, chunks_per_wg=cpw,
                                          fold_assembly=args.fold)
                                for w in windows[i::ns]], stream=s))
    ba = bas[0]
    torch.cuda.synchronize()
    tstream = trk_stream if trk_stream is not None else stream
    all_poses = {}
    feed.prime()

    def ev_on(s):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(s)
        return ev

    # the tracked leg (beside `value`, never it): local-BA windows formed from
    # the frames this bench tracks -- per step, every `ba_every` tracked pairs
    # mapped on the device (WindowMapper: k_rel_to_abs + one device map per
    # window), copied to pinned host memory, and TRK_LAG steps later turned into
    # BA problems on the host (native planner, one staged upload) and advanced
    # `ba_iters` LM iterations on the BA stream (lag-2 pipeline: the host build
    # of step k-2's windows overlaps step k's tracking on the GPU, and their
    # maps' copy to the host has completed while step k-1 ran; lag 3 measured
    # 14.3k vs 15.5-15.7k tracked frames/s, alternating runs, profiles/r5/tracked_leg)
    TRK_LAG = args.tracked_lag
    leg = {"tracked": False}
    tleg = {"wms": None, "ws": None, "build_s": [], "wait_s": [], "shapes": [], "modes": {}}

    ba_done = [None]
    step_no, pending = [0], [0]
    flush_at = {args.warmup, args.warmup + args.steps}  # step numbers that flush a launch set

    def step(marks):
        with torch.cuda.stream(tstream):
            tracked_step(marks)

    def tracked_ba(marks, tmarks, h0):
        """BA of the tracked windows of TRK_LAG steps back, on the BA stream."""
        from slam355.ba import BABatch

        # step k-TRK_LAG's maps (their copy event has fired while step k-1 ran)
        prev = tleg["wms"][(step_no[0] - TRK_LAG) % len(tleg["wms"])]
        if not prev.filled:
            if marks is not None:
                marks["track"] = tmarks
            return
        hw = time.perf_counter()
        prev.event.synchronize()  # step k-lag's maps are on the host
        hb = time.perf_counter()
        tleg["wait_s"].append(hb - hw)
        trk._ht("ba_window_wait", hw)
        # every window's observations, plan, data and descriptor staged by ONE
        # native call (slam_ba_stage_windows) into pinned buffers, uploaded by
        # one asynchronous copy per type on the BA stream (BAWindowSet.stage)
        bps = prev.stage(tleg["ws"], rig.P_l, ba_stream)
        prev.filled = False
        groups = {}
        for bp in bps:
            groups.setdefault(bp.lin_mode, []).append(bp)
        tleg["build_s"].append(time.perf_counter() - hb)
        tleg["shapes"].append([(bp.C, bp.P, bp.O) for bp in bps])
        for mode, g in groups.items():
            tleg["modes"][mode] = tleg["modes"].get(mode, 0) + len(g)
        h0 = trk._ht("ba_window_build", hb)
        bmarks = [("ba_start", ev_on(ba_stream))] if marks is not None else None
        with torch.cuda.stream(ba_stream):
            for g in groups.values():
                for i in range(0, len(g), BABatch.MAX_BATCH):
                    BABatch(g[i:i + BABatch.MAX_BATCH], stream=ba_stream).iterate(args.ba_iters)
        # BAWindowSet double-buffers its device memory: these problems stay valid
        # through the next stage() call (the one after reuses their buffers and
        # they raise from then on); the last set's states are read after the loop
        tleg["last"] = bps
        if bmarks is not None:
            bmarks.append(("local_ba", ev_on(ba_stream)))
            marks["ba"] = bmarks
            marks["track"] = tmarks
        trk._ht("ba_launch", h0)

    def tracked_step(marks):
        tmarks = [] if marks is not None else None
        if marks is not None and trk.host_times is None:
            trk.host_times = {}  # host issue time per call site, timed steps only
        h0 = time.perf_counter()
        ist = orb_stream if orb_stream is not None else tstream  # the stream that reads imgs
        fd = feeds[0]
        imgs, win = fd.next(ist)
        h0 = trk._ht("upload_issue", h0)
        if win == 0:  # a new pass over the sequence starts at frame 0
            if gchain is None:
                trk.reset_chain()
            else:
                gchain.reset(tstream)
            h0 = trk._ht("reset_chain", h0)
        if args.ba_overlap == "after-orb" and ba_done[0] is not None:
            ist.wait_event(ba_done[0])  # ORB never shares the chip with the BA chain
        if leg["tracked"]:
            wm = tleg["wms"][step_no[0] % len(tleg["wms"])]
            wm.save_pose0(tstream)
        trk.track(f0s[win], imgs=imgs, marks=tmarks, chain=gchain is None)
        if leg["tracked"]:
            wm.map_batch(tstream)
        h0 = time.perf_counter()
        if gchain is not None:
            gchain.step(trk.rvec, trk.tvec, trk.p_ninl, tstream)
            h0 = trk._ht("global_chain", h0)
        fd.release(ist)
        if tmarks is not None and orb_stream is not None:
            marks["orb"] = trk.orb_marks  # ORB's own stream: start -> done there
        if marks is None and args.keep_poses:
            all_poses[win] = trk.poses.clone()
        if leg["tracked"]:
            tracked_ba(marks, tmarks, h0)
            step_no[0] += 1
            return
        step_no[0] += 1
        pending[0] += 1
        k = step_no[0]
        if pending[0] < G and k not in flush_at:
            if marks is not None:
                marks["track"] = tmarks
            trk._ht("release_marks", h0)
            return  # this step's windows join the next step's launch set
        # (a set flushed early -- end of warmup, or a timed region of K not a
        # multiple of G -- still advances all G steps' windows: extra work, never less)
        full = pending[0] == G
        pending[0] = 0
        if args.ba_overlap == "after-orb":
            ba_stream.wait_event(trk.orb_event)
        h0 = trk._ht("release_marks", h0)
        bmarks = [("ba_start", ev_on(ba_stream))] if marks is not None and full else None
        for bt, s in zip(bas, ba_subs):
            if s is not ba_stream:
                s.wait_stream(ba_stream)
            with torch.cuda.stream(s):
                # the step's local-BA windows, all advanced together (one launch set
                # per LM iteration; windows restored to their initial state first)
                if args.no_graph:
                    bt.restore()
                    bt.iterate(args.ba_iters)
                else:
                    bt.iterate_graphed(args.ba_iters, with_restore=True)
        for s in ba_subs:
            if s is not ba_stream:
                ba_stream.wait_stream(s)
        if args.ba_overlap == "after-orb":
            ba_done[0] = ev_on(ba_stream)
        if bmarks is not None:
            bmarks.append(("local_ba", ev_on(ba_stream)))
            marks["ba"] = bmarks
        if marks is not None:
            marks["track"] = tmarks
        trk._ht("ba_graph_launch", h0)

    dt, stages = timed_loop(step, args.steps, args.warmup, world, dict_marks=True)
    # host issue time per call site over the timed steps: sum per step and the
    # slowest single call (a call that blocks on the device shows up as a max)
    host_sites = host_site_summary(trk, args.steps)
    main_step_s, main_host_s = timed_loop.step_s, timed_loop.host_s
    pcie = None
    if feed_h2d is not None:
        # the same steps with the frames uploaded from pinned host memory inside
        # the timed region (two device slots, copy stream): the PCIe-inclusive rate
        feeds[0] = feed_h2d
        feed_h2d.prime()
        flush_at.clear()
        flush_at.update({step_no[0] + args.warmup, step_no[0] + args.warmup + args.steps})
        dt_p, st_p = timed_loop(step, args.steps, args.warmup, world, dict_marks=True)
        pcie = {"frames_per_s": reduce_scalar(float(B * args.steps), world, "sum") / dt_p,
                "ms_per_step": dt_p / args.steps * 1e3,
                "host_issue_ms_per_step": timed_loop.host_s / args.steps * 1e3,
                "host_issue_sites": host_site_summary(trk, args.steps),
                "upload_bytes_per_step": float(feed_h2d.packs[0].numel()),
                "note": "frames streamed from pinned host memory inside the timed region "
                        "(copy stream, two device slots); not the headline"}
        feeds[0] = feed
    tracked = None
    if not args.no_tracked_leg and world == 1 and B % args.ba_every == 0:
        from slam355.pipeline import WindowMapper

        tleg["wms"] = [WindowMapper(trk, args.ba_every) for _ in range(TRK_LAG + 1)]
        from slam355.ba import BAWindowSet

        tleg["ws"] = BAWindowSet()
        leg["tracked"] = True
        feeds[0] = feed
        feed.prime()
        trk.host_times = None
        dt_t, st_t = timed_loop(step, args.steps, args.warmup, world, dict_marks=True)
        leg["tracked"] = False
        shp = np.array([x for s_ in tleg["shapes"][-args.steps:] for x in s_], float)
        last = tleg.get("last") or []
        sts = [bp.state() for bp in last]
        tracked = {"frames_per_s": float(B * args.steps) / dt_t, "ms_per_step": dt_t / args.steps * 1e3,
                   "host_issue_ms_per_step": timed_loop.host_s / args.steps * 1e3,
                   "host_issue_sites": host_site_summary(trk, args.steps),
                   "windows_per_step": B // args.ba_every, "pairs_per_window": args.ba_every,
                   "lm_iters": args.ba_iters,
                   "window_cams_pts_obs_mean": shp.mean(0).tolist() if len(shp) else None,
                   "window_pts_obs_max": shp.max(0)[1:].tolist() if len(shp) else None,
                   "host_build_ms_per_step": float(np.mean(tleg["build_s"][-args.steps:])) * 1e3,
                   "host_build_ms_per_window": float(np.mean(tleg["build_s"][-args.steps:])) * 1e3
                   / max(1, len(tleg["shapes"][-1]) if tleg["shapes"] else 1),
                   "host_wait_ms_per_step": float(np.mean(tleg["wait_s"][-args.steps:])) * 1e3,
                   "lin_modes": tleg["modes"], "local_ba_ms_per_step": st_t.get("local_ba"),
                   "last_set_cost_mean": float(np.mean([s_["COST"] for s_ in sts])) if sts else None,
                   "last_set_accepted_mean": float(np.mean([s_["NACCEPT"] for s_ in sts])) if sts else None,
                   "note": ("local BA on windows built from the bench's own tracked frames (lag 2: "
                            "host build of step k-2's windows overlaps step k's tracking); not the headline. "
                            "The windows hold ~1/30 of C3's observations (8 cameras x ~830 points x ~1000 "
                            "observations vs 10 x 5000 x 30000); the reference's export conventions "
                            "(camera-to-world poses fed to the world-to-camera BAL projection, KITTI's "
                            "613/185 principal point on 1280x720 frames: XXXport_files.py:51-60, "
                            "BundleAdjustment.py:317-328) make each window ill-posed (cost ~1e8, <= 3 of 10 "
                            "steps accepted), so this leg times LM throughput, not convergence")}
        torch.cuda.synchronize()
        tleg["wms"], tleg["last"] = None, None
    frames = reduce_scalar(float(B * args.steps), world, "sum")
    cnt = trk.counters()  # raises on any ORB workspace overflow since the start
    # accuracy of the tracked trajectory (the last tracked window; the device
    # chain restarts at frame 0 of the sequence with window 0) against ground truth
    last_win = (args.warmup + args.steps - 1) % n_win
    # the chain of the last global step: world * B poses from frame last_win*world*B
    est = (trk.poses if gchain is None else gchain.poses).cpu().numpy()
    f0 = last_win * world * B
    gt = np.stack([np.linalg.inv(poses[0]) @ poses[f0 + i + 1] for i in range(world * B)])
    t_err = np.linalg.norm(est[:, :3, 3] - gt[:, :3, 3], axis=1)
    # drift inside the window, relative to its first tracked frame
    rel_e = np.stack([np.linalg.inv(est[0]) @ e for e in est])
    rel_g = np.stack([np.linalg.inv(gt[0]) @ g_ for g_ in gt])
    t_err_win = np.linalg.norm(rel_e[:, :3, 3] - rel_g[:, :3, 3], axis=1)

    # roofline of the dominant stage
    n_img = 2 * B + 1
    patch_bytes = 36 * 216 * 192
    kp_mean = float(np.mean(cnt["orb"]))
    orb_bytes = n_img * (patch_bytes + kp_mean * ORB_OUT_BYTES)
    orb_ms = stages.get("orb", float("nan"))
    # one batched LM iteration advances all n_launch windows
    ba_ms_iter = stages.get("local_ba", float("nan")) / args.ba_iters
    ba_flops = n_launch * ba_flops_per_iter(*C3[:2], C3[1] * C3[2], C3[2])
    roof = {
        "orb": {"bound": "hbm", "achieved": orb_bytes / (orb_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "kernel": "k_orb_tile+k_orb_compact", "ms_per_launch": orb_ms,
                "bytes_per_launch": orb_bytes},
        "local_ba": {"bound": "mfma", "achieved": ba_flops / (ba_ms_iter * 1e-3) / 1e12,
                     "peak": F64_PEAK_TFLOPS, "unit": "TFLOP/s", "kernel": f"batched LM iteration of {n_launch} C3 windows: k_lin_mfma (assembly folded in) + k_solve_blk + k_back_trial (one HIP graph)" if args.fold else f"batched LM iteration of {n_launch} C3 windows: k_lin_mfma + k_assemble + k_solve_blk + k_back_trial (one HIP graph)",
                     "ms_per_iter": ba_ms_iter, "flops_per_iter": ba_flops},
    }
    # the stereo matcher launch (keypoint.py:44: B pairs of ~2000 x ~2000
    # descriptors): integer-VALU bound, pairs x ops / VALU peak
    oc = cnt["orb"].astype(np.int64)
    m_pairs = float((oc[:B] * oc[B + 1:2 * B + 1]).sum())
    m_ms = stages.get("stereo_knn2", float("nan"))
    roof["matcher"] = matcher_roofline(m_pairs, m_ms, trk.cap, "stereo, in the pipeline", args.valu)
    roof["matcher"]["unique_descriptor_bytes"] = float(oc[:B].sum() + oc[B + 1:2 * B + 1].sum()) * 32
    pmc = pmc_traffic()
    roof["orb"]["traffic"] = pmc_bytes(pmc, ("k_orb_tile<false>", "k_orb_compact"))
    # ORB is bound by instruction latency, not HBM: its vector-ALU issue rate
    # (wave64 VALU instructions per launch from the SQ pass x 64 lanes over the
    # launch time) against the VALU peak, beside the HBM fraction
    vi = pmc_valu("k_orb_tile<false>")
    if vi is not None:
        valu = vi[0] * 64 / (orb_ms * 1e-3) / 1e12
        roof["orb"]["valu"] = {"achieved": valu, "peak": VALU_PEAK_TOPS, "unit": "T lane-ops/s",
                               "frac": valu / VALU_PEAK_TOPS, "valu_instr_per_launch": vi[0],
                               "source": vi[1]}
    roof["local_ba"]["traffic"] = pmc_bytes(pmc, ("k_lin_mfma", "k_solve_blk", "k_back_trial<true>")
                                            + (() if args.fold else ("k_assemble",)))
    roof["matcher"]["traffic"] = pmc_bytes(pmc, (roof["matcher"]["kernel"].split()[0],))
    units = {"orb": f"bytes per ORB launch ({n_img} images), HBM, from PMC",
             "local_ba": f"bytes per batched LM iteration ({n_launch} windows), HBM, from PMC",
             "matcher": "bytes per matcher dispatch (mean of the stereo and temporal launches), HBM, from PMC"}
    for name, r in roof.items():
        r["frac"] = r["achieved"] / r["peak"]
        if r["traffic"] is not None:
            r["traffic_unit"] = units[name]
            r["traffic_source"] = pmc["path"]
    per_step = {k: v for k, v in stages.items()}
    if G > 1 and "local_ba" in per_step:  # one launch set per G steps
        per_step["local_ba_per_launch_set"] = per_step["local_ba"]
        per_step["local_ba"] /= G
    dominant = max(("orb", orb_ms), ("local_ba", per_step.get("local_ba", 0.0)), key=lambda kv: kv[1])[0]
    rec = {
        "metric": "frames/sec tracking+local-BA @1280x720",
        "value": frames / dt,
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "host_issue_ms_per_step": main_host_s / args.steps * 1e3,
        "host_issue_sites": host_sites,
        "host_issue_ms_per_step_list": [round(x * 1e3, 3) for x in main_step_s],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8+f32+f64",
        "data": (f"synthetic (seeded textured-corridor stereo sequence, {n_win * world * B + 1} "
                 f"frames 1280x720, each rank's {n_win} windows resident in its HBM; GT poses)"),
        "config": {"workload": f"C2 tracking (1280x720, {args.kp_per_tile} ORB kp/tile) + "
                               f"C3 local BA (10 KF x 5k pts x 30k obs) every {args.ba_every} frames "
                               f"x {args.ba_iters} LM iters ({n_solves} windows per step, batched" +
                               (f" over {G} steps per launch set)" if G > 1 else ")"),
                   "orb_kp_mean": kp_mean,
                   "frames_per_gpu_per_step": B, "parallelism": f"frame-pair shards x{world}",
                   "inputs": "resident in HBM before the timed region (the PCIe-inclusive "
                             "rate with the frames streamed from pinned host memory: pcie_inclusive)",
                   "local_ba_stream": "serial" if args.ba_serial else "concurrent",
                   "high_priority_stream": args.priority,
                   "ba_overlap": args.ba_overlap,
                   "tracking_cus": args.track_cus or "all",
                   "orb_stream": (f"pipelined, CUs 0..{args.orb_cus - 1}" if args.orb_cus else
                                  "pipelined, all CUs") if args.orb_pipeline else "tracking stream",
                   "local_ba_cus": args.ba_cus or "all",
                   # the headline's windows are fixed synthetic C3 problems (clean
                   # tracks, sigma 0.5 px), restored and re-solved every launch set;
                   # BA over windows built from the tracked frames is measured
                   # beside it in "tracked_source" (a timed region of its own;
                   # --ba-source tracked makes it the line's value)
                   "local_ba_source": "synthetic C3",
                   "local_ba_launch_set": (f"{n_launch} windows every {G} steps (pending steps flushed "
                                           "as a whole set at the ends of warmup and timed region)" if G > 1 else
                                           f"{n_launch} windows every step")},
        "roofline": dict(roof[dominant], stage=dominant),
        "roofline_stages": roof,
        "stage_ms_per_step": per_step,
        "ba_iters_per_s": reduce_scalar((n_solves * args.ba_iters * args.steps) / dt, world, "sum"),
        "tracking": {"orb_kp_mean": kp_mean, "stereo_matches_mean": float(np.mean(cnt["stereo"])),
                     "f_inliers_mean": float(np.mean(cnt["f_inliers"])),
                     "temporal_mean": float(np.mean(cnt["temporal"])),
                     "pnp_inliers_mean": float(np.mean(cnt["pnp_inliers"])),
                     "trajectory_t_err_m_max_from_frame0": float(t_err.max()),
                     "trajectory_t_err_m_max_in_window": float(t_err_win.max()),
                     "frames_chained": int(f0 + world * B),
                     "trajectory": ("one sequence, frame-pair shards, gathered and chained on "
                                    "every rank each step (slam355.dist.GlobalChain)"
                                    if world > 1 else "one sequence, device pose chain"),
                     # bytes of the last global step's chained poses: equal across world
                     # sizes with equal world * batch (the same pairs per global step)
                     "trajectory_sha1": hashlib.sha1(np.ascontiguousarray(est).tobytes()).hexdigest()},
    }
    if pcie is not None:
        rec["pcie_inclusive"] = pcie
    if tracked is not None:
        rec["tracked_source"] = tracked
    if args.ba_source == "tracked":
        # the line's value from the tracked-source region (opt-in; the driver's
        # default stays the BASELINE-named synthetic C3 windows)
        if tracked is None:
            raise SystemExit("--ba-source tracked needs the tracked leg (one rank, batch a "
                             "multiple of --ba-every, no --no-tracked-leg)")
        rec["synthetic_source"] = {"frames_per_s": rec["value"], "ms_per_step": rec["ms_per_step"]}
        rec["value"], rec["ms_per_step"] = tracked["frames_per_s"], tracked["ms_per_step"]
        rec["config"]["local_ba_source"] = (f"tracked: windows of {args.ba_every} tracked frame pairs, "
                                            "mapped on the device, staged by one native call, solved "
                                            f"{args.tracked_lag} steps behind tracking (tracked_source)")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline_tracking(L_np, R_np, rig, args, C3, windows[0],
                                                    pairs=CPU_PAIRS, lm_iters=CPU_PAIRS)
    if not args.no_tracked_ba:
        rec["tracked_window_ba"] = tracked_window_ba(feed, B, rig, args)
    del trk, ba, bas  # their kernels' buffers, then the masked streams themselves
    if trk_stream is not None:
        trk_stream.destroy()
    if hasattr(ba_stream, "destroy"):
        ba_stream.destroy()
    if hasattr(orb_stream, "destroy"):
        orb_stream.destroy()
    if not args.no_ba_scale:
        # the metric's second half: local-BA LM iterations/s of ONE C4 window
        # sharded over all ranks (landmarks by anchor keyframe, RCCL all-reduce
        # of the reduced camera system per iteration) -- strong scaling in N
        rec["local_ba_sharded"] = c4_sharded_iters(world, rank, steps=20, warmup=3)
    return rec


def host_site_summary(trk, steps):
    """Host issue time per call site over the timed steps (Tracker.host_times):
    sum per step and the slowest single call (a call that blocks on the device
    shows up as a large max); resets the record."""
    out = {k: {"ms_per_step": float(np.sum(v)) / steps * 1e3, "max_ms": float(np.max(v)) * 1e3,
               "calls": len(v)} for k, v in (trk.host_times or {}).items()}
    trk.host_times = None
    return out


def tracked_window_ba(feed, B, rig, args, n_pairs=8):
    """Local BA on a window built from tracked frames (main.py:120-127 ->
    XXXport_files.export_data -> BundleAdjustment): n_pairs frame pairs of the
    streamed sequence tracked on the device, their temporally matched points
    mapped by LocalMap (device rel_to_abs + appendKeyPoints on the device map),
    the BA problem formed from the map (problem_from_map) and solved with
    `ba_iters` LM iterations (one HIP graph).  Reported beside `value`: the
    host-side problem build and the device LM time."""
    from slam355.ba import BAProblem
    from slam355.pipeline import LocalMap, Tracker

    pack = feed.packs[0]
    imgs = torch.cat([pack[:n_pairs + 1], pack[B + 1:B + 1 + n_pairs]]).cuda()
    trk = Tracker(n_pairs, H_IMG, W_IMG, rig.P_l, rig.P_r, max_kp_per_tile=args.kp_per_tile, seed=0)
    lm = LocalMap(trk)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    trk.track(0, imgs=imgs)
    lm.add(0)
    torch.cuda.synchronize()
    t_map = time.perf_counter()
    BAProblem(*lm.problem(rig.P_l))  # the first build pays one-time imports (scipy Rotation)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    cams, pts, ci, pi, qs = lm.problem(rig.P_l)
    t1b = time.perf_counter()
    prob = BAProblem(cams, pts, ci, pi, qs)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    prob.iterate(1)
    cost0 = prob.state()["COST"]  # at the initial parameters
    prob.iterate_graphed(args.ba_iters)  # capture + warm
    prob.restore()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    prob.iterate_graphed(args.ba_iters)
    e1.record()
    torch.cuda.synchronize()
    st = prob.state()
    return {"frames": n_pairs + 1, "n_cams": int(len(cams)), "n_pts": int(len(pts)),
            "n_obs": int(len(ci)), "track_and_map_ms": (t_map - t0) * 1e3,
            "host_problem_build_ms": (t2 - t1) * 1e3,
            "host_problem_build_split_ms": {"problem_from_map": (t1b - t1) * 1e3,
                                            "ba_problem_plan_upload": (t2 - t1b) * 1e3},
            "lm_ms_per_iter": e0.elapsed_time(e1) / args.ba_iters, "lm_iters": args.ba_iters,
            "cost_first": cost0, "cost_final": st["COST"], "accepted": int(st["NACCEPT"]),
            "lin_mode": prob.lin_mode}


def _backend_name():
    import torch.distributed as dist

    b = dist.get_backend()
    return "RCCL (nccl)" if b == "nccl" else b


def c4_sharded_iters(world, rank, steps=20, warmup=3):
    """LM iterations/s of the C4 window (64 KF x 50k points x 300k obs) on `world`
    ranks: every rank holds all cameras and the observations of its landmark
    shard, builds its partial reduced camera system, RCCL all-reduces it
    (packed upper blocks, f64 sum) and the 2-double trial cost, and solves the
    camera system redundantly (BAProblem.step_distributed)."""
    from slam355.ba import BAProblem, upper_blocks
    from slam355.synthetic import ba_problem, perturb

    C, P, k = 64, 50000, 6
    rng = np.random.default_rng(7)  # the same global problem on every rank
    cams, pts, ci, pi, qs = ba_problem(rng, C, P, k)
    c0, p0 = perturb(rng, cams, pts)
    if world > 1:
        from slam355.dist import shard_by_anchor, shard_chunks_per_wg

        mine, keep, local_pi = shard_by_anchor(C, P, ci, pi, rank, world)
        prob = BAProblem(c0, p0[mine], ci[keep], local_pi, qs[keep],
                         block_list=upper_blocks(C, ci, pi),
                         chunks_per_wg=shard_chunks_per_wg(int(keep.sum())))
        step_fn = prob.step_distributed
        n_obs = int(keep.sum())
    else:
        prob = BAProblem(c0, p0, ci, pi, qs)
        step_fn = lambda: prob.iterate_graphed(1)  # noqa: E731
        n_obs = len(ci)
    dt, _ = timed_loop(lambda marks: step_fn(), steps, warmup, world, marks_every=False)
    return {"workload": f"C4 local BA {C} KF x {P} pts x {P * k} obs, one window over all ranks",
            "iters_per_s": steps / dt, "ms_per_iter": dt / steps * 1e3, "ranks": world,
            "obs_per_rank": n_obs, "scaling": "strong",
            "collective": (f"{_backend_name()} all_reduce (sum, f64) of the packed reduced camera "
                           "system + 2 doubles per LM iteration") if world > 1 else "none (1 GPU)",
            "final_cost": prob.state()["COST"]}


def cpu_baseline_tracking(L, R, rig, args, C3, ba_in, pairs=2, lm_iters=1):
    """The CPU oracle (C ORB/kNN/F-LMedS/PnP + numpy DLT, numpy Schur LM) on a
    bounded sample: `pairs` frame pairs of the same sequence and `lm_iters` LM
    iterations of the same C3 window, combined with the same BA schedule."""
    import oracle
    from oracle import ba as oba
    from oracle import pipeline as opl

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    t0 = time.perf_counter()
    cache = {}
    kp, octv, desc, cnt = oracle.orb_tiles_batch(np.concatenate([L[:pairs + 1], R[:pairs]]),
                                                 args.kp_per_tile, 1 << 13)
    for i in range(pairs + 1):
        cache[("L", i)] = (kp[i, :cnt[i]], octv[i, :cnt[i]], desc[i, :cnt[i]])
    for i in range(pairs):
        j = pairs + 1 + i
        cache[("R", i)] = (kp[j, :cnt[j]], octv[j, :cnt[j]], desc[j, :cnt[j]])
    for i in range(pairs):
        opl.track_pair(L[i], R[i], L[i + 1], rig.P_l, rig.P_r, max_kp=args.kp_per_tile, seed=0,
                       frame=i, orb_cache=cache)
    t_track = (time.perf_counter() - t0) / pairs
    c0, p0, ci, pi, qs = ba_in
    pr = oba._obs_pairs(ci, pi)
    t1 = time.perf_counter()
    st, oc, op = oba.LMState(), c0, p0
    for _ in range(lm_iters):
        oc, op, _ = oba.lm_iteration_schur(oc, op, ci, pi, qs, st, pr)
    t_iter = (time.perf_counter() - t1) / lm_iters
    per_frame = t_track + args.ba_iters * t_iter / args.ba_every
    return {"value": 1.0 / per_frame, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{pairs} frame pairs through the oracle chain (ORB OpenMP x{threads} "
                      f"over {2 * pairs + 1} images, rest single-thread C/numpy) = "
                      f"{t_track * 1e3:.0f} ms/frame + {lm_iters} numpy Schur LM iterations on "
                      f"the C3 window = {t_iter * 1e3:.0f} ms/iter (x{args.ba_iters}/{args.ba_every} "
                      f"per frame); sample wall {time.perf_counter() - t0:.1f} s"}


# ---------------------------------------------------------------------------- local BA
def run_ba(args, world, rank):
    from slam355.ba import BAProblem, packed, tiled_solve_flops, upper_blocks
    from slam355.synthetic import ba_problem, ba_problem_loop, perturb

    if args.ba_batch > 1:
        return run_ba_batch(args, world, rank)
    if args.c5:
        C, P, k, name = 500, 200000, 6, "C5"
    elif world == 1 and not args.c4:
        C, P, k, name = 10, 5000, 6, "C3"
    else:
        C, P, k, name = 64, 50000, 6, "C4"
    rng = np.random.default_rng(7)  # same global problem on every rank
    gen = ba_problem_loop if name == "C5" else ba_problem
    cams, pts, ci, pi, qs = gen(rng, C, P, k)
    c0, p0 = perturb(rng, cams, pts)
    if world > 1:
        from slam355.dist import shard_by_anchor, shard_chunks_per_wg

        mine, keep, local_pi = shard_by_anchor(C, P, ci, pi, rank, world)
        prob = BAProblem(c0, p0[mine], ci[keep], local_pi, qs[keep],
                         block_list=upper_blocks(C, ci, pi),
                         chunks_per_wg=shard_chunks_per_wg(int(keep.sum())))
        step_fn = prob.step_distributed
    else:
        prob = BAProblem(c0, p0, ci, pi, qs, chunks_per_wg=args.chunks_per_wg,
                         fold_assembly=args.fold)
        if args.no_graph:
            step_fn = lambda: prob.iterate(1)  # noqa: E731
        else:  # one LM iteration = one HIP-graph replay (3T + 5 launches for the tiled solver)
            step_fn = lambda: prob.iterate_graphed(1)  # noqa: E731

    pose_graph = pose_graph_solve(C) if name == "C5" and rank == 0 else None

    def step(marks):
        step_fn()

    dt, _ = timed_loop(step, args.steps, args.warmup, world, marks_every=False)
    flops = ba_flops_per_iter(C, P, P * k, k)
    if packed(C):  # tiled solver: count the tile envelope it factors, not a dense (9C)^3/3
        flops += tiled_solve_flops(C, prob.plan["blocks"]) - (9 * C) ** 3 / 3
    it_s = args.steps / dt
    achieved = flops * it_s / 1e12
    return {
        "metric": "local-BA LM iterations/sec",
        "value": it_s, "unit": "iters/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
        "scaling": "strong" if world > 1 else "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic BA problem (seeded, 6 obs/point, sigma 0.5 px)",
        "config": {"workload": f"{name} {'loop-closure global' if name == 'C5' else 'local'} BA "
                               f"{C} KF x {P} pts x {P * k} obs",
                   "packed_blocks": int(prob.plan["blocks"].shape[0]),
                   "parallelism": f"landmark shards x{world} + RCCL all-reduce" if world > 1 else "1 GPU"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": F64_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / F64_PEAK_TFLOPS, "traffic": None,
                     "kernel": "LM iteration", "flops_per_iter": flops},
        "final_cost": prob.state()["COST"],
    } | ({"pose_graph": pose_graph,
          "c5_pose_graph_plus_ba_ms": pose_graph["ms_per_solve"] + args.ba_iters * dt / args.steps * 1e3,
          "c5_sequence": f"pose-graph TRF solve to convergence, then {args.ba_iters} full-BA LM "
                         "iterations (BundleAdjustment.py:179-182, then :397-402)"}
         if pose_graph is not None else {})


def pose_graph_solve(m):
    """The pose-graph half of BASELINE config 5 (BundleAdjustment.py:107-183,
    loop_closure.py:39-52): scipy-TRF semantics on the m relative poses of a
    drifted closed loop (k_chain_trf, one workgroup), run to its ftol test;
    wall time per solve, including the host's status checks between chunks of
    64 iterations."""
    from slam355.posegraph import PoseChain
    from slam355.synthetic import pose_chain_loop

    x0 = pose_chain_loop(np.random.default_rng(11), m)
    PoseChain(x0).solve(ftol=1e-8)  # warm (module load, first launch)
    torch.cuda.synchronize()
    times = []
    for _ in range(3):
        pc = PoseChain(x0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = pc.solve(ftol=1e-8)
        times.append(time.perf_counter() - t0)
    ms = float(np.median(times)) * 1e3
    return {"frames": m, "params": 6 * m, "residuals": m + 2, "ms_per_solve": ms,
            "nfev": st["nfev"], "njev": st["njev"], "iterations": st["iterations"],
            "ms_per_iteration": ms / max(1, st["iterations"]), "status": st["message"],
            "cost0": st["cost0"], "cost": st["cost"]}


def run_ba_batch(args, world, rank):
    """--workload ba --ba-batch N: N independent C3 windows advanced together
    (slam_ba_iterate_batch, one HIP graph per LM iteration); value = window LM
    iterations/s over all ranks (each rank its own windows: weak scaling)."""
    from slam355.ba import BABatch, BAProblem
    from slam355.synthetic import ba_problem, perturb

    C, P, k = 10, 5000, 6
    rng = np.random.default_rng(7 + rank)
    probs = []
    # chunks per linearisation workgroup: with the whole GPU to itself a batch
    # of 8 windows is fastest at 5 (3 -> 46.1k, 5 -> 50.3k, 8 -> 41.0k
    # window-iters/s; 4 windows: 3 and 5 within noise, 121.5 / 123.4 us); the
    # tracking bench, which leaves BA about 40 CUs beside ORB, uses 8
    cpw = args.chunks_per_wg
    if cpw is None and args.ba_batch >= 8:
        cpw = 5
    for _ in range(args.ba_batch):
        cams, pts, ci, pi, qs = ba_problem(rng, C, P, k)
        c0, p0 = perturb(rng, cams, pts)
        probs.append(BAProblem(c0, p0, ci, pi, qs, lin_mode=args.lin_mode,
                               chunks_per_wg=cpw, fold_assembly=args.fold))
    # --ba-streams S: the windows split into S batches on S streams, so one
    # batch's latency-bound camera solve overlaps another's linearisation
    ns = max(1, min(args.ba_streams, len(probs)))
    streams = [torch.cuda.Stream() for _ in range(ns)] if ns > 1 else [None]
    bats = [BABatch(probs[i::ns], stream=streams[i]) for i in range(ns)]
    bat = bats[0]
    cur = torch.cuda.current_stream()

    def step(marks):
        if ns == 1:
            bat.iterate_graphed(1)
            return
        for b, st in zip(bats, streams):
            st.wait_stream(cur)
            b.iterate_graphed(1)
        for st in streams:
            cur.wait_stream(st)

    dt, _ = timed_loop(step, args.steps, args.warmup, world, marks_every=False)
    flops = args.ba_batch * ba_flops_per_iter(C, P, P * k, k)
    it_s = args.steps / dt
    achieved = flops * it_s / 1e12
    return {
        "metric": "local-BA LM iterations/sec (batched C3 windows)",
        "value": reduce_scalar(args.ba_batch * it_s, world, "sum"), "unit": "window-iters/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic BA windows (seeded, 6 obs/point, sigma 0.5 px)",
        "config": {"workload": f"{args.ba_batch} x C3 local BA {C} KF x {P} pts x {P * k} obs, batched",
                   "parallelism": f"window shards x{world}"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": F64_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / F64_PEAK_TFLOPS, "traffic": None,
                     "kernel": "batched LM iteration", "flops_per_iter": flops},
        "ba_streams": ns,
        "final_costs": [s["COST"] for b in bats for s in b.states()],
    }


# ---------------------------------------------------------------------------- matcher
def run_matcher(args, world, rank):
    from slam355 import matcher
    from slam355.synthetic import descriptor_batch

    if args.valu:
        from slam355 import _lib

        _lib.lib.slam_hamming_force_valu(1)
    q, nq, t, nt = descriptor_batch(args.batch, 2000, 2000, seed=rank)
    dev = torch.device("cuda")
    tq, tt = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    tnq, tnt = torch.from_numpy(nq).to(dev), torch.from_numpy(nt).to(dev)
    out = matcher.knn2_batch(tq, tnq, tt, tnt)
    stream = torch.cuda.current_stream()

    def step(marks):
        if marks is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            marks.append(("start", e))
        matcher.knn2_batch(tq, tnq, tt, tnt, out=out)
        if marks is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            marks.append(("knn2", e))

    dt, stages = timed_loop(step, args.steps, args.warmup, world)
    pairs = float((nq.astype(np.int64) * nt).sum())
    kms = stages["knn2"]
    roof = matcher_roofline(pairs, kms, t.shape[1], f"batch {args.batch}", args.valu)
    roof["frac"] = roof["achieved"] / roof["peak"]
    roof["traffic"] = None
    return {
        "metric": "BF-Hamming kNN-2 match throughput @ C2 (2000x2000 x 32 B descriptors)",
        "value": reduce_scalar(pairs * args.steps, world, "sum") / dt / 1e9, "unit": "Gpairs/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded random descriptors, 60% planted near-duplicates)",
        "config": {"workload": "C2 matcher", "batch_pairs_per_gpu": args.batch},
        "roofline": roof,
    }


# ---------------------------------------------------------------------------- LK/SGBM VO
SGBM_OPS_PER_CELL = 58  # BT cost 12 + box sums 4 + 5 paths x 7 + S/saturation 6 + argmin 1


def run_vo(args, world, rank):
    """The alternative stereo-VO front end (visual_odometry.py get_pose :188-195):
    one step = B frame pairs at 1280x720: FAST on 10x20 tiles, LK pyramids,
    pyramidal LK, SGBM on B+1 stereo pairs, disparity lookup + float32 DLT and
    the RANSAC-6 + LM pose; SGBM on a second stream, concurrent with FAST / LK."""
    from slam355 import geometry, vofront
    from slam355.synthetic import stereo_sequence

    B = args.batch
    L, R, poses, rig = stereo_sequence(B + 1, W_IMG, H_IMG, seed=rank)
    dev = torch.device("cuda")
    tl, tr = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    stream = torch.cuda.current_stream()
    # SGBM (independent of FAST / LK) runs on a second stream, concurrently
    sgbm_stream = torch.cuda.Stream()
    out = {}

    def mark(marks, lane, name, st):
        if marks is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record(st)
            marks.setdefault(lane, []).append((name, e))

    def step(marks):
        ready = torch.cuda.Event()
        ready.record(stream)
        sgbm_stream.wait_event(ready)
        with torch.cuda.stream(sgbm_stream):
            mark(marks, "sgbm", "start", sgbm_stream)
            _, dispf = vofront.sgbm(tl, tr, **vofront.SGBM)
            mark(marks, "sgbm", "sgbm", sgbm_stream)
            done = torch.cuda.Event()
            done.record(sgbm_stream)
        dispf.record_stream(stream)
        mark(marks, "main", "start", stream)
        kp, nkp = vofront.fast_tiles(tl[:B])
        mark(marks, "main", "fast", stream)
        pyr = vofront.LKPyramids(tl)
        mark(marks, "main", "lk_pyramids", stream)
        p2, st, err = vofront.lk_track(pyr, pyr, kp, nkp, prev0=0, next0=1)
        mark(marks, "main", "lk_track", stream)
        tp1, tp2, _, ntp = vofront.lk_filter(kp, p2, st, err, nkp, H_IMG, W_IMG)
        mark(marks, "main", "lk_filter", stream)
        stream.wait_event(done)
        mark(marks, "main", "wait_sgbm", stream)
        o = vofront.right_qs_3d(tp1, tp2, ntp, dispf, rig.P_l, rig.P_r)
        mark(marks, "main", "right_qs_3d", stream)
        pose, _, _, _ = geometry.vo_estimate_pose(o["q1_l64"], o["q2_l64"], o["Q1_64"],
                                                  o["Q2_64"], o["count"], rig.P_l, seed=0)
        mark(marks, "main", "pose", stream)
        out.update(nkp=nkp, ntp=ntp, cnt=o["count"], pose=pose)

    dt, stages = timed_loop(step, args.steps, args.warmup, world, dict_marks=True)
    frames = B * args.steps
    value = reduce_scalar(frames, world, "sum") / dt
    W1 = W_IMG - 32
    cells = (B + 1) * H_IMG * W1 * 32
    sgbm_ms = stages["sgbm"]
    achieved = cells * SGBM_OPS_PER_CELL / (sgbm_ms * 1e-3) / 1e12
    dof = out["pose"].cpu().numpy()
    gt_dz = [float((np.linalg.inv(poses[i]) @ poses[i + 1])[2, 3]) for i in range(B)]
    rec = {
        "metric": "frames/sec LK/SGBM stereo-VO front end @1280x720 (visual_odometry.py get_pose)",
        "value": value, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8+i16+f32+f64",
        "data": "synthetic (seeded 1280x720 stereo sequence, GT poses)",
        "config": {"workload": "LK/SGBM VO: FAST 10x20 tiles x10, LK 15x15x4 levels, SGBM 32 disp "
                               "block 11, RANSAC-6 LM pose", "frames_per_gpu_per_step": B,
                   "parallelism": f"frame-pair shards x{world}",
                   "streams": "SGBM concurrent with FAST / LK"},
        "roofline": {"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_TOPS,
                     "unit": "Tops/s", "frac": achieved / VALU_PEAK_TOPS,
                     "traffic": sgbm_traffic(),
                     "traffic_unit": "bytes per launch (33 stereo pairs), HBM, from PMC",
                     "traffic_source": "profiles/pmc_traffic_vo.json",
                     "kernel": "SGBM (k_sgbm_hsum + vert + 2 diag + row + median)",
                     "ms_per_launch": sgbm_ms, "cells_per_launch": cells,
                     "ops_per_cell": SGBM_OPS_PER_CELL},
        "stage_ms_per_step": stages,
        "vo": {"fast_kp_mean": float(out["nkp"].float().mean()),
               "tracked_mean": float(out["ntp"].float().mean()),
               "with_disparity_mean": float(out["cnt"].float().mean()),
               "t_err_max": float(np.abs(dof[:, 5] - np.array(gt_dz)).max())},
    }
    if rank == 0 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline_vo(L, R, rig)
    return rec


def sgbm_traffic():
    pmc = pmc_traffic("pmc_traffic_vo.json")
    if pmc is None:
        return None
    return pmc_bytes(pmc, tuple(k for k in pmc["kernels"] if k.startswith("k_sgbm_")))


def cpu_baseline_vo(L, R, rig, pairs=1):
    """oracle/vofront (C FAST/LK with OpenMP, C SGBM single-thread, numpy glue,
    C pose) on `pairs` frame pairs: SGBM of both frames + get_pose."""
    from oracle import vofront as vf

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    t0 = time.perf_counter()
    d0 = vf.disparity_f32(L[0], R[0])
    for i in range(pairs):
        d1 = vf.disparity_f32(L[i + 1], R[i + 1])
        vf.get_pose(L[i], L[i + 1], d0, d1, rig.P_l, rig.P_r, seed=0, frame=i)
        d0 = d1
    dt = time.perf_counter() - t0
    return {"value": pairs / dt, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{pairs} frame pair(s) through oracle/vofront: SGBM of {pairs + 1} stereo "
                      f"pairs (costs OpenMP x{threads}, paths single-thread C), FAST, LK "
                      f"(OpenMP x{threads}), numpy glue, C pose = {dt * 1e3:.0f} ms"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="tracking", choices=["tracking", "ba", "matcher", "vo"])
    ap.add_argument("--batch", type=int, default=None,
                    help="frame pairs per GPU per step (default: 64 for the tracking workload -- "
                         "in alternating runs 17.6-17.9k frames/s against 16.5-16.7k at 32 and "
                         "15.3k at 128 in the round-3 A/B, DESIGN.md §5 -- 32 elsewhere)")
    ap.add_argument("--kp-per-tile", type=int, default=64,
                    help="ORB max_number_of_kp per tile: 64 -> ~2090 kp/frame (levels 6-7 of a "
                         "216x192 patch cannot hold keypoints, so 56 gives only ~1780)")
    ap.add_argument("--windows", type=int, default=None,
                    help="global steps in the sequence, each gpus x batch frame pairs (default: "
                         "256 / (gpus x batch), at least 2: a 257-frame sequence at 1 GPU, batch 64)")
    ap.add_argument("--keep-poses", action="store_true")
    ap.add_argument("--ba-every", type=int, default=8, help="frames per local-BA solve")
    ap.add_argument("--ba-iters", type=int, default=10, help="LM iterations per local-BA solve")
    ap.add_argument("--lin-mode", default="auto", choices=["auto", "mfma", "slot"],
                    help="BA linearisation: camera-union MFMA kernel or the slot kernel")
    ap.add_argument("--chunks-per-wg", type=int, default=None,
                    help="camera-union linearisation: chunks per workgroup (default: 16 for the "
                         "tracking workload's batched windows -- 8 / 16 / 32 measured 22.0-22.3k "
                         "/ 22.3-22.5k / 21.1-21.2k frames/s, round-5 sweep profiles/r5/cpw_ab; "
                         "auto elsewhere)")
    ap.add_argument("--ba-streams", type=int, default=1,
                    help="split the local-BA windows over this many streams (tracking, and "
                         "--workload ba --ba-batch N)")
    ap.add_argument("--ba-group", type=int, default=None,
                    help="tracking: the local-BA windows of G consecutive steps advance as one "
                         "launch set (default: the fewest steps whose windows fill one batched "
                         "launch of SLAM_BA_MAX_BATCH = 16 -- 2 at batch 64, 4 at batch 32)")
    ap.add_argument("--ba-batch", type=int, default=1,
                    help="--workload ba: advance this many C3 windows together")
    ap.add_argument("--c4", action="store_true", help="--workload ba: C4 problem on 1 GPU")
    ap.add_argument("--c5", action="store_true",
                    help="--workload ba: C5 loop-closure global BA (500 KF x 200k pts)")
    ap.add_argument("--fold", action="store_true",
                    help="local BA: the assembly folded into k_lin_mfma instead of the separate "
                         "k_assemble launch (A/B; measured slower, BAProblem fold_assembly)")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch the LM iterations eagerly instead of replaying a HIP graph")
    ap.add_argument("--ba-overlap", default="full", choices=["full", "after-orb"],
                    help="tracking workload: local BA overlaps all of tracking (full), or "
                         "starts after the batch's ORB and holds the next batch's ORB back")
    ap.add_argument("--priority", default="ba", choices=["ba", "track", "equal"],
                    help="which stream gets the high HIP stream priority (tracking workload)")
    ap.add_argument("--ba-serial", action="store_true",
                    help="run local BA on the tracking stream (no overlap)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ba-scale", action="store_true",
                    help="tracking: skip the sharded C4 local-BA iterations/s measurement")
    ap.add_argument("--track-cus", type=int, default=0,
                    help="restrict the tracking stream to this many CUs (0: all); the rest run "
                         "only local-BA work, whose latency-bound kernels then do not share "
                         "SIMDs and LDS with ORB workgroups")
    ap.add_argument("--no-orb-pipeline", dest="orb_pipeline", action="store_false",
                    help="tracking: ORB on the tracking stream (default: ORB on its own stream "
                         "into double-buffered outputs, so the next batch's ORB overlaps this "
                         "batch's matching / PnP tail)")
    ap.add_argument("--orb-cus", type=int, default=0,
                    help="ORB pipeline: ORB's stream may use only the first N CUs (0: all, the "
                         "default since the camera solve fits two waves per SIMD: alternating "
                         "runs 224 / 232 / 240 / 248 / all -> 19.7-19.8k / 19.9-20.1k / "
                         "20.1-20.2k / 20.3k / 20.5k frames/s, round-4 sweep in git history at f26058c; with "
                         "the 317-register solve round 3 measured 224 best)")
    ap.add_argument("--solve-lds-floor", type=int, default=0,
                    help="LDS bytes the one-workgroup camera solve requests at least "
                         "(slam_ba_set_solve_lds_floor)")
    ap.add_argument("--orb-lds-floor", type=int, default=0,
                    help="LDS bytes k_orb_tile requests at least (slam_orb_set_lds_floor)")
    ap.add_argument("--valu", action="store_true",
                    help="matcher and tracking: force the integer-VALU kNN-2 kernel (default: fp4 "
                         "matrix cores)")
    ap.add_argument("--no-pcie-leg", action="store_true",
                    help="tracking: skip the PCIe-inclusive run (frames streamed from pinned host "
                         "memory inside the timed region) reported beside the headline")
    ap.add_argument("--ba-source", default="synthetic", choices=["synthetic", "tracked"],
                    help="local-BA windows of the line's value: the BASELINE-named synthetic C3 "
                         "windows (default; the tracked-source rate beside it) or the windows "
                         "built from the tracked frames")
    ap.add_argument("--tracked-lag", type=int, default=2,
                    help="steps between a batch's tracking and its tracked-window BA (>= 1)")
    ap.add_argument("--no-tracked-leg", action="store_true",
                    help="skip the tracked-source leg (local BA on windows built from the tracked frames)")
    ap.add_argument("--no-tracked-ba", action="store_true",
                    help="tracking: skip the local BA of a window built from tracked frames")
    ap.add_argument("--ba-cus", type=int, default=0,
                    help="disjoint CU partition: local BA on the last N CUs, tracking on the rest")
    args = ap.parse_args()
    if args.tracked_lag < 1:
        ap.error("--tracked-lag must be >= 1 (0 would stage the window mapper the same step fills)")
    if args.batch is None:
        args.batch = 64 if args.workload == "tracking" else 32
    if args.windows is None:  # global steps in the sequence (each world * batch pairs)
        args.windows = max(2, 256 // (args.batch * args.gpus))
    if args.ba_group is None:  # the fewest steps whose windows fill one batched launch
        args.ba_group = max(1, -(-16 // max(1, args.batch // args.ba_every)))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        print(f"bench.py: WORLD_SIZE={os.environ.get('WORLD_SIZE', '1')} but --gpus {args.gpus}",
              file=sys.stderr)
        sys.exit(2)
    world, rank = dist_init()
    run = {"tracking": run_tracking, "ba": run_ba, "matcher": run_matcher,
           "vo": run_vo}[args.workload]
    rec = run(args, world, rank)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()

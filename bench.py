"""slam355 benchmark — driver contract.

python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

Prints ONE JSON line on rank 0.  For N>1 it is launched by torch.distributed.run
(one process per GPU); each rank processes its own shard of frame pairs
(weak scaling) and the time is the max over ranks.
"""
from __future__ import annotations

import argparse
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

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
HBM_PEAK_GBS = 8000.0
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 78.6 T lane-ops/s (4 SIMD32 per CU)
MATCH_OPS_PER_PAIR = 19  # 8 v_xor + 8 v_bcnt(+acc) + v_lshl_or + v_min + v_med3


def dist_init():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t)
    return float(t.item())


# ---------------------------------------------------------------------------- matcher
def matcher_workload(B: int, seed: int):
    from slam355 import matcher
    from slam355.synthetic import descriptor_batch

    q, nq, t, nt = descriptor_batch(B, 2000, 2000, seed=seed)
    dev = torch.device("cuda")
    tq, tt = torch.from_numpy(q).to(dev), torch.from_numpy(t).to(dev)
    tnq, tnt = torch.from_numpy(nq).to(dev), torch.from_numpy(nt).to(dev)
    out = matcher.knn2_batch(tq, tnq, tt, tnt)
    pairs_per_step = float((nq.astype(np.int64) * nt).sum())

    def step():
        matcher.knn2_batch(tq, tnq, tt, tnt, out=out)

    return step, pairs_per_step, (q, nq, t, nt)


def cpu_baseline_matcher(host, budget_s=10.0):
    import oracle

    q, nq, t, nt = host
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    n = 1
    pairs = 0.0
    t0 = time.perf_counter()
    while True:
        k = min(n, len(nq))
        oracle.hamming_knn2_batch(q[:k], nq[:k], t[:k], nt[:k])
        pairs += float((nq[:k].astype(np.int64) * nt[:k]).sum())
        if time.perf_counter() - t0 > budget_s or k == len(nq) and n > 64:
            break
        n *= 2
    dt = time.perf_counter() - t0
    return {"value": pairs / dt / 1e9, "unit": "Gpairs/s", "cores": threads, "kind": "port",
            "sample": f"C oracle (oracle/hamming.c, OpenMP {threads} threads) on up to "
                      f"{len(nq)} 2000x2000 descriptor pairs, {dt:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="matcher", choices=["matcher"])
    ap.add_argument("--batch", type=int, default=64, help="frame pairs per rank per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world, rank = dist_init()
    step, units_per_step, host = matcher_workload(args.batch, seed=rank)
    stream = torch.cuda.current_stream()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # kernel-level timing: HIP events on the launch stream around each step
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    dt = max_over_ranks(dt, world)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))

    total_units = sum_over_ranks(units_per_step * args.steps, world)
    ops = units_per_step * MATCH_OPS_PER_PAIR
    achieved = ops / (kern_ms * 1e-3) / 1e12
    hbm_bytes = float(args.batch * (2000 + 2000) * 32 + args.batch * 2000 * 17)
    rec = {
        "metric": "BF-Hamming kNN-2 match throughput @ C2 (2000x2000 x 32B descriptors)",
        "value": total_units / dt / 1e9,
        "unit": "Gpairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded random 256-bit descriptors, 60% planted near-duplicates)",
        "config": {"workload": "C2 matcher: 1280x720-class, 2000 kp/frame, BF-Hamming kNN-2",
                   "batch_pairs_per_gpu": args.batch, "parallelism": f"frame-pair shards x{world}"},
        "roofline": {"bound": "valu", "achieved": achieved, "peak": VALU_PEAK_TOPS,
                     "unit": "Tops/s", "frac": achieved / VALU_PEAK_TOPS, "traffic": None,
                     "kernel": "knn2_kernel", "kernel_ms": kern_ms,
                     "hbm_achieved_GBs": hbm_bytes / (kern_ms * 1e-3) / 1e9,
                     "hbm_peak_GBs": HBM_PEAK_GBS,
                     "effective_scan_GBs": units_per_step * 32 / (kern_ms * 1e-3) / 1e9},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline_matcher(host)
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()

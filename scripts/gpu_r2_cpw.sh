#!/bin/bash
# camera-union linearisation: chunks per workgroup sweep (batched C3 windows alone, and in the tracking bench)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/cpw_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
for c in 1 2 3 4; do
  timeout -k 10 120 python bench.py --workload ba --ba-batch 4 --chunks-per-wg $c --steps 50 --warmup 5 > "$OUT/ba_b4_cpw$c.log" 2>&1 || exit 1
done
for c in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 20 --warmup 3 --chunks-per-wg $c > "$OUT/trk_cpw$c.log" 2>&1 || exit 1
done
timeout -k 10 120 python bench.py --workload matcher --batch 32 --steps 50 --warmup 5 > "$OUT/matcher32.log" 2>&1 || exit 1
timeout -k 10 120 python bench.py --workload matcher --batch 512 --steps 20 --warmup 3 > "$OUT/matcher512.log" 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale > "$OUT/bench_tracked.log" 2>&1 || exit 1
echo done

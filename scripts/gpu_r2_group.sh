#!/bin/bash
# default bench vs --ba-group 2 / 3, and batched-window BA lines (4 / 8 / 12 windows)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/group_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
for nb in 4 8 12; do
  timeout -k 10 120 python bench.py --workload ba --ba-batch $nb --steps 200 --warmup 20 > "$OUT/ba_b$nb.log" 2>&1 || exit 1
done
for g in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --ba-group $g --steps 12 --warmup 3 > "$OUT/bench_g$g.log" 2>&1 || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --ba-group 2 --orb-cus 200 --steps 12 --warmup 3 > "$OUT/bench_g2_o200.log" 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --ba-group 2 --orb-cus 232 --steps 12 --warmup 3 > "$OUT/bench_g2_o232.log" 2>&1 || exit 1
echo done

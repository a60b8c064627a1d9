#!/bin/bash
# Batched local-BA windows: bench lines for batch 1/4/8 (+ variants) and a
# rocprofv3 kernel-trace summary of batch 1 and batch 4 (separate runs).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
TAG="${1:-r2}"
shift || true
EXTRA="$*"
for nb in 1 4 8; do
  timeout -k 10 120 python bench.py --workload ba --ba-batch $nb --steps 200 --warmup 20 $EXTRA > "$OUT/ba_batch${nb}_$TAG.log" 2>&1 || exit 1
done
timeout -k 10 120 python bench.py --workload ba --ba-batch 4 --chunks-per-wg 2 --steps 200 --warmup 20 $EXTRA > "$OUT/ba_batch4_s2_$TAG.log" 2>&1 || exit 1
timeout -k 10 120 python bench.py --workload ba --ba-batch 4 --lin-mode slot --steps 200 --warmup 20 $EXTRA > "$OUT/ba_batch4_slot_$TAG.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for nb in 1 4; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_ba_b${nb}_$TAG" -o run \
    -- python3 "$ROOT/bench.py" --workload ba --ba-batch $nb --steps 50 --warmup 5 $EXTRA > "$OUT/ba_prof_b${nb}_$TAG.log" 2>&1 || exit 1
done
echo done

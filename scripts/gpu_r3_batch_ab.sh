#!/bin/bash
# Frame pairs per step A/B of the default tracking bench, alternating in
# separate processes (the same number of timed frames per run):
#   [BATCHES="32 64 128"] gpu_r3_batch_ab.sh TAG [ROUNDS]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
N="${2:-3}"
OUT="$ROOT/gpurun_out/batchab_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 $N); do
  for b in ${BATCHES:-32 64 128}; do
    steps=$((640 / b)); warm=$((256 / b)); [ $warm -lt 2 ] && warm=2
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --batch $b --steps $steps --warmup $warm > "$OUT/b${b}_$i.json" 2> "$OUT/b${b}_$i.err" || exit 1
  done
done
echo done

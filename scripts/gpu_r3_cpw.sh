#!/bin/bash
# Linearisation chunks per workgroup in the tracking bench (8 default vs 12 / 16),
# alternating.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/cpw_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for i in 1 2; do
  for c in 8 12 16; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --chunks-per-wg $c --steps 20 --warmup 4 > "$OUT/c${c}_$i.json" 2> "$OUT/c${c}_$i.err" || exit 1
  done
done
echo done

#!/bin/bash
# ORB pipelining: ORB CU budget sweep
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/orbpipe_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
B="python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 20 --warmup 3 --orb-pipeline"
for c in 224 208 192 176 160; do
  timeout -k 10 120 $B --orb-cus $c > "$OUT/pipe_c${c}.log" 2>&1 || exit 1
done
timeout -k 10 120 $B --orb-cus 192 --priority equal > "$OUT/pipe_c192_eq.log" 2>&1 || exit 1
echo done

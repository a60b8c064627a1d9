#!/bin/bash
# ORB pipelining with CU reservation for the latency-bound BA kernels
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/orbpipe_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
B="python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 20 --warmup 3 --orb-pipeline"
timeout -k 10 120 $B > "$OUT/pipe.log" 2>&1 || exit 1
timeout -k 10 120 $B --solve-lds-floor 86016 > "$OUT/pipe_f84.log" 2>&1 || exit 1
for c in 248 240 224; do
  timeout -k 10 120 $B --orb-cus $c --solve-lds-floor 86016 > "$OUT/pipe_c${c}_f84.log" 2>&1 || exit 1
  timeout -k 10 120 $B --orb-cus $c > "$OUT/pipe_c${c}.log" 2>&1 || exit 1
done
echo done

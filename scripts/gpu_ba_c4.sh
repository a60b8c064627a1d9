#!/bin/bash
# C4 / C5 on one GPU: bench lines + rocprofv3 kernel-trace summaries.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
TAG="${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 200 python bench.py --workload ba --c4 --steps 50 --warmup 5 > "$OUT/ba_c4_$TAG.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload ba --c5 --steps 20 --warmup 3 > "$OUT/ba_c5_$TAG.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4_$TAG" -o run \
  -- python3 "$ROOT/bench.py" --workload ba --c4 --steps 20 --warmup 3 > "$OUT/ba_c4_prof_$TAG.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5_$TAG" -o run \
  -- python3 "$ROOT/bench.py" --workload ba --c5 --steps 5 --warmup 2 > "$OUT/ba_c5_prof_$TAG.log" 2>&1 || exit 1
find "$OUT/prof_c4_$TAG" "$OUT/prof_c5_$TAG" -name "*kernel_trace.csv" -delete
echo done

#!/bin/bash
# VO front-end bench + rocprofv3 kernel-trace summary (one GPU call).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
TAG="${1:-vo}"
shift || true
timeout -k 10 300 python bench.py --workload vo "$@" > "$OUT/bench_$TAG.log" 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run \
  -- python3 "$ROOT/bench.py" --workload vo --steps 5 --warmup 2 --no-cpu-baseline "$@" \
  > "$OUT/bench_prof_$TAG.log" 2>&1
rc=$?
tail -1 "$OUT/bench_$TAG.log"
exit $rc

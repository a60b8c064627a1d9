#!/bin/bash
# rocprofv3 kernel-trace summary of a short default bench run (kernel stats only).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r2}"
shift || true
OUT="$ROOT/gpurun_out/kst_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run \
  -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-ba-scale --steps 10 --warmup 3 "$@" > "$OUT/bench.log" 2>&1 || exit 1
find "$OUT" -name "*kernel_trace.csv" -delete
echo done

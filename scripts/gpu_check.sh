#!/bin/bash
# One GPU-box pass: parity tests, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; steps are chained with && so a
# failure stops the call.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
TAG="${1:-r1}"
shift || true
BENCH_ARGS="$*"
timeout -k 10 420 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu_$TAG.log" 2>&1 && \
timeout -k 10 300 python bench.py $BENCH_ARGS > "$OUT/bench_$TAG.log" 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o run \
  -- python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline $BENCH_ARGS > "$OUT/bench_prof_$TAG.log" 2>&1
rc=$?
echo "exit=$rc"
exit $rc

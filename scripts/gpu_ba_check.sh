#!/bin/bash
# BA-only GPU pass: BA/dist parity tests, C4 bench, rocprofv3 kernel-trace summary.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
TAG="${1:-ba}"
shift || true
timeout -k 10 400 python -u -m pytest tests/test_ba.py tests/test_dist.py -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_ba_$TAG.log" 2>&1 && \
timeout -k 10 300 python bench.py --workload ba --c4 --steps 20 --warmup 3 "$@" > "$OUT/bench_ba_$TAG.log" 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_ba_$TAG" -o run \
  -- python3 "$ROOT/bench.py" --workload ba --c4 --steps 10 --warmup 2 "$@" > "$OUT/bench_ba_prof_$TAG.log" 2>&1
rc=$?
echo "exit=$rc"
exit $rc

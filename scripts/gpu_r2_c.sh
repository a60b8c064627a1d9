#!/bin/bash
# pipeline tests (tracked frames -> local BA at 3 and 8 pairs), default bench
# (with the tracked-window BA leg), matcher micro-bench at batch 32 / 512.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/c_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_pipeline.py -x -v -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest_pipeline.log" 2>&1 || exit 1
timeout -k 10 200 python bench.py > "$OUT/bench.log" 2>&1 || exit 1
timeout -k 10 120 python bench.py --workload matcher --batch 32 --steps 50 --warmup 5 > "$OUT/matcher32.log" 2>&1 || exit 1
timeout -k 10 120 python bench.py --workload matcher --batch 512 --steps 20 --warmup 3 > "$OUT/matcher512.log" 2>&1 || exit 1
echo done

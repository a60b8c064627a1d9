#!/bin/bash
# ORB parity tests + phase profile + default bench
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/orbv_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_orb.py tests/test_pipeline.py tests/test_bow.py -x -v -m gpu \
  --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
timeout -k 10 200 python scripts/orb_prof.py > "$OUT/orb_prof.log" 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 12 --warmup 3 > "$OUT/bench.log" 2>&1 || exit 1
echo done

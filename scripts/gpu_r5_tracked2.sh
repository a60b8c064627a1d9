#!/bin/bash
# Round 5: BAWindowSet test + the tracked leg.   scripts/gpu_r5_tracked2.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_ba.py tests/test_pipeline.py -x -v -m gpu -k "window_set or folded or window_mapper or stage" --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
bash scripts/gpu_r5_tracked.sh $TAG

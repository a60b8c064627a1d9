#!/bin/bash
# ORB pipelining: equality test, then the tracking bench with / without it
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/orbpipe_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_pipeline.py -x -v -m gpu -k "pipelined or corridor" --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
B="python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 20 --warmup 3"
for i in 1 2; do
  timeout -k 10 120 $B > "$OUT/trk_base$i.log" 2>&1 || exit 1
  timeout -k 10 120 $B --orb-pipeline > "$OUT/trk_pipe$i.log" 2>&1 || exit 1
done
timeout -k 10 120 $B --orb-pipeline --priority equal > "$OUT/trk_pipe_eq.log" 2>&1 || exit 1
timeout -k 10 120 $B --orb-pipeline --priority track > "$OUT/trk_pipe_track.log" 2>&1 || exit 1
echo done

#!/bin/bash
# k_solve_blk A/B: BA GPU tests on the tree's library, the per-panel timeline of
# the old and new solver (prof/libslam355_strace{_old,}.so, -DSLAM_SOLVE_TRACE),
# and the batched-window / C4 BA bench lines on the old (prof/libslam355_solve_old.so)
# and new libraries.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/solve_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_ba.py -x -q -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
for v in strace_old strace; do
  timeout -k 10 120 python scripts/solve_trace.py $v 8 > "$OUT/trace_$v.log" 2>&1 || exit 1
done
for v in solve_old ""; do
  lib=""; [ -n "$v" ] && lib="$ROOT/slam-1_amd/prof/libslam355_$v.so"
  SLAM355_LIB=$lib timeout -k 10 120 python bench.py --workload ba --ba-batch 8 --chunks-per-wg 8 --steps 30 --warmup 3 > "$OUT/ba_b8_${v:-new}.json" 2> "$OUT/ba_b8_${v:-new}.err" || exit 1
  SLAM355_LIB=$lib timeout -k 10 120 python bench.py --workload ba --c4 --steps 20 --warmup 3 > "$OUT/ba_c4_${v:-new}.json" 2> "$OUT/ba_c4_${v:-new}.err" || exit 1
done
echo done

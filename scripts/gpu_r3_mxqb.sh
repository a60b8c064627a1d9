#!/bin/bash
# Matcher query blocks per workgroup (SLAM_MX_QB 5 / 6 / 7 builds vs the tree's 8):
# bit-exact matcher tests on each build, then the C2 micro-bench (batch 32 / 512).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/mxqb_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for v in tree mxqb5 mxqb6 mxqb7; do
  lib=""; [ "$v" != tree ] && lib="$ROOT/slam-1_amd/prof/libslam355_$v.so"
  SLAM355_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_matcher.py -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_$v.log" 2>&1 || exit 1
  for b in 32 512; do
    SLAM355_LIB=$lib timeout -k 10 120 python bench.py --workload matcher --batch $b --steps 20 --warmup 3 > "$OUT/${v}_b$b.json" 2> "$OUT/${v}_b$b.err" || exit 1
  done
done
echo done

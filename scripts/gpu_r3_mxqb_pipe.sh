#!/bin/bash
# Matcher query blocks per workgroup inside the tracking pipeline: bit-exact
# matcher tests on the SLAM_MX_QB 4 / 6 builds, then the default tracking bench
# alternating tree (8) / 4 / 6 in separate processes:  gpu_r3_mxqb_pipe.sh TAG [ROUNDS]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
N="${2:-3}"
OUT="$ROOT/gpurun_out/mxqbpipe_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for v in mxqb4 mxqb6; do
  SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so timeout -k 10 200 python -u -m pytest tests/test_matcher.py -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_$v.log" 2>&1 || exit 1
done
for i in $(seq 1 $N); do
  for v in tree mxqb4 mxqb6; do
    lib=""; [ "$v" != tree ] && lib="$ROOT/slam-1_amd/prof/libslam355_$v.so"
    SLAM355_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba > "$OUT/${v}_$i.json" 2> "$OUT/${v}_$i.err" || exit 1
  done
done
echo done

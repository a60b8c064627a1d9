#!/bin/bash
# Matcher A/B: matcher GPU tests with the in-tree library, then the C2 matcher
# micro-bench (batch 32 and 512) for each named library variant.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
shift
OUT="$ROOT/gpurun_out/mxab_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_matcher.py -x -q -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
for v in "$@"; do
  for b in 32 512; do
    SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so timeout -k 10 120 python bench.py --workload matcher --batch $b --steps 20 --warmup 3 > "$OUT/m_${v}_b$b.json" 2> "$OUT/m_${v}_b$b.err" || exit 1
  done
done
echo done

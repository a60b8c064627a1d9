#!/bin/bash
# Matrix-core matcher check: matcher / pipeline GPU tests, the C2 matcher
# micro-bench (fp4 matrix cores vs the forced VALU kernel, batch 32 and 512),
# and a short tracking bench line.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/mx_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_matcher.py tests/test_pipeline.py tests/test_abi.py -x -v -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
for b in 32 512; do
  timeout -k 10 120 python bench.py --workload matcher --batch $b --steps 20 --warmup 3 > "$OUT/matcher_mx_b$b.json" 2> "$OUT/matcher_mx_b$b.err" || exit 1
  timeout -k 10 120 python bench.py --workload matcher --batch $b --steps 20 --warmup 3 --valu > "$OUT/matcher_valu_b$b.json" 2> "$OUT/matcher_valu_b$b.err" || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
echo done

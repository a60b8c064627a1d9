#!/bin/bash
# BA change check: BA / dist / pipeline GPU tests, the linearisation phase
# profile (prof/libslam355_linm.so), the batched-window BA bench (8 windows,
# 8 and 5 chunks per workgroup), C4, and a tracking bench line.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/ba_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 500 python -u -m pytest tests/test_ba.py tests/test_dist.py tests/test_pipeline.py -x -q -m gpu --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
timeout -k 10 120 python scripts/linm_prof.py 8 8 > "$OUT/linm_cpw8.log" 2>&1 || exit 1
for c in 8 5; do
  timeout -k 10 120 python bench.py --workload ba --ba-batch 8 --chunks-per-wg $c --steps 30 --warmup 3 > "$OUT/ba_b8_cpw$c.json" 2> "$OUT/ba_b8_cpw$c.err" || exit 1
done
timeout -k 10 120 python bench.py --workload ba --c4 --steps 20 --warmup 3 > "$OUT/ba_c4.json" 2> "$OUT/ba_c4.err" || exit 1
timeout -k 10 150 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 20 --warmup 3 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 1
echo done

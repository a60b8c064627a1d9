#!/bin/bash
# Camera solves with DPP row broadcasts: BA parity tests, phase timings of
# k_solve_blk (C3) and k_tl3_flow (C4 / C5), bench lines for batched C3, C4, C5.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/dpp_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 500 python -u -m pytest tests/test_ba.py tests/test_dist.py tests/test_pipeline.py -x -v -m gpu \
  --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_solveprof.so timeout -k 10 120 python scripts/ba_solve_prof.py > "$OUT/solve_prof.log" 2>&1 || exit 1
SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_flowprof.so timeout -k 10 200 python scripts/flow_prof.py > "$OUT/flow_prof.log" 2>&1 || exit 1
timeout -k 10 120 python bench.py --workload ba --ba-batch 4 --steps 200 --warmup 20 > "$OUT/ba_b4.log" 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload ba --c4 --steps 50 --warmup 5 > "$OUT/ba_c4.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload ba --c5 --steps 20 --warmup 3 > "$OUT/ba_c5.log" 2>&1 || exit 1
echo done

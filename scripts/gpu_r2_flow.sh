#!/bin/bash
# dataflow tiled solve: parity tests, then C4 / C5 bench lines and kernel stats
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/flow_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_ba.py tests/test_dist.py tests/test_pipeline.py -x -v -m gpu \
  -k "tiled or c4 or c5 or distributed or tracked" --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload ba --c4 --steps 50 --warmup 5 > "$OUT/ba_c4.log" 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload ba --c5 --steps 20 --warmup 3 > "$OUT/ba_c5.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o run \
  -- python3 "$ROOT/bench.py" --workload ba --c4 --steps 20 --warmup 3 > "$OUT/ba_c4_prof.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5" -o run \
  -- python3 "$ROOT/bench.py" --workload ba --c5 --steps 5 --warmup 2 > "$OUT/ba_c5_prof.log" 2>&1 || exit 1
find "$OUT" -name "*kernel_trace.csv" -delete
echo done

#!/bin/bash
# Round-4 baseline: GPU parity tests, smoke, the driver's bench command twice,
# and a longer timed region (60 steps) to see the steady state.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r4_base}"
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
bash scripts/gpu_r4_bench.sh "$TAG" 2 || exit 1
timeout -k 10 240 python3 bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-tracked-ba --no-ba-scale > "$OUT/bench_s60.json" 2>&1 || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench_s60.json'));print('s60', round(d['value']), round(d['ms_per_step'],3), round(d['host_issue_ms_per_step'],3))"

#!/bin/bash
# Native planner check: every BA / pipeline / dist GPU test (BAProblem now plans
# in C++ and uploads its tables in one copy), then the default bench line
# (tracked_window_ba.host_problem_build_ms).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r4_plan}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ba.py tests/test_dist.py tests/test_pipeline.py tests/test_posegraph.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]);print(round(d['value']), json.dumps(d['tracked_window_ba']))"

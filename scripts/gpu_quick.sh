#!/bin/bash
# Round-4 quick pass: selected GPU tests (pytest -k EXPR), then the driver's bench
# command, then optional extra bench workloads.  scripts/gpu_quick.sh TAG 'k-expr' [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; K="$2"; shift 2
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "$K" ]; then
  timeout -k 10 500 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(round(d['value']),round(d['ms_per_step'],3),round(d['host_issue_ms_per_step'],3), d.get('pcie_inclusive',{}).get('frames_per_s'))"

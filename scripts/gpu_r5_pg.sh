#!/bin/bash
# Round 5: pose-graph TRF (register-resident kernel) tests, A/B against the
# round-4 kernel, the C5 line; folded-BABatch test.  scripts/gpu_r5_pg.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_posegraph.py tests/test_ba.py -x -v -m gpu -k "trf or posegraph or objective or folded" --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -3 "$OUT/pytest.log"
for k in reg lds reg lds; do
  if [ $k = lds ]; then export SLAM_CHAIN_TRF=lds; else unset SLAM_CHAIN_TRF; fi
  timeout -k 10 120 python3 scripts/pg_time.py 500 5 >> "$OUT/pg_time.jsonl" 2>> "$OUT/pg_time.err" || { tail -20 "$OUT/pg_time.err"; exit 1; }
done
unset SLAM_CHAIN_TRF
cat "$OUT/pg_time.jsonl"
timeout -k 10 300 python3 bench.py --workload ba --c5 --steps 10 --warmup 3 > "$OUT/ba_c5.json" 2> "$OUT/ba_c5.err" || { tail -20 "$OUT/ba_c5.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/ba_c5.json'));print(d['value'], d['pose_graph']['ms_per_solve'], d['c5_pose_graph_plus_ba_ms'])"

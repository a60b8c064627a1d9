#!/bin/bash
# C4 / C5 BA lines and the C4 kernel stats; the tiled-solver GPU tests first.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r4_c4}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_ba.py tests/test_dist.py -x -v -m gpu -k "tiled or flow or c4 or c5 or distributed" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/c4_$i.json || exit 1
  python3 -c "import json;d=json.load(open('$OUT/c4_$i.json'));print('c4', round(d['value']), round(d['ms_per_step']*1e3,1))"
done
timeout -k 10 200 python3 bench.py --workload ba --c5 --steps 10 --warmup 2 2>/dev/null | tail -1 > $OUT/c5.json || exit 1
python3 -c "import json;d=json.load(open('$OUT/c5.json'));print('c5', round(d['value']), round(d['ms_per_step']*1e3,1), d['pose_graph']['ms_per_solve'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof -o run -- python3 $ROOT/bench.py --workload ba --c4 --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
python3 - <<PY
import csv
rows=list(csv.DictReader(open('$ROOT/$OUT/prof/run_kernel_stats.csv')))
for r in rows[:8]: print(f"{r['Name'][:50]:50s} {r['Calls']:>4} {float(r['AverageNs'])/1e3:8.1f}")
PY

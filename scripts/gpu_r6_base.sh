#!/bin/bash
# Round 6 baseline / check pass: the driver's bench command, the C4 and C5 LM
# lines, and the per-rank split (C4 / C5 at W = 1 and rank 0 of W = 8) under
# rocprofv3 kernel stats.   scripts/gpu_r6_base.sh TAG [pytest -k EXPR]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; K="$2"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$ROOT"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', round(d['value']), round(d['ms_per_step'],3))"
timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/c4.json || exit 1
timeout -k 10 200 python3 bench.py --workload ba --c5 --steps 10 --warmup 2 2>/dev/null | tail -1 > $OUT/c5.json || exit 1
python3 -c "import json;a=json.load(open('$OUT/c4.json'));b=json.load(open('$OUT/c5.json'));print('C4', round(a['value']), '| C5', round(b['value']))"
cd /tmp && export TMPDIR=/tmp
for cfg in "C4 1 0" "C4 8 0" "C5 1 0" "C5 8 0"; do
  set -- $cfg
  d=$OUT/split/${1}_w${2}_r${3}
  mkdir -p $OUT/split
  cpw=""
  if [ $2 -gt 1 ]; then cpw=$(python3 -c "import sys;sys.path[:0]=['$ROOT/slam-1_amd'];from slam355.dist import shard_chunks_per_wg as f;n=(300000 if '$1'=='C4' else 1200000)//$2;v=f(n);print(v if v else 0)"); fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 $ROOT/scripts/shard_split.py $1 $2 $3 20 $cpw > $d.json 2> $d.err || { tail -20 $d.err; exit 1; }
  find $d -name "*kernel_trace.csv" -delete
  tail -1 $d.json
done
python3 $ROOT/scripts/split_summary.py $OUT/split > $OUT/split/summary.json && python3 -c "
import json;d=json.load(open('$OUT/split/summary.json'))
for k,v in d.items(): print(k, 'div', v['divided'], 'rep', v['replicated'], 'wall', v.get('wall_us_per_iter'))"

#!/bin/bash
# Round 6: BA GPU tests (-k EXPR), then the C4 / C5 LM lines and optionally
# the per-rank split.   scripts/gpu_r6_ba.sh TAG 'k-expr' [split]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; K="$2"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"
cd "$ROOT"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_ba.py tests/test_dist.py -x -v -m gpu -k "$K" --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
for i in 1 2; do
  timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/c4_$i.json || exit 1
  timeout -k 10 200 python3 bench.py --workload ba --c5 --steps 10 --warmup 2 2>/dev/null | tail -1 > $OUT/c5_$i.json || exit 1
  python3 -c "import json;a=json.load(open('$OUT/c4_$i.json'));b=json.load(open('$OUT/c5_$i.json'));print('C4', round(a['value']), round(a['ms_per_step']*1e3,1), '| C5', round(b['value']), round(b['ms_per_step']*1e3,1))"
done
if [ "$3" = split ]; then
  cd /tmp && export TMPDIR=/tmp
  for cfg in "C4 1 0" "C4 8 0" "C5 1 0" "C5 8 0"; do
    set -- $cfg
    d=$OUT/split/${1}_w${2}_r${3}
    mkdir -p $OUT/split
    cpw=""
    if [ $2 -gt 1 ]; then cpw=$(python3 -c "import sys;sys.path[:0]=['$ROOT/slam-1_amd'];from slam355.dist import shard_chunks_per_wg as f;n=(300000 if '$1'=='C4' else 1200000)//$2;v=f(n);print(v if v else 0)"); fi
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 $ROOT/scripts/shard_split.py $1 $2 $3 20 $cpw > $d.json 2> $d.err || { tail -20 $d.err; exit 1; }
    find $d -name "*kernel_trace.csv" -delete
  done
  python3 $ROOT/scripts/split_summary.py $OUT/split > $OUT/split/summary.json && python3 -c "
import json;d=json.load(open('$OUT/split/summary.json'))
for k,v in d.items(): print(k, 'div', v['divided'], 'rep', v['replicated'], 'flow', v.get('k_tl3_flow'), 'wall', v.get('wall_us_per_iter'))"
fi

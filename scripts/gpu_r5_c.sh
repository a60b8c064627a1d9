#!/bin/bash
# Round 5 pass C: flow solve with the row-tile updates folded into the
# diagonal phase.  BA / dist GPU tests, flow timeline (HEAD vs round-4
# ba.hip), C4 / C5 A/B with the final costs compared (bit-identical iterates).
#   scripts/gpu_r5_c.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_ba.py tests/test_dist.py -x -v -m gpu -k "tiled or flow or c4 or c5 or distributed or capi or folded" --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for v in flowprof1 flowprofr4; do
  SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so timeout -k 10 200 python3 scripts/flow_prof.py > $OUT/flow_$v.log 2>&1 || { tail $OUT/flow_$v.log; exit 1; }
  echo $v; grep -E "^C|factor of" $OUT/flow_$v.log
done
for i in 1 2; do
  for v in def r4; do
    if [ $v = def ]; then unset SLAM355_LIB; else export SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so; fi
    timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/c4_${v}_$i.json || exit 1
    timeout -k 10 200 python3 bench.py --workload ba --c5 --steps 10 --warmup 2 2>/dev/null | tail -1 > $OUT/c5_${v}_$i.json || exit 1
    python3 -c "import json;a=json.load(open('$OUT/c4_${v}_$i.json'));b=json.load(open('$OUT/c5_${v}_$i.json'));print('$v', $i, 'C4', round(a['value']), round(a['ms_per_step']*1e3,1), repr(a['final_cost']), '| C5', round(b['value']), round(b['ms_per_step']*1e3,1), repr(b['final_cost']))"
  done
done

#!/bin/bash
# Round 5: software-pipelined pivot chains (tile factor + k_solve_blk panels).
# Tiled / flow / C3 BA tests, C4 / C5 / batched-C3 A/B against the HEAD build
# (prof/libslam355_head.so), flow-solve timeline of the profiling build.
#   scripts/gpu_r5_fac.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r5_fac}; VAR=slam-1_amd/prof/libslam355_head.so
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ba.py tests/test_dist.py -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for v in def head; do
    if [ $v = head ]; then export SLAM355_LIB=$ROOT/$VAR; else unset SLAM355_LIB; fi
    timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/c4_${v}_$i.json || exit 1
    timeout -k 10 200 python3 bench.py --workload ba --c5 --steps 10 --warmup 2 2>/dev/null | tail -1 > $OUT/c5_${v}_$i.json || exit 1
    timeout -k 10 120 python3 bench.py --workload ba --ba-batch 16 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/b16_${v}_$i.json || exit 1
    python3 -c "import json;a=json.load(open('$OUT/c4_${v}_$i.json'));b=json.load(open('$OUT/c5_${v}_$i.json'));c=json.load(open('$OUT/b16_${v}_$i.json'));print('$v', $i, 'C4', round(a['value']), round(a['ms_per_step']*1e3,1), a['final_cost'], '| C5', round(b['value']), round(b['ms_per_step']*1e3,1), b.get('final_cost'), '| B16', round(c['value']), round(c['ms_per_step']*1e3,1))"
  done
done
unset SLAM355_LIB
SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_flowprof.so timeout -k 10 200 python3 scripts/flow_prof.py > $OUT/flow_phases.log 2>&1 || { tail $OUT/flow_phases.log; exit 1; }
grep -E "^C|factor of" $OUT/flow_phases.log
echo ok

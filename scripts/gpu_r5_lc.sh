#!/bin/bash
# Round 5: the flow solve's child order (last child without row-tile share,
# SLAM_TL_LASTCHILD=1, default) vs the plain level order (=0): tiled / flow BA
# tests, C4 / C5 alternating, flow timelines both ways.   scripts/gpu_r5_lc.sh TAG
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r5_lc}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ba.py tests/test_dist.py -x -v -m gpu -k "tiled or flow or c4 or c5 or distributed or shard" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for v in 1 0; do
    export SLAM_TL_LASTCHILD=$v
    timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/c4_${v}_$i.json || exit 1
    timeout -k 10 200 python3 bench.py --workload ba --c5 --steps 10 --warmup 2 2>/dev/null | tail -1 > $OUT/c5_${v}_$i.json || exit 1
    python3 -c "import json;a=json.load(open('$OUT/c4_${v}_$i.json'));b=json.load(open('$OUT/c5_${v}_$i.json'));print('lastchild', $v, $i, 'C4', round(a['value']), round(a['ms_per_step']*1e3,1), a['final_cost'], '| C5', round(b['value']), round(b['ms_per_step']*1e3,1), b.get('final_cost'))"
  done
done
for v in 1 0; do
  export SLAM_TL_LASTCHILD=$v
  SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_flowprof.so timeout -k 10 200 python3 scripts/flow_prof.py > $OUT/flow_phases_$v.log 2>&1 || { tail $OUT/flow_phases_$v.log; exit 1; }
  echo "lastchild $v"; grep -E "^C" $OUT/flow_phases_$v.log
done
unset SLAM_TL_LASTCHILD

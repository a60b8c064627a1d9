#!/bin/bash
# Round-4 session-2 second pass: BA tiled-solve tests at the current library,
# C4 and C5 A/B against a variant (default: the 2x2-pivot factor alone), and
# the per-column flow-solve timeline (profiling build of the current ba.hip).
#   scripts/gpu_ab_ba.sh TAG VARIANT_SO
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${1:-r4s2b}; VAR=${2:-slam-1_amd/prof/libslam355_bafac.so}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ba.py tests/test_dist.py -x -v -m gpu -k "tiled or flow or c4 or c5 or distributed or capi" --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  for v in def var; do
    if [ $v = var ]; then export SLAM355_LIB=$ROOT/$VAR; else unset SLAM355_LIB; fi
    timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/c4_${v}_$i.json || exit 1
    timeout -k 10 200 python3 bench.py --workload ba --c5 --steps 10 --warmup 2 2>/dev/null | tail -1 > $OUT/c5_${v}_$i.json || exit 1
    python3 -c "import json;a=json.load(open('$OUT/c4_${v}_$i.json'));b=json.load(open('$OUT/c5_${v}_$i.json'));print('$v', $i, 'C4', round(a['value']), round(a['ms_per_step']*1e3,1), '| C5', round(b['value']), round(b['ms_per_step']*1e3,1))"
  done
done
unset SLAM355_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_c4 -o run -- python3 $ROOT/bench.py --workload ba --c4 --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_c5 -o run -- python3 $ROOT/bench.py --workload ba --c5 --steps 10 --warmup 2 > /dev/null 2>&1 || exit 1
find $ROOT/$OUT -name "*kernel_trace.csv" -delete
cd $ROOT
SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_flowprof.so timeout -k 10 200 python3 scripts/flow_prof.py > $OUT/flow_phases.log 2>&1 || { tail $OUT/flow_phases.log; exit 1; }
grep -E "^C|factor of" $OUT/flow_phases.log
echo ok

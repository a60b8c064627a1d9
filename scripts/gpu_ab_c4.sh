#!/bin/bash
# A/B of the C4 LM iteration: the default library vs a variant (SLAM355_LIB),
# alternating runs, then rocprof kernel stats of each.
#   scripts/gpu_ab_c4.sh TAG VARIANT_SO [bench args]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; VAR=$2; shift 2
OUT=$TAG; case $OUT in gpurun_out/*) ;; *) OUT=gpurun_out/$TAG;; esac; mkdir -p $OUT
for i in 1 2 3; do
  for v in def var; do
    if [ $v = var ]; then export SLAM355_LIB=$ROOT/$VAR; else unset SLAM355_LIB; fi
    timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 "$@" 2>/dev/null | tail -1 > $OUT/c4_${v}_$i.json || exit 1
    python3 -c "import json;d=json.load(open('$OUT/c4_${v}_$i.json'));print('$v', $i, round(d['value']), round(d['ms_per_step']*1e3,1))"
  done
done
unset SLAM355_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_def -o run -- python3 $ROOT/bench.py --workload ba --c4 --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
SLAM355_LIB=$ROOT/$VAR timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_var -o run -- python3 $ROOT/bench.py --workload ba --c4 --steps 20 --warmup 3 > /dev/null 2>&1 || exit 1
echo done

#!/bin/bash
# N-way alternating A/B of the C4 and C5 LM iteration lines:
# "def" = the default library, NAME = slam-1_amd/prof/libslam355_NAME.so.
#   scripts/gpu_ab_c4c5.sh TAG ROUNDS def NAME1 ...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; N=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $N); do
  for v in "$@"; do
    if [ $v = def ]; then unset SLAM355_LIB; else export SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so; fi
    timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/c4_${v}_$i.json || exit 1
    timeout -k 10 200 python3 bench.py --workload ba --c5 --steps 10 --warmup 2 2>/dev/null | tail -1 > $OUT/c5_${v}_$i.json || exit 1
    python3 -c "import json;a=json.load(open('$OUT/c4_${v}_$i.json'));b=json.load(open('$OUT/c5_${v}_$i.json'));print('$v', $i, 'C4', round(a['value']), round(a['ms_per_step']*1e3,1), '| C5', round(b['value']), round(b['ms_per_step']*1e3,1))"
  done
done
unset SLAM355_LIB

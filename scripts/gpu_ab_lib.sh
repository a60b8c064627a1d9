#!/bin/bash
# Alternating A/B of the default tracking bench (the driver's step counts)
# between the default library (A) and a variant library (B, SLAM355_LIB), plus
# the 16-window batched BA line of each.  scripts/gpu_ab_lib.sh TAG N VARIANT_SO
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; N=$2; VAR=$3
OUT=gpurun_out/$TAG; mkdir -p $OUT
run() {  # $1 = A|B, $2 = index
  if [ $1 = B ]; then export SLAM355_LIB=$ROOT/$VAR; else unset SLAM355_LIB; fi
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-tracked-ba --no-ba-scale --no-pcie-leg 2>/dev/null | tail -1 > $OUT/${1}_$2.json || return 1
  python3 -c "import json;d=json.load(open('$OUT/${1}_$2.json'));s=d['stage_ms_per_step'];print('$1', $2, round(d['value']), round(d['ms_per_step'],3), 'orb', round(s['orb'],2), 'ba', round(s['local_ba'],2), 'pnp', round(s['pnp'],2))"
}
for i in $(seq 1 $N); do run A $i || exit 1; run B $i || exit 1; done
for v in A B; do
  if [ $v = B ]; then export SLAM355_LIB=$ROOT/$VAR; else unset SLAM355_LIB; fi
  timeout -k 10 120 python3 bench.py --workload ba --ba-batch 16 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/b16_$v.json || exit 1
  python3 -c "import json;d=json.load(open('$OUT/b16_$v.json'));print('b16 $v', round(d['value']), round(d['ms_per_step']*1e3,1))"
done

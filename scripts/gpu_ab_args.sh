#!/bin/bash
# Alternating A/B of the default tracking bench (the driver's step counts):
#   scripts/gpu_ab_args.sh TAG N "A-args" "B-args"   (A/B args appended to bench.py)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; N=$2; A=$3; B=$4
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $N); do
  for v in A B; do
    if [ $v = A ]; then X=$A; else X=$B; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-tracked-ba --no-ba-scale --no-pcie-leg $X 2>/dev/null | tail -1 > $OUT/${v}_$i.json || exit 1
    python3 -c "import json;d=json.load(open('$OUT/${v}_$i.json'));s=d['stage_ms_per_step'];print('$v', $i, round(d['value']), round(d['ms_per_step'],3), 'orb', round(s['orb'],2), 'ba', round(s['local_ba'],2), 'pnp', round(s['pnp'],2))"
  done
done

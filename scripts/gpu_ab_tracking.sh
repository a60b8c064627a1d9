#!/bin/bash
# Alternating N-way A/B of the tracking bench (the driver's step counts):
# "def" = the default library, every other name = slam-1_amd/prof/libslam355_NAME.so.
#   scripts/gpu_ab_tracking.sh TAG ROUNDS def NAME1 NAME2 ...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; N=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $N); do
  for v in "$@"; do
    if [ $v = def ]; then unset SLAM355_LIB; else export SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-tracked-ba --no-ba-scale --no-pcie-leg 2>/dev/null | tail -1 > $OUT/${v}_$i.json || exit 1
    python3 -c "import json;d=json.load(open('$OUT/${v}_$i.json'));s=d['stage_ms_per_step'];print('$v', $i, round(d['value']), round(d['ms_per_step'],3), 'orb', round(s['orb'],2), 'ba', round(s['local_ba'],2), 'pnp', round(s['pnp'],2), 'stereo', round(s['stereo_knn2'],3))"
  done
done
unset SLAM355_LIB

#!/bin/bash
# Round 6: alternating A/B of the tracking bench (the driver's step counts, the
# headline region only) over LABEL=LIB=ARGS variants: LIB "def" or a
# slam-1_amd/prof/libslam355_LIB.so, ARGS extra bench.py arguments (',' for ' ').
#   scripts/gpu_r6_trk.sh TAG ROUNDS LABEL=LIB=ARGS...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; N=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $N); do
  for spec in "$@"; do
    lab=${spec%%=*}; rest=${spec#*=}; lib=${rest%%=*}; args=${rest#*=}; args=${args//,/ }
    if [ "$lib" = def ]; then unset SLAM355_LIB; else export SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$lib.so; fi
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-tracked-ba --no-ba-scale --no-pcie-leg --no-tracked-leg $args 2>/dev/null | tail -1 > $OUT/${lab}_$i.json || exit 1
    python3 -c "import json;d=json.load(open('$OUT/${lab}_$i.json'));s=d['stage_ms_per_step'];print('$lab', $i, round(d['value']), round(d['ms_per_step'],3), 'orb', round(s['orb'],2), 'ba', round(s['local_ba'],2), 'pnp', round(s['pnp'],2), 'stereo', round(s['stereo_knn2'],3))"
  done
done
unset SLAM355_LIB

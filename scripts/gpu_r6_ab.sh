#!/bin/bash
# Round 6: alternating A/B of (library variant, camera-solve tiling) pairs on
# the C4 / C5 LM lines.   scripts/gpu_r6_ab.sh TAG ROUNDS LIB@MODE...
# LIB: "def" (slam355/libslam355.so) or NAME (slam-1_amd/prof/libslam355_NAME.so);
# MODE: a SLAM_TL_TILES value ("-" = the default).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; N=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $N); do
  for vm in "$@"; do
    v=${vm%@*}; m=${vm#*@}
    if [ $v = def ]; then unset SLAM355_LIB; else export SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_$v.so; fi
    if [ "$m" = "-" ]; then unset SLAM_TL_TILES; else export SLAM_TL_TILES=$m; fi
    t=${v}_${m//:/_}
    timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/c4_${t}_$i.json || exit 1
    timeout -k 10 200 python3 bench.py --workload ba --c5 --steps 10 --warmup 2 2>/dev/null | tail -1 > $OUT/c5_${t}_$i.json || exit 1
    python3 -c "import json;a=json.load(open('$OUT/c4_${t}_$i.json'));b=json.load(open('$OUT/c5_${t}_$i.json'));print('$vm', $i, 'C4', round(a['value']), round(a['ms_per_step']*1e3,1), '| C5', round(b['value']), round(b['ms_per_step']*1e3,1))"
  done
done

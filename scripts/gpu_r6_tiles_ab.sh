#!/bin/bash
# Round 6: A/B of the camera solve's tiling (SLAM_TL_TILES) on the C4 / C5 LM
# lines, alternating, plus the replicated-part kernel averages of C4 / C5 at
# W = 1 per mode.   scripts/gpu_r6_tiles_ab.sh TAG ROUNDS MODE...
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=$1; N=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for i in $(seq 1 $N); do
  for m in "$@"; do
    export SLAM_TL_TILES=$m; v=${m//:/_}
    timeout -k 10 120 python3 bench.py --workload ba --c4 --steps 40 --warmup 5 2>/dev/null | tail -1 > $OUT/c4_${v}_$i.json || exit 1
    timeout -k 10 200 python3 bench.py --workload ba --c5 --steps 10 --warmup 2 2>/dev/null | tail -1 > $OUT/c5_${v}_$i.json || exit 1
    python3 -c "import json;a=json.load(open('$OUT/c4_${v}_$i.json'));b=json.load(open('$OUT/c5_${v}_$i.json'));print('$m', $i, 'C4', round(a['value']), round(a['ms_per_step']*1e3,1), '| C5', round(b['value']), round(b['ms_per_step']*1e3,1))"
  done
done
cd /tmp && export TMPDIR=/tmp
for m in "$@"; do
  export SLAM_TL_TILES=$m; v=${m//:/_}
  for c in C4 C5; do
    d=$ROOT/$OUT/split_$v/${c}_w1_r0; mkdir -p $ROOT/$OUT/split_$v
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 $ROOT/scripts/shard_split.py $c 1 0 20 > $d.json 2> $d.err || { tail -20 $d.err; exit 1; }
    find $d -name "*kernel_trace.csv" -delete
  done
  python3 $ROOT/scripts/split_summary.py $ROOT/$OUT/split_$v > $ROOT/$OUT/split_$v/summary.json && python3 -c "
import json;d=json.load(open('$ROOT/$OUT/split_$v/summary.json'))
for k,v in d.items(): print('$m', k, 'rep', v['replicated'], 'flow', v.get('k_tl3_flow'), 'wall', v.get('wall_us_per_iter'))"
done

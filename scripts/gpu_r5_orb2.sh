#!/bin/bash
# Round 5: ORB change vs the HEAD orb.hip (prof/libslam355_orbhead.so):
# ORB / pipeline GPU tests, ORB alone and the bench, alternating.
#   scripts/gpu_r5_orb2.sh TAG [bench rounds]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; N="${2:-2}"; OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
VAR=$ROOT/slam-1_amd/prof/libslam355_orbhead.so
timeout -k 10 500 python -u -m pytest tests/test_orb.py tests/test_pipeline.py -x -v -m gpu --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for i in 1 2 3; do
  for v in new head; do
    if [ $v = head ]; then export SLAM355_LIB=$VAR; else unset SLAM355_LIB; fi
    timeout -k 10 120 python3 scripts/orb_time.py >> $OUT/orb_time_$v.txt 2>> $OUT/orb_time.err || { tail -20 $OUT/orb_time.err; exit 1; }
    echo "$v $(tail -1 $OUT/orb_time_$v.txt)"
  done
done
for i in $(seq 1 $N); do
  for v in new head; do
    if [ $v = head ]; then export SLAM355_LIB=$VAR; else unset SLAM355_LIB; fi
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ba-scale --no-tracked-ba --no-pcie-leg --no-tracked-leg > $OUT/bench_${v}_$i.json 2> $OUT/bench_${v}_$i.err || { tail -20 $OUT/bench_${v}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_${v}_$i.json'));print('$v', $i, round(d['value']),round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['stage_ms_per_step'].items()})"
  done
done
unset SLAM355_LIB

#!/bin/bash
# 16 local-BA windows in ONE batched launch (library built with
# -DSLAM_BA_MAX_BATCH=16, prof/libslam355_mb16.so) every 2 steps against the
# default 8-window set every step, alternating in separate processes:
# (and, when prof/libslam355_mb32.so exists, 32 windows every 4 steps):
#   gpu_r3_mb16_ab.sh TAG [ROUNDS]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
N="${2:-3}"
OUT="$ROOT/gpurun_out/mb16_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 $N); do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba > "$OUT/default_$i.json" 2> "$OUT/default_$i.err" || exit 1
  SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_mb16.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --ba-group 2 > "$OUT/mb16g2_$i.json" 2> "$OUT/mb16g2_$i.err" || exit 1
  if [ -f "$ROOT/slam-1_amd/prof/libslam355_mb32.so" ]; then
    SLAM355_LIB=$ROOT/slam-1_amd/prof/libslam355_mb32.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --ba-group 4 > "$OUT/mb32g4_$i.json" 2> "$OUT/mb32g4_$i.err" || exit 1
  fi
done
echo done

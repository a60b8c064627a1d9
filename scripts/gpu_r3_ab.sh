#!/bin/bash
# Tracking-bench A/B of a variant library against the tree's library,
# alternating in separate processes:  gpu_r3_ab.sh TAG VARIANT [ROUNDS]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
VAR="$2"
N="${3:-3}"
OUT="$ROOT/gpurun_out/ab_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 $N); do
  for v in tree $VAR; do
    lib=""; [ "$v" != tree ] && lib="$ROOT/slam-1_amd/prof/libslam355_$v.so"
    SLAM355_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 20 --warmup 4 > "$OUT/${v}_$i.json" 2> "$OUT/${v}_$i.err" || exit 1
  done
done
echo done

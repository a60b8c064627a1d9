#!/bin/bash
# Batch-64 tracking bench: local-BA launch set of 1 vs 2 steps (--ba-group),
# alternating in separate processes:  gpu_r3_b64_ab.sh TAG [ROUNDS]
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
N="${2:-3}"
OUT="$ROOT/gpurun_out/b64ab_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 $N); do
  for g in 1 2; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --batch 64 --ba-group $g --steps 10 --warmup 4 > "$OUT/g${g}_$i.json" 2> "$OUT/g${g}_$i.err" || exit 1
  done
done
echo done

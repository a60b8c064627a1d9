#!/bin/bash
# --ba-group 2 vs 4 (8 vs 16 windows per local-BA launch set), alternating.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/groupab_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for i in 1 2 3; do
  for g in 2 4; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --ba-group $g --steps 24 --warmup 4 > "$OUT/g${g}_$i.json" 2> "$OUT/g${g}_$i.err" || exit 1
  done
done
echo done

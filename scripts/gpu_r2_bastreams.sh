#!/bin/bash
# tracking bench: local-BA windows on 1 / 2 / 4 streams (ORB pipelined, masked)
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/bastreams_${1:-r2}"
mkdir -p "$OUT"
cd "$ROOT"
B="python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 30 --warmup 3"
for i in 1 2; do
  for s in 1 2 4; do
    timeout -k 10 120 $B --ba-streams $s > "$OUT/s${s}_$i.log" 2>&1 || exit 1
  done
done
echo done

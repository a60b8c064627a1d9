#!/bin/bash
# Bench sweeps of the stream / CU split (round 3): one short bench line per
# setting, settings given as quoted argument strings.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
shift
OUT="$ROOT/gpurun_out/sweep_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
i=0
for a in "$@"; do
  i=$((i + 1))
  timeout -k 10 150 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --steps 20 --warmup 3 $a > "$OUT/s$i.json" 2> "$OUT/s$i.err" || exit 1
  echo "$a" > "$OUT/s$i.args"
done
echo done

#!/bin/bash
# Local-BA launch-set size: batched windows alone (8 / 16 windows, 8 / 5
# chunks per workgroup) and the tracking bench with --ba-group 1 / 2 / 4.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-r3}"
OUT="$ROOT/gpurun_out/bagroup_$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for nb in 8 16; do
  for c in 8 5; do
    timeout -k 10 120 python bench.py --workload ba --ba-batch $nb --chunks-per-wg $c --steps 20 --warmup 3 > "$OUT/ba_b${nb}_cpw$c.json" 2> "$OUT/ba_b${nb}_cpw$c.err" || exit 1
  done
done
for g in 2 4 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-ba-scale --no-tracked-ba --ba-group $g --steps 16 --warmup 4 > "$OUT/g$g.json" 2> "$OUT/g$g.err" || exit 1
  cat "$OUT/g$g.json" >> "$OUT/groups.jsonl"
done
echo done
